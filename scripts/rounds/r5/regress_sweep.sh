#!/bin/bash
# Round 5: regression sweep -- round-4 library vs HEAD on every ab.py workload,
# plus the general interpreter (DPEMU_X_GENERAL) and the direct macro kernel
set -o pipefail
out=gpurun_out/r5/regress
mkdir -p $out
L=ab_build/libdpemu_r4.so,ab_build/libdpemu_head.so
for wl in ramsey ar ar_sm lut_sm rb; do
  timeout -k 10 300 python -u scripts/ab.py --workload $wl --libs $L --reps 3 --steps 3 > $out/$wl.json 2> $out/$wl.err || { tail $out/$wl.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$out/$wl.json')); print('$wl', d['kernels'], d['median_ms'])"
done
for wl in ramsey ar_sm; do
  timeout -k 10 300 python -u scripts/ab.py --workload $wl --libs $L --flags 0x20,0x20 --reps 2 --steps 2 > $out/${wl}_general.json 2> $out/${wl}_general.err || { tail $out/${wl}_general.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$out/${wl}_general.json')); print('$wl general', d['kernels'], d['median_ms'])"
done
