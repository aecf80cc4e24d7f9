#!/bin/bash
# Round 5: config 3, held rows by parity slot with the round-4 wave-minimum flush (v1) vs round 4
set -o pipefail
out=gpurun_out/r5/v1_ab
mkdir -p $out
for wl in ar_sm ar; do
  timeout -k 10 240 python -u scripts/ab.py --workload $wl --libs ab_build/libdpemu_head.so,ab_build/libdpemu_v1.so --reps 10 --steps 10 \
      > $out/ab_$wl.json 2> $out/ab_$wl.err || { tail $out/ab_$wl.err; exit 1; }
  cat $out/ab_$wl.json
done
