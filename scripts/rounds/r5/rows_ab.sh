#!/bin/bash
# Round 5: branch_kernel<11,8> (config 3) -- HEAD vs uniform-row event holding
# (rows) vs the same at 7 waves per SIMD (rows_w7); same process, outputs identical.
set -o pipefail
out=gpurun_out/r5/rows_ab
mkdir -p $out
L=ab_build/libdpemu_head.so,ab_build/libdpemu_rows.so,ab_build/libdpemu_rows_w7.so
for wl in ar ar1; do
  timeout -k 10 240 python -u scripts/ab.py --workload $wl --libs $L --reps 10 --steps 10 \
      > $out/ab_$wl.json 2> $out/ab_$wl.err || { tail $out/ab_$wl.err; exit 1; }
  cat $out/ab_$wl.json
done
timeout -k 10 200 bash scripts/pmc_ab.sh ar branch_kernel ab_build/libdpemu_rows_w7.so > $out/pmc_w7.jsonl 2>&1 || { tail $out/pmc_w7.jsonl; exit 1; }
cat $out/pmc_w7.jsonl
