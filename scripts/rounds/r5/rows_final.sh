#!/bin/bash
# Round 5: the kept branch-kernel change (uniform-row event holding, 7 waves
# per SIMD) -- full -m gpu suite, then same-process A/B against HEAD.
set -o pipefail
out=gpurun_out/r5/rows_final
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
for wl in ar ar0 ar1; do
  timeout -k 10 240 python -u scripts/ab.py --workload $wl --libs ab_build/libdpemu_head.so,ab_build/libdpemu_rows_w7.so \
      --reps 10 --steps 10 > $out/ab_$wl.json 2> $out/ab_$wl.err || { tail $out/ab_$wl.err; exit 1; }
  cat $out/ab_$wl.json
done
