#!/bin/bash
# Round 5: config 3 in the bench's shot-major lane order -- round-4 branch
# kernel vs uniform-row holding at 6 and at 7 waves per SIMD.
set -o pipefail
out=gpurun_out/r5/r4w7
mkdir -p $out
L=ab_build/libdpemu_r4branch.so,ab_build/libdpemu_r4w7.so
for wl in ar_sm ar1 ar; do
  timeout -k 10 240 python -u scripts/ab.py --workload $wl --libs $L --reps 10 --steps 10 \
      > $out/ab_$wl.json 2> $out/ab_$wl.err || { tail $out/ab_$wl.err; exit 1; }
  cat $out/ab_$wl.json
done
