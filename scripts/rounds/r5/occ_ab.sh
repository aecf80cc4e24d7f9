#!/bin/bash
# Round 5: config 2 with its residency capped by extra dynamic LDS (20/40/60 KiB per workgroup)
set -o pipefail
out=gpurun_out/r5/occ_ab
mkdir -p $out
timeout -k 10 240 python -u scripts/ab.py --workload ramsey --reps 8 --steps 10 \
    --libs ab_build/libdpemu_head.so,ab_build/libdpemu_occ20.so,ab_build/libdpemu_occ40.so,ab_build/libdpemu_occ60.so \
    > $out/ab_ramsey.json 2> $out/ab_ramsey.err || { tail $out/ab_ramsey.err; exit 1; }
cat $out/ab_ramsey.json
