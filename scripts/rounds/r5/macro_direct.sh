#!/bin/bash
# Round 5: the per-lane-fetch macro_kernel (DPEMU_X_MACRO_DIRECT; what config 4
# runs when a wave spans more than MACRO_SLOTS programs, e.g. 8 shots per
# sequence) across builds: round 4, before the 3-slot macros, now
set -o pipefail
out=gpurun_out/r5/macro_direct
mkdir -p $out
timeout -k 10 400 python -u scripts/ab.py --workload rb --reps 3 --steps 2 --flags 0x40,0x40,0x40,0 \
    --libs ab_build/libdpemu_r4.so,ab_build/libdpemu_prew3.so,ab_build/libdpemu_head.so,ab_build/libdpemu_head.so \
    > $out/ab_rb.json 2> $out/ab_rb.err || { tail $out/ab_rb.err; exit 1; }
cat $out/ab_rb.json
