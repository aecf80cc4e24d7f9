#!/bin/bash
# Round 5: the 12-slot staged macro kernel vs the per-lane macro_kernel (forced
# with DPEMU_X_MACRO_DIRECT) on the launches it now takes: config 4 with 8
# shots per sequence (core-major) and with 10 shots per sequence in shot-major order
set -o pipefail
out=gpurun_out/r5/macro_wide
mkdir -p $out
lib=distributed_processor_amd/libdpemu.so
timeout -k 10 300 python -u scripts/ab.py --workload rb8 --reps 3 --steps 3 --flags 0x40,0 --libs $lib,$lib \
    > $out/ab_rb8.json 2> $out/ab_rb8.err || { tail $out/ab_rb8.err; exit 1; }
cat $out/ab_rb8.json
timeout -k 10 300 python -u scripts/ab.py --workload rb --lane-order 1 --reps 3 --steps 3 --flags 0x40,0 --libs $lib,$lib \
    > $out/ab_rb_sm.json 2> $out/ab_rb_sm.err || { tail $out/ab_rb_sm.err; exit 1; }
cat $out/ab_rb_sm.json
