#!/bin/bash
# Round 5: DDS A/B -- occupancy (round-4 kernel at 6 waves) and round-robin stripes in the single-launch kernel
set -o pipefail
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
L=distributed_processor_amd/libdpemu.so
timeout -k 10 300 python -u scripts/ab_dds.py --reps 6 --steps 20 \
    --libs $L,ab_build/libdpemu_r4.so,ab_build/libdpemu_r4w6.so,ab_build/libdpemu_st13.so,ab_build/libdpemu_st13w7.so \
    | tee gpurun_out/r5/dds_ab2.json
