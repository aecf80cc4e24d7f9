#!/bin/bash
# Round 5: the single-launch DDS kernel -- parity, then same-process A/B of
# segment sizes / occupancy against the round-4 library (index + stripes).
set -o pipefail
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_dds.py \
    "tests/test_gpu_fullsize.py::test_config5_full_launch_all_channels" > gpurun_out/r5/dds_pytest.log 2>&1 || { tail -30 gpurun_out/r5/dds_pytest.log; exit 1; }
tail -3 gpurun_out/r5/dds_pytest.log
L=distributed_processor_amd/libdpemu.so
timeout -k 10 300 python -u scripts/ab_dds.py --reps 6 --steps 20 \
    --libs $L,ab_build/libdpemu_r4.so,ab_build/libdpemu_w7s52.so,ab_build/libdpemu_w6s16.so,ab_build/libdpemu_w6s26.so,ab_build/libdpemu_w6s103.so,ab_build/libdpemu_w6s206.so \
    | tee gpurun_out/r5/dds_ab.json
