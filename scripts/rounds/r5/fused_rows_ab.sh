#!/bin/bash
# Round 5: fused DDS launch (index workgroups + tile workgroups, per-channel
# ready flags) and the branch kernel's uniform-row event holding, against
# HEAD's library: GPU parity for both paths, then same-process A/Bs.
set -o pipefail
out=gpurun_out/r5/fused_rows
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_dds.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_lane_order.py \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 240 python -u scripts/ab_dds.py --libs ab_build/libdpemu_head.so,ab_build/libdpemu_fused.so --reps 5 \
    > $out/ab_dds.json 2> $out/ab_dds.err || { tail $out/ab_dds.err; exit 1; }
cat $out/ab_dds.json
timeout -k 10 240 python -u scripts/ab.py --workload ar --libs ab_build/libdpemu_head.so,ab_build/libdpemu_fused.so --reps 5 \
    > $out/ab_ar.json 2> $out/ab_ar.err || { tail $out/ab_ar.err; exit 1; }
cat $out/ab_ar.json
