#!/bin/bash
# Round 5: MACRO_W3 (three ALU slots per macro) -- macro-path parity, then config 4 against round 4
set -o pipefail
out=gpurun_out/r5/w3
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_rb.py tests/test_kat_outputs.py tests/test_gpu_lane_order.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u scripts/ab.py --libs distributed_processor_amd/libdpemu.so,ab_build/libdpemu_w3.so,ab_build/libdpemu_r4.so \
    --workload rb --reps 4 --steps 3 | tee $out/rb_ab.json
