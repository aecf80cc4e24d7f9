# staged macro kernel: parity + same-process A/B against macro_kernel + RB bench leg
set -o pipefail
out=gpurun_out/r03c
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rb.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_lane_order.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python scripts/ab.py --libs distributed_processor_amd/libdpemu.so,distributed_processor_amd/libdpemu.so --flags 0,0x40 --workload rb --reps 3 --steps 3 > $out/ab_rb.json 2> $out/ab_rb.err || { echo "ab failed"; tail $out/ab_rb.err; exit 1; }
cat $out/ab_rb.json
