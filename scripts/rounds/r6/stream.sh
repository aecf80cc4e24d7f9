# DPEMU_X_STREAM_EVENTS: HEAD library vs the working tree's with the flag off / on (config 4 both workloads),
# then the parity + RB GPU tests on the working tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_head.so,ab_build/libdpemu_new.so,ab_build/libdpemu_new.so
timeout -k 10 300 python -u scripts/ab.py --libs $L --flags 0,0,0x80 --workload rb2q > gpurun_out/stream_rb2q.json 2> gpurun_out/stream_rb2q.err &&
timeout -k 10 300 python -u scripts/ab.py --libs $L --flags 0,0,0x80 --workload rb > gpurun_out/stream_rb.json 2> gpurun_out/stream_rb.err &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rb.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/stream_tests.log 2>&1
