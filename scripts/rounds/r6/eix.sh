# element index (ABI 9): its GPU tests, the DDS / macro tests it touches, then the bench's DDS leg
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_elem_index.py tests/test_gpu_dds.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/eix_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --legs dds --steps 20 --warmup 3 > gpurun_out/eix_bench_dds.json 2> gpurun_out/eix_bench_dds.err
