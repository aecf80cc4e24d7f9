# round-3 GPU call: VALU peak evidence, staged-macro parity + A/B, bench
set -o pipefail
out=gpurun_out/r03a
mkdir -p $out
bash scripts/valu_peak.sh $out/vp || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rb.py tests/test_gpu_parity.py -k "linear or config4 or rb or few_registers" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python scripts/ab.py --libs distributed_processor_amd/libdpemu.so,distributed_processor_amd/libdpemu.so --flags 0,0x40 --workload rb --reps 3 --steps 3 > $out/ab_rb.json 2> $out/ab_rb.err || { echo "ab failed"; tail $out/ab_rb.err; exit 1; }
cat $out/ab_rb.json
timeout -k 10 600 python bench.py --legs rb > $out/bench_rb.json 2> $out/bench_rb.err || { echo "bench failed"; tail $out/bench_rb.err; exit 1; }
