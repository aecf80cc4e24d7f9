# LUT parallel merge: parity + bench; config 4 chunk A/B
set -o pipefail
out=gpurun_out/r03g
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_lane_order.py -k "lut or fuzz or config3" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python bench.py --legs active_reset,lut --no-cpu-baseline > $out/bench_lut.json 2> $out/bench_lut.err || { tail $out/bench_lut.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench_lut.json'))
for k in ('active_reset','lut'): print(k, d[k]['kernel'], d[k]['ms_per_step'], d[k]['roofline']['kernel_ms'])"
timeout -k 10 300 python scripts/ab.py --libs ab_build/libdpemu_ch8.so,ab_build/libdpemu_ch16.so,ab_build/libdpemu_ch32.so --flags 0,0,0 --workload rb --reps 3 --steps 3 > $out/ab_ch.json 2> $out/ab_ch.err || { tail $out/ab_ch.err; exit 1; }
cat $out/ab_ch.json
