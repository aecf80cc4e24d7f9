for v in "--spg 10000" "--spg 10000 --exec-flags 1" "--spg 1" "--spg 1 --exec-flags 1"; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $v > gpurun_out/v.log 2>&1 || exit $?
  echo "$v => $(python -c "import json,sys; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print(round(d['kernel_ms'],4), 'ms', '%.3e'%d['value'], round(d['roofline']['frac'],3))")"
done
