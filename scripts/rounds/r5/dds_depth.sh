#!/bin/bash
# Round 5: the DDS leg at depth 1 / 2 / 4 (serial and pipelined on the same line), and a
# kernel trace of the depth-2 steps (do index and tile kernels of adjacent batches overlap?)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/r5/dds_depth
mkdir -p $out
for d in 2 4; do
  timeout -k 10 300 python bench.py --legs dds --no-cpu-baseline --dds-depth $d --steps 40 > $out/bench_d$d.json 2> $out/bench_d$d.err || { tail $out/bench_d$d.err; exit 1; }
  python - $out/bench_d$d.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['dds']
print({k: b.get(k) for k in ('step_mode', 'ms_per_step', 'serial_ms_per_step', 'pipelined_ms_per_step', 'kernel_ms')})
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace2 -o t --output-format csv -- python3 bench.py --legs dds --no-cpu-baseline --dds-depth 2 --steps 20 > $out/trace2.log 2>&1 || { tail $out/trace2.log; exit 1; }
echo traced
