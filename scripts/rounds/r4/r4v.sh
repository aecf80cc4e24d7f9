#!/bin/bash
# round-4 GPU bundle v: config-4 batches in flight 1 / 2 / 3 / 4 (bench rb leg only)
out=gpurun_out/r4v
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
for d in 2 3 4 2; do
timeout -k 10 300 python -u bench.py --legs rb --rb-depth $d --no-cpu-baseline --steps 20 --warmup 3 > $out/d$d.json 2> $out/d$d.err || { echo "bench d$d failed"; tail $out/d$d.err; exit 1; }
python - $out/d$d.json $d <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split('\n')[-1])
rb = d['rb']
print('depth', sys.argv[2], 'value', rb['value'], 'ms', rb['ms_per_step'], 'serial', rb.get('serial_ms_per_step'), 'kernel', rb.get('kernel_ms'))
PY
done
