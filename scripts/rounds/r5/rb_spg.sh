#!/bin/bash
# Round 5: config 4's kernel time vs shots per sequence (8: 128-B event pieces,
# 10: the BASELINE's 160-B pieces, 16: 256-B pieces) -- how much the partial
# event rows cost
set -o pipefail
out=gpurun_out/r5/rb_spg
mkdir -p $out
for spg in ${SPGS:-8 10 16}; do
  timeout -k 10 300 python bench.py --legs rb --no-cpu-baseline --rb-spg $spg --steps 10 > $out/spg$spg.json 2> $out/spg$spg.err || { tail $out/spg$spg.err; exit 1; }
  python - $out/spg$spg.json $spg <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['rb']
print(sys.argv[2], {k: b.get(k) for k in ('value', 'ms_per_step', 'kernel_ms')})
PY
done
