#!/bin/bash
# round-4 GPU bundle w: 2-rank rehearsal of the multi-GPU bench path (gloo collectives, both ranks on the one GPU; not a measurement)
out=gpurun_out/r4w
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
DPEMU_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > $out/rehearse.json 2> $out/rehearse.err || { echo "rehearsal failed"; tail -30 $out/rehearse.err; exit 1; }
python - $out/rehearse.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split('\n')[-1])
print('n_gpus', d['n_gpus'], 'world', d['collective_world_size'], d['collective_backend'], 'value', d['value'], 'legs', sorted(d['legs']), 'len', len(json.dumps(d)))
PY
