#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks on cuda:0 over
# gloo (the real N>1 runs use RCCL, one GPU per rank).  Short run, no CPU baseline.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
DPEMU_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_rehearse.log 2>&1
rc=$?; echo "rehearse rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_rehearse.log | tail -5
exit $rc
