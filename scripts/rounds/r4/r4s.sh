#!/bin/bash
# round-4 GPU bundle s: host enqueue rate of the config-1 / config-2 steps
out=gpurun_out/r4s
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
timeout -k 10 240 python -u scripts/host_rate.py > $out/host_rate.jsonl 2>&1 || { echo "host_rate failed"; tail $out/host_rate.jsonl; exit 1; }
cat $out/host_rate.jsonl
