#!/bin/bash
# round-4 GPU bundle ab: DDS store-shape probe, set b (per-tile granularity, workgroup lifetime)
out=gpurun_out/r4ab
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
timeout -k 10 120 ./scripts/micro/dds_shape_probe b > $out/shape_e.jsonl 2>&1 || { echo "probe failed"; tail $out/shape_e.jsonl; exit 1; }
cat $out/shape_e.jsonl
