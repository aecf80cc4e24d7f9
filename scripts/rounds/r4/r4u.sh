#!/bin/bash
# round-4 GPU bundle u: config-3 row flush by ballots when the stored-row count is wave-uniform (A/B)
out=gpurun_out/r4u
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm ar ar_sm; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}fb0.so,${L}fb1.so --workload $w --reps 8 --steps 10 >> $out/ab.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
done
