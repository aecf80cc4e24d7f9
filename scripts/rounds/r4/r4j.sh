#!/bin/bash
# round-4 GPU bundle j: config-3 whole-row flush (old vs new) A/B
out=gpurun_out/r4j
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm ar_sm ar; do
    timeout -k 10 240 python -u scripts/ab.py --libs ${L}br0.so,${L}br2.so --workload $w --reps 8 --steps 10 >> $out/ab_flush.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab_flush.jsonl; exit 1; }
    tail -1 $out/ab_flush.jsonl
done
