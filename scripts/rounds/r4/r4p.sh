#!/bin/bash
# round-4 GPU bundle p: config-3 row flush only at two held records (A/B)
out=gpurun_out/r4p
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 120 python -u scripts/branch_counts.py --lib ${L}bfl2c.so --workload ar_sm >> $out/counts.jsonl 2>&1 || { echo "counts failed"; tail $out/counts.jsonl; exit 1; }
tail -1 $out/counts.jsonl
for w in ar_sm ar ar_sm; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}bnew.so,${L}bfl2.so --workload $w --reps 8 --steps 10 >> $out/ab.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
done
