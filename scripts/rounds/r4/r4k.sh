#!/bin/bash
# round-4 GPU bundle k: config-3 wave tests as ballots of compares (A/B)
out=gpurun_out/r4k
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm lut_sm ar_sm; do
    timeout -k 10 240 python -u scripts/ab.py --libs ${L}br2.so,${L}br3.so,${L}br3p.so --workload $w --reps 8 --steps 10 >> $out/ab_any.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab_any.jsonl; exit 1; }
    tail -1 $out/ab_any.jsonl
done
