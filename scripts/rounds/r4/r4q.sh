#!/bin/bash
# round-4 GPU bundle q: config-2 batched-fetch probe; occupancy A/B
out=gpurun_out/r4q
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ramsey ramsey; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}sbase.so,${L}sw7.so,${L}sw8.so --workload $w --reps 8 --steps 10 >> $out/ab2.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab2.jsonl; exit 1; }
tail -1 $out/ab2.jsonl
done
