#!/bin/bash
# round-4 GPU bundle o: branch_kernel section counts; Philox xors as bitop3 (A/B)
out=gpurun_out/r4o
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm lut_sm; do
timeout -k 10 120 python -u scripts/branch_counts.py --lib ${L}bcnt.so --workload $w >> $out/counts.jsonl 2>&1 || { echo "counts $w failed"; tail $out/counts.jsonl; exit 1; }
tail -1 $out/counts.jsonl
done
for w in ar_sm lut_sm ramsey; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}base.so,${L}bnew.so --workload $w --reps 8 --steps 10 >> $out/ab.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
done
