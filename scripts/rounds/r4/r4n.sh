#!/bin/bash
# round-4 GPU bundle n: cost of the measurement generator in config 3 (probe)
out=gpurun_out/r4n
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm lut_sm; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}base.so,${L}norng.so --workload $w --reps 8 --steps 10 >> $out/ab.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
done
