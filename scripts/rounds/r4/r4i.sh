#!/bin/bash
# round-4 GPU bundle i: config-3 direct event stores, longer A/B (both shapes, LUT)
out=gpurun_out/r4i
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm lut_sm ar_sm lut_sm; do
    timeout -k 10 240 python -u scripts/ab.py --libs ${L}br0.so,${L}br1.so --workload $w --reps 8 --steps 10 >> $out/ab_br.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab_br.jsonl; exit 1; }
    tail -1 $out/ab_br.jsonl
done
