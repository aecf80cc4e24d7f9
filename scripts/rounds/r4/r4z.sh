#!/bin/bash
# round-4 GPU bundle z: config-2 probes on the bench's shot-major lanes
# (the generator's cost, occupancy, a wave-blocked event layout)
out=gpurun_out/r4z
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ramsey ramsey; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}sbase.so,${L}snorng.so,${L}sw7.so,${L}swb.so --workload $w --lane-order 1 --reps 8 --steps 10 --no-compare >> $out/ab.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
done
