#!/bin/bash
# round-4 GPU bundle r: config-2 cost of the in-loop measurement draw (probe: VGPRs 76 -> 62)
out=gpurun_out/r4r
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ramsey ramsey; do
timeout -k 10 240 python -u scripts/ab.py --libs ${L}sbase.so,${L}snorng.so --workload $w --reps 8 --steps 10 --no-compare >> $out/ab.jsonl 2>&1 || { echo "ab $w failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
done
