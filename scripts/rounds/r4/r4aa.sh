#!/bin/bash
# round-4 GPU bundle aa: config 4 -- threshold from LDS (no vmcnt drain at a
# measurement) and the producer-wave variant; small check first, then A/B
out=gpurun_out/r4aa
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 90 python -u scripts/ab.py --libs ${L}mhead.so,${L}mthr.so,${L}mprod.so --workload rb_sm --reps 2 --steps 2 > $out/small.jsonl 2>&1 || { echo "small failed"; tail $out/small.jsonl; exit 1; }
tail -1 $out/small.jsonl
grep -q '"same_outputs": true' $out/small.jsonl || { echo "outputs differ"; exit 1; }
timeout -k 10 300 python -u scripts/ab.py --libs ${L}mhead.so,${L}mthr.so,${L}mprod.so --workload rb --reps 6 --steps 4 > $out/ab.jsonl 2>&1 || { echo "ab failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
