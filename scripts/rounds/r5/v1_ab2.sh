#!/bin/bash
# Round 5: v1 confirmation -- ar_sm (bench lane order) twice more, and PMC counts
set -o pipefail
out=gpurun_out/r5/v1_ab2
mkdir -p $out
for r in 1 2; do
  timeout -k 10 240 python -u scripts/ab.py --workload ar_sm --libs ab_build/libdpemu_head.so,ab_build/libdpemu_v1.so --reps 12 --steps 10 \
      > $out/ab_ar_sm_$r.json 2> $out/ab_ar_sm_$r.err || { tail $out/ab_ar_sm_$r.err; exit 1; }
  cat $out/ab_ar_sm_$r.json
done
timeout -k 10 200 bash scripts/pmc_ab.sh ar_sm branch_kernel ab_build/libdpemu_head.so ab_build/libdpemu_v1.so > $out/pmc.jsonl 2>&1 || { tail $out/pmc.jsonl; exit 1; }
cat $out/pmc.jsonl
