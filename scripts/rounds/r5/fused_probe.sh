#!/bin/bash
# Round 5: where the fused DDS launch loses (probe builds: no release fence,
# no wait), and the branch kernel's VALU / SALU per wave, HEAD vs row holding.
set -o pipefail
out=gpurun_out/r5/fused_probe
mkdir -p $out
timeout -k 10 240 python -u scripts/ab_dds.py --reps 5 \
    --libs ab_build/libdpemu_head.so,ab_build/libdpemu_fused.so,ab_build/libdpemu_nofence.so,ab_build/libdpemu_nowait.so \
    > $out/ab_dds.json 2> $out/ab_dds.err || { tail $out/ab_dds.err; exit 1; }
cat $out/ab_dds.json
timeout -k 10 300 bash scripts/pmc_ab.sh ar branch_kernel ab_build/libdpemu_head.so ab_build/libdpemu_fused.so \
    > $out/pmc_ar.jsonl 2>&1 || { tail $out/pmc_ar.jsonl; exit 1; }
cat $out/pmc_ar.jsonl
