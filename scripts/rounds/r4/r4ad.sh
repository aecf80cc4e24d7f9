#!/bin/bash
# round-4 GPU bundle ad: DDS persistent tile workgroups over 2 / 4 / 8 / 16-tile items (A/B, I/Q must match)
out=gpurun_out/r4ad
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${L}ddsS.so,${L}ddsP4.so,${L}ddsP8.so,${L}ddsP16.so --reps 5 > $out/ab3.jsonl 2>&1 || { echo "ab failed"; tail $out/ab3.jsonl; exit 1; }
tail -1 $out/ab3.jsonl
