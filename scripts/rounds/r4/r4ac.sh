#!/bin/bash
# round-4 GPU bundle ac: DDS contiguous short stripes (4 / 8 / 16 tiles per workgroup) against the strided stripes
out=gpurun_out/r4ac
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${L}ddsS.so,${L}ddsC4.so,${L}ddsC8.so,${L}ddsC16.so --reps 5 > $out/ab.jsonl 2>&1 || { echo "ab failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
