#!/bin/bash
# round-4 GPU bundle x: DDS stripes with XCD-contiguous channel regions (A/B)
out=gpurun_out/r4x
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${L}ddsS.so,${L}ddsR.so,${L}ddsS.so,${L}ddsR.so --reps 6 > $out/ab.jsonl 2>&1 || { echo "ab failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
