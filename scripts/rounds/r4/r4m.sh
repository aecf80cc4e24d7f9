#!/bin/bash
# round-4 GPU bundle m: DDS zero-fill workgroup size sweep (A/B vs stripes)
out=gpurun_out/r4m
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 400 python -u scripts/ab_dds.py --libs ${L}ddsS7.so,${L}ddsS7t8.so,${L}ddsQ1.so,${L}ddsQ1t8.so,${L}ddsQ1t4.so,${L}ddsQ1s.so,${L}ddsQ1t8s.so,${L}ddsQ1t4s.so --reps 6 > $out/ab7.jsonl 2>&1 || { echo "ab failed"; tail $out/ab7.jsonl; exit 1; }
tail -1 $out/ab7.jsonl
