#!/bin/bash
# round-4 GPU bundle f: DDS channel dispatch order grouped by element (A/B + timelines)
out=gpurun_out/r4f
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
libs=""
for v in S7 Se Xe Be X7; do libs="$libs,${L}dds$v.so"; done
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${libs#,} > $out/ab_dds.json 2>&1 || { echo "ab_dds failed"; tail $out/ab_dds.json; exit 1; }
tail -1 $out/ab_dds.json
timeout -k 10 300 python -u scripts/dds_timeline.py --libs ${L}ddsSet.so,${L}ddsXet.so > $out/timeline.jsonl 2>&1 || { echo "timeline failed"; tail $out/timeline.jsonl; exit 1; }
tail -2 $out/timeline.jsonl
