#!/bin/bash
# round-4 GPU bundle h: config-3 direct event stores (A/B, both lane orders + LUT), DDS records read from the index (A/B)
out=gpurun_out/r4h
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
for w in ar_sm lut_sm ar; do
    timeout -k 10 240 python -u scripts/ab.py --libs ${L}br0.so,${L}br1.so --workload $w > $out/ab_br_$w.json 2>&1 || { echo "ab $w failed"; tail $out/ab_br_$w.json; exit 1; }
    tail -1 $out/ab_br_$w.json
done
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${L}ddsS7.so,${L}ddsG.so > $out/ab_dds.json 2>&1 || { echo "ab_dds failed"; tail $out/ab_dds.json; exit 1; }
tail -1 $out/ab_dds.json
