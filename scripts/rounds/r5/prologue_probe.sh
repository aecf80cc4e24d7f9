#!/bin/bash
# Round 5: what the tile workgroups' prologue loads cost (probe builds, outputs
# differ): no sine-table loads, no interp>=4 envelope loads, no record loads
set -o pipefail
out=gpurun_out/r5/prologue_probe
mkdir -p $out
timeout -k 10 300 python -u scripts/ab_dds.py --reps 5 \
    --libs ab_build/libdpemu_head.so,ab_build/libdpemu_nolut.so,ab_build/libdpemu_noenv4.so,ab_build/libdpemu_norec.so \
    > $out/ab_dds.json 2> $out/ab_dds.err || { tail $out/ab_dds.err; exit 1; }
cat $out/ab_dds.json
