#!/bin/bash
# Round 5: store-only shapes for a one-tile-per-wave DDS (scripts/micro/dds_shape_probe.hip set w)
set -o pipefail
out=gpurun_out/r5/wave_shape
mkdir -p $out
timeout -k 10 120 ./ab_build/dds_shape_probe w > $out/shape_w.jsonl 2>&1 || { tail $out/shape_w.jsonl; exit 1; }
cat $out/shape_w.jsonl
