#!/bin/bash
# Round 5: config 2's store shape, store-only, with residency capped by LDS
set -o pipefail
out=gpurun_out/r5/cfg2_shape
mkdir -p $out
timeout -k 10 120 ./ab_build/dds_shape_probe c > $out/shape_c.jsonl 2>&1 || { tail $out/shape_c.jsonl; exit 1; }
cat $out/shape_c.jsonl
