#!/bin/bash
# Round 5: rocprofv3 kernel stats of the 12-slot staged kernel vs macro_kernel (rb8 A/B launches)
set -o pipefail
out=gpurun_out/r5/macro_wide_prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
lib=distributed_processor_amd/libdpemu.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o rb8 --output-format csv -- python3 scripts/ab.py --workload rb8 --reps 3 --steps 3 \
    --flags 0x40,0 --libs $lib,$lib > $out/ab.json 2> $out/ab.err || { tail $out/ab.err; exit 1; }
cat $out/ab.json
f=$(find $out/trace -name '*kernel_stats.csv' | head -1)
cp "$f" $out/kernel_stats.csv
cut -d, -f1-5 $out/kernel_stats.csv
