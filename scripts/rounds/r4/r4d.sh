#!/bin/bash
# round-4 GPU bundle d: DDS dispatch-order A/B, then a quick bench line
out=gpurun_out/r4d
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
libs=""
for v in S7 Sw St Sc X7; do libs="$libs,${L}dds$v.so"; done
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${libs#,} > $out/ab_dds.json 2>&1 || { echo "ab_dds failed"; tail $out/ab_dds.json; exit 1; }
tail -1 $out/ab_dds.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 1; }
tail -c 2000 $out/bench.json
