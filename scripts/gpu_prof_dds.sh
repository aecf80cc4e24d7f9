#!/bin/bash
# rocprofv3 kernel trace of the config-5 DDS driver (default path), per-kernel stats.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/prof_dds_${TAG:-x}; mkdir -p $out
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 scripts/prof_dds.py 5 > $out/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; grep dds $out/trace.log | tail -3
find $out -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
