#!/bin/bash
# One GPU-box round: parity tests, smoke, bench, interleaved A/B, rocprof
# kernel trace of the bench.  Stops at the first crash / timeout.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash scripts/gpu_check.sh || exit $?
if [ -n "$PROF" ]; then
    export TMPDIR=/tmp
    mkdir -p gpurun_out/prof_$PROF
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$PROF/trace -o trace --output-format csv \
        -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$PROF/trace.log 2>&1
    rc=$?; echo "prof rc=$rc"
    find gpurun_out/prof_$PROF -name "*kernel_stats.csv" -exec cat {} \;
    exit $rc
fi
