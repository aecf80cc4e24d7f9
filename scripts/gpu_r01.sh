#!/bin/bash
# Round-1 GPU evidence: parity tests, smoke, bench, then rocprofv3 kernel trace
# and separate PMC passes over a short bench run.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/r01
mkdir -p $out
step() {   # name, timeout, command...
    local name=$1 lim=$2; shift 2
    timeout -k 10 $lim "$@" > $out/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    return $rc
}
if [ -z "$SKIP_TESTS" ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit $?
    grep -E "passed|failed" $out/pytest_gpu.log | tail -3
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
step bench 400 python -u bench.py || exit $?
grep '^{' $out/bench.log
B="--steps 10 --warmup 2 --no-cpu-baseline"
prof() {   # name, rocprofv3 options...
    local name=$1; shift
    step prof_$name 240 rocprofv3 "$@" -d $out/prof_$name -o $name --output-format csv -- python3 bench.py $B
}
prof trace --kernel-trace --stats || exit $?
find $out/prof_trace -name "*kernel_stats.csv" -exec cat {} \;
prof fetch --pmc FETCH_SIZE || exit $?
prof write --pmc WRITE_SIZE || exit $?
prof sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU || exit $?
prof sq2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE || exit $?
timeout -k 10 60 rocprofv3 -L > $out/counters_avail.txt 2>&1; echo "list rc=$?"
[ -x scripts/micro/valu_peak ] && { step valu_peak 120 scripts/micro/valu_peak || exit $?; }
python3 scripts/pmc_summary.py $out r01 || exit $?
