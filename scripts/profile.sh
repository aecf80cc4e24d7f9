#!/bin/bash
# rocprofv3 passes over the bench (kernel trace + separate PMC passes).
# usage: scripts/profile.sh <tag> [bench args...]
tag=${1:-r01}; shift
args=${@:---steps 20 --warmup 2 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/prof_$tag
mkdir -p $out
run() {   # name, rocprofv3 options...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 bench.py $args \
        > $out/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    return $rc
}
run trace --kernel-trace --stats || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES || exit $?
run pmc_busy --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
find $out -name "*.csv" | head -50
