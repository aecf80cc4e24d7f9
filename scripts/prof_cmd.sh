#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes over any python command.
# usage: scripts/prof_cmd.sh <out dir under gpurun_out> <python args...>
# e.g.   scripts/prof_cmd.sh gpurun_out/rb scripts/rb_probe.py --steps 3
# Each pass runs under its own time limit; the script stops at the first failure.
out=$1; shift
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p $out
run() {   # name, limit, rocprofv3 options...
    local name=$1 lim=$2; shift 2
    timeout -k 10 $lim rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 "${ARGS[@]}" \
        > $out/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    return $rc
}
ARGS=("$@")
run trace 300 --kernel-trace --stats || exit $?
run fetch 300 --pmc FETCH_SIZE || exit $?
run write 300 --pmc WRITE_SIZE || exit $?
run sq1 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE || exit $?
run sq2 300 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit $?
# the VALU stream's 32- / 64-bit integer split (the kernels' own VALU peak, scripts/kernel_valu_peak.py)
run sq3 300 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 GRBM_GUI_ACTIVE || exit $?
# the write path (TA -> TCP -> TCC -> EA): which unit holds a store-heavy
# kernel's waves (block limits: 2 TA, 4 TCP, 4 TCC counters per pass)
run wpath 300 --pmc TA_FLAT_WRITE_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE || exit $?
run wtcc 300 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE || exit $?
find $out/trace -name "*kernel_stats.csv" -exec cat {} \;
