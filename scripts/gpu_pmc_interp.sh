#!/bin/bash
# PMC passes over the interpreter driver (one counter group per run).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
W=${W:-config2}
out=gpurun_out/pmc_interp_$W; mkdir -p $out
run() { local name=$1; shift
    timeout -k 10 120 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 scripts/prof_interp.py $W 3 > $out/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc; }
run trace --kernel-trace --stats || exit $?
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH || exit $?
run sq2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE || exit $?
python3 scripts/pmc_summary.py $out $W
