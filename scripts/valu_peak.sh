#!/bin/bash
# VALU-peak evidence (on the GPU box): kernel trace + one PMC pass over
# scripts/micro/valu_peak (built beforehand in-tree), then the summary.
# usage: bash scripts/valu_peak.sh gpurun_out/<dir>
out=$1
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv \
    -- ./scripts/micro/valu_peak > $out/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $out/pmc -o pmc --output-format csv -- ./scripts/micro/valu_peak > $out/pmc.log 2>&1 || { echo "pmc pass failed"; exit 1; }
python3 scripts/valu_peak_summary.py $out $out/valu_peak_pmc.json
