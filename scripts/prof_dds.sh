#!/bin/bash
# rocprofv3 passes over the DDS driver: trace + PMC passes (one counter group per run).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
tag=${1:-dds}; shift
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 120 python3 scripts/prof_dds.py 3 128 4096 > $out/prologue.log 2>&1; echo "prologue rc=$?"; grep dds $out/prologue.log
run() {
    local name=$1; shift
    timeout -k 10 180 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 scripts/prof_dds.py 3 > $out/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit $?
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
run pmc_sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
find $out -name "*stats.csv" -exec cat {} \;
for f in $(find $out -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if 'dds_kernel' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    print(k, 'per-dispatch mean', sum(v) / max(1, len(set(r['Dispatch_Id'] for r in rows if 'dds_kernel' in r.get('Kernel_Name', '')))))
PY
done
