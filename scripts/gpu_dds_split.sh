#!/bin/bash
# DDS A/B per element (qdrv only, rdrv only) + seg-kernel PMC passes.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/dds_split; mkdir -p $out
for el in 0 1; do
  timeout -k 10 300 python -u scripts/ab_dds.py 3 10 128 $el > $out/ab_$el.log 2>&1 || { echo "ab $el failed"; exit 1; }
  echo "== elements $el"; grep -v amdgpu.ids $out/ab_$el.log | python3 -c "import sys,json; t=sys.stdin.read(); d=json.loads(t[t.index('{'):]); [print(k, v) for k, v in d.items()]"
done
run() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 scripts/prof_dds.py 3 > $out/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit $?
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT || exit $?
find $out -name "*kernel_stats.csv" -exec cat {} \;
python3 scripts/pmc_summary.py $out 2>/dev/null || for f in $(find $out -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in rows:
    k = r.get('Kernel_Name', '')
    if 'dds' in k:
        agg[(k[:40], r['Counter_Name'])] += float(r['Counter_Value']); disp[k[:40]].add(r['Dispatch_Id'])
for (k, c), v in sorted(agg.items()):
    print(k, c, v / max(1, len(disp[k])))
PY
done
