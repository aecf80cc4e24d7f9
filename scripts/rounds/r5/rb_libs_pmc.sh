#!/bin/bash
# Config 4: the write-path counters per library (round 4, W3, W3 + held rows):
# one rocprofv3 --pmc run per (library, counter group), per-dispatch means
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp PYTHONUNBUFFERED=1
root=gpurun_out/r5/rb_libs
mkdir -p $root
declare -A G
G[sq]="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
G[ta]="TA_FLAT_WRITE_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
G[tcc]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE"
for lib in "$@"; do
    name=$(basename $lib .so)
    for g in sq ta tcc; do
        timeout -k 10 300 rocprofv3 --pmc ${G[$g]} -d $root/${name}_$g -o pmc --output-format csv -- \
            python3 scripts/ab.py --libs $lib --workload rb --reps 2 --steps 1 \
            > $root/${name}_$g.log 2>&1 || { echo "pmc $name $g failed"; tail -5 $root/${name}_$g.log; exit 1; }
    done
done
python3 - $root "$@" <<'PY'
import csv, glob, sys, collections, json, os
root, libs = sys.argv[1], sys.argv[2:]
res = {}
for lib in libs:
    name = os.path.basename(lib)[:-3]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(root + '/' + name + '_*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'macro' in r['Kernel_Name'] and r['Counter_Name'] != 'GRBM_GUI_ACTIVE':
                acc[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
    res[name] = {k: sum(v.values()) / len(v) for k, v in sorted(acc.items())}
print(json.dumps(res, indent=1))
json.dump(res, open(root + '/summary.json', 'w'), indent=1)
PY
