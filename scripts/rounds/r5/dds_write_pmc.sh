#!/bin/bash
# Config 5: the write-path counters of dds_tile_kernel and of a plain fill of
# the same I/Q buffer (torch fill_, the store ceiling), one rocprofv3 --pmc
# run per counter group over scripts/ab_dds.py
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp PYTHONUNBUFFERED=1
root=gpurun_out/r5/dds_write
mkdir -p $root
L=distributed_processor_amd/libdpemu.so
declare -A G
G[sq]="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
G[ta]="TA_FLAT_WRITE_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
G[tcc]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE"
for g in sq ta tcc; do
    timeout -k 10 300 rocprofv3 --pmc ${G[$g]} -d $root/$g -o pmc --output-format csv -- \
        python3 scripts/ab_dds.py --libs $L --reps 2 --steps 2 > $root/$g.log 2>&1 || { echo "pmc $g failed"; tail -5 $root/$g.log; exit 1; }
done
python3 - $root <<'PY'
import csv, glob, sys, collections, json
root = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(root + '/*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']
        key = 'dds_tile' if 'dds_tile' in n else 'dds_index' if 'dds_index' in n else 'fill' if ('fill' in n or 'elementwise' in n) else None
        if key and r['Counter_Name'] != 'GRBM_GUI_ACTIVE':
            res[key][r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
out = {k: {c: sum(v.values()) / len(v) for c, v in sorted(d.items())} for k, d in res.items()}
print(json.dumps(out, indent=1))
json.dump(out, open(root + '/summary.json', 'w'), indent=1)
PY
