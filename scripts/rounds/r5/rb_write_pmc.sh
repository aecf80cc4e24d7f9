#!/bin/bash
# Config 4's write path: PMC passes over the config-4
# launch with and without event stores (dpemu_outputs.events null), so the
# counters that follow the ~1.1 ms the stores add show which unit holds the
# waves.  One counter group per rocprofv3 run (block limits: 2 TA, 4 TCP, 4 TCC).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp PYTHONUNBUFFERED=1
root=gpurun_out/r5/rb_write
mkdir -p $root
L=distributed_processor_amd/libdpemu.so
declare -A G
G[sq]="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
G[ta]="TA_FLAT_WRITE_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
G[ta2]="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
G[tcc]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE"
G[tcc2]="TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_WRITE_SECTORS_sum GRBM_GUI_ACTIVE"
for outs in summary,events,meas,hist summary,meas,hist; do
    tag=$([ $outs = summary,meas,hist ] && echo noev || echo ev)
    timeout -k 10 300 python -u scripts/ab.py --libs $L --workload rb --reps 2 --steps 3 --outputs $outs \
        > $root/time_$tag.json 2>&1 || { echo "timing $tag failed"; tail $root/time_$tag.json; exit 1; }
    cat $root/time_$tag.json | tail -1
    for g in sq ta ta2 tcc tcc2; do
        timeout -k 10 300 rocprofv3 --pmc ${G[$g]} -d $root/${tag}_$g -o pmc --output-format csv -- \
            python3 scripts/ab.py --libs $L --workload rb --reps 2 --steps 1 --outputs $outs \
            > $root/${tag}_$g.log 2>&1 || { echo "pmc $tag $g failed"; tail -5 $root/${tag}_$g.log; exit 1; }
    done
done
python3 - $root <<'PY'
import csv, glob, sys, collections, json
root = sys.argv[1]
res = {}
for tag in ('ev', 'noev'):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(root + '/' + tag + '_*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'macro' in r['Kernel_Name']:
                acc[r['Counter_Name'] + ('' if r['Counter_Name'] != 'GRBM_GUI_ACTIVE' else '@' + f.split('/')[-4])][r['Dispatch_Id']] += float(r['Counter_Value'])
    res[tag] = {k: sum(v.values()) / len(v) for k, v in sorted(acc.items())}
print(json.dumps(res, indent=1))
json.dump(res, open(root + '/summary.json', 'w'), indent=1)
PY
# the whole-row ceiling: round 4's probe build storing every record at slot =
# macro iteration (outputs differ; timing only), against round 4 and this tree
timeout -k 10 300 python -u scripts/ab.py --libs $L,ab_build/libdpemu_r4.so,ab_build/libdpemu_r4iterslot.so \
    --workload rb --reps 4 --steps 3 --no-compare > $root/iterslot_ab.json 2>&1 || { echo "iterslot ab failed"; tail $root/iterslot_ab.json; exit 1; }
tail -1 $root/iterslot_ab.json
