#!/bin/bash
# PMC counts of one kernel per A/B library: for each lib, rocprofv3 --pmc over
# scripts/ab.py on one workload, then the per-dispatch mean of each counter.
#   scripts/pmc_ab.sh <workload (scripts/ab.py's, or dds: scripts/ab_dds.py)> <kernel substring> <lib> [lib ...]
# Counters: $COUNTERS, default SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
wl=$1; kern=$2; shift 2
for lib in "$@"; do
    name=$(basename $lib .so)
    out=gpurun_out/pmc_ab/$name${TAG:+_$TAG}
    mkdir -p $out
    timeout -k 10 120 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR \
        SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU} -d $out -o pmc --output-format csv -- \
        python3 $([ "$wl" = dds ] && echo "scripts/ab_dds.py --libs $lib --reps 2 --steps 2" \
                               || echo "scripts/ab.py --libs $lib --workload $wl --reps 2 --steps 2") \
        > $out/log 2>&1 || { echo "$name failed"; exit 1; }
    python3 - "$out" "$kern" "$name" <<'PY'
import csv, glob, sys, collections, json
out, kern, name = sys.argv[1:4]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name']:
            acc[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
res = {k: sum(v.values()) / len(v) for k, v in acc.items()}
if res.get('SQ_WAVES') and 'SQ_INSTS_VALU' in res:
    res['valu_per_wave'] = res['SQ_INSTS_VALU'] / res['SQ_WAVES']
    res['salu_per_wave'] = res['SQ_INSTS_SALU'] / res['SQ_WAVES']
print(json.dumps({'lib': name, **{k: round(v, 1) for k, v in res.items()}}))
PY
done
