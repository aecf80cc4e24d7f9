#!/bin/bash
# Round 5: write-request counters of the store-only shapes (dds_shape_probe
# set w): do the fast (fill) and slow (stripes, tiles per wave) shapes differ
# in request size or DRAM stalls?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/r5/shape_pmc
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
    -d $out/p1 -o p1 --output-format csv -- ./ab_build/dds_shape_probe w > $out/p1.log 2>&1 || { tail $out/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE \
    -d $out/p2 -o p2 --output-format csv -- ./ab_build/dds_shape_probe w > $out/p2.log 2>&1 || { tail $out/p2.log; exit 1; }
python3 - $out <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'].split('(')[0]][r['Counter_Name']][f + r['Dispatch_Id']] += float(r['Counter_Value'])
res = {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
json.dump(res, open(out + '/summary.json', 'w'), indent=1)
for k, v in res.items():
    print(k[:40], {c[:22]: '%.3g' % x for c, x in v.items()})
PY
