# config 4 staged kernel after the fast-path cut: time, VALU, waits; parity of macro tests
set -o pipefail
out=gpurun_out/r03f
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rb.py tests/test_gpu_parity.py -k "linear or rb or config4 or few_registers" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 200 python scripts/rb_probe.py --steps 3 > $out/probe_staged.json 2>&1 || exit 1
timeout -k 10 200 python scripts/rb_probe.py --steps 3 --outputs summary,meas,hist > $out/probe_staged_noev.json 2>&1 || exit 1
grep -h kernel_ms $out/probe_*.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $out/sq -o sq --output-format csv -- python3 scripts/rb_probe.py --steps 2 > $out/sq.log 2>&1 || { tail $out/sq.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
d = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/r03f/sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'macro' in r['Kernel_Name']:
            d[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in d.items():
    print(k, {a: '%.4g' % b for a, b in v.items()}, 'wait/wave', v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES'])
PY
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k lut > $out/pytest_lut.log 2>&1 || { tail -30 $out/pytest_lut.log; exit 1; }
tail -2 $out/pytest_lut.log
timeout -k 10 600 python bench.py --legs active_reset,lut --no-cpu-baseline > $out/bench_lut.json 2> $out/bench_lut.err || { tail $out/bench_lut.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench_lut.json'))
for k in ('active_reset','lut'): print(k, d[k]['kernel'], d[k]['ms_per_step'], d[k]['roofline']['kernel_ms'])"
