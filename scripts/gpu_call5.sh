# config 4: staged macro kernel PMC passes; event-store share (no event output) for both macro kernels
set -o pipefail
out=gpurun_out/r03e
mkdir -p $out
timeout -k 10 200 python scripts/rb_probe.py --steps 3 > $out/probe_staged.json 2>&1 || exit 1
timeout -k 10 200 python scripts/rb_probe.py --steps 3 --outputs summary,meas,hist > $out/probe_staged_noev.json 2>&1 || exit 1
timeout -k 10 200 python scripts/rb_probe.py --steps 3 --flags 64 --outputs summary,meas,hist > $out/probe_direct_noev.json 2>&1 || exit 1
cat $out/probe_*.json
bash scripts/prof_cmd.sh $out/prof scripts/rb_probe.py --steps 2 > $out/prof.log 2>&1 || { tail $out/prof.log; exit 1; }
python scripts/pmc_summary.py $out/prof r03 $out/sum rb=macro_staged_kernel > $out/sum.log 2>&1 || { cat $out/sum.log; exit 1; }
cat $out/sum.log
