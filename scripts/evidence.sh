#!/bin/bash
# Same-box round evidence: rocprofv3 kernel trace + PMC passes over the bench,
# their per-leg summaries, then the bench line reading those summaries.
# usage (on the GPU box): bash scripts/evidence.sh gpurun_out/<dir>
out=$1
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out/profiles
bash scripts/prof_cmd.sh $out/prof bench.py --steps 20 --no-cpu-baseline > $out/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/pmc_summary.py $out/prof r03 $out/profiles > $out/pmc_summary.log 2>&1 || { echo "pmc_summary failed"; exit 1; }
cp $(find $out/prof/trace -name "*kernel_stats.csv") $out/profiles/r03_kernel_stats.csv
DPEMU_BENCH_PROFILES=$out/profiles timeout -k 10 800 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
python scripts/bench_summary.py $out/bench.json
