#!/bin/bash
# Same-box round evidence: rocprofv3 kernel trace + PMC passes over the bench,
# their per-leg summaries, then the bench line reading those summaries.
# usage (on the GPU box): bash scripts/evidence.sh gpurun_out/<dir> [tag]
# tag: the profiles/<tag>_* prefix (default: bench.py's PROFILE_TAG)
out=$1
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
tag=${2:-$(python -c "import re; print(re.search(r\"PROFILE_TAG = '(\\w+)'\", open('bench.py').read()).group(1))")}
mkdir -p $out/profiles
# (rb_shaped left out: it shares the rb leg's kernel and grid, which key the PMC summary)
bash scripts/prof_cmd.sh $out/prof bench.py --steps 8 --warmup 2 --no-cpu-baseline --legs config1,dds,active_reset,demod,lut,rb > $out/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python scripts/pmc_summary.py $out/prof $tag $out/profiles > $out/pmc_summary.log 2>&1 || { echo "pmc_summary failed"; exit 1; }
cp $(find $out/prof/trace -name "*kernel_stats.csv") $out/profiles/${tag}_kernel_stats.csv
# the raw per-dispatch CSVs are summarised now: drop them (gpurun merges back <= 64 MiB)
find $out/prof -name "*_counter_collection.csv" -delete
find $out/prof -name "*_kernel_trace.csv" -delete
# each kernel's own VALU issue peak (its opcode mix at the measured per-opcode costs)
bash scripts/kernel_mixes.sh profiles/r04_valu_peak_pmc.json $out/profiles $tag $out/profiles/${tag}_kernel_valu_peaks.json > $out/kernel_mixes.log 2>&1 || { echo "kernel_mixes failed"; tail $out/kernel_mixes.log; exit 1; }
DPEMU_BENCH_PROFILES=$out/profiles timeout -k 10 800 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
python scripts/bench_summary.py $out/bench.json
