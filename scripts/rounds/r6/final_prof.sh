# final-tree evidence, part 1: rocprofv3 kernel trace + PMC passes of the bench and their summaries
# (part 2 is the bench line reading them from profiles/: scripts/evidence.sh split in two calls)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/r6e; tag=r06
mkdir -p $out/profiles
bash scripts/prof_cmd.sh $out/prof bench.py --steps 8 --warmup 2 --no-cpu-baseline --legs config1,dds,active_reset,demod,lut,rb > $out/prof.log 2>&1 || { echo "prof failed"; tail $out/prof.log; exit 1; }
python scripts/pmc_summary.py $out/prof $tag $out/profiles > $out/pmc_summary.log 2>&1 || { echo "pmc_summary failed"; exit 1; }
cp $(find $out/prof/trace -name "*kernel_stats.csv") $out/profiles/${tag}_kernel_stats.csv
find $out/prof -name "*_counter_collection.csv" -delete
find $out/prof -name "*_kernel_trace.csv" -delete
bash scripts/kernel_mixes.sh profiles/r04_valu_peak_pmc.json $out/profiles $tag $out/profiles/${tag}_kernel_valu_peaks.json > $out/kernel_mixes.log 2>&1 || { echo "kernel_mixes failed"; tail $out/kernel_mixes.log; exit 1; }
ls $out/profiles
