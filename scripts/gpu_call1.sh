set -o pipefail
bash scripts/valu_peak.sh gpurun_out/r03vp || exit 1
timeout -k 10 300 python scripts/ab.py --libs ab_build/libdpemu_base.so,ab_build/libdpemu_nostore.so,ab_build/libdpemu_nofetch.so,ab_build/libdpemu_both.so --workload rb --no-compare --reps 3 --steps 3 > gpurun_out/r03vp/ab_probe.json 2> gpurun_out/r03vp/ab_probe.err || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r03vp/bench.json 2> gpurun_out/r03vp/bench.err
