set -o pipefail
out=gpurun_out/r03b
mkdir -p $out
timeout -k 10 400 python scripts/ab.py --libs ab_build/libdpemu_base.so,ab_build/libdpemu_nostore.so,ab_build/libdpemu_nofetch.so,ab_build/libdpemu_both.so --workload rb --no-compare --reps 3 --steps 3 > $out/ab_probe.json 2> $out/ab_probe.err || { tail $out/ab_probe.err; exit 1; }
cat $out/ab_probe.json
