# WRITE_SIZE (rocprofv3 --pmc) and an interleaved timing A/B of two A/B builds on config 3
# (direct: the kernel storing each record as emitted, the commit before the row flush; rows: profiles/r02_ar_rows_ab.json)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
for name in direct rows; do
  out=gpurun_out/wr/$name; mkdir -p $out
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out -o w --output-format csv -- python3 scripts/ab.py --libs ab_build/libdpemu_$name.so --workload ar_sm --reps 2 --steps 2 > $out/log 2>&1 || { echo "$name pmc failed"; exit 1; }
done
timeout -k 10 300 python scripts/ab.py --libs ab_build/libdpemu_direct.so,ab_build/libdpemu_rows.so --workload ar_sm --reps 25 --steps 10 > gpurun_out/wr/ab_long.json 2> gpurun_out/wr/ab_long.err
