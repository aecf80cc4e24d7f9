# config 3 in the bench's shot-major order: whole-wave nontemporal event rows in branch_kernel (b3) on the
# STATE, DEMOD and LUT launches; same-process A/B, 6 reps
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_base.so,ab_build/libdpemu_b3.so
for wl in ar_sm demod_sm lut_sm; do
  timeout -k 10 200 python -u scripts/ab.py --libs $L --reps 6 --workload $wl >> gpurun_out/branch_wave_nt.jsonl 2> gpurun_out/branch_wave_nt_$wl.err || exit 1
done
