# the measurement draw's cost: Philox4x32-10 vs a SplitMix64 probe (outputs differ)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_base.so,ab_build/libdpemu_hash.so
: > gpurun_out/hash_ab.jsonl
for w in ar_sm "ramsey --lane-order 1" rb; do
  timeout -k 10 200 python -u scripts/ab.py --libs $L --workload $w --reps 6 --no-compare >> gpurun_out/hash_ab.jsonl 2>> gpurun_out/hash_ab.err || exit 1
done
