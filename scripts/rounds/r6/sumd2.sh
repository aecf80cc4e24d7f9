# dense summary rows in the straight / branch / staged macro kernels: every bench workload, then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_base.so,ab_build/libdpemu_sumd.so
: > gpurun_out/sumd2_ab.jsonl
for w in "ramsey --lane-order 1" ar_sm lut_sm demod_sm rb; do
  timeout -k 10 200 python -u scripts/ab.py --libs $L --workload $w --reps 6 >> gpurun_out/sumd2_ab.jsonl 2>> gpurun_out/sumd2_ab.err || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sumd2_gpu.log 2>&1
