# dense summary rows (straight kernel): config 2 in the bench's shot-major order and core-major, config 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_base.so,ab_build/libdpemu_sumd.so
timeout -k 10 200 python -u scripts/ab.py --libs $L --workload ramsey --lane-order 1 --reps 6 > gpurun_out/sumd_ab.jsonl 2> gpurun_out/sumd_ab.err &&
timeout -k 10 200 python -u scripts/ab.py --libs $L --workload ramsey --lane-order 0 --reps 6 >> gpurun_out/sumd_ab.jsonl 2>> gpurun_out/sumd_ab.err &&
TAG=w COUNTERS="TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_WAVES" bash scripts/pmc_ab.sh ramsey straight $(echo $L | tr , ' ') > gpurun_out/sumd_pmc.jsonl 2>&1
