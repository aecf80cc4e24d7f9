# config 4: the product event layout vs a wave-blocked probe layout (a wave's records contiguous)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 python -u scripts/ab.py --libs ab_build/libdpemu_base.so,ab_build/libdpemu_wblk.so --workload rb --no-compare > gpurun_out/wblk_ab.json 2> gpurun_out/wblk_ab.err &&
TAG=w COUNTERS="TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum SQ_WAVES" bash scripts/pmc_ab.sh rb macro_staged ab_build/libdpemu_base.so ab_build/libdpemu_wblk.so > gpurun_out/wblk_pmc.jsonl 2>&1
