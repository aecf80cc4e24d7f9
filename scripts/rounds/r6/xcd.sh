# config 4: XCD-contiguous workgroup order in the staged macro kernel (probe) vs the product
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_base.so,ab_build/libdpemu_xcd.so
timeout -k 10 300 python -u scripts/ab.py --libs $L --workload rb --reps 6 > gpurun_out/xcd_ab.jsonl 2> gpurun_out/xcd_ab.err &&
timeout -k 10 300 python -u scripts/ab.py --libs $L --workload rb8 --reps 4 >> gpurun_out/xcd_ab.jsonl 2>> gpurun_out/xcd_ab.err &&
TAG=x COUNTERS="FETCH_SIZE" bash scripts/pmc_ab.sh rb macro_staged $(echo $L | tr , ' ') > gpurun_out/xcd_pmc.jsonl 2>&1 &&
TAG=y COUNTERS="TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" bash scripts/pmc_ab.sh rb macro_staged $(echo $L | tr , ' ') >> gpurun_out/xcd_pmc.jsonl 2>&1
