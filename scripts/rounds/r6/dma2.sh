set -o pipefail
timeout -k 10 300 python -u scripts/ab.py --libs ab_build/libdpemu_base.so,ab_build/libdpemu_dma2.so --workload rb  > gpurun_out/dma2_ab.json 2> gpurun_out/dma2_ab.err &&
TAG=w COUNTERS="TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" bash scripts/pmc_ab.sh rb macro_staged ab_build/libdpemu_base.so ab_build/libdpemu_dma2.so > gpurun_out/dma2_pmc.jsonl 2>&1
