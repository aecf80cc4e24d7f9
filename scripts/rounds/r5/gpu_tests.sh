#!/bin/bash
# Round 5: the full -m gpu suite on the cleaned product sources, then a DDS
# same-process A/B against the round-4 library (no variants left: I/Q identical, time unchanged)
set -o pipefail
out=gpurun_out/r5/${1:-tests}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -u scripts/ab_dds.py --reps 6 --steps 20 \
    --libs distributed_processor_amd/libdpemu.so,ab_build/libdpemu_r4.so | tee $out/dds_ab.json
# the box's PMC counter list (for the config-4 write-path pass)
timeout -k 10 120 rocprofv3 --list-avail > $out/counters.txt 2>&1 || true
