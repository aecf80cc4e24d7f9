#!/bin/bash
# Round 5: macro_kernel with the ALU-slot loop rolled (fix) vs before the 3-slot macros (prew3) vs HEAD
set -o pipefail
out=gpurun_out/r5/macro_direct_fix
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rb.py tests/test_gpu_parity.py \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 400 python -u scripts/ab.py --workload rb --reps 3 --steps 2 --flags 0x40,0x40,0x40,0,0 \
    --libs ab_build/libdpemu_prew3.so,ab_build/libdpemu_head.so,ab_build/libdpemu_fix.so,ab_build/libdpemu_head.so,ab_build/libdpemu_fix.so \
    > $out/ab_rb.json 2> $out/ab_rb.err || { tail $out/ab_rb.err; exit 1; }
cat $out/ab_rb.json
