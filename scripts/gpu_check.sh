#!/bin/bash
# GPU-box check: parity tests, smoke, short bench.  Stops at the first crash/timeout.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$AB" ]; then timeout -k 10 300 python -u scripts/ab_interp.py 5 10 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log | grep -v amdgpu.ids; fi
exit $rc
