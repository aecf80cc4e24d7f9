#!/bin/bash
# DDS-focused GPU call: DDS parity tests, then the interleaved kernel A/B.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dds.py -m gpu -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_dds.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_dds.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_dds.py 5 10 > gpurun_out/ab_dds.log 2>&1
rc=$?; echo "ab_dds rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_dds.log | tail -30
exit $rc
