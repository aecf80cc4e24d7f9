#!/bin/bash
# DDS GPU parity, then the config-5 A/B (event index variants).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/dds_idx; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dds.py -x -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error|mismatch" $out/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_dds.py 3 10 > $out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tr -d '\n '
exit $rc
