#!/bin/bash
# DDS parity (all paths) then the interleaved path A/B.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/dds_ab; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dds.py -v --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|Error" $out/pytest.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_dds.py 3 10 > $out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log
exit $rc
