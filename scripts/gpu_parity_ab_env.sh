#!/bin/bash
# interpreter parity, then the environment-knob A/B.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/ab_env; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error" $out/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_env.py 3 10 > $out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -20
exit $rc
