#!/bin/bash
# interpreter parity (all execution variants) then the interleaved A/B.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/interp_ab; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error" $out/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_interp.py 3 10 > $out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tr -d '\n' | sed 's/},/},\n/g'
exit $rc
