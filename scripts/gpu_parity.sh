#!/bin/bash
# interpreter + DDS GPU parity only.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/parity; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dds.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error|assert" $out/pytest.log | tail -20
exit $rc
