#!/bin/bash
# round-4 GPU bundle t: DDS parity after the index-kernel LDS change
out=gpurun_out/r4t
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dds.py tests/test_gpu_fullsize.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
