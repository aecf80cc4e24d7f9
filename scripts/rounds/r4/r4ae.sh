#!/bin/bash
# round-4 GPU bundle ae: full -m gpu suite and smoke on the final tree
out=gpurun_out/r4ae
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
