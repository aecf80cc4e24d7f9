#!/bin/bash
# Round evidence on one GPU box: full -m gpu suite, smoke, then the same-box
# rocprofv3 + PMC passes and the bench line (scripts/evidence.sh).
# usage (on the box): bash scripts/gpu_round.sh gpurun_out/<dir> [tag]
set -o pipefail
out=$1
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
# the box's clocks (boxes differ; config 4 by up to ~18 %)
timeout -k 5 30 rocm-smi --showclocks > $out/clocks.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash scripts/evidence.sh $out $2 || exit 1
