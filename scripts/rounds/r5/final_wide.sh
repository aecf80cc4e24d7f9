#!/bin/bash
# Round 5, last tree: the full -m gpu suite, smoke(), and the default bench line
set -o pipefail
out=gpurun_out/r5/final_wide
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 600 $out/bench.json
