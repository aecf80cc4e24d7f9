#!/bin/bash
# GPU parity (all -m gpu tests) then the store-pattern microbenchmark.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/store; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error|assert" $out/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 scripts/micro/store_probe > $out/store.jsonl 2>&1; rc=$?; echo "probe rc=$rc"; cat $out/store.jsonl
exit $rc
