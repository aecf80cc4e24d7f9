#!/bin/bash
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/dds_ab; mkdir -p $out
timeout -k 10 300 python -u scripts/ab_dds.py 3 10 > $out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tr -d '\n' | sed 's/},/},\n/g'
exit $rc
