#!/bin/bash
# DDS A/B incl. segment-kernel probes, full config 5 and per element.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
out=gpurun_out/dds_probe; mkdir -p $out
for el in 01 0 1; do
  timeout -k 10 300 python -u scripts/ab_dds.py 3 10 128 $el > $out/ab_$el.log 2>&1 || { echo "ab $el failed"; tail -5 $out/ab_$el.log; exit 1; }
  echo "== elements $el"; grep -v amdgpu.ids $out/ab_$el.log | python3 -c "import sys,json; t=sys.stdin.read(); d=json.loads(t[t.index('{'):]); [print(k, v) for k, v in d.items()]"
done
