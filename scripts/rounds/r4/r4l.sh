#!/bin/bash
# round-4 GPU bundle l: DDS zero-fill workgroups (parity, A/B vs stripes, timeline)
out=gpurun_out/r4l
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dds.py tests/test_gpu_fullsize.py -k "dds or config5 or synth" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${L}ddsS7.so,${L}ddsZ.so,${L}ddsS7.so,${L}ddsZ.so --reps 6 > $out/ab.jsonl 2>&1 || { echo "ab failed"; tail $out/ab.jsonl; exit 1; }
tail -1 $out/ab.jsonl
timeout -k 10 200 python -u scripts/dds_timeline.py --libs ${L}ddsS7t.so,${L}ddsZt.so > $out/tl.jsonl 2>&1 || { echo "timeline failed"; tail $out/tl.jsonl; exit 1; }
cat $out/tl.jsonl
