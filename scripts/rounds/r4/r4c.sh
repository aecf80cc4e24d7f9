#!/bin/bash
# round-4 GPU bundle c: DDS mapping x occupancy x zero-tile A/B, DDS parity
out=gpurun_out/r4c
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p $out
L=ab_build/libdpemu_
libs=""
for v in S7 S7z S8 X7 X8 B7 B8 B7z B8z; do libs="$libs,${L}dds$v.so"; done
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${libs#,} > $out/ab_dds.json 2>&1 || { echo "ab_dds failed"; tail $out/ab_dds.json; exit 1; }
tail -1 $out/ab_dds.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dds.py tests/test_gpu_fullsize.py -k "dds or config5 or pipeline or synth or sweep or edges or fallback or element or channels" > $out/pytest.log 2>&1
tail -3 $out/pytest.log
