#!/bin/bash
# Round 5: dds_index_kernel variants against HEAD (libdpemu_head.so):
# (ix2: chunks over the waves + forward scan; cnt: per-channel counts, windows found in the tile workgroups; pair: one workgroup per two channels of a lane):
# step A/B, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/r5/index_pair
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dds.py tests/test_gpu_fullsize.py \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 240 python -u scripts/ab_dds.py --libs ab_build/libdpemu_head.so,ab_build/libdpemu_pair.so --reps 7 \
    > $out/ab_dds.json 2> $out/ab_dds.err || { tail $out/ab_dds.err; exit 1; }
cat $out/ab_dds.json
for lib in pair; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/$lib -o prof --output-format csv -- \
      python3 scripts/ab_dds.py --libs ab_build/libdpemu_$lib.so --reps 3 --steps 10 > $out/$lib.log 2>&1 || { tail $out/$lib.log; exit 1; }
  echo "== $lib"; grep -i dds $(find $out/$lib -name '*kernel_stats.csv' | head -1) | cut -d, -f1-8
done
