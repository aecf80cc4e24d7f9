#!/bin/bash
# Round 5: where dds_index_kernel's ~15 us go -- rocprofv3 kernel stats of the
# product library and two probe builds (no event loads / no tile windows).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/r5/index_probe
mkdir -p $out
for lib in head ix_noload ix_nowin; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/$lib -o prof --output-format csv -- \
      python3 scripts/ab_dds.py --libs ab_build/libdpemu_$lib.so --reps 3 --steps 10 > $out/$lib.log 2>&1 || { tail $out/$lib.log; exit 1; }
  f=$(find $out/$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; grep -i dds "$f" | cut -d, -f1-8
done
