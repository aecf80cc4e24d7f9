#!/bin/bash
# round-4 GPU bundle b: DDS diagnostics (A/B + PMC), targeted parity tests, VALU opcode peaks
out=gpurun_out/r4b
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p $out
L=ab_build/libdpemu_
timeout -k 10 300 python -u scripts/ab_dds.py --libs ${L}ddsS.so,${L}ddsX1.so,${L}ddsSn.so,${L}ddsX1n.so,${L}ddsSp.so,${L}ddsX1p.so > $out/ab_dds.json 2>&1 || { echo "ab_dds failed"; tail $out/ab_dds.json; exit 1; }
tail -1 $out/ab_dds.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ref_binding.py tests/test_gpu_dds.py tests/test_gpu_fullsize.py tests/test_gpu_rb.py > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/prof_cmd.sh $out/prof scripts/ab_dds.py --libs ${L}ddsS.so,${L}ddsX1.so --reps 2 --steps 5 > $out/prof.log 2>&1 || { echo "prof failed"; tail $out/prof.log; exit 1; }
python scripts/pmc_summary.py $out/prof r04 $out/pmc "ddsS=dds_tile_kernel@6815744,ddsX1=dds_tile_kernel@4194304" > $out/pmc_summary.log 2>&1
tail -3 $out/pmc_summary.log
bash scripts/valu_peak.sh $out/valu > $out/valu.log 2>&1 || { echo "valu failed"; tail $out/valu.log; exit 1; }
tail -3 $out/valu.log
