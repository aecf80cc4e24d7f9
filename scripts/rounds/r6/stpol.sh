# record-store cache policy (lane.h StPolicy): macro_staged_kernel on config 4 (both RB workloads),
# branch_kernel on config 3 (shot-major = the bench's order, core-major); same-process A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
B=ab_build/libdpemu_
M=${B}base.so,${B}m1.so,${B}m2.so,${B}m3.so
R=${B}base.so,${B}b2.so,${B}b3.so
timeout -k 10 300 python -u scripts/ab.py --libs $M --workload rb2q > gpurun_out/stpol_rb2q.json 2> gpurun_out/stpol_rb2q.err &&
timeout -k 10 300 python -u scripts/ab.py --libs $M --workload rb > gpurun_out/stpol_rb.json 2> gpurun_out/stpol_rb.err &&
timeout -k 10 300 python -u scripts/ab.py --libs $R --workload ar_sm > gpurun_out/stpol_ar_sm.json 2> gpurun_out/stpol_ar_sm.err &&
timeout -k 10 300 python -u scripts/ab.py --libs $R --workload ar > gpurun_out/stpol_ar.json 2> gpurun_out/stpol_ar.err
