# config 4: nontemporal event / measurement stores in macro_staged_kernel, same-process A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
L=ab_build/libdpemu_base.so,ab_build/libdpemu_nt1.so,ab_build/libdpemu_nt3.so
timeout -k 10 300 python -u scripts/ab.py --libs $L --workload rb2q > gpurun_out/macro_nt_rb2q.json 2> gpurun_out/macro_nt_rb2q.err &&
timeout -k 10 300 python -u scripts/ab.py --libs $L --workload rb > gpurun_out/macro_nt_rb.json 2> gpurun_out/macro_nt_rb.err
