# config 4 (two-qubit RB) with DPEMU_X_STREAM_EVENTS on in every library: + nontemporal measurement rows (mm),
# macro-chunk DMA sc0 (sc0) or nontemporal (ntd); same-process A/B, 6 reps
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
B=ab_build/libdpemu_
timeout -k 10 400 python -u scripts/ab.py --libs ${B}base.so,${B}mm.so,${B}sc0.so,${B}ntd.so --flags 0x80,0x80,0x80,0x80 --reps 6 --workload rb2q > gpurun_out/stream2_rb2q.json 2> gpurun_out/stream2_rb2q.err
