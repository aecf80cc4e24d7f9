# why nontemporal event rows help the two-qubit RB programs and hurt the RB-shaped ones:
# L2 -> DRAM write requests and L1 -> L2 write latency, write-back (base) vs whole-wave nontemporal (m3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for wl in rb rb2q; do
  TAG=${wl}_ea COUNTERS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
    bash scripts/pmc_ab.sh $wl macro_staged ab_build/libdpemu_base.so ab_build/libdpemu_m3.so >> gpurun_out/stpol_pmc.jsonl || exit 1
  TAG=${wl}_wl COUNTERS="TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
    bash scripts/pmc_ab.sh $wl macro_staged ab_build/libdpemu_base.so ab_build/libdpemu_m3.so >> gpurun_out/stpol_pmc.jsonl || exit 1
done
