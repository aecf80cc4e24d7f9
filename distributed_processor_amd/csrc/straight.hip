// straight.hip -- the interpreter for pulse-only programs on CDNA4 (gfx950).
//
// A program whose commands are all pulse writes / pulse triggers / idles /
// done / hung opcodes (no ALU, jump, fproc or sync: op4 outside 1..7) never
// writes the register file and never moves its instruction pointer except by
// +1 (hdl/instr_ptr.v with no jump), and its qclk is never reloaded
// (hdl/qclk.v: only ALU-class commands load it).  So every lane still running
// in loop iteration k is executing command k of its program: the command
// index is wave-uniform, the fetch address is k * stride (SALU) + program
// (one VALU add), and the per-lane ip / qclk-anchor / mode state of the
// general interpreter (interp.hip) disappears.  Timing is ctrl.v's closed
// form for pulse-class commands with qclk = cycle - 1 (qclk.v after the
// two-cycle reset hold); the first command is peeled to model the hold
// (cmd_time 0 there strobes twice, oracle/fast_model.c).
//
// Outputs and their layout are identical to interp_kernel's; the launcher
// (capi.cpp) picks this kernel for pulse-only program sets whose longest
// program is shorter than the 2^16-deep cmd_mem (so ip never wraps).
//
// Commands come from the command-major image (STRAIGHT_ROWS: command k of
// program p at fetch[k * n_programs + p], with a zero = DONE row past the
// longest program, so every lane alive in iteration k <= its length reads in
// bounds), the program-major one (STRAIGHT_PROG: offsets[p] + k, guarded by
// k < length) or the workgroup's programs staged in LDS (STRAIGHT_LDS, for
// long programs on grids too small to hide global-memory latency: an LDS
// fetch does not wait for the lane's earlier event stores, which share
// vmcnt with global loads).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lane.h"

namespace dpemu {

template <int SRC>
__global__ void __launch_bounds__(BLOCK) straight_kernel(const KParams p)
{
    constexpr bool ROWS = SRC == STRAIGHT_ROWS, LDS = SRC == STRAIGHT_LDS;
    __shared__ uint32_t s_hist[HIST_LDS_MAX];
    __shared__ uint32_t s_pref[LDS ? BLOCK + 1 : 1];
    __shared__ uint32_t s_scan[BLOCK / 64];
    extern __shared__ uint4 s_prog[];
    const uint32_t tid = threadIdx.x;
    const uint32_t C = p.C;
    const uint32_t pos = blockIdx.x * BLOCK + tid;
    const bool valid = pos < p.n_lanes;
    const uint32_t core = pos & (C - 1);
    const uint32_t lane = (shot_of_pos(p, pos >> p.log2C) << p.log2C) | core;   // output lane index
    const uint64_t shot = p.shot_begin + (lane >> p.log2C);
    const uint32_t n_lanes = p.n_lanes;

    uint32_t grp = 0, prog = 0, base = 0, nprog = 0;
    if (valid) {
        grp = lane_group(p, lane);
        prog = p.prog_table[(uint64_t)grp * C + core];
        nprog = p.n_instr[prog];
        if (!ROWS) base = p.offsets[prog];
    }
    const uint32_t thr = valid ? p.p1_thr[core] : 0u;
    if (p.hist_lds) {
        for (uint32_t i = tid; i < HIST_LDS_MAX; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
    }
    if constexpr (LDS) base = stage_programs(p, s_prog, s_pref, s_scan, pos >> p.log2C);

    const uint32_t max_cycles = p.max_cycles;
    uint32_t t = 0, pe = 0, pp = 0, pa = 0;            // next DECODE cycle; pulse register image
    uint32_t flags = 0, n_ev = 0, n_meas = 0, meas_bits = 0, last_bit = 0;
    // st: 0 while running, else the finish status (| ST_TOP: stopped by the
    // max_cycles check before a fetch, so that command did not retire); k_end:
    // the command index at the finish.  A finish leaves t alone: t_end = t
    constexpr uint32_t ST_TOP = 0x100u;
    uint32_t st = valid ? 0u : ST_DONE, k_end = 0;

    // State updates below are selects, not branches: a divergent branch that
    // writes loop-carried state makes the register allocator copy that state
    // around it on every iteration.  Branches guard only stores and philox.
    //
    // pulse_iface strobe at cycle te, qclk q (kind 0: trigger, 1: phase reset)
    // with the current pulse registers, for lanes with `ok`; readout-element
    // triggers draw the measurement.  Overflow flags are derived from the
    // final counts (an event / measurement is dropped iff its count exceeds
    // the cap)
    auto emit = [&](bool ok, uint32_t te, uint32_t q, uint32_t kind) {
        if (ok && n_ev < p.event_cap) {
            const uint64_t slot = (uint64_t)n_ev * n_lanes + lane;
            if (p.ev_main) p.ev_main[slot] = make_uint4(te, q, event_word(pe, kind), pp);
            if (p.ev_amp) p.ev_amp[slot] = (uint16_t)pa;
        }
        n_ev += ok ? 1u : 0u;
        const bool is_meas = ok && kind == 0u && ((pe >> 24) & 3u) == p.meas_elem;   // meas_elem 0xFF: none
        uint32_t bit = 0;
        if (is_meas) {
            const uint32_t r = philox_u32(p.seed, shot, core, n_meas);
            bit = (thr == INF32) || (r < thr);
            if (p.meas && n_meas < p.meas_cap)
                p.meas[(uint64_t)n_meas * n_lanes + lane] = make_uint2(te + p.meas_latency, bit);
        }
        meas_bits |= (n_meas < 32u ? bit : 0u) << (n_meas & 31u);
        last_bit = is_meas ? bit : last_bit;
        n_meas += is_meas ? 1u : 0u;
    };

    // command k of a running lane (k <= its program length, so the command-major
    // fetch is in bounds)
    auto fetch = [&](uint32_t k) -> uint4 {
        if constexpr (ROWS) {
            return p.fetch[(uint64_t)(k * p.fetch_stride) + prog];
        } else {
            uint4 u = make_uint4(0u, 0u, 0u, 0u);           // past the program: op4 0 = DONE
            if (k < nprog) u = LDS ? s_prog[base + k] : p.fetch[(uint64_t)base + k];
            return u;
        }
    };

    // retire command u = k for the lanes still running: any opcode, any state
    auto retire = [&](const uint4 u, uint32_t k, bool first) {
        const bool live = st == 0u;
        const uint32_t D = t;
        const uint32_t op4 = u.y >> 28;
        // opcode classes as bit tables: cmd_time wait 9/C, pulse class 8/9/B/C,
        // strobe 9/B.  Pulse writes need no class: decode_cmd leaves the write
        // enables of every other opcode zero, so pulse_write is a no-op there
        const bool waits = (0x1200u >> op4) & 1u;
        const bool pulse_cls = (0x1B00u >> op4) & 1u;
        const bool strobe = (0x0A00u >> op4) & 1u;
        const uint32_t T = u.x;
        uint32_t wait;
        bool big = false, dbl = false;
        if (first) {
            // reset hold: qclk(0) = qclk(1) = 0 (proc.sv:125-136); cmd_time 0 strobes twice
            dbl = T == 0u;
            wait = dbl ? 0u : T + 1u;
            big = T == INF32;
        } else {
            wait = T - (D - 1u);                            // qclk(D) = D - 1 for D >= 3
        }
        const bool top = D > max_cycles;
        const bool over = waits && (big || wait > max_cycles - D);
        flags |= (live && !top && waits && (big || wait >= 0x80000000u)) ? F_LATE : 0u;
        const uint32_t fin = top ? (ST_MAX_CYCLES | ST_TOP) : over ? ST_MAX_CYCLES
                           : pulse_cls ? 0u : (op4 >= 0xDu ? ST_HUNG_OPCODE : ST_DONE);
        st = live ? fin : st;
        k_end = live ? k : k_end;
        const bool ok = live && fin == 0u;
        const uint32_t tT = D + (waits ? wait : 0u);
        pulse_write(u, pe, pp, pa);                     // pulse_reg.sv:59-97, reg_in = 0
        const bool rst = op4 == 0xBu;
        emit(ok && strobe, rst ? D : tT + 2u, rst ? (first ? 0u : D - 1u) : tT + 1u, rst ? 1u : 0u);
        if (first) {
            const bool two = ok && dbl && op4 == 0x9u;
            emit(two, tT + 3u, tT + 2u, 0u);
            flags |= two ? F_DOUBLE_STROBE : 0u;
        }
        t = ok ? tT + 3u : t;
    };

    // the cmd_time wait of a pulse / idle command after the first: past the
    // cycle budget (which includes every late cmd_time: wait >= 2^31 >
    // max_cycles - D) a running lane finishes; returns whether the lane goes
    // on, and the execution cycle tT
    auto timed = [&](const uint4 u, uint32_t k, uint32_t &tT) -> bool {
        const bool live = st == 0u;
        const uint32_t D = t;
        const uint32_t wait = u.x - (D - 1u);
        const bool stop = live && wait > max_cycles - D;
        flags |= (stop && wait >= 0x80000000u) ? F_LATE : 0u;
        st = stop ? ST_MAX_CYCLES : st;
        k_end = stop ? k : k_end;
        tT = D + wait;
        return live && !stop;
    };

    // Every lane walks the loop (finished lanes only select their old state),
    // so the loop and the per-opcode switch below branch on scalars.  The
    // running lanes share k; when they also share the opcode and none is past
    // max_cycles (the common case: the same program shape with different
    // parameters) the switch runs that opcode's straight-line semantics
    retire(fetch(0u), 0u, true);
    for (uint32_t k = 1;; k++) {
        const uint64_t running = __ballot(st == 0u);
        if (running == 0ull) break;
        const uint4 u = fetch(k);
        const uint32_t op4 = u.y >> 28;
        const uint32_t op_u = __builtin_amdgcn_readlane(op4, (int)__builtin_ctzll(running));
        const bool live = st == 0u;
        uint32_t tT;
        switch (__ballot(live && (op4 != op_u || t > max_cycles)) ? 0x10u : op_u) {
        case 0x9: {                                         // pulse write + trigger at cmd_time
            const bool ok = timed(u, k, tT);
            pulse_write(u, pe, pp, pa);
            emit(ok, tT + 2u, tT + 1u, 0u);
            t = ok ? tT + 3u : t;
            break;
        }
        case 0xC: {                                         // idle until cmd_time
            const bool ok = timed(u, k, tT);
            t = ok ? tT + 3u : t;
            break;
        }
        case 0x8:                                           // pulse write, no trigger
            pulse_write(u, pe, pp, pa);
            t = live ? t + 3u : t;
            break;
        case 0xB:                                           // phase reset strobe at decode
            emit(live, t, t - 1u, 1u);
            t = live ? t + 3u : t;
            break;
        case 0x0: case 0xA:                                 // done
            st = live ? ST_DONE : st;
            k_end = live ? k : k_end;
            break;
        default:                                            // mixed opcodes, hung, past max_cycles
            retire(u, k, false);
        }
    }
    flags |= (n_ev > p.event_cap ? F_EVENT_OVF : 0u) |
             (n_meas > min(p.meas_cap, MEAS_LOOKUP) ? F_MEAS_OVF : 0u);

    if (valid && p.summary)
        write_summary(p, lane, t, k_end, st & 0xFFu, flags, n_ev, k_end + ((st & ST_TOP) ? 0u : 1u),
                      t ? t - 1u : 0u, n_meas, meas_bits, 0u);
    if (valid && p.regs_out) {
#pragma unroll
        for (int r = 0; r < 16; r++) p.regs_out[(uint64_t)r * n_lanes + lane] = 0u;
    }
    count_outcome(p, s_hist, valid, core, grp, last_bit);
}

hipError_t launch_straight(const KParams &p, int src, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p.n_lanes + BLOCK - 1) / BLOCK);
    if (blocks == 0) return hipSuccess;
    if (src == STRAIGHT_ROWS) {
        hipLaunchKernelGGL(straight_kernel<STRAIGHT_ROWS>, dim3(blocks), dim3(BLOCK), 0, stream, p);
    } else if (src == STRAIGHT_PROG) {
        hipLaunchKernelGGL(straight_kernel<STRAIGHT_PROG>, dim3(blocks), dim3(BLOCK), 0, stream, p);
    } else {
        // programs staged in dynamic LDS beyond the default 64 KiB need the opt-in
        const size_t shmem = (size_t)p.prog_lds_words * sizeof(uint4);
        static size_t granted = 0;
        if (shmem > granted) {
            hipError_t e = hipFuncSetAttribute((const void *)straight_kernel<STRAIGHT_LDS>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
            if (e != hipSuccess) return e;
            granted = shmem;
        }
        hipLaunchKernelGGL(straight_kernel<STRAIGHT_LDS>, dim3(blocks), dim3(BLOCK), shmem, stream, p);
    }
    return hipGetLastError();
}

}  // namespace dpemu
