// straight.hip -- the interpreter for pulse-only programs on CDNA4 (gfx950).
//
// A program of pulse write / trigger, idle, pulse reset, done and hang
// commands never moves its instruction pointer except by +1
// (hdl/instr_ptr.v without a jump) and never writes a register, so qclk is
// never reloaded (hdl/qclk.v): qclk(D) = D - 1 after the two-cycle reset hold.
// Every lane still running in loop iteration k is executing command k of its
// program: the command index is wave-uniform, the per-lane ip / mode state of
// the general interpreter (interp.hip) disappears, and the next commands'
// addresses are known before the current one executes, so they are fetched
// in batches of FB (one memory latency per FB commands).  (Branch-free
// programs with reg_alu / inc_qclk run on macro.hip.)
// Timing is hdl/ctrl.v's closed form (oracle/fast_model.c); the first
// command is peeled to model the reset hold (cmd_time 0 there strobes twice).
// Outputs and their layout are identical to interp_kernel's.
//
// Commands come from the command-major image (STRAIGHT_ROWS: command k of
// program p at fetch[k * n_programs + p], zero = DONE past a program's end
// and in the guard row max_len), the program-major image (STRAIGHT_PROG:
// uops[offsets[p] + min(k, n_instr[p])], a zero guard command after every
// program) or the workgroup's programs staged in LDS with their guards
// (STRAIGHT_LDS, long programs on grids that leave LDS to spare: an LDS fetch
// does not wait for the lane's earlier event stores, which share vmcnt with
// global loads).  Every fetch is clamped in bounds, so loads are unconditional.
//
// Lanes that finish keep walking the loop with their state frozen by selects
// (a divergent branch that writes loop-carried state makes the register
// allocator copy that state around it every iteration); branches guard only
// stores, LDS register writes and philox.  When the running lanes also share
// the opcode (the batched-experiment shape: one program structure, different
// parameters) a scalar switch runs that opcode's straight-line semantics.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lane.h"

namespace dpemu {

// Cache policy of the output rows (DPEMU_ST_POLICY bits, A/B builds: 1 events,
// 2 measurements, 4 summaries nontemporal).  Events + measurements
// nontemporal is the product setting: config 2 (shot-major lanes) 0.1618 ->
// 0.1462 ms, core-major 0.1713 -> 0.1614, config 1 unchanged; either one
// alone measured neutral, and nontemporal summaries (two 16-B halves of a
// 32-B record, written by separate instructions) 0.20 ms
// (profiles/r06_straight_nt_ab.json)
#ifndef DPEMU_ST_POLICY
#define DPEMU_ST_POLICY 3
#endif

template <int SRC, int FB>
__global__ void __launch_bounds__(BLOCK) straight_kernel(const KParams p)
{
    constexpr bool ROWS = SRC == STRAIGHT_ROWS, LDS = SRC == STRAIGHT_LDS;
    __shared__ uint32_t s_hist[HIST_LDS_MAX];
    __shared__ uint32_t s_pref[LDS ? BLOCK + 1 : 1];
    __shared__ uint32_t s_scan[BLOCK / 64];
    __shared__ uint32_t s_key[BLOCK];
    extern __shared__ uint4 s_prog[];
    const uint32_t tid = threadIdx.x;
    const uint32_t C = p.C;
    uint32_t sl, core;                                // shot within the run, core (core-major workgroup)
    clear_hist_next(p);
    block_core_major(p, sl, core);
    const bool valid = sl < p.n_shots;
    const uint32_t lane = out_lane(p, sl, core);      // output lane index (core-major)
    const uint64_t shot = p.shot_begin + sl;
    const uint32_t n_lanes = p.n_lanes;

    uint32_t grp = 0, prog = 0, base = 0, nprog = 0;
    if (valid) {
        grp = shot_group(p, sl);
        prog = p.prog_table[(uint64_t)grp * C + core];
        nprog = p.n_instr[prog];
        if (!ROWS) base = p.offsets[prog];
    }
    const uint32_t thr = valid ? p.p1_thr[core] : 0u;
    if (p.hist_lds) {
        for (uint32_t i = tid; i < HIST_LDS_MAX; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
    }
    if constexpr (LDS) base = stage_programs(p, s_prog, s_pref, s_scan, sl, core);

    const uint32_t max_cycles = p.max_cycles;
    uint32_t t = 0, pe = 0, pp = 0, pa = 0;            // next DECODE cycle; pulse register image
    uint32_t flags = 0, n_ev = 0, n_meas = 0, meas_bits = 0, last_bit = 0;
    // st: 0 while running, else the finish status (| ST_TOP: stopped by the
    // max_cycles check before a fetch, so that command did not retire); k_end:
    // the command index at the finish.  A finish leaves t alone: t_end = t
    constexpr uint32_t ST_TOP = 0x100u;
    uint32_t st = valid ? 0u : ST_DONE, k_end = 0;

    // pulse_iface strobe at cycle te (kind 0: trigger, 1: phase reset) with
    // the current pulse registers, for lanes with `ok`; readout-element
    // triggers draw the measurement.  Overflow flags are derived from the
    // final counts (a record is dropped iff its count exceeds the cap)
    auto emit = [&](bool ok, uint32_t te, uint32_t kind) {
        if (ok && n_ev < p.event_cap && p.events)
            st_out(&p.events[(uint64_t)n_ev * n_lanes + lane], event_record(te, pe, pp, pa, kind), (DPEMU_ST_POLICY & 1) != 0);
        n_ev += ok ? 1u : 0u;
        const bool is_meas = ok && kind == 0u && ((pe >> 24) & 3u) == p.meas_elem;   // meas_elem 0xFF: none
        uint32_t bit = 0;
        if (is_meas) {
            bit = meas_bit(p, shot, core, n_meas, thr, pa, pe);
            if (p.meas && n_meas < p.meas_cap)
                st_out(&p.meas[(uint64_t)n_meas * n_lanes + lane], make_uint2(te + p.meas_latency, bit), (DPEMU_ST_POLICY & 2) != 0);
        }
        meas_bits |= (n_meas < 32u ? bit : 0u) << (n_meas & 31u);
        last_bit = is_meas ? bit : last_bit;
        n_meas += is_meas ? 1u : 0u;
    };

    // command k of this lane's program, zero (DONE) past its end; in bounds for any k
    auto fetch = [&](uint32_t k) -> uint4 {
        if constexpr (ROWS) {
            return p.fetch[(uint64_t)(min(k, p.max_len) * p.fetch_stride) + prog];
        } else {
            const uint32_t i = base + min(k, nprog);
            return LDS ? s_prog[i] : p.fetch[i];
        }
    };

    // retire command u = k for the lanes in `live` (running): any opcode, any state
    auto retire = [&](const uint4 u, uint32_t k, bool first, bool live) {
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
            wait = T - (D - 1u);                            // qclk(D) = D - 1 after the hold
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
        pulse_write(u, pe, pp, pa);                     // pulse_reg.sv:59-97 (reg_in reads 0)
        const bool rst = op4 == 0xBu;
        emit(ok && strobe, rst ? D : tT + 2u, rst ? 1u : 0u);
        if (first) {
            const bool two = ok && dbl && op4 == 0x9u;
            emit(two, tT + 3u, 0u);
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

    // one command for all lanes (finished ones keep their state): a scalar
    // switch on the opcode when the running lanes agree on it and none is past
    // max_cycles, else the any-opcode path.  (A waterfall over the distinct
    // opcodes of a mixed wave measured slower than the any-opcode path.)
    auto step = [&](const uint4 u, uint32_t k) {
        const uint32_t op4 = u.y >> 28;
        const uint64_t running = __ballot(st == 0u);
        const uint32_t op_u = __builtin_amdgcn_readlane(op4, (int)__builtin_ctzll(running));
        const bool live = st == 0u;
        uint32_t tT;
        switch (__ballot(live && (op4 != op_u || t > max_cycles)) ? 0x10u : op_u) {
        case 0x9: {                                         // pulse write + trigger at cmd_time
            const bool ok = timed(u, k, tT);
            pulse_write(u, pe, pp, pa);
            emit(ok, tT + 2u, 0u);
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
            emit(live, t, 1u);
            t = live ? t + 3u : t;
            break;
        case 0x0: case 0xA:                                 // done
            st = live ? ST_DONE : st;
            k_end = live ? k : k_end;
            break;
        default:                                            // mixed opcodes, hung, past max_cycles
            retire(u, k, false, live);
        }
    };

    retire(fetch(0u), 0u, true, st == 0u);
    for (uint32_t k = 1; __ballot(st == 0u); k += FB) {
        uint4 u[FB];
#pragma unroll
        for (int j = 0; j < FB; j++) u[j] = fetch(k + j);  // independent loads: one latency per batch
#pragma unroll
        for (int j = 0; j < FB; j++) {
            if (j && !__ballot(st == 0u)) break;
            step(u[j], k + j);
        }
    }
    flags |= (n_ev > p.event_cap ? F_EVENT_OVF : 0u) | (n_meas > min(p.meas_cap, MEAS_LOOKUP) ? F_MEAS_OVF : 0u);

    if (valid && p.summary)
        write_summary(p, lane, t, k_end, st & 0xFFu, flags, n_ev, k_end + ((st & ST_TOP) ? 0u : 1u),
                      t < 1u ? 0u : t - 1u, n_meas, meas_bits, 0u);
    if (valid && p.regs_out) {
#pragma unroll
        for (int r = 0; r < 16; r++) p.regs_out[(uint64_t)r * n_lanes + lane] = 0u;
    }
    count_outcome_block(p, s_hist, s_key, valid, core, sl, grp, last_bit);
}

template <int SRC, int FB>
static hipError_t launch_src(const KParams &p, uint32_t blocks, size_t shmem, hipStream_t stream)
{
    // programs staged in dynamic LDS beyond the default 64 KiB need the opt-in
    const hipError_t e = opt_in_dynamic_lds((const void *)straight_kernel<SRC, FB>, shmem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((straight_kernel<SRC, FB>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    return hipGetLastError();
}

hipError_t launch_straight(const KParams &p, int src, int fb, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p.n_lanes + BLOCK - 1) / BLOCK);
    if (blocks == 0) return hipSuccess;
    const size_t shmem = src == STRAIGHT_LDS ? (size_t)p.prog_lds_words * sizeof(uint4) : 0;
#define SRC_CASE(S)                                                                                    \
    case S: return fb == 1 ? launch_src<S, 1>(p, blocks, shmem, stream) : launch_src<S, 4>(p, blocks, shmem, stream);
    switch (src) {
    SRC_CASE(STRAIGHT_ROWS) SRC_CASE(STRAIGHT_PROG) SRC_CASE(STRAIGHT_LDS)
    }
#undef SRC_CASE
    return hipErrorInvalidValue;
}

}  // namespace dpemu
