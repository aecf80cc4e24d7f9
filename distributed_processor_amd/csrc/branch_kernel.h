// branch_kernel.h -- the interpreter for programs with jumps, fproc_meas reads
// and sync barriers (rows a1-a11; config 3, active reset) on CDNA4 (gfx950).
//
// Same lane mapping, lockstep loop and outputs as interp_kernel (interp.hip):
// one thread = one (shot, core) lane, a shot's C cores adjacent lanes of ONE
// wavefront, each iteration retires at most one command per lane and
// advances its next-DECODE cycle by hdl/ctrl.v's closed-form latency
// (oracle/fast_model.c).  What differs is how a command retires.  The
// general interpreter dispatches on the opcode; under divergence every taken
// case runs, and cases that write the loop-carried state on different paths
// cost copies of all of it per iteration.  Here:
//
//   * the commands that need no ALU -- pulse write / trigger, idle, pulse
//     reset, jump_i, sync, done, hang: almost every command of a branching
//     program -- go through ONE branch-free datapath written once through
//     selects:  wait = cmd_time - qclk(D), qclk(D) = D + qoff;  strobe at
//     tT + 2;  next decode tT + 3 / D + 4;  next ip ip + 1 / target;
//   * reg_alu, jump_cond, alu_fproc / jump_fproc, inc_qclk take a second
//     datapath (alu.v:20-50, instr_ptr.v, proc.sv:124) under a wave-uniform
//     guard, the fproc_meas lookup under its own;
//   * the cross-core phases are wave-uniform and run only when needed: the
//     fproc_meas bound before a read, the sync barrier AFTER the iteration's
//     commands, so the last arrival releases it in the same iteration;
//     group min / max are DPP within a row of 16 lanes;
//   * the reset hold (qclk(0) = qclk(1) = 0, proc.sv:125-136) can only be
//     seen by a lane's first decode: a peeled first iteration;
//   * event records are held per lane and stored a whole wave row at a
//     time (below, pend0 / pend1);
//   * no register file when no command writes one (FEAT_REGS), and the
//     workgroup's programs staged in LDS when they are short
//     (FEAT_PROG_LDS: an LDS fetch does not wait behind the lane's event
//     stores, which share vmcnt with global loads on gfx950).
//
// Branches guard only stores, LDS writes and the measurement draw.  The
// meas_lut back end (FEAT_LUT: hdl/fproc_lut.sv, core_state_mgr.sv,
// meas_lut.sv) runs the LUT FSM over the shot's merged measurement stream in
// all the shot's lanes at once (group min / ballots), where interp_kernel
// runs it serially in the shot's leader lane.

#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "lane.h"

namespace dpemu {

// cache policy of the event / measurement rows (A/B builds: bits 0-1 the
// events' StPolicy (lane.h), bit 2 measurements nontemporal)
#ifndef DPEMU_BRANCH_NT
#define DPEMU_BRANCH_NT 0
#endif
constexpr StPolicy BR_EV_POLICY = (StPolicy)(DPEMU_BRANCH_NT & 3);
constexpr bool BR_NT_MEAS = (DPEMU_BRANCH_NT & 4) != 0;

namespace {

enum : uint32_t { B_RUN = 0, B_SYNC = 1, B_LUT = 2, B_FIN = 3 };


// decode-to-decode latency per op4 past the command's base cycle (D, the
// trigger cycle tT for pulse-with-trigger / idle, the fproc ready cycle R):
// pulse 3, reg_alu / jump_i / inc_qclk / alu_fproc 4, jump_cond / jump_fproc 6
constexpr uint64_t LATENCY = 0x0003303304646440ull;

__device__ __forceinline__ uint32_t alu_eval(uint32_t op, uint32_t a, uint32_t b)
{
    // alu.v:20-50: 0 id0, 1 add, 2 sub, 3 eq, 4 le, 5 ge, 6 id1, 7 zero;
    // le = sub[31] ^ overflow == signed a < b.  A select tree on op's bits.
    const uint32_t sub = a - b;
    const uint32_t lt = (int32_t)a < (int32_t)b;
    const bool b0 = op & 1u, b1 = op & 2u;
    const uint32_t lo = b1 ? (b0 ? (uint32_t)(sub == 0u) : sub) : (b0 ? a + b : a);   // 0-3
    const uint32_t hi = b1 ? (b0 ? 0u : b) : (lt ^ (uint32_t)b0);                     // 4-7
    return (op & 4u) ? hi : lo;
}

// group reductions over the C adjacent lanes of a shot (all lanes converged):
// DPP within a row of 16 lanes (quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror and row_mirror: each step pairs every lane with one of the
// other half of its group), cross-lane permutes above 16
template <int OP>   // 0 = min, 1 = max
__device__ __forceinline__ uint32_t group_reduce(uint32_t v, uint32_t C)
{
    auto comb = [](uint32_t a, uint32_t b) { return OP == 0 ? (a < b ? a : b) : (a > b ? a : b); };
#define DPP(x, ctrl) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), (ctrl), 0xF, 0xF, false))
    if (C >= 2) v = comb(v, DPP(v, 0xB1));
    if (C >= 4) v = comb(v, DPP(v, 0x4E));
    if (C >= 8) v = comb(v, DPP(v, 0x141));
    if (C >= 16) v = comb(v, DPP(v, 0x140));
#undef DPP
    for (uint32_t m = 16; m < C; m <<= 1) v = comb(v, (uint32_t)__shfl_xor((int)v, (int)m, 64));
    return v;
}

// minimum over the whole wave (all lanes converged): DPP within each row of
// 16, then the four rows' minima by readlane
__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
    v = group_reduce<0>(v, 16u);
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return min(min(a, b), min(c, d));
}

}  // namespace

// CT: the cores per shot when fixed at compile time (8: the BASELINE
// configs), so group reductions and lane arithmetic are straight-line; 0 = p.C
template <int FEAT, int CT>
__global__ void __launch_bounds__(BLOCK) branch_kernel(const KParams p)
{
    constexpr bool FPROC = (FEAT & FEAT_FPROC) != 0;
    constexpr bool LUT = (FEAT & FEAT_LUT) != 0;     // fproc_lut back end (exclusive with FPROC)
    constexpr bool XMEAS = FPROC || LUT;             // measurements readable by the shot
    constexpr bool SYNC = (FEAT & FEAT_SYNC) != 0;
    constexpr bool REGS = (FEAT & FEAT_REGS) != 0;  // some command writes the reg_file (else it reads 0)
    constexpr bool PLDS = (FEAT & FEAT_PROG_LDS) != 0;   // the workgroup's programs staged in LDS
    constexpr bool DEMOD = (FEAT & FEAT_DEMOD) != 0;     // meas_model DPEMU_MEAS_DEMOD
    constexpr int MT = XMEAS ? MEAS_LOOKUP : 1;
    // event records stored as they arise (DIRECT) or held and stored as whole
    // wave rows (below).  Measured per back end (same-process A/Bs, outputs
    // identical; profiles/r04_branch_direct_ab.jsonl): config 3 (fproc_meas)
    // 0.446 ms held vs 0.480 direct; config 3 through the LUT 0.564 held vs
    // 0.494 direct -- the row bookkeeping's VALU costs more there than the
    // scattered partial rows it avoids.  With the DEMOD readout the held rows'
    // 10 VGPRs decide the occupancy (105 -> 95 VGPRs, 4 -> 5 waves per SIMD):
    // config 3 DEMOD 0.653 ms held vs 0.515 direct (profiles/r06_demod_ab2.json)
    constexpr bool DIRECT = LUT || DEMOD;
    constexpr int NF = LUT ? LUT_FIRE_CAP : 1;

    __shared__ uint32_t s_regs[REGS ? 16 : 1][REGS ? BLOCK : 1];
    __shared__ uint32_t s_mt[MT][BLOCK];              // measurements {valid cycle << 1 | bit}, readable by the shot
    // meas_lut (hdl/meas_lut.sv, core_state_mgr.sv): the shot's fires so
    // far, each as {fire cycle << 1 | this lane's bit of lut_out}
    __shared__ uint32_t s_fire[NF][LUT ? BLOCK : 1];
    __shared__ uint32_t s_pref[PLDS ? BLOCK + 1 : 1];
    __shared__ uint32_t s_scan[BLOCK / 64];
    // DEMOD: the lane's program's frequency tables {drv_off, drv_len, lo_off,
    // lo_len} and their index-0 words, loaded once (a global load at a readout
    // would wait behind the lane's event stores: vmcnt is shared)
    __shared__ uint32_t s_rof[DEMOD ? 6 : 1][DEMOD ? BLOCK : 1];
    // dynamic LDS: the staged programs (prog_lds_words commands), then the
    // histogram pre-aggregation bins when hist_lds
    extern __shared__ uint4 s_dyn[];
    uint4 *const s_prog = s_dyn;
    uint32_t *const s_hist = reinterpret_cast<uint32_t *>(s_dyn + (PLDS ? p.prog_lds_words : 0u));

    clear_hist_next(p);
    const uint32_t tid = threadIdx.x;
    const uint32_t C = CT ? (uint32_t)CT : p.C;
    const uint32_t log2C = CT ? (uint32_t)__builtin_ctz(CT) : p.log2C;
    const uint32_t pos = blockIdx.x * BLOCK + tid;   // thread position; a shot's cores are adjacent
    const bool valid = pos < p.n_lanes;
    const uint32_t core = pos & (C - 1);
    const uint32_t spos = pos >> log2C;
    const uint32_t lane = out_lane(p, spos, core);   // output lane index (core-major)
    const uint64_t shot = p.shot_begin + spos;
    const uint32_t wl = tid & 63;
    const uint32_t leader_tid = tid & ~(C - 1);
    const uint32_t n_lanes = p.n_lanes, max_cycles = p.max_cycles;

    uint32_t nprog = 0, grp = 0, prog = 0, base = 0;
    if (valid) {
        grp = shot_group(p, spos);
        prog = p.prog_table[(uint64_t)grp * C + core];
        base = p.offsets[prog];
        nprog = p.n_instr[prog];
    }
    // command k of this lane's program, zero (DONE) past its end, in bounds for
    // any k: the program-major image has a zero guard after every program, the
    // command-major copy zeros past each program's end and a guard row
    if constexpr (PLDS) {
        const uint32_t b = stage_programs(p, s_prog, s_pref, s_scan, spos, core);
        if (valid) base = b;
    }
    const bool cmd_major = !PLDS && p.fetch_stride != 1u;
    const uint32_t fetch_off = cmd_major ? prog : base, k_max = cmd_major ? p.max_len : nprog;
    const uint32_t thr_core = valid ? p.p1_thr[core] : 0u;
    if constexpr (DEMOD) {
        const uint4 h = valid ? p.ro_hdr[prog] : make_uint4(0u, 0u, 0u, 0u);
        s_rof[0][tid] = h.x; s_rof[1][tid] = h.y; s_rof[2][tid] = h.z; s_rof[3][tid] = h.w;
        s_rof[4][tid] = ro_freq(p, h.x, h.y, 0u);
        s_rof[5][tid] = ro_freq(p, h.z, h.w, 0u);
    }
    if (p.hist_lds) {
        for (uint32_t i = tid; i < HIST_LDS_MAX; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
    }
    if constexpr (REGS) {
#pragma unroll
        for (int r = 0; r < 16; r++) s_regs[r][tid] = 0;
    }
    if constexpr (XMEAS) {
#pragma unroll
        for (int m = 0; m < MT; m++) s_mt[m][tid] = INF32;
    }
    // meas_lut state (meas_lut.sv:27-56), the same in every lane of a shot:
    // OR-accumulated valid / measurement bits of the masked cores, the last
    // fire, fires so far; and this lane's merge cursor into its s_mt records
    uint64_t lut_valid = 0, lut_addr = 0;
    uint32_t lut_last_fire = INF32, nfire = 0, lut_cur = 0;

    uint32_t mode = valid ? B_RUN : B_FIN;
    // qclk(x) = x + qoff for every decode after the first (hdl/qclk.v: it
    // counts from 0 at cycle 1 after the reset hold; inc_qclk and the sync
    // restart reload it).  A lane's FIRST decode is the only one that can
    // fall in the reset hold (qclk(0) = qclk(1) = 0): it takes the peeled
    // first step below.
    uint32_t ip = 0, t = 0, qoff = 0xFFFFFFFFu;
    uint32_t pe = 0, pp = 0, pa = 0;                 // pulse regs: env|cfg<<24, phase|freq<<17, amp
    uint32_t wait_d = 0, status = 0, flags = 0, t_end = 0;
    uint32_t n_ev = 0, n_tr = 0, n_meas = 0, n_exec = 0, meas_bits = 0, last_bit = 0;
    const bool is_part = SYNC ? (((p.sync_mask >> core) & 1ull) != 0) : false;
    uint4 *const ev_lane = p.events + lane;          // event slot k of this lane at ev_lane[k * n_lanes]
    // Event rows written whole.  A record is held (up to two per lane) until
    // every unfinished lane of the wave has reached its slot, then the wave
    // stores the row in one instruction: lanes on different branches (config
    // 3's conditional X90 pair) reach a row in different iterations, and
    // storing each part as it comes was slower although it issued fewer
    // stores and the same bytes (config 3: 0.480 -> 0.447 ms median,
    // profiles/r02_ar_rows_ab.json).  Slots [n_st, min(n_ev, cap)) are
    // pending in pend0, pend1; a third record pushes the oldest out.
    uint4 pend0 = make_uint4(0u, 0u, 0u, 0u), pend1 = pend0;
    uint32_t n_st = 0;
    // DEMOD: the latest readout-drive strobe and pulse_reset, the last meas_valid
    RoDrive ro_d{0u, 0u, 0u};
    uint32_t ro_tref = 0, ro_ltv = 0;

    // pulse_iface strobe at cycle te (kind 0: trigger, 1: phase reset) with the
    // current pulse registers for lanes with `ok`; readout-element triggers
    // draw the measurement.  Overflow flags come from the final counts.
    auto emit = [&](bool ok, uint32_t te, uint32_t kind) __attribute__((always_inline)) {
        if (ok) {
            if (DIRECT && n_ev < p.event_cap && p.events)
                st_rec<BR_EV_POLICY>(&ev_lane[(uint64_t)n_ev * n_lanes], event_record(te, pe, pp, pa, kind));
            if (!DIRECT && n_ev < p.event_cap && p.events) {
                const uint4 rec = event_record(te, pe, pp, pa, kind);
                const bool full = n_ev - n_st == 2u;    // the oldest goes out now
                if (full) st_rec<BR_EV_POLICY>(&ev_lane[(uint64_t)n_st * n_lanes], pend0);
                pend0 = sel4(full, pend1, pend0);
                n_st += full ? 1u : 0u;
                const bool first = n_ev == n_st;
                pend0 = sel4(first, rec, pend0);
                pend1 = sel4(first, pend1, rec);
            }
            n_ev++;
            if constexpr (DEMOD) {
                if (kind == 1u) ro_tref = te;
                if (kind == 0u && ((pe >> 24) & 3u) == p.ro_drv_elem)
                    ro_d = RoDrive{te, pp & 0x03FFFFFFu, (pa & 0xFFFFu) | (((pe >> 12) & 0xFFFu) << 16) | 0x80000000u};
            }
            if (kind == 0u && ((pe >> 24) & 3u) == p.meas_elem) {   // meas_elem 0xFF: none
                uint32_t bit, tv;
                if constexpr (DEMOD) {
                    int2 a;
                    const uint32_t fi_lo = (pp >> 17) & 0x1FFu, fi_d = (ro_d.pp >> 17) & 0x1FFu;
                    const uint32_t f_lo = fi_lo ? ro_freq(p, s_rof[2][tid], s_rof[3][tid], fi_lo) : s_rof[5][tid];
                    const uint32_t f_d = fi_d ? ro_freq(p, s_rof[0][tid], s_rof[1][tid], fi_d) : s_rof[4][tid];
                    bit = demod_readout(p, shot, core, n_meas, thr_core, te, pe, pp, ro_d, ro_tref, f_lo, f_d, a);
                    tv = demod_valid(p, te, pe, ro_ltv);
                    ro_ltv = tv;
                    if (p.acc && n_meas < p.meas_cap) p.acc[(uint64_t)n_meas * n_lanes + lane] = a;
                } else {
                    bit = meas_bit(p, shot, core, n_meas, thr_core, pa, pe);
                    tv = te + p.meas_latency;
                }
                if constexpr (XMEAS) {
                    if (n_meas < (uint32_t)MT) s_mt[n_meas < (uint32_t)MT ? n_meas : 0u][tid] = (tv << 1) | bit;
                }
                if (p.meas && n_meas < p.meas_cap) st_out(&p.meas[(uint64_t)n_meas * n_lanes + lane], make_uint2(tv, bit), BR_NT_MEAS);
                meas_bits |= (n_meas < 32u ? bit : 0u) << (n_meas & 31u);
                last_bit = bit;
                n_meas++;
            }
        }
    };

    auto emit_trace = [&](bool ok, uint32_t tt, uint32_t addr, uint32_t val) __attribute__((always_inline)) {
        if (ok) {
            if (n_tr < p.trace_cap && p.trace) p.trace[(uint64_t)n_tr * n_lanes + lane] = make_uint4(tt, addr, val, 0u);
            n_tr++;
        }
    };

    // latest measurement of group lane q with valid cycle <= d.  A lane's
    // slots fill in time order (valid cycles non-decreasing, INF past the
    // last; INF >> 1 exceeds any cycle), so the scan stops at the first slot
    // later than d -- read in pairs (one ds_read2), usually one pair per
    // lane instead of MT unrolled reads and compares
    auto meas_lookup = [&](uint32_t q_tid, uint32_t d) -> uint32_t {
        static_assert(MEAS_LOOKUP % 2 == 0, "slots read in pairs");
        uint32_t res = 0;
#pragma unroll 1
        for (int m = 0; m + 1 < MT; m += 2) {
            const uint32_t e0 = s_mt[m][q_tid], e1 = s_mt[m + 1][q_tid];
            if ((e0 >> 1) > d) break;
            res = e0 & 1u;
            if ((e1 >> 1) > d) break;
            res = e1 & 1u;
        }
        return res;
    };

    // sync barrier keys: a participant's SYNC decode while it waits, its next
    // decode while it runs (a lower bound of its arrival), the earliest next
    // decode after a release while it waits on the LUT (>= wait_d + 1 + 4),
    // INF once finished
    auto sync_maxkey = [&]() -> uint32_t {
        uint32_t key = mode == B_SYNC ? wait_d : t;
        if constexpr (LUT) key = mode == B_LUT ? wait_d + 5u : key;
        key = mode == B_FIN ? INF32 : key;
        return group_reduce<1>(is_part ? key : 0u, C);
    };

    // reg_file read (hdl/reg_file.v): all zero while no command writes it
    auto reg = [&](uint32_t r) __attribute__((always_inline)) -> uint32_t {
        if constexpr (REGS) return s_regs[r & 15u][tid];
        return 0u;
    };

    auto finish = [&](bool stop, uint32_t st, uint32_t at) __attribute__((always_inline)) {
        status = stop ? st : status;
        t_end = stop ? at : t_end;
        mode = stop ? B_FIN : mode;
    };

    // store the pending rows every unfinished lane has passed (all: at the end)
    auto flush_rows = [&](bool all) __attribute__((always_inline)) {
        if (DIRECT || !p.events) return;
        const uint32_t ne = min(n_ev, p.event_cap);
        if (!__any(ne > n_st)) return;
        const uint32_t done = all ? INF32 : wave_min(mode == B_FIN ? INF32 : ne);
        // the held records [n_st, ne) are pend0, pend1: store the rows every
        // unfinished lane has passed, then shift once (not once per row)
        const bool f1 = n_st < ne && n_st < done;
        if (!__any(f1)) return;                      // most iterations complete no row
        const bool f2 = f1 && n_st + 1u < ne && n_st + 1u < done;
        if (f1) st_rec<BR_EV_POLICY>(&ev_lane[(uint64_t)n_st * n_lanes], pend0);
        if (__any(f2)) {
            if (f2) st_rec<BR_EV_POLICY>(&ev_lane[(uint64_t)(n_st + 1u) * n_lanes], pend1);
        }
        pend0 = sel4(f1 && !f2, pend1, pend0);
        n_st += (f1 ? 1u : 0u) + (f2 ? 1u : 0u);
    };

    // One lockstep iteration: every running lane retires at most one command.
    // FIRST: the peeled first iteration, where every lane decodes at cycle 0
    // inside the reset hold.  Returns whether any lane is still live.
    auto iteration = [&](auto first_tag) -> bool {
        constexpr bool FIRST = decltype(first_tag)::value;
        // max_cycles at decode
        finish(mode == B_RUN && t > max_cycles, ST_MAX_CYCLES, t);
        const bool run = mode == B_RUN;
        const uint4 u = PLDS ? s_prog[fetch_off + min(ip, k_max)]
                             : p.fetch[(uint64_t)min(ip, k_max) * p.fetch_stride + fetch_off];
        const uint32_t op = u.y >> 28;

        // ---- fproc_meas bound (FPROC): a read at D needs every meas_valid <= D
        // known, i.e. the group's lower bound on its next strobe + meas_latency > D
        bool stall = false;
        if constexpr (FPROC) {
            const bool fp = run && (op == 4u || op == 5u);
            if (__any(fp)) {
                uint32_t bound = run ? t + 2u : INF32;
                if constexpr (SYNC) {
                    if (__any(mode == B_SYNC)) {
                        const uint32_t maxkey = sync_maxkey();
                        if (mode == B_SYNC && is_part && maxkey != INF32) bound = maxkey + p.sync_latency + 5u;
                    }
                }
                const uint32_t gmin = group_reduce<0>(bound, C);
                stall = fp && !((uint64_t)gmin + p.meas_latency > (uint64_t)t);
            }
        }
        const bool go = run && !stall;
        bool sync_rel = false;                           // released from a sync barrier this iteration
        n_exec += go ? 1u : 0u;
        const uint32_t D = t;
        // qclk at this decode (0 in the reset hold)
        const uint32_t qD = FIRST ? 0u : D + qoff;

        // ---- the commands that need no ALU: one branch-free datapath ----
        // pulse write / trigger, idle, pulse reset (ctrl.v: D + 3, or tT + 3
        // after the cmd_time wait), jump_i (D + 4), sync (waits for the
        // barrier), done, hang -- almost every command of a program between
        // its measurement-conditioned branches.
        constexpr uint32_t FAST = 0xFF05u | (SYNC ? 0x80u : 0u);   // 0, 2, (7,) 8-F
        const bool pcls = (FAST >> op) & 1u;
        {
            const bool pg = go && pcls;
            const bool waits = (0x1200u >> op) & 1u;    // 9: pulse trigger, C: idle
            // tT = the first cycle >= D with qclk == cmd_time
            uint32_t wait = u.x - qD;
            bool big = false, dbl = false;
            if constexpr (FIRST) {                       // qclk(0) = qclk(1) = 0 (proc.sv:125-136)
                dbl = u.x == 0u;
                const uint64_t w = dbl ? 0ull : 1ull + u.x;
                wait = (uint32_t)w;
                big = (w >> 32) != 0ull;
            }
            const bool late = waits && (big || wait >= 0x80000000u);
            const bool over = waits && (big || wait > max_cycles - D);
            const uint32_t tT = D + (waits ? wait : 0u);
            const bool jmp = op == 2u;
            const bool to_sync = SYNC && pg && op == 7u;
            const bool cont = pg && (((0x1B04u >> op) & 1u) != 0u) && !over;   // 2, 8, 9, B, C in the budget
            // pulse_reg.sv:59-97 (write enables are zero except for 8 / 9):
            // immediates, then reg[rs0] into register-sourced fields
            // (only 8 / 9 write: skipped in iterations where no lane has one)
            if (__any(cont && ((0x300u >> op) & 1u))) {
                uint32_t pe2 = pe, pp2 = pp, pa2 = pa;
                pulse_write(u, pe2, pp2, pa2);
                if (cont && (u.w & UOP_ANY_RS)) {
                    const uint32_t r0 = reg(u.w >> 20);
                    if (u.w & UOP_RS_ENV) pe2 |= r0 & 0xFFFFFFu;
                    if (u.w & UOP_RS_PH) pp2 |= r0 & 0x1FFFFu;
                    if (u.w & UOP_RS_FR) pp2 |= (r0 & 0x1FFu) << 17;
                    if (u.w & UOP_RS_AMP) pa2 = r0 & 0xFFFFu;
                }
                pe = cont ? pe2 : pe;
                pp = cont ? pp2 : pp;
                pa = cont ? pa2 : pa;
            }
            // strobes: trigger at tT + 2 (cmd_time 0 in the reset hold strobes
            // twice), phase reset at D
            const bool rst = op == 0xBu;
            emit(cont && (op == 9u || rst), rst ? D : tT + 2u, rst ? 1u : 0u);
            if constexpr (FIRST) {
                const bool two = cont && dbl && op == 9u;
                emit(two, tT + 3u, 0u);
                flags |= two ? F_DOUBLE_STROBE : 0u;
            }
            flags |= (pg && late) ? F_LATE : 0u;
            if (__any(pg && !cont && !to_sync)) {
                finish(pg && !cont && !to_sync, over ? ST_MAX_CYCLES : op >= 0xDu ? ST_HUNG_OPCODE : ST_DONE, D);
            }
            wait_d = to_sync ? D : wait_d;
            mode = to_sync ? B_SYNC : mode;
            ip = cont ? (jmp ? (u.z & 0xFFFFu) : ((ip + 1u) & 0xFFFFu)) : ip;
            t = cont ? (jmp ? D + 4u : tT + 3u) : t;
        }
        // ---- reg_alu, jump_cond, alu_fproc / jump_fproc, inc_qclk (1, 3-6) ----
        if (__any(go && !pcls)) {
            const bool sg = go && !pcls;
            const bool is_fp = op == 4u || op == 5u;
            const uint32_t reg0 = reg(u.w >> 20);
            const uint32_t reg1 = reg(u.y >> 4);
            uint32_t data = 0;
            uint32_t R = D + 2u;                         // fproc_meas.sv:18-35: ready two cycles after the read
            bool lut_wait = false, no_meas = false;
            if constexpr (FPROC) {
                if (__any(sg && is_fp)) {
                    if (sg && is_fp) data = meas_lookup(leader_tid + (((u.z >> 16) & 0xFFu) & (C - 1u)), D);
                }
            }
            if constexpr (LUT) {
                // core_state_mgr.sv:45-69: id 0 waits for this core's next
                // meas_valid (>= D + 1: recorded already -- the core's own
                // strobes precede it -- or never), id != 0 for the LUT
                if (__any(sg && is_fp)) {
                    const bool id0 = ((u.z >> 16) & 0xFFu) == 0u;
                    lut_wait = sg && is_fp && !id0;
                    if (sg && is_fp && id0) {
                        uint32_t e = INF32;
#pragma unroll
                        for (int m = MT - 1; m >= 0; m--) {
                            const uint32_t x = s_mt[m][tid];
                            e = (x != INF32 && (x >> 1) >= D + 1u) ? x : e;
                        }
                        no_meas = e == INF32;
                        R = e >> 1;
                        data = e & 1u;
                    }
                }
            }
            const uint32_t in0 = (u.y & 8u) ? reg0 : u.x;
            const uint32_t out = alu_eval(u.y & 7u, in0, op == 6u ? qD : is_fp ? data : reg1);
            // not reached (the host picks kernels by opcode): fproc / sync without the feature
            const bool absent = (!XMEAS && is_fp) || (!SYNC && op == 7u);
            const bool r_over = XMEAS && is_fp && !lut_wait && !no_meas && R > max_cycles;
            const bool fin = r_over || absent || no_meas;
            const bool cont = sg && !fin;
            const bool to_sync = SYNC && cont && op == 7u;
            const bool to_lut = LUT && cont && lut_wait;
            const bool adv = cont && !to_sync && !to_lut;
            const uint32_t t_next = (is_fp ? R : D) + (uint32_t)((LATENCY >> (4u * op)) & 15u);
            const bool take = op == 2u || ((op == 3u || op == 5u) && (out & 1u));
            const uint32_t ip_next = take ? (u.z & 0xFFFFu) : ((ip + 1u) & 0xFFFFu);
            // reg_file write (reg_alu, alu_fproc) and the register / qclk trace
            const bool wr = adv && (op == 1u || op == 4u);
            if constexpr (REGS) {
                if (wr) s_regs[(u.y >> 8) & 15u][tid] = out;
            }
            const bool inc = adv && op == 6u;
            emit_trace(wr || inc, (op == 4u ? R : D) + 3u, inc ? TRACE_QCLK_LOAD : (u.y >> 8) & 15u,
                       inc ? out + 3u : out);
            qoff = inc ? out - D : qoff;                 // qclk(D + 3) = out + 3
            finish(sg && fin, r_over ? ST_MAX_CYCLES : ST_DEADLOCK, D);
            wait_d = (to_sync || to_lut) ? D : wait_d;
            mode = to_sync ? B_SYNC : to_lut ? B_LUT : mode;
            ip = adv ? ip_next : ip;
            t = adv ? t_next : t;
        }

        // ---- sync barrier (SYNC): complete when every participant waits; the
        // last arrival releases it in the same iteration ----
        if constexpr (SYNC) {
            if (__any(mode == B_SYNC)) {
                const uint32_t maxkey = sync_maxkey();
                const uint64_t b = __ballot(is_part && mode == B_SYNC);
                const uint64_t pm = __ballot(is_part);
                const bool all_arrived = group_bits(b, wl, C) == group_bits(pm, wl, C) && group_bits(pm, wl, C) != 0ull;
                const bool rel = mode == B_SYNC && is_part && all_arrived;
                const uint32_t S = maxkey + p.sync_latency;   // sync.ready; qclk restarts at S + 2
                const bool ok = rel && S <= max_cycles;
                emit_trace(ok, S + 2u, TRACE_QCLK_RST, 0u);
                qoff = ok ? 0u - (S + 2u) : qoff;
                ip = ok ? ((ip + 1u) & 0xFFFFu) : ip;
                t = ok ? S + 3u : t;
                mode = ok ? B_RUN : mode;
                finish(rel && !ok, ST_MAX_CYCLES, wait_d);
                sync_rel = rel;
                // a shot in which no lane retired or was released can never
                // progress (with the LUT: checked after the LUT phase below)
                if constexpr (!LUT)
                    finish(group_bits(__ballot(go || rel), wl, C) == 0ull && mode == B_SYNC, ST_DEADLOCK, wait_d);
            }
        }

        // ---- meas_lut (LUT): the shot merges its recorded
        // measurements in time order up to the horizon before which no
        // measurement can still appear (the group's bound on its next strobe
        // + meas_latency), runs the LUT FSM over them (hdl/meas_lut.sv:27-56:
        // OR-accumulate the masked cores' valid / bits, fire when every masked
        // core is valid, then clear; the cycle after a fire ignores inputs)
        // and publishes the fires; a lane waiting on the LUT (core_state_mgr
        // WAIT_LUT) takes the first fire after its read. ----
        bool lut_rel = false;
        if constexpr (LUT) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // this iteration's s_mt writes
            __builtin_amdgcn_wave_barrier();
            // merged lazily, only while some lane waits on the LUT: the
            // records stay in s_mt, and a fire matters only to a waiting lane,
            // so merging them later in the same order yields the same fires
            if (__any(mode == B_LUT)) {
                uint32_t bound = mode == B_RUN ? t + 2u : mode == B_LUT ? wait_d + 7u : INF32;
                if constexpr (SYNC) {
                    if (__any(mode == B_SYNC)) {
                        const uint32_t maxkey = sync_maxkey();
                        if (mode == B_SYNC && is_part && maxkey != INF32) bound = maxkey + p.sync_latency + 5u;
                    }
                }
                const uint32_t gmin = group_reduce<0>(bound, C);
                const bool any_run_grp = group_bits(__ballot(mode == B_RUN), wl, C) != 0ull;
                uint32_t H = INF32;
                if (any_run_grp && gmin != INF32) {
                    const uint64_t h = (uint64_t)gmin + p.meas_latency - 1u;
                    H = h > INF32 ? INF32 : (uint32_t)h;
                }
                // nothing runs: every later measurement follows a release, i.e. a fire
                const bool stop_at_fire = !any_run_grp;
                // Every lane of a shot runs the merge and the FSM on
                // group-uniform values (no serial scan by a leader): the
                // shot's next measurement cycle is the DPP group minimum over
                // each lane's own next unmerged record, its valid / bit
                // vectors are ballots
                bool fired = false, busy = valid;            // busy: this shot still merges
                while (__any(busy)) {
                    const uint32_t e = lut_cur < (uint32_t)MT ? s_mt[lut_cur < (uint32_t)MT ? lut_cur : 0u][tid] : INF32;
                    const uint32_t my = e == INF32 ? INF32 : e >> 1;
                    const uint32_t tmin = group_reduce<0>(my, C);
                    busy = busy && tmin != INF32 && tmin <= H;
                    const bool hit = busy && my == tmin;
                    const uint64_t v = group_bits(__ballot(hit), wl, C);
                    const uint64_t mv = group_bits(__ballot(hit && (e & 1u)), wl, C);
                    lut_cur += hit ? 1u : 0u;
                    const bool upd = busy && !(lut_last_fire != INF32 && tmin == lut_last_fire + 1u);
                    const uint64_t nv = lut_valid | v, na = lut_addr | (v & mv);
                    const bool fire = upd && (((uint64_t)p.lut_mask & nv) == (uint64_t)p.lut_mask);
                    if (fire) {
                        if (nfire < (uint32_t)NF) {
                            const uint64_t o = p.lut_table[na & 0xFFu];
                            s_fire[nfire < (uint32_t)NF ? nfire : 0u][tid] = (tmin << 1) | (uint32_t)((o >> core) & 1ull);
                        }
                        lut_last_fire = tmin;
                        nfire++;
                        fired = true;
                    }
                    lut_valid = fire ? 0ull : upd ? nv : lut_valid;
                    lut_addr = fire ? 0ull : upd ? na : lut_addr;
                    busy = busy && !(fire && stop_at_fire);
                }
                const uint32_t nf_grp = nfire;               // the same in every lane of the shot
                const bool grp_fired = fired;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (mode == B_LUT) {
                    const uint32_t n = nf_grp < (uint32_t)NF ? nf_grp : (uint32_t)NF;
                    for (uint32_t k = 0; k < n; k++) {
                        const uint32_t f = s_fire[k][tid], tf = f >> 1;
                        if (tf >= wait_d + 1u) {
                            // the waiting alu_fproc / jump_fproc (ip has not moved)
                            const uint4 u2 = PLDS ? s_prog[fetch_off + min(ip, k_max)]
                                                  : p.fetch[(uint64_t)min(ip, k_max) * p.fetch_stride + fetch_off];
                            const uint32_t op2 = u2.y >> 28;
                            const uint32_t in0b = (u2.y & 8u) ? reg(u2.w >> 20) : u2.x;
                            const uint32_t outb = alu_eval(u2.y & 7u, in0b, f & 1u);
                            if (tf > max_cycles) {
                                finish(true, ST_MAX_CYCLES, wait_d);
                            } else if (op2 == 4u) {
                                const uint32_t rd = (u2.y >> 8) & 15u;
                                if constexpr (REGS) s_regs[rd][tid] = outb;
                                emit_trace(true, tf + 3u, rd, outb);
                                ip = (ip + 1u) & 0xFFFFu;
                                t = tf + 4u;
                                mode = B_RUN;
                            } else {
                                ip = (outb & 1u) ? (u2.z & 0xFFFFu) : ((ip + 1u) & 0xFFFFu);
                                t = tf + 6u;
                                mode = B_RUN;
                            }
                            lut_rel = true;
                            break;
                        }
                    }
                }
                lut_rel = lut_rel || (grp_fired && tid == leader_tid);
            }
            // a shot in which no lane retired or was released can never progress
            if (__any(mode == B_SYNC || mode == B_LUT)) {
                const uint64_t pm = __ballot(go || sync_rel || lut_rel);
                finish(group_bits(pm, wl, C) == 0ull && (mode == B_SYNC || mode == B_LUT), ST_DEADLOCK, wait_d);
            }
        }
        if constexpr (XMEAS) {   // this iteration's s_mt writes before the next iteration's reads
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        flush_rows(false);
        return __any(mode != B_FIN);
    };

    if (__any(mode != B_FIN) && iteration(std::true_type{})) {
        // internal-error guard: a correct run retires an instruction of >= 3
        // cycles in some lane of every live shot each iteration, so it never trips
        for (uint32_t iter = 2; iteration(std::false_type{});) {
            if (++iter > p.iter_guard) {
                flags |= mode != B_FIN ? F_GUARD : 0u;
                finish(mode != B_FIN, ST_DEADLOCK, t);
                break;
            }
        }
    }
    flush_rows(true);
    flags |= (n_ev > p.event_cap ? F_EVENT_OVF : 0u) | (n_meas > min(p.meas_cap, MEAS_LOOKUP) ? F_MEAS_OVF : 0u) |
             ((p.trace_cap && n_tr > p.trace_cap) ? F_TRACE_OVF : 0u);

    if (valid && p.summary) {
        const uint32_t qclk_end = t_end == 0u ? 0u : t_end + qoff;   // t_end = 0: finished in the reset hold
        write_summary(p, lane, t_end, ip, status, flags, n_ev, n_exec, qclk_end, n_meas, meas_bits, n_tr);
    }
    if (valid && p.regs_out) {
#pragma unroll
        for (int r = 0; r < 16; r++) p.regs_out[(uint64_t)r * n_lanes + lane] = reg(r);
    }
    count_outcome(p, s_hist, valid, core, grp, last_bit);
}

template <int F>
static hipError_t launch_branch_f(const KParams &p, uint32_t blocks, hipStream_t stream)
{
    const size_t shmem = ((F & FEAT_PROG_LDS) ? (size_t)p.prog_lds_words * sizeof(uint4) : 0) +
                         (p.hist_lds ? HIST_LDS_MAX * sizeof(uint32_t) : 0);
    if (p.C == 8) hipLaunchKernelGGL((branch_kernel<F, 8>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    else hipLaunchKernelGGL((branch_kernel<F, 0>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
