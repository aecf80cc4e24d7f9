// macro.hip -- the interpreter for branch-free programs with register
// commands (reg_alu, inc_qclk) on CDNA4 (gfx950): RB-like programs.
//
// A program with no jump, fproc or sync command never moves its instruction
// pointer except by +1 (hdl/instr_ptr.v without a jump), so its command
// sequence is fixed before it runs.  dpemu_load_programs re-packs every such
// program into MACROS of one fixed shape (capi.cpp build_macros):
//
//     [ALU slot 0][ALU slot 1][pulse slot]          32 B
//     [imm0][ctl 0-2 packed][imm1][imm2][pulse slot]   32 B (MACRO_W3)
//
// up to two (three: MACRO_W3, images that name at most 2 registers)
// consecutive reg_alu / inc_qclk commands followed by the next other command
// (pulse write / trigger, idle, pulse reset, done, hang), each slot marked
// present or absent.  Every lane still running in loop
// iteration m executes macro m of its own program, so a wave of lanes with
// DIFFERENT programs (a depth-200 RB table: ~7 sequences per wave) runs one
// code path per iteration -- two ALU slots, one pulse slot, selects for the
// absent ones -- instead of a divergent switch per command, and retires about
// two commands per iteration.  The command semantics are unchanged: every
// slot retires one command with hdl/ctrl.v's decode-to-decode latency
// (REG_ALU / INC_QCLK D+4, pulse commands D+3 or tT+3; oracle/fast_model.c),
// checks max_cycles at its own decode and counts as one instruction.
//
// Per lane: next-decode cycle t, qclk anchor (qa_t, qa_q), pulse register
// image, counters in VGPRs; the 16 x 32-bit reg_file in LDS as [reg][lane]
// (alu.v, reg_file.v).  Finished lanes keep walking with their state frozen by
// selects; branches guard only stores, LDS writes and philox.  Outputs and
// their layout are identical to interp_kernel's.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lane.h"

// cache policy of the macro-chunk LDS DMA (A/B builds only)
#ifndef DPEMU_MACRO_DMA_AUX
#define DPEMU_MACRO_DMA_AUX 0
#endif
// cache policy of macro_staged_kernel's event / measurement rows (A/B
// builds: bits 0-1 the events' StPolicy (lane.h), bit 2 measurements
// nontemporal)
#ifndef DPEMU_MACRO_NT
#define DPEMU_MACRO_NT 0
#endif

namespace dpemu {

constexpr StPolicy MACRO_EV_POLICY = (StPolicy)(DPEMU_MACRO_NT & 3);

// alu.v:20-50; le = sub[31] ^ overflow == signed a < b
__device__ __forceinline__ uint32_t alu_macro(uint32_t op, uint32_t a, uint32_t b)
{
    const uint32_t sub = a - b;
    const uint32_t lt = (int32_t)a < (int32_t)b;
    uint32_t r = a;                 // 0: id0
    r = (op == 1) ? a + b : r;
    r = (op == 2) ? sub : r;
    r = (op == 3) ? (uint32_t)(sub == 0) : r;
    r = (op == 4) ? lt : r;
    r = (op == 5) ? (lt ^ 1u) : r;
    r = (op == 6) ? b : r;
    r = (op == 7) ? 0u : r;
    return r;
}

// alu.v:20-50 as a select tree on op's bits (no per-op compares)
__device__ __forceinline__ uint32_t alu_eval(uint32_t op, uint32_t a, uint32_t b)
{
    const uint32_t sub = a - b;
    const uint32_t lt = (int32_t)a < (int32_t)b;
    const bool b0 = op & 1u, b1 = op & 2u;
    const uint32_t lo = b1 ? (b0 ? (uint32_t)(sub == 0u) : sub) : (b0 ? a + b : a);   // 0-3
    const uint32_t hi = b1 ? (b0 ? 0u : b) : (lt ^ (uint32_t)b0);                     // 4-7
    return (op & 4u) ? hi : lo;
}

// 6 waves per SIMD: the register budget of the prefetched loop (80 VGPRs);
// same-process A/B on config 4 (scripts/ab.py): 4.76 ms vs 5.05 without the
// prefetch and 6.7 when squeezed to 7 waves (spills)
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(6))) macro_kernel(const KParams p)
{
    __shared__ uint32_t s_hist[HIST_LDS_MAX];
    __shared__ uint32_t s_regs[16][BLOCK];
    __shared__ uint32_t s_key[BLOCK];
    const uint32_t tid = threadIdx.x;
    const uint32_t C = p.C;
    uint32_t sl, core;                                // shot within the run, core (core-major workgroup)
    clear_hist_next(p);
    block_core_major(p, sl, core);
    const bool valid = sl < p.n_shots;
    const uint32_t lane = out_lane(p, sl, core);      // output lane index (core-major)
    const uint32_t n_lanes = p.n_lanes;

    uint32_t mb = 0, ml = 0;
    if (valid) {
        const uint32_t grp = shot_group(p, sl);
        const uint32_t prog = p.prog_table[(uint64_t)grp * C + core];
        mb = p.macro_off[prog];
        ml = p.macro_off[prog + 1] - 1u;             // the terminal macro
    }
    if (p.hist_lds) {
        for (uint32_t i = tid; i < HIST_LDS_MAX; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 16; r++) s_regs[r][tid] = 0;

    const uint32_t max_cycles = p.max_cycles;
    const bool tr_on = p.trace != nullptr && p.trace_cap != 0u;
    uint32_t t = 0, pe = 0, pp = 0, pa = 0;            // next DECODE cycle; pulse register image
    uint32_t qa_t = 1, qa_q = 0;                       // qclk(t) = qa_q + t - qa_t for t >= qa_t; 0 before
    uint32_t flags = 0, n_ev = 0, n_meas = 0, meas_bits = 0, last_bit = 0, n_tr = 0;
    uint32_t k = 0;                                    // commands retired = ip (no jumps)
    // st: 0 while running, else the finish status (| ST_TOP: stopped by the
    // max_cycles check before a decode, so that command did not retire).  A
    // finish leaves t alone: t_end = t, ip = k
    constexpr uint32_t ST_TOP = 0x100u;
    uint32_t st = valid ? 0u : ST_DONE;

    // qclk at cycle x: 0 in the reset hold (only the first command decodes
    // there), qa_q + x - qa_t after it
    auto qclk_at = [&](uint32_t x) __attribute__((always_inline)) -> uint32_t { return x < qa_t ? 0u : qa_q + (x - qa_t); };

    // pulse_iface strobe(s) at cycle te (kind 0: trigger, 1: phase reset) for
    // lanes with `ok`, `reps` = 2 for the reset hold's double strobe (te and
    // te + 1); readout-element triggers draw the measurement.  Overflow flags
    // come from the final counts.
    auto emit = [&](bool ok, uint32_t te, uint32_t kind, uint32_t reps) __attribute__((always_inline)) {
        for (uint32_t r = 0; r < (ok ? reps : 0u); r++) {
            if (n_ev < p.event_cap && p.events)
                p.events[(uint64_t)n_ev * n_lanes + lane] = event_record(te + r, pe, pp, pa, kind);
            n_ev++;
            const bool is_meas = kind == 0u && ((pe >> 24) & 3u) == p.meas_elem;   // meas_elem 0xFF: none
            uint32_t bit = 0;
            if (is_meas) {
                // (shot and threshold re-derived here: few registers in the loop)
                bit = meas_bit(p, p.shot_begin + sl, core, n_meas, p.p1_thr[core], pa, pe);
                if (p.meas && n_meas < p.meas_cap)
                    p.meas[(uint64_t)n_meas * n_lanes + lane] = make_uint2(te + r + p.meas_latency, bit);
            }
            meas_bits |= (n_meas < 32u ? bit : 0u) << (n_meas & 31u);
            last_bit = is_meas ? bit : last_bit;
            n_meas += is_meas ? 1u : 0u;
        }
    };

    // register-sourced pulse fields: reg[rs0] ORed into the cleared fields
    // (decode_cmd clears them; no-op for other commands and absent slots)
    auto pulse_regs = [&](const uint4 u) __attribute__((always_inline)) {
        const uint32_t reg0 = s_regs[(u.w >> 20) & 15u][tid];
        pe |= (u.w & UOP_RS_ENV) ? (reg0 & 0xFFFFFFu) : 0u;
        pp |= (u.w & UOP_RS_PH) ? (reg0 & 0x1FFFFu) : 0u;
        pp |= (u.w & UOP_RS_FR) ? ((reg0 & 0x1FFu) << 17) : 0u;
        pa = (u.w & UOP_RS_AMP) ? (reg0 & 0xFFFFu) : pa;
    };

    // ---- ALU slot {imm, ctl}: ctl = present[31] inc_qclk[30] rs0[15:12]
    // rd[11:8] rs1[7:4] in0_reg[3] alu_op[2:0] (capi.cpp build_macros).
    // reg_alu: reg[rd] = alu(in0, reg[rs1]), next decode D + 4; inc_qclk:
    // qclk = alu(in0, qclk(D)) + 3 at D + 3 (qclk.v)
    auto alu_common = [&](bool ok, uint32_t D, uint32_t ctl, uint32_t out) __attribute__((always_inline)) {
        const bool is_q = (ctl >> 30) & 1u;
        const uint32_t rd = (ctl >> 8) & 15u;
        if (ok && !is_q) s_regs[rd][tid] = out;
        if (tr_on && ok && n_tr < p.trace_cap)
            p.trace[(uint64_t)n_tr * n_lanes + lane] =
                make_uint4(D + 3u, is_q ? TRACE_QCLK_LOAD : (uint32_t)(p.reg_inv >> (4 * rd)) & 15u, is_q ? out + 3u : out, 0u);
        n_tr += ok ? 1u : 0u;
        const bool load = ok && is_q;
        qa_t = load ? D + 3u : qa_t;
        qa_q = load ? out + 3u : qa_q;
        t = ok ? D + 4u : t;
        k += ok ? 1u : 0u;
    };
    // any lane state, any ALU command (the first command included: qclk clamp)
    auto alu_general = [&](uint32_t imm, uint32_t ctl) __attribute__((always_inline)) {
        const bool live = st == 0u && (int32_t)ctl < 0;
        const uint32_t D = t;
        const bool top = D > max_cycles;
        st = (live && top) ? (ST_MAX_CYCLES | ST_TOP) : st;
        const uint32_t reg0 = s_regs[(ctl >> 12) & 15u][tid];
        const uint32_t reg1 = s_regs[(ctl >> 4) & 15u][tid];
        const uint32_t in0 = (ctl & 8u) ? reg0 : imm;
        const uint32_t out = alu_macro(ctl & 7u, in0, ((ctl >> 30) & 1u) ? qclk_at(D) : reg1);
        alu_common(live && !top, D, ctl, out);
    };
    // ---- pulse slot: a decode_cmd word (kernels.h), w bit 31 = absent; any
    // command, the first included (reset hold: qclk(0) = qclk(1) = 0,
    // proc.sv:125-136; cmd_time 0 there strobes twice)
    auto pulse_slot = [&](const uint4 u) __attribute__((always_inline)) {
        const bool live = st == 0u && (int32_t)u.w >= 0;
        const uint32_t D = t;
        const uint32_t op4 = u.y >> 28;
        // opcode classes as bit tables: cmd_time wait 9/C, pulse class 8/9/B/C,
        // strobe 9/B.  decode_cmd leaves the write enables and register-source
        // bits of every other opcode zero, and absent slots have none, so the
        // pulse write is a no-op there
        const bool waits = (0x1200u >> op4) & 1u;
        const bool pulse_cls = (0x1B00u >> op4) & 1u;
        const bool strobe = (0x0A00u >> op4) & 1u;
        const uint32_t T = u.x;
        uint32_t wait = T - qclk_at(D);
        bool big = false, dbl = false;
        if (D < qa_t) {
            dbl = T == 0u;
            const uint64_t w64 = dbl ? 0ull : (uint64_t)(qa_t - D) + (uint32_t)(T - qa_q);
            wait = (uint32_t)w64;
            big = (w64 >> 32) != 0ull;
        }
        const bool top = D > max_cycles;
        const bool over = waits && (big || wait > max_cycles - D);
        flags |= (live && !top && waits && (big || wait >= 0x80000000u)) ? F_LATE : 0u;
        const uint32_t fin = top ? (ST_MAX_CYCLES | ST_TOP) : over ? ST_MAX_CYCLES
                           : pulse_cls ? 0u : (op4 >= 0xDu ? ST_HUNG_OPCODE : ST_DONE);
        st = live ? fin : st;
        const bool ok = live && fin == 0u;
        const uint32_t tT = D + (waits ? wait : 0u);
        pulse_write(u, pe, pp, pa);        // pulse_reg.sv:59-97: immediates, then reg[rs0]
        pulse_regs(u);                     // (a finished lane's registers no longer matter)
        const bool rst = op4 == 0xBu;
        const bool two = ok && dbl && op4 == 0x9u;
        flags |= two ? F_DOUBLE_STROBE : 0u;
        emit(ok && strobe, rst ? D : tT + 2u, rst ? 1u : 0u, two ? 2u : 1u);
        t = ok ? tT + 3u : t;
        k += (live && !top) ? 1u : 0u;     // a command that decoded retires, a stop included
    };

    // one ALU slot for the wave: skipped when no running lane has it; a scalar
    // switch on the ALU op when every running lane that has it holds a reg_alu
    // with the same op and none is past max_cycles (the batched shape); else
    // the general path
    auto alu_step = [&](uint32_t imm, uint32_t ctl) __attribute__((always_inline)) {
        const bool pres = st == 0u && (int32_t)ctl < 0;
        const uint64_t pm = __ballot(pres);
        if (!pm) return;
        const uint32_t key = ctl & 0x40000007u;              // inc_qclk | op
        const uint32_t key_u = __builtin_amdgcn_readlane(key, (int)__builtin_ctzll(pm));
        if (key_u & 0x40000000u || __ballot(pres && (key != key_u || t > max_cycles))) {
            alu_general(imm, ctl);
            return;
        }
        const uint32_t D = t;
        const uint32_t in0 = (ctl & 8u) ? s_regs[(ctl >> 12) & 15u][tid] : imm;
        const uint32_t b = s_regs[(ctl >> 4) & 15u][tid];
        uint32_t out;
        switch (key_u) {                                     // alu.v:20-50
        case 0: out = in0; break;
        case 1: out = in0 + b; break;
        case 2: out = in0 - b; break;
        case 3: out = (uint32_t)(in0 == b); break;
        case 4: out = (uint32_t)((int32_t)in0 < (int32_t)b); break;
        case 5: out = (uint32_t)((int32_t)in0 >= (int32_t)b); break;
        case 6: out = b; break;
        default: out = 0u; break;
        }
        alu_common(pres, D, ctl, out);
    };

    // one pulse slot for the wave: the pulse-trigger path (the RB shape) when
    // every running lane that has the slot holds a PULSE_WRITE_TRIG, is past
    // the reset hold and not past max_cycles; else the general path
    auto pulse_step = [&](const uint4 u) __attribute__((always_inline)) {
        const bool pres = st == 0u && (int32_t)u.w >= 0;
        if (__ballot(pres && ((u.y >> 28) != 0x9u || t > max_cycles || t < qa_t))) {
            pulse_slot(u);
            return;
        }
        const uint32_t D = t;
        const uint32_t wait = u.x - (qa_q + (D - qa_t));
        const bool stop = pres && wait > max_cycles - D;     // includes every late cmd_time (wait >= 2^31)
        flags |= (stop && wait >= 0x80000000u) ? F_LATE : 0u;
        st = stop ? ST_MAX_CYCLES : st;
        const bool ok = pres && !stop;
        const uint32_t tT = D + wait;
        pulse_write(u, pe, pp, pa);                          // absent / finished lanes: no enables, or frozen
        pulse_regs(u);
        emit(ok, tT + 2u, 0u, 1u);
        t = ok ? tT + 3u : t;
        k += pres ? 1u : 0u;
    };

    // macro m of this lane's program (ALU slots, pulse slot); in bounds: the
    // terminal macro repeats
    const uint4 *mbase = p.macros;
    auto addr = [&](uint32_t m) __attribute__((always_inline)) -> const uint4 * { return mbase + 2ull * min(mb + m, ml); };

    // one macro ahead: macro m + 1 is in flight while macro m executes
    uint4 an = addr(0u)[0], un = addr(0u)[1];
    for (uint32_t m = 1; __ballot(st == 0u); m++) {
        const uint4 a = an, u = un;
        {
            const uint4 *q = addr(m);                   // the next macro: in flight during this one
            an = q[0];
            un = q[1];
        }
        // the ALU slots: three with ctl packed in a.y (MACRO_W3, uniform), else
        // two; one copy of the slot code in a rolled loop (three inlined
        // copies left the kernel's lambda state in scratch: 4.4 -> 44 ms on
        // config 4 through this kernel)
        const uint32_t n_alu = p.macro_w3 ? 3u : 2u;
#pragma unroll 1
        for (uint32_t s = 0; s < n_alu; s++) {
            const uint32_t imm = s == 0u ? a.x : s == 1u ? a.z : a.w;
            const uint32_t ctl = p.macro_w3 ? w3_ctl(a.y, (int)s) : (s == 0u ? a.y : a.w);
            alu_step(imm, ctl);
        }
        pulse_step(u);
    }
    flags |= (n_ev > p.event_cap ? F_EVENT_OVF : 0u) | (n_meas > min(p.meas_cap, MEAS_LOOKUP) ? F_MEAS_OVF : 0u) |
             (p.trace_cap && n_tr > p.trace_cap ? F_TRACE_OVF : 0u);

    if (valid && p.summary) {
        // ip = index of the finishing command; it retired unless stopped before its decode
        const uint32_t ip = (st & ST_TOP) ? k : k - 1u;
        write_summary(p, lane, t, ip, st & 0xFFu, flags, n_ev, k, qclk_at(t), n_meas, meas_bits, n_tr);
    }
    if (valid && p.regs_out) {
#pragma unroll
        for (int r = 0; r < 16; r++)
            p.regs_out[(uint64_t)r * n_lanes + lane] = ((p.reg_used >> r) & 1u) ? s_regs[(p.reg_map >> (4 * r)) & 15u][tid] : 0u;
    }
    count_outcome_block(p, s_hist, s_key, valid, core, sl, valid ? shot_group(p, sl) : 0u, last_bit);
}

// ---------------------------------------------------------------------------
// macro_staged_kernel<NR>: the same macro loop with the program memory STAGED
// IN LDS per wave (the cmd_mem analogue, sim_modules/toplevel_sim.sv:5) and
// the register file in VGPRs.
//
// A wave's 64 lanes run at most MACRO_SLOTS distinct programs (config 4:
// 64 consecutive shots of one core, 10 shots per RB sequence -> <= 8; the
// host checks the bound for the run's lane order and shots_per_group).  The
// wave assigns each distinct program a slot, and streams the programs'
// macros through a per-wave LDS chunk of MACRO_SLOTS x MACRO_CHUNK macros
// (2 KiB): every lane loads two 16-B pieces of the NEXT chunk into VGPRs
// while the wave executes the current chunk from LDS, and writes them to
// LDS at the chunk boundary.  A lane's macro fetch is then an LDS read, and
// the global loads -- which on gfx950 share vmcnt with the event stores, so
// the wait for a load also waits for every earlier store -- are waited for
// once per MACRO_CHUNK iterations instead of every iteration (macro_kernel
// fetches one macro ahead per lane).
//
// NR: register slots the macro image names (capi.cpp remaps the reg_file
// indices of the macro image to slots; RB programs name 2): NR = 2 keeps
// them in VGPRs (a select instead of an LDS round trip per access), NR = 16
// the [16][lane] LDS file.  Semantics, outputs and layout are
// macro_kernel's (hdl/alu.v, ctrl.v latencies; oracle/fast_model.c).
//
// The lane state is one struct with inlined member functions rather than
// nested lambdas: lambdas that call lambdas that capture by reference left
// their closures (and a copy of the kernel arguments) in scratch memory
// here -- 848 B per lane, every access a scratch round trip under vmcnt.

template <int NR, bool ADDID>
struct MacroLane {
    // NR == 2 images are MACRO_W3 (capi.cpp: three ALU slots whenever the
    // image names at most 2 registers); their last ALU slot decodes at t + 8,
    // the pulse slot at t + 12 (t + 4 / t + 8 with two slots)
    static constexpr bool W3 = NR == 2;
    static constexpr uint32_t SPAN = W3 ? 12u : 8u;
    const KParams &p;
    uint32_t *s_regs_lane;                 // NR == 16: &s_regs[0][tid], stride BLOCK
    uint32_t lane, sl, core;
    uint32_t rg[NR == 16 ? 2 : NR];          // (NR == 16: unused)
    uint32_t t, pe, pp, pa, qa_t, qa_q;
    uint32_t flags, n_ev, n_meas, meas_bits, last_bit, n_tr, k, st;
    uint4 *evp;                            // event slot n_ev of this lane
    bool tr_on, ev_on;
    static constexpr uint32_t ST_TOP = 0x100u;

    __device__ __forceinline__ MacroLane(const KParams &p_, uint32_t *srl, uint32_t lane_, uint32_t sl_,
                                         uint32_t core_, bool valid)
        : p(p_), s_regs_lane(srl), lane(lane_), sl(sl_), core(core_)
    {
#pragma unroll
        for (int r = 0; r < (NR == 16 ? 2 : NR); r++) rg[r] = 0;
        t = pe = pp = pa = 0;
        qa_t = 1; qa_q = 0;
        flags = n_ev = n_meas = meas_bits = last_bit = n_tr = k = 0;
        st = valid ? 0u : ST_DONE;
#ifdef DPEMU_PROBE_WAVEBLOCK
        // probe: a wave's records in one contiguous block, slot-major within
        // it (outputs differ by design)
        evp = p.events + (uint64_t)(lane >> 6) * 64u * p.event_cap + (lane & 63u);
#else
        evp = p.events + lane;
#endif
        tr_on = p.trace != nullptr && p.trace_cap != 0u;
        ev_on = p.events != nullptr;
    }

    __device__ __forceinline__ uint32_t reg_rd(uint32_t i) const
    {
        if constexpr (NR == 16) {
            return s_regs_lane[(i & 15u) * BLOCK];
        } else {
            uint32_t v = rg[0];
#pragma unroll
            for (int r = 1; r < NR; r++) v = (i == (uint32_t)r) ? rg[r] : v;
            return v;
        }
    }
    __device__ __forceinline__ void reg_wr(bool ok, uint32_t i, uint32_t v)
    {
        if constexpr (NR == 16) {
            if (ok) s_regs_lane[(i & 15u) * BLOCK] = v;
        } else {
#pragma unroll
            for (int r = 0; r < NR; r++) rg[r] = (ok && i == (uint32_t)r) ? v : rg[r];
        }
    }
    // qclk at cycle x: 0 in the reset hold, qa_q + x - qa_t after it
    __device__ __forceinline__ uint32_t qclk_at(uint32_t x) const { return x < qa_t ? 0u : qa_q + (x - qa_t); }

    // one pulse_iface strobe at te (kind 0 trigger, 1 phase reset); readout
    // triggers draw the outcome
    __device__ __forceinline__ void emit1(bool ok, uint32_t te, uint32_t kind)
    {
        if (ok) {
            if (n_ev < p.event_cap && ev_on) {
                const uint4 rec = event_record(te, pe, pp, pa, kind);
                if (p.ev_stream) st_rec<ST_NT_WAVE>(evp, rec);   // DPEMU_X_STREAM_EVENTS (uniform)
                else st_rec<MACRO_EV_POLICY>(evp, rec);
            }
#ifdef DPEMU_PROBE_WAVEBLOCK
            evp += 64u;
#else
            evp += p.n_lanes;
#endif
            n_ev++;
            if (kind == 0u && ((pe >> 24) & 3u) == p.meas_elem) {        // meas_elem 0xFF: none
                const uint32_t bit = meas_bit(p, p.shot_begin + sl, core, n_meas, p.p1_thr[core], pa, pe);
                if (p.meas && n_meas < p.meas_cap)
                    st_out(&p.meas[(uint64_t)n_meas * p.n_lanes + lane], make_uint2(te + p.meas_latency, bit),
                           (DPEMU_MACRO_NT & 4) != 0);
                meas_bits |= (n_meas < 32u ? bit : 0u) << (n_meas & 31u);
                last_bit = bit;
                n_meas++;
            }
        }
    }
    // register-sourced pulse fields (decode_cmd cleared them)
    __device__ __forceinline__ void pulse_regs(const uint4 u)
    {
        if (u.w & UOP_ANY_RS) {
            const uint32_t reg0 = reg_rd((u.w >> 20) & 15u);
            pe |= (u.w & UOP_RS_ENV) ? (reg0 & 0xFFFFFFu) : 0u;
            pp |= (u.w & UOP_RS_PH) ? (reg0 & 0x1FFFFu) : 0u;
            pp |= (u.w & UOP_RS_FR) ? ((reg0 & 0x1FFu) << 17) : 0u;
            pa = (u.w & UOP_RS_AMP) ? (reg0 & 0xFFFFu) : pa;
        }
    }
    // ALU slot {imm, ctl}: reg_alu reg[rd] = alu(in0, reg[rs1]) next decode
    // D + 4; inc_qclk qclk = alu(in0, qclk(D)) + 3 at D + 3 (qclk.v)
    __device__ __forceinline__ void alu_common(bool ok, uint32_t D, uint32_t ctl, uint32_t out)
    {
        const bool is_q = (ctl >> 30) & 1u;
        const uint32_t rd = (ctl >> 8) & 15u;
        reg_wr(ok && !is_q, rd, out);
        if (tr_on && ok && n_tr < p.trace_cap)
            p.trace[(uint64_t)n_tr * p.n_lanes + lane] =
                make_uint4(D + 3u, is_q ? TRACE_QCLK_LOAD : (uint32_t)(p.reg_inv >> (4 * rd)) & 15u,
                           is_q ? out + 3u : out, 0u);
        n_tr += ok ? 1u : 0u;
        const bool load = ok && is_q;
        qa_t = load ? D + 3u : qa_t;
        qa_q = load ? out + 3u : qa_q;
        t = ok ? D + 4u : t;
        k += ok ? 1u : 0u;
    }
    __device__ __forceinline__ void alu_general(uint32_t imm, uint32_t ctl)
    {
        const bool live = st == 0u && (int32_t)ctl < 0;
        const uint32_t D = t;
        const bool top = D > p.max_cycles;
        st = (live && top) ? (ST_MAX_CYCLES | ST_TOP) : st;
        const uint32_t reg0 = reg_rd((ctl >> 12) & 15u);
        const uint32_t reg1 = reg_rd((ctl >> 4) & 15u);
        const uint32_t in0 = (ctl & 8u) ? reg0 : imm;
        const uint32_t out = alu_macro(ctl & 7u, in0, ((ctl >> 30) & 1u) ? qclk_at(D) : reg1);
        alu_common(live && !top, D, ctl, out);
    }
    // the wave's ALU slot: skipped when no running lane has it; a scalar
    // switch when every running lane that has it holds a reg_alu with the
    // same op and none is past max_cycles; else the general path
    __device__ __forceinline__ void alu_step(uint32_t imm, uint32_t ctl)
    {
        const bool pres = st == 0u && (int32_t)ctl < 0;
        const uint64_t pm = __ballot(pres);
        if (!pm) return;
        const uint32_t key = ctl & 0x40000007u;
        const uint32_t key_u = __builtin_amdgcn_readlane(key, (int)__builtin_ctzll(pm));
        if (key_u & 0x40000000u || __ballot(pres && (key != key_u || t > p.max_cycles))) {
            alu_general(imm, ctl);
            return;
        }
        // the batched shape: every present lane runs a reg_alu with op key_u
        // within max_cycles.  Operands are read only where the op and the
        // lanes' forms need them (uniform tests), the result written to rd,
        // the register trace only when it is on
        const uint32_t D = t;
        uint32_t in0 = imm;
        if (__ballot(pres && (ctl & 8u))) in0 = (ctl & 8u) ? reg_rd((ctl >> 12) & 15u) : imm;
        const uint32_t b = (key_u == 0u || key_u == 7u) ? 0u : reg_rd((ctl >> 4) & 15u);
        uint32_t out;
        switch (key_u) {                                     // alu.v:20-50
        case 0: out = in0; break;
        case 1: out = in0 + b; break;
        case 2: out = in0 - b; break;
        case 3: out = (uint32_t)(in0 == b); break;
        case 4: out = (uint32_t)((int32_t)in0 < (int32_t)b); break;
        case 5: out = (uint32_t)((int32_t)in0 >= (int32_t)b); break;
        case 6: out = b; break;
        default: out = 0u; break;
        }
        const uint32_t rd = (ctl >> 8) & 15u;
        reg_wr(pres, rd, out);
        if (tr_on && pres && n_tr < p.trace_cap)
            p.trace[(uint64_t)n_tr * p.n_lanes + lane] = make_uint4(D + 3u, (uint32_t)(p.reg_inv >> (4 * rd)) & 15u, out, 0u);
        n_tr += pres ? 1u : 0u;
        t = pres ? D + 4u : t;
        k += pres ? 1u : 0u;
    }
    // pulse slot (a decode_cmd word, w bit 31 = absent): any command, the
    // first included (reset hold: qclk(0) = qclk(1) = 0, proc.sv:125-136;
    // cmd_time 0 there strobes twice)
    __device__ __forceinline__ void pulse_general(const uint4 u)
    {
        const bool live = st == 0u && (int32_t)u.w >= 0;
        const uint32_t D = t;
        const uint32_t op4 = u.y >> 28;
        const bool waits = (0x1200u >> op4) & 1u;
        const bool pulse_cls = (0x1B00u >> op4) & 1u;
        const bool strobe = (0x0A00u >> op4) & 1u;
        const uint32_t T = u.x;
        uint32_t wait = T - qclk_at(D);
        bool big = false, dbl = false;
        if (D < qa_t) {
            dbl = T == 0u;
            const uint64_t w64 = dbl ? 0ull : (uint64_t)(qa_t - D) + (uint32_t)(T - qa_q);
            wait = (uint32_t)w64;
            big = (w64 >> 32) != 0ull;
        }
        const uint32_t max_cycles = p.max_cycles;
        const bool top = D > max_cycles;
        const bool over = waits && (big || wait > max_cycles - D);
        flags |= (live && !top && waits && (big || wait >= 0x80000000u)) ? F_LATE : 0u;
        const uint32_t fin = top ? (ST_MAX_CYCLES | ST_TOP) : over ? ST_MAX_CYCLES
                           : pulse_cls ? 0u : (op4 >= 0xDu ? ST_HUNG_OPCODE : ST_DONE);
        st = live ? fin : st;
        const bool ok = live && fin == 0u;
        const uint32_t tT = D + (waits ? wait : 0u);
        pulse_write(u, pe, pp, pa);
        pulse_regs(u);
        const bool rst = op4 == 0xBu;
        const bool two = ok && dbl && op4 == 0x9u;
        flags |= two ? F_DOUBLE_STROBE : 0u;
        emit1(ok && strobe, rst ? D : tT + 2u, rst ? 1u : 0u);
        emit1(two, tT + 3u, 0u);
        t = ok ? tT + 3u : t;
        k += (live && !top) ? 1u : 0u;
    }
    // the wave's pulse slot: the trigger path (the RB shape) when every
    // running lane that has the slot holds a PULSE_WRITE_TRIG past the reset
    // hold and within max_cycles; else the general path
    __device__ __forceinline__ void pulse_step(const uint4 u)
    {
        const bool pres = st == 0u && (int32_t)u.w >= 0;
        if (__ballot(pres && ((u.y >> 28) != 0x9u || t > p.max_cycles || t < qa_t))) {
            pulse_general(u);
            return;
        }
        const uint32_t D = t;
        const uint32_t wait = u.x - (qa_q + (D - qa_t));
        const bool stop = pres && wait > p.max_cycles - D;   // includes every late cmd_time (wait >= 2^31)
        if (__ballot(stop)) {
            flags |= (stop && wait >= 0x80000000u) ? F_LATE : 0u;
            st = stop ? ST_MAX_CYCLES : st;
        }
        const bool ok = pres && !stop;
        const uint32_t tT = D + wait;
        pulse_write(u, pe, pp, pa);
        if (__ballot(pres && (u.w & UOP_ANY_RS))) pulse_regs(u);
        emit1(ok, tT + 2u, 0u);
        t = ok ? tT + 3u : t;
        k += pres ? 1u : 0u;
    }

    // ---- the RB-shape iteration: ONE wave-uniform test for the whole macro
    // (simple_ok), then all three slots branch-free, written through selects.
    // Holds when every running lane is past the reset hold, at least 8 cycles
    // inside max_cycles (so no slot can be stopped before its decode), its
    // ALU slots hold reg_alu (not inc_qclk), its pulse slot (if present) a
    // PULSE_WRITE_TRIG, and no register trace is requested: then the slots
    // retire exactly as alu_step / pulse_step would, without their per-slot
    // ballots and the uniform-op switch (a chain of scalar branches).
    __device__ __forceinline__ bool simple_ok(const uint4 a, const uint4 u) const
    {
        // an inc_qclk in a present ALU slot (W3: present and inc_qclk bits of the three packed fields)
        constexpr uint32_t PRES3 = (1u << W3_PRES) | (1u << (10 + W3_PRES)) | (1u << (20 + W3_PRES));
        const bool inc = W3 ? ((a.y & (a.y << (W3_PRES - W3_INC)) & PRES3) != 0u)
                            : (((int32_t)a.y < 0 && (a.y & 0x40000000u)) || ((int32_t)a.w < 0 && (a.w & 0x40000000u)));
        const bool bad = inc || ((int32_t)u.w >= 0 && (u.y >> 28) != 0x9u) || t < qa_t || t + SPAN > p.max_cycles;
        return !tr_on && !__ballot(st == 0u && bad);
    }
    __device__ __forceinline__ void alu_simple(uint32_t imm, uint32_t ctl)
    {
        const bool pres = st == 0u && (int32_t)ctl < 0;
        const uint32_t in0 = (ctl & 8u) ? reg_rd((ctl >> 12) & 15u) : imm;
        const uint32_t out = alu_eval(ctl & 7u, in0, reg_rd((ctl >> 4) & 15u));
        reg_wr(pres, (ctl >> 8) & 15u, out);
        n_tr += pres ? 1u : 0u;
        t = pres ? t + 4u : t;
        k += pres ? 1u : 0u;
    }
    // ---- the lean path (NR == 2, registers r0 / r1 in VGPRs): the macro
    // carries MACRO_SIMPLE (capi.cpp: not a program's first, so past the
    // reset hold; reg_alu ALU slots; a PULSE_WRITE_TRIG or no pulse slot) and
    // every running lane is SPAN (12) cycles or more inside max_cycles, no trace.  The
    // remapped register fields are one bit each (slot 0 / 1), so operand
    // selection and the register write are v_bfe_i32 masks and v_bitop3
    // selects, and the counters advance by masks (k - pm: +1 where present)
    __device__ __forceinline__ bool lean_ok(const uint4 u) const
    {
        return !tr_on && !__ballot(st == 0u && (!(u.w & MACRO_SIMPLE) || t + SPAN > p.max_cycles));
    }
    // ---- the lean CHUNK (NR == 2): one wave-uniform test for MACRO_CHUNK
    // macros.  `info` is the lane's chunk marker (capi.cpp mark_lean_chunks):
    // every macro MACRO_SIMPLE, the largest pulse cmd_time Tmax.  Within the
    // chunk qa is fixed (no inc_qclk), an ALU slot adds 4 cycles and a pulse
    // that does not stop the lane ends at Tc + 3 with Tc = its cmd_time +
    // qa_t - qa_q >= its decode, so by induction macro m starts at or before
    // B + 11 m, B = max(t, Tmax + qa_t - qa_q): B + 11 (CH - 1) + 8 <=
    // max_cycles keeps every macro's decodes inside max_cycles (W3: 15 m and
    // B + 15 (CH - 1) + 12; 16 CH + 8 bounds both) -- lean_ok at
    // every macro, without testing it.  (A late pulse stops its lane, which
    // the lean pulse slot handles.)  The argument holds while qclk cannot
    // wrap before max_cycles (qa_q + max_cycles - qa_t < 2^32): then a
    // cmd_time below qclk(D) waits past max_cycles and stops the lane; after a
    // wrap (an inc_qclk by a negative value) a small cmd_time would fire
    // later than B, so such lanes take the per-macro tests.
    __device__ __forceinline__ bool lean_chunk_ok(uint32_t info) const
    {
        const uint64_t tc = (uint64_t)info + qa_t;                       // Tmax's cycle + qa_q
        const uint64_t b = max((uint64_t)t, tc > qa_q ? tc - qa_q + 3u : 0ull);
        const bool no_wrap = (uint64_t)qa_q + p.max_cycles < (1ull << 32) + qa_t;
        const bool ok = info != MACRO_CHUNK_MIXED && no_wrap && b + (W3 ? 16ull : 12ull) * MACRO_CHUNK + 8u <= p.max_cycles;
        return !tr_on && !__ballot(st == 0u && !ok);
    }
    static __device__ __forceinline__ uint32_t bmask(uint32_t v, int b)     // bit b of v as 0 / ~0
    {
        return (uint32_t)(((int32_t)(v << (31 - b))) >> 31);
    }
    // ALU slot K of a MACRO_W3 macro (its packed ctl field at bit 10 K)
    template <int K>
    __device__ __forceinline__ void alu_lean_w3(uint32_t run, uint32_t imm, uint32_t pk)
    {
        constexpr int B = 10 * K;
        const uint32_t pm = run & bmask(pk, B + W3_PRES);
        const uint32_t in0 = bit_select(bmask(pk, B + W3_IN0), bit_select(bmask(pk, B + W3_RS0), rg[1], rg[0]), imm);
        const uint32_t b = bit_select(bmask(pk, B + W3_RS1), rg[1], rg[0]);
        const uint32_t out = ADDID ? in0 + (b & bmask(pk, B + W3_OP)) : alu_eval((pk >> B) & 7u, in0, b);
        const uint32_t wm = bmask(pk, B + W3_RD);
        rg[1] = bit_select(pm & wm, out, rg[1]);
        rg[0] = bit_select(pm & ~wm, out, rg[0]);
        t += pm & 4u;
        k -= pm;
        n_tr -= pm;
    }
    // one lean macro: its ALU slots (the third only when some running lane
    // has one: ~3 % of an RB image's macros), then the pulse slot
    __device__ __forceinline__ void macro_lean(const uint4 a, const uint4 u)
    {
        static_assert(W3, "the lean path is NR == 2 = MACRO_W3 only");
        const uint32_t run = st == 0u ? ~0u : 0u;
        alu_lean_w3<0>(run, a.x, a.y);
        alu_lean_w3<1>(run, a.z, a.y);
        if (__ballot(run != 0u && ((a.y >> (20 + W3_PRES)) & 1u))) alu_lean_w3<2>(run, a.w, a.y);
        pulse_lean(run, u);
    }
    __device__ __forceinline__ void pulse_lean(uint32_t run, const uint4 u)
    {
        const bool pres = run != 0u && (int32_t)u.w >= 0;
        const uint32_t D = t;
        const uint32_t wait = u.x - (qa_q + (D - qa_t));
        const bool stop = pres && wait > p.max_cycles - D;   // includes every late cmd_time (wait >= 2^31)
        flags |= (stop && wait >= 0x80000000u) ? F_LATE : 0u;
        st = stop ? ST_MAX_CYCLES : st;
        const bool ok = pres && !stop;
        pulse_write(u, pe, pp, pa);
        // register-sourced fields (decode_cmd cleared them), only those the image uses
        const uint32_t rs = p.macro_rs;
        if (rs) {
            const uint32_t reg0 = bit_select(bmask(u.w, 20), rg[1], rg[0]);
            if (rs & UOP_RS_ENV) pe |= reg0 & bmask(u.w, 16) & 0xFFFFFFu;
            if (rs & UOP_RS_PH) pp |= reg0 & bmask(u.w, 17) & 0x1FFFFu;
            if (rs & UOP_RS_FR) pp |= (reg0 << 17) & bmask(u.w, 18) & (0x1FFu << 17);
            if (rs & UOP_RS_AMP) pa = bit_select(bmask(u.w, 19), reg0 & 0xFFFFu, pa);
        }
        emit1(ok, D + wait + 2u, 0u);
        t = ok ? D + wait + 3u : t;
        k += pres ? 1u : 0u;
    }

    __device__ __forceinline__ void pulse_simple(const uint4 u)
    {
        const bool pres = st == 0u && (int32_t)u.w >= 0;
        const uint32_t D = t;
        const uint32_t wait = u.x - (qa_q + (D - qa_t));
        const bool stop = pres && wait > p.max_cycles - D;   // includes every late cmd_time (wait >= 2^31)
        flags |= (stop && wait >= 0x80000000u) ? F_LATE : 0u;
        st = stop ? ST_MAX_CYCLES : st;
        const bool ok = pres && !stop;
        pulse_write(u, pe, pp, pa);
        const uint32_t reg0 = reg_rd((u.w >> 20) & 15u);     // register-sourced fields (cleared by decode_cmd)
        pe |= (u.w & UOP_RS_ENV) ? (reg0 & 0xFFFFFFu) : 0u;
        pp |= (u.w & UOP_RS_PH) ? (reg0 & 0x1FFFFu) : 0u;
        pp |= (u.w & UOP_RS_FR) ? ((reg0 & 0x1FFu) << 17) : 0u;
        pa = (u.w & UOP_RS_AMP) ? (reg0 & 0xFFFFu) : pa;
        emit1(ok, D + wait + 2u, 0u);
        t = ok ? D + wait + 3u : t;
        k += pres ? 1u : 0u;
    }
};

#ifdef DPEMU_PROBE_WAVETIME
// probe builds only (scripts/wavetime_probe.py): per wave, its start and end on
// the 100-MHz wall clock, HW_ID and XCC_ID, so the occupancy of the launch over
// time (its tail) can be read back
__device__ uint32_t g_wavetime[4u << 18];
__device__ __forceinline__ void probe_wavetime(uint32_t t0, uint32_t wv)
{
    const uint32_t w = blockIdx.x * (BLOCK / 64) + wv;
    if ((threadIdx.x & 63) == 0 && w < (1u << 18)) {
        const uint32_t t1 = (uint32_t)wall_clock64();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        *(uint4 *)&g_wavetime[4u * w] = make_uint4(t0, t1, hw, xcc);
    }
}
extern "C" int dpemu_probe_wavetime(void *dst, size_t bytes, int reset)
{
    if (reset) {
        void *a = nullptr;
        if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_wavetime)) != hipSuccess) return -1;
        return hipMemset(a, 0, sizeof(g_wavetime)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wavetime), bytes < sizeof(g_wavetime) ? bytes : sizeof(g_wavetime)) ==
                   hipSuccess ? 0 : -1;
}
#endif

// NSL: program slots per wave -- MACRO_SLOTS, or MACRO_SLOTS_WIDE (NR == 2
// only) for runs whose waves span more programs (fewer shots per program);
// the wide chunks (48 KiB per workgroup) hold 3 workgroups per CU
template <int NR, bool ADDID, int NSL>
__global__ void __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(NR == 16 || NSL > (int)MACRO_SLOTS ? 3 : 4))) macro_staged_kernel(const KParams p)
{
    constexpr uint32_t NW = BLOCK / 64, CH = MACRO_CHUNK, NS = NSL;
    constexpr uint32_t PIECES = NS * CH * 2;          // 16-B pieces of a chunk
    constexpr uint32_t PL = PIECES / 64;              // pieces per lane
    static_assert(PIECES % 64 == 0 && (CH & (CH - 1)) == 0, "whole pieces per lane, power-of-two chunk");
    // the staging loop maps lane wl to macro (wl >> 1) & (CH - 1) in every load
    // round, which is the round's macro only while a round covers <= CH macros
    static_assert(CH <= 32, "staging assumes at most 32 macros per chunk");
    __shared__ uint4 s_chunk0[NW][PIECES];            // [wave][slot][macro][2], double-buffered
    __shared__ uint4 s_chunk1[NW][PIECES];
    __shared__ uint32_t s_smb[NW][NS], s_sml[NW][NS]; // slot -> first / terminal macro
    __shared__ uint32_t s_scb[NW][NS];                // slot -> its first lean-chunk marker (macro_coff)
    __shared__ uint32_t s_info0[NW][NS], s_info1[NW][NS];   // the staged chunk's markers, per slot
    __shared__ uint32_t s_regs[NR == 16 ? 16 : 1][NR == 16 ? BLOCK : 1];
    __shared__ uint32_t s_key[BLOCK];
    extern __shared__ uint32_t s_hist[];              // HIST_LDS_MAX words when p.hist_lds (dynamic)
    const uint32_t tid = threadIdx.x, wv = tid >> 6, wl = tid & 63;
    const uint32_t C = p.C;
#ifdef DPEMU_PROBE_WAVETIME
    const uint32_t pt0 = (uint32_t)wall_clock64();
#endif
    uint32_t sl, core;
    clear_hist_next(p);
    block_core_major(p, sl, core);
    const bool valid = sl < p.n_shots;
    const uint32_t lane = out_lane(p, sl, core);

    uint32_t prog = 0, mb = 0, ml = 0, cb = 0;
    if (valid) {
        const uint32_t grp = shot_group(p, sl);
        prog = p.prog_table[(uint64_t)grp * C + core];
        mb = p.macro_off[prog];
        ml = p.macro_off[prog + 1] - 1u;
        if constexpr (NR == 2) cb = p.macro_coff[prog];
    }
    if (p.hist_lds) {
        for (uint32_t i = tid; i < HIST_LDS_MAX; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
    }
    if constexpr (NR == 16) {
#pragma unroll
        for (int r = 0; r < 16; r++) s_regs[r][tid] = 0;
    }
    MacroLane<NR, ADDID> L(p, NR == 16 ? &s_regs[0][tid] : nullptr, lane, sl, core, valid);

    // ---- the wave's distinct programs -> slots (a uniform waterfall) ----
    uint32_t slot = 0, nslots = 0;
    {
        uint64_t rem = __ballot(valid);
        while (rem) {
            const int ld = (int)__builtin_ctzll(rem);
            const uint32_t lp = __builtin_amdgcn_readlane(prog, ld);
            const bool mine = valid && prog == lp;
            if (mine) slot = nslots;
            if (wl == 0 && nslots < NS) {
                s_smb[wv][nslots] = __builtin_amdgcn_readlane(mb, ld);
                s_sml[wv][nslots] = __builtin_amdgcn_readlane(ml, ld);
                s_scb[wv][nslots] = __builtin_amdgcn_readlane(cb, ld);
            }
            rem &= ~__ballot(mine);
            nslots++;
        }
    }
    // more programs than slots: the host's bound was wrong (internal error):
    // those lanes share slot NS - 1's macros, their outputs are flagged
    L.flags |= slot >= NS ? F_GUARD : 0u;
    slot = min(slot, NS - 1u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // chunk c of every slot (macros [c CH, (c + 1) CH), the terminal macro
    // repeating) goes global -> LDS directly (global_load_lds_dwordx4: no
    // VGPRs hold it in flight), into the buffer the wave is NOT reading; lane
    // wl of load instruction r fetches piece e = r * 64 + wl = slot e / 16,
    // macro (e / 2) % 8, half e % 2 (the LDS image is lane-linear)
    // piece r of this lane: e = r * 64 + wl = slot e / (2 CH), macro (e / 2) % CH, half e % 2
    const uint32_t pj = (wl >> 1) & (CH - 1u), ph = wl & 1u;
    const uint4 *const mbase = p.macros;
    // Only the lanes of the wave's nslots slots load (s_smb / s_sml of the
    // others were never written -- all of them in a wave with no valid lane);
    // the other pieces of the LDS image are never read.
    // (NR == 2: lane sr < nslots also fetches slot sr's lean-chunk marker of
    // chunk c, clamped to the program's last chunk, into info[sr])
    auto stage = [&](uint32_t c, uint4 *buf, uint32_t *info) __attribute__((always_inline)) {
        const uint32_t m = c * CH + pj;
#pragma unroll
        for (uint32_t r = 0; r < PL; r++) {
            const uint32_t sr = (r * 64u + wl) / (2u * CH);
            if (sr < nslots) {
                const uint32_t b0 = s_smb[wv][sr], l0 = s_sml[wv][sr];
                __builtin_amdgcn_global_load_lds(mbase + 2ull * min(b0 + m, l0) + ph, buf + r * 64u, 16, 0, DPEMU_MACRO_DMA_AUX);
            }
        }
        if constexpr (NR == 2) {
            if (wl < min(nslots, NS)) {
                const uint32_t ci = min(c, (s_sml[wv][wl] - s_smb[wv][wl]) / CH);
                __builtin_amdgcn_global_load_lds(p.macro_chunk + s_scb[wv][wl] + ci, info, 4, 0, 0);
            }
        }
    };
    const uint32_t moff = slot * (CH * 2);
    // the chunk loop, two phases per round so every LDS read names one
    // buffer statically (the compiler then needs no vmcnt wait for the DMA
    // into the other): phase A executes chunk c from s_chunk0 while chunk
    // c + 1 streams into s_chunk1, phase B the reverse.  A phase always runs
    // its CH macros (finished lanes are frozen); the DMA of the next chunk
    // is waited for (vmcnt(0)) once per phase
    auto phase = [&](const uint4 *buf, const uint32_t *info) __attribute__((always_inline)) {
        const uint4 *const cur = buf + moff;
        if constexpr (NR == 2) {
            // one wave test for the whole chunk, then CH macros with no test
            // and no branch between them but the stores' own
            if (L.lean_chunk_ok(info[slot])) {
#pragma unroll 2
                for (uint32_t i = 0; i < CH; i++) L.macro_lean(cur[2 * i], cur[2 * i + 1]);
                return;
            }
        }
#pragma unroll 1
        for (uint32_t i = 0; i < CH; i++) {
            const uint4 a = cur[2 * i], u = cur[2 * i + 1];
            if constexpr (NR == 2) {
                if (L.lean_ok(u)) {
                    L.macro_lean(a, u);
                    continue;
                }
            }
            constexpr bool W3 = MacroLane<NR, ADDID>::W3;
            const uint32_t c0 = W3 ? w3_ctl(a.y, 0) : a.y, c1 = W3 ? w3_ctl(a.y, 1) : a.w;
            const uint32_t i1 = a.z;
            if (L.simple_ok(a, u)) {
                L.alu_simple(a.x, c0);
                L.alu_simple(i1, c1);
                if (W3) L.alu_simple(a.w, w3_ctl(a.y, 2));
                L.pulse_simple(u);
            } else {
                L.alu_step(a.x, c0);
                L.alu_step(i1, c1);
                if (W3) L.alu_step(a.w, w3_ctl(a.y, 2));
                L.pulse_step(u);
            }
        }
    };
    stage(0u, s_chunk0[wv], s_info0[wv]);
    for (uint32_t c = 0; __ballot(L.st == 0u); c += 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        stage(c + 1u, s_chunk1[wv], s_info1[wv]);
#ifdef DPEMU_PROBE_DMA2
        stage(c + 1u, s_chunk1[wv], s_info1[wv]);   // probe: every chunk fetched twice
#endif
        phase(s_chunk0[wv], s_info0[wv]);
        if (!__ballot(L.st == 0u)) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        stage(c + 2u, s_chunk0[wv], s_info0[wv]);
#ifdef DPEMU_PROBE_DMA2
        stage(c + 2u, s_chunk0[wv], s_info0[wv]);
#endif
        phase(s_chunk1[wv], s_info1[wv]);
    }
    // no LDS DMA may still be in flight when the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    L.flags |= (L.n_ev > p.event_cap ? F_EVENT_OVF : 0u) | (L.n_meas > min(p.meas_cap, MEAS_LOOKUP) ? F_MEAS_OVF : 0u) |
               (p.trace_cap && L.n_tr > p.trace_cap ? F_TRACE_OVF : 0u);

    if (valid && p.summary) {
        const uint32_t ip = (L.st & MacroLane<NR, ADDID>::ST_TOP) ? L.k : L.k - 1u;
        write_summary(p, lane, L.t, ip, L.st & 0xFFu, L.flags, L.n_ev, L.k, L.qclk_at(L.t), L.n_meas, L.meas_bits,
                      L.n_tr);
    }
    if (valid && p.regs_out) {
#pragma unroll
        for (int r = 0; r < 16; r++)
            p.regs_out[(uint64_t)r * p.n_lanes + lane] =
                ((p.reg_used >> r) & 1u) ? L.reg_rd((uint32_t)(p.reg_map >> (4 * r)) & 15u) : 0u;
    }
    count_outcome_block(p, s_hist, s_key, valid, core, sl, valid ? shot_group(p, sl) : 0u, L.last_bit);
#ifdef DPEMU_PROBE_WAVETIME
    probe_wavetime(pt0, wv);
#endif
}

hipError_t launch_macro(const KParams &p, uint32_t slots, int nr, bool addid, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p.n_lanes + BLOCK - 1) / BLOCK);
    if (blocks == 0) return hipSuccess;
    const size_t shmem = p.hist_lds ? HIST_LDS_MAX * sizeof(uint32_t) : 0;
    constexpr int S = MACRO_SLOTS, SW = MACRO_SLOTS_WIDE;
    if (slots == 0u) hipLaunchKernelGGL(macro_kernel, dim3(blocks), dim3(BLOCK), 0, stream, p);
    else if (slots > MACRO_SLOTS && nr == 2 && addid)
        hipLaunchKernelGGL((macro_staged_kernel<2, true, SW>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    else if (slots > MACRO_SLOTS && nr == 2)
        hipLaunchKernelGGL((macro_staged_kernel<2, false, SW>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    else if (slots > MACRO_SLOTS)
        return hipErrorInvalidValue;                     // (the host offers wide slots to NR == 2 images only)
    else if (nr == 2 && addid) hipLaunchKernelGGL((macro_staged_kernel<2, true, S>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    else if (nr == 2) hipLaunchKernelGGL((macro_staged_kernel<2, false, S>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    else hipLaunchKernelGGL((macro_staged_kernel<16, false, S>), dim3(blocks), dim3(BLOCK), shmem, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
