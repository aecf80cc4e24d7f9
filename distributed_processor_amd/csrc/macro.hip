// macro.hip -- the interpreter for branch-free programs with register
// commands (reg_alu, inc_qclk) on CDNA4 (gfx950): RB-like programs.
//
// A program with no jump, fproc or sync command never moves its instruction
// pointer except by +1 (hdl/instr_ptr.v without a jump), so its command
// sequence is fixed before it runs.  dpemu_load_programs re-packs every such
// program into MACROS of one fixed shape (capi.cpp build_macros):
//
//     [ALU slot 0][ALU slot 1][pulse slot]          32 B
//
// up to two consecutive reg_alu / inc_qclk commands followed by the next
// other command (pulse write / trigger, idle, pulse reset, done, hang),
// each slot marked present or absent.  Every lane still running in loop
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

namespace dpemu {

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
#ifdef MACRO_PROBE_NOSTORE                              // A/B probe only (scripts/ab_libs.sh): no event stores
            if (n_ev == 0xFFFFFFFFu)
#else
            if (n_ev < p.event_cap && p.events)
#endif
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
                make_uint4(D + 3u, is_q ? TRACE_QCLK_LOAD : rd, is_q ? out + 3u : out, 0u);
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
#ifdef MACRO_PROBE_NOFETCH                              // A/B probe only: every fetch hits macro 0..1 (L1)
    auto addr = [&](uint32_t m) __attribute__((always_inline)) -> const uint4 * { return mbase + 2ull * min(mb + (m & 1u), ml); };
#else
    auto addr = [&](uint32_t m) __attribute__((always_inline)) -> const uint4 * { return mbase + 2ull * min(mb + m, ml); };
#endif

    // one macro ahead: macro m + 1 is in flight while macro m executes
    uint4 an = addr(0u)[0], un = addr(0u)[1];
    for (uint32_t m = 1; __ballot(st == 0u); m++) {
        const uint4 a = an, u = un;
        {
            const uint4 *q = addr(m);                   // the next macro: in flight during this one
            an = q[0];
            un = q[1];
        }
        alu_step(a.x, a.y);
        alu_step(a.z, a.w);
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
        for (int r = 0; r < 16; r++) p.regs_out[(uint64_t)r * n_lanes + lane] = s_regs[r][tid];
    }
    count_outcome_block(p, s_hist, s_key, valid, core, sl, valid ? shot_group(p, sl) : 0u, last_bit);
}

hipError_t launch_macro(const KParams &p, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p.n_lanes + BLOCK - 1) / BLOCK);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(macro_kernel, dim3(blocks), dim3(BLOCK), 0, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
