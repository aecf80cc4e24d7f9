// interp.hip -- lockstep ISA interpreter for the QubiC distributed processor
// on CDNA4 (gfx950).
//
// One thread = one (shot, core) lane.  Lane L = shot_local * C + core with C a
// power of two <= 64, so the C cores of a shot are adjacent lanes of ONE
// wavefront: every cross-core interaction of the gateware -- fproc reads of
// another core's measurement (hdl/fproc_meas.sv), the meas_lut syndrome FSM
// (hdl/core_state_mgr.sv, hdl/meas_lut.sv) and the sync barrier
// (hdl/sync_iface.sv + build-defined controller) -- is resolved inside the
// wave with shuffles, ballots and LDS; nothing crosses a workgroup.
//
// Each loop iteration retires at most one instruction per lane and advances
// that lane's next-DECODE cycle by the closed-form latency of hdl/ctrl.v
// (see oracle/fast_model.c for the restatement this kernel is pinned to).
// Per-lane state lives in VGPRs (ip, next-decode cycle t, qclk anchor, pulse
// register image, counters); the 16 x 32-bit reg_file lives in LDS as
// [reg][lane] so a runtime register index is one ds_read_b32 with no bank
// conflict.  Measurements (valid cycle << 1 | bit) live in LDS [slot][lane]
// so other cores of the shot can read them.
//
// Cross-core ordering: a read of qubit q at DECODE cycle D (fproc_meas) needs
// every meas_valid with cycle <= D.  Each lane publishes a lower bound of its
// next readout strobe; the read proceeds once min(bound) + meas_latency > D.
// The lane with the smallest pending read is never blocked by another read,
// so the shot always progresses (a group with no progress is a true deadlock).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "lane.h"

namespace dpemu {

enum : uint32_t { M_RUN = 0, M_SYNC = 1, M_LUT = 2, M_FIN = 3 };

__device__ __forceinline__ uint32_t alu_op(uint32_t op, uint32_t a, uint32_t b)
{
    // alu.v:20-50; le = sub[31] ^ overflow == signed a < b
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

// group reductions over the C adjacent lanes of a shot (all lanes converged)
template <int OP>   // 0 = min, 1 = max
__device__ __forceinline__ uint32_t group_reduce(uint32_t v, uint32_t C)
{
    for (uint32_t m = 1; m < C; m <<= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, (int)m, 64);
        v = OP == 0 ? (o < v ? o : v) : (o > v ? o : v);
    }
    return v;
}

__device__ __forceinline__ void wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int FEAT>
__global__ void __launch_bounds__(BLOCK) interp_kernel(const KParams p)
{
    constexpr bool FPROC = (FEAT & FEAT_FPROC) != 0;
    constexpr bool SYNC = (FEAT & FEAT_SYNC) != 0;
    constexpr bool LUT = (FEAT & FEAT_LUT) != 0;
    constexpr bool PLDS = (FEAT & FEAT_PROG_LDS) != 0;   // programs staged in LDS
    // pulse / idle / done only: no ALU writes, so every register reads 0
    constexpr bool STRAIGHT = (FEAT & FEAT_STRAIGHT) != 0;
    constexpr bool XMEAS = FPROC || LUT;             // measurements readable by other lanes
    constexpr int MT = XMEAS ? MEAS_LOOKUP : 1;
    constexpr int NF = LUT ? LUT_FIRE_CAP : 1;

    __shared__ uint32_t s_regs[STRAIGHT ? 1 : 16][STRAIGHT ? 1 : BLOCK];
    __shared__ uint32_t s_mt[MT][BLOCK];
    // meas_lut per shot (slots indexed by the shot leader's tid)
    __shared__ uint32_t s_cur[LUT ? BLOCK : 1];       // merge cursor into lane's s_mt
    __shared__ uint32_t s_fire_t[NF][LUT ? BLOCK : 1];
    __shared__ uint64_t s_fire_o[NF][LUT ? BLOCK : 1];
    // programs of this workgroup's (group, core) slots: the analogue of each core's cmd_mem
    __shared__ uint32_t s_pref[PLDS ? BLOCK + 1 : 1];
    __shared__ uint32_t s_scan[BLOCK / 64];
    extern __shared__ uint4 s_prog[];

    clear_hist_next(p);
    const uint32_t tid = threadIdx.x;
    const uint32_t C = p.C;
    const uint32_t pos = blockIdx.x * BLOCK + tid;   // thread position; a shot's cores are adjacent
    const bool valid = pos < p.n_lanes;
    const uint32_t core = pos & (C - 1);
    const uint32_t spos = pos >> p.log2C;
    const uint32_t lane = out_lane(p, spos, core);   // output lane index (core-major)
    const uint64_t shot = p.shot_begin + spos;
    const uint32_t wl = tid & 63;                    // lane within the wavefront
    const uint32_t leader_tid = tid & ~(C - 1);

    uint32_t base = 0, nprog = 0, grp = 0, prog = 0;
    if (valid) {
        grp = shot_group(p, spos);
        prog = p.prog_table[(uint64_t)grp * C + core];
        base = p.offsets[prog];
        nprog = p.n_instr[prog];
    }
    // command ip of this lane's program in the fetch image (KParams::fetch)
    const uint32_t fetch_off = p.fetch_stride == 1u ? base : prog;
    const uint32_t thr_core = valid ? p.p1_thr[core] : 0u;
    __shared__ uint32_t s_hist[HIST_LDS_MAX];
    if (p.hist_lds) {
        for (uint32_t i = tid; i < HIST_LDS_MAX; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
    }
    if constexpr (PLDS) {
        const uint32_t b = stage_programs(p, s_prog, s_pref, s_scan, spos, core);
        if (valid) base = b;
    }
    if constexpr (!STRAIGHT) {
#pragma unroll
        for (int r = 0; r < 16; r++) s_regs[r][tid] = 0;
    }
    if constexpr (XMEAS) {
#pragma unroll
        for (int m = 0; m < MT; m++) s_mt[m][tid] = INF32;
    }
    if constexpr (LUT) s_cur[tid] = 0;

    // lane state
    uint32_t mode = valid ? M_RUN : M_FIN;
    uint32_t ip = 0, t = 0, qa_t = 1, qa_q = 0;      // qclk(0) = qclk(1) = 0: reset hold
    uint32_t pe = 0, pp = 0, pa = 0;                 // pulse regs: env|cfg<<24, phase|freq<<17, amp
    uint32_t wait_d = 0, status = 0, flags = 0;
    uint32_t n_ev = 0, n_tr = 0, n_meas = 0, n_exec = 0, meas_bits = 0, last_bit = 0;
    uint32_t t_end = 0;
    // DEMOD (run-time: this kernel is the general path): the latest
    // readout-drive strobe and pulse_reset, the last meas_valid
    const bool demod = p.meas_model == DPEMU_MEAS_DEMOD;
    RoDrive ro_d{0u, 0u, 0u};
    uint32_t ro_tref = 0, ro_ltv = 0;
    // leader-only meas_lut state
    uint64_t lut_valid = 0, lut_addr = 0;
    uint32_t lut_last_fire = INF32, nfire = 0;

    const uint64_t n_lanes = p.n_lanes;
    const bool is_part = SYNC ? (((p.sync_mask >> core) & 1ull) != 0) : false;

    // a finished lane's ip and qclk anchor never change again: ip and qclk at
    // t_end are read when the summary is written
    auto finish = [&](uint32_t st, uint32_t at) {
        status = st; mode = M_FIN; t_end = at;
    };

    // (always_inline: with the DEMOD readout an out-of-line call would keep the
    // kernel's state in scratch, tests/test_kernel_resources.py)
    auto emit_event = [&](uint32_t te, uint32_t kind) __attribute__((always_inline)) {
        if (n_ev < p.event_cap) {
            if (p.events) p.events[(uint64_t)n_ev * n_lanes + lane] = event_record(te, pe, pp, pa, kind);
        } else flags |= F_EVENT_OVF;
        n_ev++;
        if (demod) {
            if (kind == 1u) ro_tref = te;
            if (kind == 0u && ((pe >> 24) & 3u) == p.ro_drv_elem)
                ro_d = RoDrive{te, pp & 0x03FFFFFFu, (pa & 0xFFFFu) | (((pe >> 12) & 0xFFFu) << 16) | 0x80000000u};
        }
        if (kind == 0 && p.meas_elem != 0xFFu && ((pe >> 24) & 3u) == p.meas_elem) {
            uint32_t bit, tv;
            if (demod) {
                int2 a;
                const uint4 h = p.ro_hdr[prog];              // drv_off, drv_len, lo_off, lo_len
                bit = demod_readout(p, shot, core, n_meas, thr_core, te, pe, pp, ro_d, ro_tref,
                                    ro_freq(p, h.z, h.w, (pp >> 17) & 0x1FFu),
                                    ro_freq(p, h.x, h.y, (ro_d.pp >> 17) & 0x1FFu), a);
                tv = demod_valid(p, te, pe, ro_ltv);
                ro_ltv = tv;
                if (p.acc && n_meas < p.meas_cap) p.acc[(uint64_t)n_meas * n_lanes + lane] = a;
            } else {
                bit = meas_bit(p, shot, core, n_meas, thr_core, pa, pe);
                tv = te + p.meas_latency;
            }
            if constexpr (XMEAS) {
                if (n_meas < MEAS_LOOKUP) s_mt[n_meas < MT ? n_meas : 0][tid] = (tv << 1) | bit;
            }
            if (n_meas < p.meas_cap) {
                if (p.meas) p.meas[(uint64_t)n_meas * n_lanes + lane] = make_uint2(tv, bit);
            } else flags |= F_MEAS_OVF;
            if (n_meas >= MEAS_LOOKUP) flags |= F_MEAS_OVF;
            if (n_meas < 32 && bit) meas_bits |= 1u << n_meas;
            last_bit = bit;
            n_meas++;
        }
    };

    auto emit_trace = [&](uint32_t tt, uint32_t addr, uint32_t val) __attribute__((always_inline)) {
        if (n_tr < p.trace_cap) {
            if (p.trace) p.trace[(uint64_t)n_tr * n_lanes + lane] = make_uint4(tt, addr, val, 0u);
        } else if (p.trace_cap) flags |= F_TRACE_OVF;
        n_tr++;
    };

    // latest measurement of group lane q with valid cycle <= d (slots sorted, INF = empty)
    auto meas_lookup = [&](uint32_t q_tid, uint32_t d) -> uint32_t {
        uint32_t res = 0;
#pragma unroll
        for (int m = 0; m < MT; m++) {
            const uint32_t e = s_mt[m][q_tid];
            if (e != INF32 && (e >> 1) <= d) res = e & 1u;
        }
        return res;
    };

    uint32_t iter = 0;
    for (;;) {
        if (!__any(mode != M_FIN)) break;
        // internal-error guard: a correct run retires an instruction of >= 3 cycles
        // in some lane of every live shot each iteration, so it never gets here
        if (++iter > p.iter_guard) {
            if (mode != M_FIN) { flags |= F_GUARD; finish(ST_DEADLOCK, t); }
            break;
        }

        // ---------------- fetch (RUN lanes) ----------------
        bool run = (mode == M_RUN);
        if (run && t > p.max_cycles) { finish(ST_MAX_CYCLES, t); run = false; }
        uint4 u = make_uint4(0u, 0u, 0u, 0u);             // past the program: op4 0 = DONE
        if (run && ip < nprog) u = PLDS ? s_prog[base + ip] : p.fetch[(uint64_t)ip * p.fetch_stride + fetch_off];
        const uint32_t op4 = u.y >> 28;
        const bool is_fproc = run && (op4 == 4u || op4 == 5u);

        // fproc_meas read at D = t (pending in a running lane): it needs every
        // meas_valid <= D known, i.e. the group's strobe bound + meas_latency > D
        auto fproc_stall = [&](uint32_t gmin) -> bool {
            if constexpr (FPROC) {
                if (is_fproc && p.fproc_mode == 0u) return !((uint64_t)gmin + p.meas_latency > (uint64_t)t);
            }
            return false;
        };

        // Retire the fetched command u (opcode op) in a running, unstalled
        // lane: hdl/ctrl.v's decode-to-decode latency in closed form
        // (DESIGN.md §2).  Called with a wave-uniform op from the fast path
        // (a scalar switch: only that opcode's code runs) and with the lane's
        // own op4 from the general path.  Registers are read where a command
        // uses them.
        auto retire = [&](const uint32_t op) {
            n_exec++;
            const uint32_t D = t;
            const uint32_t alu = u.y & 7u;
            auto reg = [&](uint32_t r) -> uint32_t { return STRAIGHT ? 0u : s_regs[r & 15u][tid]; };
            auto in0 = [&]() -> uint32_t { return (u.y & 8u) ? reg(u.w >> 20) : u.x; };
            auto qclk = [&](uint32_t d) -> uint32_t { return (d < qa_t) ? 0u : qa_q + (d - qa_t); };
            switch (op) {
            case 0x0: case 0xA:
                finish(ST_DONE, D);
                break;
            case 0xB:
                emit_event(D, 1u);
                ip = (ip + 1u) & 0xFFFFu; t = D + 3u;
                break;
            case 0x8: case 0x9: case 0xC: {
                bool go = true;
                uint32_t tT = D;
                bool dbl = false;
                if (op != 0x8) {
                    const uint32_t T = u.x;
                    uint64_t wait;
                    if (D < qa_t) { dbl = (T == 0u); wait = dbl ? 0ull : (uint64_t)(qa_t - D) + (uint32_t)(T - qa_q); }
                    else wait = (uint32_t)(T - qclk(D));
                    if (wait >= 0x80000000ull) flags |= F_LATE;
                    if (wait > (uint64_t)(p.max_cycles - D)) { finish(ST_MAX_CYCLES, D); go = false; }
                    else tT = D + (uint32_t)wait;
                }
                if (go && op != 0xC) {
                    // pulse_reg.sv:59-97: immediates, then reg[rs0] into register-sourced fields
                    pulse_write(u, pe, pp, pa);
                    if (!STRAIGHT && (u.w & UOP_ANY_RS)) {
                        const uint32_t r0 = reg(u.w >> 20);
                        if (u.w & UOP_RS_ENV) pe |= r0 & 0xFFFFFFu;
                        if (u.w & UOP_RS_PH) pp |= r0 & 0x1FFFFu;
                        if (u.w & UOP_RS_FR) pp |= (r0 & 0x1FFu) << 17;
                        if (u.w & UOP_RS_AMP) pa = r0 & 0xFFFFu;
                    }
                }
                if (go) {
                    if (op == 0x9) {
                        emit_event(tT + 2u, 0u);
                        if (dbl) { emit_event(tT + 3u, 0u); flags |= F_DOUBLE_STROBE; }
                    }
                    ip = (ip + 1u) & 0xFFFFu;
                    t = tT + 3u;
                }
                break;
            }
            case 0x1: {
                if constexpr (!STRAIGHT) {
                    const uint32_t out = alu_op(alu, in0(), reg(u.y >> 4));
                    const uint32_t rd = (u.y >> 8) & 15u;
                    s_regs[rd][tid] = out;
                    emit_trace(D + 3u, rd, out);
                    ip = (ip + 1u) & 0xFFFFu; t = D + 4u;
                }
                break;
            }
            case 0x2:
                ip = u.z & 0xFFFFu; t = D + 4u;
                break;
            case 0x3: {
                const uint32_t out = alu_op(alu, in0(), reg(u.y >> 4));
                ip = (out & 1u) ? (u.z & 0xFFFFu) : ((ip + 1u) & 0xFFFFu);
                t = D + 6u;
                break;
            }
            case 0x6: {
                const uint32_t out = alu_op(alu, in0(), qclk(D));
                qa_t = D + 3u; qa_q = out + 3u;
                emit_trace(D + 3u, TRACE_QCLK_LOAD, out + 3u);
                ip = (ip + 1u) & 0xFFFFu; t = D + 4u;
                break;
            }
            case 0x7:
                if constexpr (SYNC) { mode = M_SYNC; wait_d = D; }
                else { finish(ST_DEADLOCK, D); }   // not reached: host selects SYNC kernels
                break;
            case 0x4: case 0x5: {
                const uint32_t id = (u.z >> 16) & 0xFFu;
                bool have = false;
                uint32_t R = 0, data = 0;
                if constexpr (XMEAS) {
                    if (p.fproc_mode == 0u) {
                        R = D + 2u;
                        data = meas_lookup(leader_tid + (id & (C - 1)), D);
                        have = true;
                    } else if (id == 0u) {
                        // core_state_mgr WAIT_MEAS: first own meas_valid at >= D + 1
#pragma unroll
                        for (int m = MT - 1; m >= 0; m--) {
                            const uint32_t e = s_mt[m][tid];
                            if (e != INF32 && (e >> 1) >= D + 1u) { R = e >> 1; data = e & 1u; have = true; }
                        }
                        if (!have) { finish(ST_DEADLOCK, D); }
                    } else {
                        mode = M_LUT; wait_d = D;
                    }
                } else {
                    finish(ST_DEADLOCK, D);          // not reached: host selects FPROC kernels
                }
                if (have) {
                    if (R > p.max_cycles) finish(ST_MAX_CYCLES, D);
                    else {
                        const uint32_t out = alu_op(alu, in0(), data);
                        if (op == 4u) {
                            const uint32_t rd = (u.y >> 8) & 15u;
                            s_regs[rd][tid] = out;
                            emit_trace(R + 3u, rd, out);
                            ip = (ip + 1u) & 0xFFFFu; t = R + 4u;
                        } else {
                            ip = (out & 1u) ? (u.z & 0xFFFFu) : ((ip + 1u) & 0xFFFFu);
                            t = R + 6u;
                        }
                    }
                }
                break;
            }
            default:                                     // 0xD-0xF: hang in DECODE
                finish(ST_HUNG_OPCODE, D);
                break;
            }
        };

        // ---------------- fast path: one opcode for the whole wave ----------------
        // Every live lane runs and all fetched the same opcode (the batched-
        // experiment shape: one program structure, per-core / per-group
        // parameters): no lane waits in a barrier or on the LUT, so the
        // cross-core phase reduces to the fproc bound, and a scalar switch runs
        // only that opcode's semantics.
        if constexpr (!LUT && !STRAIGHT) {
            const uint64_t run_m = __ballot(run);
            if (run_m) {
                const uint32_t op_u = __builtin_amdgcn_readlane(op4, (int)__builtin_ctzll(run_m));
                if (!__ballot(mode != M_FIN && !(run && op4 == op_u))) {
                    uint32_t gmin = INF32;
                    if (op_u == 4u || op_u == 5u) gmin = group_reduce<0>(run ? t + 2u : INF32, C);
                    if (run && !fproc_stall(gmin)) retire(op_u);
                    if constexpr (FPROC || XMEAS) wave_fence();
                    continue;
                }
            }
        }

        // ---------------- cross-core phase (converged) ----------------
        uint32_t gmin = INF32;
        bool any_run_grp = true;
        bool released = false;
        if constexpr (SYNC || XMEAS) {
            // wave-uniform guards: gmin only matters to a pending fproc_meas read (or the
            // LUT leader), the barrier only while some lane waits in SYNC -- most iterations
            // of a branching program skip both group reductions
            const bool need_g = LUT || __any(is_fproc);
            if constexpr (SYNC) {
              if (need_g || __any(mode == M_SYNC)) {
                // barrier: complete when every participant is in SYNC_WAIT
                const uint32_t key = is_part ? ((mode == M_SYNC) ? wait_d : (mode == M_RUN) ? t
                                             : (mode == M_LUT) ? wait_d + 5u : INF32) : 0u;
                const uint32_t maxkey = group_reduce<1>(key, C);
                const uint64_t b = __ballot(is_part && mode == M_SYNC);
                const uint64_t pm = __ballot(is_part);
                const bool all_arrived = group_bits(b, wl, C) == group_bits(pm, wl, C) &&
                                         group_bits(pm, wl, C) != 0ull;
                if (mode == M_SYNC && is_part && all_arrived) {
                    const uint32_t S = maxkey + p.sync_latency;
                    if (S > p.max_cycles) finish(ST_MAX_CYCLES, wait_d);
                    else {
                        qa_t = S + 2u; qa_q = 0u;
                        emit_trace(S + 2u, TRACE_QCLK_RST, 0u);
                        ip = (ip + 1u) & 0xFFFFu;
                        t = S + 3u;
                        mode = M_RUN;
                    }
                    released = true;
                }
                // strobe bound of a waiting participant
                if (need_g) {
                    uint32_t bound = INF32;
                    if (mode == M_RUN) bound = t + 2u;
                    else if (mode == M_LUT) bound = wait_d + 7u;
                    else if (mode == M_SYNC && is_part && maxkey != INF32)
                        bound = maxkey + p.sync_latency + 5u;
                    gmin = group_reduce<0>(bound, C);
                }
              }
            } else if (need_g) {
                const uint32_t bound = (mode == M_RUN) ? t + 2u : (mode == M_LUT) ? wait_d + 7u : INF32;
                gmin = group_reduce<0>(bound, C);
            }
            if constexpr (LUT) any_run_grp = group_bits(__ballot(mode == M_RUN), wl, C) != 0ull;
        }

        // ---------------- execute (any opcode per lane) ----------------
        bool executed = false;
        if constexpr (STRAIGHT) {
            // pulse / idle / pulse_reset / done / hang only: the timing of ctrl.v in
            // closed form with few state merges (the generic switch costs ~2x
            // the VALU instructions per command)
            if (run) {
                n_exec++;
                const uint32_t D = t;
                const uint32_t qD = (D < qa_t) ? 0u : qa_q + (D - qa_t);
                const bool pw = op4 == 0x8u || op4 == 0x9u;
                const bool waits = op4 == 0x9u || op4 == 0xCu;
                const bool pulse_cls = pw || op4 == 0xBu || op4 == 0xCu;
                const uint32_t T = u.x;
                uint32_t wait = T - qD;
                bool dbl = false, big = false;
                if (D < qa_t) {            // reset hold: qclk(0) = qclk(1) = 0 (proc.sv:125-136)
                    dbl = T == 0u;
                    const uint64_t wl = dbl ? 0ull : (uint64_t)(qa_t - D) + (uint32_t)(T - qa_q);
                    wait = (uint32_t)wl;
                    big = (wl >> 32) != 0ull;
                }
                if (waits && (big || wait >= 0x80000000u)) flags |= F_LATE;
                const bool over = waits && (big || wait > p.max_cycles - D);
                const uint32_t tT = D + (waits ? wait : 0u);
                if (!pulse_cls || over) {
                    finish(over ? ST_MAX_CYCLES : (op4 >= 0xDu ? ST_HUNG_OPCODE : ST_DONE), D);
                } else {
                    if (pw) {
                        // pulse_reg.sv:59-97 with reg_in = 0
                        pulse_write(u, pe, pp, pa);
                    }
                    if (op4 == 0x9u || op4 == 0xBu) {
                        emit_event(op4 == 0xBu ? D : tT + 2u, op4 == 0xBu ? 1u : 0u);
                        if (dbl && op4 == 0x9u) { emit_event(tT + 3u, 0u); flags |= F_DOUBLE_STROBE; }
                    }
                    ip = (ip + 1u) & 0xFFFFu;
                    t = tT + 3u;
                }
            }
        } else if (run && !fproc_stall(gmin)) {
            executed = true;
            retire(op4);
        }

        // ---------------- meas_lut (per shot, by the shot's leader lane) ----------------
        if constexpr (LUT) {
            wave_fence();
            bool fired = false;
            if (tid == leader_tid && valid) {
                uint32_t H = INF32;
                if (any_run_grp && gmin != INF32) {
                    const uint64_t h = (uint64_t)gmin + p.meas_latency - 1u;
                    H = h > INF32 ? INF32 : (uint32_t)h;
                }
                const bool stop_at_fire = !any_run_grp;
                for (;;) {
                    uint32_t tmin = INF32;
                    for (uint32_t c = 0; c < C; c++) {
                        const uint32_t cur = s_cur[leader_tid + c];
                        if (cur < (uint32_t)MT) {
                            const uint32_t e = s_mt[cur < (uint32_t)MT ? cur : 0][leader_tid + c];
                            if (e != INF32 && (e >> 1) < tmin) tmin = e >> 1;
                        }
                    }
                    if (tmin == INF32 || tmin > H) break;
                    uint64_t v = 0, mv = 0;
                    for (uint32_t c = 0; c < C; c++) {
                        const uint32_t cur = s_cur[leader_tid + c];
                        if (cur < (uint32_t)MT) {
                            const uint32_t e = s_mt[cur < (uint32_t)MT ? cur : 0][leader_tid + c];
                            if (e != INF32 && (e >> 1) == tmin) {
                                v |= 1ull << c;
                                if (e & 1u) mv |= 1ull << c;
                                s_cur[leader_tid + c] = cur + 1u;
                            }
                        }
                    }
                    // meas_lut.sv:40-56: LUT_READY the cycle after a fire ignores inputs
                    if (lut_last_fire != INF32 && tmin == lut_last_fire + 1u) continue;
                    const uint64_t nv = lut_valid | v, na = lut_addr | (v & mv);
                    if (((uint64_t)p.lut_mask & nv) == (uint64_t)p.lut_mask) {
                        lut_last_fire = tmin;
                        if (nfire < (uint32_t)NF) {
                            s_fire_t[nfire < (uint32_t)NF ? nfire : 0][tid] = tmin;
                            s_fire_o[nfire < (uint32_t)NF ? nfire : 0][tid] = p.lut_table[na & 0xFFu];
                        }
                        nfire++;
                        lut_valid = 0; lut_addr = 0;
                        fired = true;
                        if (stop_at_fire) break;
                    } else { lut_valid = nv; lut_addr = na; }
                }
            }
            // publish the leader's fire count to the group
            const uint32_t nf_grp = (uint32_t)__shfl((int)nfire, (int)(wl & ~(C - 1)), 64);
            const bool grp_fired = group_bits(__ballot(fired), wl, C) != 0ull;
            wave_fence();
            if (mode == M_LUT) {
                const uint32_t n = nf_grp < (uint32_t)NF ? nf_grp : (uint32_t)NF;
                for (uint32_t k = 0; k < n; k++) {
                    const uint32_t tf = s_fire_t[k][leader_tid];
                    if (tf >= wait_d + 1u) {
                        const uint64_t out_bits = s_fire_o[k][leader_tid];
                        // the waiting fproc command
                        const uint4 u2 = PLDS ? s_prog[base + ip] : p.uops[base + ip];
                        const uint32_t op4b = u2.y >> 28, alub = u2.y & 7u;
                        // both operands loaded, then selected: a select of the two
                        // addresses would be one flat_load (generic pointer)
                        const uint32_t rs0v = s_regs[(u2.w >> 20) & 15u][tid];
                        const uint32_t in0b = (u2.y & 8u) ? rs0v : u2.x;
                        if (tf > p.max_cycles) { finish(ST_MAX_CYCLES, wait_d); }
                        else {
                            const uint32_t out = alu_op(alub, in0b, (uint32_t)((out_bits >> core) & 1ull));
                            if (op4b == 4u) {
                                const uint32_t rd = (u2.y >> 8) & 15u;
                                s_regs[rd][tid] = out;
                                emit_trace(tf + 3u, rd, out);
                                ip = (ip + 1u) & 0xFFFFu; t = tf + 4u;
                            } else {
                                ip = (out & 1u) ? (u2.z & 0xFFFFu) : ((ip + 1u) & 0xFFFFu);
                                t = tf + 6u;
                            }
                            mode = M_RUN;
                        }
                        released = true;
                        break;
                    }
                }
            }
            if (grp_fired) released = released || (tid == leader_tid);
        }

        // ---------------- deadlock: a shot with no progress can never progress ----------------
        if constexpr (SYNC || LUT) {
            if (__any(mode == M_SYNC || mode == M_LUT)) {       // wave-uniform: only waiting lanes can deadlock
                const uint64_t prog = __ballot(executed || released);
                if (group_bits(prog, wl, C) == 0ull && (mode == M_SYNC || mode == M_LUT))
                    finish(ST_DEADLOCK, wait_d);
            }
        }
        if constexpr (FPROC || XMEAS) wave_fence();
    }

    if (valid && p.summary) {
        const uint32_t qclk_end = (t_end < qa_t) ? 0u : qa_q + (t_end - qa_t);
        write_summary(p, lane, t_end, ip, status, flags, n_ev, n_exec, qclk_end, n_meas, meas_bits, n_tr);
    }
    if (valid && p.regs_out) {
#pragma unroll
        for (int r = 0; r < 16; r++) p.regs_out[(uint64_t)r * n_lanes + lane] = STRAIGHT ? 0u : s_regs[r][tid];
    }
    count_outcome(p, s_hist, valid, core, grp, last_bit);
}

// out[i] += sum of the R replicas; thread = (bin, slice of 8 replicas), loads independent
// hist[i] (+)= the sum of the R replicas' bin i; every replica word read is
// left zero for the next run.  A thread sums one slice of 8 replicas of one
// bin.  Adding: a u64 atomic per slice.  Storing (hist_assign): the G >=
// slices lanes of a bin are adjacent, their sums are combined with
// cross-lane shuffles and the group's first lane stores the bin.
__global__ void __launch_bounds__(BLOCK) hist_reduce_kernel(uint32_t *rep, uint32_t R, uint64_t stride,
                                                           uint64_t bins, uint32_t G, unsigned long long *hist)
{
    const uint32_t slices = (R + 7) / 8;
    const uint32_t per = G ? G : slices;                     // threads per bin
    const uint64_t n = bins * per;
    for (uint64_t x = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; x - threadIdx.x < n; x += (uint64_t)gridDim.x * BLOCK) {
        const bool in = x < n;
        const uint64_t i = G ? x / G : x % bins;
        const uint32_t sl = G ? (uint32_t)(x % G) : (uint32_t)(x / bins);
        const uint32_t r0 = sl * 8;
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = (in && r0 + k < R) ? rep[(uint64_t)(r0 + k) * stride + i] : 0u;
        unsigned long long acc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            acc += v[k];
            if (v[k]) rep[(uint64_t)(r0 + k) * stride + i] = 0u;
        }
        if (G) {                                             // uniform: every lane of the wave shuffles
            for (uint32_t m = 1; m < G; m <<= 1) {
                const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)acc, (int)m, 64);
                const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(acc >> 32), (int)m, 64);
                acc += ((unsigned long long)hi << 32) | lo;
            }
            if (in && sl == 0) hist[i] = acc;
        } else if (in && acc) {
            atomicAdd(&hist[i], acc);
        }
    }
}

hipError_t launch_hist_reduce(uint32_t *rep, uint32_t R, uint64_t stride, uint64_t bins, bool assign,
                              unsigned long long *hist, hipStream_t stream)
{
    uint32_t G = 0;                                          // storing: lanes per bin, a power of two >= slices
    if (assign) {
        G = 1;
        while (G < (R + 7) / 8) G <<= 1;                     // R <= 64: G <= 8
    }
    const uint64_t n = bins * (assign ? G : (R + 7) / 8);
    const uint64_t blocks = std::min<uint64_t>((n + BLOCK - 1) / BLOCK, 8192);
    hipLaunchKernelGGL(hist_reduce_kernel, dim3((uint32_t)blocks), dim3(BLOCK), 0, stream, rep, R, stride, bins, G,
                       hist);
    return hipGetLastError();
}

template <int F>
static void launch_one(const KParams &p, uint32_t blocks, size_t shmem, hipStream_t stream)
{
    hipLaunchKernelGGL(interp_kernel<F>, dim3(blocks), dim3(BLOCK), shmem, stream, p);
}

hipError_t launch_interp(const KParams &p, int feat, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p.n_lanes + BLOCK - 1) / BLOCK);
    if (blocks == 0) return hipSuccess;
    const size_t shmem = (feat & FEAT_PROG_LDS) ? (size_t)p.prog_lds_words * sizeof(uint4) : 0;
    switch (feat) {
#define CASE(F) case F: launch_one<F>(p, blocks, shmem, stream); break;
    CASE(FEAT_STRAIGHT) CASE(FEAT_STRAIGHT | FEAT_PROG_LDS)
    CASE(0) CASE(FEAT_FPROC) CASE(FEAT_SYNC) CASE(FEAT_FPROC | FEAT_SYNC) CASE(FEAT_LUT) CASE(FEAT_LUT | FEAT_SYNC)
    CASE(FEAT_PROG_LDS) CASE(FEAT_PROG_LDS | FEAT_FPROC) CASE(FEAT_PROG_LDS | FEAT_SYNC)
    CASE(FEAT_PROG_LDS | FEAT_FPROC | FEAT_SYNC) CASE(FEAT_PROG_LDS | FEAT_LUT)
    CASE(FEAT_PROG_LDS | FEAT_LUT | FEAT_SYNC)
#undef CASE
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dpemu
