// lane.h -- per-lane helpers shared by the interpreter kernels (interp.hip:
// the general lockstep interpreter; straight.hip: pulse-only programs).
#pragma once

#include "kernels.h"

namespace dpemu {

// per-component select (keeps the pending event records in registers)
__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b)
{
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}


#define INF32 0xFFFFFFFFu

// pulse_reg.sv:59-97 for a pre-decoded pulse command (decode_cmd): each field
// with its write enable takes its immediate (register-sourced fields are zero
// here and ORed in by the caller).  Enables are sign-extended to masks
// (v_bfe_i32) and merged with 3-input bit selects (v_bitop3_b32 0xCA = a ? b : c
// per bit): 10 VALU.  pe[31:28] picks up the opcode and pa[31:16] other
// command bits: consumers mask them (pe & 0x0FFFFFFF, (uint16_t)pa).
__device__ __forceinline__ uint32_t bit_select(uint32_t m, uint32_t a, uint32_t b)
{
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}

__device__ __forceinline__ void pulse_write(const uint4 u, uint32_t &pe, uint32_t &pp, uint32_t &pa)
{
    const int32_t w = (int32_t)u.w;
    const uint32_t m_env = (uint32_t)((w << 7) >> 31);      // enable bit 24
    const uint32_t m_cfg = (uint32_t)((w << 6) >> 31);      // 25
    const uint32_t m_ph = (uint32_t)((w << 5) >> 31);       // 26
    const uint32_t m_fr = (uint32_t)((w << 4) >> 31);       // 27
    const uint32_t m_amp = (uint32_t)((w << 3) >> 31);      // 28
    pe = bit_select(bit_select(0x00FFFFFFu, m_env, m_cfg), u.y, pe);
    pp = bit_select(bit_select(0x0001FFFFu, m_ph, m_fr), u.z, pp);
    pa = bit_select(m_amp, u.w, pa);
}

// event word 2: env[23:0] cfg[27:24] kind[31:28]
__device__ __forceinline__ uint32_t event_word(uint32_t pe, uint32_t kind)
{
    return (pe & 0x0FFFFFFFu) | (kind << 28);
}

// a * b as 64 bits in ONE v_mad_u64_u32 (hipcc emits a v_mul_lo_u32 +
// v_mul_hi_u32 pair for lo / __umulhi: scripts/micro/mul_rate.hip measured a
// Philox round 1.3x faster this way on gfx950, profiles/r03_mul_rate.jsonl)
__device__ __forceinline__ uint64_t mul_wide(uint32_t a, uint32_t b)
{
    uint64_t r, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(carry) : "v"(a), "s"(b));
    return r;
}

// Philox4x32-10, output words 0..2 (counter = shot_lo, shot_hi, core, m; key = seed)
__device__ __forceinline__ uint3 philox3(uint64_t seed, uint64_t shot, uint32_t core, uint32_t m)
{
    uint32_t c0 = (uint32_t)shot, c1 = (uint32_t)(shot >> 32), c2 = core, c3 = m;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = mul_wide(c0, 0xD2511F53u), p1 = mul_wide(c2, 0xCD9E8D57u);
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        // 3-input xors as one v_bitop3_b32 each (0x96 = a ^ b ^ c)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint3(c0, c1, c2);
}

// measurement outcome (oracle/philox.c oracle_meas_bit; include/dpemu.h): the
// prepared state against thr, or with meas_model READOUT the discriminated
// readout x = +-(ro_sep * amp >> 16) + (z * ro_sigma >> 16) > ro_thr, z the
// centred Irwin-Hall(4) sum of the 16-bit halves of Philox words 1 and 2;
// with ro_win the separation scales by min(W, ro_win) * floor(2^24 / ro_win)
// / 2^24, W = the env word's length field (bits 23:12)
__device__ __forceinline__ uint32_t meas_bit(const KParams &p, uint64_t shot, uint32_t core, uint32_t m,
                                             uint32_t thr, uint32_t amp, uint32_t env)
{
    const uint3 r = philox3(p.seed, shot, core, m);
    const uint32_t state = (thr == 0xFFFFFFFFu) || (r.x < thr);
    if (p.meas_model != DPEMU_MEAS_READOUT) return state;
    const int64_t z = (int64_t)((r.y & 0xFFFFu) + (r.y >> 16) + (r.z & 0xFFFFu) + (r.z >> 16)) - 131070;
    int64_t s = ((int64_t)p.ro_sep * (int64_t)(amp & 0xFFFFu)) >> 16;
    const uint32_t w = (env >> 12) & 0xFFFu;
    if (p.ro_win && w) {    // W = 0: a CW envelope, no window scaling; floor(2^24 / ro_win) from the host
        s = (s * (int64_t)((w < p.ro_win ? w : p.ro_win) * p.ro_wrecip)) >> 24;
    }
    const int64_t x = (state ? s : -s) + ((z * (int64_t)p.ro_sigma) >> 16);
    return x > (int64_t)p.ro_thr;
}

// ---- readout demodulation model (meas_model DPEMU_MEAS_DEMOD) --------------
// The closed form of include/dpemu.h / DESIGN.md §2, restated for the CPU in
// oracle/readout.c (that file's header is the normative spec).  Integer
// arithmetic only; every intermediate is the oracle's value.

// sin(2 pi x / 2^33) * 2^61 (x mod 2^33): quarter-wave reduction, then
// y * P(y^2) with P the Q30 Taylor polynomial of sin(pi/2 t) / t, t = y / 2^31
// (each Horner step one v_mad_i64_i32; every P value fits int32)
__device__ __forceinline__ int64_t sin33(uint64_t x)
{
    const uint32_t q = (uint32_t)(x >> 31) & 3u;
    const uint32_t f = (uint32_t)x & 0x7FFFFFFFu;
    const uint32_t y = (q & 1u) ? 0x80000000u - f : f;      // <= 2^31
    const int32_t z = (int32_t)(uint32_t)(((uint64_t)y * y) >> 32);   // t^2, Q30
    int32_t P = -3864;
    P = 172272 + (int32_t)(((int64_t)P * z) >> 30);
    P = -5026995 + (int32_t)(((int64_t)P * z) >> 30);
    P = 85569306 + (int32_t)(((int64_t)P * z) >> 30);
    P = -693598668 + (int32_t)(((int64_t)P * z) >> 30);
    P = 1686629713 + (int32_t)(((int64_t)P * z) >> 30);     // > 0
    const int64_t s = (int64_t)((uint64_t)y * (uint32_t)P);  // Q61
    return (q & 2u) ? -s : s;
}

// sin(n b pi / 2^32) / sin(b pi / 2^32) in Q16, b = (int32) beta, n >= 1: the
// modulus of the sum of n unit phasors advancing by beta per clock
__device__ __forceinline__ int64_t dirichlet_q16(uint32_t n, uint32_t beta)
{
    const int32_t b = (int32_t)beta;
    if (b == 0) return (int64_t)n << 16;
    const int64_t den = sin33((uint64_t)(int64_t)b);
    const int64_t num = sin33((uint64_t)((int64_t)n * b));
    uint64_t ad = (uint64_t)(den < 0 ? -den : den), an = (uint64_t)(num < 0 ? -num : num);
    const int bl = 64 - __clzll((long long)ad);               // ad > 0
    const int sh = bl > 31 ? bl - 31 : 0;                     // the divisor below 2^31
    ad >>= sh;
    an >>= sh;
    const int64_t qv = (int64_t)((an << 16) / ad);
    return ((num < 0) != (den < 0)) ? -qv : qv;
}

// env length field (bits 23:12) in env words, 0 (a CW envelope) = 4096
__device__ __forceinline__ uint32_t ro_words(uint32_t env) { const uint32_t L = (env >> 12) & 0xFFFu; return L ? L : 4096u; }

// meas_valid of a readout strobe at t_lo after the lane's previous one at
// last_tv (0: none): its window, then meas_latency, in order
__device__ __forceinline__ uint32_t demod_valid(const KParams &p, uint32_t t_lo, uint32_t pe, uint32_t last_tv)
{
    const uint32_t tv = t_lo + ro_words(pe) * p.ro_cpw + p.meas_latency;
    return tv > last_tv ? tv : last_tv + 1u;
}

// the lane's latest readout-drive strobe: its cycle, phase | freq << 17, and
// amp[15:0] | env length[27:16] | seen[31]
struct RoDrive {
    uint32_t t, pp, al;
};

// frequency word of freq index fi from a program's table {off, len}
// (dpemu_load_readout_freqs): 0 past its end
__device__ __forceinline__ uint32_t ro_freq(const KParams &p, uint32_t off, uint32_t len, uint32_t fi)
{
    return fi < len ? p.ro_fq[off + fi] : 0u;
}

// outcome of readout m (strobe at t_lo with pulse registers pe / pp, LO
// frequency word f_lo; the drive's f_d); acc = the accumulated {I, Q}.
// t_ref: the lane's latest pulse_reset
__device__ __forceinline__ uint32_t demod_readout(const KParams &p, uint64_t shot, uint32_t core, uint32_t m,
                                                  uint32_t thr, uint32_t t_lo, uint32_t pe, uint32_t pp,
                                                  const RoDrive d, uint32_t t_ref, uint32_t f_lo, uint32_t f_d,
                                                  int2 &acc)
{
    const uint3 r = philox3(p.seed, shot, core, m);
    const uint32_t s = (thr == 0xFFFFFFFFu) || (r.x < thr);
    int64_t sig_i = 0, sig_q = 0;
    if (d.al >> 31) {
        const uint32_t n_lo = ro_words(pe) * p.ro_cpw, n_d = ro_words(d.al >> 16 << 12) * p.ro_cpw;
        const uint32_t r0 = d.t + p.ro_delay;                   // the return starts (< 2^32: t < 2^31)
        const uint32_t a = max(r0, t_lo), e = min(t_lo + n_lo, r0 + n_d);
        if (e > a) {
            const uint32_t n = e - a;
            const uint32_t beta = f_d - f_lo;
            const uint32_t th = s ? p.ro_theta1 : p.ro_theta0;
            const uint32_t alpha = beta * (a - t_ref) - f_d * p.ro_delay + (((d.pp & 0x1FFFFu) - (pp & 0x1FFFFu)) << 15) + th;
            const uint32_t gamma = alpha + (uint32_t)(uint64_t)(((int64_t)(n - 1u) * (int32_t)beta) >> 1);
            const int64_t dq = dirichlet_q16(n, beta);
            const int64_t c15 = (sin33(((uint64_t)gamma << 1) + 0x80000000ull) + (1ll << 45)) >> 46;
            const int64_t s15 = (sin33((uint64_t)gamma << 1) + (1ll << 45)) >> 46;
            const int64_t amp = (int64_t)(((uint64_t)(d.al & 0xFFFFu) * (s ? p.ro_gain1 : p.ro_gain0)) >> 16);
            const int64_t M = amp * dq;
            sig_i = (M * c15 + (1ll << 31)) >> 32;
            sig_q = (M * s15 + (1ll << 31)) >> 32;
        }
    }
    const int32_t u0 = (int32_t)(r.y & 0xFFFFu), u1 = (int32_t)(r.y >> 16);
    const int32_t u2 = (int32_t)(r.z & 0xFFFFu), u3 = (int32_t)(r.z >> 16);
    const int64_t zi = u0 + u1 - u2 - u3, zq = u0 - u1 + u2 - u3;
    acc.x = (int32_t)(sig_i + ((zi * (int64_t)p.ro_sigma) >> 16));
    acc.y = (int32_t)(sig_q + ((zq * (int64_t)p.ro_sigma) >> 16));
    const uint32_t ax = p.ro_axis[core];
    const int64_t x = ((int64_t)acc.x * (int16_t)(ax & 0xFFFFu) + (int64_t)acc.y * (int16_t)(ax >> 16)) >> 15;
    return x > (int64_t)p.ro_thr;
}

__device__ __forceinline__ uint64_t group_bits(uint64_t ballot, uint32_t lane_in_wave, uint32_t C)
{
    const uint32_t base = lane_in_wave & ~(C - 1);
    const uint64_t gm = (C >= 64) ? ~0ull : ((1ull << C) - 1);
    return (ballot >> base) & gm;
}

__device__ __forceinline__ uint32_t fast_div(uint32_t n, const uint32_t d[3])
{
    const uint32_t t = __umulhi(d[0], n);
    return (t + ((n - t) >> d[1])) >> d[2];
}

// program group of the run's shot sl: (shot / spg) % n_groups from the run's
// first shot (g0, r0 from the host) in 32-bit arithmetic, the divisions by
// multiply-high with host-made constants (kernels.h fast_div_init); a u64
// division would cost ~150 VALU instructions per lane, a u32 one ~20
// (r0 + sl) / spg: the group step of run shot sl past the run's first group
__device__ __forceinline__ uint32_t group_q(const KParams &p, uint32_t sl)
{
    const uint64_t num = (uint64_t)p.grp_r0 + sl;
    return (num >> 32) ? (uint32_t)(num / p.shots_per_group) : fast_div((uint32_t)num, p.spg_div);
}

__device__ __forceinline__ uint32_t shot_group(const KParams &p, uint32_t sl)
{
    const uint32_t q = group_q(p, sl);
    const uint32_t g = p.grp_g0 + (q - fast_div(q, p.ng_div) * p.n_groups);   // < 2 n_groups <= 2^32
    return g >= p.n_groups ? g - p.n_groups : g;
}

// index of the program-group "step" of shot sp relative to shot sp0 of the run
__device__ __forceinline__ uint32_t group_step(const KParams &p, uint32_t sp, uint32_t sp0)
{
    if (p.n_groups == 1) return 0;
    // (shot_begin + x) / spg = shot_begin / spg + (r0 + x) / spg
    return group_q(p, sp) - group_q(p, sp0);
}

// output lane of (run shot sl, core) (include/dpemu.h): core-major, or
// shot-major with lane_order DPEMU_LANES_SHOT_MAJOR
__device__ __forceinline__ uint32_t out_lane(const KParams &p, uint32_t sl, uint32_t core)
{
    return p.shot_major ? (sl << p.log2C) + core : core * p.n_shots + sl;
}

// an output store, nontemporal (streaming: written whole, never read back
// by the kernel) when nt
typedef uint32_t st_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t st_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_out(uint4 *dst, const uint4 v, bool nt)
{
    if (nt) __builtin_nontemporal_store(st_u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<st_u32x4 *>(dst));
    else *dst = v;
}
__device__ __forceinline__ void st_out(uint2 *dst, const uint2 v, bool nt)
{
    if (nt) __builtin_nontemporal_store(st_u32x2{v.x, v.y}, reinterpret_cast<st_u32x2 *>(dst));
    else *dst = v;
}

// cache policy of a 16-B record store from a possibly partial wave: ST_WB
// write-back (L2 merges partial lines of later stores), ST_NT nontemporal,
// ST_NT_LINE nontemporal for the lanes whose 8-lane group -- one 128-B line
// of consecutive lanes -- all store (the rest write-back), ST_NT_WAVE
// nontemporal when the whole wave stores
enum StPolicy { ST_WB = 0, ST_NT = 1, ST_NT_LINE = 2, ST_NT_WAVE = 3 };
template <StPolicy P>
__device__ __forceinline__ void st_rec(uint4 *dst, const uint4 v)
{
    if constexpr (P == ST_WB || P == ST_NT) {
        st_out(dst, v, P == ST_NT);
    } else {
        const uint64_t m = __builtin_amdgcn_read_exec();
        const bool full = P == ST_NT_WAVE ? m == ~0ull : ((m >> (__lane_id() & 56u)) & 0xFFull) == 0xFFull;
        if (full) st_out(dst, v, true);
        else *dst = v;
    }
}

// the 16-B event record (include/dpemu.h): pulse_iface snapshot at cycle te
__device__ __forceinline__ uint4 event_record(uint32_t te, uint32_t pe, uint32_t pp, uint32_t pa, uint32_t kind)
{
    return make_uint4(te, event_word(pe, kind), pp, pa & 0xFFFFu);
}

// Stage the programs of this workgroup's (group, core) slots in LDS -- the
// analogue of each core's cmd_mem -- each with its zero guard command, and
// return the LDS command index of program slot (group of shot position spos,
// core).  Slots k = step * C + c
// run over the block's consecutive program groups (at most BLOCK slots and
// the footprint within the dynamic LDS: host-checked).  Every thread of the
// workgroup calls it (barriers).  s_pref: BLOCK + 1 words, s_scan: BLOCK / 64.
__device__ __forceinline__ uint32_t stage_programs(const KParams &p, uint4 *s_prog, uint32_t *s_pref,
                                                   uint32_t *s_scan, uint32_t spos, uint32_t my_core)
{
    const uint32_t tid = threadIdx.x, C = p.C;
    const uint32_t n_shots = p.n_lanes >> p.log2C;
    const uint32_t sp0 = (blockIdx.x * BLOCK) >> p.log2C;
    const uint32_t spl = min(sp0 + (BLOCK >> p.log2C), n_shots) - 1u;
    const uint32_t g0 = shot_group(p, sp0);
    const uint32_t nslots = (group_step(p, spl, sp0) + 1u) * C;
    uint32_t len = 0;
    if (tid < nslots) {
        const uint32_t gx = g0 + tid / C;
        const uint32_t g = gx - fast_div(gx, p.ng_div) * p.n_groups;
        len = p.n_instr[p.prog_table[(uint64_t)g * C + (tid & (C - 1))]] + 1u;   // + guard
    }
    uint32_t total;
    const uint32_t pre = block_exclusive_scan(len, s_scan, &total);
    if (tid < nslots) s_pref[tid] = pre;
    if (tid == 0) s_pref[nslots] = total;
    __syncthreads();
    for (uint32_t idx = tid; idx < total; idx += BLOCK) {
        uint32_t lo = 0, hi = nslots;                    // largest k with s_pref[k] <= idx
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pref[mid] <= idx) lo = mid; else hi = mid;
        }
        const uint32_t gx = g0 + lo / C;
        const uint32_t g = gx - fast_div(gx, p.ng_div) * p.n_groups;
        const uint32_t prog = p.prog_table[(uint64_t)g * C + (lo & (C - 1))];
        s_prog[idx] = p.uops[p.offsets[prog] + (idx - s_pref[lo])];
    }
    __syncthreads();
    const uint32_t sp = min(spos, spl);                  // threads past the run: any slot
    return s_pref[group_step(p, sp, sp0) * C + my_core];
}

// Thread -> (shot, core) of the branch-free kernels (straight.hip, macro.hip):
// workgroup b covers the run's shots [b S, (b + 1) S), S = BLOCK / C, all C
// cores, in the output's lane order inside the workgroup: core-major lanes
// (thread = core * S + shot) put consecutive shots of one core in a wave,
// shot-major lanes (thread = shot * C + core) whole shots -- either way a
// wave's lanes are consecutive output lanes, so every event / summary store
// of a wave is one contiguous run.  The slot of the thread's shot in the
// workgroup (count_outcome_block) is shot_slot.
__device__ __forceinline__ void block_core_major(const KParams &p, uint32_t &sl, uint32_t &core)
{
    const uint32_t S_log2 = 8u - p.log2C;                // BLOCK = 256
    if (p.shot_major) {
        core = threadIdx.x & (p.C - 1u);
        sl = (blockIdx.x << S_log2) + (threadIdx.x >> p.log2C);
    } else {
        core = threadIdx.x >> S_log2;
        sl = (blockIdx.x << S_log2) + (threadIdx.x & ((1u << S_log2) - 1u));
    }
}

__device__ __forceinline__ uint32_t shot_slot(const KParams &p)
{
    return p.shot_major ? threadIdx.x >> p.log2C : threadIdx.x & ((1u << (8u - p.log2C)) - 1u);
}

// dpemu_outputs.hist_next: the caller's next histogram buffer set to zero in
// passing (vector stores, one u64 per thread of the first workgroups; it is
// disjoint from this run's hist, so no ordering with the counting is needed)
__device__ __forceinline__ void clear_hist_next(const KParams &p)
{
    if (!p.hist_next) return;
    const uint64_t n = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < p.hist_bins; i += n) p.hist_next[i] = 0ull;
}

// the outcome histogram for block_core_major workgroups: each lane ORs its
// last measurement into its shot's key in LDS, then one thread per shot
// counts the key (every thread of the workgroup calls it: barriers)
__device__ __forceinline__ void count_outcome_block(const KParams &p, uint32_t *s_hist, uint32_t *s_key, bool valid,
                                                    uint32_t core, uint32_t sl, uint32_t grp, uint32_t last_bit)
{
    if (!p.hist && !p.hist_rep) return;                  // uniform
    const uint32_t tid = threadIdx.x, S_log2 = 8u - p.log2C, S = 1u << S_log2;
    const uint32_t slot = shot_slot(p);
    if (tid < S) s_key[tid] = 0u;
    __syncthreads();
    if (valid && last_bit) atomicOr(&s_key[slot], 1u << core);
    __syncthreads();
    const bool mine = valid && core == 0u;               // thread (core 0, shot): the shot's count
    const uint32_t key = mine ? s_key[slot] : 0u;
    const uint64_t bin = (uint64_t)grp * (1ull << p.C) + key;
    if (p.hist_rep) {
        uint32_t *rep = p.hist_rep + (uint64_t)(blockIdx.x % p.hist_reps) * p.hist_stride;
        if (p.hist_lds) {
            if (mine) atomicAdd(&s_hist[bin], 1u);
            __syncthreads();
            const uint32_t bins = p.n_groups << p.C;
            for (uint32_t i = tid; i < bins; i += BLOCK)
                if (s_hist[i]) atomicAdd(&rep[i], s_hist[i]);
        } else if (mine) {
            atomicAdd(&rep[bin], 1u);
        }
    } else if (mine) {
        atomicAdd(&p.hist[bin], 1ull);
    }
    (void)sl;
}

// dpemu_outputs::summary row of a lane (include/dpemu.h)
__device__ __forceinline__ void write_summary(const KParams &p, uint32_t lane, uint32_t t_end, uint32_t ip,
                                              uint32_t status, uint32_t flags, uint32_t n_ev, uint32_t n_exec,
                                              uint32_t qclk_end, uint32_t n_meas, uint32_t meas_bits, uint32_t n_tr)
{
    uint4 *s = reinterpret_cast<uint4 *>(p.summary + 8ull * lane);
    const uint4 s0 = make_uint4(t_end, (ip & 0xFFFFu) | ((status & 0xFFu) << 16) | ((flags & 0xFFu) << 24), n_ev, n_exec);
    const uint4 s1 = make_uint4(qclk_end, n_meas, meas_bits, n_tr);
#if defined(DPEMU_ST_POLICY) && (DPEMU_ST_POLICY & 4)
    st_out(s, s0, true);
    st_out(s + 1, s1, true);
#else
    s[0] = s0;
    s[1] = s1;
#endif
}

// outcome histogram: bit c of the key = last measurement of core c; one count per
// shot into bin grp << C | key (direct u64 atomics, or a privatised u32 replica
// with optional LDS pre-aggregation; capi.cpp chooses).  Called by every thread
// of the workgroup (the LDS path has a barrier).
__device__ __forceinline__ void count_outcome(const KParams &p, uint32_t *s_hist, bool valid, uint32_t core,
                                              uint32_t grp, uint32_t last_bit)
{
    const uint32_t C = p.C, tid = threadIdx.x, wl = tid & 63;
    if (p.hist_rep) {
        const uint64_t key = group_bits(__ballot(last_bit != 0u), wl, C);
        const uint64_t bin = (uint64_t)grp * (1ull << C) + key;
        uint32_t *rep = p.hist_rep + (uint64_t)(blockIdx.x % p.hist_reps) * p.hist_stride;
        if (p.hist_lds) {
            // small histogram: aggregate the workgroup's shots in LDS first
            if (valid && core == 0u) atomicAdd(&s_hist[bin], 1u);
            __syncthreads();
            const uint32_t bins = p.n_groups << C;
            for (uint32_t i = tid; i < bins; i += BLOCK)
                if (s_hist[i]) atomicAdd(&rep[i], s_hist[i]);
        } else if (valid && core == 0u) {
            atomicAdd(&rep[bin], 1u);
        }
    } else if (p.hist) {
        const uint64_t key = group_bits(__ballot(last_bit != 0u), wl, C);
        if (valid && core == 0u) atomicAdd(&p.hist[(uint64_t)grp * (1ull << C) + key], 1ull);
    }
}

}  // namespace dpemu
