// dds.hip -- fixed-point DDS I/Q synthesis from emulated pulse events (gfx950).
//
// Spec: DESIGN.md §4.3 and oracle/dds_ref.c (CPU restatement, bit-exact).
// Inputs are the interpreter's outputs in HBM (lane summaries + slot-major
// event records) and the assembler's env / freq buffers (asmparse.py:46-86
// formats).  HBM-write-bound by design: 4 B per output sample.
//
// Two launches per synthesis:
//   * dds_index_kernel (one wave per channel) compacts the lane's strobes
//     of the channel's element and its pulse_resets (time-sorted: a core emits
//     them in time order) once, channel-contiguous, plus each chunk's window;
//   * dds_chunk_kernel, grid (sample chunks, channels).  A workgroup loads its
//     window of records, stages the sine table and the channel's env / freq
//     tables in LDS -- as (E, E') / (R, R') pairs for the Y-form products --
//     and sweeps its chunk with no global loads in the loop: on gfx950 stores
//     count in vmcnt, and a load in the loop would make every tile wait for
//     the previous tile's stores.  A pulse's fields are decoded once per
//     thread, the carrier once per 4 or 8 samples.  The production
//     instances (LSPT = 4 / 8, the "lean" kernel) hold only that path plus
//     the generic per-sample sweep, so they fit 64 VGPRs (8 waves per SIMD).
//     Default: LSPT = 4 (each thread one 16-B store per tile, 1 KiB dense
//     per wave-instruction).
//
// Store layout: thread-contiguous 4 (default) or 8 samples.  A/B history
// (scripts/ab_dds.py, config 5, 1.72 GB per launch, medians incl. the index
// kernel's 0.018 ms; a torch fill of the same buffer takes 0.245-0.25 ms):
//   * every workgroup compacting its own events (slot-major loads, one line
//     per event) vs the index kernel: 0.36 vs 0.35 ms at 32 Ki-sample chunks;
//     the index is what makes shorter chunks affordable;
//   * lean kernel, 16 Ki-sample chunks: LSPT 4: 0.322-0.342 ms; LSPT 8:
//     0.325-0.349 walking the strobes, 0.332-0.336 with the per-chunk cycle
//     table (fewer VALU, 8 KiB more LDS: fewer resident workgroups);
//     8 / 24 / 32 Ki chunks: 0.37-0.45 / 0.36 / 0.36-0.37;
//   * the general kernel (89 VGPRs, 5 waves per SIMD), X/Y form: 0.352-0.358
//     at 32 Ki chunks, 0.397 at 16 Ki;
//   * the same grid and prologue with zero stores: 0.343 ms (general kernel,
//     16 Ki); bare chunk-shaped stores 0.29-0.30 (scripts/micro/
//     store_probe.hip): short 1-D fill-shaped workgroups (4-16 KiB) reach
//     6.5-7.0 TB/s, 128-KiB chunks 5.6-6.0, persistent grids 4.8-5.4.  The
//     kernel sits on its store pattern, not on its arithmetic;
//   * a two-kernel design with a per-tile segment table and one short
//     fill-like workgroup per 1-8 KiB tile lost (3.2-3.5 TB/s): every tile
//     paid a chain of dependent table lookups.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.h"

namespace dpemu {

constexpr uint32_t DDS_CYC_CHUNK_MAX = 64 * BLOCK;   // the lean kernel's cycle table: 8 entries per thread, spc >= 8

#ifndef LWAVES
#define LWAVES 8            // waves per SIMD the lean chunk kernel is register-budgeted for
#endif

// a.lo * b.lo + a.hi * b.hi + c on packed int16 pairs: one VOP3P
// v_dot2_i32_i16 with the rounding constant in an SGPR
__device__ __forceinline__ int32_t dot2(uint32_t a, uint32_t b, int32_t c)
{
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

__device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return min(max(v, lo), hi); }

// {lo[15:0], hi[15:0]} in one v_perm_b32
__device__ __forceinline__ uint32_t pack16(int32_t lo, int32_t hi)
{
    return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}

// Complex products as dot2 pairs.  Words hold I in the high and Q in the low
// half.  With X = {lo: -bq, hi: bi} and Y = {lo: bi, hi: bq}:
//   (a (x) b).re = ai*bi - aq*bq = dot2(a, X),  .im = ai*bq + aq*bi = dot2(a, Y).
// bq is never -32768 here (table and rotated carriers are symmetric), so -bq
// fits in int16, and every sum stays inside int32.
struct Carrier {
    uint32_t X, Y;
};

// a0 = (c0 * amp + 2^15) >> 16 from the carrier (cos, sin) = table entries
__device__ __forceinline__ Carrier carrier_cs(int32_t c, int32_t s, int32_t amp)
{
    const int32_t a16 = amp & 0xFFFF;           // |c0| < 2^15, amp < 2^16: v_mad_i32_i24
    const int32_t ai = (c * a16 + (1 << 15)) >> 16;
    const int32_t aq = (s * a16 + (1 << 15)) >> 16;
    return Carrier{pack16(-aq, ai), pack16(ai, aq)};
}

// from the Q15 table at theta >> 20
__device__ __forceinline__ Carrier carrier(const int16_t *lut, uint32_t theta, int32_t amp)
{
    const uint32_t idx = theta >> 20;
    return carrier_cs(lut[(idx + 1024) & 4095], lut[idx], amp);
}

// the Q15 table is exactly antisymmetric (sin[i + 2048] = -sin[i]: built from
// the first quadrant, dpemu_dds_sin_lut), so the lean kernel stages half of it
__device__ __forceinline__ int32_t lut_half(const int16_t *lut, uint32_t i)
{
    const int32_t v = lut[i & 2047u];
    return (i & 2048u) ? -v : v;
}

__device__ __forceinline__ Carrier carrier_half(const int16_t *lut, uint32_t theta, int32_t amp)
{
    const uint32_t idx = theta >> 20;
    return carrier_cs(lut_half(lut, (idx + 1024) & 4095), lut_half(lut, idx), amp);
}

// a = symsat((a0 (x) R_k + 2^14) >> 15)
__device__ __forceinline__ Carrier rotate(Carrier a0, uint32_t rw)
{
    const int32_t cr = clampi(dot2(rw, a0.X, 1 << 14) >> 15, -32767, 32767);
    const int32_t cq = clampi(dot2(rw, a0.Y, 1 << 14) >> 15, -32767, 32767);
    return Carrier{pack16(-cq, cr), pack16(cr, cq)};
}

typedef short short2_t __attribute__((ext_vector_type(2)));

// sat16((env (x) a + 2^14) >> 15), packed {I low, Q high}: the two
// saturations and the pack are one v_cvt_pk_i16_i32
__device__ __forceinline__ uint32_t mix(uint32_t ew, Carrier a)
{
    const short2_t r = __builtin_amdgcn_cvt_pk_i16(dot2(ew, a.X, 1 << 14) >> 15, dot2(ew, a.Y, 1 << 14) >> 15);
    return __builtin_bit_cast(uint32_t, r);
}

// last index i < n with t[i] <= x, or -1
__device__ __forceinline__ int last_le(const uint32_t *t, int n, uint32_t x)
{
    int lo = 0, hi = n;                 // first index with t > x
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (t[mid] <= x) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store4(uint32_t *out, uint32_t j0, uint32_t c_end, const uint32_t v[4])
{
    if (j0 + 3 < c_end) {
        const u32x4 w = {v[0], v[1], v[2], v[3]};
        *reinterpret_cast<u32x4 *>(out + j0) = w;
    } else {
        for (int s = 0; s < 4 && j0 + s < c_end; s++) out[j0 + s] = v[s];
    }
}

// ---------------------------------------------------------------------------
// Event compaction: the channel's strobes (kind 0, cfg & 3 ==
// elem) and the lane's pulse_resets, in event (= time) order, into LDS.
// Every global load of the events is issued before the first barrier.
// ---------------------------------------------------------------------------
// sink(i, ev, amp) stores strobe i (ev = {t, -, env | cfg | kind, phase | freq index}).
template <class StrobeSink>
__device__ __forceinline__ void compact_events(const DDSParams &p, uint32_t lane, uint32_t elem, StrobeSink sink,
                                               uint32_t *rs_t, uint32_t *s_tmp, uint32_t *s_cnt, int *n_st, int *n_rs)
{
    const uint32_t tid = threadIdx.x, wl = tid & 63, wv = tid >> 6;
    uint32_t n_ev = min(p.summary[8ull * lane + 2], p.event_cap);
    constexpr int EV_PASSES = DDS_MAX_EVENTS / BLOCK;
    uint4 evr[EV_PASSES];
    uint32_t ampr[EV_PASSES];
#pragma unroll
    for (int ps = 0; ps < EV_PASSES; ps++) {
        const uint32_t e = ps * BLOCK + tid;
        evr[ps] = make_uint4(0, 0, 0, 0);
        ampr[ps] = 0;
        if (e < n_ev) {
            evr[ps] = p.ev_main[(uint64_t)e * p.n_lanes + lane];
            ampr[ps] = p.ev_amp[(uint64_t)e * p.n_lanes + lane];
        }
    }
    if (tid == 0) { s_cnt[0] = 0; s_cnt[1] = 0; }
    __syncthreads();
#pragma unroll
    for (int ps = 0; ps < EV_PASSES; ps++) {
        if ((uint32_t)ps * BLOCK >= n_ev) break;    // uniform
        const uint32_t e = ps * BLOCK + tid;
        const uint4 ev = evr[ps];
        const uint32_t kind = ev.z >> 28;
        const bool is_st = e < n_ev && kind == 0u && ((ev.z >> 24) & 3u) == elem;
        const bool is_rs = e < n_ev && kind == 1u;
        const uint64_t bs = __ballot(is_st), br = __ballot(is_rs);
        const uint64_t below = (wl == 0) ? 0ull : (~0ull >> (64 - wl));
        if (wl == 0) { s_tmp[wv] = (uint32_t)__popcll(bs); s_tmp[BLOCK / 64 + wv] = (uint32_t)__popcll(br); }
        __syncthreads();
        uint32_t os = s_cnt[0], orr = s_cnt[1], ts = 0, tr = 0;
        for (uint32_t k = 0; k < BLOCK / 64; k++) {
            os += (k < wv) ? s_tmp[k] : 0u;
            orr += (k < wv) ? s_tmp[BLOCK / 64 + k] : 0u;
            ts += s_tmp[k];
            tr += s_tmp[BLOCK / 64 + k];
        }
        if (is_st) sink(os + (uint32_t)__popcll(bs & below), ev, ampr[ps]);
        if (is_rs) rs_t[orr + (uint32_t)__popcll(br & below)] = ev.x;
        __syncthreads();
        if (tid == 0) { s_cnt[0] += ts; s_cnt[1] += tr; }
        __syncthreads();
    }
    *n_st = (int)s_cnt[0];
    *n_rs = (int)s_cnt[1];
}

// ---------------------------------------------------------------------------
// Y-form complex products (the segment kernel and the chunk kernel's quad
// sweep; see the comment above dds_seg_kernel)
// ---------------------------------------------------------------------------
typedef short short2v __attribute__((ext_vector_type(2)));

// {lo: hi, hi: -lo} of an I16|Q16 word
__device__ __forceinline__ uint32_t neg_swap(uint32_t w) { return (w >> 16) | (((0u - w) & 0xFFFFu) << 16); }

// dot2 results (+2^14) >> 15 of two components -> {lo, hi} saturated to int16
__device__ __forceinline__ uint32_t pk_sat(int32_t lo, int32_t hi)
{
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(lo >> 15, hi >> 15));
}

// a0 (x) R_k, symsat, Y form
__device__ __forceinline__ uint32_t rot_y(uint32_t y0, uint32_t r, uint32_t rp)
{
    const short2v v = __builtin_bit_cast(short2v, pk_sat(dot2(rp, y0, 1 << 14), dot2(r, y0, 1 << 14)));
    const short2v lo = {-32767, -32767};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, lo));
}

// sat16(E (x) a), packed {I low, Q high}
__device__ __forceinline__ uint32_t mix_y(uint32_t e, uint32_t ep, uint32_t y)
{
    return pk_sat(dot2(ep, y, 1 << 14), dot2(e, y, 1 << 14));
}

// ===========================================================================
// Chunk path
// ===========================================================================
struct QuadArgs {
    const int16_t *lut;
    const uint32_t *st_t, *st_env, *st_pf;
    const uint16_t *st_amp;
    const uint32_t *rs_t;
    int n_st, n_rs;
    uint32_t spc, spc_sh, interp, int_sh;
    const uint32_t *env;            // channel's env table (LDS)
    uint32_t env_len;
    const uint32_t *freq;           // channel's freq table (LDS)
    uint32_t freq_len;
    uint32_t *out;
    uint32_t c_end;                 // end of this workgroup's samples
    const uint32_t *cyc;            // optional cycle table: entry n - n_first = (strobe + 1) | (reset + 1) << 16
    uint32_t n_first;
};

// Quad sweep: a thread's SPT consecutive samples (SPT | spc) share one
// emulated cycle.  The tile stride SPT * BLOCK is a multiple of spc, so a
// thread's sub-sample slot k0 is fixed and its SPT rotation words change only
// with the pulse.
template <int SPT>
__device__ __forceinline__ void sweep_quad(const QuadArgs &q, uint32_t j_first)
{
    constexpr int NV = SPT / 4;
    const uint32_t k0 = j_first & (q.spc - 1);
    int si = last_le(q.st_t, q.n_st, j_first >> q.spc_sh), ri = last_le(q.rs_t, q.n_rs, j_first >> q.spc_sh);
    int cur = -2;                                   // strobe whose fields are cached
    bool act = false;                               // strobe plays (freq entry valid)
    uint32_t base = 0, lim = 0, emask = 0, F0 = 0, ph15 = 0;
    int32_t amp = 0;
    uint32_t r[SPT];                                // rotation words R_{k0+s}
#pragma unroll
    for (int s = 0; s < SPT; s++) r[s] = 0;
    const uint32_t *envp = q.env;
    for (uint32_t j0 = j_first; j0 < q.c_end; j0 += SPT * BLOCK) {
        const uint32_t n = j0 >> q.spc_sh;
        while (si + 1 < q.n_st && q.st_t[si + 1] <= n) si++;
        while (ri + 1 < q.n_rs && q.rs_t[ri + 1] <= n) ri++;
        uint32_t v[SPT];
#pragma unroll
        for (int s = 0; s < SPT; s++) v[s] = 0;
        if (si != cur) {                            // new pulse: decode its fields once
            cur = si;
            act = false;
            if (si >= 0) {
                const uint32_t env_w = q.st_env[si], pf = q.st_pf[si];
                const uint32_t A = env_w & 0xFFFu, L = (env_w >> 12) & 0xFFFu, fi = pf >> 17;
                base = q.st_t[si] * q.spc;          // sample index of the strobe
                // samples d = j - base with env index (d >> int_sh) & emask inside the
                // pulse and the table: d < lim
                const uint32_t room = q.env_len > 4 * A ? q.env_len - 4 * A : 0u;
                if (L) {
                    emask = 0xFFFFFFFFu;
                    const uint32_t n_env = min(4 * L, room);
                    lim = n_env << q.int_sh;
                    if ((lim >> q.int_sh) != n_env) lim = 0xFFFFFFFFu;   // no overflow past 2^32
                } else {
                    emask = 0u;                     // CW: env word 4A forever
                    lim = room ? 0xFFFFFFFFu : 0u;
                }
                envp = q.env + 4 * A;
                act = 16 * fi + 15 < q.freq_len;
                if (act) {
                    const uint32_t *frp = q.freq + 16 * fi;
                    F0 = frp[0];
#pragma unroll
                    for (int h = 0; h < NV; h++) {
                        const uint4 rw = *reinterpret_cast<const uint4 *>(frp + k0 + 4 * h);
                        r[4 * h] = rw.x; r[4 * h + 1] = rw.y; r[4 * h + 2] = rw.z; r[4 * h + 3] = rw.w;
                    }
                }
                ph15 = (pf & 0x1FFFFu) << 15;
                amp = q.st_amp[si];
            }
        }
        if (act) {
            const uint32_t t_ref = ri >= 0 ? q.rs_t[ri] : 0u;
            const Carrier a0 = carrier(q.lut, F0 * (n - t_ref) + ph15, amp);
            uint32_t ew[SPT];
            const uint32_t d0 = j0 - base;
            if (q.interp == 1 && d0 + (SPT - 1) < lim && emask) {
#pragma unroll
                for (int h = 0; h < NV; h++) {
                    const uint4 e4 = *reinterpret_cast<const uint4 *>(envp + d0 + 4 * h);
                    ew[4 * h] = e4.x; ew[4 * h + 1] = e4.y; ew[4 * h + 2] = e4.z; ew[4 * h + 3] = e4.w;
                }
            } else {
#pragma unroll
                for (int s = 0; s < SPT; s++)
                    ew[s] = d0 + s < lim ? envp[((d0 + s) >> q.int_sh) & emask] : 0u;
            }
#pragma unroll
            for (int s = 0; s < SPT; s++) {
                Carrier a = rotate(a0, r[s]);
                if (s == 0 && k0 == 0) a = a0;      // sub-sample 0 is the unrotated carrier
                v[s] = mix(ew[s], a);
            }
            if (d0 + (SPT - 1) >= lim) {            // the pulse ends inside these samples
#pragma unroll
                for (int s = 0; s < SPT; s++) v[s] = d0 + s < lim ? v[s] : 0u;
            }
        }
#pragma unroll
        for (int h = 0; h < NV; h++) store4(q.out, j0 + 4 * h, q.c_end, v + 4 * h);
    }
}

// Quad sweep in Y form: the same walk as sweep_quad, with the rotation pairs
// (R, R') staged in LDS and the env words as (E, E') pairs (PAIRS, interp 1)
// or single words (E' formed per word), so a sample costs 2 dot2 + pack +
// max for the rotation and 2 dot2 + pack for the mix.  Needs every staged
// eq, rq != -32768 (the workgroup's tables; else the generic sweep runs).
template <int SPT, bool PAIRS, bool HALF>
__device__ __forceinline__ void sweep_quad_y(const QuadArgs &q, uint32_t j_first)
{
    const uint32_t k0 = j_first & (q.spc - 1);
    int si = last_le(q.st_t, q.n_st, j_first >> q.spc_sh), ri = last_le(q.rs_t, q.n_rs, j_first >> q.spc_sh);
    int cur = -2;
    bool act = false;
    uint32_t base = 0, lim = 0, emask = 0, F0 = 0, ph15 = 0;
    int32_t a16 = 0;
    uint32_t R[SPT], Rp[SPT];
#pragma unroll
    for (int s = 0; s < SPT; s++) R[s] = Rp[s] = 0;
    const uint32_t *envp = q.env;
    for (uint32_t j0 = j_first; j0 < q.c_end; j0 += SPT * BLOCK) {
        const uint32_t n = j0 >> q.spc_sh;
        if (q.cyc) {                                // one LDS word instead of walking the strobes
            const uint32_t w = q.cyc[n - q.n_first];
            si = (int)(w & 0xFFFFu) - 1;
            ri = (int)(w >> 16) - 1;
        } else {
            while (si + 1 < q.n_st && q.st_t[si + 1] <= n) si++;
            while (ri + 1 < q.n_rs && q.rs_t[ri + 1] <= n) ri++;
        }
        uint32_t v[SPT];
#pragma unroll
        for (int s = 0; s < SPT; s++) v[s] = 0;
        if (si != cur) {                            // new pulse: decode its fields once
            cur = si;
            act = false;
            if (si >= 0) {
                const uint32_t env_w = q.st_env[si], pf = q.st_pf[si];
                const uint32_t A = env_w & 0xFFFu, L = (env_w >> 12) & 0xFFFu, fi = pf >> 17;
                base = q.st_t[si] * q.spc;
                const uint32_t room = q.env_len > 4 * A ? q.env_len - 4 * A : 0u;
                if (L) {
                    emask = 0xFFFFFFFFu;
                    const uint32_t n_env = min(4 * L, room);
                    lim = n_env << q.int_sh;
                    if ((lim >> q.int_sh) != n_env) lim = 0xFFFFFFFFu;
                } else {
                    emask = 0u;
                    lim = room ? 0xFFFFFFFFu : 0u;
                }
                envp = q.env + (PAIRS ? 8 * A : 4 * A);
                act = 16 * fi + 15 < q.freq_len;
                if (act) {
                    const uint32_t *frp = q.freq + 32 * fi;     // (R, R') pairs; pair 0 = (F0, 0)
                    F0 = frp[0];
#pragma unroll
                    for (int h = 0; h < SPT / 2; h++) {
                        const uint4 w = *reinterpret_cast<const uint4 *>(frp + 2 * k0 + 4 * h);
                        R[2 * h] = w.x; Rp[2 * h] = w.y; R[2 * h + 1] = w.z; Rp[2 * h + 1] = w.w;
                    }
                }
                ph15 = (pf & 0x1FFFFu) << 15;
                a16 = q.st_amp[si];
            }
        }
        if (act && j0 - base < lim) {               // (a finished pulse plays zeros)
            const uint32_t t_ref = ri >= 0 ? q.rs_t[ri] : 0u;
            const uint32_t idx = (F0 * (n - t_ref) + ph15) >> 20;
            const int32_t c = HALF ? lut_half(q.lut, (idx + 1024) & 4095) : q.lut[(idx + 1024) & 4095];
            const int32_t sn = HALF ? lut_half(q.lut, idx) : q.lut[idx];
            const uint32_t y0 = pack16((c * a16 + (1 << 15)) >> 16, (sn * a16 + (1 << 15)) >> 16);
            uint32_t E[SPT], Ep[SPT];
            const uint32_t d0 = j0 - base;
            const bool inside = d0 + (SPT - 1) < lim;
            if (PAIRS && inside && emask) {
#pragma unroll
                for (int h = 0; h < SPT / 2; h++) {
                    const uint4 w = *reinterpret_cast<const uint4 *>(envp + 2 * d0 + 4 * h);
                    E[2 * h] = w.x; Ep[2 * h] = w.y; E[2 * h + 1] = w.z; Ep[2 * h + 1] = w.w;
                }
            } else if (PAIRS) {
#pragma unroll
                for (int s = 0; s < SPT; s++) {
                    const uint32_t wi = (d0 + s) & emask;
                    E[s] = d0 + s < lim ? envp[2 * wi] : 0u;
                    Ep[s] = d0 + s < lim ? envp[2 * wi + 1] : 0u;
                }
            } else if (inside && (((d0 >> q.int_sh) == ((d0 + SPT - 1) >> q.int_sh)) || !emask)) {
                const uint32_t e = envp[(d0 >> q.int_sh) & emask], ep = neg_swap(e);   // one word for all
#pragma unroll
                for (int s = 0; s < SPT; s++) { E[s] = e; Ep[s] = ep; }
            } else {
#pragma unroll
                for (int s = 0; s < SPT; s++) {
                    E[s] = d0 + s < lim ? envp[((d0 + s) >> q.int_sh) & emask] : 0u;
                    Ep[s] = neg_swap(E[s]);
                }
            }
#pragma unroll
            for (int s = 0; s < SPT; s++) {
                uint32_t y = rot_y(y0, R[s], Rp[s]);
                if (s == 0 && k0 == 0) y = y0;              // sub-sample 0 is the unrotated carrier
                v[s] = mix_y(E[s], Ep[s], y);
            }
            if (!inside) {                                  // the pulse ends inside these samples
#pragma unroll
                for (int s = 0; s < SPT; s++) v[s] = d0 + s < lim ? v[s] : 0u;
            }
        }
#pragma unroll
        for (int h = 0; h < SPT / 4; h++) store4(q.out, j0 + 4 * h, q.c_end, v + 4 * h);
    }
}

// Row sweep: per tile iteration a thread produces R quads, quad h at
// j0 + h * ROW (ROW = 4 * BLOCK samples, a multiple of spc), so every store
// instruction of a wave writes 1 KiB contiguous -- measured 5-7 % faster
// for bare stores than the thread-contiguous 32 B of sweep_quad<8>, whose
// two store instructions each leave every other 16 B of a line for the
// other (scripts/ab_dds.py probes).  Each row keeps its own pulse cursor.
struct RowCursor {
    int si, ri, cur;
    bool act;
    uint32_t base, lim, emask, F0, ph15, amp;
    uint32_t r[4];                  // rotation words R_{k0 .. k0+3}
    const uint32_t *envp;
};

__device__ __forceinline__ void row_init(const QuadArgs &q, RowCursor &c, uint32_t j_first)
{
    c.si = last_le(q.st_t, q.n_st, j_first >> q.spc_sh);
    c.ri = last_le(q.rs_t, q.n_rs, j_first >> q.spc_sh);
    c.cur = -2;
    c.act = false;
    c.base = c.lim = c.emask = c.F0 = c.ph15 = c.amp = 0;
#pragma unroll
    for (int s = 0; s < 4; s++) c.r[s] = 0;
    c.envp = q.env;
}

__device__ __forceinline__ void row_step(const QuadArgs &q, RowCursor &c, uint32_t j0, uint32_t k0, uint32_t v[4])
{
    const uint32_t n = j0 >> q.spc_sh;
    while (c.si + 1 < q.n_st && q.st_t[c.si + 1] <= n) c.si++;
    while (c.ri + 1 < q.n_rs && q.rs_t[c.ri + 1] <= n) c.ri++;
#pragma unroll
    for (int s = 0; s < 4; s++) v[s] = 0;
    if (c.si != c.cur) {                            // new pulse: decode its fields once
        c.cur = c.si;
        c.act = false;
        if (c.si >= 0) {
            const uint32_t env_w = q.st_env[c.si], pf = q.st_pf[c.si];
            const uint32_t A = env_w & 0xFFFu, L = (env_w >> 12) & 0xFFFu, fi = pf >> 17;
            c.base = q.st_t[c.si] * q.spc;
            const uint32_t room = q.env_len > 4 * A ? q.env_len - 4 * A : 0u;
            if (L) {
                c.emask = 0xFFFFFFFFu;
                const uint32_t n_env = min(4 * L, room);
                c.lim = n_env << q.int_sh;
                if ((c.lim >> q.int_sh) != n_env) c.lim = 0xFFFFFFFFu;
            } else {
                c.emask = 0u;
                c.lim = room ? 0xFFFFFFFFu : 0u;
            }
            c.envp = q.env + 4 * A;
            c.act = 16 * fi + 15 < q.freq_len;
            if (c.act) {
                const uint32_t *frp = q.freq + 16 * fi;
                c.F0 = frp[0];
                const uint4 rw = *reinterpret_cast<const uint4 *>(frp + k0);
                c.r[0] = rw.x; c.r[1] = rw.y; c.r[2] = rw.z; c.r[3] = rw.w;
            }
            c.ph15 = (pf & 0x1FFFFu) << 15;
            c.amp = q.st_amp[c.si];
        }
    }
    if (c.act) {
        const uint32_t t_ref = c.ri >= 0 ? q.rs_t[c.ri] : 0u;
        const Carrier a0 = carrier(q.lut, c.F0 * (n - t_ref) + c.ph15, (int32_t)c.amp);
        uint32_t ew[4];
        const uint32_t d0 = j0 - c.base;
        if (q.interp == 1 && d0 + 3 < c.lim && c.emask) {
            const uint4 e4 = *reinterpret_cast<const uint4 *>(c.envp + d0);
            ew[0] = e4.x; ew[1] = e4.y; ew[2] = e4.z; ew[3] = e4.w;
        } else {
#pragma unroll
            for (int s = 0; s < 4; s++) ew[s] = d0 + s < c.lim ? c.envp[((d0 + s) >> q.int_sh) & c.emask] : 0u;
        }
#pragma unroll
        for (int s = 0; s < 4; s++) {
            Carrier a = rotate(a0, c.r[s]);
            if (s == 0 && k0 == 0) a = a0;          // sub-sample 0 is the unrotated carrier
            v[s] = mix(ew[s], a);
        }
        if (d0 + 3 >= c.lim) {
#pragma unroll
            for (int s = 0; s < 4; s++) v[s] = d0 + s < c.lim ? v[s] : 0u;
        }
    }
}

template <int R>
__device__ __forceinline__ void sweep_rows(const QuadArgs &q, uint32_t c_begin)
{
    constexpr uint32_t ROW = 4 * BLOCK;
    const uint32_t j_first = c_begin + 4 * threadIdx.x;
    const uint32_t k0 = j_first & (q.spc - 1);      // the same in every row and tile
    RowCursor c[R];
#pragma unroll
    for (int h = 0; h < R; h++) row_init(q, c[h], j_first + h * ROW);
    for (uint32_t j0 = j_first; j0 < q.c_end; j0 += R * ROW) {
        uint32_t v[R][4];
#pragma unroll
        for (int h = 0; h < R; h++) row_step(q, c[h], j0 + h * ROW, k0, v[h]);
#pragma unroll
        for (int h = 0; h < R; h++)
            if (j0 + h * ROW < q.c_end) store4(q.out, j0 + h * ROW, q.c_end, v[h]);
    }
}

// LSPT = 0: the general kernel (every path, probe and A/B knob).  LSPT = 4 / 8:
// the lean production instance -- event index + Y-form quad sweep with LSPT
// samples per thread per tile (4 where spc is not a multiple of LSPT), the
// generic sweep for everything else -- whose register budget allows
// amdgpu_waves_per_eu(LWAVES) (more resident store streams per SIMD).
template <int LSPT>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(LSPT ? LWAVES : 1)))
dds_chunk_kernel(const DDSParams p)
{
    constexpr bool LEAN = LSPT != 0;
    // dynamic LDS (dds_lds_bytes): sine table | compacted strobes / resets |
    // staged env table | staged freq table
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    // (lean: half the sine table, dds_lds_bytes - 4096)
    constexpr uint32_t LUT_BYTES = LEAN ? 4096 : 8192;
    int16_t *s_lut = reinterpret_cast<int16_t *>(s_dyn);
    uint32_t *s_st_t = reinterpret_cast<uint32_t *>(s_dyn + LUT_BYTES);
    uint32_t *s_st_env = s_st_t + p.ev_lds;
    uint32_t *s_st_pf = s_st_env + p.ev_lds;
    uint32_t *s_rs_t = s_st_pf + p.ev_lds;
    uint32_t *s_env = s_rs_t + p.ev_lds;
    uint32_t *s_freq = s_env + p.env_lds;
    uint16_t *s_st_amp = reinterpret_cast<uint16_t *>(s_freq + p.freq_lds);
    __shared__ uint32_t s_tmp[2 * (BLOCK / 64)];
    __shared__ uint32_t s_cnt[2];

    const uint32_t tid = threadIdx.x;
    const uint32_t ch = blockIdx.y;
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
    if (d[1] & DDS_SEG_FLAG) return;        // synthesised by dds_seg_kernel
    const uint32_t lane = d[0], elem = d[1] & 3u, spc = d[2], interp = d[3] ? d[3] : 1u;
    const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
    const bool spc_p2 = (spc & (spc - 1)) == 0, int_p2 = (interp & (interp - 1)) == 0;
    const uint32_t spc_sh = __ffs(spc) - 1, int_sh = __ffs(interp) - 1;
    const bool yf = p.yform != 0;           // Y-form quad sweep: (R, R') and interp-1 (E, E') pairs staged
    const bool staged = yf ? (interp == 1 ? 2 * env_len : env_len) <= p.env_lds && 2 * freq_len <= p.freq_lds
                           : env_len <= p.env_lds && freq_len <= p.freq_lds;

    // prologue: every global load of the workgroup up front (compact_events
    // issues the event loads before its first barrier)
    // probes 8..11 (A/B only): the contiguous-store probe minus parts of the
    // prologue -- 8: no sine table, 9: no env / freq tables, 10: no event
    // window, 11: none of them, 12: none and no index kernel
    const uint32_t pr = p.probe;
    if (pr != 8 && pr < 11)
        for (uint32_t i = tid; i < LUT_BYTES / 16; i += BLOCK)
            reinterpret_cast<uint4 *>(s_lut)[i] = reinterpret_cast<const uint4 *>(p.sin_lut)[i];
    bool bad = false;                       // a staged eq or rq is -32768: no Y form
    if (pr == 9 || pr >= 11) {
    } else if (staged && yf) {
        if (interp == 1) {
            for (uint32_t i = tid; i < env_len; i += BLOCK) {
                const uint32_t e = p.env[env_off + i];
                bad |= (e & 0xFFFFu) == 0x8000u;
                reinterpret_cast<uint2 *>(s_env)[i] = make_uint2(e, neg_swap(e));
            }
        } else {
            for (uint32_t i = tid; i < env_len; i += BLOCK) {
                const uint32_t e = p.env[env_off + i];
                bad |= (e & 0xFFFFu) == 0x8000u;
                s_env[i] = e;
            }
        }
        for (uint32_t i = tid; i < freq_len; i += BLOCK) {
            const uint32_t w = p.freq[freq_off + i];
            const bool rot = (i & 15u) != 0;
            bad |= rot && (w & 0xFFFFu) == 0x8000u;
            reinterpret_cast<uint2 *>(s_freq)[i] = make_uint2(w, rot ? neg_swap(w) : 0u);
        }
    } else if (staged) {
        for (uint32_t i = tid; i < env_len; i += BLOCK) s_env[i] = p.env[env_off + i];
        for (uint32_t i = tid; i < freq_len; i += BLOCK) s_freq[i] = p.freq[freq_off + i];
    }
    int n_st = 0, n_rs = 0;
    if (!LEAN && pr >= 10) {
        __syncthreads();
    } else if (LEAN || p.xs) {     // indexed: this chunk's window of the channel's compacted events
        const uint4 w = p.win[(uint64_t)ch * gridDim.x + blockIdx.x];
        n_st = (int)w.y;
        n_rs = (int)w.w;
        const uint4 *xs = p.xs + (uint64_t)ch * p.ev_lds + w.x;
        const uint32_t *xr = p.xr + (uint64_t)ch * p.ev_lds + w.z;
        for (uint32_t i = tid; i < w.y; i += BLOCK) {
            const uint4 r = xs[i];
            s_st_t[i] = r.x; s_st_env[i] = r.y; s_st_pf[i] = r.z; s_st_amp[i] = (uint16_t)r.w;
        }
        for (uint32_t i = tid; i < w.w; i += BLOCK) s_rs_t[i] = xr[i];
        bad = __syncthreads_or(bad);
    } else if constexpr (!LEAN) {
        compact_events(
            p, lane, elem,
            [&](uint32_t i, const uint4 &ev, uint32_t amp) {
                s_st_t[i] = ev.x; s_st_env[i] = ev.z & 0xFFFFFFu; s_st_pf[i] = ev.w; s_st_amp[i] = (uint16_t)amp;
            },
            s_rs_t, s_tmp, s_cnt, &n_st, &n_rs);
        if (yf) bad = __syncthreads_or(bad);
    }

    uint32_t *out = p.iq + (uint64_t)ch * p.n_samples;
    const uint32_t c_begin = blockIdx.x * p.chunk;
    const uint32_t c_end = min(c_begin + p.chunk, p.n_samples);
    if (!LEAN && (p.probe == 3 || p.probe == 4 || p.probe >= 8)) {   // probes: zero stores of the sweep, 8 samples per thread per tile
        const uint32_t z[4] = {0, 0, 0, (uint32_t)(n_st + n_rs) & 0u};
        if (p.probe != 4 && p.rows == 0) {   // thread-contiguous 32 B (two half-dense store instructions)
            for (uint32_t j0 = c_begin + 8 * tid; j0 < c_end; j0 += 8 * BLOCK) {
                store4(out, j0, c_end, z);
                store4(out, j0 + 4, c_end, z);
            }
        } else {                 // rows: each store instruction dense (1 KiB per wave)
            for (uint32_t j0 = c_begin + 4 * tid; j0 < c_end; j0 += 8 * BLOCK) {
                store4(out, j0, c_end, z);
                store4(out, j0 + 4 * BLOCK, c_end, z);
            }
        }
        return;
    }
    const bool quad = staged && (spc & 3u) == 0 && spc_p2 && int_p2 && (interp == 1 || interp >= 4);
    const uint32_t n_c0 = c_begin >> spc_sh;     // the chunk's first cycle (power-of-two spc)
    uint32_t *s_cyc = nullptr;
    if (LEAN && LSPT == 8 && quad && !bad && (spc & 7u) == 0 && p.chunk <= DDS_CYC_CHUNK_MAX && p.cyc) {
        // cycle table of the chunk (<= chunk / 8 cycles): entry r = (1 + latest strobe at or
        // before cycle n_first + r) | (1 + latest reset) << 16, window indices, 0 = none.
        // Scatter each strobe / reset to its cycle (strobe and reset times are
        // strictly increasing; only window entry 0 can precede the chunk), then
        // an inclusive max-scan of both halves at once (v_pk_max_u16).
        s_cyc = reinterpret_cast<uint32_t *>(s_dyn + dds_lds_bytes(p.ev_lds, p.env_lds, p.freq_lds) - (8192 - LUT_BYTES));
        const uint32_t n_last = (c_end - 1) >> spc_sh;
        uint16_t *c16 = reinterpret_cast<uint16_t *>(s_cyc);
        reinterpret_cast<uint4 *>(s_cyc)[2 * tid] = make_uint4(0, 0, 0, 0);   // 8 entries per thread
        reinterpret_cast<uint4 *>(s_cyc)[2 * tid + 1] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        for (int i = (int)tid; i < n_st; i += BLOCK) {
            const uint32_t t = s_st_t[i];
            if (t <= n_last) c16[2 * (t > n_c0 ? t - n_c0 : 0u)] = (uint16_t)(i + 1);
        }
        for (int i = (int)tid; i < n_rs; i += BLOCK) {
            const uint32_t t = s_rs_t[i];
            if (t <= n_last) c16[2 * (t > n_c0 ? t - n_c0 : 0u) + 1] = (uint16_t)(i + 1);
        }
        __syncthreads();
        constexpr uint32_t PER = 8;                  // entries per thread (chunk / 8 <= 8 * BLOCK)
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        uint32_t e[PER];
        const uint4 w0 = reinterpret_cast<const uint4 *>(s_cyc)[2 * tid];
        const uint4 w1 = reinterpret_cast<const uint4 *>(s_cyc)[2 * tid + 1];
        e[0] = w0.x; e[1] = w0.y; e[2] = w0.z; e[3] = w0.w; e[4] = w1.x; e[5] = w1.y; e[6] = w1.z; e[7] = w1.w;
        auto pmax = [](uint32_t a, uint32_t b) {
            return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(us2, a),
                                                                         __builtin_bit_cast(us2, b)));
        };
#pragma unroll
        for (uint32_t k = 1; k < PER; k++) e[k] = pmax(e[k], e[k - 1]);
        const uint32_t wl = tid & 63, wv = tid >> 6;
        uint32_t m = e[PER - 1];
#pragma unroll
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(m, off);
            if (wl >= off) m = pmax(m, y);
        }
        if (wl == 63) s_tmp[wv] = m;
        uint32_t ex = __shfl_up(m, 1);
        if (wl == 0) ex = 0;
        __syncthreads();
        for (uint32_t k = 0; k < wv; k++) ex = pmax(ex, s_tmp[k]);
#pragma unroll
        for (uint32_t k = 0; k < PER; k++) e[k] = pmax(e[k], ex);
        reinterpret_cast<uint4 *>(s_cyc)[2 * tid] = make_uint4(e[0], e[1], e[2], e[3]);
        reinterpret_cast<uint4 *>(s_cyc)[2 * tid + 1] = make_uint4(e[4], e[5], e[6], e[7]);
        __syncthreads();
    }
    if (LEAN && p.probe == 13) {            // probe (A/B only): the lean kernel's prologue + zero stores
        const uint32_t z[4] = {0, 0, 0, (uint32_t)(n_st + n_rs) & 0u};
        for (uint32_t j0 = c_begin + 4 * tid; j0 < c_end; j0 += 4 * BLOCK) store4(out, j0, c_end, z);
        return;
    }
    if (quad && (LEAN || yf) && !bad) {
        const QuadArgs q{s_lut, s_st_t, s_st_env, s_st_pf, s_st_amp, s_rs_t, n_st, n_rs, spc, spc_sh, interp, int_sh,
                         s_env, env_len, s_freq, freq_len, out, c_end, s_cyc, n_c0};
        if (LSPT != 4 && (spc & 7u) == 0) {
            if (interp == 1) sweep_quad_y<8, true, LEAN>(q, c_begin + 8 * tid);
            else sweep_quad_y<8, false, LEAN>(q, c_begin + 8 * tid);
        } else {
            if (interp == 1) sweep_quad_y<4, true, LEAN>(q, c_begin + 4 * tid);
            else sweep_quad_y<4, false, LEAN>(q, c_begin + 4 * tid);
        }
        return;
    }
    if (!LEAN && quad && !yf) {
        const QuadArgs q{s_lut, s_st_t, s_st_env, s_st_pf, s_st_amp, s_rs_t, n_st, n_rs, spc, spc_sh, interp, int_sh,
                         s_env, env_len, s_freq, freq_len, out, c_end, nullptr, 0};
        switch (p.rows) {
        case 1: sweep_rows<1>(q, c_begin); break;
        case 2: sweep_rows<2>(q, c_begin); break;
        case 4: sweep_rows<4>(q, c_begin); break;
        default:
            if ((spc & 7u) == 0) sweep_quad<8>(q, c_begin + 8 * tid);
            else sweep_quad<4>(q, c_begin + 4 * tid);
        }
        return;
    }

    // ---- generic sweep: the per-sample definition ----
    // cursors: latest strobe / reset at or before the current cycle.  A
    // thread's samples only move forward, so after one binary search at the
    // first sample the cursors advance by a short linear scan per tile.
    const uint32_t j_first = c_begin + 4 * tid;
    const uint32_t n_first = spc_p2 ? (j_first >> spc_sh) : j_first / spc;
    int si = last_le(s_st_t, n_st, n_first), ri = last_le(s_rs_t, n_rs, n_first);
    for (uint32_t j0 = j_first; j0 < c_end; j0 += 4 * BLOCK) {
        uint32_t v[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t j = j0 + s;
            const uint32_t n = spc_p2 ? (j >> spc_sh) : j / spc, k = j - n * spc;
            while (si + 1 < n_st && s_st_t[si + 1] <= n) si++;
            while (ri + 1 < n_rs && s_rs_t[ri + 1] <= n) ri++;
            uint32_t o = 0;
            if (si >= 0) {
                const uint32_t env_w = s_st_env[si], pf = s_st_pf[si];
                const uint32_t A = env_w & 0xFFFu, L = (env_w >> 12) & 0xFFFu;
                const uint32_t r = j - s_st_t[si] * spc;
                const uint32_t es = L ? (int_p2 ? (r >> int_sh) : r / interp) : 0u;
                const uint32_t widx = 4 * A + es;
                const uint32_t fi = pf >> 17, phase = pf & 0x1FFFFu;
                if ((!L || es < 4 * L) && widx < env_len && 16 * fi + 15 < freq_len) {
                    const uint32_t *fr = p.freq + freq_off + 16 * fi;
                    const uint32_t t_ref = ri >= 0 ? s_rs_t[ri] : 0u;
                    const Carrier a0 = LEAN ? carrier_half(s_lut, fr[0] * (n - t_ref) + (phase << 15), s_st_amp[si])
                                            : carrier(s_lut, fr[0] * (n - t_ref) + (phase << 15), s_st_amp[si]);
                    o = mix(p.env[env_off + widx], k ? rotate(a0, fr[k]) : a0);
                }
            }
            v[s] = o;
        }
        store4(out, j0, c_end, v);
    }
}

// Event index of the chunk path: one wave per channel compacts the
// lane's strobes of the channel's element and its pulse_resets once (instead
// of once per chunk: the slot-major event loads are one 16-B line access per
// event), writes them channel-contiguous, and for every chunk the window of
// strobes / resets its sweep can see: from the latest one at or before the
// chunk's first cycle to the latest one at or before its last cycle.  The
// chunk kernel then loads only its window, coalesced.
__global__ void __launch_bounds__(BLOCK) dds_index_kernel(const DDSParams p)
{
    // one wave per channel, BLOCK / 64 channels per workgroup, no workgroup
    // barrier: each lane issues all its event loads (8 per lane cover 512
    // events) before the wave compacts them with ballot / popc straight into
    // the global index; the strobe / reset times also go to the wave's LDS
    // slice for the window searches
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    const uint32_t wl = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t ch = blockIdx.x * (BLOCK / 64) + wv;
    if (ch >= p.n_channels) return;                         // the whole wave
    uint32_t *s_st_t = reinterpret_cast<uint32_t *>(s_dyn) + (uint64_t)wv * 2 * p.ev_lds;
    uint32_t *s_rs_t = s_st_t + p.ev_lds;
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
    const uint32_t lane = d[0], elem = d[1] & 3u, spc = d[2];
    const uint32_t n_ev = min(p.summary[8ull * lane + 2], p.event_cap);
    uint4 *xs = p.xs + (uint64_t)ch * p.ev_lds;
    uint32_t *xr = p.xr + (uint64_t)ch * p.ev_lds;
    const uint64_t below = wl ? (~0ull >> (64 - wl)) : 0ull;
    uint32_t ns = 0, nr = 0;
    constexpr int K = 8;
    for (uint32_t e0 = 0; e0 < n_ev; e0 += 64 * K) {
        uint4 ev[K];
        uint32_t am[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint32_t e = e0 + 64 * k + wl;
            ev[k] = make_uint4(0, 0, 0, 0);
            am[k] = 0;
            if (e < n_ev) {
                ev[k] = p.ev_main[(uint64_t)e * p.n_lanes + lane];
                am[k] = p.ev_amp[(uint64_t)e * p.n_lanes + lane];
            }
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint32_t e = e0 + 64 * k + wl;
            const uint32_t kind = ev[k].z >> 28;
            const bool is_st = e < n_ev && kind == 0u && ((ev[k].z >> 24) & 3u) == elem;
            const bool is_rs = e < n_ev && kind == 1u;
            const uint64_t bs = __ballot(is_st), br = __ballot(is_rs);
            if (is_st) {
                const uint32_t i = ns + (uint32_t)__popcll(bs & below);
                xs[i] = make_uint4(ev[k].x, ev[k].z & 0xFFFFFFu, ev[k].w, am[k]);
                s_st_t[i] = ev[k].x;
            }
            if (is_rs) {
                const uint32_t i = nr + (uint32_t)__popcll(br & below);
                xr[i] = ev[k].x;
                s_rs_t[i] = ev[k].x;
            }
            ns += (uint32_t)__popcll(bs);
            nr += (uint32_t)__popcll(br);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the wave's LDS writes before its reads
    __builtin_amdgcn_wave_barrier();
    const int n_st = (int)ns, n_rs = (int)nr;
    const uint32_t chunks = (p.n_samples + p.chunk - 1) / p.chunk;
    for (uint32_t c = wl; c < chunks; c += 64) {
        const uint64_t c0 = (uint64_t)c * p.chunk, c1 = min(c0 + p.chunk, (uint64_t)p.n_samples) - 1;
        const uint32_t n0 = (uint32_t)(c0 / spc), n1 = (uint32_t)(c1 / spc);
        const int s0 = last_le(s_st_t, n_st, n0), s1 = last_le(s_st_t, n_st, n1);
        const int r0 = last_le(s_rs_t, n_rs, n0), r1 = last_le(s_rs_t, n_rs, n1);
        const int sl = max(s0, 0), rl = max(r0, 0);
        p.win[(uint64_t)ch * chunks + c] = make_uint4((uint32_t)sl, (uint32_t)(s1 + 1 - sl), (uint32_t)rl,
                                                     (uint32_t)(r1 + 1 - rl));
    }
}

// ===========================================================================
// Segment path: dds_seg_kernel (channels with spc in {8, 16}, power-of-two
// interp, env / freq tables staged in LDS; DDS_SEG_FLAG in the descriptor).
//
// The chunk kernel's sweep re-finds and re-decodes the current pulse on every
// tile, and on pulse-dense channels (RB qdrv: a 16-cycle X90 every 16 cycles,
// while a thread's tiles are 128 cycles apart) that is every tile.  Here the
// prologue does it once per workgroup:
//   * per strobe, a 32-B record {b, e, env base | cw | amp, phase<<15, F0,
//     rotation-table base}: b = strobe sample, e = end of the samples it
//     plays (b + lim; b when its freq entry is invalid);
//   * per 8-sample group of the chunk, the latest strobe and pulse_reset
//     (u16 + u16), found by one binary search per thread and a forward walk.
// Strobes and resets sit on cycle boundaries (8 | spc), so a group never
// straddles one; it can straddle only a pulse end that is not a multiple of
// 8 samples, handled by the per-sample path.
//
// The sweep then costs per group: the table word, the record, t_ref, one
// carrier, and per sample 6 VALU for the rotation and 5 for the mix:
//   with Y = {lo: ai, hi: aq}, R = {lo: rq, hi: ri}, R' = {lo: ri, hi: -rq}:
//     (a (x) R).re = dot2(R', Y),  .im = dot2(R, Y)
//   and with E = {lo: eq, hi: ei}, E' = {lo: ei, hi: -eq}:
//     (E (x) a).re = dot2(E', a),  .im = dot2(E, a)
// so only Y-form words are ever packed (one v_cvt_pk_i16_i32 + one
// v_pk_max_i16 for symsat).  R' / E' need rq, eq != -32768; a workgroup whose
// tables hold one falls back to the per-sample X/Y path for every group.
// ===========================================================================
struct SegArgs {
    const int16_t *lut;
    const uint4 *rec;               // 2 x uint4 per strobe
    const uint32_t *rs_t;
    const uint32_t *gseg;           // per group: (strobe + 1) | (reset + 1) << 16
    const uint32_t *env;            // ISH == 0: (E, E') pairs; else E
    const uint32_t *fr2;            // per freq entry 16 (R, R') pairs; pair 0 = (F0, 0)
    uint32_t spc_sh, int_sh, c_begin, c_end, ng;
    uint32_t *out;
    bool bad;                       // some eq or rq == -32768: per-sample X/Y path
};

// the definition, sample by sample (X/Y form): straddling groups and bad tables
template <int ISH>
__device__ __forceinline__ void seg_group_slow(const SegArgs &q, uint32_t j0, const uint4 ra, const uint4 rb,
                                            uint32_t t_ref, uint32_t v[8])
{
    const uint32_t n = j0 >> q.spc_sh, k0 = j0 & ((1u << q.spc_sh) - 1u);
    const Carrier a0 = carrier(q.lut, rb.x * (n - t_ref) + ra.w, (int32_t)(ra.z >> 16));
    const uint32_t eb = ra.z & 0x3FFFu;
    const bool cw = (ra.z >> 15) & 1u;
    for (int s = 0; s < 8; s++) {
        const uint32_t j = j0 + s;
        v[s] = 0;
        if (j < ra.y) {
            const uint32_t widx = eb + (cw ? 0u : ((j - ra.x) >> q.int_sh));
            const uint32_t e = ISH == 0 ? q.env[2 * widx] : q.env[widx];
            const uint32_t k = k0 + s;
            v[s] = mix(e, k ? rotate(a0, q.fr2[rb.y + 2 * k]) : a0);
        }
    }
}

template <int ISH>
__device__ __forceinline__ void sweep_seg(const SegArgs &q)
{
    const uint32_t spc_m = (1u << q.spc_sh) - 1u;
    for (uint32_t g = threadIdx.x; g < q.ng; g += BLOCK) {
        const uint32_t j0 = q.c_begin + 8 * g;
        const uint32_t gs = q.gseg[g];
        const int si = (int)(gs & 0xFFFFu) - 1, ri = (int)(gs >> 16) - 1;
        uint32_t v[8];
#pragma unroll
        for (int s = 0; s < 8; s++) v[s] = 0;
        if (si >= 0) {
            const uint4 ra = q.rec[2 * si];
            if (j0 < ra.y) {
                const uint4 rb = q.rec[2 * si + 1];
                const uint32_t t_ref = ri >= 0 ? q.rs_t[ri] : 0u;
                if (j0 + 8 <= ra.y && !q.bad) {
                    const uint32_t n = j0 >> q.spc_sh, k0 = j0 & spc_m;
                    const uint32_t idx = (rb.x * (n - t_ref) + ra.w) >> 20;
                    const int32_t c = q.lut[(idx + 1024) & 4095], sn = q.lut[idx];
                    const int32_t a16 = (int32_t)(ra.z >> 16);
                    const uint32_t y0 = pack16((c * a16 + (1 << 15)) >> 16, (sn * a16 + (1 << 15)) >> 16);
                    // rotation pairs (R_k, R'_k), k = k0 .. k0 + 7
                    const uint4 *rp = reinterpret_cast<const uint4 *>(q.fr2 + rb.y + 2 * k0);
                    uint32_t R[8], Rp[8], E[8], Ep[8];
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        const uint4 w = rp[h];
                        R[2 * h] = w.x; Rp[2 * h] = w.y; R[2 * h + 1] = w.z; Rp[2 * h + 1] = w.w;
                    }
                    const uint32_t eb = ra.z & 0x3FFFu, d0 = j0 - ra.x;
                    if ((ra.z >> 15) & 1u) {                       // CW: env word 4A throughout
                        const uint32_t e = ISH == 0 ? q.env[2 * eb] : q.env[eb];
                        const uint32_t ep = ISH == 0 ? q.env[2 * eb + 1] : neg_swap(e);
#pragma unroll
                        for (int s = 0; s < 8; s++) { E[s] = e; Ep[s] = ep; }
                    } else if (ISH == 0) {                         // 8 (E, E') pairs
                        const uint4 *ep4 = reinterpret_cast<const uint4 *>(q.env + 2 * (eb + d0));
#pragma unroll
                        for (int h = 0; h < 4; h++) {
                            const uint4 w = ep4[h];
                            E[2 * h] = w.x; Ep[2 * h] = w.y; E[2 * h + 1] = w.z; Ep[2 * h + 1] = w.w;
                        }
                    } else if (ISH == 1) {                         // 4 words, 2 samples each
                        const uint4 w = *reinterpret_cast<const uint4 *>(q.env + eb + (d0 >> 1));
                        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                        for (int s = 0; s < 8; s++) { E[s] = ww[s >> 1]; Ep[s] = neg_swap(ww[s >> 1]); }
                    } else if (ISH == 2) {                         // 2 words, 4 samples each
                        const uint2 w = *reinterpret_cast<const uint2 *>(q.env + eb + (d0 >> 2));
                        const uint32_t e0 = w.x, e1 = w.y, p0 = neg_swap(e0), p1 = neg_swap(e1);
#pragma unroll
                        for (int s = 0; s < 8; s++) { E[s] = s < 4 ? e0 : e1; Ep[s] = s < 4 ? p0 : p1; }
                    } else {                                       // one word for all 8
                        const uint32_t e = q.env[eb + (d0 >> q.int_sh)], ep = neg_swap(e);
#pragma unroll
                        for (int s = 0; s < 8; s++) { E[s] = e; Ep[s] = ep; }
                    }
#pragma unroll
                    for (int s = 0; s < 8; s++) {
                        uint32_t y = rot_y(y0, R[s], Rp[s]);
                        if (s == 0) y = k0 == 0 ? y0 : y;         // sub-sample 0 is the unrotated carrier
                        v[s] = mix_y(E[s], Ep[s], y);
                    }
                } else {
                    seg_group_slow<ISH>(q, j0, ra, rb, t_ref, v);
                }
            }
        }
        store4(q.out, j0, q.c_end, v);
        store4(q.out, j0 + 4, q.c_end, v + 4);
    }
}

// strobe i's 32-B segment record (t = strobe cycle, env_w = env word, pf =
// phase | freq index, amp); F0 comes from the staged (R, R') pairs
__device__ __forceinline__ void seg_record(uint4 *rec, const uint32_t *fr2, uint32_t i, uint32_t t, uint32_t env_w,
                                           uint32_t pf, uint32_t amp, uint32_t spc, uint32_t ish, uint32_t env_len,
                                           uint32_t freq_len)
{
    const uint32_t A = env_w & 0xFFFu, L = (env_w >> 12) & 0xFFFu, fi = pf >> 17;
    const uint32_t b = t * spc;
    const uint32_t room = env_len > 4 * A ? env_len - 4 * A : 0u;
    uint32_t lim;
    if (L) {
        const uint32_t n_env = min(4 * L, room);
        lim = n_env << ish;
        if ((lim >> ish) != n_env) lim = 0xFFFFFFFFu;
    } else {
        lim = room ? 0xFFFFFFFFu : 0u;
    }
    const bool act = 16 * fi + 15 < freq_len;
    const uint32_t e = !act ? b : (lim > 0xFFFFFFFFu - b ? 0xFFFFFFFFu : b + lim);
    rec[2 * i] = make_uint4(b, e, (4 * A) | ((L ? 0u : 1u) << 15) | ((amp & 0xFFFFu) << 16), (pf & 0x1FFFFu) << 15);
    rec[2 * i + 1] = make_uint4(act ? fr2[32 * fi] : 0u, 32 * fi, 0u, 0u);
}

// Persistent: gridDim.x workgroups (all resident) each take a contiguous
// range of the (segment channel, sub-chunk) items, channel-major, so a
// workgroup stages the sine table once and compacts a channel's events once
// per channel it visits (2-3 per workgroup at config 5) instead of once per
// chunk; per sub-chunk it only rebuilds the group table.
__global__ void __launch_bounds__(BLOCK) dds_seg_kernel(const DDSParams p)
{
    // dynamic LDS (dds_seg_lds_bytes): sine table | strobe records | strobe
    // times | reset times | group table | env | (R, R') freq pairs
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    int16_t *s_lut = reinterpret_cast<int16_t *>(s_dyn);
    uint4 *s_rec = reinterpret_cast<uint4 *>(s_dyn + 8192);
    uint32_t *s_st_t = reinterpret_cast<uint32_t *>(s_rec + 2 * p.ev_lds);
    uint32_t *s_rs_t = s_st_t + p.ev_lds;
    uint32_t *s_gseg = s_rs_t + p.ev_lds;
    uint32_t *s_env = s_gseg + p.chunk / 8;
    uint32_t *s_fr2 = s_env + p.env_lds;
    __shared__ uint32_t s_tmp[2 * (BLOCK / 64)];
    __shared__ uint32_t s_cnt[2];

    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 4096 / 8; i += BLOCK)
        reinterpret_cast<uint4 *>(s_lut)[i] = reinterpret_cast<const uint4 *>(p.sin_lut)[i];

    const uint32_t n_sub = (p.n_samples + p.chunk - 1) / p.chunk;
    const uint64_t total = (uint64_t)p.n_seg * n_sub;
    const uint64_t per = (total + gridDim.x - 1) / gridDim.x;
    const uint64_t it_end = min((uint64_t)(blockIdx.x + 1) * per, total);
    uint32_t cur = 0xFFFFFFFFu, ch = 0, spc_sh = 0, int_sh = 0, spc_c = 1, env_len_c = 0, freq_len_c = 0;
    int n_st = 0, n_rs = 0;
    bool bad = false;
    if (p.probe == 5) {                     // probe: the sweep's stores alone (zeros)
        for (uint64_t it = (uint64_t)blockIdx.x * per; it < it_end; it++) {
            const uint32_t ci = (uint32_t)(it / n_sub), sub = (uint32_t)(it - (uint64_t)ci * n_sub);
            const uint32_t c_begin = sub * p.chunk, c_end = min(c_begin + p.chunk, p.n_samples);
            uint32_t *out = p.iq + (uint64_t)p.seg_list[ci] * p.n_samples;
            const uint32_t z[4] = {0, 0, 0, 0};
            for (uint32_t j0 = c_begin + 8 * tid; j0 < c_end; j0 += 8 * BLOCK) {
                store4(out, j0, c_end, z);
                store4(out, j0 + 4, c_end, z);
            }
        }
        return;
    }
    for (uint64_t it = (uint64_t)blockIdx.x * per; it < it_end; it++) {
        const uint32_t ci = (uint32_t)(it / n_sub), sub = (uint32_t)(it - (uint64_t)ci * n_sub);
        __syncthreads();                    // the previous sweep is done with the tables
        if (ci != cur) {                    // new channel: stage its tables, compact its events
            cur = ci;
            ch = p.seg_list[ci];
            const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
            const uint32_t lane = d[0], elem = d[1] & 3u, spc = d[2], interp = d[3] ? d[3] : 1u;
            const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
            spc_sh = __ffs(spc) - 1;
            int_sh = __ffs(interp) - 1;
            bad = false;
            if (int_sh == 0) {              // E' beside E
                for (uint32_t i = tid; i < env_len; i += BLOCK) {
                    const uint32_t e = p.env[env_off + i];
                    bad |= (e & 0xFFFFu) == 0x8000u;
                    reinterpret_cast<uint2 *>(s_env)[i] = make_uint2(e, neg_swap(e));
                }
            } else {
                for (uint32_t i = tid; i < env_len; i += BLOCK) {
                    const uint32_t e = p.env[env_off + i];
                    bad |= (e & 0xFFFFu) == 0x8000u;
                    s_env[i] = e;
                }
            }
            for (uint32_t i = tid; i < freq_len; i += BLOCK) {   // R' beside R
                const uint32_t w = p.freq[freq_off + i];
                const bool rot = (i & 15u) != 0;
                bad |= rot && (w & 0xFFFFu) == 0x8000u;
                reinterpret_cast<uint2 *>(s_fr2)[i] = make_uint2(w, rot ? neg_swap(w) : 0u);
            }
            env_len_c = env_len; freq_len_c = freq_len; spc_c = spc;
            if (!p.xs)
                compact_events(
                    p, lane, elem,
                    [&](uint32_t i, const uint4 &ev, uint32_t amp) {
                        s_st_t[i] = ev.x;
                        seg_record(s_rec, s_fr2, i, ev.x, ev.z & 0xFFFFFFu, ev.w, amp, spc, int_sh, env_len, freq_len);
                    },
                    s_rs_t, s_tmp, s_cnt, &n_st, &n_rs);
            bad = __syncthreads_or(bad);    // (index path: also publishes s_fr2 for the records)
        }
        if (p.xs) {                         // indexed: this sub-chunk's window of the channel's events
            const uint4 w = p.win[(uint64_t)ch * n_sub + sub];
            n_st = (int)w.y;
            n_rs = (int)w.w;
            const uint4 *xs = p.xs + (uint64_t)ch * p.ev_lds + w.x;
            const uint32_t *xr = p.xr + (uint64_t)ch * p.ev_lds + w.z;
            for (uint32_t i = tid; i < w.y; i += BLOCK) {
                const uint4 r = xs[i];
                s_st_t[i] = r.x;
                seg_record(s_rec, s_fr2, i, r.x, r.y, r.z, r.w, spc_c, int_sh, env_len_c, freq_len_c);
            }
            for (uint32_t i = tid; i < w.w; i += BLOCK) s_rs_t[i] = xr[i];
            __syncthreads();
        }

        // group table of the sub-chunk: thread tid owns groups [g0, g1)
        const uint32_t c_begin = sub * p.chunk;
        const uint32_t c_end = min(c_begin + p.chunk, p.n_samples);
        const uint32_t ng = (c_end - c_begin + 7) / 8;
        const uint32_t gper = (ng + BLOCK - 1) / BLOCK;
        const uint32_t g0 = min(tid * gper, ng), g1 = min(g0 + gper, ng);
        if (g0 < g1) {
            uint32_t n = (c_begin + 8 * g0) >> spc_sh;
            int si = last_le(s_st_t, n_st, n), ri = last_le(s_rs_t, n_rs, n);
            for (uint32_t g = g0; g < g1; g++) {
                n = (c_begin + 8 * g) >> spc_sh;
                while (si + 1 < n_st && s_st_t[si + 1] <= n) si++;
                while (ri + 1 < n_rs && s_rs_t[ri + 1] <= n) ri++;
                s_gseg[g] = (uint32_t)(si + 1) | ((uint32_t)(ri + 1) << 16);
            }
        }
        __syncthreads();

        const SegArgs q{s_lut, s_rec, s_rs_t, s_gseg, s_env, s_fr2, spc_sh, int_sh, c_begin, c_end, ng,
                        p.iq + (uint64_t)ch * p.n_samples, bad};
        if (p.probe == 6 || p.probe == 7) {  // probes: tables built; stores of zeros / of the group words
            for (uint32_t g = tid; g < ng; g += BLOCK) {
                const uint32_t j0 = c_begin + 8 * g;
                const uint32_t w = p.probe == 7 ? s_gseg[g] : 0u;
                const uint32_t z[4] = {w, w, w, w};
                store4(q.out, j0, c_end, z);
                store4(q.out, j0 + 4, c_end, z);
            }
            continue;
        }
        switch (int_sh) {
        case 0: sweep_seg<0>(q); break;
        case 1: sweep_seg<1>(q); break;
        case 2: sweep_seg<2>(q); break;
        default: sweep_seg<3>(q); break;
        }
    }
}

// dynamic LDS above 64 KiB needs an opt-in per kernel, raised as requests grow
static hipError_t opt_in_lds(const void *fn, uint32_t bytes, uint32_t *granted)
{
    if (bytes <= 64 * 1024 || bytes <= *granted) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) *granted = bytes;
    return e;
}

hipError_t launch_dds_index(const DDSParams &p, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples || !p.xs) return hipSuccess;
    const uint32_t ilds = (BLOCK / 64) * 2 * p.ev_lds * 4;   // per wave: strobe and reset times
    static uint32_t granted = 0;
    const hipError_t e = opt_in_lds(reinterpret_cast<const void *>(dds_index_kernel), ilds, &granted);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dds_index_kernel, dim3((p.n_channels + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), ilds,
                       stream, p);
    return hipGetLastError();
}

hipError_t launch_dds(const DDSParams &p, const DDSParams &ps, bool any_seg, bool any_chunk, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples) return hipSuccess;
    if (any_seg && ps.n_seg) {
        const uint32_t lds = dds_seg_lds_bytes(ps.ev_lds, ps.env_lds, ps.freq_lds, ps.chunk) + ps.lds_pad;
        static uint32_t granted = 0;
        hipError_t e = opt_in_lds(reinterpret_cast<const void *>(dds_seg_kernel), lds, &granted);
        if (e != hipSuccess) return e;
        // one resident wave of workgroups: CUs x workgroups per CU (occupancy,
        // or ps.grid_per_cu when set), never more than there are items
        int dev = 0, cus = 0, per_cu = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dds_seg_kernel, BLOCK, lds)) != hipSuccess)
            return e;
        if (ps.grid_per_cu) per_cu = std::min<int>(per_cu, (int)ps.grid_per_cu);
        const uint64_t items = (uint64_t)ps.n_seg * ((ps.n_samples + ps.chunk - 1) / ps.chunk);
        // indexed: one item per workgroup (no per-channel compaction to amortise)
        const uint32_t grid = ps.xs ? (uint32_t)items
                                    : (uint32_t)std::min<uint64_t>(items, (uint64_t)std::max(1, cus * std::max(1, per_cu)));
        hipLaunchKernelGGL(dds_seg_kernel, dim3(grid), dim3(BLOCK), lds, stream, ps);
    }
    if (any_chunk) {
        const uint32_t chunks = (p.n_samples + p.chunk - 1) / p.chunk;
        const bool lean = p.xs && p.yform && !p.rows && (!p.probe || p.probe == 13);
        // lean SPT-8 kernel: + the cycle table (chunk / 8 u32 entries, 8 per thread)
        const uint32_t lds = dds_lds_bytes(p.ev_lds, p.env_lds, p.freq_lds) + p.lds_pad - (lean ? 4096u : 0u) +
                             (lean && p.spt != 4 && p.cyc ? 32 * BLOCK : 0u);
        const void *fn = !lean ? reinterpret_cast<const void *>(dds_chunk_kernel<0>)
                         : p.spt == 4 ? reinterpret_cast<const void *>(dds_chunk_kernel<4>)
                                      : reinterpret_cast<const void *>(dds_chunk_kernel<8>);
        static uint32_t granted[3] = {0, 0, 0};
        const hipError_t e = opt_in_lds(fn, lds, &granted[!lean ? 0 : p.spt == 4 ? 1 : 2]);
        if (e != hipSuccess) return e;
        if (!lean) hipLaunchKernelGGL(dds_chunk_kernel<0>, dim3(chunks, p.n_channels), dim3(BLOCK), lds, stream, p);
        else if (p.spt == 4) hipLaunchKernelGGL(dds_chunk_kernel<4>, dim3(chunks, p.n_channels), dim3(BLOCK), lds, stream, p);
        else hipLaunchKernelGGL(dds_chunk_kernel<8>, dim3(chunks, p.n_channels), dim3(BLOCK), lds, stream, p);
    }
    return hipGetLastError();
}

}  // namespace dpemu
