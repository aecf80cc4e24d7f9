// dds.hip -- fixed-point DDS I/Q synthesis from emulated pulse events (gfx950).
//
// Spec: DESIGN.md §4.5 and oracle/dds_ref.c (CPU restatement, bit-exact).
// Inputs are the interpreter's outputs in HBM (lane summaries + slot-major
// 16-B event records) and the assembler's env / freq buffers
// (asmparse.py:46-86 formats).  HBM-write-bound by design: 4 B per output
// sample, nothing else leaves the chip.
//
// Two launches per synthesis:
//   * dds_index_kernel (one workgroup per channel, or per two channels of one
//     lane) compacts the lane's strobes of the channel's element and its
//     pulse_resets (time-sorted: a core emits them in time order) once,
//     channel-contiguous, and writes the channel's two counts;
//   * dds_tile_kernel, grid (stripes, channels).  A channel's 1,024-sample
//     tiles go round-robin to its stripe workgroups, so at any time the
//     stripes of a channel write ADJACENT tiles.  A workgroup stages the
//     quarter-wave sine table, the channel's env / freq tables -- as
//     (E, E') / (R, R') pairs for the Y-form products, the env pairs in
//     bank-swizzled chunks -- and the channel's records (up to rec_lds; a
//     denser channel is read from the global index) in LDS, finds each of its
//     tiles' window of records (the ones the tile's samples can see), then
//     sweeps with no global loads in the loop (on gfx950 stores count in
//     vmcnt, so a load there would wait for the previous tile's stores).
//     At 16 samples per clock (the RFSoC rate) a lane makes one whole cycle
//     per tile -- window search, record decode, theta and carrier once per
//     16 samples -- and the wave's 4 KiB goes out through a 1-KiB LDS
//     transpose as 1-KiB dense store instructions; at other rates a lane
//     makes 4 consecutive samples (one 16-B store).
// Channels whose sample rate or tables do not fit the quad sweep take the
// generic per-sample sweep (the definition, sample by sample).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.h"

namespace dpemu {


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

// the Q15 table is built from its first quadrant with exact symmetry
// (dpemu_dds_sin_lut): sin[2048 - i] = sin[i], sin[i + 2048] = -sin[i], so
// the tile kernel stages the quarter wave, entries 0..1024 (2 KiB of LDS)
__device__ __forceinline__ int32_t lut_quarter(const int16_t *lut, uint32_t i)
{
    const uint32_t r = i & 1023u;
    const int32_t v = lut[(i & 1024u) ? 1024u - r : r];
    return (i & 2048u) ? -v : v;
}

__device__ __forceinline__ Carrier carrier_quarter(const int16_t *lut, uint32_t theta, int32_t amp)
{
    const uint32_t idx = theta >> 20;
    return carrier_cs(lut_quarter(lut, (idx + 1024) & 4095), lut_quarter(lut, idx), amp);
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
// I/Q stores nontemporal (A/B builds only)
#ifndef DPEMU_DDS_NT
#define DPEMU_DDS_NT 0
#endif

__device__ __forceinline__ void store4(uint32_t *out, uint32_t j0, uint32_t c_end, const uint32_t v[4])
{
    if (j0 + 3 < c_end) {
        const u32x4 w = {v[0], v[1], v[2], v[3]};
#if DPEMU_DDS_NT
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(out + j0));
#else
        *reinterpret_cast<u32x4 *>(out + j0) = w;
#endif
    } else {
        for (int s = 0; s < 4 && j0 + s < c_end; s++) out[j0 + s] = v[s];
    }
}

// The interp-1 envelope is staged as (E, E') pairs, two pairs per 16-B chunk,
// chunk c at physical chunk c ^ ((c >> 4) & 7).  The cycle sweep's lanes read
// chunks 8 apart (16 samples = 8 chunks per cycle); unswizzled, the 16 lanes
// of a ds_read_b128 pass would hit 2 bank groups (8-way conflicts), swizzled
// they hit all 16 -- for any pulse start A.
__device__ __forceinline__ uint32_t env_chunk(uint32_t c) { return c ^ ((c >> 4) & 7u); }
// word index of pair q's E in that layout (E' at + 1)
__device__ __forceinline__ uint32_t env_pair(uint32_t q) { return (env_chunk(q >> 1) << 2) | ((q & 1u) << 1); }

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
// Event index: one workgroup per channel.  Event chunk q (64 events) goes to
// wave q % 4 (chunks 4 k + w are wave w's k-th), so every wave loads from the
// first chunk on and the loads of short lists spread over the waves; all
// loaded up front.  The 16 chunks' strobe / reset counts are scanned in LDS,
// each wave writes its records at their offsets in event order, and the
// channel's two counts go out; the tile workgroups find their tiles' windows
// in the records they stage.  (Round 4 wrote every tile's window here, 4.5 us
// of the kernel's 14.8; one wave per channel with per-lane tile cursors
// measured 1 % slower per step.)
// ===========================================================================
__global__ void __launch_bounds__(BLOCK) dds_index_kernel(const DDSParams p)
{
    constexpr int W = BLOCK / 64;
    constexpr int K = DDS_MAX_EVENTS / BLOCK;           // event chunks per wave
    __shared__ uint32_t s_cnt[3][K * W + 1];            // strobes of channel 0 / 1, resets
    const uint32_t tid = threadIdx.x, wl = tid & 63u, wv = tid >> 6;
    // the workgroup's channels: ch0 and, when p.pair_lanes, ch0 + 1 (same lane)
    const uint32_t G = p.pair_lanes ? 2u : 1u;
    const uint32_t ch0 = blockIdx.x * G;
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch0;
    const uint32_t lane = d[0], elem0 = d[1] & 3u, elem1 = G == 2u ? d[DDS_CH_WORDS + 1] & 3u : 0xFFu;
    const uint32_t n_ev = min(p.summary[8ull * lane + 2], p.event_cap);
    const uint64_t below = wl ? (~0ull >> (64 - wl)) : 0ull;
    uint4 ev[K];
    bool is_s0[K], is_s1[K], is_rs[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t e = (k * W + wv) * 64u + wl;
        ev[k] = e < n_ev ? p.events[(uint64_t)e * p.n_lanes + lane] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t e = (k * W + wv) * 64u + wl;
        const uint32_t kind = ev[k].y >> 28, el = (ev[k].y >> 24) & 3u;
        is_s0[k] = e < n_ev && kind == 0u && el == elem0;
        is_s1[k] = e < n_ev && kind == 0u && el == elem1;
        is_rs[k] = e < n_ev && kind == 1u;
        const uint32_t n0 = (uint32_t)__popcll(__ballot(is_s0[k])), n1 = (uint32_t)__popcll(__ballot(is_s1[k]));
        const uint32_t nr = (uint32_t)__popcll(__ballot(is_rs[k]));
        if (wl == 0) { s_cnt[0][k * W + wv] = n0; s_cnt[1][k * W + wv] = n1; s_cnt[2][k * W + wv] = nr; }
    }
    __syncthreads();
    if (tid < 3) {                                      // exclusive scans of the chunk counts (+ totals)
        uint32_t acc = 0;
        for (int q = 0; q < K * W; q++) { const uint32_t c = s_cnt[tid][q]; s_cnt[tid][q] = acc; acc += c; }
        s_cnt[tid][K * W] = acc;
    }
    __syncthreads();
    uint4 *xs0 = p.xs + (uint64_t)ch0 * p.ev_lds, *xs1 = xs0 + p.ev_lds;
    uint32_t *xr0 = p.xr + (uint64_t)ch0 * p.ev_lds, *xr1 = xr0 + p.ev_lds;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t q = k * W + wv;                  // records in the chunks before: s_cnt[.][q]
        const uint64_t b0 = __ballot(is_s0[k]), b1 = __ballot(is_s1[k]), br = __ballot(is_rs[k]);
        const uint4 rec = make_uint4(ev[k].x, ev[k].y & 0xFFFFFFu, ev[k].z, ev[k].w & 0xFFFFu);
        if (is_s0[k]) xs0[s_cnt[0][q] + (uint32_t)__popcll(b0 & below)] = rec;
        if (is_s1[k]) xs1[s_cnt[1][q] + (uint32_t)__popcll(b1 & below)] = rec;
        if (is_rs[k]) {
            const uint32_t i = s_cnt[2][q] + (uint32_t)__popcll(br & below);
            xr0[i] = ev[k].x;
            if (G == 2u) xr1[i] = ev[k].x;
        }
    }
    if (tid == 0) p.cnt[ch0] = make_uint2(s_cnt[0][K * W], s_cnt[2][K * W]);
    if (tid == 0 && G == 2u) p.cnt[ch0 + 1] = make_uint2(s_cnt[1][K * W], s_cnt[2][K * W]);
}

// the latest strobe record with t <= x among rec[0, n) (time-sorted), or -1
__device__ __forceinline__ int last_le_rec(const uint4 *rec, int n, uint32_t x)
{
    int lo = 0, hi = n;                 // first index with t > x
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rec[mid].x <= x) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}

// a tile's window from its raw search results {a0, a1, b0, b1} (a0 / b0:
// strobes / resets at or before the tile's first cycle, a1 / b1: at or
// before its last): from the latest record at or before the first cycle
// (the first record when none is) to the latest at or before the last
__device__ __forceinline__ uint4 tile_window(uint4 raw)
{
    const uint32_t sl = raw.x ? raw.x - 1u : 0u, rl = raw.z ? raw.z - 1u : 0u;
    return make_uint4(sl, raw.y - sl, rl, raw.w - rl);
}

// the latest record at or before cycle n inside a window {lo, count} of a
// staged time array (base = the staged array's first index), or -1
__device__ __forceinline__ int window_find(const uint32_t *t, uint32_t lo, uint32_t count, uint32_t base, uint32_t n)
{
    const int r = last_le(t + (lo - base), (int)count, n);
    return r < 0 ? -1 : (int)(lo - base) + r;
}

// the same over staged strobe records {t, ...} (windows hold 1-3 records)
__device__ __forceinline__ int window_find_rec(const uint4 *rec, uint32_t lo, uint32_t count, uint32_t base,
                                               uint32_t n)
{
    int a = 0, b = (int)count;                       // first index with t > n
    const uint4 *r = rec + (lo - base);
    while (a < b) {
        const int mid = (a + b) >> 1;
        if (r[mid].x <= n) a = mid + 1; else b = mid;
    }
    return a == 0 ? -1 : (int)(lo - base) + a - 1;
}

// The tiles a workgroup sweeps: grid (stripes, channels), stripe s of channel
// ch takes the channel's tiles s, s + stripes, ... (local tile i is tile
// c_first + i step, whose first sample is tile * DDS_TILE)
struct TileMap {
    uint32_t ch, c_first, step, n_t;
    __device__ __forceinline__ uint32_t tile(uint32_t i) const { return c_first + i * step; }
    __device__ __forceinline__ uint32_t first(uint32_t i) const { return tile(i) * DDS_TILE; }
};

__device__ __forceinline__ TileMap tile_map(const DDSParams &p)
{
    TileMap m;
    m.ch = blockIdx.y;
    m.c_first = blockIdx.x;
    m.step = gridDim.x;
    m.n_t = (p.tiles - blockIdx.x + gridDim.x - 1) / gridDim.x;
    return m;
}

// the LDS-resident part of a tile workgroup
struct TileLds {
    const int16_t *lut;
    const uint4 *win;
    const uint32_t *env, *freq;
    uint4 *xpose;
};

// The sweep over a stripe's n_t tiles.  st / rs_t: the strobe records and
// reset times, staged in LDS (base = the first staged index) or the global
// index (base 0); inlined at both call sites so each keeps its address space.
__device__ __forceinline__ void tile_sweep(const DDSParams &p, const TileLds &L, const uint32_t *d, const TileMap &M,
                                           bool quad, const uint4 *st, uint32_t st_lo, const uint32_t *rs_t,
                                           uint32_t rs_lo)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t ch = M.ch, n_t = M.n_t;
    const uint32_t spc = d[2], interp = d[3] ? d[3] : 1u;
    const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
    const bool spc_p2 = (spc & (spc - 1)) == 0, int_p2 = (interp & (interp - 1)) == 0;
    const uint32_t spc_sh = __ffs(spc) - 1, int_sh = __ffs(interp) - 1;
    const int16_t *s_lut = L.lut;
    const uint32_t *s_env = L.env, *s_freq = L.freq;
    uint32_t *out = p.iq + (uint64_t)ch * p.n_samples;
    if (quad && spc == 16u) {
        // ---- cycle sweep (16 samples / clk, the RFSoC rate): a lane makes one
        // whole cycle, so the window search, record decode, theta and carrier
        // are done once per 16 samples; wave w takes the stripe's tiles w, w + 4, ...
        const uint32_t wv = tid >> 6, ln = tid & 63u;
        for (uint32_t i = wv; i < n_t; i += BLOCK / 64) {
            const uint32_t tb = M.first(i);                                 // the tile's first sample (16 | tb)
            const uint32_t js = tb + 16 * ln;                               // this lane's cycle n = js / 16
            const uint32_t n = js >> 4;
            const uint4 w = tile_window(L.win[i]);
            uint32_t v[16];
#pragma unroll
            for (int q = 0; q < 16; q++) v[q] = 0u;
            const int si = js < p.n_samples ? window_find_rec(st, w.x, w.y, st_lo, n) : -1;
            if (si >= 0) {
                const uint4 rec = st[si];                            // {t, env word, phase | freq << 17, amp}
                const uint32_t A = rec.y & 0xFFFu, Lw = (rec.y >> 12) & 0xFFFu, fi = rec.z >> 17;
                const uint32_t room = env_len > 4 * A ? env_len - 4 * A : 0u;
                uint32_t lim, emask;
                if (Lw) {
                    emask = 0xFFFFFFFFu;
                    const uint32_t n_env = min(4 * Lw, room);
                    lim = n_env << int_sh;
                    if ((lim >> int_sh) != n_env) lim = 0xFFFFFFFFu;
                } else {
                    emask = 0u;
                    lim = room ? 0xFFFFFFFFu : 0u;
                }
                const uint32_t d0 = 16 * (n - rec.x);                // samples since the strobe's first
                if (16 * fi + 15 < freq_len && d0 < lim) {
                    const int ri = window_find(rs_t, w.z, w.w, rs_lo, n);
                    const uint32_t t_ref = ri >= 0 ? rs_t[ri] : 0u;
                    const uint32_t *frp = s_freq + 32 * fi;          // (R, R') pairs; pair 0 = (F0, 0)
                    const uint32_t idx = (frp[0] * (n - t_ref) + ((rec.z & 0x1FFFFu) << 15)) >> 20;
                    const int32_t c = lut_quarter(s_lut, (idx + 1024) & 4095), sn = lut_quarter(s_lut, idx);
                    const int32_t a16 = (int32_t)(rec.w & 0xFFFFu);
                    const uint32_t y0 = pack16((c * a16 + (1 << 15)) >> 16, (sn * a16 + (1 << 15)) >> 16);
                    const bool inside = d0 + 15 < lim && emask;
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        uint32_t R[4], Rp[4], E[4], Ep[4];
#pragma unroll
                        for (int h = 0; h < 2; h++) {
                            const uint4 rw = *reinterpret_cast<const uint4 *>(frp + 8 * g + 4 * h);
                            R[2 * h] = rw.x; Rp[2 * h] = rw.y; R[2 * h + 1] = rw.z; Rp[2 * h + 1] = rw.w;
                        }
                        if (interp == 1) {
                            if (inside) {
#pragma unroll
                                for (int h = 0; h < 2; h++) {
                                    const uint4 ew = *reinterpret_cast<const uint4 *>(
                                        s_env + 4 * env_chunk(2 * A + (d0 >> 1) + 2 * g + h));
                                    E[2 * h] = ew.x; Ep[2 * h] = ew.y; E[2 * h + 1] = ew.z; Ep[2 * h + 1] = ew.w;
                                }
                            } else {
#pragma unroll
                                for (int s2 = 0; s2 < 4; s2++) {
                                    const uint32_t dd = d0 + 4 * g + s2;
                                    const uint32_t wi = env_pair(4 * A + (dd & emask));
                                    E[s2] = dd < lim ? s_env[wi] : 0u;
                                    Ep[s2] = dd < lim ? s_env[wi + 1] : 0u;
                                }
                            }
                        } else {                                     // interp >= 4: one env word for 4 samples
                            const uint32_t e = d0 + 4 * g < lim ? s_env[4 * A + (((d0 + 4 * g) >> int_sh) & emask)] : 0u;
                            const uint32_t ep = neg_swap(e);
#pragma unroll
                            for (int s2 = 0; s2 < 4; s2++) { E[s2] = e; Ep[s2] = ep; }
                        }
#pragma unroll
                        for (int s2 = 0; s2 < 4; s2++) {
                            const uint32_t y = (g == 0 && s2 == 0) ? y0 : rot_y(y0, R[s2], Rp[s2]);
                            // E = E' = 0 past the pulse end makes the mix 0 (interp 1: the
                            // loads above; interp >= 4: 4-sample groups lie wholly in or out)
                            v[4 * g + s2] = mix_y(E[s2], Ep[s2], y);
                        }
                    }
                }
            }
            // transpose through the wave's 1-KiB LDS slice so every store
            // instruction writes 1 KiB dense (lane-per-cycle stores would be 64 B
            // apart): round r, lanes 16 r .. 16 r + 15 put their 4 chunks
            // (lane l's chunk q at slot 4 (l & 15) + (q ^ (l >> 2 & 3)):
            // conflict-free both ways), every lane takes one chunk and stores
            uint4 *xp = L.xpose + 64 * wv;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if ((ln >> 4) == (uint32_t)r) {
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        xp[4 * (ln & 15u) + (q ^ ((ln >> 2) & 3u))] =
                            make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t lc = ln >> 2;                            // source lane 16 r + lc
                const uint4 x = xp[4 * lc + ((ln & 3u) ^ ((lc >> 2) & 3u))];
                const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
                store4(out, tb + 4 * (64u * r + ln), p.n_samples, w4);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the next writes
                __builtin_amdgcn_wave_barrier();
            }
        }
        return;
    }
    const uint32_t k0 = (4 * tid) & (spc - 1);     // sub-sample slot: fixed (tiles start at multiples of 16)
    for (uint32_t i = 0; i < n_t; i++) {
        const uint32_t j0 = M.first(i) + 4 * tid;
        if (j0 >= p.n_samples) continue;
        const uint4 w = tile_window(L.win[i]);
        uint32_t v[4] = {0u, 0u, 0u, 0u};
        if (quad) {
            const uint32_t n = j0 >> spc_sh;                         // the thread's 4 samples share cycle n
            const int si = window_find_rec(st, w.x, w.y, st_lo, n);
            if (si >= 0) {
                const uint4 rec = st[si];                            // {t, env word, phase | freq << 17, amp}
                const uint32_t A = rec.y & 0xFFFu, Lw = (rec.y >> 12) & 0xFFFu, fi = rec.z >> 17;
                const uint32_t base = rec.x << spc_sh;               // sample index of the strobe
                // samples dd = j - base with env index (dd >> int_sh) & emask inside
                // the pulse and the table: dd < lim
                const uint32_t room = env_len > 4 * A ? env_len - 4 * A : 0u;
                uint32_t lim, emask;
                if (Lw) {
                    emask = 0xFFFFFFFFu;
                    const uint32_t n_env = min(4 * Lw, room);
                    lim = n_env << int_sh;
                    if ((lim >> int_sh) != n_env) lim = 0xFFFFFFFFu;   // no overflow past 2^32
                } else {
                    emask = 0u;                                      // CW: env word 4A forever
                    lim = room ? 0xFFFFFFFFu : 0u;
                }
                const uint32_t d0 = j0 - base;
                if (16 * fi + 15 < freq_len && d0 < lim) {           // (a finished pulse plays zeros)
                    const int ri = window_find(rs_t, w.z, w.w, rs_lo, n);
                    const uint32_t t_ref = ri >= 0 ? rs_t[ri] : 0u;
                    const uint32_t *frp = s_freq + 32 * fi;          // (R, R') pairs; pair 0 = (F0, 0)
                    const uint32_t idx = (frp[0] * (n - t_ref) + ((rec.z & 0x1FFFFu) << 15)) >> 20;
                    const int32_t c = lut_quarter(s_lut, (idx + 1024) & 4095), sn = lut_quarter(s_lut, idx);
                    const int32_t a16 = (int32_t)(rec.w & 0xFFFFu);
                    const uint32_t y0 = pack16((c * a16 + (1 << 15)) >> 16, (sn * a16 + (1 << 15)) >> 16);
                    uint32_t R[4], Rp[4], E[4], Ep[4];
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint4 rw = *reinterpret_cast<const uint4 *>(frp + 2 * k0 + 4 * h);
                        R[2 * h] = rw.x; Rp[2 * h] = rw.y; R[2 * h + 1] = rw.z; Rp[2 * h + 1] = rw.w;
                    }
                    const bool inside = d0 + 3 < lim;
                    if (interp == 1) {
                        // (E, E') pairs, swizzled chunks (env_pair); pair 4A + dd
                        if (inside && emask) {
#pragma unroll
                            for (int h = 0; h < 2; h++) {
                                const uint4 ew = *reinterpret_cast<const uint4 *>(
                                    s_env + 4 * env_chunk(2 * A + (d0 >> 1) + h));
                                E[2 * h] = ew.x; Ep[2 * h] = ew.y; E[2 * h + 1] = ew.z; Ep[2 * h + 1] = ew.w;
                            }
                        } else {
#pragma unroll
                            for (int s = 0; s < 4; s++) {
                                const uint32_t wi = env_pair(4 * A + ((d0 + s) & emask));
                                E[s] = d0 + s < lim ? s_env[wi] : 0u;
                                Ep[s] = d0 + s < lim ? s_env[wi + 1] : 0u;
                            }
                        }
                    } else {                                         // interp >= 4: one env word for the 4
                        const uint32_t e = s_env[4 * A + ((d0 >> int_sh) & emask)], ep = neg_swap(e);
#pragma unroll
                        for (int s = 0; s < 4; s++) { E[s] = e; Ep[s] = ep; }
                    }
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        uint32_t y = rot_y(y0, R[s], Rp[s]);
                        if (s == 0 && k0 == 0) y = y0;               // sub-sample 0 is the unrotated carrier
                        v[s] = d0 + s < lim ? mix_y(E[s], Ep[s], y) : 0u;
                    }
                }
            }
        } else {
            // ---- generic sweep: the per-sample definition (oracle/dds_ref.c) ----
#pragma unroll 1
            for (int s = 0; s < 4; s++) {
                const uint32_t j = j0 + s;
                if (j >= p.n_samples) break;
                const uint32_t n = spc_p2 ? (j >> spc_sh) : j / spc, k = j - n * spc;
                const int si = window_find_rec(st, w.x, w.y, st_lo, n);
                if (si < 0) continue;
                const uint4 rec = st[si];
                const uint32_t A = rec.y & 0xFFFu, Lw = (rec.y >> 12) & 0xFFFu;
                const uint32_t r = j - rec.x * spc;
                const uint32_t es = Lw ? (int_p2 ? (r >> int_sh) : r / interp) : 0u;
                const uint32_t widx = 4 * A + es;
                const uint32_t fi = rec.z >> 17, phase = rec.z & 0x1FFFFu;
                if ((!Lw || es < 4 * Lw) && widx < env_len && 16 * fi + 15 < freq_len) {
                    const int ri = window_find(rs_t, w.z, w.w, rs_lo, n);
                    const uint32_t *fr = p.freq + freq_off + 16 * fi;
                    const uint32_t t_ref = ri >= 0 ? rs_t[ri] : 0u;
                    const Carrier a0 = carrier_quarter(s_lut, fr[0] * (n - t_ref) + (phase << 15), (int32_t)(rec.w & 0xFFFFu));
                    v[s] = mix(p.env[env_off + widx], k ? rotate(a0, fr[k]) : a0);
                }
            }
        }
        store4(out, j0, p.n_samples, v);
    }
}

// ===========================================================================
// Tile sweep.  Workgroup (stripe, ch) synthesises its stripe of channel ch
// (stripe_tile).  Per tile a thread finds its pulse in the tile's window
// (binary search over a few LDS entries), decodes it and makes its samples:
//   Y-form quad / cycle sweep (spc a power of two >= 4, interp 1 or >= 4 and
//   a power of two, tables staged, no -32768 in the staged eq / rq): a =
//   symsat(a0 (x) R_k) as 2 v_dot2_i32_i16 + v_cvt_pk_i16_i32 + v_pk_max_i16,
//   the mix sat16(E (x) a) as 2 v_dot2_i32_i16 + v_cvt_pk_i16_i32;
//   else the generic per-sample sweep (X/Y form, tables read where they lie).
// ===========================================================================
// waves per SIMD the register allocation targets: 7 (69 VGPRs, spill-free);
// forcing 8 (64 VGPRs) spills 10 VGPRs and measured 15 % slower
// (profiles/r04_dds_variants_ab.json)
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(7))) dds_tile_kernel(const DDSParams p)
{
    // dynamic LDS (dds_lds_bytes): quarter sine table | strobe records |
    // reset times | tile windows | env | freq | store transpose
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    int16_t *s_lut = reinterpret_cast<int16_t *>(s_dyn);
    uint4 *s_st = reinterpret_cast<uint4 *>(s_dyn + DDS_LUT_BYTES);
    uint32_t *s_rs_t = reinterpret_cast<uint32_t *>(s_st + p.rec_lds);
    uint4 *s_win = reinterpret_cast<uint4 *>(s_rs_t + p.rec_lds);
    uint32_t *s_env = reinterpret_cast<uint32_t *>(s_win + p.wg_tiles);
    uint32_t *s_freq = s_env + p.env_lds;
    uint4 *s_xpose = reinterpret_cast<uint4 *>(s_freq + p.freq_lds);   // DDS_XPOSE_BYTES, 16-B aligned

    const uint32_t tid = threadIdx.x;
    const TileMap M = tile_map(p);
    if (M.n_t == 0) return;                          // (workgroup-uniform)
    const uint32_t ch = M.ch, n_t = M.n_t;
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
    const uint32_t spc = d[2], interp = d[3] ? d[3] : 1u;
    const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
    const bool spc_p2 = (spc & (spc - 1)) == 0, int_p2 = (interp & (interp - 1)) == 0;
    const bool staged = (interp == 1 ? dds_env_pairs_words(env_len) : env_len) <= p.env_lds && 2 * freq_len <= p.freq_lds;
    // the channel's strobes / resets (a stripe's tiles span the channel)
    const uint2 cnt = p.cnt[ch];
    const uint32_t st_n = cnt.x, rs_n = cnt.y;
    const bool fits = st_n <= p.rec_lds && rs_n <= p.rec_lds;    // workgroup-uniform

    // prologue: every global load of the workgroup up front
    if (tid < DDS_LUT_BYTES / 16)                                      // entries 0..1031 (1024 needed)
        reinterpret_cast<uint4 *>(s_lut)[tid] = reinterpret_cast<const uint4 *>(p.sin_lut)[tid];
    bool bad = false;                       // a staged eq or rq is -32768: no Y form
    if (staged) {
        if (interp == 1) {
            for (uint32_t i = tid; i < env_len; i += BLOCK) {
                const uint32_t e = p.env[env_off + i];
                bad |= (e & 0xFFFFu) == 0x8000u;
                *reinterpret_cast<uint2 *>(s_env + env_pair(i)) = make_uint2(e, neg_swap(e));
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
    }
    const uint4 *xs = p.xs + (uint64_t)ch * p.ev_lds;
    const uint32_t *xr = p.xr + (uint64_t)ch * p.ev_lds;
    if (fits) {
        for (uint32_t i = tid; i < st_n; i += BLOCK) s_st[i] = xs[i];
        for (uint32_t i = tid; i < rs_n; i += BLOCK) s_rs_t[i] = xr[i];
    }
    bad = __syncthreads_or(bad);
    // the tiles' windows: 4 searches per tile, one per thread (raw counts,
    // tile_window in the sweep)
    const uint32_t spc_sh = __ffs(spc) - 1;
    for (uint32_t q = tid; q < 4 * n_t; q += BLOCK) {
        const uint32_t j0 = M.first(q >> 2), j1 = min(j0 + DDS_TILE, p.n_samples) - 1, j = (q & 1u) ? j1 : j0;
        const uint32_t n = spc_p2 ? j >> spc_sh : j / spc;
        int r;
        if (q & 2u) r = fits ? last_le(s_rs_t, (int)rs_n, n) : last_le(xr, (int)rs_n, n);
        else r = fits ? last_le_rec(s_st, (int)st_n, n) : last_le_rec(xs, (int)st_n, n);
        reinterpret_cast<uint32_t *>(s_win)[q] = (uint32_t)(r + 1);
    }
    __syncthreads();

    const bool quad = staged && !bad && (spc & 3u) == 0 && spc_p2 && int_p2 && (interp == 1 || interp >= 4);
    const TileLds L{s_lut, s_win, s_env, s_freq, s_xpose};
    if (fits)
        tile_sweep(p, L, d, M, quad, s_st, 0u, s_rs_t, 0u);
    else
        tile_sweep(p, L, d, M, quad, xs, 0u, xr, 0u);
}

hipError_t launch_dds_index(const DDSParams &p, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples) return hipSuccess;
    // a workgroup per channel, or per pair of channels on one lane (pair_lanes)
    hipLaunchKernelGGL(dds_index_kernel, dim3(p.pair_lanes ? p.n_channels / 2 : p.n_channels), dim3(BLOCK), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_dds(const DDSParams &p, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples) return hipSuccess;
    const uint32_t lds = dds_lds_bytes(p.rec_lds, p.wg_tiles, p.env_lds, p.freq_lds);
    const hipError_t e = opt_in_dynamic_lds(reinterpret_cast<const void *>(dds_tile_kernel), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dds_tile_kernel, dim3(p.stripes, p.n_channels), dim3(BLOCK), lds, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
