// dds.hip -- fixed-point DDS I/Q synthesis from emulated pulse events (gfx950).
//
// Spec: DESIGN.md §4.7 and oracle/dds_ref.c (CPU restatement, bit-exact).
// Inputs are the interpreter's outputs in HBM (lane summaries + slot-major
// 16-B event records) and the assembler's env / freq buffers
// (asmparse.py:46-86 formats).  HBM-write-bound by design: 4 B per output
// sample, nothing else leaves the chip.
//
// ONE launch per synthesis: dds_synth_kernel, one workgroup per (channel,
// segment of seg_tiles 1,024-sample tiles).  A workgroup
//   * stages the quarter-wave sine table and the channel's env / freq tables
//     in LDS -- as (E, E') / (R, R') pairs for the Y-form products, the env
//     pairs in bank-swizzled chunks;
//   * scans the lane's event records once (4 per thread, ballot / popc
//     compaction) and stages the element's strobes and the pulse_resets its
//     segment can see: from the latest one at or before the segment's first
//     cycle, up to `rec` of each (a denser segment is swept in several passes,
//     each restaging from its first tile);
//   * sweeps its tiles with no global load in the loop (on gfx950 stores
//     count in vmcnt, so a load there would wait for the previous tile's
//     stores).  Wave w takes tiles w, w + 4, ..., so the workgroup writes 4
//     adjacent 4-KiB tiles at a time; a wave finds a tile's window of records
//     with a ballot over the staged times from its own cursor (tiles come in
//     increasing order).  At 16 samples per clock (the RFSoC rate) a lane
//     makes one whole cycle -- record lookup, theta and carrier once per 16
//     samples -- and the wave's 4 KiB goes out through a 1-KiB LDS transpose
//     as 1-KiB dense store instructions; at other rates a lane makes 4
//     consecutive samples per round (one 16-B store), 4 rounds per tile.
// Round 4's design (a per-channel index kernel writing every tile's window to
// HBM, then 13 stripe workgroups per channel each re-staging it) took two
// launches and ~50 MB of index traffic per config-5 step.
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

// the Q15 table is built from its first quadrant with exact symmetry
// (dpemu_dds_sin_lut): sin[2048 - i] = sin[i], sin[i + 2048] = -sin[i], so
// the kernel stages the quarter wave, entries 0..1024 (2 KiB of LDS)
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

// The interp-1 envelope is staged as (E, E') pairs, two pairs per 16-B chunk,
// chunk c at physical chunk c ^ ((c >> 4) & 7).  The cycle sweep's lanes read
// chunks 8 apart (16 samples = 8 chunks per cycle); unswizzled, the 16 lanes
// of a ds_read_b128 pass would hit 2 bank groups (8-way conflicts), swizzled
// they hit all 16 -- for any pulse start A.
__device__ __forceinline__ uint32_t env_chunk(uint32_t c) { return c ^ ((c >> 4) & 7u); }
// word index of pair q's E in that layout (E' at + 1)
__device__ __forceinline__ uint32_t env_pair(uint32_t q) { return (env_chunk(q >> 1) << 2) | ((q & 1u) << 1); }

// ---------------------------------------------------------------------------
// Y-form complex products (the quad and cycle sweeps)
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
// Record lookups.  A lane needs, for its cycle n, the latest strobe of the
// channel's element with t <= n (ties: the later event) and the latest
// pulse_reset with t <= n (its time t_ref, else 0) -- oracle/dds_ref.c's
// cursor, exact for a lane's events in time order (as dpemu_run writes them).
// ===========================================================================

// LDS-staged records, restricted to one tile's window: strobes st[s_lo, s_lo
// + s_n) and reset times rs[r_lo, r_lo + r_n), where the window starts at the
// latest record at or before the tile's first cycle (windows hold 1-3 records)
struct LdsLookup {
    const uint4 *st;
    const uint32_t *rs;
    uint32_t s_lo, s_n, r_lo, r_n;

    __device__ __forceinline__ bool strobe(uint32_t n, uint4 &rec) const
    {
        const uint4 *r = st + s_lo;
        int a = 0, b = (int)s_n;                         // first index with t > n
        while (a < b) {
            const int mid = (a + b) >> 1;
            if (r[mid].x <= n) a = mid + 1; else b = mid;
        }
        if (a == 0) return false;
        rec = r[a - 1];
        return true;
    }
    __device__ __forceinline__ uint32_t t_ref(uint32_t n) const
    {
        const uint32_t *r = rs + r_lo;
        int a = 0, b = (int)r_n;
        while (a < b) {
            const int mid = (a + b) >> 1;
            if (r[mid] <= n) a = mid + 1; else b = mid;
        }
        return a ? r[a - 1] : 0u;
    }
};

// The lane's raw event records in HBM (a tile that needs more records than a
// workgroup stages; dpemu_run's timelines never do -- strobes and resets of a
// lane are >= 3 cycles apart -- but hand-built event arrays may): a binary
// search over the time-ordered events, then a walk back to the kind asked for.
struct GlobalLookup {
    const uint4 *ev;
    uint32_t n_lanes, lane, n_ev, elem;

    __device__ __forceinline__ int last_le(uint32_t n) const
    {
        int a = 0, b = (int)n_ev;
        while (a < b) {
            const int mid = (a + b) >> 1;
            if (ev[(uint64_t)mid * n_lanes + lane].x <= n) a = mid + 1; else b = mid;
        }
        return a - 1;
    }
    __device__ __forceinline__ bool strobe(uint32_t n, uint4 &rec) const
    {
        for (int e = last_le(n); e >= 0; e--) {
            const uint4 x = ev[(uint64_t)e * n_lanes + lane];
            if ((x.y >> 28) == 0u && ((x.y >> 24) & 3u) == elem) {
                rec = make_uint4(x.x, x.y & 0xFFFFFFu, x.z, x.w & 0xFFFFu);
                return true;
            }
        }
        return false;
    }
    __device__ __forceinline__ uint32_t t_ref(uint32_t n) const
    {
        for (int e = last_le(n); e >= 0; e--) {
            const uint4 x = ev[(uint64_t)e * n_lanes + lane];
            if ((x.y >> 28) == 1u) return x.x;
        }
        return 0u;
    }
};

// ===========================================================================
// One wave-tile: DDS_TILE samples of a channel starting at sample c DDS_TILE.
// ===========================================================================
struct Chan {
    uint32_t spc, interp, env_off, env_len, freq_off, freq_len, spc_sh, int_sh;
    bool spc_p2, int_p2, quad;
};

struct Tables {                 // LDS-resident
    const int16_t *lut;
    const uint32_t *env, *freq;
    uint4 *xpose;               // this wave's 1-KiB transpose slice
};

template <class LK>
__device__ __forceinline__ void sweep_tile(const DDSParams &p, const Chan &C, const Tables &T, uint32_t *out,
                                           uint32_t c, const LK &lk)
{
    const uint32_t ln = threadIdx.x & 63u;
    const uint32_t tb = c * DDS_TILE;                                   // the tile's first sample
    const int16_t *s_lut = T.lut;
    const uint32_t *s_env = T.env, *s_freq = T.freq;
    if (C.quad && C.spc == 16u) {
        // ---- cycle sweep (16 samples / clk, the RFSoC rate): a lane makes one
        // whole cycle, so the record lookup, theta and carrier are done once
        // per 16 samples
        const uint32_t js = tb + 16 * ln;                               // this lane's cycle n = js / 16
        const uint32_t n = js >> 4;
        uint32_t v[16];
#pragma unroll
        for (int q = 0; q < 16; q++) v[q] = 0u;
        uint4 rec;
        if (js < p.n_samples && lk.strobe(n, rec)) {                    // {t, env word, phase | freq << 17, amp}
            const uint32_t A = rec.y & 0xFFFu, Lw = (rec.y >> 12) & 0xFFFu, fi = rec.z >> 17;
            const uint32_t room = C.env_len > 4 * A ? C.env_len - 4 * A : 0u;
            uint32_t lim, emask;
            if (Lw) {
                emask = 0xFFFFFFFFu;
                const uint32_t n_env = min(4 * Lw, room);
                lim = n_env << C.int_sh;
                if ((lim >> C.int_sh) != n_env) lim = 0xFFFFFFFFu;
            } else {
                emask = 0u;
                lim = room ? 0xFFFFFFFFu : 0u;
            }
            const uint32_t d0 = 16 * (n - rec.x);                       // samples since the strobe's first
            if (16 * fi + 15 < C.freq_len && d0 < lim) {
                const uint32_t t_ref = lk.t_ref(n);
                const uint32_t *frp = s_freq + 32 * fi;                 // (R, R') pairs; pair 0 = (F0, 0)
                const uint32_t idx = (frp[0] * (n - t_ref) + ((rec.z & 0x1FFFFu) << 15)) >> 20;
                const int32_t cc = lut_quarter(s_lut, (idx + 1024) & 4095), sn = lut_quarter(s_lut, idx);
                const int32_t a16 = (int32_t)(rec.w & 0xFFFFu);
                const uint32_t y0 = pack16((cc * a16 + (1 << 15)) >> 16, (sn * a16 + (1 << 15)) >> 16);
                const bool inside = d0 + 15 < lim && emask;
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    uint32_t R[4], Rp[4], E[4], Ep[4];
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint4 rw = *reinterpret_cast<const uint4 *>(frp + 8 * g + 4 * h);
                        R[2 * h] = rw.x; Rp[2 * h] = rw.y; R[2 * h + 1] = rw.z; Rp[2 * h + 1] = rw.w;
                    }
                    if (C.interp == 1) {
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
                    } else {                                             // interp >= 4: one env word for 4 samples
                        const uint32_t e = d0 + 4 * g < lim ? s_env[4 * A + (((d0 + 4 * g) >> C.int_sh) & emask)] : 0u;
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
        uint4 *xp = T.xpose;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if ((ln >> 4) == (uint32_t)r) {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    xp[4 * (ln & 15u) + (q ^ ((ln >> 2) & 3u))] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t lc = ln >> 2;                                // source lane 16 r + lc
            const uint4 x = xp[4 * lc + ((ln & 3u) ^ ((lc >> 2) & 3u))];
            const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
            store4(out, tb + 4 * (64u * r + ln), p.n_samples, w4);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");      // reads done before the next writes
            __builtin_amdgcn_wave_barrier();
        }
        return;
    }
    // ---- 4 rounds of 256 samples, 4 consecutive samples per lane (one 16-B store)
    const uint32_t k0 = (4 * ln) & (C.spc - 1);     // sub-sample slot (power-of-two spc; tiles start at multiples of 16)
#pragma unroll 1
    for (uint32_t r = 0; r < 4; r++) {
        const uint32_t j0 = tb + 256 * r + 4 * ln;
        if (j0 >= p.n_samples) break;
        uint32_t v[4] = {0u, 0u, 0u, 0u};
        uint4 rec;
        if (C.quad) {
            const uint32_t n = j0 >> C.spc_sh;                          // the lane's 4 samples share cycle n
            if (lk.strobe(n, rec)) {
                const uint32_t A = rec.y & 0xFFFu, Lw = (rec.y >> 12) & 0xFFFu, fi = rec.z >> 17;
                const uint32_t base = rec.x << C.spc_sh;                // sample index of the strobe
                // samples dd = j - base with env index (dd >> int_sh) & emask inside
                // the pulse and the table: dd < lim
                const uint32_t room = C.env_len > 4 * A ? C.env_len - 4 * A : 0u;
                uint32_t lim, emask;
                if (Lw) {
                    emask = 0xFFFFFFFFu;
                    const uint32_t n_env = min(4 * Lw, room);
                    lim = n_env << C.int_sh;
                    if ((lim >> C.int_sh) != n_env) lim = 0xFFFFFFFFu;  // no overflow past 2^32
                } else {
                    emask = 0u;                                         // CW: env word 4A forever
                    lim = room ? 0xFFFFFFFFu : 0u;
                }
                const uint32_t d0 = j0 - base;
                if (16 * fi + 15 < C.freq_len && d0 < lim) {            // (a finished pulse plays zeros)
                    const uint32_t t_ref = lk.t_ref(n);
                    const uint32_t *frp = s_freq + 32 * fi;             // (R, R') pairs; pair 0 = (F0, 0)
                    const uint32_t idx = (frp[0] * (n - t_ref) + ((rec.z & 0x1FFFFu) << 15)) >> 20;
                    const int32_t cc = lut_quarter(s_lut, (idx + 1024) & 4095), sn = lut_quarter(s_lut, idx);
                    const int32_t a16 = (int32_t)(rec.w & 0xFFFFu);
                    const uint32_t y0 = pack16((cc * a16 + (1 << 15)) >> 16, (sn * a16 + (1 << 15)) >> 16);
                    uint32_t R[4], Rp[4], E[4], Ep[4];
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint4 rw = *reinterpret_cast<const uint4 *>(frp + 2 * k0 + 4 * h);
                        R[2 * h] = rw.x; Rp[2 * h] = rw.y; R[2 * h + 1] = rw.z; Rp[2 * h + 1] = rw.w;
                    }
                    const bool inside = d0 + 3 < lim;
                    if (C.interp == 1) {
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
                    } else {                                             // interp >= 4: one env word for the 4
                        const uint32_t e = s_env[4 * A + ((d0 >> C.int_sh) & emask)], ep = neg_swap(e);
#pragma unroll
                        for (int s = 0; s < 4; s++) { E[s] = e; Ep[s] = ep; }
                    }
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        uint32_t y = rot_y(y0, R[s], Rp[s]);
                        if (s == 0 && k0 == 0) y = y0;                  // sub-sample 0 is the unrotated carrier
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
                const uint32_t n = C.spc_p2 ? (j >> C.spc_sh) : j / C.spc, k = j - n * C.spc;
                if (!lk.strobe(n, rec)) continue;
                const uint32_t A = rec.y & 0xFFFu, Lw = (rec.y >> 12) & 0xFFFu;
                const uint32_t rr = j - rec.x * C.spc;
                const uint32_t es = Lw ? (C.int_p2 ? (rr >> C.int_sh) : rr / C.interp) : 0u;
                const uint32_t widx = 4 * A + es;
                const uint32_t fi = rec.z >> 17, phase = rec.z & 0x1FFFFu;
                if ((!Lw || es < 4 * Lw) && widx < C.env_len && 16 * fi + 15 < C.freq_len) {
                    const uint32_t *fr = p.freq + C.freq_off + 16 * fi;
                    const uint32_t t_ref = lk.t_ref(n);
                    const Carrier a0 = carrier_quarter(s_lut, fr[0] * (n - t_ref) + (phase << 15), (int32_t)(rec.w & 0xFFFFu));
                    v[s] = mix(p.env[C.env_off + widx], k ? rotate(a0, fr[k]) : a0);
                }
            }
        }
        store4(out, j0, p.n_samples, v);
    }
}

// index of the latest staged time <= n, from a wave-uniform cursor at or
// below it (times sorted): a ballot over the next 64 entries per step
template <class TimeAt>
__device__ __forceinline__ int advance_le(TimeAt time_at, int cur, uint32_t cnt, uint32_t n)
{
    const uint32_t ln = threadIdx.x & 63u;
    for (;;) {
        const uint32_t i = (uint32_t)(cur + 1) + ln;
        const bool v = i < cnt && time_at(i) <= n;
        const int k = __popcll(__ballot(v));
        cur += k;
        if (k < 64) return cur;
    }
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// the cycle of sample j
__device__ __forceinline__ uint32_t cycle_of(const Chan &C, uint64_t j)
{
    return (uint32_t)(C.spc_p2 ? (j >> C.spc_sh) : j / C.spc);
}

// A workgroup's record staging area and the lane it reads
struct Work {
    uint8_t *rec;               // staging area, p.rec_bytes: strobe records {t, env word, phase | freq << 17,
                                //   amp} (16 B), then reset times (4 B)
    uint32_t (*cnt)[BLOCK / 64];
    uint32_t *stop;             // [2]: the first strobe / reset time not staged
    uint32_t lane, elem, n_ev;
};

struct Staged {
    const uint4 *st;
    const uint32_t *rs;
    uint32_t ns, nr, t_stop;    // staged counts; the first record time not staged (~0: none)
};

// Stage the strobes / resets with t <= n1 that cycles [n0, n1] can see: from
// the latest at or before n0 (events 4 per thread, ballot / popc compaction,
// the waves' counts combined in LDS).  MULTI = false: the host guarantees
// 16 event_cap <= rec_bytes, so all of them fit (strobes, then resets right
// behind).  MULTI: up to rec_bytes / 20 of each; t_stop = the first time left
// out.  *bad: OR-reduced over the workgroup (the tables' flag rides on the
// first barrier).
template <bool MULTI>
__device__ __forceinline__ Staged stage(const DDSParams &p, const Work &W, uint32_t n0, uint32_t n1, bool *bad)
{
    const uint32_t tid = threadIdx.x, wl = tid & 63u, wv = tid >> 6;
    const uint64_t below = wl ? (~0ull >> (64 - wl)) : 0ull;
    constexpr int K = DDS_MAX_EVENTS / BLOCK;                       // events per thread
    uint4 ev[K];
    bool is_st[K], is_rs[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t e = (wv * K + k) * 64u + wl;
        ev[k] = e < W.n_ev ? p.events[(uint64_t)e * p.n_lanes + W.lane] : make_uint4(0, 0, 0, 0);
    }
    uint32_t cnt[4] = {0u, 0u, 0u, 0u};                             // strobes, resets (t <= n1); those <= n0
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t e = (wv * K + k) * 64u + wl;
        const uint32_t kind = ev[k].y >> 28;
        const bool in = e < W.n_ev && ev[k].x <= n1;
        is_st[k] = in && kind == 0u && ((ev[k].y >> 24) & 3u) == W.elem;
        is_rs[k] = in && kind == 1u;
        cnt[0] += (uint32_t)__popcll(__ballot(is_st[k]));
        cnt[1] += (uint32_t)__popcll(__ballot(is_rs[k]));
        cnt[2] += (uint32_t)__popcll(__ballot(is_st[k] && ev[k].x <= n0));
        cnt[3] += (uint32_t)__popcll(__ballot(is_rs[k] && ev[k].x <= n0));
    }
    if (wl == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++) W.cnt[q][wv] = cnt[q];
    }
    if (MULTI && tid == 0) { W.stop[0] = 0xFFFFFFFFu; W.stop[1] = 0xFFFFFFFFu; }
    *bad = __syncthreads_or(*bad);
    uint32_t os = 0, orr = 0, tot[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t w = 0; w < BLOCK / 64; w++) {
        os += w < wv ? W.cnt[0][w] : 0u;
        orr += w < wv ? W.cnt[1][w] : 0u;
#pragma unroll
        for (int q = 0; q < 4; q++) tot[q] += W.cnt[q][w];
    }
    const uint32_t base_s = tot[2] ? tot[2] - 1 : 0u, base_r = tot[3] ? tot[3] - 1 : 0u;
    const uint32_t cap = MULTI ? (p.rec_bytes / 20) & ~7u : 0xFFFFFFFFu;
    const uint32_t ns = min(cap, tot[0] - base_s), nr = min(cap, tot[1] - base_r);
    uint4 *st = reinterpret_cast<uint4 *>(W.rec);
    uint32_t *rs = reinterpret_cast<uint32_t *>(st + (MULTI ? cap : ns));
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint64_t bs = __ballot(is_st[k]), br = __ballot(is_rs[k]);
        if (is_st[k]) {
            const uint32_t i = os + (uint32_t)__popcll(bs & below) - base_s;   // (wraps below base_s)
            if (i < ns) st[i] = make_uint4(ev[k].x, ev[k].y & 0xFFFFFFu, ev[k].z, ev[k].w & 0xFFFFu);
            if (MULTI && i == ns) W.stop[0] = ev[k].x;
        }
        if (is_rs[k]) {
            const uint32_t i = orr + (uint32_t)__popcll(br & below) - base_r;
            if (i < nr) rs[i] = ev[k].x;
            if (MULTI && i == nr) W.stop[1] = ev[k].x;
        }
        os += (uint32_t)__popcll(bs);
        orr += (uint32_t)__popcll(br);
    }
    __syncthreads();
    return Staged{st, rs, ns, nr, MULTI ? min(W.stop[0], W.stop[1]) : 0xFFFFFFFFu};
}

// tiles c < stop_tile end before the first unstaged record: every record they can see is staged
__device__ __forceinline__ uint32_t stop_tile(const Chan &C, const Staged &S, uint32_t c_end)
{
    return S.t_stop == 0xFFFFFFFFu ? c_end : (uint32_t)umin64(c_end, (uint64_t)S.t_stop * C.spc / DDS_TILE);
}

__device__ __forceinline__ uint32_t last_cycle(const DDSParams &p, const Chan &C, uint32_t c_end)
{
    return cycle_of(C, umin64((uint64_t)c_end * DDS_TILE, p.n_samples) - 1);
}

// tiles [c0, c1) from the staged records: wave w takes c0 + w, c0 + w + 4, ...
// and finds each tile's window with its cursors
__device__ __forceinline__ void sweep_staged(const DDSParams &p, const Chan &C, const Tables &T, uint32_t *out,
                                             uint32_t c0, uint32_t c1, const Staged &S)
{
    const uint4 *s_st = S.st;
    const uint32_t *s_rs = S.rs;
    const auto st_time = [=](uint32_t i) { return s_st[i].x; };
    const auto rs_time = [=](uint32_t i) { return s_rs[i]; };
    int cs = -1, cr = -1;                                           // the wave's cursors
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);    // (wave-uniform)
#pragma unroll 1
    for (uint32_t c = c0 + wv; c < c1; c += BLOCK / 64) {
        const uint32_t na = cycle_of(C, (uint64_t)c * DDS_TILE);
        const uint32_t nb = cycle_of(C, umin64((uint64_t)c * DDS_TILE + DDS_TILE, p.n_samples) - 1);
        cs = advance_le(st_time, cs, S.ns, na);
        const int se = advance_le(st_time, cs, S.ns, nb);
        cr = advance_le(rs_time, cr, S.nr, na);
        const int re = advance_le(rs_time, cr, S.nr, nb);
        const uint32_t slo = (uint32_t)max(cs, 0), rlo = (uint32_t)max(cr, 0);
        const LdsLookup lk{s_st, s_rs, slo, (uint32_t)(se + 1) - slo, rlo, (uint32_t)(re + 1) - rlo};
        sweep_tile(p, C, T, out, c, lk);
    }
}

#ifdef DDS_STRIPE_AB
__device__ __forceinline__ void sweep_stripe(const DDSParams &p, const Chan &C, const Tables &T, uint32_t *out,
                                             uint32_t s0, uint32_t step, uint32_t tiles, const Staged &S)
{
    const uint4 *s_st = S.st;
    const uint32_t *s_rs = S.rs;
    const auto st_time = [=](uint32_t i) { return s_st[i].x; };
    const auto rs_time = [=](uint32_t i) { return s_rs[i]; };
    int cs = -1, cr = -1;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll 1
    for (uint32_t c = s0 + wv * step; c < tiles; c += (BLOCK / 64) * step) {
        const uint32_t na = cycle_of(C, (uint64_t)c * DDS_TILE);
        const uint32_t nb = cycle_of(C, umin64((uint64_t)c * DDS_TILE + DDS_TILE, p.n_samples) - 1);
        cs = advance_le(st_time, cs, S.ns, na);
        const int se = advance_le(st_time, cs, S.ns, nb);
        cr = advance_le(rs_time, cr, S.nr, na);
        const int re = advance_le(rs_time, cr, S.nr, nb);
        const uint32_t slo = (uint32_t)max(cs, 0), rlo = (uint32_t)max(cr, 0);
        const LdsLookup lk{s_st, s_rs, slo, (uint32_t)(se + 1) - slo, rlo, (uint32_t)(re + 1) - rlo};
        sweep_tile(p, C, T, out, c, lk);
    }
}
#endif

// ===========================================================================
// dds_synth_kernel: workgroup = (channel, segment of seg_tiles tiles).
// MULTI (the host's choice when 16 event_cap > rec_bytes): a segment whose
// records do not fit one staging is swept in passes, each restaging from its
// first tile, and a tile that alone needs more than the area holds looks its
// records up in the lane's raw events (GlobalLookup).
// ===========================================================================
#ifndef DDS_WAVES
#define DDS_WAVES 6
#endif
template <bool MULTI>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(DDS_WAVES))) dds_synth_kernel(const DDSParams p)
{
    // dynamic LDS (dds_lds_bytes): quarter sine table | record area (rec_bytes) |
    // env | freq | store transpose (1 KiB per wave)
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    __shared__ uint32_t s_cnt[4][BLOCK / 64];
    __shared__ uint32_t s_stop[2];
    int16_t *s_lut = reinterpret_cast<int16_t *>(s_dyn);
    uint8_t *s_rec = s_dyn + DDS_LUT_BYTES;
    uint32_t *s_env = reinterpret_cast<uint32_t *>(s_rec + p.rec_bytes);
    uint32_t *s_freq = s_env + p.env_lds;
    uint4 *s_xpose = reinterpret_cast<uint4 *>(s_freq + p.freq_lds);

    const uint32_t tid = threadIdx.x;
    const uint32_t ch = blockIdx.x / p.segs, seg = blockIdx.x - ch * p.segs;
    const uint32_t c_begin = seg * p.seg_tiles, c_end = min(c_begin + p.seg_tiles, p.tiles);
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
    Chan C;
    C.spc = d[2];
    C.interp = d[3] ? d[3] : 1u;
    C.env_off = d[4]; C.env_len = d[5]; C.freq_off = d[6]; C.freq_len = d[7];
    C.spc_p2 = (C.spc & (C.spc - 1)) == 0;
    C.int_p2 = (C.interp & (C.interp - 1)) == 0;
    C.spc_sh = __ffs(C.spc) - 1;
    C.int_sh = __ffs(C.interp) - 1;
    const bool staged = (C.interp == 1 ? dds_env_pairs_words(C.env_len) : C.env_len) <= p.env_lds &&
                        2 * C.freq_len <= p.freq_lds;
    const Work W{s_rec, s_cnt, s_stop, d[0], d[1] & 3u, min(p.summary[8ull * d[0] + 2], p.event_cap)};

    // ---- tables (the only global loads besides the event scan)
    if (tid < DDS_LUT_BYTES / 16)                                      // entries 0..1031 (1024 needed)
        reinterpret_cast<uint4 *>(s_lut)[tid] = reinterpret_cast<const uint4 *>(p.sin_lut)[tid];
    bool bad = false;                       // a staged eq or rq is -32768: no Y form
    if (staged) {
        if (C.interp == 1) {
            for (uint32_t i = tid; i < C.env_len; i += BLOCK) {
                const uint32_t e = p.env[C.env_off + i];
                bad |= (e & 0xFFFFu) == 0x8000u;
                *reinterpret_cast<uint2 *>(s_env + env_pair(i)) = make_uint2(e, neg_swap(e));
            }
        } else {
            for (uint32_t i = tid; i < C.env_len; i += BLOCK) {
                const uint32_t e = p.env[C.env_off + i];
                bad |= (e & 0xFFFFu) == 0x8000u;
                s_env[i] = e;
            }
        }
        for (uint32_t i = tid; i < C.freq_len; i += BLOCK) {
            const uint32_t w = p.freq[C.freq_off + i];
            const bool rot = (i & 15u) != 0;
            bad |= rot && (w & 0xFFFFu) == 0x8000u;
            reinterpret_cast<uint2 *>(s_freq)[i] = make_uint2(w, rot ? neg_swap(w) : 0u);
        }
    }
    // ---- the segment's records (the tables' flag rides on the stage's barrier)
#ifdef DDS_STRIPE_AB
    if (!MULTI) {
        Staged S = stage<MULTI>(p, W, cycle_of(C, (uint64_t)seg * DDS_TILE), last_cycle(p, C, p.tiles), &bad);
        C.quad = staged && !bad && (C.spc & 3u) == 0 && C.spc_p2 && C.int_p2 && (C.interp == 1 || C.interp >= 4);
        const Tables T{s_lut, s_env, s_freq, s_xpose + 64 * __builtin_amdgcn_readfirstlane(tid >> 6)};
        sweep_stripe(p, C, T, p.iq + (uint64_t)ch * p.n_samples, seg, p.segs, p.tiles, S);
        return;
    }
#endif
    const uint32_t n_last = last_cycle(p, C, c_end);
    Staged S = stage<MULTI>(p, W, cycle_of(C, (uint64_t)c_begin * DDS_TILE), n_last, &bad);
    C.quad = staged && !bad && (C.spc & 3u) == 0 && C.spc_p2 && C.int_p2 && (C.interp == 1 || C.interp >= 4);
    const Tables T{s_lut, s_env, s_freq, s_xpose + 64 * __builtin_amdgcn_readfirstlane(tid >> 6)};
    uint32_t *out = p.iq + (uint64_t)ch * p.n_samples;
    if (!MULTI) {
        sweep_staged(p, C, T, out, c_begin, c_end, S);
        return;
    }
#pragma unroll 1
    for (uint32_t c0 = c_begin;;) {                                    // passes (workgroup-uniform)
        uint32_t c1 = stop_tile(C, S, c_end);
        if (c1 <= c0) {
            // tile c0 alone needs more records than the area holds
            if ((tid >> 6) == 0) {
                const GlobalLookup lk{p.events, p.n_lanes, W.lane, W.n_ev, W.elem};
                sweep_tile(p, C, T, out, c0, lk);
            }
            c1 = c0 + 1;
        } else {
            sweep_staged(p, C, T, out, c0, c1, S);
        }
        c0 = c1;
        if (c0 >= c_end) return;
        __syncthreads();                                               // every wave is done with the staged records
        S = stage<MULTI>(p, W, cycle_of(C, (uint64_t)c0 * DDS_TILE), n_last, &bad);
    }
}

hipError_t launch_dds(const DDSParams &p, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples) return hipSuccess;
    const uint32_t lds = dds_lds_bytes(p.rec_bytes, p.env_lds, p.freq_lds);
    const bool multi = 16ull * p.event_cap > p.rec_bytes;
    const void *fn = multi ? reinterpret_cast<const void *>(dds_synth_kernel<true>)
                           : reinterpret_cast<const void *>(dds_synth_kernel<false>);
    const hipError_t e = opt_in_dynamic_lds(fn, lds);
    if (e != hipSuccess) return e;
    if (multi)
        hipLaunchKernelGGL(dds_synth_kernel<true>, dim3(p.n_channels * p.segs), dim3(BLOCK), lds, stream, p);
    else
        hipLaunchKernelGGL(dds_synth_kernel<false>, dim3(p.n_channels * p.segs), dim3(BLOCK), lds, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
