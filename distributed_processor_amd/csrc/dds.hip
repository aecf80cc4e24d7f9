// dds.hip -- fixed-point DDS I/Q synthesis from emulated pulse events (gfx950).
//
// Spec: DESIGN.md §DDS and oracle/dds_ref.c (CPU restatement, bit-exact).
// Inputs are the interpreter's outputs in HBM (lane summaries + slot-major
// event records) and the assembler's env / freq buffers (asmparse.py:46-86
// formats).  HBM-write-bound by design: 4 B per output sample, everything
// else is read once per workgroup (events -> LDS) or hits L2 (env / freq
// tables), so the sample loop is budgeted in VALU ops per sample.
//
// Grid: (sample chunks, channels).  A workgroup compacts its channel's
// events into LDS -- strobes of the channel's element and pulse_resets, both
// time-sorted because a core emits them in time order -- then sweeps its
// chunk in 1024-sample tiles; a thread produces 4 consecutive samples per
// tile and stores them with one 16-byte global_store_dwordx4 (a wave writes
// 1 KiB contiguous).
//
// Two sweeps, chosen per channel:
//  * quad  (spc % 4 == 0, interp 1 or a power of two >= 4, tables 16-B
//          aligned -- every QubiC element): the 4 samples of a thread share
//          one emulated cycle, so theta / carrier / amplitude are computed
//          once per 4 samples and strobe fields once per pulse; env and
//          rotation words arrive as single 16-B loads.  Per sample: 4
//          v_dot2_i32_i16, 4 shifts, 4 clamps, 3 packs.
//  * generic  (anything else the ABI accepts): the per-sample definition.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.h"

namespace dpemu {

typedef short s16x2 __attribute__((ext_vector_type(2)));

// a.lo * b.lo + a.hi * b.hi + c on packed int16 pairs: one v_dot2_i32_i16
__device__ __forceinline__ int32_t dot2(uint32_t a, uint32_t b, int32_t c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), c, false);
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

// a0 = (c0 * amp + 2^15) >> 16 from the Q15 table at theta >> 20
__device__ __forceinline__ Carrier carrier(const int16_t *lut, uint32_t theta, int32_t amp)
{
    const uint32_t idx = theta >> 20;
    const int32_t ai = (__mul24((int32_t)lut[(idx + 1024) & 4095], amp) + (1 << 15)) >> 16;
    const int32_t aq = (__mul24((int32_t)lut[idx], amp) + (1 << 15)) >> 16;
    return Carrier{pack16(-aq, ai), pack16(ai, aq)};
}

// a = symsat((a0 (x) R_k + 2^14) >> 15)
__device__ __forceinline__ Carrier rotate(Carrier a0, uint32_t rw)
{
    const int32_t cr = clampi(dot2(rw, a0.X, 1 << 14) >> 15, -32767, 32767);
    const int32_t cq = clampi(dot2(rw, a0.Y, 1 << 14) >> 15, -32767, 32767);
    return Carrier{pack16(-cq, cr), pack16(cr, cq)};
}

// sat16((env (x) a + 2^14) >> 15), packed {I low, Q high}
__device__ __forceinline__ uint32_t mix(uint32_t ew, Carrier a)
{
    return pack16(clampi(dot2(ew, a.X, 1 << 14) >> 15, -32768, 32767),
                  clampi(dot2(ew, a.Y, 1 << 14) >> 15, -32768, 32767));
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

__device__ __forceinline__ void store4(uint32_t *out, uint32_t j0, uint32_t c_end, const uint32_t v[4])
{
    if (j0 + 3 < c_end) {
        *reinterpret_cast<uint4 *>(out + j0) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
        for (int s = 0; s < 4 && j0 + s < c_end; s++) out[j0 + s] = v[s];
    }
}

__global__ void __launch_bounds__(BLOCK) dds_kernel(const DDSParams p)
{
    __shared__ int16_t s_lut[4096];
    __shared__ uint32_t s_st_t[DDS_MAX_EVENTS], s_st_env[DDS_MAX_EVENTS], s_st_pf[DDS_MAX_EVENTS];
    __shared__ uint16_t s_st_amp[DDS_MAX_EVENTS];
    __shared__ uint32_t s_rs_t[DDS_MAX_EVENTS];
    __shared__ uint32_t s_tmp[2 * (BLOCK / 64)];
    __shared__ uint32_t s_cnt[2];

    const uint32_t tid = threadIdx.x, wl = tid & 63, wv = tid >> 6;
    const uint32_t ch = blockIdx.y;
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
    const uint32_t lane = d[0], elem = d[1], spc = d[2], interp = d[3] ? d[3] : 1u;
    const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
    const bool spc_p2 = (spc & (spc - 1)) == 0, int_p2 = (interp & (interp - 1)) == 0;
    const uint32_t spc_sh = __ffs(spc) - 1, int_sh = __ffs(interp) - 1;

    for (uint32_t i = tid; i < 4096; i += BLOCK) s_lut[i] = p.sin_lut[i];
    uint32_t n_ev = p.summary[8ull * lane + 2];
    n_ev = min(n_ev, p.event_cap);
    if (tid == 0) { s_cnt[0] = 0; s_cnt[1] = 0; }
    __syncthreads();

    // ---- compact this channel's strobes and the lane's pulse_resets into LDS ----
    for (uint32_t b = 0; b < n_ev; b += BLOCK) {
        const uint32_t e = b + tid;
        uint4 ev = make_uint4(0, 0, 0, 0);
        uint16_t amp = 0;
        if (e < n_ev) {
            ev = p.ev_main[(uint64_t)e * p.n_lanes + lane];
            amp = p.ev_amp[(uint64_t)e * p.n_lanes + lane];
        }
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
        if (is_st) {
            const uint32_t i = os + (uint32_t)__popcll(bs & below);
            s_st_t[i] = ev.x; s_st_env[i] = ev.z & 0xFFFFFFu; s_st_pf[i] = ev.w; s_st_amp[i] = amp;
        }
        if (is_rs) s_rs_t[orr + (uint32_t)__popcll(br & below)] = ev.x;
        __syncthreads();
        if (tid == 0) { s_cnt[0] += ts; s_cnt[1] += tr; }
        __syncthreads();
    }
    const int n_st = (int)s_cnt[0], n_rs = (int)s_cnt[1];

    uint32_t *out = p.iq + (uint64_t)ch * p.n_samples;
    const uint32_t c_begin = blockIdx.x * DDS_CHUNK;
    const uint32_t c_end = min(c_begin + DDS_CHUNK, p.n_samples);
    // cursors: latest strobe / reset at or before the current cycle.  A
    // thread's samples only move forward, so after one binary search at the
    // first sample the cursors advance by a short linear scan per tile.
    const uint32_t j_first = c_begin + 4 * tid;
    const uint32_t n_first = spc_p2 ? (j_first >> spc_sh) : j_first / spc;
    int si = last_le(s_st_t, n_st, n_first), ri = last_le(s_rs_t, n_rs, n_first);

    const bool quad = (spc & 3u) == 0 && spc_p2 && int_p2 && (interp == 1 || interp >= 4) &&
                      (env_off & 3u) == 0 && (freq_off & 3u) == 0 &&
                      (((uintptr_t)p.env | (uintptr_t)p.freq) & 15u) == 0;
    if (quad) {
        // ---- quad sweep: one cycle per thread per tile ----
        int cur = -2;                                   // strobe whose fields are cached
        bool act = false;                               // strobe plays (freq entry valid)
        uint32_t base = 0, lim = 0, emask = 0, F0 = 0, ph15 = 0;
        int32_t amp = 0;
        const uint32_t *envp = p.env, *frp = p.freq;
        for (uint32_t j0 = j_first; j0 < c_end; j0 += 4 * BLOCK) {
            const uint32_t n = j0 >> spc_sh, k0 = j0 & (spc - 1);
            while (si + 1 < n_st && s_st_t[si + 1] <= n) si++;
            while (ri + 1 < n_rs && s_rs_t[ri + 1] <= n) ri++;
            uint32_t v[4] = {0, 0, 0, 0};
            if (si != cur) {                            // new pulse: decode its fields once
                cur = si;
                act = false;
                if (si >= 0) {
                    const uint32_t env_w = s_st_env[si], pf = s_st_pf[si];
                    const uint32_t A = env_w & 0xFFFu, L = (env_w >> 12) & 0xFFFu, fi = pf >> 17;
                    base = s_st_t[si] * spc;            // sample index of the strobe
                    // samples d = j - base with env index (d >> int_sh) & emask inside the
                    // pulse and the table: d < lim
                    const uint32_t room = env_len > 4 * A ? env_len - 4 * A : 0u;
                    if (L) {
                        emask = 0xFFFFFFFFu;
                        const uint32_t n_env = min(4 * L, room);
                        lim = n_env << int_sh;
                        if ((lim >> int_sh) != n_env) lim = 0xFFFFFFFFu;   // no overflow past 2^32
                    } else {
                        emask = 0u;                     // CW: env word 4A forever
                        lim = room ? 0xFFFFFFFFu : 0u;
                    }
                    envp = p.env + env_off + 4 * A;
                    frp = p.freq + freq_off + 16 * fi;
                    act = 16 * fi + 15 < freq_len;
                    F0 = act ? frp[0] : 0u;
                    ph15 = (pf & 0x1FFFFu) << 15;
                    amp = s_st_amp[si];
                }
            }
            if (act) {
                const uint32_t t_ref = ri >= 0 ? s_rs_t[ri] : 0u;
                const Carrier a0 = carrier(s_lut, F0 * (n - t_ref) + ph15, amp);
                const uint4 rw = *reinterpret_cast<const uint4 *>(frp + k0);
                const uint32_t d0 = j0 - base;
                uint32_t ew[4];
                if (interp == 1 && d0 + 3 < lim && emask) {
                    const uint4 e4 = *reinterpret_cast<const uint4 *>(envp + d0);
                    ew[0] = e4.x; ew[1] = e4.y; ew[2] = e4.z; ew[3] = e4.w;
                } else {
#pragma unroll
                    for (int s = 0; s < 4; s++)
                        ew[s] = d0 + s < lim ? envp[((d0 + s) >> int_sh) & emask] : 0u;
                }
                const uint32_t r[4] = {rw.x, rw.y, rw.z, rw.w};
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const Carrier a = (k0 + s == 0) ? a0 : rotate(a0, r[s]);
                    v[s] = d0 + s < lim ? mix(ew[s], a) : 0u;
                }
            }
            store4(out, j0, c_end, v);
        }
        return;
    }

    // ---- generic sweep: the per-sample definition ----
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
                    const Carrier a0 = carrier(s_lut, fr[0] * (n - t_ref) + (phase << 15), s_st_amp[si]);
                    o = mix(p.env[env_off + widx], k ? rotate(a0, fr[k]) : a0);
                }
            }
            v[s] = o;
        }
        store4(out, j0, c_end, v);
    }
}

hipError_t launch_dds(const DDSParams &p, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples) return hipSuccess;
    const uint32_t chunks = (p.n_samples + DDS_CHUNK - 1) / DDS_CHUNK;
    hipLaunchKernelGGL(dds_kernel, dim3(chunks, p.n_channels), dim3(BLOCK), 0, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
