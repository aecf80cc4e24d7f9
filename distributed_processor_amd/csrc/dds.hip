// dds.hip -- fixed-point DDS I/Q synthesis from emulated pulse events (gfx950).
//
// Spec: DESIGN.md §DDS and oracle/dds_ref.c (CPU restatement, bit-exact).
// Inputs are the interpreter's outputs in HBM (lane summaries + slot-major
// event records) and the assembler's env / freq buffers (asmparse.py:46-86
// formats).  HBM-write-bound by design: 4 B per output sample; everything
// else is read once per workgroup into LDS (the channel's events, env and
// freq tables, the sine table), so the sample loop issues no global loads --
// on gfx950 stores count in vmcnt, and a load in the loop would make every
// tile wait for the previous tile's stores.
//
// Grid: (sample chunks, channels).  A workgroup compacts its channel's
// events into LDS -- strobes of the channel's element and pulse_resets, both
// time-sorted because a core emits them in time order -- then sweeps its
// chunk in 1024-sample tiles; a thread produces 4 consecutive samples per
// tile and stores them with one 16-byte global_store_dwordx4 (a wave writes
// 1 KiB contiguous).
//
// Two sweeps, chosen per channel:
//  * quad  (spc % 4 == 0, interp 1 or a power of two >= 4, tables staged in
//          LDS -- every QubiC element): the 4 (or 8, when 8 | spc) samples
//          of a thread share one emulated cycle, so theta / carrier /
//          amplitude are computed once per cycle; strobe fields and the
//          thread's rotation words (its sub-sample slot never changes) once
//          per pulse; env words arrive as 16-B LDS reads.  Per sample:
//          4 v_dot2_i32_i16, 4 shifts, 4 clamps, 3 packs, 1 select.
//  * generic  (anything else the ABI accepts): the per-sample definition,
//          reading env / freq tables from global memory.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.h"

namespace dpemu {

// a.lo * b.lo + a.hi * b.hi + c on packed int16 pairs: one VOP3P
// v_dot2_i32_i16 with the rounding constant in an SGPR (the builtin lowers to
// v_dot2c + a v_mov of the accumulator per product)
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

// a0 = (c0 * amp + 2^15) >> 16 from the Q15 table at theta >> 20
__device__ __forceinline__ Carrier carrier(const int16_t *lut, uint32_t theta, int32_t amp)
{
    const uint32_t idx = theta >> 20;
    // |c0| < 2^15, amp < 2^16: v_mad_i32_i24
    const int32_t a16 = amp & 0xFFFF;
    const int32_t ai = ((int32_t)lut[(idx + 1024) & 4095] * a16 + (1 << 15)) >> 16;
    const int32_t aq = ((int32_t)lut[idx] * a16 + (1 << 15)) >> 16;
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store4(uint32_t *out, uint32_t j0, uint32_t c_end, const uint32_t v[4], bool nt = false)
{
    if (j0 + 3 < c_end) {
        const u32x4 w = {v[0], v[1], v[2], v[3]};
        if (nt)
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(out + j0));
        else
            *reinterpret_cast<u32x4 *>(out + j0) = w;
    } else {
        for (int s = 0; s < 4 && j0 + s < c_end; s++) out[j0 + s] = v[s];
    }
}

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
    uint32_t tiles_step;            // tile stride: 1 (chunked) or gridDim.x (interleaved)
    bool nt;
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
    for (uint32_t j0 = j_first; j0 < q.c_end; j0 += q.tiles_step * (SPT * BLOCK)) {
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
                v[s] = mix(ew[s], a) & (d0 + s < lim ? 0xFFFFFFFFu : 0u);
            }
        }
#pragma unroll
        for (int h = 0; h < NV; h++) store4(q.out, j0 + 4 * h, q.c_end, v + 4 * h, q.nt);
    }
}

__global__ void __launch_bounds__(BLOCK) dds_kernel(const DDSParams p)
{
    // dynamic LDS (dds_lds_bytes): sine table | compacted strobes / resets |
    // staged env table | staged freq table
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    int16_t *s_lut = reinterpret_cast<int16_t *>(s_dyn);
    uint32_t *s_st_t = reinterpret_cast<uint32_t *>(s_dyn + 8192);
    uint32_t *s_st_env = s_st_t + p.ev_lds;
    uint32_t *s_st_pf = s_st_env + p.ev_lds;
    uint32_t *s_rs_t = s_st_pf + p.ev_lds;
    uint32_t *s_env = s_rs_t + p.ev_lds;
    uint32_t *s_freq = s_env + p.env_lds;
    uint16_t *s_st_amp = reinterpret_cast<uint16_t *>(s_freq + p.freq_lds);
    __shared__ uint32_t s_tmp[2 * (BLOCK / 64)];
    __shared__ uint32_t s_cnt[2];

    const uint32_t tid = threadIdx.x, wl = tid & 63, wv = tid >> 6;
    const uint32_t ch = blockIdx.y;
    const uint32_t *d = p.ch + DDS_CH_WORDS * ch;
    const uint32_t lane = d[0], elem = d[1], spc = d[2], interp = d[3] ? d[3] : 1u;
    const uint32_t env_off = d[4], env_len = d[5], freq_off = d[6], freq_len = d[7];
    const bool spc_p2 = (spc & (spc - 1)) == 0, int_p2 = (interp & (interp - 1)) == 0;
    const uint32_t spc_sh = __ffs(spc) - 1, int_sh = __ffs(interp) - 1;
    const bool staged = env_len <= p.env_lds && freq_len <= p.freq_lds;
    if (p.probe == 5) {                         // probe: persistent grid, flattened 4-KiB tiles
        const uint64_t total = (uint64_t)p.n_channels * p.n_samples;
        const uint64_t G = (uint64_t)gridDim.x * gridDim.y, wg = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
        const u32x4 z = {0, 0, 0, 0};
        for (uint64_t j = (wg * BLOCK + tid) * 4; j + 3 < total; j += G * BLOCK * 4)
            *reinterpret_cast<u32x4 *>(p.iq + j) = z;
        return;
    }
    if (p.probe >= 3) {                         // probe: flat zero stores over the whole output,
        // workgroup-contiguous spans of (probe == 3 ? chunk : 4 * BLOCK) samples
        const uint64_t total = (uint64_t)p.n_channels * p.n_samples;
        const uint64_t span = p.probe == 3 ? p.chunk : 4 * BLOCK;
        const uint64_t wg = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
        const u32x4 z = {0, 0, 0, 0};
        for (uint64_t b = wg * span; b < total; b += (uint64_t)gridDim.x * gridDim.y * span)
            for (uint64_t j = b + 4 * tid; j < b + span && j + 3 < total; j += 4 * BLOCK)
                *reinterpret_cast<u32x4 *>(p.iq + j) = z;
        return;
    }
    if (p.probe == 2) {                         // probe: the grid's zero stores alone
        uint32_t *o = p.iq + (uint64_t)ch * p.n_samples;
        const uint32_t z[4] = {0, 0, 0, 0};
        if (p.ilv) {
            for (uint32_t j0 = blockIdx.x * 4 * BLOCK + 4 * tid; j0 < p.n_samples; j0 += gridDim.x * 4 * BLOCK)
                store4(o, j0, p.n_samples, z, p.nt);
        } else {
            const uint32_t e = min(blockIdx.x * p.chunk + p.chunk, p.n_samples);
            for (uint32_t j0 = blockIdx.x * p.chunk + 4 * tid; j0 < e; j0 += 4 * BLOCK) store4(o, j0, e, z, p.nt);
        }
        return;
    }

    // ---- prologue: issue every global load of the workgroup up front ----
    uint32_t n_ev = p.summary[8ull * lane + 2];
    n_ev = min(n_ev, p.event_cap);
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
    for (uint32_t i = tid; i < 4096 / 8; i += BLOCK)
        reinterpret_cast<uint4 *>(s_lut)[i] = reinterpret_cast<const uint4 *>(p.sin_lut)[i];
    if (staged) {
        for (uint32_t i = tid; i < env_len; i += BLOCK) s_env[i] = p.env[env_off + i];
        for (uint32_t i = tid; i < freq_len; i += BLOCK) s_freq[i] = p.freq[freq_off + i];
    }
    if (tid == 0) { s_cnt[0] = 0; s_cnt[1] = 0; }
    __syncthreads();

    // ---- compact this channel's strobes and the lane's pulse_resets into LDS ----
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
        if (is_st) {
            const uint32_t i = os + (uint32_t)__popcll(bs & below);
            s_st_t[i] = ev.x; s_st_env[i] = ev.z & 0xFFFFFFu; s_st_pf[i] = ev.w; s_st_amp[i] = (uint16_t)ampr[ps];
        }
        if (is_rs) s_rs_t[orr + (uint32_t)__popcll(br & below)] = ev.x;
        __syncthreads();
        if (tid == 0) { s_cnt[0] += ts; s_cnt[1] += tr; }
        __syncthreads();
    }
    const int n_st = (int)s_cnt[0], n_rs = (int)s_cnt[1];

    uint32_t *out = p.iq + (uint64_t)ch * p.n_samples;
    // Chunked: workgroup x owns samples [x * chunk, (x + 1) * chunk) and sweeps
    // them tile by tile.  Interleaved (p.ilv): workgroup x owns tiles x, x + X,
    // x + 2X, ... of its channel, so the X workgroups of a channel -- dispatched
    // together -- write one contiguous, advancing window.
    const uint32_t X = gridDim.x;
    const uint32_t c_begin = p.ilv ? 0u : blockIdx.x * p.chunk;
    const uint32_t c_end = p.ilv ? p.n_samples : min(c_begin + p.chunk, p.n_samples);
    const uint32_t tstep = p.ilv ? X : 1u;
    // first sample of this thread for SPT samples per thread
    auto first = [&](uint32_t spt) { return (p.ilv ? blockIdx.x * spt * BLOCK : c_begin) + spt * tid; };

    if (p.probe == 1) {                         // probe: prologue, then zero stores
        const uint32_t z[4] = {0, 0, 0, (uint32_t)(n_st + n_rs) & 0u};
        for (uint32_t j0 = first(4); j0 < c_end; j0 += tstep * 4 * BLOCK) store4(out, j0, c_end, z, p.nt);
        return;
    }
    const bool quad = staged && (spc & 3u) == 0 && spc_p2 && int_p2 && (interp == 1 || interp >= 4);
    if (quad) {
        const QuadArgs q{s_lut, s_st_t, s_st_env, s_st_pf, s_st_amp, s_rs_t, n_st, n_rs, spc, spc_sh, interp, int_sh,
                         s_env, env_len, s_freq, freq_len, out, c_end, tstep, p.nt != 0};
        if ((spc & 7u) == 0 && p.spt8)
            sweep_quad<8>(q, first(8));
        else
            sweep_quad<4>(q, first(4));
        return;
    }

    // ---- generic sweep: the per-sample definition ----
    // cursors: latest strobe / reset at or before the current cycle.  A
    // thread's samples only move forward, so after one binary search at the
    // first sample the cursors advance by a short linear scan per tile.
    const uint32_t j_first = first(4);
    const uint32_t n_first = spc_p2 ? (j_first >> spc_sh) : j_first / spc;
    int si = last_le(s_st_t, n_st, n_first), ri = last_le(s_rs_t, n_rs, n_first);
    for (uint32_t j0 = j_first; j0 < c_end; j0 += tstep * 4 * BLOCK) {
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
        store4(out, j0, c_end, v, p.nt);
    }
}

hipError_t launch_dds(const DDSParams &p, hipStream_t stream)
{
    if (!p.n_channels || !p.n_samples) return hipSuccess;
    const uint32_t chunks = (p.n_samples + p.chunk - 1) / p.chunk;
    if (p.probe == 5) {
        hipLaunchKernelGGL(dds_kernel, dim3(p.chunk / 64, 1), dim3(BLOCK), dds_lds_bytes(p.ev_lds, p.env_lds, p.freq_lds),
                           stream, p);
        return hipGetLastError();
    }
    if (p.probe == 4) {                         // probe: fill-like grid, one 16-B store per thread
        const uint64_t total = (uint64_t)p.n_channels * p.n_samples;
        const uint64_t blocks = (total + 4 * BLOCK - 1) / (4 * BLOCK);
        hipLaunchKernelGGL(dds_kernel, dim3(65535, (uint32_t)((blocks + 65534) / 65535)), dim3(BLOCK), 0, stream, p);
        return hipGetLastError();
    }
    const uint32_t lds = dds_lds_bytes(p.ev_lds, p.env_lds, p.freq_lds);
    if (lds > 64 * 1024) {
        static bool attr = false;               // opt in to > 64 KiB of dynamic LDS once
        if (!attr) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(dds_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            attr = true;
        }
    }
    hipLaunchKernelGGL(dds_kernel, dim3(chunks, p.n_channels), dim3(BLOCK), lds, stream, p);
    return hipGetLastError();
}

}  // namespace dpemu
