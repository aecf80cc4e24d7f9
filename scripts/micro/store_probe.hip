// HBM streaming-store pattern microbenchmark for the DDS output (1.72 GB per
// launch at config 5: 2048 channels x 209952 int16-I/Q samples).  Every
// variant writes the same bytes; only which workgroup writes which 16-B piece,
// and when, changes.  Question it answers: is the DDS kernel's store floor
// (5.4-5.8 TB/s for its chunk layout) set by chip-wide address locality?
//
//   chunk_contig : grid (chunks, channels); a WG owns 32 Ki contiguous samples,
//                  a thread 8 contiguous samples per tile (the current kernel)
//   chunk_rows   : same ownership, every store instruction 1 KiB dense
//   ileave_G     : G WGs per channel; tile = 2048 samples; WG w writes tiles
//                  w, w+G, w+2G ... (the channel's WGs advance together)
//   fill_T       : 1-D grid, WG b writes tile b of T samples (torch-fill-like)
//   persist      : 2048 WGs sweep the whole buffer tile by tile, grid-stride
//   *_nt         : the same with nontemporal stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 256;

template <bool NT>
__device__ __forceinline__ void st(uint32_t *p, uint32_t v)
{
    const u32x4 w = {v, v + 1, v + 2, v + 3};
    if (NT) __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
    else *reinterpret_cast<u32x4 *>(p) = w;
}

// a WG's samples [b, e): 2048 samples per tile, thread = 2 x 16 B
template <bool NT, bool ROWS>
__device__ __forceinline__ void tile(uint32_t *out, uint32_t b, uint32_t e)
{
    const uint32_t t = threadIdx.x;
    if (ROWS) {
        const uint32_t j = b + 4 * t;
        if (j + 3 < e) st<NT>(out + j, j);
        if (j + 4 * BLOCK + 3 < e) st<NT>(out + j + 4 * BLOCK, j);
    } else {
        const uint32_t j = b + 8 * t;
        if (j + 3 < e) st<NT>(out + j, j);
        if (j + 7 < e) st<NT>(out + j + 4, j);
    }
}

template <bool NT, bool ROWS>
__global__ void __launch_bounds__(BLOCK) chunk_k(uint32_t *iq, uint32_t n_samples, uint32_t chunk)
{
    uint32_t *out = iq + (uint64_t)blockIdx.y * n_samples;
    const uint32_t c0 = blockIdx.x * chunk, c1 = min(c0 + chunk, n_samples);
    for (uint32_t b = c0; b < c1; b += 2048) tile<NT, ROWS>(out, b, c1);
}

template <bool NT>
__global__ void __launch_bounds__(BLOCK) ileave_k(uint32_t *iq, uint32_t n_samples, uint32_t G)
{
    uint32_t *out = iq + (uint64_t)blockIdx.y * n_samples;
    for (uint32_t b = blockIdx.x * 2048; b < n_samples; b += G * 2048) tile<NT, true>(out, b, n_samples);
}

template <bool NT>
__global__ void __launch_bounds__(BLOCK) fill_k(uint32_t *iq, uint64_t total, uint32_t T)
{
    const uint64_t b0 = (uint64_t)blockIdx.x * T;
    for (uint32_t o = 0; o < T; o += 2048) {
        const uint64_t b = b0 + o;
        if (b >= total) return;
        const uint32_t j = 4 * threadIdx.x;
        if (b + j + 3 < total) st<NT>(iq + b + j, j);
        if (b + j + 4 * BLOCK + 3 < total) st<NT>(iq + b + j + 4 * BLOCK, j);
    }
}

template <bool NT>
__global__ void __launch_bounds__(BLOCK) persist_k(uint32_t *iq, uint64_t total)
{
    for (uint64_t b = (uint64_t)blockIdx.x * 2048; b < total; b += (uint64_t)gridDim.x * 2048) {
        const uint32_t j = 4 * threadIdx.x;
        if (b + j + 3 < total) st<NT>(iq + b + j, j);
        if (b + j + 4 * BLOCK + 3 < total) st<NT>(iq + b + j + 4 * BLOCK, j);
    }
}

// one 16-B store per thread, WG of B threads: the torch elementwise-fill shape
template <int B>
__global__ void __launch_bounds__(B) fill1_k(uint32_t *iq, uint64_t total)
{
    const uint64_t j = ((uint64_t)blockIdx.x * B + threadIdx.x) * 4;
    if (j + 3 < total) st<false>(iq + j, (uint32_t)j);
}

// U 16-B row stores per thread (each instruction 1 KiB dense per wave), WG of 256
template <int U>
__global__ void __launch_bounds__(BLOCK) fillU_k(uint32_t *iq, uint64_t total)
{
    const uint64_t b = (uint64_t)blockIdx.x * (U * 4 * BLOCK);
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t j = b + 4 * threadIdx.x + (uint64_t)u * 4 * BLOCK;
        if (j + 3 < total) st<false>(iq + j, (uint32_t)j);
    }
}

// the dds_tile_kernel store shape: grid (stripes, channels), 1024-sample tiles
// (4 KiB, four 1-KiB row stores per wave), wave w of stripe s takes local
// tiles w, w + 4, ... of its stripe; RR: local tile i = tile s + i * stripes,
// else the stripe's contiguous run s * TPS + i
template <bool RR>
__global__ void __launch_bounds__(BLOCK) ddsshape_k(uint32_t *iq, uint32_t n_samples, uint32_t tps)
{
    const uint32_t tiles = (n_samples + 1023) / 1024, stripes = gridDim.x, s = blockIdx.x;
    uint32_t *out = iq + (uint64_t)blockIdx.y * n_samples;
    const uint32_t n_t = RR ? (tiles - s + stripes - 1) / stripes : min(tps, tiles - s * tps);
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t i = wv; i < n_t; i += 4) {
        const uint32_t t = RR ? s + i * stripes : s * tps + i;
        for (int r = 0; r < 4; r++) {
            const uint32_t j = t * 1024 + 4 * (64 * r + ln);
            if (j + 3 < n_samples) st<false>(out + j, j);
        }
    }
}

// flattened buffer, 1024-sample tiles; WG b writes T consecutive tiles, wave w tiles w, w + 4, ...
__global__ void __launch_bounds__(BLOCK) wgtiles_k(uint32_t *iq, uint64_t total, uint32_t T)
{
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t i = wv; i < T; i += 4) {
        const uint64_t t = (uint64_t)blockIdx.x * T + i;
        for (int r = 0; r < 4; r++) {
            const uint64_t j = t * 1024 + 4 * (64 * r + ln);
            if (j + 3 < total) st<false>(iq + j, (uint32_t)j);
        }
    }
}

// WG b = tiles 4b .. 4b + 3 of channel b / tpc (tpc = WGs per channel), one tile per wave
__global__ void __launch_bounds__(BLOCK) wavetile_k(uint32_t *iq, uint32_t n_samples, uint32_t tpc)
{
    const uint32_t ch = blockIdx.x / tpc, tw = blockIdx.x % tpc;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    uint32_t *out = iq + (uint64_t)ch * n_samples;
    const uint32_t t = 4 * tw + wv;
    for (int r = 0; r < 4; r++) {
        const uint32_t j = t * 1024 + 4 * (64 * r + ln);
        if (j + 3 < n_samples) st<false>(out + j, j);
    }
}

// the dds_tile_kernel stripes, but the workgroup writes each tile together:
// for the stripe's local tiles 4m .. 4m + 3, round r stores tile 4m + r with
// wave w writing its row w (1 KiB), so every round is one dense 4 KiB
template <bool RR>
__global__ void __launch_bounds__(BLOCK) ddswg_k(uint32_t *iq, uint32_t n_samples, uint32_t tps)
{
    const uint32_t tiles = (n_samples + 1023) / 1024, stripes = gridDim.x, s = blockIdx.x;
    uint32_t *out = iq + (uint64_t)blockIdx.y * n_samples;
    const uint32_t n_t = RR ? (tiles - s + stripes - 1) / stripes : min(tps, tiles - s * tps);
    for (uint32_t i = 0; i < n_t; i++) {
        const uint32_t t = RR ? s + i * stripes : s * tps + i;
        const uint32_t j = t * 1024 + 4 * threadIdx.x;
        if (j + 3 < n_samples) st<false>(out + j, j);
    }
}

// balanced contiguous stripes: channel tiles split into `ns` near-equal runs,
// wave w of stripe s takes local tiles w, w + 4, ...
__global__ void __launch_bounds__(BLOCK) ddsbal_k(uint32_t *iq, uint32_t n_samples, uint32_t ns)
{
    const uint32_t tiles = (n_samples + 1023) / 1024, s = blockIdx.x;
    uint32_t *out = iq + (uint64_t)blockIdx.y * n_samples;
    const uint32_t t0 = (uint32_t)((uint64_t)tiles * s / ns), t1 = (uint32_t)((uint64_t)tiles * (s + 1) / ns);
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t t = t0 + wv; t < t1; t += 4) {
        for (int r = 0; r < 4; r++) {
            const uint32_t j = t * 1024 + 4 * (64 * r + ln);
            if (j + 3 < n_samples) st<false>(out + j, j);
        }
    }
}

static double timeit(void (*launch)(void *), void *a, uint64_t bytes)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch(a);
    hipDeviceSynchronize();
    float best = 1e30f, sum = 0;
    const int R = 10;
    for (int r = 0; r < R; r++) {
        hipEventRecord(e0);
        launch(a);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
        sum += ms;
    }
    hipEventDestroy(e0); hipEventDestroy(e1);
    return bytes / (best * 1e-3) / 1e12;
}

struct A { uint32_t *iq; uint32_t ns, nch, p; };
static A g;

int main(int argc, char **argv)
{
    g.nch = 2048; g.ns = 209952;
    const uint64_t total = (uint64_t)g.nch * g.ns, bytes = total * 4;
    if (hipMalloc(&g.iq, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    auto report = [&](const char *name, void (*fn)(void *)) {
        const double tbs = timeit(fn, &g, bytes);
        printf("{\"variant\": \"%s\", \"TB_s\": %.3f, \"ms\": %.4f}\n", name, tbs, bytes / (tbs * 1e12) * 1e3);
        fflush(stdout);
    };
    {
        const uint32_t tiles = (g.ns + 1023) / 1024;
        static const uint32_t TPSs[] = {16, 8, 32};
        for (uint32_t T : TPSs) {
            char nm[64];
            g.p = T;
            snprintf(nm, sizeof nm, "ddsshape_rr_%u", T);
            report(nm, [](void *) { const uint32_t tl = (g.ns + 1023) / 1024; ddsshape_k<true><<<dim3((tl + g.p - 1) / g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
            snprintf(nm, sizeof nm, "ddsshape_cont_%u", T);
            report(nm, [](void *) { const uint32_t tl = (g.ns + 1023) / 1024; ddsshape_k<false><<<dim3((tl + g.p - 1) / g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
            snprintf(nm, sizeof nm, "ddswg_rr_%u", T);
            report(nm, [](void *) { const uint32_t tl = (g.ns + 1023) / 1024; ddswg_k<true><<<dim3((tl + g.p - 1) / g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
            snprintf(nm, sizeof nm, "ddswg_cont_%u", T);
            report(nm, [](void *) { const uint32_t tl = (g.ns + 1023) / 1024; ddswg_k<false><<<dim3((tl + g.p - 1) / g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
            snprintf(nm, sizeof nm, "wgtiles_%u", T);
            report(nm, [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; wgtiles_k<<<(uint32_t)((t / 1024 + g.p - 1) / g.p), BLOCK>>>(g.iq, t, g.p); });
        }
        report("wavetile", [](void *) { const uint32_t tl = (g.ns + 1023) / 1024, tpc = (tl + 3) / 4; wavetile_k<<<g.nch * tpc, BLOCK>>>(g.iq, g.ns, tpc); });
        report("fill1_256_again", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fill1_k<256><<<(uint32_t)((t / 4 + 255) / 256), 256>>>(g.iq, t); });
        static const uint32_t NSs[] = {2, 3, 4, 6, 13};
        for (uint32_t NS : NSs) {
            char nm[64];
            g.p = NS;
            snprintf(nm, sizeof nm, "ddsbal_%u", NS);
            report(nm, [](void *) { ddsbal_k<<<dim3(g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
        }
        (void)tiles;
    }
    const uint32_t chunks = (g.ns + 32767) / 32768;
    {
        const uint64_t tot = (uint64_t)g.nch * g.ns;
        report("fill1_64", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fill1_k<64><<<(uint32_t)((t / 4 + 63) / 64), 64>>>(g.iq, t); });
        report("fill1_128", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fill1_k<128><<<(uint32_t)((t / 4 + 127) / 128), 128>>>(g.iq, t); });
        report("fill1_256", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fill1_k<256><<<(uint32_t)((t / 4 + 255) / 256), 256>>>(g.iq, t); });
        report("fill1_512", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fill1_k<512><<<(uint32_t)((t / 4 + 511) / 512), 512>>>(g.iq, t); });
        report("fillU_2", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fillU_k<2><<<(uint32_t)((t + 2047) / 2048), BLOCK>>>(g.iq, t); });
        report("fillU_4", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fillU_k<4><<<(uint32_t)((t + 4095) / 4096), BLOCK>>>(g.iq, t); });
        report("fillU_8", [](void *) { const uint64_t t = (uint64_t)g.nch * g.ns; fillU_k<8><<<(uint32_t)((t + 8191) / 8192), BLOCK>>>(g.iq, t); });
        (void)tot;
    }
    report("chunk_contig", [](void *) { chunk_k<false, false><<<dim3((g.ns + 32767) / 32768, g.nch), BLOCK>>>(g.iq, g.ns, 32768); });
    report("chunk_rows", [](void *) { chunk_k<false, true><<<dim3((g.ns + 32767) / 32768, g.nch), BLOCK>>>(g.iq, g.ns, 32768); });
    report("chunk_contig_nt", [](void *) { chunk_k<true, false><<<dim3((g.ns + 32767) / 32768, g.nch), BLOCK>>>(g.iq, g.ns, 32768); });
    report("chunk_rows_nt", [](void *) { chunk_k<true, true><<<dim3((g.ns + 32767) / 32768, g.nch), BLOCK>>>(g.iq, g.ns, 32768); });
    static const uint32_t Gs[] = {7, 16, 32, 64, 103};
    for (uint32_t G : Gs) {
        char nm[64];
        g.p = G;
        snprintf(nm, sizeof nm, "ileave_%u", G);
        report(nm, [](void *) { ileave_k<false><<<dim3(g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
        snprintf(nm, sizeof nm, "ileave_%u_nt", G);
        report(nm, [](void *) { ileave_k<true><<<dim3(g.p, g.nch), BLOCK>>>(g.iq, g.ns, g.p); });
    }
    static const uint32_t Ts[] = {2048, 8192, 32768};
    for (uint32_t T : Ts) {
        char nm[64];
        g.p = T;
        snprintf(nm, sizeof nm, "fill_%u", T);
        report(nm, [](void *) {
            const uint64_t tot = (uint64_t)g.nch * g.ns;
            fill_k<false><<<(uint32_t)((tot + g.p - 1) / g.p), BLOCK>>>(g.iq, tot, g.p);
        });
        snprintf(nm, sizeof nm, "fill_%u_nt", T);
        report(nm, [](void *) {
            const uint64_t tot = (uint64_t)g.nch * g.ns;
            fill_k<true><<<(uint32_t)((tot + g.p - 1) / g.p), BLOCK>>>(g.iq, tot, g.p);
        });
    }
    static const uint32_t Ps[] = {1024, 2048, 4096};
    for (uint32_t P : Ps) {
        char nm[64];
        g.p = P;
        snprintf(nm, sizeof nm, "persist_%u", P);
        report(nm, [](void *) { persist_k<false><<<g.p, BLOCK>>>(g.iq, (uint64_t)g.nch * g.ns); });
        snprintf(nm, sizeof nm, "persist_%u_nt", P);
        report(nm, [](void *) { persist_k<true><<<g.p, BLOCK>>>(g.iq, (uint64_t)g.nch * g.ns); });
    }
    (void)chunks;
    hipFree(g.iq);
    return 0;
}
