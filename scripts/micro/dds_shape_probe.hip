// Store-shape probe for the config-5 DDS output (2048 channels x 209952
// samples x 4 B = 1.72 GB, [channel][sample]).  Every variant writes the same
// bytes; only which workgroup writes which 16-B piece, and when, changes.
// Question: which channel-bound shape (a workgroup owns ONE channel, so it
// can stage that channel's tables once) stores as fast as the torch fill?
//
//   fill     : WG b writes 4-KiB block b (one 16-B store per thread)
//   cur      : the round-3 dds_tile_kernel shape: 13 stripes x 16 tiles per
//              channel, channel-local 1024-sample tiles round-robin over the
//              stripes, wave w of a stripe takes its tiles w, w + 4, ...
//   cx<K><W|G>[s] : WG (ch, k, r), linear id (ch * K + k) * 8 + r, so that
//              WGs dealt round-robin over the 8 XCDs put residue r on one XCD;
//              it writes the GLOBAL 4-KiB blocks B of its channel with
//              B % 8 == r, the i-th such block when i % K == k.  W: wave w
//              takes its list entries w, w + 4, ... (a wave = one block);
//              G: the workgroup writes each block together (wave w = row w).
//              s: residue (r + 5 ch) % 8 instead -- the same shape with every
//              XCD writing every residue (the XCD-affinity control).
//   cc<K>W   : like cx<K>W but the K workgroups of (ch, r) take contiguous
//              runs of the residue list instead of interleaving
// The channel-boundary blocks are written partly by each channel's WG
// (16-B granular masks), as a channel-bound kernel would.
// Set "w" (round 5): one tile per wave in address order (wave_tile_k).
// Also records s_getreg(XCC_ID) per WG of one launch to check that WG g and
// g + 8 share an XCD (MI355X_MICROARCH.md, workgroup dispatch).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 256;
constexpr uint32_t NCH = 2048, NS = 209952;

__device__ __forceinline__ void st16(uint32_t *p, uint32_t v)
{
    const u32x4 w = {v, v + 1, v + 2, v + 3};
    *reinterpret_cast<u32x4 *>(p) = w;
}

__device__ __forceinline__ uint32_t xcc_id()
{
    // HW_REG_XCC_ID (id 20), bits [3:0]
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
}

__global__ void __launch_bounds__(BLOCK) fill_k(uint32_t *iq, uint64_t total)
{
    const uint64_t j = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) * 4;
    if (j + 3 < total) st16(iq + j, (uint32_t)j);
}

__global__ void __launch_bounds__(BLOCK) cur_k(uint32_t *iq, uint32_t stripes, uint32_t *xcc)
{
    const uint32_t ch = blockIdx.x / stripes, s = blockIdx.x % stripes;
    const uint32_t tiles = (NS + 1023) / 1024;
    uint32_t *out = iq + (uint64_t)ch * NS;
    const uint32_t n_t = (tiles - s + stripes - 1) / stripes;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    if (xcc && threadIdx.x == 0) xcc[blockIdx.x] = xcc_id();
    for (uint32_t i = wv; i < n_t; i += 4) {
        const uint32_t t = s + i * stripes;
        for (int r = 0; r < 4; r++) {
            const uint32_t j = t * 1024 + 4 * (64 * r + ln);
            if (j + 3 < NS) st16(out + j, j);
        }
    }
}

// (set "w") the stripes shape with channel rows PITCH samples apart (NS
// written per row): pitch 216 Ki samples puts every row on a 4-KiB boundary
__global__ void __launch_bounds__(BLOCK) curP_k(uint32_t *iq, uint32_t stripes, uint32_t pitch)
{
    const uint32_t ch = blockIdx.x / stripes, s = blockIdx.x % stripes;
    const uint32_t tiles = (NS + 1023) / 1024;
    uint32_t *out = iq + (uint64_t)ch * pitch;
    const uint32_t n_t = (tiles - s + stripes - 1) / stripes;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t i = wv; i < n_t; i += 4) {
        const uint32_t t = s + i * stripes;
        for (int r = 0; r < 4; r++) {
            const uint32_t j = t * 1024 + 4 * (64 * r + ln);
            if (j + 3 < NS) st16(out + j, j);
        }
    }
}

// (round 4, set "b") the stripes shape with the whole workgroup on each tile
// (thread t writes 16 B at 4 t of the tile) instead of a wave per tile
__global__ void __launch_bounds__(BLOCK) curG_k(uint32_t *iq, uint32_t stripes)
{
    const uint32_t ch = blockIdx.x / stripes, s = blockIdx.x % stripes;
    const uint32_t tiles = (NS + 1023) / 1024;
    uint32_t *out = iq + (uint64_t)ch * NS;
    const uint32_t n_t = (tiles - s + stripes - 1) / stripes;
    for (uint32_t i = 0; i < n_t; i++) {
        const uint32_t j = (s + i * stripes) * 1024 + 4 * threadIdx.x;
        if (j + 3 < NS) st16(out + j, j);
    }
}

// (set "b") the stripes shape with each workgroup starting its tile loop at a
// workgroup-dependent rotation (ROT: rot = (g * 7) mod n_t; 1: g mod n_t)
__global__ void __launch_bounds__(BLOCK) curR_k(uint32_t *iq, uint32_t stripes, uint32_t mode)
{
    const uint32_t ch = blockIdx.x / stripes, s = blockIdx.x % stripes;
    const uint32_t tiles = (NS + 1023) / 1024;
    uint32_t *out = iq + (uint64_t)ch * NS;
    const uint32_t n_t = (tiles - s + stripes - 1) / stripes;
    const uint32_t rot = mode == 0 ? (blockIdx.x * 7u) % n_t : blockIdx.x % n_t;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t i0 = wv; i0 < n_t; i0 += 4) {
        const uint32_t i = (i0 + rot) % n_t;
        const uint32_t t = s + i * stripes;
        for (int r = 0; r < 4; r++) {
            const uint32_t j = t * 1024 + 4 * (64 * r + ln);
            if (j + 3 < NS) st16(out + j, j);
        }
    }
}

// (set "b") stripe items (ch, s) = item / 13, item % 13 (the cur shape's
// workgroups) taken M at a time by one workgroup: WG g does items
// g M .. g M + M - 1 (curM), or -- persistent, P workgroups -- items g, g + P, ...
__global__ void __launch_bounds__(BLOCK) curM_k(uint32_t *iq, uint32_t M, uint32_t P)
{
    const uint32_t stripes = 13, tiles = (NS + 1023) / 1024, n_items = NCH * stripes;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    const uint32_t i_begin = P ? blockIdx.x : blockIdx.x * M, i_step = P ? P : 1u;
    const uint32_t i_end = P ? n_items : min(n_items, blockIdx.x * M + M);
    for (uint32_t it = i_begin; it < i_end; it += i_step) {
        const uint32_t ch = it / stripes, s = it % stripes;
        uint32_t *out = iq + (uint64_t)ch * NS;
        const uint32_t n_t = (tiles - s + stripes - 1) / stripes;
        for (uint32_t i = wv; i < n_t; i += 4) {
            const uint32_t t = s + i * stripes;
            for (int r = 0; r < 4; r++) {
                const uint32_t j = t * 1024 + 4 * (64 * r + ln);
                if (j + 3 < NS) st16(out + j, j);
            }
        }
    }
}

// (set "b") long-lived fill, rotated: WG b writes its N blocks starting at (b * 7) mod N
__global__ void __launch_bounds__(BLOCK) blkR_k(uint32_t *iq, uint64_t total, uint32_t N)
{
    const uint64_t b0 = (uint64_t)blockIdx.x * N;
    const uint32_t rot = (blockIdx.x * 7u) % N;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    for (uint32_t i0 = wv; i0 < N; i0 += 4) {
        const uint32_t i = (i0 + rot) % N;
        for (int q = 0; q < 4; q++) {
            const uint64_t j = (b0 + i) * 1024 + 4 * (64 * q + ln);
            if (j + 3 < total) st16(iq + j, (uint32_t)j);
        }
    }
}

// (set "b") long-lived fill: WG b writes N consecutive global 4-KiB blocks;
// WAVE: wave w takes blocks w, w + 4, ... (4 x 1-KiB stores each), else the
// whole workgroup writes each block in turn
template <bool WAVE>
__global__ void __launch_bounds__(BLOCK) blk_k(uint32_t *iq, uint64_t total, uint32_t N)
{
    const uint64_t b0 = (uint64_t)blockIdx.x * N;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    if (WAVE) {
        for (uint32_t i = wv; i < N; i += 4)
            for (int q = 0; q < 4; q++) {
                const uint64_t j = (b0 + i) * 1024 + 4 * (64 * q + ln);
                if (j + 3 < total) st16(iq + j, (uint32_t)j);
            }
    } else {
        for (uint32_t i = 0; i < N; i++) {
            const uint64_t j = (b0 + i) * 1024 + 4 * threadIdx.x;
            if (j + 3 < total) st16(iq + j, (uint32_t)j);
        }
    }
}

// WG (ch, k, r): global blocks B of channel ch with B % 8 == res, list index i
// (B = base8 + 8 i + res) with i % K == k (INTERLEAVE) or i in run k (contiguous)
template <bool WAVE, bool INTERLEAVE>
__global__ void __launch_bounds__(BLOCK) cx_k(uint32_t *iq, uint32_t K, uint32_t scramble, uint32_t *xcc)
{
    const uint32_t g = blockIdx.x;
    const uint32_t r = g & 7u, k = (g >> 3) % K, ch = (g >> 3) / K;
    const uint32_t res = scramble ? (r + 5 * ch) & 7u : r;
    if (xcc && threadIdx.x == 0) xcc[g] = xcc_id();
    const uint64_t j_lo = (uint64_t)ch * NS, j_hi = j_lo + NS;       // global samples of the channel
    const uint64_t b_lo = j_lo / 1024, b_hi = (j_hi - 1) / 1024;     // its global blocks (inclusive)
    const uint64_t base8 = b_lo & ~7ull;
    const uint32_t n_list = (uint32_t)((b_hi - base8 - res) / 8 + 1); // i = 0 .. n_list-1 (B <= b_hi)
    uint32_t i0, di, i1;
    if (INTERLEAVE) { i0 = k; di = K; i1 = n_list; }
    else { const uint32_t per = (n_list + K - 1) / K; i0 = k * per; di = 1; i1 = min(n_list, i0 + per); }
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    if (WAVE) {
        for (uint32_t i = i0 + wv * di; i < i1; i += 4 * di) {
            const uint64_t B = base8 + 8ull * i + res;
            if (B < b_lo) continue;
            for (int q = 0; q < 4; q++) {
                const uint64_t j = B * 1024 + 4 * (64 * q + ln);
                if (j >= j_lo && j < j_hi) st16(iq + j, (uint32_t)j);
            }
        }
    } else {
        for (uint32_t i = i0; i < i1; i += di) {
            const uint64_t B = base8 + 8ull * i + res;
            if (B < b_lo) continue;
            const uint64_t j = B * 1024 + 4 * threadIdx.x;
            if (j >= j_lo && j < j_hi) st16(iq + j, (uint32_t)j);
        }
    }
}

// (set "w") one channel-local 1024-sample tile per wave: WG (ch, g) of W
// waves takes tiles g W .. g W + W - 1 of channel ch, channel-major (so the
// grid writes the buffer in address order, like the fill); each wave sleeps
// SLEEP x 64 clocks before its 4 x 1-KiB stores (a stand-in for its compute)
template <int W, int SLEEP>
__global__ void __launch_bounds__(64 * W) wave_tile_k(uint32_t *iq, uint32_t per_ch)
{
    const uint32_t tiles = (NS + 1023) / 1024;
    const uint32_t ch = blockIdx.x / per_ch, g = blockIdx.x % per_ch;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    const uint32_t t = g * W + wv;
    if (t >= tiles) return;
    for (int k = 0; k < SLEEP; k++) __builtin_amdgcn_s_sleep(1);
    uint32_t *out = iq + (uint64_t)ch * NS;
    for (int q = 0; q < 4; q++) {
        const uint32_t j = t * 1024 + 4 * (64 * q + ln);
        if (j + 3 < NS) st16(out + j, j);
    }
}

// (set "w") channel-contiguous stripes: stripe s of a channel takes the
// channel's tiles [s T, s T + T) (T = ceil(tiles / S)), wave w of the
// workgroup its tiles w, w + 4, ... (4 x 1-KiB stores each)
__global__ void __launch_bounds__(BLOCK) contig_k(uint32_t *iq, uint32_t S)
{
    const uint32_t tiles = (NS + 1023) / 1024, T = (tiles + S - 1) / S;
    const uint32_t ch = blockIdx.x / S, st = blockIdx.x % S;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    uint32_t *out = iq + (uint64_t)ch * NS;
    for (uint32_t i = wv; i < T; i += 4) {
        const uint32_t t = st * T + i;
        if (t >= tiles) break;
        for (int q = 0; q < 4; q++) {
            const uint32_t j = t * 1024 + 4 * (64 * q + ln);
            if (j + 3 < NS) st16(out + j, j);
        }
    }
}

// (set "w") channel-local tiles in global (channel-major) order, written by
// whole workgroups (thread t: 16 B at 4 t of the tile):
//   gtile   : workgroup b writes tile b and exits (the fill, channel-local)
//   gstride : G persistent workgroups, workgroup g takes tiles g, g + G, ...
//             (at any time the grid writes a window of ~G tiles)
//   gstrideW: the same with each WAVE on its own tile (window ~4 G tiles)
__global__ void __launch_bounds__(BLOCK) gtile_k(uint32_t *iq, uint32_t n_tiles, uint32_t G, uint32_t wave_mode,
                                                uint32_t pitch = NS)
{
    const uint32_t tiles = (NS + 1023) / 1024;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    if (!wave_mode) {
        for (uint32_t t = blockIdx.x; t < n_tiles; t += G) {
            const uint32_t ch = t / tiles, c = t - ch * tiles;
            const uint32_t j = c * 1024 + 4 * threadIdx.x;
            if (j + 3 < NS) st16(iq + (uint64_t)ch * pitch + j, j);
        }
    } else {
        for (uint32_t t = 4 * blockIdx.x + wv; t < n_tiles; t += 4 * G) {
            const uint32_t ch = t / tiles, c = t - ch * tiles;
            for (int q = 0; q < 4; q++) {
                const uint32_t j = c * 1024 + 4 * (64 * q + ln);
                if (j + 3 < NS) st16(iq + (uint64_t)ch * pitch + j, j);
            }
        }
    }
}

// (set "w") persistent fill: G workgroups, workgroup g writes global 4-KiB
// blocks g, g + G, ... one 16-B store per thread per block (the fill's
// address stream from long-lived workgroups); SLEEP x 64 clocks per block
template <int SLEEP>
__global__ void __launch_bounds__(BLOCK) gblk_k(uint32_t *iq, uint64_t total, uint32_t G)
{
    const uint64_t nblk = total / 1024;
    for (uint64_t b = blockIdx.x; b < nblk; b += G) {
        for (int k = 0; k < SLEEP; k++) __builtin_amdgcn_s_sleep(1);
        const uint64_t j = b * 1024 + 4 * threadIdx.x;
        st16(iq + j, (uint32_t)j);
    }
}

// (set "c") config 2's store shape (0.96 GB: per lane 32-B summary, 5
// event records of 16 B in slot-major rows, one 8-B measurement row), 8M
// lanes, one workgroup per 256 lanes; residency capped by dynamic LDS
__global__ void __launch_bounds__(BLOCK) cfg2_k(uint32_t *base, uint32_t order)
{
    extern __shared__ uint32_t s_pad[];
    const uint64_t n = 8000000ull, lane = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (lane >= n) return;
    if (threadIdx.x == 1023) s_pad[0] = 0;              // (never: keeps the LDS allocation)
    uint32_t *summ = base, *ev = base + n * 8, *meas = ev + n * 4 * 5;
    const uint32_t v = (uint32_t)lane;
    if (order == 0) {
        for (int k = 0; k < 5; k++) st16(ev + ((uint64_t)k * n + lane) * 4, v + k);
        *reinterpret_cast<uint2 *>(meas + lane * 2) = make_uint2(v, 1);
        st16(summ + lane * 8, v); st16(summ + lane * 8 + 4, v);
    } else {                                            // one stream at a time per workgroup: rows in turn
        st16(summ + lane * 8, v); st16(summ + lane * 8 + 4, v);
        __syncthreads();
        for (int k = 0; k < 5; k++) { st16(ev + ((uint64_t)k * n + lane) * 4, v + k); __syncthreads(); }
        *reinterpret_cast<uint2 *>(meas + lane * 2) = make_uint2(v, 1);
    }
}

// the fill with 64-thread workgroups (one 16-B store per thread)
__global__ void __launch_bounds__(64) fill64_k(uint32_t *iq, uint64_t total)
{
    const uint64_t j = ((uint64_t)blockIdx.x * 64 + threadIdx.x) * 4;
    if (j + 3 < total) st16(iq + j, (uint32_t)j);
}

static uint32_t *g_iq;
static uint32_t g_K, g_scr;

template <typename F>
static void bench(const char *name, F launch)
{
    const uint64_t bytes = (uint64_t)NCH * NS * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch();
    hipDeviceSynchronize();
    std::vector<float> t;
    for (int r = 0; r < 15; r++) {
        hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("{\"variant\": \"%s\", \"ms_min\": %.4f, \"ms_med\": %.4f, \"TB_s_min\": %.3f, \"TB_s_med\": %.3f}\n", name,
           t[0], t[t.size() / 2], bytes / (t[0] * 1e-3) / 1e12, bytes / (t[t.size() / 2] * 1e-3) / 1e12);
    fflush(stdout);
    hipEventDestroy(e0); hipEventDestroy(e1);
}

// one launch with XCC ids recorded: fraction of WGs whose XCC == (g + c) % 8
static void check_xcc(uint32_t n_wg, void (*launch)(uint32_t *), const char *name)
{
    uint32_t *d;
    hipMalloc(&d, n_wg * 4);
    launch(d);
    hipDeviceSynchronize();
    std::vector<uint32_t> h(n_wg);
    hipMemcpy(h.data(), d, n_wg * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    const uint32_t c = (h[0] + 8 - 0) & 7u;
    uint32_t ok = 0;
    for (uint32_t g = 0; g < n_wg; g++) ok += h[g] == ((g + c) & 7u);
    printf("{\"xcc_check\": \"%s\", \"wgs\": %u, \"xcc_of_wg0\": %u, \"frac_round_robin\": %.5f}\n", name, n_wg, h[0],
           (double)ok / n_wg);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const uint64_t total = (uint64_t)NCH * NS, bytes = total * 4;
    if (hipMalloc(&g_iq, (uint64_t)NCH * 210944u * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    if (argc > 1 && argv[1][0] == 'c') {                 // round-5 set: config 2's store shape
        const uint64_t bytes2 = 8000000ull * 120;
        for (int rep = 0; rep < 2; rep++) {
            bench("fill_0.96GB", [&] { fill_k<<<(uint32_t)(bytes2 / 16 / BLOCK), BLOCK>>>(g_iq, bytes2 / 4); });
            for (uint32_t lds : {0u, 20u * 1024, 40u * 1024, 60u * 1024}) {
                for (uint32_t order : {0u, 1u}) {
                    g_K = lds; g_scr = order;
                    char nm[48];
                    snprintf(nm, sizeof nm, "cfg2_lds%uK_o%u", lds / 1024, order);
                    bench(nm, [&] { cfg2_k<<<8000000 / BLOCK, BLOCK, g_K>>>(g_iq, g_scr); });
                }
            }
        }
        hipFree(g_iq);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'w') {                 // round-5 set: one tile per wave, address order
        const uint32_t tiles = (NS + 1023) / 1024;
        for (int rep = 0; rep < 2; rep++) {
            bench("fill", [&] { fill_k<<<(uint32_t)(total / 4 / BLOCK), BLOCK>>>(g_iq, total); });
            bench("fill64", [&] { fill64_k<<<(uint32_t)(total / 4 / 64), 64>>>(g_iq, total); });
            bench("cur", [&] { cur_k<<<NCH * 13, BLOCK>>>(g_iq, 13, nullptr); });
            bench("wave1", [&] { wave_tile_k<1, 0><<<NCH * tiles, 64>>>(g_iq, tiles); });
            bench("wave4", [&] { wave_tile_k<4, 0><<<NCH * ((tiles + 3) / 4), 256>>>(g_iq, (tiles + 3) / 4); });
            bench("wave1_s16", [&] { wave_tile_k<1, 16><<<NCH * tiles, 64>>>(g_iq, tiles); });
            bench("wave1_s48", [&] { wave_tile_k<1, 48><<<NCH * tiles, 64>>>(g_iq, tiles); });
            bench("wave4_s16", [&] { wave_tile_k<4, 16><<<NCH * ((tiles + 3) / 4), 256>>>(g_iq, (tiles + 3) / 4); });
            bench("wave4_s48", [&] { wave_tile_k<4, 48><<<NCH * ((tiles + 3) / 4), 256>>>(g_iq, (tiles + 3) / 4); });
            for (uint32_t G : {1024u, 1792u, 2048u, 4096u, 8192u}) {
                g_K = G;
                char nm[32];
                snprintf(nm, sizeof nm, "gblk%u", G);
                bench(nm, [&] { gblk_k<0><<<g_K, BLOCK>>>(g_iq, total, g_K); });
                snprintf(nm, sizeof nm, "gblk%u_s8", G);
                bench(nm, [&] { gblk_k<8><<<g_K, BLOCK>>>(g_iq, total, g_K); });
            }
            {
                const uint32_t nt = NCH * tiles;
                bench("gtile", [&] { gtile_k<<<nt, BLOCK>>>(g_iq, nt, nt, 0); });
                for (uint32_t P : {210176u, 210944u, 210048u}) {   // 1-KiB, 4-KiB, 512-B aligned rows
                    g_K = P;
                    char nm[40];
                    snprintf(nm, sizeof nm, "gtile_p%u", P);
                    bench(nm, [&] { gtile_k<<<nt, BLOCK>>>(g_iq, nt, nt, 0, g_K); });
                    snprintf(nm, sizeof nm, "gstrideW2048_p%u", P);
                    bench(nm, [&] { gtile_k<<<2048, BLOCK>>>(g_iq, nt, 2048, 1, g_K); });
                    snprintf(nm, sizeof nm, "curP_p%u", P);
                    bench(nm, [&] { curP_k<<<NCH * 13, BLOCK>>>(g_iq, 13, g_K); });
                }
                for (uint32_t G : {1024u, 1792u, 2048u, 4096u}) {
                    g_K = G;
                    char nm[32];
                    snprintf(nm, sizeof nm, "gstride%u", G);
                    bench(nm, [&] { gtile_k<<<g_K, BLOCK>>>(g_iq, nt, g_K, 0); });
                    snprintf(nm, sizeof nm, "gstrideW%u", G);
                    bench(nm, [&] { gtile_k<<<g_K, BLOCK>>>(g_iq, nt, g_K, 1); });
                }
            }
            bench("curP_ns", [&] { curP_k<<<NCH * 13, BLOCK>>>(g_iq, 13, NS); });
            bench("curP_210944", [&] { curP_k<<<NCH * 13, BLOCK>>>(g_iq, 13, 210944u); });
            bench("curP_209984", [&] { curP_k<<<NCH * 13, BLOCK>>>(g_iq, 13, 209984u); });
            bench("curP_210048", [&] { curP_k<<<NCH * 13, BLOCK>>>(g_iq, 13, 210048u); });
            for (uint32_t S : {1u, 2u, 4u, 7u, 13u, 26u}) {
                g_K = S;
                char nm[32];
                snprintf(nm, sizeof nm, "contig%u", S);
                bench(nm, [&] { contig_k<<<NCH * g_K, BLOCK>>>(g_iq, g_K); });
            }
        }
        hipFree(g_iq);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'b') {                 // round-4 set: per-tile granularity, WG lifetime
        const uint32_t nblk = (uint32_t)((total + 1023) / 1024);
        for (int rep = 0; rep < 2; rep++) {
            bench("fill", [&] { fill_k<<<(uint32_t)(total / 4 / BLOCK), BLOCK>>>(g_iq, total); });
            bench("cur", [&] { cur_k<<<NCH * 13, BLOCK>>>(g_iq, 13, nullptr); });
            bench("curG", [&] { curG_k<<<NCH * 13, BLOCK>>>(g_iq, 13); });
            bench("cur2", [&] { curM_k<<<(NCH * 13 + 1) / 2, BLOCK>>>(g_iq, 2, 0); });
            bench("cur4", [&] { curM_k<<<(NCH * 13 + 3) / 4, BLOCK>>>(g_iq, 4, 0); });
            bench("curP2048", [&] { curM_k<<<2048, BLOCK>>>(g_iq, 0, 2048); });
            bench("curP4096", [&] { curM_k<<<4096, BLOCK>>>(g_iq, 0, 4096); });
            bench("curR7", [&] { curR_k<<<NCH * 13, BLOCK>>>(g_iq, 13, 0); });
            bench("curR1", [&] { curR_k<<<NCH * 13, BLOCK>>>(g_iq, 13, 1); });
            bench("blk16R", [&] { blkR_k<<<(nblk + 15) / 16, BLOCK>>>(g_iq, total, 16); });
            for (uint32_t N : {2u, 4u, 8u, 16u, 32u, 64u, 128u, 256u}) {
                g_K = N;
                char nm[32];
                snprintf(nm, sizeof nm, "blk%uW", N);
                bench(nm, [&] { blk_k<true><<<(nblk + g_K - 1) / g_K, BLOCK>>>(g_iq, total, g_K); });
                snprintf(nm, sizeof nm, "blk%uG", N);
                bench(nm, [&] { blk_k<false><<<(nblk + g_K - 1) / g_K, BLOCK>>>(g_iq, total, g_K); });
            }
        }
        hipFree(g_iq);
        return 0;
    }
    check_xcc(NCH * 8, [](uint32_t *x) { cx_k<true, true><<<NCH * 8, BLOCK>>>(g_iq, 1, 0, x); }, "cx1W");
    check_xcc(NCH * 13, [](uint32_t *x) { cur_k<<<NCH * 13, BLOCK>>>(g_iq, 13, x); }, "cur");
    for (int rep = 0; rep < 2; rep++) {
        bench("fill", [&] { fill_k<<<(uint32_t)(total / 4 / BLOCK), BLOCK>>>(g_iq, total); });
        bench("cur", [&] { cur_k<<<NCH * 13, BLOCK>>>(g_iq, 13, nullptr); });
        for (uint32_t K : {1u, 2u, 4u}) {
            g_K = K;
            char nm[32];
            snprintf(nm, sizeof nm, "cx%uW", K);
            bench(nm, [&] { cx_k<true, true><<<NCH * 8 * g_K, BLOCK>>>(g_iq, g_K, 0, nullptr); });
            snprintf(nm, sizeof nm, "cx%uG", K);
            bench(nm, [&] { cx_k<false, true><<<NCH * 8 * g_K, BLOCK>>>(g_iq, g_K, 0, nullptr); });
            snprintf(nm, sizeof nm, "cx%uWs", K);
            bench(nm, [&] { cx_k<true, true><<<NCH * 8 * g_K, BLOCK>>>(g_iq, g_K, 1, nullptr); });
            if (K > 1) {
                snprintf(nm, sizeof nm, "cc%uW", K);
                bench(nm, [&] { cx_k<true, false><<<NCH * 8 * g_K, BLOCK>>>(g_iq, g_K, 0, nullptr); });
            }
        }
    }
    hipFree(g_iq);
    return 0;
}
