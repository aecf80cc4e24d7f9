// Store-shape probe for config 2's outputs (8M lanes: a 32-B summary, five
// 16-B event rows and one 8-B measurement row per lane, slot-major rows,
// one workgroup per 256 lanes), with the distance between the rows varied.
// Question: is the 0.158-0.165 ms store floor of that shape (against 0.140 for
// a fill of the same 0.96 GB, profiles/r05_config2_store_shape.jsonl) set by
// the rows' address distance (DRAM bank / channel aliasing of the seven
// concurrent row streams, n_lanes * 16 = 128,000,000 B apart), so that a row
// pitch parameter in the ABI would buy it back?
//
//   fill         : WG b writes 4-KiB block b of 0.96 GB
//   pitch<P>     : the config-2 shape, every row P lanes long (P >= n): event
//                  row k at k * P * 16, summary / measurement regions after
//   pitch<P>_ev  : events only (5 rows), same pitch
//   rowsN        : N rows of 16 B per lane only, pitch n (N = 1 is a fill)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 256;
constexpr uint64_t N = 8000000ull;

__device__ __forceinline__ void st16(uint32_t *p, uint32_t v)
{
    const u32x4 w = {v, v + 1, v + 2, v + 3};
    *reinterpret_cast<u32x4 *>(p) = w;
}

__global__ void __launch_bounds__(BLOCK) fill_k(uint32_t *base, uint64_t words)
{
    const uint64_t j = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) * 4;
    if (j + 3 < words) st16(base + j, (uint32_t)j);
}

// rows: event rows at k * P lanes; summary region (P lanes x 32 B) and the
// measurement row (P lanes x 8 B) after them
__global__ void __launch_bounds__(BLOCK) cfg2_k(uint32_t *base, uint64_t P, uint32_t n_rows, uint32_t with_sm)
{
    const uint64_t lane = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (lane >= N) return;
    uint32_t *ev = base, *summ = base + 4 * P * n_rows, *meas = summ + 8 * P;
    const uint32_t v = (uint32_t)lane;
    for (uint32_t k = 0; k < n_rows; k++) st16(ev + (k * P + lane) * 4, v + k);
    if (with_sm) {
        *reinterpret_cast<uint2 *>(meas + lane * 2) = make_uint2(v, 1);
        st16(summ + lane * 8, v);
        st16(summ + lane * 8 + 4, v);
    }
}

static void bench(const char *name, uint64_t bytes, void (*launch)(void *), void *arg)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch(arg);
    hipDeviceSynchronize();
    std::vector<float> t;
    for (int r = 0; r < 15; r++) {
        hipEventRecord(e0);
        launch(arg);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("{\"variant\": \"%s\", \"bytes\": %llu, \"ms_min\": %.4f, \"ms_med\": %.4f, \"TB_s_med\": %.3f}\n", name,
           (unsigned long long)bytes, t[0], t[t.size() / 2], bytes / (t[t.size() / 2] * 1e-3) / 1e12);
    fflush(stdout);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

struct Arg {
    uint32_t *base;
    uint64_t P;
    uint32_t rows, sm;
};

int main()
{
    uint32_t *base;
    const uint64_t max_bytes = 1400ull << 20;
    if (hipMalloc(&base, max_bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    static Arg a;
    a.base = base;
    const uint32_t grid = (uint32_t)((N + BLOCK - 1) / BLOCK);
    for (int rep = 0; rep < 2; rep++) {
        bench("fill_0.96GB", N * 120, [](void *) { fill_k<<<(uint32_t)(N * 120 / 16 / BLOCK), BLOCK>>>(a.base, N * 30); },
              nullptr);
        // pads in lanes: 0, 4 KiB, 64 KiB, 1 MiB, 2 MiB + 4 KiB, 8 MiB + 1 KiB, 32 MiB
        for (uint64_t pad : {0ull, 256ull, 4096ull, 65536ull, 131328ull, 524352ull, 2097152ull}) {
            a.P = N + pad;
            if ((a.P * 120) > max_bytes) continue;
            char nm[64];
            a.rows = 5;
            a.sm = 1;
            snprintf(nm, sizeof nm, "pitch_pad%llu", (unsigned long long)pad);
            bench(nm, N * 120, [](void *) { cfg2_k<<<(uint32_t)((N + BLOCK - 1) / BLOCK), BLOCK>>>(a.base, a.P, a.rows, a.sm); },
                  nullptr);
            a.sm = 0;
            snprintf(nm, sizeof nm, "pitch_pad%llu_ev", (unsigned long long)pad);
            bench(nm, N * 80, [](void *) { cfg2_k<<<(uint32_t)((N + BLOCK - 1) / BLOCK), BLOCK>>>(a.base, a.P, a.rows, a.sm); },
                  nullptr);
        }
        for (uint32_t rows : {1u, 2u, 3u, 5u, 7u}) {
            a.P = N;
            a.rows = rows;
            a.sm = 0;
            char nm[64];
            snprintf(nm, sizeof nm, "rows%u", rows);
            bench(nm, N * 16 * rows, [](void *) { cfg2_k<<<(uint32_t)((N + BLOCK - 1) / BLOCK), BLOCK>>>(a.base, a.P, a.rows, a.sm); },
                  nullptr);
        }
    }
    (void)grid;
    hipFree(base);
    return 0;
}
