// XCD-locality store probe: 4-KiB blocks (a 256-thread workgroup x 16 B) of a
// 1.72-GB buffer.  Workgroup b runs on XCD b % 8 (round-robin dispatch).
//   ident   : WG b writes block b (torch-fill shape: XCD k writes blocks = k mod 8)
//   scramble: WG b writes block b ^ ((b >> 3) & 7) (each XCD writes every residue)
//   local_T : WG b writes T blocks, all = b mod 8 (multi-store waves, XCD-aligned)
//   mixed_T : WG b writes T consecutive blocks (multi-store, every residue)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) blocks_k(uint32_t *buf, uint64_t n_blocks, uint32_t T)
{
    const uint64_t b = blockIdx.x;
    const u32x4 w = {(uint32_t)b, 1u, 2u, 3u};
    for (uint32_t j = 0; j < T; j++) {
        uint64_t blk;
        if (MODE == 0) blk = b;
        else if (MODE == 1) blk = b ^ ((b >> 3) & 7);
        else if (MODE == 2) blk = (b & 7) + 8 * ((uint64_t)j + (uint64_t)T * (b >> 3));
        else blk = b * T + j;
        if (blk < n_blocks) *reinterpret_cast<u32x4 *>(buf + blk * 1024 + threadIdx.x * 4) = w;
    }
}

int main()
{
    const uint64_t bytes = 1719926784ull, n_blocks = bytes / 4096;
    uint32_t *buf;
    if (hipMalloc(&buf, bytes + 65536) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto bench = [&](const char *name, int T, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 10; r++) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("{\"variant\": \"%s\", \"T\": %d, \"ms\": %.4f, \"TB_s\": %.3f}\n", name, T, best, n_blocks * 4096.0 / (best * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; rep++) {
        bench("ident", 1, [&] { blocks_k<0><<<(uint32_t)n_blocks, 256>>>(buf, n_blocks, 1); });
        bench("scramble", 1, [&] { blocks_k<1><<<(uint32_t)n_blocks, 256>>>(buf, n_blocks, 1); });
        for (int T : {2, 4, 16}) {
            const uint32_t g = (uint32_t)((n_blocks + T - 1) / T);
            const uint32_t gl = (uint32_t)(((n_blocks + 8 * T - 1) / (8 * T)) * 8);
            bench("local", T, [&] { blocks_k<2><<<gl, 256>>>(buf, n_blocks, T); });
            bench("mixed", T, [&] { blocks_k<3><<<g, 256>>>(buf, n_blocks, T); });
        }
    }
    return 0;
}
