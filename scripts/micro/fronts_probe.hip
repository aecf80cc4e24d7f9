// Store-front microbenchmark for the interpreter's slot-major outputs: every
// wave writes F rows of 1 KiB (64 lanes x 16 B), row f at f * S bytes past row
// 0, as the straight kernel writes event slot f of its 64 lanes (S = n_lanes *
// 16 B = 2^27 at config 2), plus optionally a 2-KiB summary block.  Question:
// do power-of-two row strides (fronts that map to the same HBM channel / bank)
// cost bandwidth, and how does a wave's store count change the rate?
#include <hip/hip_runtime.h>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) fronts_k(uint32_t *base, uint64_t stride_words, uint32_t F, uint32_t *summ)
{
    const uint64_t lane = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const u32x4 w = {(uint32_t)lane, 1u, 2u, 3u};
    for (uint32_t f = 0; f < F; f++)
        *reinterpret_cast<u32x4 *>(base + f * stride_words + lane * 4) = w;
    if (summ) {
        *reinterpret_cast<u32x4 *>(summ + lane * 8) = w;
        *reinterpret_cast<u32x4 *>(summ + lane * 8 + 4) = w;
    }
}

int main()
{
    const uint64_t n_lanes = 8u << 20;                     // config 2: 10^6 shots x 8 cores ~ 2^23
    const uint64_t pad_max = 64 * 1024;                    // words
    uint32_t *buf, *summ;
    const uint64_t words = 6 * (n_lanes * 4 + pad_max);
    if (hipMalloc(&buf, words * 4) != hipSuccess || hipMalloc(&summ, n_lanes * 32) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const uint64_t pads[] = {0, 64, 256, 1024, 4096, 16384};   // words added to the 2^25-word row stride
    for (int with_s = 0; with_s < 2; with_s++)
    for (uint32_t F : {1u, 2u, 5u}) {
        for (uint64_t pad : pads) {
            const uint64_t stride = n_lanes * 4 + pad;
            auto launch = [&]() { fronts_k<<<(uint32_t)(n_lanes / 256), 256>>>(buf, stride, F, with_s ? summ : nullptr); };
            launch();
            hipDeviceSynchronize();
            float best = 1e30f;
            for (int r = 0; r < 10; r++) {
                hipEventRecord(e0);
                launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            const double bytes = (double)n_lanes * 16 * F + (with_s ? n_lanes * 32.0 : 0.0);
            printf("{\"F\": %u, \"summary\": %d, \"pad_words\": %llu, \"ms\": %.4f, \"TB_s\": %.3f}\n", F, with_s,
                   (unsigned long long)pad, best, bytes / (best * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return 0;
}
