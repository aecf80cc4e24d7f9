// VALU issue-rate microbenchmark (re-measure the int32 VALU peak).
// Each lane runs CH independent add/xor chains for ITERS iterations; the VALU
// instruction count per wave is read from the disassembly (printed by the
// driver script) and divided by the hipEvent-timed kernel duration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int CH>
__global__ void __launch_bounds__(256) valu_kernel(uint32_t *out, uint32_t iters, uint32_t k) {
    uint32_t a[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x * (c + 1) + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            a[c] = (a[c] + k) ^ (a[c] >> 3);
            a[c] = (a[c] - k) ^ (a[c] << 5);
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
static void run(const char *name, uint32_t blocks, uint32_t iters, uint32_t *d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    valu_kernel<CH><<<blocks, 256>>>(d, iters, 7u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        valu_kernel<CH><<<blocks, 256>>>(d, iters, 7u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double waves = blocks * 4.0;
    // each chain step: add, shr, xor, sub, shl, xor = 6 ops (the compiler may fuse to 4: v_add, v_xad/ v_lshl_xor...)
    printf("{\"kernel\": \"%s\", \"chains\": %d, \"blocks\": %u, \"iters\": %u, \"ms\": %.4f, \"wave_iters_per_s\": %.4e}\n",
           name, CH, blocks, iters, best, waves * iters * CH / (best * 1e-3));
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 256u * 65536u * 4u);
    // 256 CU x 4 SIMD x w waves/SIMD = 256*w blocks of 4 waves
    for (int w : {1, 2, 4, 8}) {
        run<8>("ch8", 256 * w, 4096, d);
        run<2>("ch2", 256 * w, 16384, d);
        run<1>("ch1", 256 * w, 16384, d);
    }
    hipFree(d);
    return 0;
}
