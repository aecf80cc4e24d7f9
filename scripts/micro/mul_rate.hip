// Integer multiply issue rates on gfx950 (sizing the Philox measurement draw,
// lane.h philox3): wave64 instructions/s of v_add_u32, v_mul_lo_u32,
// v_mul_hi_u32 and v_mad_u64_u32 over 8 independent chains per lane at full
// occupancy.  One JSON line per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void __launch_bounds__(256) mul_kernel(uint32_t *out, uint32_t iters, uint32_t k)
{
    uint32_t a[8];
#pragma unroll
    for (int c = 0; c < 8; c++) a[c] = threadIdx.x * (c + 3) + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "s"(k));
            if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "s"(k));
            if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "s"(k));
            if constexpr (OP == 3) {
                uint64_t r;
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a[c]), "s"(k) : "vcc");
                a[c] = (uint32_t)r ^ (uint32_t)(r >> 32);
            }
            if constexpr (OP == 4) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "s"(k));
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
static void run(const char *name, uint32_t blocks, uint32_t iters, uint32_t *d)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    mul_kernel<OP><<<blocks, 256>>>(d, iters, 0x9E3779B9u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        mul_kernel<OP><<<blocks, 256>>>(d, iters, 0x9E3779B9u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double n = blocks * 4.0 * iters * 8;   // wave-instructions of the op (mad: + 1 xor each)
    printf("{\"op\": \"%s\", \"blocks\": %u, \"ms\": %.4f, \"wave_insts_per_s\": %.4e}\n", name, blocks, best,
           n / (best * 1e-3));
}

int main()
{
    uint32_t *d;
    hipMalloc(&d, 256u * 8192u * 4u);
    const uint32_t blocks = 8192, iters = 512;
    run<0>("v_add_u32", blocks, iters, d);
    run<1>("v_mul_lo_u32", blocks, iters, d);
    run<2>("v_mul_hi_u32", blocks, iters, d);
    run<3>("v_mad_u64_u32+v_xor", blocks, iters, d);
    run<4>("v_mul_u32_u24", blocks, iters, d);
    hipFree(d);
    return 0;
}
