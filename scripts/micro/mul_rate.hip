// mul_rate.hip -- throughput of the Philox round's 32x32 -> 64-bit products on
// gfx950: v_mul_hi_u32 + v_mul_lo_u32 pairs (what hipcc emits for __umulhi and
// a * b) against one v_mad_u64_u32 per product.  One JSON line per variant:
// ms and products per second over the whole chip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ void __launch_bounds__(256) rounds(uint32_t *out, uint32_t n)
{
    uint32_t c0 = threadIdx.x, c1 = blockIdx.x, c2 = c0 ^ 0x55u, c3 = c1 * 7u;
    uint32_t k0 = 1u, k1 = 2u;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t hi0, lo0, hi1, lo1;
        if constexpr (MODE == 0) {
            hi0 = __umulhi(0xD2511F53u, c0); lo0 = 0xD2511F53u * c0;
            hi1 = __umulhi(0xCD9E8D57u, c2); lo1 = 0xCD9E8D57u * c2;
        } else {
            uint64_t a, b, ca, cb;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a), "=s"(ca) : "v"(c0), "s"(0xD2511F53u));
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(b), "=s"(cb) : "v"(c2), "s"(0xCD9E8D57u));
            hi0 = (uint32_t)(a >> 32); lo0 = (uint32_t)a; hi1 = (uint32_t)(b >> 32); lo1 = (uint32_t)b;
        }
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3;
}

int main()
{
    const uint32_t blocks = 256 * 16, n = 4096;
    uint32_t *out;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; rep++) {
        for (int mode = 0; mode < 2; mode++) {
            hipEventRecord(a);
            if (mode == 0) hipLaunchKernelGGL(rounds<0>, dim3(blocks), dim3(256), 0, 0, out, n);
            else hipLaunchKernelGGL(rounds<1>, dim3(blocks), dim3(256), 0, 0, out, n);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double products = 2.0 * n * blocks * 256;
            if (rep) printf("{\"variant\": \"%s\", \"ms\": %.4f, \"products_per_s\": %.4g}\n",
                            mode == 0 ? "mul_hi+mul_lo" : "mad_u64_u32", ms, products / (ms * 1e-3));
        }
    }
    hipFree(out);
    return 0;
}
