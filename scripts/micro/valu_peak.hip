// VALU issue-rate microbenchmark (re-measure the int32 VALU
// peak, VERDICT r02 "next" item 1).  Each lane runs CH independent integer
// chains (add / shift / xor: the interpreter's instruction mix) for ITERS
// iterations, at W waves per SIMD (256 * W workgroups of 4 waves).  The
// instruction count is NOT inferred here: rocprofv3 --pmc SQ_INSTS_VALU
// GRBM_GUI_ACTIVE (one pass, scripts/valu_peak_summary.py) gives the VALU
// instructions per launch and the shader clock, and the kernel trace the
// duration; this program only launches each variant REPS times (and prints
// its HIP-event time so a run without the profiler is still informative).
//
//   ./valu_peak [iters]          kernels valu_kernel<CH, W> for CH in {1,2,4,8}, W in {1,2,4,8}
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int CH, int W>
__global__ void __launch_bounds__(256) valu_kernel(uint32_t *out, uint32_t iters, uint32_t k)
{
    uint32_t a[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x * (c + 1) + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                a[c] = (a[c] + k) ^ (a[c] >> 3);
                a[c] = (a[c] - k) ^ (a[c] << 5);
            }
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// the same shape with one instruction type (inline asm, so nothing folds):
// v_add_u32 only (int), v_fma_f32 only (float)
template <int CH, int W>
__global__ void __launch_bounds__(256) add_kernel(uint32_t *out, uint32_t iters, uint32_t k)
{
    uint32_t a[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = threadIdx.x * (c + 1) + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 12; u++) {
#pragma unroll
            for (int c = 0; c < CH; c++) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[c]) : "s"(k));
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH, int W>
__global__ void __launch_bounds__(256) fma_kernel(uint32_t *out, uint32_t iters, uint32_t k)
{
    float a[CH];
    const float m = 1.0f + 1e-7f * (float)k, q = 1e-3f * (float)k;
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = (float)(threadIdx.x * (c + 1) + blockIdx.x);
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 12; u++) {
#pragma unroll
            for (int c = 0; c < CH; c++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "s"(m), "s"(q));
        }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; c++) s += a[c];
    out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(s);
}

template <int CH, int W>
static void run_other(uint32_t iters, uint32_t *d)
{
    const uint32_t blocks = 256u * W, it = iters / CH;
    hipLaunchKernelGGL((add_kernel<CH, W>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
    hipLaunchKernelGGL((fma_kernel<CH, W>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL((add_kernel<CH, W>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
        hipLaunchKernelGGL((fma_kernel<CH, W>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
    }
    CHECK(hipDeviceSynchronize());
}

template <int CH, int W>
static void run(uint32_t iters, uint32_t *d, int reps)
{
    const uint32_t blocks = 256u * W;          // 256 CUs x 4 SIMDs x W waves = 256 W blocks of 4 waves
    const uint32_t it = iters / CH;            // about the same instructions per lane for every CH
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((valu_kernel<CH, W>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; r++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((valu_kernel<CH, W>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    printf("{\"kernel\": \"valu_kernel<%d, %d>\", \"chains\": %d, \"waves_per_simd\": %d, \"blocks\": %u, "
           "\"iters\": %u, \"ms_min\": %.5f, \"ms_mean\": %.5f}\n", CH, W, CH, W, blocks, it, best, sum / reps);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

template <int W>
static void run_w(uint32_t iters, uint32_t *d, int reps)
{
    run<1, W>(iters, d, reps);
    run<2, W>(iters, d, reps);
    run<4, W>(iters, d, reps);
    run<8, W>(iters, d, reps);
}

int main(int argc, char **argv)
{
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 8192;
    uint32_t *d;
    CHECK(hipMalloc(&d, 256u * 8u * 256u * 4u));
    run_w<1>(iters, d, 5);
    run_w<2>(iters, d, 5);
    run_w<4>(iters, d, 5);
    run_w<8>(iters, d, 5);
    run_other<1, 8>(iters, d);
    run_other<4, 8>(iters, d);
    run_other<8, 8>(iters, d);
    CHECK(hipFree(d));
    return 0;
}
