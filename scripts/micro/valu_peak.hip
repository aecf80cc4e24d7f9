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
//   ./valu_peak [iters [ops]]    kernels valu_kernel<CH, W> for CH in {1,2,4,8}, W in {1,2,4,8},
//                                add / fma chains, and (ops != 0) the single-opcode op_kernel<OP>
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

// ---- single-opcode chains (VERDICT r03 "next" item 4): the opcodes that make
// up >= 90 % of branch_kernel<11,8>'s and macro_staged_kernel<2,true>'s VALU
// text (scripts/valu_mix.py), each alone: CH = 4 independent chains per lane,
// 12 instructions per chain and iteration, 8 waves per SIMD (2048 workgroups
// of 4 waves).  Kernel op_kernel<OP> for OP in the table below; the summary
// (scripts/valu_peak_summary.py) names them by the opcode.
enum {
    OP_XOR, OP_ADD, OP_SUB, OP_AND, OP_LSHR, OP_LSHL, OP_MIN, OP_MOV, OP_CNDMASK, OP_BFE, OP_BITOP3,
    OP_MAD64, OP_LSHLADD64, OP_CMPEQ, OP_READLANE, OP_MULLO, OP_MULHI, OP_ASHR64, OP_N
};
template <int OP>
__device__ __forceinline__ void op1(uint32_t &a, uint32_t &b, uint64_t &w, uint32_t k, uint64_t m)
{
    if constexpr (OP == OP_XOR) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_ADD) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_SUB) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_AND) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_LSHR) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_LSHL) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_MIN) asm volatile("v_min_u32 %0, %1, %0" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b));
    else if constexpr (OP == OP_CNDMASK) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m));
    else if constexpr (OP == OP_BFE) asm volatile("v_bfe_i32 %0, %0, 3, 7" : "+v"(a));
    else if constexpr (OP == OP_BITOP3) a = __builtin_amdgcn_bitop3_b32(a, b, k, 0xCA);
    else if constexpr (OP == OP_MAD64) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w), "=s"(c) : "v"(a), "s"(k));
    } else if constexpr (OP == OP_LSHLADD64) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(w) : "s"(m));
    else if constexpr (OP == OP_CMPEQ) {
        uint64_t c;
        asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(c) : "v"(a), "s"(k));
        asm volatile("" :: "s"(c));
    } else if constexpr (OP == OP_READLANE) {
        uint32_t c;
        asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(c) : "v"(a));
        asm volatile("" :: "s"(c));
    } else if constexpr (OP == OP_MULLO) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_MULHI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "s"(k));
    else if constexpr (OP == OP_ASHR64) asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(w));
}

template <int OP>
__global__ void __launch_bounds__(256) op_kernel(uint32_t *out, uint32_t iters, uint32_t k)
{
    constexpr int CH = 4;
    uint32_t a[CH], b[CH];
    uint64_t w[CH];
    const uint64_t m = 0x5555555555555555ull ^ k;
#pragma unroll
    for (int c = 0; c < CH; c++) {
        a[c] = threadIdx.x * (c + 1) + blockIdx.x;
        b[c] = a[c] ^ 0x9E3779B9u;
        w[c] = ((uint64_t)a[c] << 32) | b[c];
    }
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 12; u++) {
#pragma unroll
            for (int c = 0; c < CH; c++) op1<OP>(a[c], b[c], w[c], k, m);
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= a[c] ^ b[c] ^ (uint32_t)w[c] ^ (uint32_t)(w[c] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
static void run_op(uint32_t iters, uint32_t *d)
{
    const uint32_t blocks = 256u * 8u, it = iters / 4;
    for (int r = 0; r < 4; r++) hipLaunchKernelGGL((op_kernel<OP>), dim3(blocks), dim3(256), 0, 0, d, it, 7u);
    CHECK(hipDeviceSynchronize());
    if constexpr (OP + 1 < OP_N) run_op<OP + 1>(iters, d);
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
    if (argc <= 2 || atoi(argv[2])) run_op<0>(iters, d);
    CHECK(hipFree(d));
    return 0;
}
