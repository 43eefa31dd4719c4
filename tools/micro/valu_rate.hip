// VALU issue-rate microbenchmark (gfx950, test infrastructure): cycles per wave64 instruction per SIMD for the
// instruction kinds the extraction kernels are built from.  One workgroup of 4 x W waves per CU (W waves on each
// SIMD, all co-resident: a workgroup never spans CUs); every wave runs ITER x 16 instructions of one kind in 16
// independent chains, clocked with s_memtime.  Per workgroup: window = max end - min start over its waves;
// cycles per instruction per SIMD = window / (ITER * 16 * W); the median over the workgroups is printed.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/valu_rate tools/micro/valu_rate.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define ITER 128
#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__);           \
            return 1;                                                            \
        }                                                                        \
    } while (0)

// %0 = the chain register (read and written), %1 / %2 = loop-invariant sources
#define OPS(X)                                                     \
    X(0, "v_add_u32 %0, %0, %1")                                   \
    X(1, "v_sub_u32 %0, %0, %1")                                   \
    X(2, "v_and_b32 %0, %0, %1")                                   \
    X(3, "v_or_b32 %0, %0, %1")                                    \
    X(4, "v_xor_b32 %0, %0, %1")                                   \
    X(5, "v_lshlrev_b32 %0, 1, %0")                                \
    X(6, "v_max_u32 %0, %0, %1")                                   \
    X(7, "v_min_u32 %0, %0, %1")                                   \
    X(8, "v_max_i32 %0, %0, %1")                                   \
    X(9, "v_max_f32 %0, %0, %1")                                   \
    X(10, "v_add_f32 %0, %0, %1")                                  \
    X(11, "v_fma_f32 %0, %0, %1, %2")                              \
    X(12, "v_max3_u32 %0, %0, %1, %2")                             \
    X(13, "v_max3_f32 %0, %0, %1, %2")                             \
    X(14, "v_med3_u32 %0, %0, %1, %2")                             \
    X(15, "v_perm_b32 %0, %0, %1, %2")                             \
    X(16, "v_or3_b32 %0, %0, %1, %2")                              \
    X(17, "v_add3_u32 %0, %0, %1, %2")                             \
    X(18, "v_lshl_or_b32 %0, %0, 2, %1")                           \
    X(19, "v_alignbyte_b32 %0, %0, %1, 1")                         \
    X(20, "v_bfe_u32 %0, %0, 3, 5")                                \
    X(21, "v_mul_u32_u24 %0, %0, %1")                              \
    X(22, "v_mad_u32_u24 %0, %0, %1, %2")                          \
    X(23, "v_mul_lo_u32 %0, %0, %1")                               \
    X(24, "v_cndmask_b32 %0, %0, %1, vcc")                         \
    X(25, "v_mbcnt_lo_u32_b32 %0, -1, %0")                         \
    X(26, "v_cmp_gt_u32 vcc, %0, %1")                              \
    X(27, "v_cmp_gt_u32_e64 s[40:41], %0, %1")                     \
    X(28, "v_max_u16 %0, %0, %1")                                  \
    X(29, "v_max_f16 %0, %0, %1")                                  \
    X(30, "v_pk_max_u16 %0, %0, %1")                               \
    X(31, "v_pk_min_u16 %0, %0, %1")                               \
    X(32, "v_pk_add_u16 %0, %0, %1")                               \
    X(33, "v_pk_sub_u16 %0, %0, %1")                               \
    X(34, "v_pk_max_i16 %0, %0, %1")                               \
    X(35, "v_pk_max_f16 %0, %0, %1")                               \
    X(36, "v_pk_add_f16 %0, %0, %1")                               \
    X(37, "v_pk_fma_f16 %0, %0, %1, %2")                           \
    X(38, "v_pk_maximum3_f16 %0, %0, %1, %2")                      \
    X(39, "v_pk_minimum3_f16 %0, %0, %1, %2")                      \
    X(40, "v_maximum3_f32 %0, %0, %1, %2")                         \
    X(41, "v_sad_u8 %0, %0, %1, %2")                               \
    X(42, "v_max_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0") \
    X(43, "v_max_u32_sdwa %0, %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_0") \
    X(44, "v_mov_b32 %0, %1")                                      \
    X(45, "v_cvt_f32_ubyte1 %0, %0")                               \
    X(46, "v_add_u16 %0, %0, %1")                                  \
    X(47, "v_lshrrev_b32 %0, 3, %0")

#define NOPS 49

template <int K>
__device__ __forceinline__ void body(unsigned (&r)[16], unsigned k0, unsigned k1);
#define DEF_BODY(n, fmt)                                                                              \
    template <>                                                                                       \
    __device__ __forceinline__ void body<n>(unsigned(&r)[16], unsigned k0, unsigned k1)               \
    {                                                                                                 \
        _Pragma("unroll") for (int c = 0; c < 16; c++) __asm__ volatile(fmt : "+v"(r[c]) : "v"(k0), "v"(k1) : "vcc", "s40", "s41"); \
    }
OPS(DEF_BODY)

// the packed-f32 op needs 64-bit operands
template <>
__device__ __forceinline__ void body<48>(unsigned (&r)[16], unsigned k0, unsigned k1)
{
    double d[8];
    for (int c = 0; c < 8; c++) d[c] = __builtin_bit_cast(double, ((unsigned long long)r[2 * c + 1] << 32) | r[2 * c]);
    const double a = __builtin_bit_cast(double, ((unsigned long long)k1 << 32) | k0);
    for (int rep = 0; rep < 2; rep++)
#pragma unroll
        for (int c = 0; c < 8; c++) __asm__ volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d[c]) : "v"(a), "v"(a));
    for (int c = 0; c < 8; c++) {
        const unsigned long long u = __builtin_bit_cast(unsigned long long, d[c]);
        r[2 * c] = (unsigned)u;
        r[2 * c + 1] = (unsigned)(u >> 32);
    }
}

template <int K>
__global__ __launch_bounds__(1024) void valu_kernel(unsigned long long* t, unsigned* out, unsigned seed)
{
    unsigned r[16];
    for (int i = 0; i < 16; i++) r[i] = seed * (threadIdx.x + 3 * i + 1);
    const unsigned k0 = (seed ^ threadIdx.x) | 0x3c003c00u, k1 = seed + 7;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) body<K>(r, k0, k1);
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0);
    unsigned acc = 0;
    for (int i = 0; i < 16; i++) acc ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        t[2 * w] = t0;
        t[2 * w + 1] = t1;
    }
}

static const char* NAMES[NOPS] = {
#define NAME(n, fmt) fmt,
    OPS(NAME)
#undef NAME
    "v_pk_fma_f32 (64-bit operands)"};

template <int K>
static int run(int ncu, double (&res)[3])
{
    const int wpsv[3] = {1, 2, 4};
    for (int vi = 0; vi < 3; vi++) {
        const int wps = wpsv[vi], nt = 256 * wps, nw = ncu * 4 * wps;
        unsigned long long* d_t;
        unsigned* d_out;
        CHK(hipMalloc(&d_t, nw * 16));
        CHK(hipMalloc(&d_out, ncu * nt * 4));
        std::vector<double> win;
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(valu_kernel<K>, dim3(ncu), dim3(nt), 0, 0, d_t, d_out, 12345u + rep);
            CHK(hipDeviceSynchronize());
            if (rep == 0) continue;
            std::vector<unsigned long long> t(2 * nw);
            CHK(hipMemcpy(t.data(), d_t, nw * 16, hipMemcpyDeviceToHost));
            for (int b = 0; b < ncu; b++) {
                unsigned long long lo = ~0ull, hi = 0;
                for (int w = 0; w < 4 * wps; w++) {
                    lo = std::min(lo, t[2 * (b * 4 * wps + w)]);
                    hi = std::max(hi, t[2 * (b * 4 * wps + w) + 1]);
                }
                win.push_back((double)(hi - lo));
            }
        }
        std::sort(win.begin(), win.end());
        res[vi] = win[win.size() / 2] / (ITER * 16.0 * wps);
        CHK(hipFree(d_t));
        CHK(hipFree(d_out));
    }
    return 0;
}

template <int K>
static int run_all(int ncu)
{
    if constexpr (K < NOPS) {
        double r[3];
        if (run<K>(ncu, r)) return 1;
        printf("%-100s  W=1 %5.2f  W=2 %5.2f  W=4 %5.2f\n", NAMES[K], r[0], r[1], r[2]);
        fflush(stdout);
        return run_all<K + 1>(ncu);
    }
    return 0;
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    printf("%s, %d CUs; cycles per wave64 instruction per SIMD at W waves per SIMD (s_memtime window, median)\n",
           p.gcnArchName, p.multiProcessorCount);
    return run_all<0>(p.multiProcessorCount);
}
