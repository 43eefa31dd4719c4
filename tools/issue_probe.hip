// Issue-rate probe (measurement infrastructure, GPU box): how many SALU and VALU instructions a CU retires per
// cycle with 1..8 waves per SIMD, alone and interleaved, so the FAST / describe / octree instruction mixes can be
// priced.  Each kernel runs ITER iterations of an unrolled block of independent instructions (4 chains each, so no
// dependent-latency stall); every workgroup is 256 threads (4 waves, one per SIMD), launched with 256 * W
// workgroups for W waves per SIMD.  Output: one JSON line per (kernel, W) with instructions per cycle per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o tools/issue_probe && ./tools/issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

#define ITER 4096
// 16 instructions per block, 4 independent chains
#define S4 "s_add_u32 %0, %0, %4\n\ts_add_u32 %1, %1, %4\n\ts_add_u32 %2, %2, %4\n\ts_add_u32 %3, %3, %4\n\t"
#define V4 "v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t"
#define M4 "s_add_u32 %0, %0, %8\n\tv_add_u32 %4, %4, %9\n\ts_add_u32 %1, %1, %8\n\tv_add_u32 %5, %5, %9\n\t" \
           "s_add_u32 %2, %2, %8\n\tv_add_u32 %6, %6, %9\n\ts_add_u32 %3, %3, %8\n\tv_add_u32 %7, %7, %9\n\t"

__global__ __launch_bounds__(256) void salu_k(unsigned* out, unsigned inc)
{
    unsigned a = threadIdx.x >> 6, b = a + 1, c = a + 2, d = a + 3;
    a = __builtin_amdgcn_readfirstlane(a);
    b = __builtin_amdgcn_readfirstlane(b);
    c = __builtin_amdgcn_readfirstlane(c);
    d = __builtin_amdgcn_readfirstlane(d);
    for (int i = 0; i < ITER; i++)
        __asm__ volatile(S4 S4 S4 S4 : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(inc) : "scc");
    if ((a ^ b ^ c ^ d) == 0x12345678u) out[blockIdx.x] = a;
}

__global__ __launch_bounds__(256) void valu_k(unsigned* out, unsigned inc)
{
    unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    for (int i = 0; i < ITER; i++)
        __asm__ volatile(V4 V4 V4 V4 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(inc));
    if ((a ^ b ^ c ^ d) == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = a;
}

// 16 SALU + 16 VALU interleaved per block
__global__ __launch_bounds__(256) void mixed_k(unsigned* out, unsigned inc)
{
    unsigned a = threadIdx.x >> 6, b = a + 1, c = a + 2, d = a + 3;
    a = __builtin_amdgcn_readfirstlane(a);
    b = __builtin_amdgcn_readfirstlane(b);
    c = __builtin_amdgcn_readfirstlane(c);
    d = __builtin_amdgcn_readfirstlane(d);
    unsigned e = threadIdx.x, f = e + 1, g = e + 2, h = e + 3;
    for (int i = 0; i < ITER; i++)
        __asm__ volatile(M4 M4 M4 M4
                         : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                         : "s"(inc), "v"(inc)
                         : "scc");
    if ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = a;
}

int main()
{
    unsigned* out;
    CHECK(hipMalloc(&out, 256 * 256 * 64 * 4));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const double clk_ghz = prop.clockRate * 1e-6;  // kHz -> GHz (the nominal peak clock)
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct K {
        const char* name;
        void (*fn)(unsigned*, unsigned);
        int salu, valu;  // instructions per block per wave
    } ks[] = {{"salu", salu_k, 16, 0}, {"valu", valu_k, 0, 16}, {"mixed", mixed_k, 16, 16}};
    for (const K& k : ks) {
        for (int W = 1; W <= 8; W *= 2) {
            const int grid = cus * W;  // 4 waves per workgroup, one per SIMD: W waves per SIMD
            hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, 1u);  // warm-up
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, 1u);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double waves = 5.0 * grid * 4.0;
            const double cyc = ms * 1e-3 * clk_ghz * 1e9;  // at the nominal clock
            const double insts = waves * ITER * 16.0;   // per instruction type in the block
            printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"salu_per_cu_cycle\": %.3f, "
                   "\"valu_per_cu_cycle\": %.3f, \"clock_ghz_nominal\": %.2f}\n",
                   k.name, W, ms, k.salu ? insts / cyc / cus : 0.0, k.valu ? insts / cyc / cus : 0.0, clk_ghz);
        }
    }
    CHECK(hipFree(out));
    return 0;
}
