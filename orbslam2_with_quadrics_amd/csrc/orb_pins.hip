// orb_pins.hip -- exhaustive device-side pins of the restated glibc functions (orb_math_dev.h): og_sincosf
// (rBRIEF rotation, src/ORBextractor.cc:113) and og_logf (MapPoint::PredictScale, src/MapPoint.cc:410) are
// evaluated on every float of a bit range and folded into chunked order-free hashes, which tests compare with
// the host libm's (tools/libm_chunk_hash.c, tests/golden/libm_chunks.json).  Diagnostics entry point only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_math_dev.h"
#include "orbgpu_internal.h"

__device__ __forceinline__ unsigned long long og_hash_mix(unsigned long long z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

#define PIN_NT 256
#define PIN_PER 16  // consecutive inputs per thread: a workgroup covers 4096, never straddling a chunk (log2 >= 12)

// fn 0: sincosf -> (sin bits << 32 | cos bits); fn 1: logf -> log bits.  out[c - c0] += sum over the chunk.
__global__ __launch_bounds__(PIN_NT) void og_math_hash_kernel(int fn, unsigned long long begin,
                                                              unsigned long long end, int chunk_log2,
                                                              unsigned long long c0, unsigned long long* out)
{
    const unsigned long long base = ((begin >> 12) + blockIdx.x) << 12;  // 4096-aligned span of this workgroup
    unsigned long long acc = 0;
    for (int k = 0; k < PIN_PER; k++) {
        const unsigned long long u = base + (unsigned long long)threadIdx.x * PIN_PER + k;
        if (u < begin || u >= end) continue;
        const float x = __uint_as_float((uint32_t)u);
        unsigned long long v;
        if (fn == 0) {
            float s, c;
            og_sincosf(x, &s, &c);
            v = ((unsigned long long)__float_as_uint(s) << 32) | __float_as_uint(c);
        } else {
            v = __float_as_uint(og_logf(x));
        }
        acc += og_hash_mix(v + u * 0x9E3779B97F4A7C15ull);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    __shared__ unsigned long long ws[PIN_NT / 64];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < PIN_NT / 64; w++) t += ws[w];
        atomicAdd(&out[(base >> chunk_log2) - c0], t);
    }
}

hipError_t og_math_hash(int fn, unsigned long long begin, unsigned long long end, int chunk_log2,
                        unsigned long long* d_out, hipStream_t s)
{
    const unsigned long long nblk = ((end + 4095) >> 12) - (begin >> 12);
    hipLaunchKernelGGL(og_math_hash_kernel, dim3((unsigned)nblk), dim3(PIN_NT), 0, s, fn, begin, end, chunk_log2,
                       begin >> chunk_log2, d_out);
    return hipGetLastError();
}
