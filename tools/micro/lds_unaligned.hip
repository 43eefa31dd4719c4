// LDS reads at 2-byte-aligned addresses on gfx950 (test infrastructure): each lane reads 4 dwords starting at u16
// index 2 * lane + 1 of a known u16 ramp with ds_read_b32 x4, ds_read2_b32 x2, ds_read_b64 x2 and ds_read_b128, and
// checks every dword against the ramp.  Prints the mismatch count of each form.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/lds_unaligned tools/micro/lds_unaligned.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out)
{
    __shared__ unsigned short s[1200];
    for (int i = threadIdx.x; i < 1200; i += blockDim.x) s[i] = (unsigned short)(i * 7 + 3);
    __syncthreads();
    const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)s;
    const int l = threadIdx.x;
    const unsigned a = base + 2u * (2u * l + 1u);
    unsigned v[4][4];
    __asm__ volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:4\n\tds_read_b32 %2, %4 offset:8\n\t"
                     "ds_read_b32 %3, %4 offset:12\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(v[0][0]), "=v"(v[0][1]), "=v"(v[0][2]), "=v"(v[0][3]) : "v"(a));
    __asm__ volatile("ds_read2_b32 %0, %2 offset1:1\n\tds_read2_b32 %1, %2 offset0:2 offset1:3\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(*(unsigned long long*)&v[1][0]), "=v"(*(unsigned long long*)&v[1][2]) : "v"(a));
    __asm__ volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(*(unsigned long long*)&v[2][0]), "=v"(*(unsigned long long*)&v[2][2]) : "v"(a));
    __asm__ volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(*(uint4*)&v[3][0]) : "v"(a));
    for (int f = 0; f < 4; f++) {
        unsigned bad = 0;
        for (int j = 0; j < 4; j++) {
            const int u = 2 * l + 1 + 2 * j;
            const unsigned want = (unsigned)s[u] | ((unsigned)s[u + 1] << 16);
            bad += v[f][j] != want;
        }
        out[f * 256 + l] = bad;
    }
}

int main()
{
    unsigned* d;
    if (hipMalloc(&d, 1024 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d);
    unsigned h[1024];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[4] = {"ds_read_b32 x4", "ds_read2_b32 x2", "ds_read_b64 x2", "ds_read_b128"};
    for (int f = 0; f < 4; f++) {
        int bad = 0;
        for (int i = 0; i < 256; i++) bad += h[f * 256 + i];
        printf("%-16s at 2-byte alignment: %d wrong dwords of 1024\n", names[f], bad);
    }
    return 0;
}
