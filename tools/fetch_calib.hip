// FETCH_SIZE calibration (measurement infrastructure, GPU box): streaming reads of a known byte count at 4, 8 and
// 16 bytes per lane, and the FAST ROI pattern (rows of dword loads at a row pitch, overlapping halos), each kernel
// launched alone so a `rocprofv3 --pmc FETCH_SIZE` pass prices it per dispatch.  The ratio of the counter's bytes
// to the bytes actually read is the correction for that access width (tools/pmc_summary.py).
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib && ./tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// every element read once; one dword per workgroup written (vector store) so nothing is optimised away
template <typename T>
__global__ __launch_bounds__(256) void stream_read(const T* __restrict__ src, size_t n, unsigned* __restrict__ out)
{
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const T v = src[i];
        const unsigned* w = (const unsigned*)&v;
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 4); k++) acc ^= w[k];
    }
    __shared__ unsigned red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned s = 0;
        for (int k = 0; k < 256; k++) s ^= red[k];
        out[blockIdx.x] = s;
    }
}

// FAST-like 2-D tiles: each workgroup reads a (rows x cols-byte) window of a pitched image with dword loads, the
// windows of neighbouring workgroups overlapping by `halo` pixels on each side (as the FAST blocks' ROIs do)
__global__ __launch_bounds__(256) void tile_read(const unsigned char* __restrict__ img, int pitch, int tw, int th,
                                                 int halo, int ntx, unsigned* __restrict__ out)
{
    const int tx = blockIdx.x % ntx, ty = blockIdx.x / ntx;
    const int x0 = tx * tw - halo, y0 = ty * th - halo;
    const int wd = (tw + 2 * halo + 3) / 4 + 1, rows = th + 2 * halo;
    unsigned acc = 0;
    for (int i = threadIdx.x; i < wd * rows; i += 256) {
        const int r = i / wd, c = i - r * wd;
        const long long a = (long long)(y0 + r) * pitch + ((x0 & ~3) + 4 * c);
        acc ^= *(const unsigned*)(img + a);
    }
    __shared__ unsigned red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned s = 0;
        for (int k = 0; k < 256; k++) s ^= red[k];
        out[blockIdx.x] = s;
    }
}

int main()
{
    const size_t bytes = 1ull << 30;
    unsigned char* src;
    unsigned* out;
    CHECK(hipMalloc(&src, bytes + (1 << 20)));
    CHECK(hipMemset(src, 1, bytes + (1 << 20)));
    CHECK(hipMalloc(&out, 1 << 24));
    const int grid = 256 * 32;
    // warm-up launch of each so the PMC pass sees steady-state dispatches; then the measured one
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(stream_read<unsigned>, dim3(grid), dim3(256), 0, 0, (const unsigned*)src, bytes / 4, out);
        hipLaunchKernelGGL(stream_read<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)src, bytes / 8, out);
        hipLaunchKernelGGL(stream_read<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)src, bytes / 16, out);
    }
    // tiles: a 16384-px-pitched image of 16384 rows (256 MiB); 62 x 62 tiles with a 12-px halo (FAST 2x2 cells +
    // the ROI border), and the same without halo
    const int pitch = 16384, H = 16384;
    const int tw = 62, th = 62, ntx = (pitch - 64) / tw, nty = (H - 64) / th;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(tile_read, dim3(ntx * nty), dim3(256), 0, 0, src + 32 * pitch + 32, pitch, tw, th, 12, ntx,
                           out);
        hipLaunchKernelGGL(tile_read, dim3(ntx * nty), dim3(256), 0, 0, src + 32 * pitch + 32, pitch, tw, th, 0, ntx,
                           out);
    }
    CHECK(hipDeviceSynchronize());
    const double halo_bytes = (double)ntx * nty * (th + 24) * 4.0 * ((tw + 24 + 3) / 4 + 1);
    const double nohalo_bytes = (double)ntx * nty * th * 4.0 * ((tw + 3) / 4 + 1);
    const double unique = (double)(ntx * tw + 24) * (nty * th + 24);
    printf("{\"stream_bytes\": %zu, \"tile_halo_bytes_requested\": %.0f, \"tile_nohalo_bytes_requested\": %.0f, "
           "\"tile_unique_bytes\": %.0f, \"order\": [\"stream4\", \"stream8\", \"stream16\", \"tile_halo\", "
           "\"tile_nohalo\"], \"reps\": 2}\n",
           bytes, halo_bytes, nohalo_bytes, unique);
    CHECK(hipFree(src));
    CHECK(hipFree(out));
    return 0;
}
