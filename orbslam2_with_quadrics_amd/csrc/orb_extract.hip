// orb_extract.hip -- gfx950 kernels of ORBextractor::operator() (src/ORBextractor.cc:1043-1105).
//
//   k1 og_resize_kernel    : one chained pyramid level (cv::resize INTER_LINEAR 8U; vertical form per
//                            ORBGPU_SEM_RESIZE_*)
//   k2 og_fast_quad_kernel: one 512-thread workgroup per block of up to 2x2 FAST cells: ROI -> LDS,
//                            threshold-free quick test, FAST-9 score, same-cell 3x3 NMS, the reference's
//                            per-cell 20 -> 7 fallback, ballot compaction into the (frame, level) slots
//   k3 og_octree_kernel    : one 1024-thread workgroup per (frame, level): the DistributeOctTree list
//                            simulation as data-parallel rounds (LDS node table, block scans)
//   k4 og_describe_kernel  : one wave per keypoint: 43x43 raw patch -> LDS, IC angle, fused 7x7
//                            Gaussian to a 37x37 patch, rBRIEF 256 tests, ballot-packed 32 B
//   k5 og_grid_kernel      : Frame::AssignFeaturesToGrid, CSR grid per frame
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstddef>
#include <type_traits>

#include "orb_math_dev.h"
#include "orbgpu_internal.h"
#include "orbgpu_launch.h"

typedef unsigned long long u64;

#include "orb_pattern.inc"  // static const signed char oo_orb_pattern[1024]
__constant__ signed char og_pattern[1024];
__constant__ float4 og_pattern_f[256];  // the same tests as floats (x0, y0, x1, y1): one 16-byte load, no conversions
static bool g_pattern_uploaded_dev[64] = {false};

// Lane masks straight from one v_cmp each (LLVM lowers ballot(a && b) as v_cmp(v_cndmask(mask), 0): two VALU
// per ballot); compound conditions are ANDs of these masks on the scalar unit.  Inactive lanes read 0.
#define OG_ICMP_EQ 32
#define OG_ICMP_NE 33
#define OG_ICMP_SGT 38
#define OG_ICMP_SLT 40
__device__ __forceinline__ u64 og_lanes_ne(unsigned a, unsigned b) { return __builtin_amdgcn_uicmp(a, b, OG_ICMP_NE); }
__device__ __forceinline__ u64 og_lanes_eq(unsigned a, unsigned b) { return __builtin_amdgcn_uicmp(a, b, OG_ICMP_EQ); }
__device__ __forceinline__ u64 og_lanes_lt(int a, int b) { return __builtin_amdgcn_sicmp(a, b, OG_ICMP_SLT); }
__device__ __forceinline__ u64 og_lanes_gt(int a, int b) { return __builtin_amdgcn_sicmp(a, b, OG_ICMP_SGT); }
__device__ __forceinline__ u64 og_ballot(bool b) { return __ballot(b); }
// number of set bits of m below this lane (v_mbcnt: 2 VALU instead of masking and two popcounts)
__device__ __forceinline__ int og_rank(u64 m, int base = 0)  // + base, for free
{
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, (unsigned)base));
}

// XCD-aware bijective remap (cdna_hip_programming.md §5.5 T1): workgroups are dealt round-robin over
// the 8 XCDs (separate L2s); give each XCD one contiguous chunk of the logical index space so that
// neighbouring FAST cells / keypoints, which share cache lines, hit the same L2.  Speed only.
// LDS byte address of a __shared__ object
template <typename T>
__device__ __forceinline__ uint32_t og_lds_addr(T* p)
{
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p;
}

__device__ __forceinline__ unsigned og_xcd_remap(unsigned orig, unsigned nwg)
{
    const unsigned q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ------------------------------------------------------------------------------------------------
// k1: pyramid level l from level l-1 (src/ORBextractor.cc:1120)
// ------------------------------------------------------------------------------------------------
// cv::resize's vertical pass on the horizontal sums d0, d1 (<= 255 * 2048) with weights b0 + b1 = 2048:
//   FX = false: OpenCV's 8U specialisation of VResizeLinear (SSE2 mulhi body and scalar tail alike):
//               ((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2
//   FX = true : the generic FixedPtCast form (b0 * d0 + b1 * d1 + 2^21) >> 22
// All terms are >= 0 and < 2^32 (products < 2^27 after the shift, 2^31 before), results <= 255.
template <bool FX>
__device__ __forceinline__ uint32_t og_rz_vert(uint32_t b0, uint32_t d0, uint32_t b1, uint32_t d1)
{
    if (FX) return min((__umul24(b0, d0) + __umul24(b1, d1) + (1u << 21)) >> 22, 255u);
    return min(((__umul24(b0, d0 >> 4) >> 16) + (__umul24(b1, d1 >> 4) >> 16) + 2u) >> 2, 255u);
}

// og_resize2_kernel's form of og_rz_vert: with FX = false its horizontal weights are pre-scaled by 16
// (og_rz_weights; <= 2048 * 16 = 32768 fits the u16 dot operand), so D = 16 d and D & ~0xff = (d >> 4) << 8, and
// v_mul_hi_u32_u24(b << 8, (d >> 4) << 8) = (b * (d >> 4)) >> 16 exactly (operands < 2^24: b <= 2049,
// D <= 255 * 2049 * 16): two ops per term instead of three.  FX = true is og_rz_vert.
__device__ __forceinline__ uint32_t og_mulhi_u24(uint32_t a, uint32_t b)
{
    uint32_t r;
    __asm__("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <bool FX>
__device__ __forceinline__ uint32_t og_rz_vert16(uint32_t b0, uint32_t D0, uint32_t b1, uint32_t D1)
{
    if (FX) return og_rz_vert<FX>(b0, D0, b1, D1);  // unscaled weights: D = d
    return min((og_mulhi_u24(b0 << 8, D0 & ~0xffu) + og_mulhi_u24(b1 << 8, D1 & ~0xffu) + 2u) >> 2,
               255u);
}

// (s >> 2) into byte k of `packed`, the other bytes preserved (one SDWA shift; byte 0 clears the rest).  For the FX = false form's sums
// s = t0 + t1 + 2 the result is <= 255 without a clamp: both weight pairs sum to <= 2049 (two cvRound of
// complementary products, og_plan_tables), so x = d >> 4 <= 2049 * 255 / 16 and t0 + t1 <= 2049 * x / 2^16 < 1021
__device__ __forceinline__ void og_rz_put_shr2(uint32_t& packed, uint32_t s, int k)
{
    if (k == 0)  // (the first byte zeroes the others: `packed` needs no initial value)
        __asm__("v_lshrrev_b32_sdwa %0, %2, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD"
                : "=v"(packed) : "v"(s), "s"(2u));
    else if (k == 1)
        __asm__("v_lshrrev_b32_sdwa %0, %2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                : "+v"(packed) : "v"(s), "s"(2u));
    else if (k == 2)
        __asm__("v_lshrrev_b32_sdwa %0, %2, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                : "+v"(packed) : "v"(s), "s"(2u));
    else
        __asm__("v_lshrrev_b32_sdwa %0, %2, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                : "+v"(packed) : "v"(s), "s"(2u));
}

#define RZ_NT 256
#define RZ_TW 256                      // output columns per workgroup (64 lanes x 4)
#define RZ_TH 16                       // output rows per workgroup (4 waves x 4 rows)
#define RZ_SROWS 28                    // >= source rows a 16-row tile touches (15 * 1.6 + 2, scale <= 1.6)
#define RZ_SC 448                      // LDS row stride: >= 255 * 1.6 + 2 source bytes + 15 alignment slack
typedef unsigned short og_rz_u16x2 __attribute__((ext_vector_type(2)));

// One workgroup = 16 output rows x 256 output columns of one frame (balanced tiles: a 1111-px level is 5
// tiles, not 1024 + 87).  The source rows/columns the tile touches are staged in LDS with 16-byte loads
// from 16-byte aligned addresses, all issued before the first LDS store; each source row keeps its own
// misalignment (mis[r]), so any pitch and any frame stride take the same path.  Each output pixel costs
// 4 LDS byte reads; the arithmetic is the scalar fixed-point form of cv::resize INTER_LINEAR (DESIGN.md
// §3.1).  The aligned 16-byte blocks read never leave the 16-byte block holding a pixel of the row.
template <bool FX>
__global__ __launch_bounds__(RZ_NT) void og_resize_kernel(const uint8_t* __restrict__ src, long long src_pitch,
                                                          long long src_fstride, uint8_t* __restrict__ dst,
                                                          long long dst_pitch, long long dst_fstride, int sw,
                                                          int sh, int dw, int dh, const int4* __restrict__ xtab,
                                                          const int4* __restrict__ ytab, int xmax,
                                                          int* __restrict__ status)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[RZ_SROWS * RZ_SC];
    __shared__ int mis[RZ_SROWS];
    __shared__ int4 YT[RZ_TH];  // ytab rows of the tile (read once, not once per row by every thread)
    const int f = blockIdx.z, tid = threadIdx.x;
    const int dy0 = blockIdx.y * RZ_TH, dx0 = blockIdx.x * RZ_TW;
    const int ny = min(RZ_TH, dh - dy0), nx = min(RZ_TW, dw - dx0);
    const int sy0 = ytab[dy0].x, sy1 = ytab[dy0 + ny - 1].y;   // clipped rows, monotone in dy
    const int sx0 = xtab[dx0].x;
    const int sx1 = min(xtab[dx0 + nx - 1].x + 1, sw - 1);
    const uint8_t* base = src + (long long)f * src_fstride;
    const int nrows = sy1 - sy0 + 1, ncols = sx1 - sx0 + 1;
    const int nch = (ncols + 15 + 15) >> 4;                      // 16-byte chunks per row incl. misalignment
    if (nrows > RZ_SROWS || nch * 16 > RZ_SC) {                 // unreachable: scaleFactor <= 1.6 on the host
        if (tid == 0) atomicOr(status, 8);
        return;
    }
    {
        if (tid < ny) YT[tid] = ytab[dy0 + tid];
        uint4 buf[4];
        const int q = tid & 31;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int r = (tid >> 5) + 8 * k;
            buf[k] = make_uint4(0u, 0u, 0u, 0u);
            if (r < nrows && q < nch) {
                const uintptr_t a = (uintptr_t)(base + (long long)(sy0 + r) * src_pitch + sx0);
                const uintptr_t a16 = a & ~(uintptr_t)15;
                if (a16 + 16 * q <= a + (uintptr_t)(ncols - 1)) buf[k] = *(const uint4*)(a16 + 16 * q);
                if (q == 0) mis[r] = (int)(a - a16);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int r = (tid >> 5) + 8 * k;
            if (r < nrows && q < nch) *(uint4*)&S[r * RZ_SC + 16 * q] = buf[k];
        }
    }
    __syncthreads();
    const int c = tid & 63, rg = tid >> 6;
    const int dxt = dx0 + 4 * c;
    if (dxt >= dw) return;
    int sx[4], a0[4], a1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int dx = min(dxt + k, dw - 1);
        const int4 xt = xtab[dx];
        sx[k] = xt.x - sx0;
        if (dx < xmax) {
            a0[k] = xt.y;
            a1[k] = xt.z;
        } else {                                                // right border: S[sx]*2048
            a0[k] = 2048;
            a1[k] = 0;
        }
    }
    const int n = min(4, dw - dxt);
    uint8_t* D = dst + (long long)f * dst_fstride + dxt;
    auto store = [&](int r, uint32_t packed) {
        uint8_t* Dr = D + (long long)(dy0 + r) * dst_pitch;
        if (n == 4 && ((((uintptr_t)Dr) & 3) == 0)) {
            *(uint32_t*)Dr = packed;
        } else {
            for (int k = 0; k < n; k++) Dr[k] = (uint8_t)(packed >> (8 * k));
        }
    };
    if ((src_pitch & 15) == 0) {
        // every staged row has the same misalignment: the (S[sx], S[sx+1]) pair of column k is one v_perm of
        // the two LDS dwords around it (selector fixed per thread), the horizontal pass one v_dot2_u32_u16
        const int m0 = mis[0];
        int dwk[4];
        uint32_t sel[4];
        og_rz_u16x2 wt[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int bp = m0 + sx[k];
            const unsigned o = (unsigned)(bp & 3);
            dwk[k] = bp >> 2;
            sel[k] = o | 0x0c00u | ((o + 1u) << 16) | 0x0c000000u;
            // a1 = 0 at the right border; FX = false: pre-scaled by 16 for the multiply-high form (og_rz_vert16)
            wt[k] = og_rz_u16x2{(unsigned short)(a0[k] << (FX ? 0 : 4)), (unsigned short)(a1[k] << (FX ? 0 : 4))};
        }
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            const int r = 4 * rg + rr;
            if (r >= ny) break;
            const int4 yt = YT[r];
            const uint32_t* R0 = (const uint32_t*)(S + (yt.x - sy0) * RZ_SC);
            const uint32_t* R1 = (const uint32_t*)(S + (yt.y - sy0) * RZ_SC);
            uint32_t packed = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t p0 = __builtin_amdgcn_perm(R0[dwk[k] + 1], R0[dwk[k]], sel[k]);
                const uint32_t p1 = __builtin_amdgcn_perm(R1[dwk[k] + 1], R1[dwk[k]], sel[k]);
                const uint32_t d0 = __builtin_amdgcn_udot2(__builtin_bit_cast(og_rz_u16x2, p0), wt[k], 0u, false);
                const uint32_t d1 = __builtin_amdgcn_udot2(__builtin_bit_cast(og_rz_u16x2, p1), wt[k], 0u, false);
                if (!FX)  // og_rz_vert16 (its clamp never binds, og_rz_put_shr2)
                    og_rz_put_shr2(packed, og_mulhi_u24((unsigned)yt.z << 8, d0 & ~0xffu) + og_mulhi_u24((unsigned)yt.w << 8, d1 & ~0xffu) + 2u, k);
                else
                    packed |= og_rz_vert<FX>((unsigned)yt.z, d0, (unsigned)yt.w, d1) << (8 * k);
            }
            store(r, packed);
        }
        return;
    }
#pragma unroll
    for (int rr = 0; rr < 4; rr++) {
        const int r = 4 * rg + rr;
        if (r >= ny) break;
        const int4 yt = YT[r];
        const int r0 = yt.x - sy0, r1 = yt.y - sy0;
        const uint8_t* R0 = S + r0 * RZ_SC + mis[r0];
        const uint8_t* R1 = S + r1 * RZ_SC + mis[r1];
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // (a1 == 0 at the right border, where sx+1 may be the column past the tile: reads 0-weighted)
            const int d0 = R0[sx[k]] * a0[k] + (a1[k] ? R0[sx[k] + 1] * a1[k] : 0);
            const int d1 = R1[sx[k]] * a0[k] + (a1[k] ? R1[sx[k] + 1] * a1[k] : 0);
            packed |= og_rz_vert<FX>((unsigned)yt.z, (unsigned)d0, (unsigned)yt.w, (unsigned)d1) << (8 * k);
        }
        store(r, packed);
    }
}

// ------------------------------------------------------------------------------------------------
// k1': two chained pyramid levels per launch (A = level l from S = level l-1, then B = level l+1 from A).
// One workgroup = one 16 x 256 tile of B.  The A rows/columns the tile reads are computed into LDS from the
// staged S region (never re-read from HBM); the A pixels the tile OWNS are also stored.  Ownership of A
// follows B's tiles through the source index of their first row/column (ytabB[y].x, xtabB[x].x, monotone):
// tile [y0, y1) x [x0, x1) owns A rows [ytabB[y0].x, ytabB[y1].x) and columns [xtabB[x0].x, xtabB[x1].x),
// the last tile of a row/column up to the level edge -- a partition of A, so every A pixel is stored once.
// The arithmetic is og_resize_kernel's (cv::resize INTER_LINEAR fixed point, og_rz_vert).
// ------------------------------------------------------------------------------------------------

// 4 horizontally adjacent outputs of one row from two LDS source rows: sx = byte offsets in the rows, weights
// (a0, a1) per column (a1 = 0 at the right border), vertical weights (yz, yw) -- for FX = false already shifted left
// by 8 (the multiply-high operand of og_rz_vert16; og_resize2_kernel stages its y table that way)
template <bool FX>
__device__ __forceinline__ uint32_t og_rz_quad(const uint8_t* R0, const uint8_t* R1, const int* sx,
                                               const og_rz_u16x2* wt, unsigned yz, unsigned yw)
{
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t p0 = (uint32_t)R0[sx[k]] | ((uint32_t)R0[sx[k] + 1] << 16);
        const uint32_t p1 = (uint32_t)R1[sx[k]] | ((uint32_t)R1[sx[k] + 1] << 16);
        const uint32_t d0 = __builtin_amdgcn_udot2(__builtin_bit_cast(og_rz_u16x2, p0), wt[k], 0u, false);
        const uint32_t d1 = __builtin_amdgcn_udot2(__builtin_bit_cast(og_rz_u16x2, p1), wt[k], 0u, false);
        if (!FX)  // og_rz_vert16 (its clamp never binds, og_rz_put_shr2): the final shift writes byte k of `packed`
            og_rz_put_shr2(packed, og_mulhi_u24(yz, d0 & ~0xffu) + og_mulhi_u24(yw, d1 & ~0xffu) + 2u, k);
        else
            packed |= og_rz_vert16<FX>(yz, d0, yw, d1) << (8 * k);
    }
    return packed;
}

// (og_resize2_kernel: FX = false pre-scales the weights by 16 for og_rz_vert16)
template <bool FX>
__device__ __forceinline__ void og_rz_weights(const int4* xtab, int xmax, int dx, int base, int* sx, og_rz_u16x2* wt,
                                              int k)
{
    const int4 xt = xtab[dx];
    sx[k] = xt.x - base;
    const int sh = FX ? 0 : 4;
    wt[k] = dx < xmax ? og_rz_u16x2{(unsigned short)(xt.y << sh), (unsigned short)(xt.z << sh)}
                      : og_rz_u16x2{(unsigned short)(2048 << sh), 0};
}

#define RZ2_U 3  // staging chunks per thread per round of og_resize2_kernel

__device__ __forceinline__ void og_rz_store4(uint8_t* Dr, uint32_t packed, int n)
{
    if (n == 4 && ((((uintptr_t)Dr) & 3) == 0)) {
        *(uint32_t*)Dr = packed;
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < n) Dr[k] = (uint8_t)(packed >> (8 * k));
    }
}

template <bool FX>
__global__ __launch_bounds__(RZ2_NT) void og_resize2_kernel(const uint8_t* __restrict__ src, long long src_pitch,
                                                           long long src_fstride, uint8_t* __restrict__ dstA,
                                                           long long pitchA, uint8_t* __restrict__ dstB,
                                                           long long pitchB, long long dst_fstride, OgRz2Geom g,
                                                           int* __restrict__ status)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t rz2_lds[];
    // LDS layout (og_rz2_lds_bytes): the tile's rows of the A pass's y table, then S, A and the row misalignments (the
    // B pass reads its wave-uniform y-table rows with scalar loads)
    int4* YA = (int4*)rz2_lds;                     // [AR]  ytabA[ar0 + i]
    uint8_t* S = (uint8_t*)(YA + g.AR);             // [SR][SC] staged source rows (own misalignment each)
    uint8_t* A = S + g.SR * g.SC;                  // [AR][AC] level-A region, column ac0 at byte 0
    int* mis = (int*)(A + g.AR * g.AC);            // [SR]
    const int f = blockIdx.z, tid = threadIdx.x;
    const int by0 = blockIdx.y * RZ2_TH, bx0 = blockIdx.x * RZ_TW;
    const int nyB = min(RZ2_TH, g.bh - by0);
    // A region (what B's tile reads, plus the A pixels it owns) and the S region it reads: replayed on the host
    // from the tables (orbgpu_capi.cpp), one load instead of a chain of dependent table lookups
    const int4* T = g.tiles + 3 * (blockIdx.y * gridDim.x + blockIdx.x);
    const int4 t0 = T[0], t1 = T[1], t2 = T[2];
    const int ar0 = t0.x, ar1 = t0.y, own_r1 = t0.z, ac0 = t0.w;
    const int ac1 = t1.x, own_c1 = t1.y, sr0 = t1.z, sr1 = t1.w;
    const int sc0 = t2.x, sc1 = t2.y;
    const int nrS = sr1 - sr0 + 1, ncS = sc1 - sc0 + 1, nrA = ar1 - ar0 + 1, ncA = ac1 - ac0 + 1;
    const int nch = (ncS + 15 + 15) >> 4;
    if (nrS > g.SR || nch * 16 > g.SC - 16 || nrA > g.AR || ((ncA + 3) & ~3) > g.AC - 16 || nrA > RZ2_NT ||
        ncA > 4 * RZ2_NT) {  // host maxima; one thread per A row / column quad
        if (tid == 0) atomicOr(status, 8);
        return;
    }
    // the A pass's x weights, loaded before the staging so that they are in flight with it.  A pass: thread =
    // one fixed column quad (qa) x every G-th row of the region; B pass: column quad cth, 4 rows.
    const int nqA = (ncA + 3) >> 2;                // <= RZ2_NT (checked above)
    const int G = RZ2_NT / nqA;
    const int qa = tid % nqA, rga = tid / nqA;
    const int cA = ac0 + 4 * qa;
    int sxA[4], sxB[4];
    og_rz_u16x2 wtA[4], wtB[4];
    const int cth = tid & 63, rg = tid >> 6;
    const int dxt = bx0 + 4 * cth;
#pragma unroll
    for (int k = 0; k < 4; k++) og_rz_weights<FX>(g.xtabA, g.xmaxA, min(cA + k, ac1), sc0, sxA, wtA, k);
    // staging addresses: the region's first row (wave-uniform, SGPRs) rounded down to 16 bytes plus a 32-bit lane
    // offset; chunk -> (row, chunk) with the exact float quotient (nIt < 2^14)
    const uint8_t* rbase = src + (long long)f * src_fstride + (long long)sr0 * src_pitch + sc0;
    const unsigned mb = (unsigned)((uintptr_t)rbase & 15);
    const uint8_t* abase = rbase - mb;
    const unsigned upitch = (unsigned)src_pitch & (OG_MAX_PITCH - 1);  // < 2^24 (checked on the host)
    const float rn = 1.0f / (float)nch, hn = 0.5f * rn;
    // RZ2_U chunks per thread per round, all loads issued before the first LDS store; the y-table rows of the
    // tile ride along (each pass below reads its vertical weights from LDS, not from a global load per row)
    const int nIt = nrS * nch;
    const int4 ya = tid < nrA ? g.ytabA[ar0 + tid] : make_int4(0, 0, 0, 0);
    for (int it0 = tid; it0 < nIt; it0 += RZ2_NT * RZ2_U) {
        uint4 v[RZ2_U];
#pragma unroll
        for (int u = 0; u < RZ2_U; u++) {
            const int it = it0 + u * RZ2_NT;
            v[u] = make_uint4(0u, 0u, 0u, 0u);
            if (it < nIt) {
                const int r = (int)__builtin_fmaf((float)it, rn, hn) & 127, q = it - (int)__umul24((unsigned)r, (unsigned)nch & 0xfffu);
                const unsigned o = __umul24((unsigned)r, upitch) + mb;  // row start relative to abase (upitch < 2^24)
                const unsigned c16 = (o & ~15u) + 16u * (unsigned)q;  // this chunk, 16-byte aligned
                if (c16 <= o + (unsigned)(ncS - 1)) v[u] = *(const uint4*)(abase + c16);
            }
        }
#pragma unroll
        for (int u = 0; u < RZ2_U; u++) {
            const int it = it0 + u * RZ2_NT;
            if (it < nIt) {
                const int r = (int)__builtin_fmaf((float)it, rn, hn) & 127, q = it - (int)__umul24((unsigned)r, (unsigned)nch & 0xfffu);
                *(uint4*)&S[__umul24((unsigned)r, (unsigned)g.SC) + 16 * q] = v[u];
                if (q == 0) mis[r] = (int)((__umul24((unsigned)r, upitch) + mb) & 15u);
            }
        }
    }
    // the A pass's table rows relative to the staged region (row - sr0) and, for FX = false, with the vertical weights
    // pre-shifted for the multiply-high form: once per tile instead of once per row and thread
    if (tid < nrA) YA[tid] = make_int4(ya.x - sr0, ya.y - sr0, FX ? ya.z : ya.z << 8, FX ? ya.w : ya.w << 8);
    __syncthreads();
    // ---- level A region -> LDS (and the owned part -> HBM)
    uint8_t* DA = dstA + (long long)f * dst_fstride;
    if (rga < G) {
        // ac0 is a multiple of 4 (host plan): every quad left of own_c1 is one aligned dword store
        const bool own_c = cA < own_c1;
        const int nown = min(4, own_c1 - cA);
        if ((upitch & 15u) == 0) {
            // a 16-byte multiple pitch gives every staged row the first row's misalignment mb: folded into the lane's
            // column offsets once, so a row's four byte addresses are one multiply-add and four adds
            int sxm[4];
#pragma unroll
            for (int k = 0; k < 4; k++) sxm[k] = sxA[k] + (int)mb;
            for (int rr = rga; rr < nrA; rr += G) {
                const int4 yt = YA[rr];
                const int r = ar0 + rr;
                const int r0 = yt.x, r1 = yt.y;
                const uint32_t packed = og_rz_quad<FX>(S + __umul24((unsigned)r0, (unsigned)g.SC),
                                                       S + __umul24((unsigned)r1, (unsigned)g.SC), sxm, wtA,
                                                       (unsigned)yt.z, (unsigned)yt.w);
                *(uint32_t*)&A[rr * g.AC + 4 * qa] = packed;
                if (r < own_r1 && own_c) og_rz_store4(DA + (__umul24((unsigned)r, (unsigned)pitchA) + (unsigned)cA), packed, nown);
            }
        } else {
            for (int rr = rga; rr < nrA; rr += G) {
                const int4 yt = YA[rr];
                const int r = ar0 + rr;
                const int r0 = yt.x, r1 = yt.y;
                const unsigned m0 = (unsigned)mis[r0], m1 = (unsigned)mis[r1];
                const uint32_t packed = og_rz_quad<FX>(S + __umul24((unsigned)r0, (unsigned)g.SC) + m0,
                                                       S + __umul24((unsigned)r1, (unsigned)g.SC) + m1, sxA, wtA,
                                                       (unsigned)yt.z, (unsigned)yt.w);
                *(uint32_t*)&A[rr * g.AC + 4 * qa] = packed;
                if (r < own_r1 && own_c) og_rz_store4(DA + (__umul24((unsigned)r, (unsigned)pitchA) + (unsigned)cA), packed, nown);
            }
        }
    }
    __syncthreads();
    // ---- level B tile from the A region
    if (dxt >= g.bw) return;
#pragma unroll
    for (int k = 0; k < 4; k++) og_rz_weights<FX>(g.xtabB, g.xmaxB, min(dxt + k, g.bw - 1), ac0, sxB, wtB, k);
    const int n = min(4, g.bw - dxt);
    uint8_t* DB = dstB + (long long)f * dst_fstride + dxt;
    // the wave's 4 output rows read nondecreasing A rows, and consecutive outputs share one (a 1.2 downscale: ~5
    // distinct rows for 4 outputs): each distinct row's 4 horizontal sums are formed once and kept for the next
    // output (the rows are wave-uniform, so every reuse test is a scalar branch)
    const int rgu = __builtin_amdgcn_readfirstlane(rg);
    constexpr bool MH = !FX;  // sums kept as (d >> 4) << 8 for the multiply-high vertical form
    auto hsum = [&](int row, uint32_t (&h)[4]) {
        const uint8_t* R = A + __umul24((unsigned)(row - ar0), (unsigned)g.AC);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t pr = (uint32_t)R[sxB[k]] | ((uint32_t)R[sxB[k] + 1] << 16);
            const uint32_t d = __builtin_amdgcn_udot2(__builtin_bit_cast(og_rz_u16x2, pr), wtB[k], 0u, false);
            h[k] = MH ? (d & ~0xffu) : d;
        }
    };
    uint32_t hx[4] = {0u, 0u, 0u, 0u}, hy[4] = {0u, 0u, 0u, 0u};  // sums of rows rx < ry, the last output's two rows
    int rx = -1, ry = -1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = 4 * rgu + q;
        if (r >= nyB) break;
        // the row's table entry is wave-uniform: one scalar load (constant address space) into SGPRs, so its row
        // addresses and reuse tests are scalar work
#if defined(__HIP_DEVICE_COMPILE__)
        const int4 yt = ((const __attribute__((address_space(4))) int4*)g.ytabB)[by0 + r];
#else
        const int4 yt = g.ytabB[by0 + r];  // (host pass of the device function: never called)
#endif
        uint32_t h0[4], h1[4];
        if (yt.x == ry) {
#pragma unroll
            for (int k = 0; k < 4; k++) h0[k] = hy[k];
        } else if (yt.x == rx) {
#pragma unroll
            for (int k = 0; k < 4; k++) h0[k] = hx[k];
        } else {
            hsum(yt.x, h0);
        }
        if (yt.y == yt.x) {
#pragma unroll
            for (int k = 0; k < 4; k++) h1[k] = h0[k];
        } else if (yt.y == ry) {
#pragma unroll
            for (int k = 0; k < 4; k++) h1[k] = hy[k];
        } else {
            hsum(yt.y, h1);
        }
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (MH)
                og_rz_put_shr2(packed, og_mulhi_u24((unsigned)yt.z << 8, h0[k]) + og_mulhi_u24((unsigned)yt.w << 8, h1[k]) + 2u, k);
            else
                packed |= og_rz_vert<FX>((unsigned)yt.z, h0[k], (unsigned)yt.w, h1[k]) << (8 * k);
        }
        og_rz_store4(DB + __umul24((unsigned)(by0 + r), (unsigned)pitchB), packed, n);
        rx = yt.x;
        ry = yt.y;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            hx[k] = h0[k];
            hy[k] = h1[k];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k2: FAST cells (src/ORBextractor.cc:789-829 + cv::FAST TYPE_9_16 with nonmax suppression)
// ------------------------------------------------------------------------------------------------
// M(p) = max over the 16 contiguous 9-arcs and both polarities of min |I(p) - I(arc)|; the pixel is a
// FAST corner at threshold t iff M > t and then cornerScore<16> == M - 1.  Per polarity on the
// circle values themselves: the dark score is v - A with A = min_k max_arc c, the bright one B - v with
// B = max_k min_arc c.  The bright score is the dark form on complemented values, so one polarity's instructions
// serve both.  A survivor of the quick test at tq
// that fails one polarity's quick test has that polarity's score <= tq, and scores <= tq never decide anything
// (a kept corner needs M > max(t, 1) >= tq and then beats every neighbour <= tq), so the passing polarity's
// score stands for M; the rare survivors passing both take the max of the two.  Each 9-arc [k, k+8] is the
// max3 of the 3-arcs at k, k+3, k+6, exact.  (The scalar integer form of this score, og_fast_M1, was the reference
// og_fast_Mpk was checked against bit for bit until round 5; it is in git history.  The CPU restatement of
// cornerScore<16> is the checker the GPU tests hold every keypoint response to.)


// The same score on the f16-biased quad ROI (0x6400 | pixel = the f16 value 1024 + pixel) with packed f16 ops: the
// opposite samples (c_k, c_k+8) share a dword, so one v_pk_maximum3_f16 forms two 3-arc maxima (k and k + 8) and
// the arcs that wrap past c_15 take the swapped halves (op_sel).  The polarity is a per-lane sign: the bright score
// B - v = max_k min_arc(c) - v is the dark form v' - min_k max_arc(c') on c' = -c, v' = -v, so both polarities run
// the same instructions.  All values are integers of magnitude < 2048 (exact in f16): exact integer arithmetic.
// p = the centre's u16 in the quad ROI; SX = element step of one column, st = of one row.
typedef _Float16 og_h2 __attribute__((ext_vector_type(2)));
// base = LDS byte address of the sample 3 rows up and 3 columns left of the centre; FQ_S_ = row stride in qwords
// (one pixel column of the quad ROI is 4 u16 = 8 bytes).  The compiler packs each pair (c_k, c_k+8) with one v_perm
// (D16 loads cannot do it here: with SRAMECC, gfx950's ds_read_u16_d16[_hi] clear the other half).
#define OG_MPK_OFF(dy, dx) (8 * ((3 + (dy)) * FQ_S_ + 3 + (dx)))
template <int FQ_S_>
__device__ __forceinline__ int og_fast_Mpk(uint32_t base, uint32_t sgm)
{
    uint32_t w[8];
    uint32_t vc;
    {
        typedef const __attribute__((address_space(3))) _Float16 lds_h;
        lds_h* q = (lds_h*)(uintptr_t)(base + OG_MPK_OFF(0, 0));
        constexpr int st = 4 * FQ_S_, SX = 4;
        const _Float16 c[16] = {q[3 * st],      q[1 * SX + 3 * st], q[2 * SX + 2 * st],  q[3 * SX + 1 * st],
                                q[3 * SX],      q[3 * SX - 1 * st], q[2 * SX - 2 * st],  q[1 * SX - 3 * st],
                                q[-3 * st],     q[-1 * SX - 3 * st], q[-2 * SX - 2 * st], q[-3 * SX - 1 * st],
                                q[-3 * SX],     q[-3 * SX + 1 * st], q[-2 * SX + 2 * st], q[-1 * SX + 3 * st]};
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = __builtin_bit_cast(uint32_t, og_h2{c[k], c[k + 8]});
        vc = __builtin_bit_cast(uint16_t, q[0]);
    }
    // the polarity as a sign flip of both halves (sgm = 0 or 0x80008000): one 2-cycle v_xor_b32 per pair where a
    // v_pk_mul_f16 by -1 is a 4-cycle one (profiles/r05_valu_issue_rates.txt); -x is exactly x * -1, zeros included
    og_h2 P[8];
#pragma unroll
    for (int k = 0; k < 8; k++) P[k] = __builtin_bit_cast(og_h2, w[k] ^ sgm);
    const _Float16 v = __builtin_bit_cast(og_h2, vc ^ sgm).x;
#define OG_SW(a) __builtin_shufflevector(a, a, 1, 0)
#define OG_MX3(a, b, c) __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c)
#define OG_MN3(a, b, c) __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c)
    // X_k = (max c_k..c_k+2, max c_k+8..c_k+10)
    const og_h2 X0 = OG_MX3(P[0], P[1], P[2]), X1 = OG_MX3(P[1], P[2], P[3]), X2 = OG_MX3(P[2], P[3], P[4]);
    const og_h2 X3 = OG_MX3(P[3], P[4], P[5]), X4 = OG_MX3(P[4], P[5], P[6]), X5 = OG_MX3(P[5], P[6], P[7]);
    const og_h2 X6 = OG_MX3(P[6], P[7], OG_SW(P[0])), X7 = OG_MX3(P[7], OG_SW(P[0]), OG_SW(P[1]));
    // Y_k = (max of the 9-arc at k, at k + 8) = max(X_k, X_k+3, X_k+6)
    const og_h2 Y0 = OG_MX3(X0, X3, X6), Y1 = OG_MX3(X1, X4, X7), Y2 = OG_MX3(X2, X5, OG_SW(X0));
    const og_h2 Y3 = OG_MX3(X3, X6, OG_SW(X1)), Y4 = OG_MX3(X4, X7, OG_SW(X2));
    const og_h2 Y5 = OG_MX3(X5, OG_SW(X0), OG_SW(X3)), Y6 = OG_MX3(X6, OG_SW(X1), OG_SW(X4));
    const og_h2 Y7 = OG_MX3(X7, OG_SW(X2), OG_SW(X5));
    const og_h2 Z = OG_MN3(OG_MN3(Y0, Y1, Y2), OG_MN3(Y3, Y4, Y5), __builtin_elementwise_minimum(Y6, Y7));
#undef OG_SW
#undef OG_MX3
#undef OG_MN3
    const _Float16 A = __builtin_elementwise_minimum(Z.x, Z.y);
    const int M = (int)(short)(v - A);  // an integer in [-255, 255]
    return M > 0 ? M : 0;
}
#undef OG_MPK_OFF

// OpenCV FAST_t quick rejection (src: cv::FAST, pairs {k, k+8}): a pixel can only be a corner at
// threshold t if for every opposite pair one pixel is darker than v-t (resp. brighter than v+t).
// Necessary condition => every pixel that fails it has M <= t.  Restated threshold-free:
//   dark(t)   <=>  max_k min(c_k, c_k+8) < v - t,   bright(t) <=> min_k max(c_k, c_k+8) > v + t.
// Two pixels at once: each dword holds two pixels as u16 halves 0x6400 | pixel = the f16 value 1024 + pixel
// (exact, monotone), so the packed f16 ops of gfx950 apply and v_pk_maximum3/minimum3_f16 reduce the 8 pair
// minima (maxima) in 4 ops.  All values are integers below 2048 (exact in f16) and x - x = +0, so a half of the
// returned {dmax - (v - t), (v + t) - bmin} dwords is negative (sign bit set) iff that pixel passes that
// polarity's test, and a half of their packed minimum iff the pixel passes either.
typedef unsigned short og_u16x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------------------------
// k2: FAST over blocks of up to 2x2 cells.  The cells' detection areas tile a level without overlap
// (cell j covers [minB + j*wCell + 3, minB + (j+1)*wCell + 3); only the last row/column is clipped), so a
// block's detection area is the union and a pixel's cell is (i >= hCell, j >= wCell).  Every per-cell rule
// of src/ORBextractor.cc:789-829 + cv::FAST is kept: the NMS only sees corners of the same cell, and each
// cell falls back to minThFAST on its own.  One 512-thread workgroup per block: 4x fewer workgroups, one
// global reservation per block, 15 % less halo than per-cell ROIs.
// ------------------------------------------------------------------------------------------------
#define FB_NT 512
#define FB_NW (FB_NT / 64)
#define FB_MW 80                 // detection height capacity of a block (2 x 40 or 1 x 64); width <= 64
#define FB_MSW (FB_MW + 3)       // score map stride: a zero gap column before, between and after the cells
#define FB_MSZ ((FB_MSW * FB_MSW + 15) & ~15)  // 16-byte multiple: zeroed by 16-byte stores
#define FB_FCHUNK 64u            // frames per dispatch chunk of og_fast_quad_kernel (a multiple of 8; 16-128 measured,
                                 // profiles/sweeps/r06_ab_fast_chunk_size.txt)

// score-map index of detection pixel (i, j): one zero row/column separates the block's cells and surrounds
// them, so a pixel's 8 neighbours outside its cell (or outside the detection area) read 0 without checks
__device__ __forceinline__ int og_ms_idx(int i, int j, int wC, int hC)
{
    return (i + 1 + (i >= hC)) * FB_MSW + (j + 1 + (j >= wC));
}

// c[k] = circle sample k (f16-biased pixel pairs, cv::FAST's offsets; only the opposite pairs {k, k+8} matter),
// pv = centre.  The pair minima / maxima reduce as trees (depth 3 instead of a chain of 8).
__device__ __forceinline__ uint2 og_fast_quick2v(const uint32_t (&c)[16], uint32_t pv, og_u16x2 tt)
{
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 v = __builtin_bit_cast(h2, pv);
    const h2 t = {(_Float16)tt.x, (_Float16)tt.y};
    h2 mn[8], mx[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        mn[k] = __builtin_elementwise_minimum(__builtin_bit_cast(h2, c[k]), __builtin_bit_cast(h2, c[k + 8]));
        mx[k] = __builtin_elementwise_maximum(__builtin_bit_cast(h2, c[k]), __builtin_bit_cast(h2, c[k + 8]));
    }
#define OG_MAX3(a, b, c) __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c)
#define OG_MIN3(a, b, c) __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c)
    const h2 dmax = OG_MAX3(OG_MAX3(mn[0], mn[1], mn[2]), OG_MAX3(mn[3], mn[4], mn[5]), __builtin_elementwise_maximum(mn[6], mn[7]));
    const h2 bmin = OG_MIN3(OG_MIN3(mx[0], mx[1], mx[2]), OG_MIN3(mx[3], mx[4], mx[5]), __builtin_elementwise_minimum(mx[6], mx[7]));
#undef OG_MAX3
#undef OG_MIN3
    const h2 dark = dmax - (v - t), bright = (v + t) - bmin;  // negative: passes
    return make_uint2(__builtin_bit_cast(uint32_t, dark), __builtin_bit_cast(uint32_t, bright));
}

// lanes whose u16 low half is negative as an i16 (one v_cmp on the low 16 bits)
__device__ __forceinline__ u64 og_lanes_lo16_neg(uint32_t a)
{
    u64 m;
    __asm__("v_cmp_gt_i16_e64 %0, 0, %1" : "=s"(m) : "v"(a));
    return m;
}

// block table reads through the constant address space: uniform, so one scalar load (through a generic pointer
// the compiler cannot prove the table unclobbered by the kernel's own stores and falls back to vector loads).  The
// fields are taken from the 8 dwords with shifts (a bit_cast to the mixed-width struct costs ~50 scalar byte ops).
typedef unsigned int og_u32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ og_u32x8 og_fast_block(const OgFastBlk* blocks, int b)
{
    static_assert(sizeof(OgFastBlk) == 32, "OgFastBlk is read as one dwordx8");
    static_assert(offsetof(OgFastBlk, y0) == 8 && offsetof(OgFastBlk, rw) == 12 && offsetof(OgFastBlk, cand_off) == 16 &&
                      offsetof(OgFastBlk, ox) == 24 && offsetof(OgFastBlk, colw) == 28,
                  "OgFastBlk field offsets");
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(4))) og_u32x8*)blocks)[b];
#else
    og_u32x8 r;
    __builtin_memcpy(&r, blocks + b, 32);  // (host pass of the device function: never called)
    return r;
#endif
}

// Survivor stores of one stage-1 iteration: entry v_k to LDS byte address a_k from the lanes of m_k only (entries
// 1 and 3 from the high halves of v_1, v_3).  One exec save, then exec = saved & m_k around each store, one restore.
__device__ __forceinline__ void og_ds_write_b16_x4(u64 m0, uint32_t a0, uint32_t v0, u64 m1, uint32_t a1, uint32_t v1,
                                                   u64 m2, uint32_t a2, uint32_t v2, u64 m3, uint32_t a3, uint32_t v3)
{
    u64 sv;
    __asm__ volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_and_b64 exec, %0, %1\n\tds_write_b16 %2, %3\n\t"
        "s_and_b64 exec, %0, %4\n\tds_write_b16_d16_hi %5, %6\n\t"
        "s_and_b64 exec, %0, %7\n\tds_write_b16 %8, %9\n\t"
        "s_and_b64 exec, %0, %10\n\tds_write_b16_d16_hi %11, %12\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(sv)
        : "s"(m0), "v"(a0), "v"(v0), "s"(m1), "v"(a1), "v"(v1), "s"(m2), "v"(a2), "v"(v2), "s"(m3), "v"(a3), "v"(v3)
        : "memory");
}

// One FAST block as the kernel works on it, decoded from its OgFastBlk record (scalar registers)
struct OgFB {
    int l, rw, rh, dw, dh, wC, hC, cand_off, cand_cap, ox, oy, mis;
    unsigned colw;       // OgFastBlk::colw
    unsigned upitch;     // < 2^24 (checked on the host)
    bool aligned;        // row pitch a multiple of 4
    const uint8_t* row0; // ROI pixel (0, 0) of frame f
};

__device__ __forceinline__ OgFB og_fast_decode(const OgFastBlk* blocks, int p, unsigned f, const uint8_t* img0,
                                               long long pitch0, long long fstride0, const uint8_t* pyr,
                                               long long pyr_per_frame)
{
    const og_u32x8 bk = og_fast_block(blocks, p);
    OgFB b;
    b.l = (int)bk[2] >> 16;
    b.rw = bk[3] & 255;
    b.rh = (bk[3] >> 8) & 255;
    b.dw = b.rw - 6;
    b.dh = b.rh - 6;
    b.wC = (bk[3] >> 16) & 255;
    b.hC = bk[3] >> 24;
    b.cand_off = (int)bk[4];
    b.cand_cap = (int)bk[5];
    b.ox = (int)(short)(bk[6] & 0xffffu);
    b.oy = (int)bk[6] >> 16;
    b.colw = bk[7];
    if (b.l == 0) {
        b.upitch = (unsigned)pitch0 & (OG_MAX_PITCH - 1);
        b.row0 = img0 + (unsigned long long)f * (unsigned long long)fstride0 +
                 (unsigned long long)((bk[2] & 0xffffu) * b.upitch) + bk[0];
    } else {
        b.upitch = bk[1];
        b.row0 = pyr + (unsigned long long)f * (unsigned long long)pyr_per_frame + bk[0];
    }
    b.aligned = (b.upitch & 3) == 0;
    b.mis = b.aligned ? (int)((uintptr_t)b.row0 & 3) : 0;
    return b;
}

// ------------------------------------------------------------------------------------------------
// k2 (quad layout): the ROI is stored as u16 quads: qword (r, x) of roiq holds ROI pixels (r, x), (r, x + 16),
// (r, x + 32), (r, x + 48).  One ds_read_b64 (2 LDS cycles) then gives one circle sample of four pixels.
// Lane L of a wave takes quad column c = L & 15 of ROI row R + {0, 4, 1, 5}[L >> 4]: the two 16-lane row groups of
// each 32-lane LDS access are 4 rows = 112 qwords = 16 (mod 32) apart, so every b64 access is bank-conflict free.
// ------------------------------------------------------------------------------------------------
#define FQ_S 28     // quad-ROI row stride in qwords (>= 16 + 6 + 3 misalignment; 4 * FQ_S = 16 mod 32)
#define FQ_ROWS 86  // ROI rows (detection <= 80 + 6)

__device__ __forceinline__ void og_fastq_roi_load(const OgFB& b, int tid, uint32_t (&s)[2][4])
{
    // item (row, group of 4 qwords): 4 dword loads (one per 16-column segment), 8 v_perm into 4 quads, two 16-byte
    // LDS stores.  Columns past the ROI hold image bytes to its right (never read by a detection pixel); rows past it
    // are not stored.  The loads are unconditional (no exec branches): rows past the ROI re-read its last row.
    // Addresses: the block's uniform row base (SGPRs) plus a 32-bit per-lane offset (saddr + voffset loads).  The
    // pitch test is one uniform branch around all the loads (not one per load), and every load of a path is issued
    // before the first use.
    const int nq4 = (16 + 6 + b.mis + 3) >> 2;  // groups of 4 qwords per row (<= 7)
    const int q4 = min(tid & 7, nq4 - 1);
    const uint8_t* rbase = b.row0 - b.mis;
    unsigned off[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int r = min((tid >> 3) + 64 * k, b.rh - 1);
        off[k] = __umul24((unsigned)r, b.upitch) + 4u * (unsigned)q4;  // upitch < 2^24, r < 128
        __asm__("" : "+v"(off[k]));  // a 32-bit lane offset (saddr + voffset loads)
    }
    if (b.aligned) {
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int g = 0; g < 4; g++) s[k][g] = *(const uint32_t*)(rbase + off[k] + 16u * g);
    } else {
        // odd pitch: two aligned loads funnel-shifted by the row's offset
        const unsigned mb = (unsigned)((uintptr_t)rbase & 3);
        const uint8_t* abase = rbase - mb;
        uint32_t lo[2][4], hi[2][4];
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const unsigned o = off[k] + 16u * g + mb;
                const uint32_t* a = (const uint32_t*)(abase + (o & ~3u));
                lo[k][g] = a[0];
                hi[k][g] = a[1];
            }
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int g = 0; g < 4; g++) s[k][g] = __builtin_amdgcn_alignbyte(hi[k][g], lo[k][g], (off[k] + mb) & 3u);
    }
}

__device__ __forceinline__ void og_fastq_roi_put(const OgFB& b, int tid, const uint32_t (&s)[2][4], uint2* roiq)
{
    const int nq4 = (16 + 6 + b.mis + 3) >> 2;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int r = (tid >> 3) + 64 * k;
        if (r < b.rh && (tid & 7) < nq4) {
            uint32_t w[8];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                // quad t: byte t of segments 0..3 as four u16 (f16 1024 + pixel, og_fast_quick2v)
                const uint32_t sel = 0x0c000c00u | ((4u + t) << 16) | t;
                w[2 * t] = __builtin_amdgcn_perm(s[k][1], s[k][0], sel) | 0x64006400u;
                w[2 * t + 1] = __builtin_amdgcn_perm(s[k][3], s[k][2], sel) | 0x64006400u;
            }
            uint4* d = (uint4*)&roiq[r * FQ_S + 4 * (tid & 7)];
            d[0] = make_uint4(w[0], w[1], w[2], w[3]);
            d[1] = make_uint4(w[4], w[5], w[6], w[7]);
        }
    }
}

#ifndef OG_FAST_PROFILE
#define OG_FAST_PROFILE 0  // 1: diagnostic clocks (variant "fastprof", tests/test_gpu_variants.py)
#endif
#if OG_FAST_PROFILE  // diagnostic builds only (tools/fast_profile.py): per-phase clocks of every block of the middle frame
__device__ unsigned long long og_fast_prof[4096 * 8];
#define FAST_PROF(slot)                                                                                         \
    do {                                                                                                        \
        if (tid == 0 && f == (unsigned)nframes / 2 && p < 4096) og_fast_prof[p * 8 + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define FAST_PROF(slot) \
    do {                \
    } while (0)
#endif

// One block per workgroup.  Stage 1: quick test of every detection pixel and a survivor list; stage 2: exact scores
// into the score map; stage 3: same-cell NMS at both thresholds and per-cell counts; stage 4: the reference's
// per-cell 20 -> 7 fallback, one global reservation per block and the candidate stores.
// (8 waves per SIMD: 64 VGPRs.  Prefetching a second block's ROI under a relaxed budget of 4 waves per SIMD measured
// 2.2x (registers) and 1.6x (LDS-DMA) the FAST time: profiles/sweeps/r05_ab_fast_cell_prefetch_describe_kp2_mono.txt)
__global__ __launch_bounds__(FB_NT) __attribute__((amdgpu_waves_per_eu(8, 8))) void og_fast_quad_kernel(
    const OgFastBlk* __restrict__ blocks, int nb, const uint8_t* __restrict__ img0, long long pitch0, long long fstride0,
    const uint8_t* __restrict__ pyr, long long pyr_per_frame, u64* __restrict__ cand, long long cand_per_frame,
    int* __restrict__ cand_count, int nlevels, int thr, int* __restrict__ status, int nframes)
{
    __shared__ __attribute__((aligned(16))) uint2 roiq[FQ_ROWS * FQ_S];
    __shared__ __attribute__((aligned(16))) uint8_t Ms[FB_MSZ];
    __shared__ uint16_t lst[FB_MW * FB_MW];    // survivors (i << 7) | j; bits 14/15: dark/bright passes (stages 1-2),
                                               // then kept at t1/t2 (stages 3-4)
    __shared__ int sh_ns;
    __shared__ __attribute__((aligned(16))) int wk[FB_NW][8];  // per wave: kept at t1 per cell [0..3], at t2 [4..7]
    __shared__ int sh_base, sh_nk, sh_out;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    // grid (G, blocks, chunks), G = min(B, FB_FCHUNK): the dispatch order (x fastest) interleaves the G frames of a
    // chunk, so every block of frame f runs on XCD f % 8 and shares that L2 with its neighbours (G a multiple of 8
    // when B >= 8; FAST -0.7 % against frame-major order, profiles/sweeps/r05_ab_fast_frame_interleave.txt), and a
    // frame's neighbouring blocks, which share halo lines, are dispatched G workgroups apart rather than B.  With the
    // frames interleaved over a whole 512-frame batch the launch fetched 9.8 GB, 3.1x its pixel bytes; chunks of 64
    // fetch 3.2 GB (profiles/sweeps/r06_ab_fast_chunk.txt).  No division in the index.
    const unsigned f = blockIdx.z * gridDim.x + blockIdx.x;
    if (f >= (unsigned)nframes) return;  // the last chunk's unused frame slots
    const int t1 = thr & 255, t2 = (thr >> 8) & 255;  // clamped to [0, 255] on the host
    const int tq = min(t1, t2);
    const og_u16x2 tt = {(unsigned short)tq, (unsigned short)tq};
    const int tA = max(t1, 1), tB = max(t2, 1);
    const uint32_t a_ns = og_lds_addr(&sh_ns), a_lst = og_lds_addr(&lst[0]);
    const int p = (int)blockIdx.y;
    // every kernel argument the block decode reads is fetched before the first of them is used: one scalar-cache round
    // trip (the compiler's order took three before the block record)
    __asm__ volatile("" ::"s"(blocks), "s"(nb), "s"(img0), "s"(pitch0), "s"(fstride0), "s"(pyr), "s"(pyr_per_frame));
    if (p >= nb) return;
    const OgFB b = og_fast_decode(blocks, p, f, img0, pitch0, fstride0, pyr, pyr_per_frame);
    FAST_PROF(0);
    uint32_t sroi[2][4];
    og_fastq_roi_load(b, tid, sroi);
    {
        // zero only the score-map rows the block reads (dh + 3: gap rows included), while the ROI loads are in flight
        const int msz = min(FB_MSZ, ((b.dh + 3) * FB_MSW + 15) & ~15);
        for (int idx = tid * 16; idx < msz; idx += FB_NT * 16) *(uint4*)&Ms[idx] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid == 0) sh_ns = 0;
    og_fastq_roi_put(b, tid, sroi, roiq);
    __syncthreads();
    FAST_PROF(1);
    const int dh = b.dh, wC = b.wC, hC = b.hC;  // (the block's width enters through its column masks, b.colw)
    const uint2* Tq = roiq + b.mis;  // Tq[r * FQ_S + x] = quad (x, x + 16, x + 32, x + 48) of ROI row r
    // ---- stage 1: quick test on every detection pixel, four per lane.  Unit u = (row group g = u >> 1, half
    // h = u & 1) covers ROI rows 8g + 2h + {0, 4, 1, 5} (the lane's 16-lane group picks one); wave w takes units
    // w, w + 8, ...  Column masks are per-block constants, row masks scalars; one LDS reservation per unit.
    {
        const int lg = lane >> 4, c = lane & 15;
        const int lrow = ((lg & 1) << 2) | (lg >> 1);  // 0, 4, 1, 5
        const uint2* Tl = &Tq[(lrow + 3) * FQ_S + (c + 3)];
        const uint32_t e_lane = (uint32_t)((lrow << 7) | c), e_hi = (e_lane + 16u) << 16;
        // lanes whose column c (lane & 15) is below segment k's column count (the block record's byte k, in [0, 16]),
        // in all four 16-lane groups
        auto cmask = [&](int k) -> u64 {
            const unsigned m16 = (1u << ((b.colw >> (8 * k)) & 31u)) - 1u;
            const unsigned m32 = m16 * 0x10001u;
            return ((u64)m32 << 32) | m32;
        };
        const u64 col0 = cmask(0), col1 = cmask(1), col2 = cmask(2), col3 = cmask(3);
        const int nunits = ((dh + 7) >> 3) * 2;
        // wave w takes units u = w, w + 8, ...: their first rows R = 8 (u >> 1) + 2 (u & 1) step by 32 (uniform)
        const int Rlim = 8 * (nunits >> 1) + 2 * (wvu & 1);
        for (int R = 8 * (wvu >> 1) + 2 * (wvu & 1); R < Rlim; R += 4 * FB_NW) {
            const bool full = R + 5 < dh;
            // (tail: lanes whose row is past the area read rows below the ROI -- inside the LDS allocation, at most
            // 11 rows past row 80 -- and are masked out)
            const uint2* q = Tl + R * FQ_S;
            uint32_t c0[16], c1[16];
            unsigned long long w[17];
            {
                // volatile 64-bit loads: never paired into ds_read2_b64 (8 cycles per pair instead of 2 per read),
                // issued in order (opposite samples k, k + 8 adjacent, centre first), each waited for only where it
                // is used (partial lgkmcnt waits)
                const int st = FQ_S;
                const int off[17] = {3 * st,      1 + 3 * st,  2 + 2 * st,  3 + 1 * st, 3,          3 - 1 * st,
                                     2 - 2 * st,  1 - 3 * st,  -3 * st,     -1 - 3 * st, -2 - 2 * st, -3 - 1 * st,
                                     -3,          -3 + 1 * st, -2 + 2 * st, -1 + 3 * st, 0};
                typedef const volatile __attribute__((address_space(3))) unsigned long long lds_u64;
                lds_u64* q64 = (lds_u64*)(uintptr_t)og_lds_addr(q);
                w[16] = q64[0];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    w[k] = q64[off[k]];
                    w[k + 8] = q64[off[k + 8]];
                }
            }
#pragma unroll
            for (int k = 0; k < 16; k++) {
                c0[k] = (uint32_t)w[k];
                c1[k] = (uint32_t)(w[k] >> 32);
            }
            const uint2 ctr = make_uint2((uint32_t)w[16], (uint32_t)(w[16] >> 32));
            const uint2 r0 = og_fast_quick2v(c0, ctr.x, tt);  // pixels c, c + 16
            const uint2 r1 = og_fast_quick2v(c1, ctr.y, tt);  // pixels c + 32, c + 48
            // the column masks, restricted in a tail unit to its rows inside the area
            u64 cm0 = col0, cm1 = col1, cm2 = col2, cm3 = col3;
            if (!full) {
                const u64 rows = (R < dh ? 0xffffull : 0ull) | (R + 4 < dh ? 0xffff0000ull : 0ull) |
                                 (R + 1 < dh ? 0xffff00000000ull : 0ull) | (R + 5 < dh ? 0xffff000000000000ull : 0ull);
                cm0 &= rows;
                cm1 &= rows;
                cm2 &= rows;
                cm3 &= rows;
            }
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            auto pkmin = [](uint32_t x, uint32_t y) -> uint32_t {
                return __builtin_bit_cast(uint32_t, __builtin_elementwise_minimum(__builtin_bit_cast(h2, x),
                                                                                   __builtin_bit_cast(h2, y)));
            };
            const uint32_t a0 = pkmin(r0.x, r0.y), a1 = pkmin(r1.x, r1.y);
            const u64 m[4] = {og_lanes_lo16_neg(a0) & cm0, og_lanes_lt((int)a0, 0) & cm1, og_lanes_lo16_neg(a1) & cm2,
                              og_lanes_lt((int)a1, 0) & cm3};
            int cnt[4], n = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                cnt[k] = __popcll(m[k]);
                n += cnt[k];
            }
            if (n) {
                uint32_t old;
                u64 sv;
                // the reservation is issued, and waited for only after the entries and ranks are formed
                __asm__ volatile(
                    "s_mov_b64 %1, exec\n\ts_mov_b64 exec, 1\n\tds_add_rtn_u32 %0, %2, %3\n\ts_mov_b64 exec, %1"
                    : "=&v"(old), "=&s"(sv)
                    : "v"(a_ns), "v"(n)
                    : "memory");
                // entries: bits 14 / 15 of each half = the dark / bright sign bits of that pixel; the high pixels'
                // entries are built in the high half and stored by ds_write_b16_d16_hi
                const uint32_t base = e_lane + (uint32_t)(R << 7), hbase = e_hi + ((uint32_t)R << 23);
                const uint32_t X0 = ((r0.x >> 1) & 0x40004000u) | (r0.y & 0x80008000u);
                const uint32_t X1 = ((r1.x >> 1) & 0x40004000u) | (r1.y & 0x80008000u);
                const uint32_t v[4] = {X0 | base, X0 | hbase, X1 | (base + 32u), X1 | (hbase + (32u << 16))};
                const int c1 = cnt[0], c2 = c1 + cnt[1], c3 = c2 + cnt[2];
                const uint32_t k0 = (uint32_t)og_rank(m[0]), k1 = (uint32_t)og_rank(m[1], c1),
                               k2 = (uint32_t)og_rank(m[2], c2), k3 = (uint32_t)og_rank(m[3], c3);
                __asm__ volatile("s_waitcnt lgkmcnt(0)" : "+v"(old) : : "memory");
                const uint32_t ab = a_lst + 2u * (uint32_t)__builtin_amdgcn_readfirstlane(old);
                og_ds_write_b16_x4(m[0], ab + 2u * k0, v[0], m[1], ab + 2u * k1, v[1], m[2], ab + 2u * k2, v[2], m[3],
                                   ab + 2u * k3, v[3]);
            }
        }
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the asm list stores are not tracked by the compiler
    __syncthreads();
    FAST_PROF(2);
    const int ns = sh_ns;
    if (tid == 0) {
        sh_nk = 0;
        sh_out = 0;
    }
    // ---- stage 2: exact M for every survivor; single pixels are u16 reads of the quad layout (element step 4)
    const uint16_t* T16 = (const uint16_t*)Tq;
    for (int e = tid; e < ns; e += FB_NT) {
        const int ent = lst[e];
        const int i = (ent >> 7) & 127, j = ent & 127;
        const uint16_t* pc = &T16[4 * ((i + 3) * FQ_S + ((j & 15) + 3)) + (j >> 4)];
        const bool dark = (ent & 0x4000) != 0, bright = (ent & 0x8000) != 0;
        // the exact score with packed f16 pair ops (og_fast_Mpk)
        const uint32_t pb = og_lds_addr(pc) - 8u * (3u * FQ_S + 3u);
        int M = og_fast_Mpk<FQ_S>(pb, dark ? 0u : 0x80008000u);
        if (dark && bright) M = max(M, og_fast_Mpk<FQ_S>(pb, 0x80008000u));
        Ms[og_ms_idx(i, j, wC, hC)] = (uint8_t)M;
    }
    __syncthreads();
    FAST_PROF(3);
    // ---- stage 3: same-cell 3x3 NMS at both thresholds; each wave walks every 8th 64-entry chunk of the list.  The
    // entries kept at either threshold are compacted into the ROI buffer (free after stage 2) as (entry | kept at t1
    // << 14 | kept at t2 << 15 | M << 16), so that the emission walks those few instead of every survivor (a strict
    // 3x3 maximum per cell: at most 20 x 16 per cell, 1280 per block, against 4816 u32 of the buffer)
    int c1[4] = {0, 0, 0, 0}, c2[4] = {0, 0, 0, 0};
    uint32_t* kl = (uint32_t*)roiq;
    const uint32_t a_nk = og_lds_addr(&sh_nk);
    for (int e0 = wvu * 64; e0 < ns; e0 += FB_NT) {
        const int e = e0 + lane;
        int ent = 0, mc = 0, nbm = 0;
        if (e < ns) {
            ent = lst[e] & 0x3fff;
            const uint8_t* q = &Ms[og_ms_idx(ent >> 7, ent & 127, wC, hC) - FB_MSW - 1];
            mc = q[FB_MSW + 1];
            nbm = max(max(max(q[0], q[1]), max(q[2], q[FB_MSW])),
                      max(max(q[FB_MSW + 2], q[2 * FB_MSW]), max(q[2 * FB_MSW + 1], q[2 * FB_MSW + 2])));
        }
        const u64 top = og_lanes_gt(mc, nbm);
        const u64 K1 = og_lanes_gt(mc, tA) & top, K2 = og_lanes_gt(mc, tB) & top;
        const u64 ci = og_lanes_gt(ent >> 7, hC - 1), cj = og_lanes_gt(ent & 127, wC - 1);
        const u64 cm[4] = {~ci & ~cj, ~ci & cj, ci & ~cj, ci & cj};
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
            c1[cc] += __popcll(K1 & cm[cc]);
            c2[cc] += __popcll(K2 & cm[cc]);
        }
        const u64 K = K1 | K2;
        if (K) {  // wave-uniform
            uint32_t old;
            u64 sv;
            const int nk = __popcll(K);
            __asm__ volatile(
                "s_mov_b64 %1, exec\n\ts_mov_b64 exec, 1\n\tds_add_rtn_u32 %0, %2, %3\n\ts_mov_b64 exec, %1"
                : "=&v"(old), "=&s"(sv)
                : "v"(a_nk), "v"(nk)
                : "memory");
            // the entry and its rank while the reservation is in flight
            const uint32_t v = (uint32_t)ent | ((uint32_t)mc << 16) | (mc > tA ? 0x4000u : 0u) | (mc > tB ? 0x8000u : 0u);
            const int rk = og_rank(K);
            __asm__ volatile("s_waitcnt lgkmcnt(0)" : "+v"(old) : : "memory");
            const int kb = __builtin_amdgcn_readfirstlane(old);
            if ((K >> lane) & 1ull) kl[kb + rk] = v;
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
            wk[wv][cc] = c1[cc];
            wk[wv][4 + cc] = c2[cc];
        }
    }
    __syncthreads();
    FAST_PROF(4);
    // per cell: iniThFAST unless the cell is empty at it (src/ORBextractor.cc:809-816)
    const int qw = (lane >> 2) & (FB_NW - 1), qc = lane & 3;
    const int v1 = wk[qw][qc], v2 = wk[qw][4 + qc];
    const u64 nz1 = og_lanes_ne((unsigned)v1, 0u) & 0xffffffffull;
    unsigned useT2 = 0;
#pragma unroll
    for (int cc = 0; cc < 4; cc++) useT2 |= ((nz1 & (0x11111111ull << cc)) ? 0u : 1u) << cc;
    const int kw = ((useT2 >> qc) & 1u) ? v2 : v1;
    int ks = kw + __builtin_amdgcn_mov_dpp(kw, 0xb1, 0xf, 0xf, false);
    ks = ks + __builtin_amdgcn_mov_dpp(ks, 0x4e, 0xf, 0xf, false);
    const int kx = __shfl(ks, 4 * (lane & 7));
    int sc = kx;
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x111, 0xf, 0xf, true);
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x112, 0xf, 0xf, true);
    sc += __builtin_amdgcn_update_dpp(0, sc, 0x114, 0xf, 0xf, true);
    const int total = __builtin_amdgcn_readlane(sc, FB_NW - 1);
    const int nk = sh_nk;  // (written before the stage-3 barrier)
    // ---- stage 4: one reservation per block; each wave writes its kept entries at its offset
    int sb = 0;
    if (total != 0) {  // block-uniform
        if (tid == 0) {
            const int bb = atomicAdd(&cand_count[f * nlevels + b.l], total);
            if (bb + total > b.cand_cap) atomicOr(status, 1);  // cannot happen: cap is the exact NMS bound
            sh_base = bb;
        }
        __syncthreads();
        sb = sh_base;
    }
    FAST_PROF(5);
    // ---- emission: the kept entries of the compacted list (the cell's threshold picks the flag), each wave's at an
    // offset from one LDS counter (a block's candidates are unordered: every consumer orders them itself)
    const bool emit = total != 0 && sb + total <= b.cand_cap;
    u64* out = cand + (unsigned long long)f * (unsigned long long)cand_per_frame + (unsigned)(b.cand_off + sb);
    const uint32_t a_out = og_lds_addr(&sh_out);
    if (emit) {
        for (int e0 = wvu * 64; e0 < nk; e0 += FB_NT) {
            const int e = e0 + lane;
            const uint32_t ent = e < nk ? kl[e] : 0u;
            const int i = (ent >> 7) & 127, j = ent & 127;
            const int cell = (i >= hC) * 2 + (j >= wC);
            const unsigned kbit = ent & (((useT2 >> cell) & 1u) ? 0x8000u : 0x4000u);
            const u64 mask = og_lanes_ne(kbit, 0u);
            if (mask) {  // wave-uniform
                uint32_t old;
                u64 sv;
                const int n = __popcll(mask);
                __asm__ volatile(
                    "s_mov_b64 %1, exec\n\ts_mov_b64 exec, 1\n\tds_add_rtn_u32 %0, %2, %3\n\ts_mov_b64 exec, %1"
                    : "=&v"(old), "=&s"(sv)
                    : "v"(a_out), "v"(n)
                    : "memory");
                const u64 cv = og_pack_cand(b.ox + j, b.oy + i, (int)(ent >> 16) - 1);
                const int rk = og_rank(mask);
                __asm__ volatile("s_waitcnt lgkmcnt(0)" : "+v"(old) : : "memory");
                const int ob = __builtin_amdgcn_readfirstlane(old);
                if (kbit) out[ob + rk] = cv;
            }
        }
    }
#if OG_FAST_PROFILE
    __builtin_amdgcn_s_waitcnt(0);  // the candidate stores issued
    FAST_PROF(6);
    if (tid == 0 && f == (unsigned)nframes / 2 && p < 4096) og_fast_prof[p * 8 + 7] = (unsigned long long)ns | ((unsigned long long)b.l << 32);
#endif
}

hipError_t og_read_fast_prof(unsigned long long* out, int n)
{
#if OG_FAST_PROFILE
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(og_fast_prof), sizeof(unsigned long long) * (size_t)std::min(n, 4096 * 8));
#else
    (void)out;
    (void)n;
    return hipErrorNotSupported;
#endif
}

// ------------------------------------------------------------------------------------------------
// k2b (option ORBGPU_SEM_SCORE_HARRIS, include/orbgpu.h; not part of ORB-SLAM2): the Harris response of every
// FAST candidate replaces its FAST score as the octree's ranking key.  The response is OpenCV's ORB
// HARRIS_SCORE (features2d orb.cpp HarrisResponses, blockSize 7, harris_k 0.04) at the candidate's level pixel;
// the candidate keeps its slot, only the key word (bits 32-63) is rewritten.
// ------------------------------------------------------------------------------------------------
// float -> u32 with the same order (the octree's atomicMax ranks keys); -0 (not produced: a, b >= 0) as +0
__device__ __forceinline__ unsigned og_harris_key(float r)
{
    const unsigned u = __float_as_uint(r);
    if (u == 0x80000000u) return 0x80000000u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float og_harris_unkey(unsigned k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// the response from the integer structure-tensor sums, in the published operation order, each product and sum
// rounded to float (no contraction): ((a*b - c*c) - (k*(a+b))*(a+b)) * scale^4, scale = 1/(4*7*255)
__device__ __forceinline__ float og_harris_response(int a, int b, int c)
{
#pragma clang fp contract(off)
    const float scale = 1.f / ((1 << 2) * 7 * 255.f);
    const float s4 = scale * scale * scale * scale;
    const float fa = (float)a, fb = (float)b, fc = (float)c;
    return (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * s4;
}

#define HR_NT 256
// workgroups per (frame, level): one per 2^15 candidate slots (the level's area / 4), 1 .. 32
__host__ __device__ inline int og_harris_groups(int cand_cap)
{
    const int g = cand_cap >> 15;
    return g < 1 ? 1 : (g > 32 ? 32 : g);
}

// one thread per candidate of levels [lb, le); grid (sum over those levels of og_harris_groups, B)
__global__ __launch_bounds__(HR_NT) void og_harris_kernel(OgPlan P, const uint8_t* __restrict__ img0, long long pitch0,
                                                          long long fstride0, const uint8_t* __restrict__ pyr,
                                                          u64* __restrict__ cand, const int* __restrict__ cand_count,
                                                          int lb, int le)
{
    const int f = blockIdx.y;
    int l = lb, g = blockIdx.x, ng = 1;
    for (; l < le; l++) {
        ng = og_harris_groups(P.lv[l].cand_cap);
        if (g < ng) break;
        g -= ng;
    }
    if (l >= le) return;
    const OgLevel& L = P.lv[l];
    const int n = min(cand_count[f * P.nlevels + l], L.cand_cap);
    const uint8_t* img;
    long long pitch;
    if (l == 0) {
        img = img0 + (long long)f * fstride0;
        pitch = pitch0;
    } else {
        img = pyr + (long long)f * P.pyr_per_frame + L.pyr_off;
        pitch = L.pitch;
    }
    uint32_t* K32 = (uint32_t*)(cand + (long long)f * P.cand_per_frame + L.cand_off);
    for (int k = g * HR_NT + (int)threadIdx.x; k < n; k += ng * HR_NT) {
        const uint32_t xy = K32[2 * k];
        // candidates lie >= 19 px inside the level (minB + 3), the 9 x 9 window reaches 4: no border handling
        const int x = (int)(xy & 0xffff) + L.minB, y = (int)(xy >> 16) + L.minB;
        int p[9][9];
#pragma unroll
        for (int r = 0; r < 9; r++) {
            // row r of the window from three aligned dwords (any pitch: each row has its own misalignment)
            const uint8_t* rp = img + (long long)(y - 4 + r) * pitch + (x - 4);
            const unsigned m = (unsigned)((uintptr_t)rp & 3);
            const uint32_t* q = (const uint32_t*)(rp - m);
            const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
            const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, m), w1 = __builtin_amdgcn_alignbyte(d2, d1, m);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                p[r][j] = (int)((w0 >> (8 * j)) & 0xff);
                p[r][4 + j] = (int)((w1 >> (8 * j)) & 0xff);
            }
            p[r][8] = (int)((d2 >> (8 * m)) & 0xff);
        }
        // 7 x 7 block of 3x3 Sobel-form gradients (integer sums: any order)
        int sa = 0, sb = 0, sc = 0;
#pragma unroll
        for (int i = 1; i < 8; i++)
#pragma unroll
            for (int j = 1; j < 8; j++) {
                const int ix = (p[i][j + 1] - p[i][j - 1]) * 2 + (p[i - 1][j + 1] - p[i - 1][j - 1]) +
                               (p[i + 1][j + 1] - p[i + 1][j - 1]);
                const int iy = (p[i + 1][j] - p[i - 1][j]) * 2 + (p[i + 1][j - 1] - p[i - 1][j - 1]) +
                               (p[i + 1][j + 1] - p[i - 1][j + 1]);
                sa += ix * ix;
                sb += iy * iy;
                sc += ix * iy;
            }
        K32[2 * k + 1] = og_harris_key(og_harris_response(sa, sb, sc));
    }
}

// ------------------------------------------------------------------------------------------------
// k3: octree (src/ORBextractor.cc:481-537, 539-763), one workgroup per (frame, level)
// ------------------------------------------------------------------------------------------------
struct OctNode {
    short x0, y0, x1, y1;
    int cnt;
    int cid;  // creation order == allocation order of the reference's list nodes
};

#define OCT_NT 1024

// inclusive scan over the 64 lanes (all active) with DPP, no LDS round trips: row_shr 1, 2, 4, 8 within rows of 16,
// then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the row totals
__device__ __forceinline__ int og_wave_incl_scan(int x)
{
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}

// exclusive block scan of one int per thread; returns the exclusive prefix, *total = sum.  Every wave scans the
// per-wave totals itself (no third barrier for a wave-0 pass).
__device__ __forceinline__ int og_block_excl_scan(int v, int* wsum, int* total)
{
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x = og_wave_incl_scan(v);
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    const int nw = blockDim.x >> 6;
    const int s = og_wave_incl_scan(lane < nw ? wsum[lane] : 0);
    const int before = w ? __builtin_amdgcn_readlane(s, w - 1) : 0;
    *total = __builtin_amdgcn_readlane(s, nw - 1);
    __syncthreads();
    return before + x - v;
}

__device__ __forceinline__ int og_quadrant(int x, int y, const OctNode& n)
{
    const int halfX = (n.x1 - n.x0 + 1) >> 1;  // ceil((float)(UR.x-UL.x)/2), exact for ints
    const int halfY = (n.y1 - n.y0 + 1) >> 1;
    const int mx = n.x0 + halfX, my = n.y0 + halfY;
    return x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
}

__device__ __forceinline__ OctNode og_child(const OctNode& p, int q)
{
    const int halfX = (p.x1 - p.x0 + 1) >> 1, halfY = (p.y1 - p.y0 + 1) >> 1;
    const int mx = p.x0 + halfX, my = p.y0 + halfY;
    OctNode c;
    c.x0 = (short)((q & 1) ? mx : p.x0);
    c.x1 = (short)((q & 1) ? p.x1 : mx);
    c.y0 = (short)((q & 2) ? my : p.y0);
    c.y1 = (short)((q & 2) ? p.y1 : my);
    c.cnt = 0;
    c.cid = 0;
    return c;
}

// candidate order key: (cell row, cell col, row in cell, col in cell) == vToDistributeKeys order
__device__ __forceinline__ unsigned og_cand_order(int x, int y, const OgLevel& L)
{
    const int ci = (y - 3) / L.hCell, cj = (x - 3) / L.wCell;
    const int ly = y - 3 - ci * L.hCell, lx = x - 3 - cj * L.wCell;
    return (unsigned)(((ci * L.nCols + cj) * L.hCell + ly) * L.wCell + lx);
}

// og_cand_order with the two divisions as multiply-high by m = floor((2^32 - 1) / d) + 1 (exact for n < 2^16 and
// d < 2^16; wCell, hCell <= 255 and level coordinates < 2^16 are checked by the plan)
__device__ __forceinline__ unsigned og_cand_order_m(int x, int y, const OgLevel& L, unsigned mW, unsigned mH)
{
    const unsigned yy = (unsigned)(y - 3), xx = (unsigned)(x - 3);
    const unsigned ci = __umulhi(yy, mH), cj = __umulhi(xx, mW);
    const unsigned ly = yy - ci * (unsigned)L.hCell, lx = xx - cj * (unsigned)L.wCell;
    return ((ci * (unsigned)L.nCols + cj) * (unsigned)L.hCell + ly) * (unsigned)L.wCell + lx;
}

// atomicMax(&ctr[addr], v) for every active lane, one LDS atomic per run of equal addresses: a segmented max with
// DPP (row_shr 1/2/4/8, then row_bcast 15/31, each step taking the shifted lane's value only when its address is
// the lane's own), after which the last lane of every run holds the run's maximum.  A shifted lane of another run
// with the same address only adds a value of the same counter, so merging it is harmless.  Wave-uniform control
// flow.  The final key pass's per-node maximum: its keys arrive in candidate order, so a wave's lanes fall into a
// few nodes and plain atomics serialise on them (~45 % of that pass, tools/octree_profile.py --variant noatom).
__device__ __forceinline__ void og_wave_max32(unsigned* ctr, int addr, unsigned v, bool act)
{
    const int a = act ? addr : -1;
    unsigned x = act ? v : 0u;
#define OG_SEGMAX_STEP(ctrl, rm)                                                                     \
    {                                                                                                \
        const int sa = __builtin_amdgcn_update_dpp(-2, a, ctrl, rm, 0xf, false);                     \
        const unsigned sx = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rm, 0xf, false); \
        x = (sa == a && sx > x) ? sx : x;                                                            \
    }
    OG_SEGMAX_STEP(0x111, 0xf)
    OG_SEGMAX_STEP(0x112, 0xf)
    OG_SEGMAX_STEP(0x114, 0xf)
    OG_SEGMAX_STEP(0x118, 0xf)
    OG_SEGMAX_STEP(0x142, 0xa)
    OG_SEGMAX_STEP(0x143, 0xc)
#undef OG_SEGMAX_STEP
    const int nxt = __builtin_amdgcn_update_dpp(-2, a, 0x130, 0xf, 0xf, false);  // wave_shl:1 (lane + 1)
    if (act && nxt != a) atomicMax(&ctr[addr], x);
}

// atomicAdd(&ctr[addr], 1) for every active lane, one LDS atomic per run of equal addresses among the active lanes:
// the wave's keys are consecutive FAST outputs (one block's corners), so neighbours share nodes and plain atomics
// would serialise on the same counters.  The first lane of each run adds the run's length.  Wave-uniform control
// flow; exact counts.  (The round-3 form, ballots over the two most common addresses and then plain atomics, is in
// git history.)
__device__ __forceinline__ void og_wave_count(int* ctr, int addr, bool act)
{
    const int lane = threadIdx.x & 63;
    const int a = act ? addr : -1;
    const int prev = __builtin_amdgcn_update_dpp(-1, a, 0x138, 0xf, 0xf, false);  // wave_shr:1 (lane - 1)
    const bool head = act && (lane == 0 || prev != a);
    const u64 heads = og_ballot(head);
    const u64 actm = og_ballot(act);
    if (head) {
        const u64 after = lane == 63 ? 0ull : (heads >> (lane + 1)) << (lane + 1);
        const int end = after ? __builtin_ctzll(after) : 64;  // next head (or past the wave)
        const u64 span = (end == 64 ? ~0ull : ((1ull << end) - 1ull)) & ~((1ull << lane) - 1ull);
        atomicAdd(&ctr[addr], (int)__popcll(actm & span));
    }
}

#define OCT_U 4  // candidates per thread per pass with all loads hoisted (latency batching; 8 and 16 measured in
                 // the table-mode count pass: profiles/sweeps/r05_ab_octree_count_unroll.txt)

#ifndef OG_OCT_PROFILE
#define OG_OCT_PROFILE 0  // l + 1: diagnostic clocks of level l (variant "octprof0", tests/test_gpu_variants.py)
#endif
#if OG_OCT_PROFILE  // diagnostic builds only (tools/octree_profile.py): per-round clocks of (frame 0, level OG_OCT_PROFILE - 1)
__device__ unsigned long long og_oct_prof[256];
#define OCT_PROF(slot, v)                                                                                    \
    do {                                                                                                     \
        if (tid == 0 && f == 0 && l == OG_OCT_PROFILE - 1 && (slot) < 256) og_oct_prof[(slot)] = (v);      \
    } while (0)
#else
#define OCT_PROF(slot, v) \
    do {                  \
    } while (0)
#endif

// levels [l0, l0 + gridDim.x / frames) of the launch, level-major, one list node per thread (OG_OCT_MAXL)
__global__ __launch_bounds__(OCT_NT) __attribute__((amdgpu_waves_per_eu(8, 8))) void og_octree_kernel(OgPlan P, int l0, const u64* __restrict__ cand,
                                                           const int* __restrict__ cand_count,
                                                           uint16_t* __restrict__ node_of,
                                                           unsigned* __restrict__ oct_best,
                                                           uint32_t* __restrict__ oct_xy,
                                                           uint32_t* __restrict__ oct_resp,
                                                           int* __restrict__ oct_count, int* __restrict__ status,
                                                           int nlaunch)
{
    __shared__ OctNode nodes[2][OG_OCT_MAXL];
    __shared__ uint8_t fresh[2][OG_OCT_MAXL];
    __shared__ int splitRank[OG_OCT_MAXL];
    __shared__ int splitNode[OG_OCT_MAXL];
    __shared__ int newPos[OG_OCT_MAXL];
    __shared__ int aux[OG_OCT_MAXL];
    // child counts, indexed 4*node + quadrant: one buffer -- a round's counts are consumed (split set,
    // children) before the key pass accumulates the next round's, with barriers in between; the last key
    // pass keeps the best key per node in the same storage.  ~74 KB of LDS in total: 2 workgroups per CU.
    __shared__ __attribute__((aligned(16))) int childCnt[4 * OG_OCT_MAXL];
    __shared__ __attribute__((aligned(16))) uint16_t childPos[4 * OG_OCT_MAXL];
    // final-phase planning only: the candidates' (size, creation id) keys, in the previous round's (dead) childPos
    u64* skey = (u64*)childPos;
    u64* best = (u64*)childCnt;  // [OG_OCT_MAXL], final key pass only
    // table mode (below): each list node's index in the depth tables (childCnt) / position table (childPos)
    __shared__ uint16_t npath[2][OG_OCT_MAXL];
    __shared__ int wsum[32];
    __shared__ int sv[16];

    // level-major dispatch order, level 0 first: the finest level has the most candidates (and rounds), so
    // its workgroups start in the first wave of residency instead of being interleaved with the short ones
    const int nb = (int)gridDim.x / nlaunch;  // frames in the launch
    const int l = l0 + (int)blockIdx.x / nb, f = (int)blockIdx.x % nb, tid = threadIdx.x;
    const OgLevel& L = P.lv[l];
    const int C = min(cand_count[f * P.nlevels + l], L.cand_cap);
    const u64* K = cand + (long long)f * P.cand_per_frame + L.cand_off;
    const uint32_t* K32 = (const uint32_t*)K;  // [2k] = x | y << 16, [2k+1] = response
    uint16_t* NO = node_of + (long long)f * P.cand_per_frame + L.cand_off;
    const int N = L.N;
    const int nIni = L.nIni;
    const int H = L.maxBY - L.minB;

    OCT_PROF(0, clock64());
    OCT_PROF(1, (unsigned long long)C);
    // ---- table mode.  A node's bounds follow from its root by the fixed halving of DivideNode (:481-537), so the
    // node containing a key at depth d is a function of the key alone: path p_0 = root, p_d = 4 p_(d-1) + quadrant.
    // ONE key pass counts every key at its depth-D node (D = the deepest depth whose tables of all depths fit the
    // 4 x OG_OCT_MAXL ints of childCnt); the counts of depths < D are sums of their children.  The rounds then read
    // their children counts from the tables instead of re-reading the keys (no per-round key pass), and NO[k] holds
    // the key's depth-D table index.  The last pass maps that index to the key's final node through a position
    // table (childPos) filled down from each listed node to its depth-D descendants.  A round whose next split
    // candidates include a depth-D node leaves table mode: one key pass moves NO[] to list positions and counts the
    // next children as the per-round passes below do (og_octree_profile: the level-0 workgroup's key passes were
    // ~60 % of its time, and each re-read every key -- DESIGN.md §5).
    int D = 0;
    {
        int tot = nIni, w = nIni;
        while (D < 7 && tot + 4 * w <= 4 * OG_OCT_MAXL) {
            w *= 4;
            tot += w;
            D++;
        }
    }
    // first table index of depth d: nIni (4^d - 1) / 3, and (4^d - 1) / 3 is 0b0101...01 (d ones)
    auto tbase = [nIni](int d) { return nIni * (int)(0x55555555u & ((1u << (2 * d)) - 1u)); };
    // a list node's npath entry: table index | depth << 12 (indices < 4 OG_OCT_MAXL = 2^12)
    auto tchild = [&](int e, int q) {  // the npath entry of child q
        const int t = e & 0xfff, d = e >> 12;
        return (tbase(d + 1) + 4 * (t - tbase(d)) + q) | ((d + 1) << 12);
    };
    const int Ttot = tbase(D + 1);
    bool tmode = D >= 1;  // workgroup-uniform
    const unsigned mW = 0xffffffffu / (unsigned)L.wCell + 1u, mH = 0xffffffffu / (unsigned)L.hCell + 1u;
    // the per-node best key in 32 bits when it fits: FAST score (8 bits) << 24 | 0xffffff - candidate order (the
    // order is below nRows hCell nCols wCell <= 2^24); the Harris option's 32-bit keys keep the 64-bit form
    const bool k32 = !(P.sem & ORBGPU_SEM_SCORE_HARRIS) &&
                     (unsigned)(L.nRows * L.hCell) * (unsigned)(L.nCols * L.wCell) <= 0xffffffu;
    unsigned* best32 = (unsigned*)childCnt;
    // cell-best table (table mode, 32-bit keys): the counting pass also keeps every depth-D cell's best key (in the
    // node buffers' LDS, free until the roots are listed) and parks the table in HBM (OG_OCT_BEST_CELLS u32 per frame
    // and level); the final phase then takes each listed node's best from its cells through the position table -- no
    // second pass over the keys.  Used when the keys outweigh the table (workgroup-uniform).
#ifndef OG_OCT_BESTTAB
#define OG_OCT_BESTTAB 1  // 0: the final key pass instead of the cell-best table (variant "octbt0", tests/test_gpu_variants.py)
#endif
    const int bD0 = tbase(D), cellsD = Ttot - bD0;
    const bool btab = OG_OCT_BESTTAB && tmode && k32 && C >= cellsD;
    unsigned* cellbest = (unsigned*)&nodes[0][0];
    static_assert(sizeof(nodes) >= 3 * OG_OCT_MAXL * sizeof(unsigned), "depth-D cells fit the node buffers");
    unsigned* BT = oct_best + (long long)(f * P.nlevels + l) * OG_OCT_BEST_CELLS;
    // one pass over the cells: every cell's best goes to the list node that holds it (position table in childPos)
    auto cell_pass = [&]() {
        for (int c0 = 0; c0 < cellsD; c0 += OCT_NT) {  // uniform trip count: og_wave_max32 wants whole waves
            const int c = c0 + tid;
            const unsigned key = c < cellsD ? BT[c] : 0u;
            og_wave_max32(best32, c < cellsD ? (int)childPos[bD0 + c] : 0, key, key != 0u);
        }
    };
    // a key's depth-D path (og_quadrant / og_child from its root): the leave pass's form when NO[] was not written
    auto dpath = [&](int x, int y) {
        const int r = min((int)((float)x / L.hX), nIni - 1);
        int x0 = (int)(L.hX * (float)r), x1 = (int)(L.hX * (float)(r + 1)), y0 = 0, y1 = H;
        int pth = r;
        for (int d = 0; d < D; d++) {
            const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
            const int qx = x >= mx, qy = y >= my;
            x0 = qx ? mx : x0;
            x1 = qx ? x1 : mx;
            y0 = qy ? my : y0;
            y1 = qy ? y1 : my;
            pth = 4 * pth + qx + 2 * qy;
        }
        return pth;
    };
    if (tmode) {
        for (int q = tid; q < Ttot; q += OCT_NT) childCnt[q] = 0;
        if (btab)
            for (int q = tid; q < cellsD; q += OCT_NT) cellbest[q] = 0u;
        // the depth-D path is separable: x alone picks the root and the x halves, y alone the y halves.  Per-column
        // and per-row tables (in childPos, free until the position table) hold them with the quadrant bits already
        // spread (x at even bit positions with the root above them, y at odd): path = XT[x] | YT[y]
        const int Wx = L.maxBX - L.minB + 1, Hy = H + 1;
        const bool xyt = Wx + Hy <= 4 * OG_OCT_MAXL;  // workgroup-uniform
        uint16_t* XT = childPos;
        uint16_t* YT = childPos + Wx;
        if (xyt) {
            for (int x = tid; x < Wx; x += OCT_NT) {
                const int r = min((int)((float)x / L.hX), nIni - 1);
                int x0 = (int)(L.hX * (float)r), x1 = (int)(L.hX * (float)(r + 1)), m = r;
                for (int d = 0; d < D; d++) {
                    const int mx = x0 + ((x1 - x0 + 1) >> 1), qx = x >= mx;
                    x0 = qx ? mx : x0;
                    x1 = qx ? x1 : mx;
                    m = (m << 2) | qx;
                }
                XT[x] = (uint16_t)m;
            }
            for (int y = tid; y < Hy; y += OCT_NT) {
                int y0 = 0, y1 = H, m = 0;
                for (int d = 0; d < D; d++) {
                    const int my = y0 + ((y1 - y0 + 1) >> 1), qy = y >= my;
                    y0 = qy ? my : y0;
                    y1 = qy ? y1 : my;
                    m = (m << 2) | (qy << 1);
                }
                YT[y] = (uint16_t)m;
            }
        }
        __syncthreads();
        const int bD = tbase(D);
        for (int base = tid; base < C; base += OCT_NT * OCT_U) {
            uint32_t kv[OCT_U], kr[OCT_U];
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                if (btab) {  // the whole key: the response joins the cell's best (same lines as the xy half)
                    const u64 kk = k < C ? K[k] : 0ull;
                    kv[u] = (uint32_t)kk;
                    kr[u] = (uint32_t)(kk >> 32);
                } else {
                    kv[u] = k < C ? K32[2 * k] : 0u;
                    kr[u] = 0u;
                }
            }
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                int a = 0;
                unsigned key32 = 0;
                if (k < C) {
                    const int x = (int)(kv[u] & 0xffff), y = (int)(kv[u] >> 16);
                    if (btab) key32 = (kr[u] << 24) | (0xffffffu - og_cand_order_m(x, y, L, mW, mH));
                    int pth;
                    if (xyt) {
                        pth = XT[x] | YT[y];
                    } else {
                        const int r = min((int)((float)x / L.hX), nIni - 1);
                        int x0 = (int)(L.hX * (float)r), x1 = (int)(L.hX * (float)(r + 1)), y0 = 0, y1 = H;
                        pth = r;
                        for (int d = 0; d < D; d++) {  // og_quadrant / og_child
                            const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
                            const int qx = x >= mx, qy = y >= my;
                            x0 = qx ? mx : x0;
                            x1 = qx ? x1 : mx;
                            y0 = qy ? my : y0;
                            y1 = qy ? y1 : my;
                            pth = 4 * pth + qx + 2 * qy;
                        }
                    }
                    a = bD + pth;
                    if (!btab) NO[k] = (uint16_t)a;  // (with the cell table only a leave pass needs it: recomputed)
                }
                og_wave_count(childCnt, a, k < C);  // (one LDS atomicAdd per key instead: 3 % slower)
                // the cell's best key: one LDS atomicMax per key (a segmented wave maximum first, og_wave_max32, was 2 %
                // slower: its 6 DPP steps cost more VALU than the same-address atomics serialise,
                // profiles/sweeps/r06_ab_octree_plain_atomics.txt)
                if (btab && k < C) atomicMax(&cellbest[a - bD], key32);
            }
        }
        __syncthreads();
        if (btab)  // (before the roots overwrite the node buffers; read back by cell_pass after barriers)
            for (int q = tid; q < cellsD; q += OCT_NT) BT[q] = cellbest[q];
        for (int d = D - 1; d >= 0; d--) {  // counts of shallower depths: sums of the four children
            const int b0 = tbase(d), b1 = tbase(d + 1), n = b1 - b0;
            for (int e = tid; e < n; e += OCT_NT)
                childCnt[b0 + e] = childCnt[b1 + 4 * e] + childCnt[b1 + 4 * e + 1] + childCnt[b1 + 4 * e + 2] +
                                   childCnt[b1 + 4 * e + 3];
            __syncthreads();
        }
        if (tid == 0) {
            int Ln = 0;
            for (int r = 0; r < nIni; r++) {
                const int c = childCnt[r];
                if (c > 0) {
                    OctNode n;
                    n.x0 = (short)(int)(L.hX * (float)r);
                    n.x1 = (short)(int)(L.hX * (float)(r + 1));
                    n.y0 = 0;
                    n.y1 = (short)H;
                    n.cnt = c;
                    n.cid = r;
                    nodes[0][Ln] = n;
                    fresh[0][Ln] = 0;
                    npath[0][Ln] = (uint16_t)r;
                    Ln++;
                }
            }
            sv[0] = Ln;
            sv[1] = 0;
            sv[2] = nIni;
            sv[3] = Ln == 0;
            sv[4] = 0;
            sv[8] = 0;
        }
        __syncthreads();
    }
    // position table of list `lst` (childPos): every depth-D index -> the list position of its listed ancestor
    auto pos_table = [&](int lst, int Lcount) {
        uint16_t* PT = childPos;
        for (int e = tid; e < Ttot; e += OCT_NT) PT[e] = 0xffff;
        __syncthreads();
        for (int q = tid; q < Lcount; q += OCT_NT) PT[npath[lst][q] & 0xfff] = (uint16_t)q;
        __syncthreads();
        for (int d = 1; d <= D; d++) {
            const int b0 = tbase(d - 1), b1 = tbase(d), n = tbase(d + 1) - b1;
            for (int e = tid; e < n; e += OCT_NT)
                if (PT[b1 + e] == 0xffff) PT[b1 + e] = PT[b0 + (e >> 2)];
            __syncthreads();
        }
    };
    // ---- (no table mode) roots (src/ORBextractor.cc:552-585) and the children of the first pass's splits, in ONE key pass:
    // each key's root r = x / hX and its quadrant in that root are counted together (childCnt[4r + q]); a root's
    // size is the sum of its four quadrant counts.  NO[k] holds the root id until the first round's key pass,
    // which maps it to the root's list position through aux[] (`noRoot`).
    if (!tmode) {
    for (int q = tid; q < 4 * nIni; q += OCT_NT) childCnt[q] = 0;
    __syncthreads();
    for (int base = tid; base < C; base += OCT_NT * OCT_U) {
        uint32_t kv[OCT_U];
#pragma unroll
        for (int u = 0; u < OCT_U; u++) {
            const int k = base + u * OCT_NT;
            kv[u] = k < C ? K32[2 * k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < OCT_U; u++) {
            const int k = base + u * OCT_NT;
            int a = 0;
            if (k < C) {
                const int x = (int)(kv[u] & 0xffff), y = (int)(kv[u] >> 16);
                const int r = min((int)((float)x / L.hX), nIni - 1);
                NO[k] = (uint16_t)r;
                OctNode rn;
                rn.x0 = (short)(int)(L.hX * (float)r);
                rn.x1 = (short)(int)(L.hX * (float)(r + 1));
                rn.y0 = 0;
                rn.y1 = (short)H;
                a = 4 * r + og_quadrant(x, y, rn);
            }
            og_wave_count(childCnt, a, k < C);
        }
    }
    __syncthreads();
    if (tid == 0) {
        int Ln = 0;
        for (int r = 0; r < nIni; r++) {
            const int c0 = childCnt[4 * r], c1 = childCnt[4 * r + 1], c2 = childCnt[4 * r + 2], c3 = childCnt[4 * r + 3];
            const int c = c0 + c1 + c2 + c3;
            if (c > 0) {
                OctNode n;
                n.x0 = (short)(int)(L.hX * (float)r);
                n.x1 = (short)(int)(L.hX * (float)(r + 1));
                n.y0 = 0;
                n.y1 = (short)H;
                n.cnt = c;
                n.cid = r;
                nodes[0][Ln] = n;
                fresh[0][Ln] = 0;
                // quadrant counts follow the root to its list position (Ln <= r: a forward in-place move)
                childCnt[4 * Ln] = c0;
                childCnt[4 * Ln + 1] = c1;
                childCnt[4 * Ln + 2] = c2;
                childCnt[4 * Ln + 3] = c3;
                aux[r] = Ln++;
            } else {
                aux[r] = -1;
            }
        }
        for (int q = 4 * Ln; q < 4 * nIni; q++) childCnt[q] = 0;
        sv[0] = Ln;      // list length
        sv[1] = 0;       // mode of the coming round: 0 normal pass, 1 final phase
        sv[2] = nIni;    // next creation id
        sv[3] = Ln == 0; // done (an empty list can never grow)
        sv[4] = 0;       // current node buffer
        sv[8] = 0;       // `best` filled by a key pass
    }
    __syncthreads();
    }
    bool noRoot = !tmode;  // NO[] holds root ids (workgroup-uniform)

    OCT_PROF(2, clock64());
    for (int round = 0; round < 4096; round++) {
        if (sv[3]) break;
        const int Ln = sv[0], mode = sv[1], cur = sv[4];
        OCT_PROF(8 + 4 * round, clock64());
        OCT_PROF(9 + 4 * round, (unsigned long long)Ln | ((unsigned long long)mode << 32));
        OctNode* cn = nodes[cur];
        uint8_t* cf = fresh[cur];
        OctNode* nn = nodes[cur ^ 1];
        uint8_t* nf = fresh[cur ^ 1];
        const int* CC = childCnt;
        int* NCC = childCnt;
        if (tid == 0) sv[10] = 0;  // table-mode leave flags of this round
        __syncthreads();
        // ---- the split set of this round and its order
        const int i = tid;
        int S, exSplit = 0;
        if (mode == 0) {
            const bool flag = i < Ln && cn[i].cnt > 1;
            const int rank = og_block_excl_scan(flag ? 1 : 0, wsum, &S);
            exSplit = rank;
            if (i < Ln) splitRank[i] = flag ? rank : -1;
            if (flag) splitNode[rank] = i;
        } else {
            // vSizeAndPointerToNode of the previous round sorted ascending by (size, ptr) and walked from
            // the back (src/ORBextractor.cc:684-685): order = descending (cnt, creation id)
            const bool flag = i < Ln && cf[i] && cn[i].cnt > 1;
            const int c = og_block_excl_scan(flag ? 1 : 0, wsum, &S);
            u64 mk = 0;
            if (flag) {
                mk = ((u64)(uint32_t)cn[i].cnt << 32) | (u64)(uint32_t)cn[i].cid;  // (size, ptr) order, unique
                skey[c] = mk;
            }
            __syncthreads();
            if (i < Ln) splitRank[i] = -1;
            if (flag) {
                // rank = number of candidates with a larger key: every lane reads the same key (broadcast), no
                // dependent lookups, so the loop pipelines
                int rank = 0;
#pragma unroll 8
                for (int q = 0; q < S; q++) rank += skey[q] > mk;
                splitRank[i] = rank;
                splitNode[rank] = i;
            }
        }
        OCT_PROF(200 + 8 * (round & 3), clock64());
        if (S == 0) {  // nothing to split: size == prevSize -> bFinish
            if (tid == 0) sv[3] = 1;
            __syncthreads();
            break;
        }
        __syncthreads();
        // ---- per split (in split order): non-empty children, the final phase's break point (:730-731)
        int nc = 0, nexp = 0, sn = 0;
        if (i < S) {
            sn = splitNode[i];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int c = tmode ? CC[tchild(npath[cur][sn], q) & 0xfff] : CC[4 * sn + q];
                nc += c > 0;
                nexp += c > 1;
            }
        }
        OCT_PROF(201 + 8 * (round & 3), clock64());
        // one scan for the children counts and (mode 0) the expandable children: both sums <= 4 OG_OCT_MAXL < 2^16
        int totP;
        const int exP = og_block_excl_scan(nc | (nexp << 16), wsum, &totP);
        const int exNc = exP & 0xffff;
        int A = S, T = totP & 0xffff;
        if (mode == 1) {
            const bool reach = i < S && (Ln + exNc + nc - (i + 1) >= N);
            if (tid == 0) sv[5] = S;
            __syncthreads();
            if (reach) atomicMin(&sv[5], i + 1);
            __syncthreads();
            A = sv[5];
            if (i == A - 1) sv[6] = exNc + nc;
            __syncthreads();
            T = sv[6];
        }
        OCT_PROF(202 + 8 * (round & 3), clock64());
        // ---- children: groups in reverse split order, each n4,n3,n2,n1 (push_front, :621-660)
        if (i < A) {
            const OctNode par = cn[sn];
            const int groupStart = T - (exNc + nc);
            const int cidBase = sv[2] + exNc;
            // the key pass's remap record of node sn: its split point here, its children's positions below
            newPos[sn] = (par.x0 + ((par.x1 - par.x0 + 1) >> 1)) | ((par.y0 + ((par.y1 - par.y0 + 1) >> 1)) << 16);
            int before = 0;  // non-empty children among q' < q (creation order n1..n4)
            const int tp = tmode ? (int)npath[cur][sn] : 0;
            for (int q = 0; q < 4; q++) {
                const int tc = tmode ? tchild(tp, q) : 0;
                const int c = tmode ? CC[tc & 0xfff] : CC[4 * sn + q];
                if (c > 0) {
                    const int pos = groupStart + (nc - before - 1);
                    OctNode ch = og_child(par, q);
                    ch.cnt = c;
                    ch.cid = cidBase + before;
                    if (!tmode) childPos[4 * sn + q] = (uint16_t)pos;
                    if (pos < OG_OCT_MAXL) {
                        nn[pos] = ch;
                        nf[pos] = 1;
                        npath[cur ^ 1][pos] = (uint16_t)tc;
                    }
                    if (tmode && c > 1 && (tc >> 12) >= D) atomicOr(&sv[10], 1);  // a fresh split candidate at depth D
                    before++;
                }
            }
        }
        // ---- kept nodes follow, in their old order (mode 0: every unsplit node, ranked by the split-set scan)
        const bool kept = i < Ln && (splitRank[i] < 0 || splitRank[i] >= A);
        int keptTot, kr;
        if (mode == 0) {
            kr = i - exSplit;
            keptTot = Ln - S;
        } else {
            kr = og_block_excl_scan(kept ? 1 : 0, wsum, &keptTot);
        }
        if (kept) {
            const int pos = T + kr;
            // remap record of a kept node: split point (0, 0) selects quadrant 3, and all four entries are pos
            newPos[i] = 0;
            if (!tmode) ((u64*)childPos)[i] = (u64)(uint16_t)pos * 0x0001000100010001ull;
            if (pos < OG_OCT_MAXL) {
                nn[pos] = cn[i];
                nf[pos] = 0;
                npath[cur ^ 1][pos] = npath[cur][i];
            }
            if (tmode && cn[i].cnt > 1 && (npath[cur][i] >> 12) >= D) atomicOr(&sv[10], 2);  // splits if mode 0
        }
        const int expTot = totP >> 16;  // mode 0 (A = S): expandable children of all splits
        OCT_PROF(203 + 8 * (round & 3), clock64());
        __syncthreads();  // the new list and the leave flags are complete
        OCT_PROF(204 + 8 * (round & 3), clock64());
        const int Lnew = T + keptTot;
        if (Lnew > OG_OCT_MAXL) {
            if (tid == 0) {
                atomicOr(status, 2);
                sv[3] = 1;
                sv[0] = 0;
            }
            __syncthreads();
            break;
        }
        // ---- termination / next mode (src/ORBextractor.cc:669-677, 734-735), decided before the key pass
        int done = 0, nextMode = mode;
        if (mode == 0) {
            if (Lnew >= N || Lnew == Ln) done = 1;
            else if (Lnew + expTot * 3 > N) nextMode = 1;
        } else {
            if (Lnew >= N || Lnew == Ln) done = 1;
        }
        // table mode: leave it when a next-round split candidate is a depth-D node (its children have no table):
        // a fresh child with more than one key, or (the next round splits every such node) a kept one
        bool leave = false;
        if (tmode && !done) {
            const int lf = sv[10];
            leave = (lf & 1) || (nextMode == 0 && (lf & 2));
        }
        if (!tmode || leave)
            for (int q = tid; q < 4 * Lnew; q += OCT_NT) NCC[q] = 0;
        if (done) {
            for (int q = tid; q < Lnew; q += OCT_NT) best[q] = 0ull;
        } else if (!tmode || leave) {
            // counting record of every node of the new list (splitRank is dead until the next round's plan):
            // split point x | y << 15, bit 30 = the node is a split candidate of the next round
            for (int q = tid; q < Lnew; q += OCT_NT) {
                const OctNode& nd = nn[q];
                const int countable = nd.cnt > 1 && (nextMode == 0 || nf[q]);
                splitRank[q] = (nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1)) | ((nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1)) << 15) |
                               (countable << 30);
            }
        }
        __syncthreads();
        OCT_PROF(10 + 4 * round, clock64());
        OCT_PROF(11 + 4 * round, (unsigned long long)S | ((unsigned long long)A << 32));
        if (tmode && !done && !leave) {  // table mode: the next round's counts are in the tables, no key pass
            if (tid == 0) {
                sv[0] = Lnew;
                sv[1] = nextMode;
                sv[2] += T;
                sv[3] = 0;
                sv[4] = cur ^ 1;
            }
            __syncthreads();
            continue;
        }
        if (tmode) pos_table(cur ^ 1, Lnew);  // NO[k] (depth-D index) -> new list position
        if (btab && tmode && done) {  // the last round in table mode: bests from the cell table, no key pass
            cell_pass();
            __syncthreads();
            tmode = false;
            if (tid == 0) {
                sv[0] = Lnew;
                sv[1] = nextMode;
                sv[2] += T;
                sv[3] = 1;
                sv[4] = cur ^ 1;
                sv[8] = 1;
            }
            __syncthreads();
            break;
        }
        // ---- one pass over the keys: move to the new list position, and either count the children of
        // the next round's split candidates or (last round) keep the best key per node (:744-760)
        for (int base = tid; base < C; base += OCT_NT * OCT_U) {
            u64 kv[OCT_U];  // the whole 8-byte key (its response is read by the last pass): same lines as its xy half
            int no[OCT_U];
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                kv[u] = k < C ? K[k] : 0ull;
                no[u] = k < C && !(tmode && btab) ? NO[k] : 0;
            }
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                int a = 0;
                bool cnt = false;
                unsigned key32 = 0;
                if (k < C) {
                    const int x = (int)(kv[u] & 0xffff), y = (int)((kv[u] >> 16) & 0xffff);
                    int n2;
                    if (tmode) {
                        n2 = childPos[btab ? bD0 + dpath(x, y) : no[u]];
                    } else {
                        const int n = noRoot ? aux[no[u]] : no[u];
                        // remap record: the node's split point (newPos) and its four target positions (childPos)
                        const int mm = newPos[n];
                        const u64 tp = ((const u64*)childPos)[n];
                        const int q = (x >= (mm & 0xffff) ? 1 : 0) | (y >= (mm >> 16) ? 2 : 0);  // og_quadrant
                        n2 = (int)((tp >> (16 * q)) & 0xffffu);
                    }
                    if (!done) NO[k] = (uint16_t)n2;
                    if (done) {
                        const unsigned resp = (unsigned)(kv[u] >> 32);
                        if (k32) {
                            key32 = (resp << 24) | (0xffffffu - og_cand_order_m(x, y, L, mW, mH));
                            a = n2;
                        } else {
                            atomicMax(&best[n2],
                                      ((u64)resp << 32) | (u64)(0xffffffffu - og_cand_order_m(x, y, L, mW, mH)));
                        }
                    } else {
                        const int rc = splitRank[n2];
                        cnt = (rc >> 30) & 1;
                        a = 4 * n2 + ((x >= (rc & 0x7fff) ? 1 : 0) | (y >= ((rc >> 15) & 0x7fff) ? 2 : 0));
                    }
                }
                if (!done) og_wave_count(NCC, a, cnt);  // `done`, k32 are workgroup-uniform
                else if (k32 && k < C) atomicMax(&best32[a], key32);  // (plain LDS atomics: see the count pass)
            }
        }
        __syncthreads();
        noRoot = false;
        tmode = false;  // NO[] now holds list positions (or the pass was the last one)
        if (tid == 0) {
            sv[0] = Lnew;
            sv[1] = nextMode;
            sv[2] += T;
            sv[3] = done;
            sv[4] = cur ^ 1;
            sv[8] = done;  // `best` is valid
        }
        __syncthreads();
    }
    __syncthreads();
    OCT_PROF(3, clock64());
    const int Ln = sv[0];
    if (!sv[8] && btab && tmode) {  // finished in table mode without a final round: bests from the cell table
        pos_table(sv[4], Ln);
        for (int n = tid; n < Ln; n += OCT_NT) best[n] = 0ull;
        __syncthreads();
        cell_pass();
        __syncthreads();
    } else if (!sv[8]) {  // finished without a final key pass (empty split set): one pass for the best key
        if (tmode) pos_table(sv[4], Ln);  // (childPos: dead after the plan)
        for (int n = tid; n < Ln; n += OCT_NT) best[n] = 0ull;
        __syncthreads();
        for (int base = tid; base < C; base += OCT_NT * OCT_U) {
            u64 kv[OCT_U];
            int no[OCT_U];
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                kv[u] = k < C ? K[k] : 0ull;
                no[u] = k < C ? NO[k] : 0;
            }
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                int n = 0;
                unsigned key32 = 0;
                if (k < C) {
                    const int x = (int)(kv[u] & 0xffff), y = (int)((kv[u] >> 16) & 0xffff);
                    const unsigned resp = (unsigned)(kv[u] >> 32);
                    n = tmode ? (int)childPos[no[u]] : (noRoot ? aux[no[u]] : no[u]);
                    if (k32)
                        key32 = (resp << 24) | (0xffffffu - og_cand_order_m(x, y, L, mW, mH));
                    else
                        atomicMax(&best[n], ((u64)resp << 32) | (u64)(0xffffffffu - og_cand_order_m(x, y, L, mW, mH)));
                }
                if (k32 && k < C) atomicMax(&best32[n], key32);
            }
        }
        __syncthreads();
    }
    const int nout = min(Ln, L.kcap);
    for (int n = tid; n < nout; n += OCT_NT) {
        const u64 b = k32 ? ((u64)(best32[n] >> 24) << 32) | (0xff000000u | (best32[n] & 0xffffffu)) : best[n];
        const unsigned ord = 0xffffffffu - (unsigned)(b & 0xffffffffu);
        const int lx = ord % L.wCell;
        unsigned t2 = ord / L.wCell;
        const int ly = t2 % L.hCell;
        t2 /= L.hCell;
        const int cj = t2 % L.nCols, ci = t2 / L.nCols;
        const int x = cj * L.wCell + 3 + lx + L.minB, y = ci * L.hCell + 3 + ly + L.minB;
        const long long o = (long long)f * P.kcap_total + L.koff + n;
        oct_xy[o] = (uint32_t)x | ((uint32_t)y << 16);
        oct_resp[o] = (uint32_t)(b >> 32);
    }
    if (tid == 0) {
        oct_count[f * P.nlevels + l] = nout;
        if (Ln > L.kcap) atomicOr(status, 4);
    }
    OCT_PROF(4, clock64());
    OCT_PROF(5, (unsigned long long)Ln);
}

// exclusive block scan of NPT ints per thread, thread t holding items t*NPT .. t*NPT + NPT-1 (in order)
template <int NPT>
__device__ __forceinline__ void og_block_excl_scan_n(const int (&v)[NPT], int (&ex)[NPT], int* wsum, int* total)
{
    int s = 0;
#pragma unroll
    for (int j = 0; j < NPT; j++) s += v[j];
    int e = og_block_excl_scan(s, wsum, total);
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        ex[j] = e;
        e += v[j];
    }
}

// og_octree_kernel with a list capacity of MAXL = OG_OCT_MAXL_BIG nodes, NPT = MAXL / OCT_NT of them per thread in the
// per-node phases, for levels of more than ~1000 features (5000+ features per frame).  The 1024-node kernel above
// keeps its own one-node-per-thread form: the generic one measured 22 % slower at NPT = 1 (0.60 -> 0.73 ms per 512
// frames at config 3, same instruction count; not explained)
template <int MAXL>
__global__ __launch_bounds__(OCT_NT) void og_octree_big_kernel(OgPlan P, int l0, const u64* __restrict__ cand,
                                                           const int* __restrict__ cand_count,
                                                           uint16_t* __restrict__ node_of,
                                                           uint32_t* __restrict__ oct_xy,
                                                           uint32_t* __restrict__ oct_resp,
                                                           int* __restrict__ oct_count, int* __restrict__ status,
                                                           int nlaunch)
{
    constexpr int OG_OCT_MAXL_T = MAXL;
    constexpr int NPT = MAXL / OCT_NT;  // list nodes per thread in the per-node phases
    static_assert(NPT * OCT_NT == MAXL, "list capacity is a multiple of the workgroup");
    __shared__ OctNode nodes[2][MAXL];
    __shared__ uint8_t fresh[2][MAXL];
    __shared__ int splitRank[MAXL];
    __shared__ int splitNode[MAXL];
    __shared__ int newPos[MAXL];
    __shared__ int aux[MAXL];
    // child counts, indexed 4*node + quadrant: one buffer -- a round's counts are consumed (split set,
    // children) before the key pass accumulates the next round's, with barriers in between; the last key
    // pass keeps the best key per node in the same storage.  ~74 KB of LDS in total: 2 workgroups per CU.
    __shared__ __attribute__((aligned(16))) int childCnt[4 * MAXL];
    __shared__ __attribute__((aligned(16))) uint16_t childPos[4 * MAXL];
    // final-phase planning only: the candidates' (size, creation id) keys, in the previous round's (dead) childPos
    u64* skey = (u64*)childPos;
    u64* best = (u64*)childCnt;  // [MAXL], final key pass only
    __shared__ int wsum[32];
    __shared__ int sv[16];

    // level-major dispatch order, level 0 first: the finest level has the most candidates (and rounds), so
    // its workgroups start in the first wave of residency instead of being interleaved with the short ones
    const int nb = (int)gridDim.x / nlaunch;  // frames in the launch
    const int l = l0 + (int)blockIdx.x / nb, f = (int)blockIdx.x % nb, tid = threadIdx.x;
    const OgLevel& L = P.lv[l];
    const int C = min(cand_count[f * P.nlevels + l], L.cand_cap);
    const u64* K = cand + (long long)f * P.cand_per_frame + L.cand_off;
    const uint32_t* K32 = (const uint32_t*)K;  // [2k] = x | y << 16, [2k+1] = response
    uint16_t* NO = node_of + (long long)f * P.cand_per_frame + L.cand_off;
    const int N = L.N;
    const int nIni = L.nIni;
    const int H = L.maxBY - L.minB;

    OCT_PROF(0, clock64());
    OCT_PROF(1, (unsigned long long)C);
    // ---- roots (src/ORBextractor.cc:552-585) and the children of the first pass's splits, in ONE key pass:
    // each key's root r = x / hX and its quadrant in that root are counted together (childCnt[4r + q]); a root's
    // size is the sum of its four quadrant counts.  NO[k] holds the root id until the first round's key pass,
    // which maps it to the root's list position through aux[] (`noRoot`).
    for (int q = tid; q < 4 * nIni; q += OCT_NT) childCnt[q] = 0;
    __syncthreads();
    for (int base = tid; base < C; base += OCT_NT * OCT_U) {
        uint32_t kv[OCT_U];
#pragma unroll
        for (int u = 0; u < OCT_U; u++) {
            const int k = base + u * OCT_NT;
            kv[u] = k < C ? K32[2 * k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < OCT_U; u++) {
            const int k = base + u * OCT_NT;
            int a = 0;
            if (k < C) {
                const int x = (int)(kv[u] & 0xffff), y = (int)(kv[u] >> 16);
                const int r = min((int)((float)x / L.hX), nIni - 1);
                NO[k] = (uint16_t)r;
                OctNode rn;
                rn.x0 = (short)(int)(L.hX * (float)r);
                rn.x1 = (short)(int)(L.hX * (float)(r + 1));
                rn.y0 = 0;
                rn.y1 = (short)H;
                a = 4 * r + og_quadrant(x, y, rn);
            }
            og_wave_count(childCnt, a, k < C);
        }
    }
    __syncthreads();
    if (tid == 0) {
        int Ln = 0;
        for (int r = 0; r < nIni; r++) {
            const int c0 = childCnt[4 * r], c1 = childCnt[4 * r + 1], c2 = childCnt[4 * r + 2], c3 = childCnt[4 * r + 3];
            const int c = c0 + c1 + c2 + c3;
            if (c > 0) {
                OctNode n;
                n.x0 = (short)(int)(L.hX * (float)r);
                n.x1 = (short)(int)(L.hX * (float)(r + 1));
                n.y0 = 0;
                n.y1 = (short)H;
                n.cnt = c;
                n.cid = r;
                nodes[0][Ln] = n;
                fresh[0][Ln] = 0;
                // quadrant counts follow the root to its list position (Ln <= r: a forward in-place move)
                childCnt[4 * Ln] = c0;
                childCnt[4 * Ln + 1] = c1;
                childCnt[4 * Ln + 2] = c2;
                childCnt[4 * Ln + 3] = c3;
                aux[r] = Ln++;
            } else {
                aux[r] = -1;
            }
        }
        for (int q = 4 * Ln; q < 4 * nIni; q++) childCnt[q] = 0;
        sv[0] = Ln;      // list length
        sv[1] = 0;       // mode of the coming round: 0 normal pass, 1 final phase
        sv[2] = nIni;    // next creation id
        sv[3] = Ln == 0; // done (an empty list can never grow)
        sv[4] = 0;       // current node buffer
        sv[8] = 0;       // `best` filled by a key pass
    }
    __syncthreads();
    bool noRoot = true;  // NO[] holds root ids (workgroup-uniform)

    OCT_PROF(2, clock64());
    for (int round = 0; round < 4096; round++) {
        if (sv[3]) break;
        const int Ln = sv[0], mode = sv[1], cur = sv[4];
        OCT_PROF(8 + 4 * round, clock64());
        OCT_PROF(9 + 4 * round, (unsigned long long)Ln | ((unsigned long long)mode << 32));
        OctNode* cn = nodes[cur];
        uint8_t* cf = fresh[cur];
        OctNode* nn = nodes[cur ^ 1];
        uint8_t* nf = fresh[cur ^ 1];
        const int* CC = childCnt;
        int* NCC = childCnt;
        __syncthreads();
        // ---- the split set of this round and its order.  List node i = NPT * tid + j (j < NPT): each thread owns
        // NPT consecutive nodes, so thread-local prefixes plus one block scan keep the list order.
        int S;
        if (mode == 0) {
            int fl[NPT], rk[NPT];
#pragma unroll
            for (int j = 0; j < NPT; j++) {
                const int i = NPT * tid + j;
                fl[j] = i < Ln && cn[i].cnt > 1;
            }
            og_block_excl_scan_n<NPT>(fl, rk, wsum, &S);
#pragma unroll
            for (int j = 0; j < NPT; j++) {
                const int i = NPT * tid + j;
                if (i < Ln) splitRank[i] = fl[j] ? rk[j] : -1;
                if (fl[j]) splitNode[rk[j]] = i;
            }
        } else {
            // vSizeAndPointerToNode of the previous round sorted ascending by (size, ptr) and walked from
            // the back (src/ORBextractor.cc:684-685): order = descending (cnt, creation id)
            int fl[NPT], cx[NPT];
            u64 mk[NPT];
#pragma unroll
            for (int j = 0; j < NPT; j++) {
                const int i = NPT * tid + j;
                fl[j] = i < Ln && cf[i] && cn[i].cnt > 1;
            }
            og_block_excl_scan_n<NPT>(fl, cx, wsum, &S);
#pragma unroll
            for (int j = 0; j < NPT; j++) {
                const int i = NPT * tid + j;
                mk[j] = 0;
                if (fl[j]) {
                    mk[j] = ((u64)(uint32_t)cn[i].cnt << 32) | (u64)(uint32_t)cn[i].cid;  // (size, ptr) order, unique
                    skey[cx[j]] = mk[j];
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < NPT; j++) {
                const int i = NPT * tid + j;
                if (i < Ln) splitRank[i] = -1;
                if (fl[j]) {
                    // rank = number of candidates with a larger key: every lane reads the same key (broadcast), no
                    // dependent lookups, so the loop pipelines
                    int rank = 0;
#pragma unroll 8
                    for (int q = 0; q < S; q++) rank += skey[q] > mk[j];
                    splitRank[i] = rank;
                    splitNode[rank] = i;
                }
            }
        }
        if (S == 0) {  // nothing to split: size == prevSize -> bFinish
            if (tid == 0) sv[3] = 1;
            __syncthreads();
            break;
        }
        __syncthreads();
        // ---- per split (in split order): non-empty children, the final phase's break point (:730-731)
        int nc[NPT], nexp[NPT], sn[NPT], exNc[NPT];
#pragma unroll
        for (int j = 0; j < NPT; j++) {
            const int i = NPT * tid + j;
            nc[j] = 0;
            nexp[j] = 0;
            sn[j] = 0;
            if (i < S) {
                sn[j] = splitNode[i];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int c = CC[4 * sn[j] + q];
                    nc[j] += c > 0;
                    nexp[j] += c > 1;
                }
            }
        }
        int totNc;
        og_block_excl_scan_n<NPT>(nc, exNc, wsum, &totNc);
        int A = S;
        if (mode == 1) {
            if (tid == 0) sv[5] = S;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < NPT; j++) {
                const int i = NPT * tid + j;
                if (i < S && (Ln + exNc[j] + nc[j] - (i + 1) >= N)) atomicMin(&sv[5], i + 1);
            }
            __syncthreads();
            A = sv[5];
        }
#pragma unroll
        for (int j = 0; j < NPT; j++)
            if (NPT * tid + j == A - 1) sv[6] = exNc[j] + nc[j];
        __syncthreads();
        const int T = sv[6];
        // ---- children: groups in reverse split order, each n4,n3,n2,n1 (push_front, :621-660)
#pragma unroll
        for (int j = 0; j < NPT; j++) {
            const int i = NPT * tid + j;
            if (i >= A) continue;
            const OctNode par = cn[sn[j]];
            const int groupStart = T - (exNc[j] + nc[j]);
            const int cidBase = sv[2] + exNc[j];
            // the key pass's remap record of node sn: its split point here, its children's positions below
            newPos[sn[j]] = (par.x0 + ((par.x1 - par.x0 + 1) >> 1)) | ((par.y0 + ((par.y1 - par.y0 + 1) >> 1)) << 16);
            int before = 0;  // non-empty children among q' < q (creation order n1..n4)
            for (int q = 0; q < 4; q++) {
                const int c = CC[4 * sn[j] + q];
                if (c > 0) {
                    const int pos = groupStart + (nc[j] - before - 1);
                    OctNode ch = og_child(par, q);
                    ch.cnt = c;
                    ch.cid = cidBase + before;
                    childPos[4 * sn[j] + q] = (uint16_t)pos;
                    if (pos < MAXL) {
                        nn[pos] = ch;
                        nf[pos] = 1;
                    }
                    before++;
                }
            }
        }
        // ---- kept nodes follow, in their old order
        int kept[NPT], kr[NPT], ne[NPT], dummy[NPT];
#pragma unroll
        for (int j = 0; j < NPT; j++) {
            const int i = NPT * tid + j;
            kept[j] = i < Ln && (splitRank[i] < 0 || splitRank[i] >= A);
            ne[j] = i < A ? nexp[j] : 0;
        }
        int keptTot;
        og_block_excl_scan_n<NPT>(kept, kr, wsum, &keptTot);
#pragma unroll
        for (int j = 0; j < NPT; j++) {
            const int i = NPT * tid + j;
            if (!kept[j]) continue;
            const int pos = T + kr[j];
            // remap record of a kept node: split point (0, 0) selects quadrant 3, and all four entries are pos
            newPos[i] = 0;
            ((u64*)childPos)[i] = (u64)(uint16_t)pos * 0x0001000100010001ull;
            if (pos < MAXL) {
                nn[pos] = cn[i];
                nf[pos] = 0;
            }
        }
        int expTot;
        og_block_excl_scan_n<NPT>(ne, dummy, wsum, &expTot);
        const int Lnew = T + keptTot;
        if (Lnew > MAXL) {
            if (tid == 0) {
                atomicOr(status, 2);
                sv[3] = 1;
                sv[0] = 0;
            }
            __syncthreads();
            break;
        }
        // ---- termination / next mode (src/ORBextractor.cc:669-677, 734-735), decided before the key pass
        int done = 0, nextMode = mode;
        if (mode == 0) {
            if (Lnew >= N || Lnew == Ln) done = 1;
            else if (Lnew + expTot * 3 > N) nextMode = 1;
        } else {
            if (Lnew >= N || Lnew == Ln) done = 1;
        }
        for (int q = tid; q < 4 * Lnew; q += OCT_NT) NCC[q] = 0;
        if (done) {
            for (int q = tid; q < Lnew; q += OCT_NT) best[q] = 0ull;
        } else {
            // counting record of every node of the new list (splitRank is dead until the next round's plan):
            // split point x | y << 15, bit 30 = the node is a split candidate of the next round
            for (int q = tid; q < Lnew; q += OCT_NT) {
                const OctNode& nd = nn[q];
                const int countable = nd.cnt > 1 && (nextMode == 0 || nf[q]);
                splitRank[q] = (nd.x0 + ((nd.x1 - nd.x0 + 1) >> 1)) | ((nd.y0 + ((nd.y1 - nd.y0 + 1) >> 1)) << 15) |
                               (countable << 30);
            }
        }
        __syncthreads();
        OCT_PROF(10 + 4 * round, clock64());
        OCT_PROF(11 + 4 * round, (unsigned long long)S | ((unsigned long long)A << 32));
        // ---- one pass over the keys: move to the new list position, and either count the children of
        // the next round's split candidates or (last round) keep the best key per node (:744-760)
        for (int base = tid; base < C; base += OCT_NT * OCT_U) {
            uint32_t kv[OCT_U];
            int no[OCT_U];
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                kv[u] = k < C ? K32[2 * k] : 0u;
                no[u] = k < C ? NO[k] : 0;
            }
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                int a = 0;
                bool cnt = false;
                if (k < C) {
                    const int n = noRoot ? aux[no[u]] : no[u];
                    const int x = (int)(kv[u] & 0xffff), y = (int)(kv[u] >> 16);
                    // remap record: the node's split point (newPos) and its four target positions (childPos)
                    const int mm = newPos[n];
                    const u64 tp = ((const u64*)childPos)[n];
                    const int q = (x >= (mm & 0xffff) ? 1 : 0) | (y >= (mm >> 16) ? 2 : 0);  // og_quadrant
                    const int n2 = (int)((tp >> (16 * q)) & 0xffffu);
                    NO[k] = (uint16_t)n2;
                    if (done) {
                        const unsigned resp = K32[2 * k + 1];
                        atomicMax(&best[n2], ((u64)resp << 32) | (u64)(0xffffffffu - og_cand_order(x, y, L)));
                    } else {
                        const int rc = splitRank[n2];
                        cnt = (rc >> 30) & 1;
                        a = 4 * n2 + ((x >= (rc & 0x7fff) ? 1 : 0) | (y >= ((rc >> 15) & 0x7fff) ? 2 : 0));
                    }
                }
                if (!done) og_wave_count(NCC, a, cnt);  // `done` is workgroup-uniform
            }
        }
        __syncthreads();
        noRoot = false;
        if (tid == 0) {
            sv[0] = Lnew;
            sv[1] = nextMode;
            sv[2] += T;
            sv[3] = done;
            sv[4] = cur ^ 1;
            sv[8] = done;  // `best` is valid
        }
        __syncthreads();
    }
    __syncthreads();
    OCT_PROF(3, clock64());
    const int Ln = sv[0];
    if (!sv[8]) {  // finished without a final key pass (empty split set): one pass for the best key
        for (int n = tid; n < Ln; n += OCT_NT) best[n] = 0ull;
        __syncthreads();
        for (int base = tid; base < C; base += OCT_NT * OCT_U) {
            u64 kv[OCT_U];
            int no[OCT_U];
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                kv[u] = k < C ? K[k] : 0ull;
                no[u] = k < C ? NO[k] : 0;
            }
#pragma unroll
            for (int u = 0; u < OCT_U; u++) {
                const int k = base + u * OCT_NT;
                if (k < C) {
                    const int x = (int)(kv[u] & 0xffff), y = (int)((kv[u] >> 16) & 0xffff);
                    const unsigned resp = (unsigned)(kv[u] >> 32);
                    atomicMax(&best[noRoot ? aux[no[u]] : no[u]],
                              ((u64)resp << 32) | (u64)(0xffffffffu - og_cand_order(x, y, L)));
                }
            }
        }
        __syncthreads();
    }
    (void)OG_OCT_MAXL_T;
    const int nout = min(Ln, L.kcap);
    for (int n = tid; n < nout; n += OCT_NT) {
        const u64 b = best[n];
        const unsigned ord = 0xffffffffu - (unsigned)(b & 0xffffffffu);
        const int lx = ord % L.wCell;
        unsigned t2 = ord / L.wCell;
        const int ly = t2 % L.hCell;
        t2 /= L.hCell;
        const int cj = t2 % L.nCols, ci = t2 / L.nCols;
        const int x = cj * L.wCell + 3 + lx + L.minB, y = ci * L.hCell + 3 + ly + L.minB;
        const long long o = (long long)f * P.kcap_total + L.koff + n;
        oct_xy[o] = (uint32_t)x | ((uint32_t)y << 16);
        oct_resp[o] = (uint32_t)(b >> 32);
    }
    if (tid == 0) {
        oct_count[f * P.nlevels + l] = nout;
        if (Ln > L.kcap) atomicOr(status, 4);
    }
    OCT_PROF(4, clock64());
    OCT_PROF(5, (unsigned long long)Ln);
}

// ------------------------------------------------------------------------------------------------
// k4: orientation + blur + rBRIEF + assembly (src/ORBextractor.cc:77-147, 851-852, 1076-1104)
// ------------------------------------------------------------------------------------------------
// BORDER_REFLECT_101 for an index at most n - 2 outside [0, n): one reflection (the describe window of a keypoint at
// least 19 px inside its level overshoots by a few pixels), no loop
__device__ __forceinline__ int og_reflect101_1(int i, int n)
{
    return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

// sum over the 64 lanes (all active) with DPP: quad_perm [1,0,3,2] and [2,3,0,1] (quads), row_half_mirror (8),
// row_mirror (16), row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3; lane 63 then holds the sum.
// Six VALU ops instead of six ds_bpermute shuffles and adds.
__device__ __forceinline__ int og_wave_sum(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0xb1, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x4e, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    return __builtin_amdgcn_readlane(v, 63);
}

#define DK_WAVES 4  // keypoint waves per workgroup (1 and 2 measured: profiles/sweeps/r04_ab_dk_waves.txt)
#define RAW_W 43
#define RAW_S 52  // 43 + 3 misalignment bytes, dword multiple; 13 dwords: conflict-free lane-per-row reads
#define BL_W 37   // the blurred window the tests can reach (only its 512 samples are formed)
#define HP_ROWS 22  // row pairs of the horizontal pass (43 rows -> 22 pairs)
#define HP_S 40     // pair-row stride in dwords (10 groups of 4 columns)
#define DK_BORDER_RB 22  // border windows: rows of byte loads in flight per batch

// IC_Angle (src/ORBextractor.cc:77-104) by disk rows with v_dot4: item t < 279 = (disk row v = t / 9 - 15, window
// dword j = t % 9, which holds window columns 4 + 4j .. 7 + 4j, i.e. u = 4j - 17 .. 4j - 14).  Per item: the byte mask
// of the columns inside the disk row (|u| <= umax[|v|]; umax depends only on HALF_PATCH_SIZE = 15, :454-469, and the
// host checks that its table equals OG_UMAX), the weights u + 16 of those bytes (in [1, 31]; bytes outside the disk
// are masked to 0 first), and the dword's LDS byte offset | v << 16.  m10 = sum (u + 16) I - 16 sum I, m01 = sum v
// sum I.
#define OG_IC_ITEMS 320  // 279 items padded to 5 x 64 lanes (padding: mask 0)
struct OgIcTab {
    uint32_t mask[OG_IC_ITEMS], wt[OG_IC_ITEMS], ov[OG_IC_ITEMS];
};
constexpr OgIcTab og_make_ic()
{
    OgIcTab t{};
    constexpr int umax[16] = {OG_UMAX};
    for (int i = 0; i < 279; i++) {
        const int v = i / 9 - 15, j = i % 9, av = v < 0 ? -v : v;
        uint32_t m = 0, w = 0;
        for (int k = 0; k < 4; k++) {
            const int u = 4 * j + k - 17;
            const int au = u < 0 ? -u : u;
            if (au <= umax[av]) {
                m |= 0xffu << (8 * k);
                w |= (uint32_t)(u + 16) << (8 * k);
            }
        }
        t.mask[i] = m;
        t.wt[i] = w;
        t.ov[i] = (uint32_t)((21 + v) * 52 + 4 + 4 * j) | ((uint32_t)(v & 0xffff) << 16);  // RAW_S = 52
    }
    return t;
}
// the table lane-major: lane i's items i, i + 64, .. i + 256 as (mask, wt, ov) triples in 16 words, loaded at kernel
// start with four 16-byte loads from one base (in flight over the level search and the window load)
struct OgIcLane {
    uint32_t w[64][16];
};
constexpr OgIcLane og_make_icl()
{
    const OgIcTab t = og_make_ic();
    OgIcLane l{};
    for (int i = 0; i < 64; i++)
        for (int it = 0; it < OG_IC_ITEMS / 64; it++) {
            l.w[i][3 * it] = t.mask[i + 64 * it];
            l.w[i][3 * it + 1] = t.wt[i + 64 * it];
            l.w[i][3 * it + 2] = t.ov[i + 64 * it];
        }
    return l;
}
__constant__ OgIcLane og_icl = og_make_icl();
// GaussianBlur 7x7 sigma 2 integer kernels by ORBGPU_SEM_BLUR_* variant, c0 | c1 << 8 | c2 << 16 | c3 << 24 for
// [c0,c1,c2,c3,c2,c1,c0]: cvRound(256 g) (sum 257) twice, the bit-exact kernel with centre 256 - 2 sum(sides),
// the error-diffused bit-exact kernel
constexpr uint32_t og_blur_coefs[4] = {18u | 34u << 8 | 49u << 16 | 55u << 24, 18u | 34u << 8 | 49u << 16 | 55u << 24,
                                          18u | 34u << 8 | 49u << 16 | 54u << 24, 18u | 34u << 8 | 48u << 16 | 56u << 24};

// The describe kernel's waves share no LDS: each wave owns its raw window and horizontal sums.  A wave only has to
// see its own LDS writes before it reads them back, so it synchronises with itself (LDS counter drained, no
// reordering across the point) instead of with the other waves of the workgroup; a wave that finished its loads does
// not wait for a neighbour's global loads (-2 % describe time against workgroup barriers).
__device__ __forceinline__ void og_dk_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores have landed
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// BV = ORBGPU_SEM_BLUR_* variant >> ORBGPU_SEM_BLUR_SHIFT, NOFMA = ORBGPU_SEM_BRIEF_NOFMA: compile-time, so every
// variant keeps its kernel taps as literal operands and only the SSE2 variant carries the tie test
template <int BV, bool NOFMA>
__global__ __launch_bounds__(64 * DK_WAVES) void og_describe_kernel(OgPlan P, const uint8_t* __restrict__ img0,
                                                                    long long pitch0, long long fstride0,
                                                                    const uint8_t* __restrict__ pyr,
                                                                    const uint32_t* __restrict__ oct_xy,
                                                                    const uint32_t* __restrict__ oct_resp,
                                                                    const int* __restrict__ oct_count,
                                                                    orbgpu_kp_dev* __restrict__ kps,
                                                                    uint8_t* __restrict__ desc,
                                                                    int* __restrict__ counts, unsigned dmagic)
{
    __shared__ __attribute__((aligned(16))) uint8_t raw[DK_WAVES][RAW_W * RAW_S];
    __shared__ __attribute__((aligned(16))) uint32_t hp[DK_WAVES][HP_ROWS * HP_S];
    // w is wave-uniform: made explicit, so the keypoint index, its level and its window origin live in SGPRs
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // the lane's IC_Angle items, loaded first: in flight over the level search and the window load
    uint4 icq[4] = {};
#if defined(__HIP_DEVICE_COMPILE__)
    {
        typedef const __attribute__((address_space(1))) uint4 g_u4;
        g_u4* ib = (g_u4*)&og_icl.w[0][0];
        __asm__("" : "+s"(ib));  // one SGPR base: a lane offset and 16-byte immediate steps
#pragma unroll
        for (int k = 0; k < 4; k++) icq[k] = ib[4 * lane + k];
    }
#endif
    const unsigned gx = gridDim.x, gy = gridDim.y;
    const int nlv = P.nlevels, kct = P.kcap_total;
    const unsigned lin = og_xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy);
    // frame = lin / gridDim.x by the host's multiply-high constant (exact for every lin of the launch, checked on the
    // host; 0: the division)
    const unsigned fq = dmagic ? __umulhi(lin, dmagic) : lin / gx;
    const int f = (int)fq;
    const int g = (int)(lin - fq * gx) * DK_WAVES + w;
    // which level does keypoint g belong to (levels concatenated 0..L-1, :1076-1104); with 8 levels the frame's
    // counts are one 32-byte scalar load and the search is unrolled (per keypoint wave: the scalar unit is shared)
    int l = -1, li = 0, total = 0;
    if (nlv == 8) {
#if defined(__HIP_DEVICE_COMPILE__)
        // one 32-byte scalar load of the frame's 8 level counts (a DPP scan over a per-lane vector load was 3 % slower:
        // the vector load's round trip at the kernel's start).  The level is the number of prefix sums <= g (they are
        // nondecreasing) and its first keypoint the last such prefix sum: 4 scalar instructions per level, the compare's
        // SCC feeding both the select and the add-with-carry
        const og_u32x8 c8 = ((const __attribute__((address_space(4))) og_u32x8*)(oct_count + 8 * f))[0];
        int nl = 0, st = 0;
        const int gu = __builtin_amdgcn_readfirstlane(g);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int c = (int)c8[q];
            __asm__("s_add_i32 %0, %0, %3\n\t"
                    "s_cmp_ge_i32 %4, %0\n\t"
                    "s_cselect_b32 %2, %0, %2\n\t"
                    "s_addc_u32 %1, %1, 0"
                    : "+s"(total), "+s"(nl), "+s"(st)
                    : "s"(c), "s"(gu)
                    : "scc");
        }
        if (nl < 8) {
            l = nl;
            li = g - st;
        }
#endif
    } else {
        for (int q = 0; q < nlv; q++) {
            const int c = oct_count[f * nlv + q];
            if (l < 0 && g < total + c) {
                l = q;
                li = g - total;
            }
            total += c;
        }
    }
    // wave-uniform by construction: SGPRs, so that P.lv[l] below is a scalar load, not a vector load from the kernarg
    // segment (the generic branch's loop would otherwise make them VGPRs)
    l = __builtin_amdgcn_readfirstlane(l);
    li = __builtin_amdgcn_readfirstlane(li);
    total = __builtin_amdgcn_readfirstlane(total);
    if (g == 0 && lane == 0) counts[f] = total;
    const bool active = l >= 0;
    uint8_t* R = raw[w];
    uint32_t* Hp = hp[w];
    int cx = 0, cy = 0, lw = 1, lh = 1;
    unsigned resp = 0;  // response key (og_harris_key under ORBGPU_SEM_SCORE_HARRIS, else the FAST score)
    if (active) {
        const OgLevel& L = P.lv[l];
        const int koff = L.koff, Lp = L.pitch;
        const long long Lpo = L.pyr_off;
        lw = L.w;
        lh = L.h;
        const unsigned o = (unsigned)f * (unsigned)kct + (unsigned)(koff + li);  // < 2^31 (host plan)
        const uint32_t xy = oct_xy[o];
        cx = (int)(xy & 0xffff);
        cy = (int)(xy >> 16);
        resp = oct_resp[o];
        // the image origin by selects, not a branch
        const uint8_t* img = l == 0 ? img0 + (long long)f * fstride0 : pyr + ((long long)f * P.pyr_per_frame + Lpo);
        const long long pitch = l == 0 ? pitch0 : (long long)Lp;
        if (cx >= 21 && cy >= 21 && cx + 28 < lw && cy + 21 < lh) {
            // interior (almost every keypoint): 43 rows x 11 dwords, lanes 0-54 = 5 rows x 11 dwords stepping 5 rows
            // per iteration (offsets advance by a uniform 5 * pitch).  Each dword comes from two aligned loads
            // funnel-shifted by the row's own misalignment (any pitch, e.g. a contiguous 1241-px KITTI image); the
            // farthest byte read is x = cx + 26, inside the row (level starts are 256-B aligned, so the rounded-down
            // first load never precedes the image).  All loads of a lane are issued before the first use; addresses
            // are the window origin rounded down to 4 bytes (wave-uniform, SGPRs) plus a 32-bit lane offset.
            const uint8_t* src0 = img + (long long)(cy - 21) * pitch + (cx - 21);
            const unsigned m0 = (unsigned)((uintptr_t)src0 & 3);
            const uint8_t* abase = src0 - m0;
            const unsigned upitch = (unsigned)pitch & (OG_MAX_PITCH - 1);  // < 2^24 (checked on the host)
            constexpr int NIT = (RAW_W + 4) / 5;  // 9 iterations of 5 rows
            const int lr = (lane * 5958) >> 16;  // lane / 11 (lanes 55-63: row 5, inactive)
            unsigned l11 = __umul24((unsigned)lr, 11u);
            __asm__("" : "+v"(l11));
            const int q = lane - (int)l11;
            const bool lact = lane < 55;
            const unsigned off0 = __umul24((unsigned)min(lr, 4), upitch) + 4u * (unsigned)q + m0;  // upitch < 2^24
            const unsigned step = __umul24(5u, upitch);
            uint32_t lo[NIT], hi[NIT];
            unsigned sh[NIT];
#pragma unroll
            for (int k = 0; k < NIT; k++) {
                // rows past the window (lr + 5 k > 42) re-read row 42's place: the last row + the lane's column
                const unsigned kk = (unsigned)min(k, (RAW_W - 1 - min(lr, 4)) / 5);
                unsigned off = off0 + kk * step;
                __asm__("" : "+v"(off));  // a 32-bit lane offset (saddr + voffset loads)
                const uint32_t* a = (const uint32_t*)(abase + (off & ~3u));
                sh[k] = off & 3u;
                lo[k] = a[0];
                hi[k] = a[1];
            }
#pragma unroll
            for (int k = 0; k < NIT; k++) {
                const int r = lr + 5 * k;
                if (lact && r < RAW_W) *(uint32_t*)&R[r * RAW_S + 4 * q] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh[k]);
            }
        } else {
            // within 21 px of the border: BORDER_REFLECT_101.  Lane c < 43 owns window column c (its reflected image
            // column, once); each row's reflected image row is wave-uniform.  The loads of a batch of rows are issued
            // before their stores: 2 memory round trips instead of the 29 of a pixel-per-lane loop.  One reflection
            // is exact: keypoints lie in [19, size - 19) of their level, so the window spans [-2, size + 1] and a
            // level holding a keypoint is at least 39 px.
            unsigned xx = (unsigned)og_reflect101_1(cx - 21 + min(lane, RAW_W - 1), lw);
            // loads from the uniform base of the lowest row the window can reflect to, plus a 32-bit lane offset
            // (saddr + voffset loads; < 47 rows x 2^24)
            const int y0r = max(cy - 23, 0);
            const uint8_t* wbase = img + (long long)y0r * pitch;
            for (int r0 = 0; r0 < RAW_W; r0 += DK_BORDER_RB) {
                uint32_t v[DK_BORDER_RB];
#pragma unroll
                for (int k = 0; k < DK_BORDER_RB; k++) {
                    const int yy = og_reflect101_1(cy - 21 + min(r0 + k, RAW_W - 1), lh);
                    unsigned off = __umul24((unsigned)(yy - y0r), (unsigned)pitch & (OG_MAX_PITCH - 1)) + xx;
                    __asm__("" : "+v"(off));
                    v[k] = wbase[off];
                }
#pragma unroll
                for (int k = 0; k < DK_BORDER_RB; k++)
                    if (lane < RAW_W && r0 + k < RAW_W) R[(r0 + k) * RAW_S + lane] = (uint8_t)v[k];
            }
        }
    }
    og_dk_sync();
    const uint8_t* Rb = R;  // Rb[r * RAW_S + c] = window pixel (r, c)
    // ---- IC_Angle on the unblurred level (:77-104); integer moments are order-independent
    int m01 = 0, m10 = 0;
    if (active) {
        static_assert(RAW_S == 52, "og_make_ic's row stride");
        const uint32_t rb = og_lds_addr(Rb);
        int a10 = 0, a01 = 0;
#pragma unroll
        for (int it = 0; it < OG_IC_ITEMS / 64; it++) {
            auto word = [&](int i) -> uint32_t {
                const uint4 q = icq[i >> 2];
                return (i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w;
            };
            const uint32_t msk = word(3 * it), wt = word(3 * it + 1), ov = word(3 * it + 2);
            typedef const __attribute__((address_space(3))) uint32_t lds_u32;
            const uint32_t d = *(lds_u32*)(uintptr_t)(rb + (ov & 0xffffu)) & msk;
            const int s0 = (int)__builtin_amdgcn_udot4(d, 0x01010101u, 0u, false);
            a10 += (int)__builtin_amdgcn_udot4(d, wt, 0u, false) - 16 * s0;
            a01 += ((int)ov >> 16) * s0;
        }
        m01 = og_wave_sum(a01);
        m10 = og_wave_sum(a10);
    }
    const float angle = og_fast_atan2((float)m01, (float)m10);
    // ---- 7x7 Gaussian (sigma 2, BORDER_REFLECT_101) at the rBRIEF samples.  Integer weights gk[i]*gk[j] summed
    // exactly and rounded once, so any factoring is exact.  The kernel [c0,c1,c2,c3,c2,c1,c0] and the rounding follow
    // the context's ORBGPU_SEM_BLUR_* variant: (acc + 2^15) >> 16, except that the SSE2 variant
    // rounds ties half-to-even in columns x < 4*floor(w/4) (OpenCV 3.x SymmColumnVec_32s8u: float sums, cvtps2dq).
    // Horizontal pass over the window with v_dot4_u32_u8: item = (row pair rp, 4-column group g): rows 2rp, 2rp+1,
    // outputs 4g..4g+3, stored as (row 2rp, row 2rp+1) u16 pairs Hp[rp][col] (<= 257 * 255 = 65535, exact in u16)
    constexpr uint32_t gc = og_blur_coefs[BV];  // c0 | c1 << 8 | c2 << 16 | c3 << 24
    constexpr uint32_t c0 = gc & 0xff, c1 = (gc >> 8) & 0xff, c2 = (gc >> 16) & 0xff, c3 = gc >> 24;
    // the lane's four rBRIEF test pairs, loaded here: in flight over the blur pass
    float4 pfs[4] = {};
#if defined(__HIP_DEVICE_COMPILE__)
    {
        typedef const __attribute__((address_space(1))) float4 g_f4;
        g_f4* pb = (g_f4*)og_pattern_f;
        __asm__("" : "+s"(pb));  // one SGPR base: a lane offset and 1 KB immediate steps
#pragma unroll
        for (int t = 0; t < 4; t++) pfs[t] = pb[lane + 64 * t];
    }
#endif
    if (active) {
        // item it = lane + 64 k = (row pair rp, 4-column group g) for k = 0..3 (220 items): from one item to the lane's
        // next, rp advances by 6 and g by 4, with one wrap of g past 10 into rp; the item's raw-window and Hp byte
        // addresses advance with them (adds and one select per step instead of a division and multiplies per item)
        int g = lane % 10, rp = lane / 10;
        uint32_t ar = (uint32_t)(2 * rp * RAW_S + 4 * g);    // byte offset in the raw window: row 2 rp, dword g
        uint32_t ah = (uint32_t)(4 * (rp * HP_S + 4 * g));   // byte offset of Hp[rp][4 g]
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (k < 3 || lane + 64 * k < HP_ROWS * 10) {
                uint32_t hv[2][4];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    // row 2 rp + h, clamped to row 42 (pair 21's high half, row 43, is never read)
                    const uint32_t a = h == 0 || rp < HP_ROWS - 1 ? ar + (uint32_t)(h * RAW_S) : ar;
                    const uint32_t* rr = (const uint32_t*)(Rb + a);
                    const uint32_t d0 = rr[0], d1 = rr[1], d2 = rr[2];
                    // output k = sum over the window bytes k .. k+6 of d0:d1:d2: the weights shift, not the data --
                    // 2, 2, 3, 3 dot4 for k = 0..3
                    constexpr uint32_t W00 = c0 | c1 << 8 | c2 << 16 | c3 << 24, W01 = c2 | c1 << 8 | c0 << 16;
                    constexpr uint32_t W10 = c0 << 8 | c1 << 16 | c2 << 24, W11 = c3 | c2 << 8 | c1 << 16 | c0 << 24;
                    constexpr uint32_t W20 = c0 << 16 | c1 << 24, W21 = c2 | c3 << 8 | c2 << 16 | c1 << 24, W22 = c0;
                    constexpr uint32_t W30 = c0 << 24, W31 = c1 | c2 << 8 | c3 << 16 | c2 << 24, W32 = c1 | c0 << 8;
                    hv[h][0] = __builtin_amdgcn_udot4(d1, W01, __builtin_amdgcn_udot4(d0, W00, 0u, false), false);
                    hv[h][1] = __builtin_amdgcn_udot4(d1, W11, __builtin_amdgcn_udot4(d0, W10, 0u, false), false);
                    hv[h][2] = __builtin_amdgcn_udot4(d2, W22, __builtin_amdgcn_udot4(d1, W21, __builtin_amdgcn_udot4(d0, W20, 0u, false), false), false);
                    hv[h][3] = __builtin_amdgcn_udot4(d2, W32, __builtin_amdgcn_udot4(d1, W31, __builtin_amdgcn_udot4(d0, W30, 0u, false), false), false);
                }
                // (row 2 rp, row 2 rp + 1) u16 pairs: one v_perm each (sums <= 65535)
                *(uint4*)((uint8_t*)Hp + ah) = make_uint4(__builtin_amdgcn_perm(hv[1][0], hv[0][0], 0x05040100u),
                                                     __builtin_amdgcn_perm(hv[1][1], hv[0][1], 0x05040100u),
                                                     __builtin_amdgcn_perm(hv[1][2], hv[0][2], 0x05040100u),
                                                     __builtin_amdgcn_perm(hv[1][3], hv[0][3], 0x05040100u));
            }
            if (k < 3) {
                const bool wrap = g >= 6;  // g + 4 >= 10
                g += wrap ? 4 - 10 : 4;
                rp += wrap ? 7 : 6;
                ar += wrap ? 6 * 2 * RAW_S + 16 + 2 * RAW_S - 40 : 6 * 2 * RAW_S + 16;
                ah += 4 * (6 * HP_S + 4 * 4);  // (7 HP_S - 4 * 6 when g wraps: the same 256 dwords)
            }
        }
    }
    og_dk_sync();
    if (!active) return;
    // ---- rBRIEF (:108-147)
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float a, b;
    og_sincosf(angle * factorPI, &b, &a);
    constexpr bool nofma = NOFMA;
    // The tests read 512 blurred pixels of the 37x37 window; each is the vertical 7-tap sum over the row-pair
    // horizontal sums Hp at its own column: 4 dword reads and 4 v_dot2 (even rows taps (g0,g1)(g2,g3)(g4,g5)(g6,0),
    // odd rows (0,g0)(g1,g2)(g3,g4)(g5,g6)), rounded by the context's variant.
    typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
    const int xsimd_s = BV == 0 ? ((lw & ~3) - (cx - 18)) : 0;  // window columns < xsimd_s round half-to-even
    // ALLEVEN: every window column is < xsimd_s (the usual case away from the level's right edge)
    // y = 18 + row, xw = 18 + col: window coordinates of a sample at offsets |row|, |col| <= 18 from the centre
    const uint32_t hpb = og_lds_addr(Hp);
    auto blurred = [&](unsigned y, unsigned xw, auto alleven) -> int {
        // LDS byte address of Hp[(y >> 1) * HP_S + xw]: one 24-bit multiply-add and one shift-add (v_mul_lo_u32 is
        // quarter rate); the four tap rows are the immediate offsets of two ds_read2_b32
        typedef const __attribute__((address_space(3))) uint32_t lds_u32;
        lds_u32* h = (lds_u32*)(uintptr_t)((__umul24(y >> 1, HP_S) + xw) * 4u + hpb);
        // the tap weights by row parity, each one v_alignbyte of two constants (the odd form, and the even form's high
        // half): a 16-bit funnel shift for even rows ((2y + 2) & 3 = 2 iff y is even), none for odd rows
        // (asm: the high dword is an inline constant and the low one an SGPR; the compiler's own choice re-creates each
        // low constant in a VGPR with a v_mov per sample)
        const unsigned sh = 2u * y + 2u;
        auto wsel = [&](auto hi, uint32_t lo) -> u16x2v {
            uint32_t r;
            __asm__("v_alignbyte_b32 %0, %1, %2, %3" : "=v"(r) : "n"(decltype(hi)::value), "s"(lo), "v"(sh));
            return __builtin_bit_cast(u16x2v, r);
        };
        const u16x2v w0 = wsel(std::integral_constant<uint32_t, c1>{}, c0 << 16);
        const u16x2v w1 = wsel(std::integral_constant<uint32_t, c3>{}, c1 | c2 << 16);
        const u16x2v w2 = wsel(std::integral_constant<uint32_t, c1>{}, c3 | c2 << 16);
        const u16x2v w3 = wsel(std::integral_constant<uint32_t, 0u>{}, c1 | c0 << 16);
        uint32_t acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, h[0]), w0, 0u, false);
        acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, h[HP_S]), w1, acc, false);
        acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, h[2 * HP_S]), w2, acc, false);
        acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, h[3 * HP_S]), w3, acc, false);
        uint32_t v;
        if (BV == 0) {
            const uint32_t up = decltype(alleven)::value ? 0u : ((int)xw < xsimd_s ? 0u : 1u);
            v = (acc + 0x7fffu + (__builtin_amdgcn_ubfe(acc, 16, 1) | up)) >> 16;
        } else {
            v = (acc + (1u << 15)) >> 16;
        }
        return (int)min(v, 255u);
    };
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v ab = {a, b}, ba = {b, a};
    auto brief_words = [&](auto alleven, u64 (&words)[4]) {
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const float4 pf = pfs[t];
            const f2v xy[2] = {f2v{pf.x, pf.y}, f2v{pf.z, pf.w}};
            int val[2];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                // GCC -O3 -march=native contracts the first product of GET_VALUE into an FMA; a build
                // without contraction rounds both products (the kernels are compiled -ffp-contract=off).
                // (row, col) = (x b + y a, x a - y b) as one pair of packed f32 ops: the products, the sums and the FMAs
                // round exactly as the scalar statements of the reference.  op_sel picks x or y out of the (x, y) pair
                // for both halves, neg_hi negates y b in the high half only.
                f2v yab, rc;
                __asm__("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(yab) : "v"(xy[q]), "v"(ab));
                if (nofma) {
                    f2v xba;
                    __asm__("v_pk_mul_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1]" : "=v"(xba) : "v"(xy[q]), "v"(ba));
                    __asm__("v_pk_add_f32 %0, %1, %2 neg_lo:[0,0] neg_hi:[0,1]" : "=v"(rc) : "v"(xba), "v"(yab));
                } else {
                    __asm__("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1] neg_lo:[0,0,0] neg_hi:[0,0,1]"
                            : "=v"(rc)
                            : "v"(xy[q]), "v"(ba), "v"(yab));
                }
                val[q] = blurred(og_cvround_plus(rc.x, 18), og_cvround_plus(rc.y, 18), alleven);
            }
            words[t] = og_ballot(val[0] < val[1]);
        }
    };
    u64 words[4];
    if (BV == 0 && xsimd_s >= BL_W)  // wave-uniform: the whole window rounds half-to-even
        brief_words(std::integral_constant<bool, true>{}, words);
    else
        brief_words(std::integral_constant<bool, false>{}, words);
    const unsigned o = (unsigned)f * (unsigned)P.frame_cap + (unsigned)g;  // < 2^31 (host plan)
    if (lane < 4) {
        u64 v = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
        ((u64*)(desc + (size_t)o * 32))[lane] = v;
    }
    if (lane == 0) {
        const OgLevel& L = P.lv[l];
        orbgpu_kp_dev k;
        float x = (float)cx, y = (float)cy;
        if (l != 0) {
            x = x * L.scale;
            y = y * L.scale;
        }
        k.x = x;
        k.y = y;
        k.size = (float)L.patch_size;
        k.angle = angle;
        k.response = (P.sem & ORBGPU_SEM_SCORE_HARRIS) ? og_harris_unkey(resp) : (float)resp;
        k.octave = l;
        k.class_id = -1;
        kps[o] = k;
    }
}

// ------------------------------------------------------------------------------------------------
// k5: Frame::AssignFeaturesToGrid (src/Frame.cc:230-245, PosInGrid :382-392)
// ------------------------------------------------------------------------------------------------
// OG_GRID_LDS_ITEMS (orbgpu_internal.h): the frame capacity the plan enforces, so every frame's items fit in LDS
// insertion sort of one cell's item indices [b, e) (a few items per cell)
template <typename T>
__device__ __forceinline__ void og_sort_cell(T* SI, int b, int e)
{
    for (int p = b + 1; p < e; p++) {
        const int v = SI[p];
        int q = p - 1;
        while (q >= b && SI[q] > v) {
            SI[q + 1] = SI[q];
            q--;
        }
        SI[q + 1] = v;
    }
}
#define GRID_NT 1024
// one 1024-thread workgroup per frame, everything in LDS (~72 KB): each keypoint's cell is computed once (kept in
// cellOf), counted, scanned, scattered into LDS, and the per-cell insertion sort restores index order.
// record_refused (the extraction's grid launch only): frame 0 now holds an extracted frame, so the context's
// "frame 0 came from a refused record" word (status[1], og_record_check_kernel) is cleared
__global__ __launch_bounds__(GRID_NT) void og_grid_kernel(const orbgpu_kp_dev* __restrict__ kps,
                                                          const int* __restrict__ counts, int frame_cap,
                                                          OgGridGeom G, int* __restrict__ cell_start,
                                                          int* __restrict__ cell_items, int* __restrict__ status,
                                                          int* __restrict__ record_refused)
{
    if (record_refused && blockIdx.x == 0 && threadIdx.x == 0) *record_refused = 0;
    __shared__ int cnt[OG_GRID_CELLS + 1];
    __shared__ int wsum[32];
    __shared__ int starts[OG_GRID_CELLS + 1];
    __shared__ int sitems[OG_GRID_LDS_ITEMS];
    __shared__ uint16_t cellOf[OG_GRID_LDS_ITEMS];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = counts[f];
    const orbgpu_kp_dev* K = kps + (long long)f * frame_cap;
    int* CS = cell_start + (long long)f * (OG_GRID_CELLS + 1);
    int* CI = cell_items + (long long)f * frame_cap;
    // every frame's items fit: counts[f] <= frame_cap <= OG_GRID_LDS_ITEMS (build_plan); checked, never trusted
    if (n < 0 || n > min(frame_cap, OG_GRID_LDS_ITEMS)) {
        if (tid == 0) atomicOr(status, 64);
        return;
    }
    constexpr int per = OG_GRID_CELLS / GRID_NT;
    static_assert(per * GRID_NT == OG_GRID_CELLS, "cells per thread");
#pragma unroll
    for (int q = 0; q < per; q++) cnt[tid * per + q] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += GRID_NT) {
        const int px = (int)roundf((K[i].x - G.minX) * G.invW);
        const int py = (int)roundf((K[i].y - G.minY) * G.invH);
        int c = 0xffff;
        if (px >= 0 && px < OG_GRID_COLS && py >= 0 && py < OG_GRID_ROWS) {  // PosInGrid, src/Frame.cc:382-392
            c = px * OG_GRID_ROWS + py;
            atomicAdd(&cnt[c], 1);
        }
        cellOf[i] = (uint16_t)c;
    }
    __syncthreads();
    int local[per];
    int sum = 0;
#pragma unroll
    for (int q = 0; q < per; q++) {
        local[q] = sum;
        sum += cnt[tid * per + q];
    }
    int tot;
    const int ex = og_block_excl_scan(sum, wsum, &tot);
#pragma unroll
    for (int q = 0; q < per; q++) {
        CS[tid * per + q] = starts[tid * per + q] = ex + local[q];
        cnt[tid * per + q] = ex + local[q];  // cursors (each thread rewrites only its own cells)
    }
    if (tid == 0) CS[OG_GRID_CELLS] = starts[OG_GRID_CELLS] = tot;
    __syncthreads();
    const int nin = tot;
    for (int i = tid; i < n; i += GRID_NT) {
        const int c = cellOf[i];
        if (c != 0xffff) {
            const int pos = atomicAdd(&cnt[c], 1);
            if (pos >= 0 && pos < nin) sitems[pos] = i;
            else atomicOr(status, 64);
        }
    }
    __syncthreads();
    // restore ascending index order inside each cell (push_back order of the reference): an insertion sort per
    // cell (a few items each) in LDS.  Ranges are checked: DS instructions drop out-of-range LDS accesses
    // silently, so a bad range raises status bit 64 instead of passing unnoticed.
#pragma unroll
    for (int q = 0; q < per; q++) {
        const int c = tid * per + q;
        const int b = starts[c], e = starts[c + 1];
        if (b < 0 || b > e || e > nin) {
            atomicOr(status, 64);
            continue;
        }
        og_sort_cell(sitems, b, e);
    }
    __syncthreads();
    for (int p = tid; p < nin; p += GRID_NT) {
        const int v = sitems[p];
        if (v < 0 || v >= n) atomicOr(status, 64);  // every item is a keypoint index of this frame
        CI[p] = v;
    }
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
hipError_t og_upload_pattern(int device)
{
    if (device >= 0 && device < 64 && g_pattern_uploaded_dev[device]) return hipSuccess;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(og_pattern), oo_orb_pattern, sizeof(oo_orb_pattern), 0,
                                     hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        float pf[1024];
        for (int i = 0; i < 1024; i++) pf[i] = (float)oo_orb_pattern[i];
        e = hipMemcpyToSymbol(HIP_SYMBOL(og_pattern_f), pf, sizeof(pf), 0, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && device >= 0 && device < 64) g_pattern_uploaded_dev[device] = true;
    return e;
}

hipError_t og_read_oct_prof(unsigned long long* out, int n)
{
#if OG_OCT_PROFILE
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(og_oct_prof), sizeof(unsigned long long) * (size_t)std::min(n, 256));
#else
    (void)out;
    (void)n;
    return hipErrorNotSupported;
#endif
}

void og_launch_resize(hipStream_t s, const uint8_t* src, long long src_pitch, long long src_fstride, uint8_t* dst,
                      long long dst_pitch, long long dst_fstride, int sw, int sh, int dw, int dh, const int4* xtab,
                      const int4* ytab, int xmax, int* status, int B, int sem)
{
    dim3 grid((dw + RZ_TW - 1) / RZ_TW, (dh + RZ_TH - 1) / RZ_TH, B);
    if (sem & ORBGPU_SEM_RESIZE_FIXEDPT)
        hipLaunchKernelGGL(og_resize_kernel<true>, grid, dim3(RZ_NT), 0, s, src, src_pitch, src_fstride, dst, dst_pitch,
                           dst_fstride, sw, sh, dw, dh, xtab, ytab, xmax, status);
    else
        hipLaunchKernelGGL(og_resize_kernel<false>, grid, dim3(RZ_NT), 0, s, src, src_pitch, src_fstride, dst,
                           dst_pitch, dst_fstride, sw, sh, dw, dh, xtab, ytab, xmax, status);
}

// the fused resize takes up to 64 KB of dynamic LDS: set once per device (the attribute is per device), from
// orbgpu_create after hipSetDevice
hipError_t og_prepare_device()
{
    hipError_t e = hipFuncSetAttribute((const void*)og_resize2_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)og_resize2_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                64 * 1024);
    if (e == hipSuccess) e = og_prepare_device_match();
    if (e == hipSuccess) e = og_prepare_device_bow();
    return e;
}

void og_launch_resize2(hipStream_t s, const uint8_t* src, long long src_pitch, long long src_fstride, uint8_t* dstA,
                       long long pitchA, uint8_t* dstB, long long pitchB, long long dst_fstride, const OgRz2Geom& g,
                       int* status, int B, int sem)
{
    const size_t shm = og_rz2_lds_bytes(g.SR, g.SC, g.AR, g.AC);
    dim3 grid((g.bw + RZ_TW - 1) / RZ_TW, (g.bh + RZ2_TH - 1) / RZ2_TH, B);
    if (sem & ORBGPU_SEM_RESIZE_FIXEDPT)
        hipLaunchKernelGGL(og_resize2_kernel<true>, grid, dim3(RZ2_NT), shm, s, src, src_pitch, src_fstride, dstA,
                           pitchA, dstB, pitchB, dst_fstride, g, status);
    else
        hipLaunchKernelGGL(og_resize2_kernel<false>, grid, dim3(RZ2_NT), shm, s, src, src_pitch, src_fstride, dstA,
                           pitchA, dstB, pitchB, dst_fstride, g, status);
}

void og_launch_fast(hipStream_t s, const OgPlan& P, int lb, int le, const OgFastBlk* table, const uint8_t* img0,
                    long long pitch0, long long fstride0, const uint8_t* pyr, u64* cand, int* cand_count, int* status,
                    int B)
{
    le = std::min(le, P.nlevels);
    if (lb >= le || B <= 0) return;
    const int thr = std::min(std::max(P.iniTh, 0), 255) | (std::min(std::max(P.minTh, 0), 255) << 8);
    // the levels' table range (level-major); the kernel interleaves the frames of each 64-frame chunk in dispatch
    // order, so a frame's blocks share one XCD
    const int p0 = P.lv[lb].fb_off, p1 = le < P.nlevels ? P.lv[le].fb_off : P.fast_blocks;
    if (p1 <= p0) return;
    const int G = std::min(B, (int)FB_FCHUNK);
    hipLaunchKernelGGL(og_fast_quad_kernel, dim3(G, p1 - p0, (B + G - 1) / G), dim3(FB_NT), 0, s, table + p0, p1 - p0,
                       img0, pitch0, fstride0, pyr, P.pyr_per_frame, cand, P.cand_per_frame, cand_count, P.nlevels, thr,
                       status, B);
}

void og_launch_harris(hipStream_t s, const OgPlan& P, int lb, int le, const uint8_t* img0, long long pitch0,
                      long long fstride0, const uint8_t* pyr, u64* cand, const int* cand_count, int B)
{
    le = std::min(le, P.nlevels);
    int g = 0;
    for (int l = lb; l < le; l++) g += og_harris_groups(P.lv[l].cand_cap);
    if (g <= 0 || B <= 0) return;
    hipLaunchKernelGGL(og_harris_kernel, dim3(g, B), dim3(HR_NT), 0, s, P, img0, pitch0, fstride0, pyr, cand,
                       cand_count, lb, le);
}

void og_launch_octree(hipStream_t s, const OgPlan& P, int lb, int le, const u64* cand, const int* cand_count,
                      uint16_t* node_of, unsigned* oct_best, uint32_t* oct_xy, uint32_t* oct_resp, int* oct_count,
                      int* status, int B)
{
    // levels whose list may exceed OG_OCT_MAXL (more than ~1000 features: the finest levels, P.oct_big of them)
    // take the 2-nodes-per-thread kernel; the rest the 1-node-per-thread one
    le = std::min(le, P.nlevels);
    const int b0 = lb, b1 = std::min(le, P.oct_big), s0 = std::max(lb, P.oct_big), s1 = le;
    if (b1 > b0)
        hipLaunchKernelGGL(og_octree_big_kernel<OG_OCT_MAXL_BIG>, dim3((b1 - b0) * B), dim3(OCT_NT), 0, s, P, b0, cand,
                           cand_count, node_of, oct_xy, oct_resp, oct_count, status, b1 - b0);
    if (s1 > s0)
        hipLaunchKernelGGL(og_octree_kernel, dim3((s1 - s0) * B), dim3(OCT_NT), 0, s, P, s0, cand,
                           cand_count, node_of, oct_best, oct_xy, oct_resp, oct_count, status, s1 - s0);
}

void og_launch_describe(hipStream_t s, const OgPlan& P, const uint8_t* img0, long long pitch0, long long fstride0,
                        const uint8_t* pyr, const uint32_t* oct_xy, const uint32_t* oct_resp, const int* oct_count,
                        orbgpu_kp_dev* kps, uint8_t* desc, int* counts, int B)
{
    const int blocks = (P.frame_cap + DK_WAVES - 1) / DK_WAVES;
    const int bv = (P.sem >> ORBGPU_SEM_BLUR_SHIFT) & 3;
    const bool nofma = (P.sem & ORBGPU_SEM_BRIEF_NOFMA) != 0;
    // the 8 (blur variant, rotation form) instantiations
    using K = void (*)(OgPlan, const uint8_t*, long long, long long, const uint8_t*, const uint32_t*, const uint32_t*,
                       const int*, orbgpu_kp_dev*, uint8_t*, int*, unsigned);
    static const K table[8] = {og_describe_kernel<0, false>, og_describe_kernel<1, false>, og_describe_kernel<2, false>,
                               og_describe_kernel<3, false>, og_describe_kernel<0, true>,  og_describe_kernel<1, true>,
                               og_describe_kernel<2, true>,  og_describe_kernel<3, true>};
    // lin / blocks == mulhi(lin, floor(2^32 / blocks) + 1) for every lin < blocks * B when blocks^2 * B < 2^32
    const unsigned long long d = (unsigned long long)blocks;
    const unsigned dmagic = (d > 1 && d * d * (unsigned long long)B < (1ull << 32)) ? (unsigned)((1ull << 32) / d + 1) : 0u;
    hipLaunchKernelGGL(table[bv + 4 * nofma], dim3(blocks, B), dim3(64 * DK_WAVES), 0, s, P, img0, pitch0, fstride0,
                       pyr, oct_xy, oct_resp, oct_count, kps, desc, counts, dmagic);
}

// the batch's per-(frame, level) candidate counters to zero: a kernel rather than hipMemsetAsync, so that a batch's
// launch sequence holds kernels only (a captured memset node replayed after synchronous device-to-host copies
// faulted under the runtime's graph packet capture)
__global__ __launch_bounds__(256) void og_zero_kernel(int* __restrict__ p, int n)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = 0;
}

void og_launch_zero(hipStream_t s, int* p, int n)
{
    if (n > 0) hipLaunchKernelGGL(og_zero_kernel, dim3(std::min((n + 255) / 256, 1024)), dim3(256), 0, s, p, n);
}

void og_launch_grid(hipStream_t s, const orbgpu_kp_dev* kps, const int* counts, int frame_cap, OgGridGeom G,
                    int* cell_start, int* cell_items, int* status, int B, int* record_refused)
{
    hipLaunchKernelGGL(og_grid_kernel, dim3(B), dim3(GRID_NT), 0, s, kps, counts, frame_cap, G, cell_start, cell_items,
                       status, record_refused);
}
