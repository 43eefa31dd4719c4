// orb_stereo.hip -- gfx950 kernels of Frame::ComputeStereoMatches (src/Frame.cc:466-640).
//
//   og_stereo_rows_kernel   : vRowIndices (:476-493) as a CSR over image rows, right keypoints of each
//                             row in index order (one workgroup per frame pair)
//   og_stereo_match16_kernel: 16 lanes per left keypoint: row-band Hamming search (levels +-1, u-range,
//                             strict-< first minimum, :504-549), 11x121 SAD sliding window on both
//                             pyramids with DPP row reductions (exact integers), parabola sub-pixel fit,
//                             disparity / depth (:552-622)
//   og_stereo_filter_kernel : median of the SAD distances by two-pass radix select, 2.1 x median
//                             rejection (:626-639)
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "orb_math_dev.h"
#include "orbgpu_internal.h"
#include "orbgpu_launch.h"

typedef unsigned long long u64;

#define ST_TH_HIGH 100
#define ST_TH_LOW 50
#define ST_MAXROWS 8192

// vRowIndices (src/Frame.cc:476-493): right keypoint iR is pushed to every row of its band
// [floor(y - 2 sf), ceil(y + 2 sf)] in index order.  Band ends live in LDS; row counts come from LDS atomics and
// a block scan; then each row is filled by one thread that walks the keypoints in index order (LDS broadcast
// reads), so every row list is in push_back order without sorting.
#define ST_NT 1024
#define ST_MAXR 8192      // right keypoints held in LDS
__global__ __launch_bounds__(ST_NT) void og_stereo_rows_kernel(OgStereoDev S)
{
    __shared__ int cnt[ST_MAXROWS + 1];
    __shared__ short lo_[ST_MAXR], hi_[ST_MAXR];
    __shared__ int wsum[ST_NT / 64];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int Nr = min(S.R.counts[b], ST_MAXR);
    const orbgpu_kp_dev* KR = S.R.kps + (long long)b * S.R.frame_cap;
    int* RS = S.row_start + (long long)b * (S.nRows + 1);
    int* RI = S.row_items + (long long)b * S.row_cap;
    for (int y = tid; y <= S.nRows; y += ST_NT) cnt[y] = 0;
    __syncthreads();
    for (int iR = tid; iR < Nr; iR += ST_NT) {
        const float kpY = KR[iR].y;
        const float r = 2.0f * S.sf[KR[iR].octave];
        const int lo = max((int)floorf(kpY - r), 0), hi = min((int)ceilf(kpY + r), S.nRows - 1);
        lo_[iR] = (short)lo;
        hi_[iR] = (short)hi;
        for (int yi = lo; yi <= hi; yi++) atomicAdd(&cnt[yi], 1);
    }
    __syncthreads();
    // exclusive scan of cnt[0..nRows) in chunks of ST_NT
    int carry = 0;
    for (int y0 = 0; y0 < S.nRows; y0 += ST_NT) {
        const int y = y0 + tid;
        const int v = y < S.nRows ? cnt[y] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(x, o);
            if (lane >= o) x += t;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        int before = carry, tot = 0;
        for (int q = 0; q < ST_NT / 64; q++) {
            if (q < wv) before += wsum[q];
            tot += wsum[q];
        }
        if (y < S.nRows) RS[y] = before + x - v;
        __syncthreads();
        carry += tot;
    }
    if (tid == 0) RS[S.nRows] = carry;
    __syncthreads();
    __threadfence_block();
    // each row's list in index order: the wave takes the keypoints 64 at a time, ballots the ones whose band holds
    // the row and writes them at their rank (index order within the ballot, the ballots in index order)
    for (int y = wv; y < S.nRows; y += ST_NT / 64) {
        int pos = RS[y];
        const int end = min(pos + cnt[y], S.row_cap);
        for (int c = 0; c < Nr && pos < end; c += 64) {
            const int iR = c + lane;
            const bool in = iR < Nr && lo_[iR] <= y && y <= hi_[iR];
            const u64 m = __ballot(in);
            const int r = __popcll(m & ((1ull << lane) - 1ull));
            if (in && pos + r < end) RI[pos + r] = iR;
            pos += __popcll(m);
        }
    }
}

// ---- og_stereo_match16_kernel: one left keypoint per 16 lanes (4 keypoints per wave, 16 per 256-thread workgroup):
// row-band Hamming search (levels +-1, u-range, strict-< first minimum, src/Frame.cc:504-549), 11x121 SAD sliding
// window on both pyramids (exact integers), parabola sub-pixel fit, disparity / depth (:552-622).  Every cross-lane step stays inside a 16-lane DPP row (row_ror / quad_perm
// min and add reductions: VALU, no LDS round trips), and the SAD is computed from registers: lane r < 11 loads row
// r - 5 of the 11-pixel left window and of the 21-pixel right band (all 11 window positions), then forms its 11 row
// sums with v_sad_u32.
__device__ __forceinline__ unsigned og_row16_min(unsigned v)
{
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));  // row_ror:8
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false));  // row_ror:4
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
    return v;
}
__device__ __forceinline__ int og_row16_sum(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x4e, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0xb1, 0xf, 0xf, false);
    return v;
}

__global__ __launch_bounds__(256) void og_stereo_match16_kernel(OgStereoDev S)
{
    const int b = blockIdx.y, l = threadIdx.x & 15;
    const int iL = blockIdx.x * 16 + (threadIdx.x >> 4);
    const int N = S.L.counts[b];
    if (iL >= N) return;  // whole 16-lane groups leave together
    float* UR = S.uright + (long long)b * S.L.frame_cap;
    float* DE = S.depth + (long long)b * S.L.frame_cap;
    int* SAD = S.sad + (long long)b * S.L.frame_cap;
    if (l == 0) {
        UR[iL] = -1.0f;
        DE[iL] = -1.0f;
        SAD[iL] = -1;
    }
    const orbgpu_kp_dev kpL = S.L.kps[(long long)b * S.L.frame_cap + iL];
    const orbgpu_kp_dev* KR = S.R.kps + (long long)b * S.R.frame_cap;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;
    if (row < 0 || row >= S.nRows) return;
    const int* RS = S.row_start + (long long)b * (S.nRows + 1);
    const int* RI = S.row_items + (long long)b * S.row_cap;
    const int cb = RS[row], ce = min(RS[row + 1], S.row_cap);
    if (cb == ce) return;
    const float minZ = S.mb, minD = 0;
    const float maxD = S.mbf / minZ;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) return;
    // ---- row-band Hamming search: the first strict minimum below TH_HIGH in candidate order
    uint4 da, db;
    {
        const uint4* q = (const uint4*)(S.L.desc + ((long long)b * S.L.frame_cap + iL) * 32);
        da = q[0];
        db = q[1];
    }
    // (dist << 16) | (candidate position): smallest distance, then first in order.  The position is the index in one
    // row list, which holds at most ST_MAXR right keypoints, so it fits the low 16 bits.
    static_assert(ST_MAXR <= 65535, "row-list positions are packed into 16 bits");
    unsigned best = 0xffffffffu;
#define OG_ST_BAND_U 4  // band candidates per lane whose dependent loads (list entry, keypoint, descriptor) are batched
    // each stage's loads for OG_ST_BAND_U candidates are issued together: 3 memory round trips per batch instead of 3
    // per candidate (the candidate order only enters through the packed position, so the batching is exact)
    for (int c0 = cb + l; c0 < ce; c0 += 16 * OG_ST_BAND_U) {
        int iR[OG_ST_BAND_U];
#pragma unroll
        for (int u = 0; u < OG_ST_BAND_U; u++) {
            const int c = c0 + 16 * u;
            iR[u] = c < ce ? RI[c] : -1;
        }
        bool pass[OG_ST_BAND_U];
#pragma unroll
        for (int u = 0; u < OG_ST_BAND_U; u++) {
            pass[u] = false;
            if (iR[u] >= 0) {
                const orbgpu_kp_dev* kr = KR + iR[u];
                const int oct = kr->octave;
                const float uR = kr->x;
                pass[u] = !(oct < levelL - 1 || oct > levelL + 1) && uR >= minU && uR <= maxU;
            }
        }
        uint4 qa[OG_ST_BAND_U], qb[OG_ST_BAND_U];
#pragma unroll
        for (int u = 0; u < OG_ST_BAND_U; u++) {
            qa[u] = qb[u] = make_uint4(0u, 0u, 0u, 0u);
            if (pass[u]) {
                const uint4* q = (const uint4*)(S.R.desc + ((long long)b * S.R.frame_cap + iR[u]) * 32);
                qa[u] = q[0];
                qb[u] = q[1];
            }
        }
#pragma unroll
        for (int u = 0; u < OG_ST_BAND_U; u++) {
            if (pass[u]) {
                const int dist = og_hamming(da, db, qa[u], qb[u]);
                if (dist < ST_TH_HIGH) best = min(best, ((unsigned)dist << 16) | (unsigned)(c0 + 16 * u - cb));
            }
        }
    }
    best = og_row16_min(best);
    const int thOrbDist = (ST_TH_HIGH + ST_TH_LOW) / 2;
    if (best == 0xffffffffu || (int)(best >> 16) >= thOrbDist) return;
    const int bestIdxR = RI[cb + (int)(best & 0xffffu)];
    // ---- SAD sliding window on the keypoint's pyramid level (:552-592)
    const float uR0 = KR[bestIdxR].x;
    const float scaleFactor = S.isf[levelL];
    const float scaleduL = roundf(kpL.x * scaleFactor);
    const float scaledvL = roundf(kpL.y * scaleFactor);
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const int w = 5, Lw = 5;
    const float iniu = scaleduR0 + Lw - w;
    const float endu = scaleduR0 + Lw + w + 1;
    const int rcols = S.lvl_w[levelL];
    if (iniu < 0 || endu >= rcols) return;
    const uint8_t* IL;
    const uint8_t* IR;
    long long pl, pr;
    if (levelL == 0) {
        IL = S.L0 + (long long)b * S.L0_fstride;
        pl = S.L0_pitch;
        IR = S.R0 + (long long)b * S.R0_fstride;
        pr = S.R0_pitch;
    } else {
        IL = S.Lpyr + (long long)b * S.pyr_fstride + S.lvl_off[levelL];
        IR = S.Rpyr + (long long)b * S.pyr_fstride + S.lvl_off[levelL];
        pl = pr = S.lvl_pitch[levelL];
    }
    const int ivL = (int)scaledvL, iuL = (int)scaleduL, iuR0 = (int)scaleduR0;
    const int ry = min(l, 2 * w) - w;  // window row of this lane (lanes 11-15 repeat row +5 and contribute 0)
    const uint8_t* lrow = IL + (long long)(ivL + ry) * pl + (iuL - w);
    const uint8_t* rrow = IR + (long long)(ivL + ry) * pr + (iuR0 - Lw - w);
    const uint8_t* rctr = IR + (long long)ivL * pr + (iuR0 - Lw);
    const int cL = IL[(long long)ivL * pl + iuL];
    unsigned lv[11], rv[21], cR[11];
#pragma unroll
    for (int x = 0; x < 11; x++) lv[x] = lrow[x];
#pragma unroll
    for (int x = 0; x < 21; x++) rv[x] = rrow[x];
#pragma unroll
    for (int i = 0; i < 11; i++) cR[i] = rctr[i];
    // |(L - cL) - (R - cR_i)| = |(L - cL + cR_i + 512) - (R + 512)|: both operands in [0, 1022], two window pixels
    // per 16-bit half pair, so one v_sad_u16 adds two terms (the 11th pixel pairs with a zero half)
    unsigned LP[6], RP[20];
#pragma unroll
    for (int p = 0; p < 5; p++) LP[p] = lv[2 * p] | (lv[2 * p + 1] << 16);
    LP[5] = lv[10];
#pragma unroll
    for (int x = 0; x < 20; x++) RP[x] = (rv[x] | (rv[x + 1] << 16)) + 0x02000200u;
    int sums[11];
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const unsigned off = cR[i] + 512u - (unsigned)cL;  // in [257, 767]
        unsigned s = 0;
#pragma unroll
        for (int p = 0; p < 5; p++) s = __builtin_amdgcn_sad_u16(LP[p] + off * 0x10001u, RP[2 * p + i], s);
        s = __builtin_amdgcn_sad_u16(LP[5] + off, rv[10 + i] + 512u, s);
        sums[i] = l <= 2 * w ? (int)s : 0;
    }
    int bestD = INT_MAX, bestincR = 0;
    float vDists[11];
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const float dist = (float)og_row16_sum(sums[i]);  // cv::norm(IL, IR, NORM_L1): exact integer
        if (dist < bestD) {
            bestD = (int)dist;
            bestincR = i - Lw;
        }
        vDists[i] = dist;
    }
    if (bestincR == -Lw || bestincR == Lw) return;
    const float dist1 = vDists[Lw + bestincR - 1];
    const float dist2 = vDists[Lw + bestincR];
    const float dist3 = vDists[Lw + bestincR + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) return;
    float bestuR = S.sf[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = (uL - bestuR);
    if (disparity >= minD && disparity < maxD) {
        if (disparity <= 0) {
            disparity = 0.01f;
            bestuR = (float)((double)uL - 0.01);
        }
        if (l == 0) {
            DE[iL] = S.mbf / disparity;
            UR[iL] = bestuR;
            SAD[iL] = bestD;
        }
    }
}

// median of the valid SAD distances (radix select on 16-bit values: <= 121 * 510 = 61710), then the
// 1.5 * 1.4 * median rejection, which removes exactly the entries with (float)dist >= thDist (:626-639)
__global__ __launch_bounds__(256) void og_stereo_filter_kernel(OgStereoDev S)
{
    __shared__ int hist[256];
    __shared__ int sel[4];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int N = S.L.counts[b];
    float* UR = S.uright + (long long)b * S.L.frame_cap;
    float* DE = S.depth + (long long)b * S.L.frame_cap;
    const int* SAD = S.sad + (long long)b * S.L.frame_cap;
    hist[tid] = 0;
    if (tid < 4) sel[tid] = 0;
    __syncthreads();
    int nv = 0;
    for (int i = tid; i < N; i += 256) {
        const int d = SAD[i];
        if (d >= 0) {
            atomicAdd(&hist[(d >> 8) & 255], 1);
            nv++;
        }
    }
    atomicAdd(&sel[0], nv);
    __syncthreads();
    const int n = sel[0];
    if (n == 0) {
        if (tid == 0) S.nmatches[b] = 0;
        return;
    }
    const int k = n / 2;  // vDistIdx[size/2].first
    if (tid == 0) {
        int acc = 0, bin = 0;
        for (; bin < 256; bin++) {
            if (acc + hist[bin] > k) break;
            acc += hist[bin];
        }
        sel[1] = bin;
        sel[2] = k - acc;
    }
    __syncthreads();
    const int hiBin = sel[1], k2 = sel[2];
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < N; i += 256) {
        const int d = SAD[i];
        if (d >= 0 && ((d >> 8) & 255) == hiBin) atomicAdd(&hist[d & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int acc = 0, bin = 0;
        for (; bin < 256; bin++) {
            if (acc + hist[bin] > k2) break;
            acc += hist[bin];
        }
        sel[3] = (hiBin << 8) | bin;
    }
    __syncthreads();
    const float median = (float)sel[3];
    const float thDist = 1.5f * 1.4f * median;
    int rej = 0;
    for (int i = tid; i < N; i += 256) {
        const int d = SAD[i];
        if (d >= 0 && !((float)d < thDist)) {
            UR[i] = -1;
            DE[i] = -1;
            rej++;
        }
    }
    __shared__ int rsum;
    if (tid == 0) rsum = 0;
    __syncthreads();
    atomicAdd(&rsum, rej);
    __syncthreads();
    if (tid == 0) S.nmatches[b] = n - rsum;
}

void og_launch_stereo(hipStream_t s, const OgStereoDev& S, int B)
{
    hipLaunchKernelGGL(og_stereo_rows_kernel, dim3(B), dim3(ST_NT), 0, s, S);
    hipLaunchKernelGGL(og_stereo_match16_kernel, dim3((S.L.frame_cap + 15) / 16, B), dim3(256), 0, s, S);
    hipLaunchKernelGGL(og_stereo_filter_kernel, dim3(B), dim3(256), 0, s, S);
}
