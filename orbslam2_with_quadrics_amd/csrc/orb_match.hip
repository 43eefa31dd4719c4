// orb_match.hip -- gfx950 kernels of the per-frame Hamming matchers.
//
//   og_search_init_kernel : ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:405-520), one
//       64-lane wave per (F1, F2) pair.  Queries run in the reference's order (the vMatchedDistance /
//       vnMatches21 state couples them, :444, :463-470); the candidates of one query are scored in
//       parallel (XOR + popcount over 8 u32) and reduced to (best, second) with a lexicographic
//       (distance, candidate position) wave min -- exactly the reference's strict-< update order.
//   og_projb_fill/resolve : ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)
//       (src/ORBmatcher.cc:45-137) for B frames.  Candidate lists + distances are built in one parallel pass
//       (one thread per map point); the order-dependent claims (:87-89, :123) are resolved by a parallel
//       fixed-point iteration of the triangular claim system over LDS-staged lists (og_projb_resolve_kernel).
#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>
#include <stdint.h>

#include "orb_math_dev.h"
#include "orbgpu_internal.h"
#include "orbgpu_launch.h"

typedef unsigned long long u64;

#define TH_HIGH 100
#define TH_LOW 50
#define HISTO_LENGTH 30

// ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1601-1642) -> (ind1, ind2, ind3), -1 = none
__device__ __forceinline__ int3 og_three_maxima(const int* h)
{
    int max1 = 0, max2 = 0, max3 = 0;
    int ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = h[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    return make_int3(ind1, ind2, ind3);
}

struct OgCellRange {
    int x0, x1, y0, y1;  // inclusive; empty if x0 > x1
};

// Frame::GetFeaturesInArea cell window (src/Frame.cc:332-346)
__device__ __forceinline__ OgCellRange og_cell_range(const OgGridGeom& G, float x, float y, float r)
{
    OgCellRange c;
    c.x0 = max(0, (int)floorf((x - G.minX - r) * G.invW));
    c.x1 = min(OG_GRID_COLS - 1, (int)ceilf((x - G.minX + r) * G.invW));
    c.y0 = max(0, (int)floorf((y - G.minY - r) * G.invH));
    c.y1 = min(OG_GRID_ROWS - 1, (int)ceilf((y - G.minY + r) * G.invH));
    if (c.x0 >= OG_GRID_COLS || c.x1 < 0 || c.y0 >= OG_GRID_ROWS || c.y1 < 0) c.x0 = 1, c.x1 = 0;
    return c;
}

__device__ __forceinline__ void og_load_desc(const uint8_t* p, uint4& a, uint4& b)
{
    const uint4* q = (const uint4*)p;
    a = q[0];
    b = q[1];
}

__device__ __forceinline__ u64 og_wave_min_u64(u64 v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const u64 w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ int og_wave_sum(int v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------------------------------------------------------
// SearchForInitialization, two phases:
//  A. og_init_cand_kernel  -- one wave per (pair, F1 keypoint): Frame::GetFeaturesInArea on F2's grid
//     (src/Frame.cc:327-380: cells ix-major, then iy, then cell order), level filter, window test,
//     Hamming distance; the list {dist:16 | i2:16} is written in candidate order.  Fully parallel.
//  B. og_init_resolve_kernel -- one wave per pair replays the reference's ordered loop
//     (src/ORBmatcher.cc:418-487): only the state-dependent vMatchedDistance filter (:444), the
//     best/second reduction and the steal/rot-hist bookkeeping remain sequential.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void og_init_cand_kernel(OgFrameDev F1, int ref, OgFrameDev F2, OgGridGeom G,
                                                           int windowSize, int dkeep, const float* __restrict__ prev_xy,
                                                           int prev_stride, uint32_t* __restrict__ lists,
                                                           int list_cap, int* __restrict__ list_n)
{
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int i1 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n1 = F1.counts[ref];
    if (i1 >= F1.frame_cap) return;
    int* NC = list_n + (long long)b * F1.frame_cap;
    if (i1 >= n1) return;
    const orbgpu_kp_dev* K1 = F1.kps + (long long)ref * F1.frame_cap;
    const int level1 = K1[i1].octave;
    if (level1 > 0) {
        if (lane == 0) NC[i1] = 0;
        return;
    }
    const float* PV = prev_xy + (long long)b * prev_stride;
    const float x = PV[2 * i1], y = PV[2 * i1 + 1];
    const float r = (float)windowSize;
    const OgCellRange cr = og_cell_range(G, x, y, r);
    if (cr.x0 > cr.x1) {
        if (lane == 0) NC[i1] = 0;
        return;
    }
    const uint8_t* D1 = F1.desc + (long long)ref * F1.frame_cap * 32;
    const orbgpu_kp_dev* K2 = F2.kps + (long long)b * F2.frame_cap;
    const uint8_t* D2 = F2.desc + (long long)b * F2.frame_cap * 32;
    const int* CS = F2.cell_start + (long long)b * (OG_GRID_CELLS + 1);
    const int* CI = F2.cell_items + (long long)b * F2.frame_cap;
    uint32_t* LST = lists + ((long long)b * F1.frame_cap + i1) * list_cap;
    uint4 da, db;
    og_load_desc(D1 + (long long)i1 * 32, da, db);
    const int ncy = cr.y1 - cr.y0 + 1;
    const int ncells = (cr.x1 - cr.x0 + 1) * ncy;
    int n = 0;
    for (int c0 = 0; c0 < ncells; c0 += 64) {
        const int c = c0 + lane;
        int cell = 0, cnt = 0;
        if (c < ncells) {
            cell = (cr.x0 + c / ncy) * OG_GRID_ROWS + (cr.y0 + c % ncy);
            cnt = CS[cell + 1] - CS[cell];
        }
        // inclusive scan of the cell counts with DPP (row_shr 1/2/4/8, then row_bcast 15/31), no LDS round trips
        int incl = cnt;
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xf, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xa, 0xf, false);
        incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xc, 0xf, false);
        const int T = __builtin_amdgcn_readlane(incl, 63);
        const int cellStart = c < ncells ? CS[cell] : 0;
        for (int e = lane; e - lane < T; e += 64) {
            const int ee = min(e, T - 1);
            int lo = 0;  // binary lifting: number of lanes whose inclusive count is <= ee
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const int v = __shfl(incl, lo + step - 1);
                if (v <= ee) lo += step;
            }
            const int ownerIncl = __shfl(incl, lo), ownerCnt = __shfl(cnt, lo), ownerStart = __shfl(cellStart, lo);
            bool valid = false;
            uint32_t entry = 0;
            if (e < T) {
                const int i2 = CI[ownerStart + e - (ownerIncl - ownerCnt)];
                const orbgpu_kp_dev kp2 = K2[i2];
                if (kp2.octave >= level1 && kp2.octave <= level1) {  // src/Frame.cc:361-368
                    const float distx = kp2.x - x, disty = kp2.y - y;
                    if (fabsf(distx) < r && fabsf(disty) < r) {
                        uint4 ea, eb;
                        og_load_desc(D2 + (long long)i2 * 32, ea, eb);
                        const int dist = og_hamming(da, db, ea, eb);
                        entry = ((uint32_t)dist << 16) | (uint32_t)i2;
                        valid = dist <= dkeep;  // og_init_keep_bound: farther candidates cannot change the result
                    }
                }
            }
            const u64 mask = __ballot(valid);
            const int pos = n + __popcll(mask & ((1ull << lane) - 1ull));
            if (valid && pos < list_cap) LST[pos] = entry;
            n += __popcll(mask);
        }
    }
    if (lane == 0) NC[i1] = min(n, list_cap) | (n > list_cap ? (int)0x80000000 : 0);
}

// wave-wide min of a u32 (all 64 lanes active): DPP row_shr prefix minima inside each 16-lane row, then
// the four row results via readlane -- no LDS round trips (ds_bpermute) on the sequential critical path
__device__ __forceinline__ uint32_t og_wave_min_u32(uint32_t v)
{
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return min(min(a, b), min(c, d));
}

#define INIT_NT 256

// One workgroup per pair.  All four waves stage the pair's candidate lists (compacted), the keypoint
// angles and the per-query offsets into LDS; wave 0 then replays the reference's ordered loop
// (src/ORBmatcher.cc:418-487).  The only state a later query reads is vMatchedDistance (:444), so the
// loop keeps just that (u16 in LDS, 0xffff == INT_MAX) and logs every accepted match (i1, i2); the
// next query's entries and their vMatchedDistance values are loaded one query ahead and the single
// entry the current match changes is patched in registers.  Steals (:463-470), the final
// vnMatches12, nmatches and the rotation histogram (including stolen matches' stale entries, :478)
// follow from the log in a parallel pass: vnMatches12[i1] = i2 iff i1 is the last claimant of i2.
__global__ __launch_bounds__(INIT_NT) void og_init_resolve_kernel(
    OgFrameDev F1, int ref, OgFrameDev F2, float nnratio, int checkOri, float* __restrict__ prev_xy,
    int prev_stride, const uint32_t* __restrict__ lists, int list_cap, const int* __restrict__ list_n,
    int* __restrict__ matches12, int match_stride, int* __restrict__ nmatches, int* __restrict__ status, int ecap,
    const int* __restrict__ ref_status, int qcap)
{
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // F1 from another context whose frame 0 now holds a refused frame record (ref_status[1], og_record_check_kernel:
    // F1 was left empty) is reported by this context's next status check too (bit 256), not only as zero matches
    if (ref_status && b == 0 && tid == 0 && ref_status[1]) atomicOr(status, 256);
    const int n1 = F1.counts[ref];
    const int n2 = F2.counts[b];
    const int c1 = F1.frame_cap, c2 = F2.frame_cap;
    float* a1 = (float*)smem;                   // F1 angles               [c1]
    float* a2 = a1 + c1;                        // F2 angles               [c2]
    int* offs = (int*)(a2 + c2);                // list offsets of the active queries [c1 + 1]
    int* own = offs + c1 + 1;                   // last log entry claiming i2 [c2]
    uint32_t* E = (uint32_t*)(own + c2);        // staged entries          [ecap]
    uint16_t* vMD = (uint16_t*)(E + ecap);      // vMatchedDistance        [c2]
    short* m12 = (short*)(vMD + c2);            // vnMatches12             [c1]
    short* log1 = m12 + c1;                     // match log: i1           [c1]
    short* log2 = log1 + c1;                    // match log: i2           [c1]
    short* act = log2 + c1;                     // active queries (F1 indices) [c1]
    signed char* binOf = (signed char*)(act + c1);  // rot-hist bin of i1's match, -1 = none [c1]
    __shared__ int hist[HISTO_LENGTH];
    __shared__ int wsum[INIT_NT / 64];
    __shared__ int wact[INIT_NT / 64];
    __shared__ int sh_nlog;
    const orbgpu_kp_dev* K1 = F1.kps + (long long)ref * c1;
    const orbgpu_kp_dev* K2 = F2.kps + (long long)b * c2;
    const int* NC = list_n + (long long)b * c1;
    const uint32_t* LB = lists + (long long)b * c1 * list_cap;
    for (int i = tid; i < n2; i += INIT_NT) {
        vMD[i] = 0xffff;
        own[i] = -1;
        a2[i] = K2[i].angle;
    }
    for (int i = tid; i < n1; i += INIT_NT) {
        m12[i] = -1;
        binOf[i] = -1;
        a1[i] = K1[i].angle;
    }
    if (tid < HISTO_LENGTH) hist[tid] = 0;
    // the queries that have candidates (octave-0 F1 keypoints with a non-empty window), in order, with
    // the exclusive prefix of their list lengths (overflowed lists count 0 and are reported)
    int na;
    {
        int carry = 0, acarry = 0;
        for (int base = 0; base < n1; base += INIT_NT) {
            const int i = base + tid;
            int v = 0;
            if (i < n1 && i < qcap) {  // (F1 keypoints from qcap on are past level 0: no candidate kernel wave)
                const int raw = NC[i];
                if (raw < 0) atomicOr(status, 16);
                v = raw < 0 ? 0 : raw;
            }
            const u64 am = __ballot(v > 0);
            int x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            if (lane == 63) wsum[wv] = x;
            if (lane == 0) wact[wv] = __popcll(am);
            __syncthreads();
            int before = carry, abefore = acarry;
            for (int q = 0; q < wv; q++) before += wsum[q], abefore += wact[q];
            if (v > 0) {
                const int k = abefore + __popcll(am & ((1ull << lane) - 1ull));
                act[k] = (short)i;
                offs[k] = before + x - v;
            }
            int tot = 0, atot = 0;
            for (int q = 0; q < INIT_NT / 64; q++) tot += wsum[q], atot += wact[q];
            __syncthreads();
            carry += tot;
            acarry += atot;
        }
        na = acarry;
        if (tid == 0) offs[na] = carry;
    }
    __syncthreads();
    int nlog = 0;  // wave 0's register copy of the log length
    // chunks of queries whose entries fit the LDS staging buffer (one list never exceeds ecap)
    for (int qa = 0; qa < na;) {
        int qb;
        {
            int lo = qa, hi = na;  // largest qb with offs[qb] - offs[qa] <= ecap
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (offs[mid] - offs[qa] <= ecap) lo = mid;
                else hi = mid - 1;
            }
            qb = lo;
        }
        const int ebase = offs[qa], tot = offs[qb] - ebase;
        auto src_of = [&](int t) -> long long {  // list slot of staged element t (last q with offs[q] <= g)
            const int g = ebase + t;
            int lo = qa, hi = qb - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (offs[mid] <= g) lo = mid;
                else hi = mid - 1;
            }
            return (long long)act[lo] * list_cap + (g - offs[lo]);
        };
        for (int t0 = 0; t0 < tot; t0 += INIT_NT * 4) {
            const int ta = t0 + tid, tb = ta + INIT_NT, tc = tb + INIT_NT, td = tc + INIT_NT;
            const long long sa = ta < tot ? src_of(ta) : 0, sb = tb < tot ? src_of(tb) : 0;
            const long long sc = tc < tot ? src_of(tc) : 0, sd = td < tot ? src_of(td) : 0;
            const uint32_t va = ta < tot ? LB[sa] : 0u, vb = tb < tot ? LB[sb] : 0u;
            const uint32_t vc = tc < tot ? LB[sc] : 0u, vd = td < tot ? LB[sd] : 0u;
            if (ta < tot) E[ta] = va;
            if (tb < tot) E[tb] = vb;
            if (tc < tot) E[tc] = vc;
            if (td < tot) E[td] = vd;
        }
        __syncthreads();
        if (wv == 0 && qa < qb) {
            // pipeline registers of the next query: its first 64 entries and their vMatchedDistance
            int nOff = offs[qa] - ebase, nCnt = offs[qa + 1] - offs[qa];
            uint32_t nEnt = lane < nCnt ? E[nOff + lane] : 0u;
            int nVmd = lane < nCnt ? (int)vMD[nEnt & 0xffff] : 0;
            int nI1 = act[qa];
            for (int k = qa; k < qb; k++) {
                const int i1 = nI1, eo = nOff, nc = nCnt;
                const uint32_t ent0 = nEnt;
                const int vmd0 = nVmd;
                if (k + 1 < qb) {
                    nI1 = act[k + 1];
                    nOff = offs[k + 1] - ebase;
                    nCnt = offs[k + 2] - offs[k + 1];
                    nEnt = lane < nCnt ? E[nOff + lane] : 0u;
                    nVmd = lane < nCnt ? (int)vMD[nEnt & 0xffff] : 0;
                }
                uint32_t best1 = 0xffffffffu, best2 = 0xffffffffu;  // lane-local two smallest (dist:16 | pos:16)
                int best1i2 = 0;
                for (int e0 = 0; e0 < nc; e0 += 64) {
                    const int e = e0 + lane;
                    if (e < nc) {
                        const uint32_t ent = e0 == 0 ? ent0 : E[eo + e];
                        const int i2 = (int)(ent & 0xffff), dist = (int)(ent >> 16);
                        const int vmd = e0 == 0 ? vmd0 : (int)vMD[i2];
                        if (!(vmd <= dist)) {  // src/ORBmatcher.cc:444 (0xffff == INT_MAX)
                            const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)e;
                            if (key < best1) {
                                best2 = best1;
                                best1 = key;
                                best1i2 = i2;
                            } else if (key < best2) {
                                best2 = key;
                            }
                        }
                    }
                }
                const uint32_t gbest = og_wave_min_u32(best1);
                if (gbest == 0xffffffffu) continue;
                const uint32_t gsecond = og_wave_min_u32(best1 == gbest ? best2 : best1);
                const int bestDist = (int)(gbest >> 16);
                const int bestDist2 = gsecond == 0xffffffffu ? INT_MAX : (int)(gsecond >> 16);
                if (bestDist <= TH_LOW && bestDist < (float)bestDist2 * nnratio) {
                    const int bestIdx2 = __builtin_amdgcn_readlane(best1i2, (int)(gbest & 63));
                    if (lane == 0) {
                        vMD[bestIdx2] = (uint16_t)bestDist;
                        log1[nlog] = (short)i1;
                        log2[nlog] = (short)bestIdx2;
                    }
                    nlog++;
                    if (lane < nCnt && (int)(nEnt & 0xffff) == bestIdx2) nVmd = bestDist;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        __syncthreads();
        qa = qb;
    }
    if (tid == 0) sh_nlog = nlog;
    __syncthreads();
    nlog = sh_nlog;
    // ---- replay the log in parallel: last claimant per i2, rotation histogram of every match
    const float factor = 1.0f / HISTO_LENGTH;
    for (int j = tid; j < nlog; j += INIT_NT) {
        atomicMax(&own[log2[j]], j);
        if (checkOri) {
            const int i1 = log1[j], i2 = log2[j];
            float rot = a1[i1] - a2[i2];
            if (rot < 0.0) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            binOf[i1] = (signed char)bin;
            atomicAdd(&hist[bin], 1);
        }
    }
    __syncthreads();
    int live = 0;
    for (int j = tid; j < nlog; j += INIT_NT) {
        const int i2 = log2[j];
        if (own[i2] == j) {
            m12[log1[j]] = (short)i2;
            live++;
        }
    }
    __syncthreads();
    if (checkOri) {
        const int3 im = og_three_maxima(hist);
        for (int i = tid; i < n1; i += INIT_NT) {
            const int bin = binOf[i];
            if (bin >= 0 && bin != im.x && bin != im.y && bin != im.z && m12[i] >= 0) {
                m12[i] = -1;
                live--;
            }
        }
    }
    live = og_wave_sum(live);
    if (lane == 0) wsum[wv] = live;
    __syncthreads();
    int* M = matches12 + (long long)b * match_stride;
    float* PV = prev_xy + (long long)b * prev_stride;
    for (int i = tid; i < n1; i += INIT_NT) {
        const int j = m12[i];
        M[i] = j;
        if (j >= 0) {  // update vbPrevMatched (src/ORBmatcher.cc:515-517)
            PV[2 * i] = K2[j].x;
            PV[2 * i + 1] = K2[j].y;
        }
    }
    if (tid == 0) nmatches[b] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

size_t og_init_resolve_lds(int cap1, int cap2, int ecap)
{
    // a1, a2, offs, own, E, vMD, m12, log1, log2, act, binOf (see og_init_resolve_kernel), 16-B aligned
    const size_t b = 4 * (size_t)cap1 + 4 * (size_t)cap2 + 4 * ((size_t)cap1 + 1) + 4 * (size_t)cap2 +
                     4 * (size_t)ecap + 2 * (size_t)cap2 + 4 * 2 * (size_t)cap1 + (size_t)cap1;
    return (b + 15) & ~(size_t)15;
}

// Largest candidate distance that can still change SearchForInitialization's outcome.  A candidate at d > TH_LOW
// is never the accepted best, and if TH_LOW < (float)d * nnratio then every acceptable best b <= TH_LOW passes
// the ratio test against it (b < (float)d * nnratio), so as a second-best it never causes a rejection; the
// same holds for every larger d (the float product is monotonic).  Dropping such candidates therefore leaves
// the best candidate, the accept/reject decision and every vMatchedDistance update of the reference loop
// (src/ORBmatcher.cc:430-462) unchanged, while the lists shrink to the near matches.
int og_init_keep_bound(float nnratio)
{
    if (!(nnratio > 0.0f)) return 255;
    for (int d = TH_LOW + 1; d <= 256; d++)
        if ((float)TH_LOW < (float)d * nnratio) return d - 1;
    return 256;
}

void og_launch_search_init(hipStream_t s, OgFrameDev F1, int ref, OgFrameDev F2, OgGridGeom G, float nnratio,
                           int checkOri, int windowSize, float* prev_xy, int prev_stride, int* matches12,
                           int match_stride, int* nmatches, uint32_t* lists, int list_cap, int* list_n, int* status,
                           int B, const int* ref_status, int qcap)
{
    // queries: F1 keypoints [0, qcap) (only octave-0 keypoints have candidates, :419-421; a frame extracted here
    // lists its levels in order, so its octave-0 keypoints are the first <= kcap_0)
    qcap = qcap > 0 ? std::min(qcap, F1.frame_cap) : F1.frame_cap;
    hipLaunchKernelGGL(og_init_cand_kernel, dim3((qcap + 3) / 4, B), dim3(256), 0, s, F1, ref, F2, G,
                       windowSize, og_init_keep_bound(nnratio), prev_xy, prev_stride, lists, list_cap, list_n);
    const size_t fixed = og_init_resolve_lds(F1.frame_cap, F2.frame_cap, 0);
    // staging for the (pruned, short) lists: a few KB keep several workgroups per CU; one list (<= list_cap)
    // must always fit, longer query ranges are staged in chunks
    const int ecap = (int)std::min<size_t>(std::max(list_cap, 2048), (OG_INIT_LDS_MAX - fixed) / 4);
    const size_t shm = og_init_resolve_lds(F1.frame_cap, F2.frame_cap, ecap);
    hipLaunchKernelGGL(og_init_resolve_kernel, dim3(B), dim3(INIT_NT), shm, s, F1, ref, F2, nnratio, checkOri,
                       prev_xy, prev_stride, lists, list_cap, list_n, matches12, match_stride, nmatches, status,
                       ecap, ref_status, qcap);
}

// Tracking::MonocularInitialization (src/Tracking.cc:573-575): vbPrevMatched[i] = F1.mvKeysUn[i].pt,
// replicated for every frame of a batch.
__global__ __launch_bounds__(256) void og_prev_from_frame_kernel(OgFrameDev F1, int ref, float* prev_xy,
                                                                 int prev_stride)
{
    const int b = blockIdx.y;
    const int n1 = F1.counts[ref];
    const orbgpu_kp_dev* K1 = F1.kps + (long long)ref * F1.frame_cap;
    float* PV = prev_xy + (long long)b * prev_stride;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n1; i += gridDim.x * blockDim.x) {
        PV[2 * i] = K1[i].x;
        PV[2 * i + 1] = K1[i].y;
    }
}

void og_launch_prev_from_frame(hipStream_t s, OgFrameDev F1, int ref, float* prev_xy, int prev_stride, int B)
{
    hipLaunchKernelGGL(og_prev_from_frame_kernel, dim3(4, B), dim3(256), 0, s, F1, ref, prev_xy, prev_stride);
}

// ------------------------------------------------------------------------------------------------
// SearchByProjection(Frame&, const vector<MapPoint*>&, th)
// ------------------------------------------------------------------------------------------------
// Candidates of map point m in GetFeaturesInArea order (src/Frame.cc:327-380: cells ix-major, then iy, then cell
// order) after the static filters of SearchByProjection (levels, window, stereo check, src/ORBmatcher.cc:53-104),
// with their Hamming distances; the dynamic filter (claims, :87-89) is applied by the caller.  visit(idx, dist,
// octave) is called in order for every candidate with dist <= dkeep (og_proj_keep_bound).
// Keypoint geometry as the enumeration reads it: straight from the frame's arrays in HBM ...
struct OgGeomGlobal {
    const OgFrameDev& F;
    __device__ int cs(int c) const { return F.cell_start[c]; }
    __device__ int item(int j) const { return F.cell_items[j]; }
    __device__ float x(int i) const { return F.kps[i].x; }
    __device__ float y(int i) const { return F.kps[i].y; }
    __device__ int oct(int i) const { return F.kps[i].octave; }
    __device__ bool has_ur() const { return F.uright != nullptr; }
    __device__ float ur(int i) const { return F.uright[i]; }
};
// ... or from the frame's copy in LDS (og_projb_fill_kernel)
struct OgGeomLds {
    const int* CS;
    const uint16_t* CI;
    const float2* XY;
    const uint8_t* OC;
    const float* UR;  // nullptr without mvuRight
    __device__ int cs(int c) const { return CS[c]; }
    __device__ int item(int j) const { return CI[j]; }
    __device__ float x(int i) const { return XY[i].x; }
    __device__ float y(int i) const { return XY[i].y; }
    __device__ int oct(int i) const { return OC[i]; }
    __device__ bool has_ur() const { return UR != nullptr; }
    __device__ float ur(int i) const { return UR[i]; }
};

// Candidates of map point m in GetFeaturesInArea order (src/Frame.cc:327-380: cells ix-major, then iy, then cell
// order) after the static filters of SearchByProjection (levels, window, stereo check, src/ORBmatcher.cc:53-104),
// with their Hamming distances (descriptors from HBM); the dynamic filter (claims, :87-89) is applied by the caller.
// visit(idx, dist, octave) is called in order for every candidate with dist <= dkeep (og_proj_keep_bound).
template <class Geom, class Visit>
__device__ __forceinline__ void og_proj_visit(const Geom& K, const uint8_t* fdesc, const OgGridGeom& G, const float* sf,
                                              const OgMapPointsDev& mp, int m, float th, int dkeep, Visit visit)
{
    if (!mp.track_in_view[m] || mp.is_bad[m]) return;
    const int lvl = mp.level[m];
    float r = mp.view_cos[m] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos, :131-137
    if (th != 1.0) r *= th;
    const float R = r * sf[lvl];
    const float x = mp.proj_x[m], y = mp.proj_y[m];
    const OgCellRange cr = og_cell_range(G, x, y, R);
    if (cr.x0 > cr.x1) return;
    const int minLevel = lvl - 1, maxLevel = lvl;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    uint4 da, db;
    og_load_desc(mp.desc + (long long)m * 32, da, db);
    for (int ix = cr.x0; ix <= cr.x1; ix++)
        for (int iy = cr.y0; iy <= cr.y1; iy++) {
            const int cell = ix * OG_GRID_ROWS + iy;
            const int je = K.cs(cell + 1);
            for (int j = K.cs(cell); j < je; j++) {
                const int idx = K.item(j);
                const int oct = K.oct(idx);
                if (bCheckLevels) {
                    if (oct < minLevel) continue;
                    if (maxLevel >= 0 && oct > maxLevel) continue;
                }
                const float distx = K.x(idx) - x, disty = K.y(idx) - y;
                if (!(fabsf(distx) < R && fabsf(disty) < R)) continue;
                if (K.has_ur() && K.ur(idx) > 0) {
                    const float er = fabsf(mp.proj_xr[m] - K.ur(idx));
                    if (er > r * sf[lvl]) continue;
                }
                uint4 ea, eb;
                og_load_desc(fdesc + (long long)idx * 32, ea, eb);
                const int dist = og_hamming(da, db, ea, eb);
                if (dist > dkeep) continue;  // og_proj_keep_bound
                visit(idx, dist, oct);
            }
        }
}

// og_proj_visit with the candidates' descriptor loads batched: up to 4 candidates that pass the geometric filters are
// queued (in order) and their descriptors loaded together, so a point's window costs one memory round trip per 4
// candidates instead of one per candidate.  Same candidates, same order, same visits.
template <class Geom, class Visit>
__device__ __forceinline__ void og_proj_visit_b(const Geom& K, const uint8_t* fdesc, const OgGridGeom& G, const float* sf,
                                                const OgMapPointsDev& mp, int m, float th, int dkeep, Visit visit)
{
    if (!mp.track_in_view[m] || mp.is_bad[m]) return;
    const int lvl = mp.level[m];
    float r = mp.view_cos[m] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos, :131-137
    if (th != 1.0) r *= th;
    const float R = r * sf[lvl];
    const float x = mp.proj_x[m], y = mp.proj_y[m];
    const OgCellRange cr = og_cell_range(G, x, y, R);
    if (cr.x0 > cr.x1) return;
    const int minLevel = lvl - 1, maxLevel = lvl;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    uint4 da, db;
    og_load_desc(mp.desc + (long long)m * 32, da, db);
    int q0 = 0, q1 = 0, q2 = 0, q3 = 0, o0 = 0, o1 = 0, o2 = 0, o3 = 0, nq = 0;
    auto flush = [&]() {
        uint4 a0 = {}, b0 = {}, a1 = {}, b1 = {}, a2 = {}, b2 = {}, a3 = {}, b3 = {};
        if (nq > 0) og_load_desc(fdesc + (long long)q0 * 32, a0, b0);
        if (nq > 1) og_load_desc(fdesc + (long long)q1 * 32, a1, b1);
        if (nq > 2) og_load_desc(fdesc + (long long)q2 * 32, a2, b2);
        if (nq > 3) og_load_desc(fdesc + (long long)q3 * 32, a3, b3);
        if (nq > 0) {
            const int d = og_hamming(da, db, a0, b0);
            if (d <= dkeep) visit(q0, d, o0);  // og_proj_keep_bound
        }
        if (nq > 1) {
            const int d = og_hamming(da, db, a1, b1);
            if (d <= dkeep) visit(q1, d, o1);
        }
        if (nq > 2) {
            const int d = og_hamming(da, db, a2, b2);
            if (d <= dkeep) visit(q2, d, o2);
        }
        if (nq > 3) {
            const int d = og_hamming(da, db, a3, b3);
            if (d <= dkeep) visit(q3, d, o3);
        }
        nq = 0;
    };
    for (int ix = cr.x0; ix <= cr.x1; ix++)
        for (int iy = cr.y0; iy <= cr.y1; iy++) {
            const int cell = ix * OG_GRID_ROWS + iy;
            const int je = K.cs(cell + 1);
            for (int j = K.cs(cell); j < je; j++) {
                const int idx = K.item(j);
                const int oct = K.oct(idx);
                if (bCheckLevels) {
                    if (oct < minLevel) continue;
                    if (maxLevel >= 0 && oct > maxLevel) continue;
                }
                const float distx = K.x(idx) - x, disty = K.y(idx) - y;
                if (!(fabsf(distx) < R && fabsf(disty) < R)) continue;
                if (K.has_ur() && K.ur(idx) > 0) {
                    const float er = fabsf(mp.proj_xr[m] - K.ur(idx));
                    if (er > r * sf[lvl]) continue;
                }
                if (nq == 0) {
                    q0 = idx;
                    o0 = oct;
                } else if (nq == 1) {
                    q1 = idx;
                    o1 = oct;
                } else if (nq == 2) {
                    q2 = idx;
                    o2 = oct;
                } else {
                    q3 = idx;
                    o3 = oct;
                }
                if (++nq == 4) flush();
            }
        }
    flush();
}

// a kept candidate as one dword: keypoint index (15 bits: the claim table of a frame holds < 2^15 keypoints,
// orbgpu_search_by_projection checks it), distance (9 bits, <= 256), octave (8 bits)
__device__ __forceinline__ uint32_t og_pj_pack(int idx, int dist, int oct)
{
    return (uint32_t)idx | ((uint32_t)dist << 15) | ((uint32_t)oct << 24);
}

__global__ __launch_bounds__(1024) void og_scan_kernel(const int* cnt, int n, int* off)
{
    // single-workgroup exclusive scan (n is the map-point count, a few thousand)
    __shared__ int wsum[16];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < n ? cnt[i] : 0;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            int s = 0;
            for (int q = 0; q < 16; q++) {
                const int t = wsum[q];
                wsum[q] = s;
                s += t;
            }
        }
        __syncthreads();
        if (i < n) off[i] = carry + wsum[w] + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += wsum[15] + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) off[n] = carry;
}

// Largest candidate distance that can change the outcome: a candidate at d > TH_HIGH is never the accepted
// best, and if TH_HIGH <= nnratio * (float)d then no acceptable best b <= TH_HIGH satisfies b > nnratio * d, so as
// a second-best it never triggers the ratio rejection (src/ORBmatcher.cc:115-121); the same holds for every
// larger d.  Dropping those candidates leaves every point's decision and bestIdx unchanged.
int og_proj_keep_bound(float nnratio)
{
    if (!(nnratio > 0.0f)) return 256;
    for (int d = TH_HIGH + 1; d <= 256; d++)
        if ((float)TH_HIGH <= nnratio * (float)d) return d - 1;
    return 256;
}

__device__ __forceinline__ OgFrameDev og_frame_of(const OgFrameDev& F, int b)
{
    OgFrameDev f = F;
    f.kps += (long long)b * F.frame_cap;
    f.desc += (long long)b * F.frame_cap * 32;
    f.counts += b;
    f.cell_start += (long long)b * (OG_GRID_CELLS + 1);
    f.cell_items += (long long)b * F.frame_cap;
    if (F.uright) f.uright += (long long)b * F.frame_cap;
    return f;
}

__device__ __forceinline__ OgMapPointsDev og_mp_of(const OgMapPointsDev& mp, int b, int stride)
{
    const long long o = (long long)b * stride;
    const long long om = mp.shared_map ? 0 : o;  // the map's own fields: per frame, or one map for all frames
    OgMapPointsDev q = mp;
    q.track_in_view += o;
    q.is_bad += om;
    q.level += o;
    q.view_cos += o;
    q.proj_x += o;
    q.proj_y += o;
    q.proj_xr += o;
    q.n_obs += om;
    q.desc += om * 32;
    return q;
}

// ---- one enumeration pass.  A workgroup of PF_NT threads takes every PF_WG-th block of PF_NT map points of one
// frame; it first copies the frame's keypoint geometry (x, y, octave, mvuRight) and grid into LDS with coalesced
// loads, so the window enumeration reads LDS and only the candidates' descriptors come from HBM.  The first OG_PJ_K
// kept candidates of a point go to its slots, stored k-major (slot k of points m, m + 1, ... adjacent); kept[] = the
// point's full kept count (> OG_PJ_K: the resolve re-enumerates that point itself).  Frames whose geometry does not
// fit the LDS take the same enumeration from HBM.
#define PF_NT 512
#define PF_WG 4  // workgroups per frame
// the cell starts (OG_GRID_CELLS + 1 ints) padded to a 16-byte multiple, so the float2 XY array after them is
// 8-byte aligned (ds_read_b64, no split accesses)
#define PF_CS_INTS (((OG_GRID_CELLS + 1) + 3) & ~3)
__host__ __device__ inline size_t og_projb_fill_lds(int frame_cap, bool ur)
{
    return (size_t)PF_CS_INTS * 4 + (size_t)frame_cap * (8 + 1 + 2 + (ur ? 4 : 0)) + 16;
}

__global__ __launch_bounds__(PF_NT) void og_projb_fill_kernel(OgFrameDev Fb, OgGridGeom G, const float* sf,
                                                              OgMapPointsDev mp, int stride, float th, int dkeep,
                                                              int use_lds, uint32_t* __restrict__ slots,
                                                              int* __restrict__ kept)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t pf_lds[];
    const int b = blockIdx.y, tid = threadIdx.x;
    const OgFrameDev F = og_frame_of(Fb, b);
    const OgMapPointsDev q = og_mp_of(mp, b, stride);
    uint32_t* S = slots + (long long)b * OG_PJ_K * stride;
    int* KEPT = kept + (long long)b * stride;
    auto run = [&](const auto& K) {
        for (int m = blockIdx.x * PF_NT + tid; m < q.m; m += PF_WG * PF_NT) {
            int n = 0;
            auto put = [&](int idx, int dist, int oct) {
                if (n < OG_PJ_K) S[(long long)n * stride + m] = og_pj_pack(idx, dist, oct);
                n++;
            };
            og_proj_visit_b(K, F.desc, G, sf, q, m, th, dkeep, put);
            KEPT[m] = n;
        }
    };
    if (!use_lds) {  // uniform (host decision from frame_cap)
        run(OgGeomGlobal{F});
        return;
    }
    const int n = min(F.counts[0], F.frame_cap);
    int* CS = (int*)pf_lds;
    float2* XY = (float2*)(CS + PF_CS_INTS);
    float* UR = (float*)(XY + F.frame_cap);
    uint16_t* CI = (uint16_t*)(UR + (F.uright ? F.frame_cap : 0));
    uint8_t* OC = (uint8_t*)(CI + F.frame_cap);
    for (int c = tid; c <= OG_GRID_CELLS; c += PF_NT) CS[c] = F.cell_start[c];
    for (int i = tid; i < n; i += PF_NT) {
        const orbgpu_kp_dev* kp = F.kps + i;
        XY[i] = make_float2(kp->x, kp->y);
        OC[i] = (uint8_t)kp->octave;
        CI[i] = (uint16_t)F.cell_items[i];
        if (F.uright) UR[i] = F.uright[i];
    }
    __syncthreads();
    run(OgGeomLds{CS, CI, XY, OC, F.uright ? UR : nullptr});
}

// The reference's ordered loop over map points (src/ORBmatcher.cc:53-129) couples points only through the
// claims: point m skips keypoint i while it is held by a map point with Observations() > 0 (:87-89).  In the
// sequential run such a holder is the FIRST accepted claimant with observations (later points cannot take the
// keypoint from it), so with  FO[i] = -1 for a keypoint held before the call by a point with observations, else
// the smallest accepted point with observations whose best is i  the decision of point m is a function of
// { i : FO[i] < m } alone.  That system is triangular (m depends on points < m only): iterating "decide every
// point from FO; rebuild FO from the decisions" (Jacobi) reaches its unique fixed point -- the sequential
// result -- after at most (longest dependency chain + 1) rounds, and a round that leaves FO unchanged is that
// fixed point.  One workgroup per frame; every point's decision within a round is independent.
// Final ownership: keypoint i belongs to the LAST accepted claimant (assignment order), else keeps its holder.
//
// The candidate lists are staged once into LDS (compacted by a block scan of the kept counts), so the rounds read
// no global memory; a frame whose lists exceed the LDS budget reads its slots instead, and a point with more than
// OG_PJ_K kept candidates re-enumerates them (og_proj_visit) in every round.
#define PJ_NT 1024
__device__ __forceinline__ int og_block_exclusive_scan(int v, int* wsum, int& total)
{
    // PJ_NT threads; wsum: PJ_NT / 64 + 1 ints of LDS
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int q = 0; q < PJ_NT / 64; q++) {
            const int t = wsum[q];
            wsum[q] = acc;
            acc += t;
        }
        wsum[PJ_NT / 64] = acc;
    }
    __syncthreads();
    total = wsum[PJ_NT / 64];
    const int r = wsum[w] + x - v;
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(PJ_NT) void og_projb_resolve_kernel(OgFrameDev Fb, OgGridGeom G, const float* sf,
                                                                 OgMapPointsDev mp, int stride, float th, int dkeep,
                                                                 const uint32_t* __restrict__ slots,
                                                                 const int* __restrict__ kept, float nnratio,
                                                                 int lds_bytes, int stage_ok, int* owner,
                                                                 int* owner_obs, int* nmatches, int* res, int* status)
{
    extern __shared__ int pj_lds[];
    const int frame_cap = Fb.frame_cap;
    int* FO = pj_lds;               // [frame_cap] current round
    int* NF = pj_lds + frame_cap;   // [frame_cap] next round / final owner
    int* PO = NF + frame_cap;       // [M + 1] list offsets (staged mode)
    __shared__ int sh_changed, sh_nm;
    __shared__ int wsum[PJ_NT / 64 + 1];
    const int b = blockIdx.x, tid = threadIdx.x;
    const OgFrameDev F = og_frame_of(Fb, b);
    const int n = F.counts[0];
    const OgMapPointsDev q = og_mp_of(mp, b, stride);
    const int M = q.m;
    const int* KEPT = kept + (long long)b * stride;
    const uint32_t* SL = slots + (long long)b * OG_PJ_K * stride;
    int* OWN = owner + (long long)b * frame_cap;
    int* OBS = owner_obs + (long long)b * frame_cap;
    int* RES = res + (long long)b * stride;
    // ---- stage the lists: per-point counts (0 for overflowed points: they re-enumerate), block scan, copy
    const int ppt = (M + PJ_NT - 1) / PJ_NT;  // points per thread, contiguous: m in [tid * ppt, tid * ppt + ppt)
    int my = 0;
    for (int k = 0; k < ppt; k++) {
        const int m = tid * ppt + k;
        if (m < M) {
            const int c = KEPT[m];
            my += c <= OG_PJ_K ? c : 0;
        }
    }
    int T = 0;
    const int base = og_block_exclusive_scan(my, wsum, T);
    uint32_t* LST = (uint32_t*)(PO + M + 1);
    const int cap_entries = (lds_bytes - (int)sizeof(int) * (2 * frame_cap + M + 1)) / 4;
    const bool staged = stage_ok && M > 0 && T <= cap_entries &&
                        (2 * frame_cap + M + 1) * (int)sizeof(int) <= lds_bytes;  // uniform
    if (staged) {
        int o = base;
        for (int k = 0; k < ppt; k++) {
            const int m = tid * ppt + k;
            if (m < M) {
                PO[m] = o;
                const int c = KEPT[m];
                o += c <= OG_PJ_K ? c : 0;
            }
        }
        if (tid == 0) PO[M] = T;
    }
    for (int i = tid; i < n; i += PJ_NT) {
        FO[i] = (OWN[i] >= 0 && OBS[i]) ? -1 : INT_MAX;  // round 0 starts from the pre-call claims only
        NF[i] = FO[i];
    }
    if (tid == 0) sh_changed = 1;
    __syncthreads();
    if (staged) {  // copy slot k of every point with more than k staged entries (k-major: coalesced reads)
        for (int k = 0; k < OG_PJ_K; k++) {
            for (int m = tid; m < M; m += PJ_NT) {
                const int c = KEPT[m];
                if (c <= OG_PJ_K && k < c) LST[PO[m] + k] = SL[(long long)k * stride + m];
            }
        }
    }
    __syncthreads();
    int rounds = 0;
    for (;;) {
        for (int m = tid; m < M; m += PJ_NT) {
            int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
            auto take = [&](int idx, int dist, int oct) {
                if (FO[idx] < m) return;  // :87-89
                if (dist < bestDist) {
                    bestDist2 = bestDist;
                    bestDist = dist;
                    bestLevel2 = bestLevel;
                    bestLevel = oct;
                    bestIdx = idx;
                } else if (dist < bestDist2) {
                    bestLevel2 = oct;
                    bestDist2 = dist;
                }
            };
            const int nc = KEPT[m];
            if (nc > OG_PJ_K) {
                og_proj_visit(OgGeomGlobal{F}, F.desc, G, sf, q, m, th, dkeep, take);
            } else if (staged) {
                const uint32_t* L = LST + PO[m];
                for (int c = 0; c < nc; c++) {
                    const uint32_t e = L[c];
                    take((int)(e & 0x7fff), (int)((e >> 15) & 0x1ff), (int)(e >> 24));
                }
            } else {
                for (int c = 0; c < nc; c++) {
                    const uint32_t e = SL[(long long)c * stride + m];
                    take((int)(e & 0x7fff), (int)((e >> 15) & 0x1ff), (int)(e >> 24));
                }
            }
            int r = -1;
            if (bestDist <= TH_HIGH && !(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2)) r = bestIdx;
            RES[m] = r;
            if (r >= 0 && q.n_obs[m] > 0) atomicMin(&NF[r], m);
        }
        __syncthreads();
        int ch = 0;
        for (int i = tid; i < n; i += PJ_NT) {
            const int v = NF[i];
            ch |= v != FO[i];
            FO[i] = v;
            NF[i] = (OWN[i] >= 0 && OBS[i]) ? -1 : INT_MAX;
        }
        if (tid == 0) sh_changed = 0;
        __syncthreads();
        if (ch) sh_changed = 1;
        __syncthreads();
        const bool again = sh_changed != 0;
        __syncthreads();
        if (!again) break;
        if (++rounds > M + 1) {  // cannot happen (triangular system); reported, never silent
            if (tid == 0) atomicOr(status, 32);
            break;
        }
    }
    // final ownership and the count of assignments
    for (int i = tid; i < n; i += PJ_NT) NF[i] = -1;
    if (tid == 0) sh_nm = 0;
    __syncthreads();
    int cnt = 0;
    for (int m = tid; m < M; m += PJ_NT) {
        const int r = RES[m];
        if (r >= 0) {
            atomicMax(&NF[r], m);
            cnt++;
        }
    }
    cnt = og_wave_sum(cnt);
    if ((tid & 63) == 0) atomicAdd(&sh_nm, cnt);
    __syncthreads();
    for (int i = tid; i < n; i += PJ_NT) {
        const int o = NF[i];
        if (o >= 0) {
            OWN[i] = o;
            OBS[i] = q.n_obs[o] > 0;
        }
    }
    if (tid == 0) nmatches[b] = sh_nm;
}

void og_launch_projb(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgMapPointsDev mp, int stride,
                     float nnratio, float th, int B, uint32_t* slots, int* kept, int* res, int* owner, int* owner_obs,
                     int* nmatches, int* status, int dbg)
{
    // dbg (orbgpu_debug_set_projection_paths, tests only): 1 = enumerate from HBM geometry, 2 = resolve from the
    // slots in HBM (no LDS-staged lists); both are the paths of frames too large for the LDS
    if (B <= 0) return;
    const int dkeep = og_proj_keep_bound(nnratio);
    if (mp.m > 0) {
        // cell items are u16 in LDS: frames of at most 65535 keypoints (the host form checks far less)
        const size_t lds = og_projb_fill_lds(F.frame_cap, F.uright != nullptr);
        const int use_lds = !(dbg & 1) && lds <= OG_PJ_LDS && F.frame_cap <= 65535;
        hipLaunchKernelGGL(og_projb_fill_kernel, dim3(PF_WG, B), dim3(PF_NT), use_lds ? lds : 0, s, F, G, sf, mp, stride,
                           th, dkeep, use_lds, slots, kept);
    }
    hipLaunchKernelGGL(og_projb_resolve_kernel, dim3(B), dim3(PJ_NT), OG_PJ_LDS, s, F, G, sf, mp, stride, th, dkeep,
                       slots, kept, nnratio, (int)OG_PJ_LDS, (dbg & 2) ? 0 : 1, owner, owner_obs, nmatches, res, status);
}

// ------------------------------------------------------------------------------------------------
// Frame::isInFrustum + MapPoint::PredictScale (src/Frame.cc:269-325, src/MapPoint.cc:402-417), one thread
// per map point.  cv::Mat algebra as pinned in DESIGN.md §3 (R*x + t left to right in float; norm
// and dot accumulate in double); the reference's own u/v/ur expressions are GCC-contracted FMAs.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void og_rx_t(const float* R, const float* x, const float* t, float* o)
{
#pragma unroll
    for (int r = 0; r < 3; r++) {
        float s = __fmul_rn(R[3 * r], x[0]);
        s = __fadd_rn(s, __fmul_rn(R[3 * r + 1], x[1]));
        s = __fadd_rn(s, __fmul_rn(R[3 * r + 2], x[2]));
        o[r] = __fadd_rn(s, t[r]);
    }
}

__device__ __forceinline__ void og_frustum_point(const OgCameraDev& cam, const OgMapGeomDev& mp, int m, float limit,
                                                OgFrustumOut out);

__global__ __launch_bounds__(256) void og_frustum_kernel(OgCameraDev cam, OgMapGeomDev mp, float limit,
                                                         OgFrustumOut out)
{
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= mp.m) return;
    og_frustum_point(cam, mp, m, limit, out);
}

// one camera per blockIdx.y (the pose / intrinsics of orbgpu_camera, read from device memory), one shared map
__global__ __launch_bounds__(256) void og_frustum_batch_kernel(const float* __restrict__ cams, float minX, float maxX,
                                                               float minY, float maxY, OgMapGeomDev mp, float limit,
                                                               OgFrustumOut out, int stride)
{
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= mp.m) return;
    const int b = blockIdx.y;
    const float* c = cams + 23 * (long long)b;  // orbgpu_camera: 22 floats + int nlevels
    OgCameraDev cam;
#pragma unroll
    for (int k = 0; k < 9; k++) cam.R[k] = c[k];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        cam.t[k] = c[9 + k];
        cam.Ow[k] = c[12 + k];
    }
    cam.fx = c[15];
    cam.fy = c[16];
    cam.cx = c[17];
    cam.cy = c[18];
    cam.mbf = c[19];
    cam.mb = c[20];
    cam.scale_factor = c[21];
    cam.nlevels = __float_as_int(c[22]);
    cam.minX = minX;
    cam.maxX = maxX;
    cam.minY = minY;
    cam.maxY = maxY;
    const long long o = (long long)b * stride;
    OgFrustumOut ob{out.in_view + o, out.proj_x + o, out.proj_y + o, out.proj_xr + o, out.level + o,
                    out.view_cos + o, nullptr};
    og_frustum_point(cam, mp, m, limit, ob);
}

void og_launch_frustum_batch(hipStream_t s, const void* d_cams, int B, float minX, float maxX, float minY, float maxY,
                             OgMapGeomDev mp, float viewingCosLimit, OgFrustumOut out, int stride)
{
    if (mp.m > 0 && B > 0)
        hipLaunchKernelGGL(og_frustum_batch_kernel, dim3((mp.m + 255) / 256, B), dim3(256), 0, s,
                           (const float*)d_cams, minX, maxX, minY, maxY, mp, viewingCosLimit, out, stride);
}

// Frame::isInFrustum + MapPoint::PredictScale of map point m for one camera (src/Frame.cc:269-325,
// src/MapPoint.cc:402-417)
__device__ __forceinline__ void og_frustum_point(const OgCameraDev& cam, const OgMapGeomDev& mp, int m, float limit,
                                                OgFrustumOut out)
{
    bool in = false;
    float u = 0, v = 0, ur = 0, vc = 0;
    int lvl = 0;
    do {
        const float P[3] = {mp.pos[3 * m], mp.pos[3 * m + 1], mp.pos[3 * m + 2]};
        float Pc[3];
        og_rx_t(cam.R, P, cam.t, Pc);
        if (Pc[2] < 0.0f) break;
        const float invz = __fdiv_rn(1.0f, Pc[2]);
        u = __fmaf_rn(__fmul_rn(cam.fx, Pc[0]), invz, cam.cx);
        v = __fmaf_rn(__fmul_rn(cam.fy, Pc[1]), invz, cam.cy);
        if (u < cam.minX || u > cam.maxX) break;
        if (v < cam.minY || v > cam.maxY) break;
        const float maxD = __fmul_rn(1.2f, mp.max_dist[m]);
        const float minD = __fmul_rn(0.8f, mp.min_dist[m]);
        const float PO[3] = {__fsub_rn(P[0], cam.Ow[0]), __fsub_rn(P[1], cam.Ow[1]), __fsub_rn(P[2], cam.Ow[2])};
        double ss = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) ss = __dadd_rn(ss, __dmul_rn((double)PO[k], (double)PO[k]));
        const float dist = (float)__dsqrt_rn(ss);
        if (dist < minD || dist > maxD) break;
        double dot = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) dot = __dadd_rn(dot, __dmul_rn((double)PO[k], (double)mp.normal[3 * m + k]));
        vc = (float)__ddiv_rn(dot, (double)dist);
        if (vc < limit) break;
        const float ratio = __fdiv_rn(mp.max_dist[m], dist);
        int ns = (int)ceilf(__fdiv_rn(og_logf(ratio), og_logf(cam.scale_factor)));
        ns = ns < 0 ? 0 : (ns >= cam.nlevels ? cam.nlevels - 1 : ns);
        lvl = ns;
        ur = __fmaf_rn(-cam.mbf, invz, u);
        in = true;
    } while (0);
    out.in_view[m] = in ? 1 : 0;
    if (in) {
        out.proj_x[m] = u;
        out.proj_y[m] = v;
        out.proj_xr[m] = ur;
        out.level[m] = lvl;
        out.view_cos[m] = vc;
    }
    if (out.n_in_view) {
        const u64 b = __ballot(in);
        if ((threadIdx.x & 63) == 0 && b) atomicAdd(out.n_in_view, __popcll(b));
    }
}

void og_launch_frustum(hipStream_t s, OgCameraDev cam, OgMapGeomDev mp, float viewingCosLimit, OgFrustumOut out)
{
    if (mp.m > 0)
        hipLaunchKernelGGL(og_frustum_kernel, dim3((mp.m + 255) / 256), dim3(256), 0, s, cam, mp, viewingCosLimit,
                           out);
}

// ------------------------------------------------------------------------------------------------
// ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
// (src/ORBmatcher.cc:1328-1470).  Projection + GetFeaturesInArea + static filters (stereo check) +
// distances in parallel per last-frame point; the claim order (:1384-1386, :1411) and the rotation
// histogram (:1414-1443) replay in one ordered pass.
// ------------------------------------------------------------------------------------------------
template <bool FILL>
__device__ int og_last_enum(const OgFrameDev& F, const OgGridGeom& G, const float* sf, const OgCameraDev& cam,
                            const OgLastFrameDev& LF, int i, float th, int mode, OgLastCand* out)
{
    if (!LF.has_mp[i] || LF.outlier[i]) return 0;
    const float P[3] = {LF.pos[3 * i], LF.pos[3 * i + 1], LF.pos[3 * i + 2]};
    float x3[3];
    og_rx_t(cam.R, P, cam.t, x3);
    const float invzc = (float)__ddiv_rn(1.0, (double)x3[2]);
    if (invzc < 0) return 0;
    const float u = __fmaf_rn(__fmul_rn(cam.fx, x3[0]), invzc, cam.cx);
    const float v = __fmaf_rn(__fmul_rn(cam.fy, x3[1]), invzc, cam.cy);
    if (u < G.minX || u > G.maxX) return 0;
    if (v < G.minY || v > G.maxY) return 0;
    if (u != u || v != v) return 0;
    const int o = LF.kps[i].octave;
    const float radius = __fmul_rn(th, sf[o]);
    int minLevel, maxLevel;
    if (mode == 1) minLevel = o, maxLevel = -1;
    else if (mode == 2) minLevel = 0, maxLevel = o;
    else minLevel = o - 1, maxLevel = o + 1;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const OgCellRange cr = og_cell_range(G, u, v, radius);
    if (cr.x0 > cr.x1) return 0;
    const float ur = __fmaf_rn(-cam.mbf, invzc, u);
    uint4 da, db;
    if (FILL) og_load_desc(LF.desc + (long long)i * 32, da, db);
    int n = 0;
    for (int ix = cr.x0; ix <= cr.x1; ix++)
        for (int iy = cr.y0; iy <= cr.y1; iy++) {
            const int cell = ix * OG_GRID_ROWS + iy;
            for (int j = F.cell_start[cell]; j < F.cell_start[cell + 1]; j++) {
                const int idx = F.cell_items[j];
                const orbgpu_kp_dev kp = F.kps[idx];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = __fsub_rn(kp.x, u), disty = __fsub_rn(kp.y, v);
                if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
                if (F.uright && F.uright[idx] > 0) {
                    if (fabsf(__fsub_rn(ur, F.uright[idx])) > radius) continue;
                }
                if (FILL) {
                    uint4 ea, eb;
                    og_load_desc(F.desc + (long long)idx * 32, ea, eb);
                    out[n] = OgLastCand{idx, og_hamming(da, db, ea, eb)};
                }
                n++;
            }
        }
    return n;
}

__global__ __launch_bounds__(256) void og_last_count_kernel(OgFrameDev F, OgGridGeom G, const float* sf,
                                                            OgCameraDev cam, OgLastFrameDev LF, float th, int mode,
                                                            int* cnt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LF.n) return;
    cnt[i] = og_last_enum<false>(F, G, sf, cam, LF, i, th, mode, nullptr);
}

__global__ __launch_bounds__(256) void og_last_fill_kernel(OgFrameDev F, OgGridGeom G, const float* sf,
                                                           OgCameraDev cam, OgLastFrameDev LF, float th, int mode,
                                                           const int* off, OgLastCand* cands)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= LF.n) return;
    og_last_enum<true>(F, G, sf, cam, LF, i, th, mode, cands + off[i]);
}

// ent: LF.n ints -- the rotation-histogram pushes in order, packed (bin << 24) | keypoint index
// blockAny: any claim blocks a keypoint (relocalisation, :1543-1544) instead of claims by map points with
// observations (:1384-1386); thAccept: TH_HIGH or the caller's ORBdist; owner_obs may be nullptr.
__global__ __launch_bounds__(64) void og_last_resolve_kernel(OgFrameDev F, OgLastFrameDev LF, int checkOri,
                                                             int blockAny, int thAccept, const int* off,
                                                             const OgLastCand* cands, int* ent, int* owner,
                                                             int* owner_obs, int* nmatches)
{
    __shared__ int hist[HISTO_LENGTH];
    __shared__ int sh[4];
    const int lane = threadIdx.x;
    if (lane < HISTO_LENGTH) hist[lane] = 0;
    __syncthreads();
    if (lane == 0) {
        int nm = 0, ne = 0;
        const float factor = 1.0f / HISTO_LENGTH;
        for (int i = 0; i < LF.n; i++) {
            const int b = off[i], e = off[i + 1];
            if (b == e) continue;
            int bestDist = 256, bestIdx2 = -1;
            for (int c = b; c < e; c++) {
                const OgLastCand cc = cands[c];
                if (owner[cc.idx] >= 0 && (blockAny || owner_obs[cc.idx])) continue;
                if (cc.dist < bestDist) {
                    bestDist = cc.dist;
                    bestIdx2 = cc.idx;
                }
            }
            if (bestDist <= thAccept) {
                owner[bestIdx2] = i;
                if (owner_obs) owner_obs[bestIdx2] = LF.n_obs ? LF.n_obs[i] > 0 : 1;
                nm++;
                if (checkOri) {
                    float rot = __fsub_rn(LF.kps[i].angle, F.kps[bestIdx2].angle);
                    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                    int bin = (int)roundf(__fmul_rn(rot, factor));
                    if (bin == HISTO_LENGTH) bin = 0;
                    hist[bin]++;
                    ent[ne++] = (bin << 24) | bestIdx2;
                }
            }
        }
        sh[0] = nm;
        sh[1] = ne;
        int i1 = -1, i2 = -1, i3 = -1;
        if (checkOri) {
            const int3 im = og_three_maxima(hist);
            i1 = im.x, i2 = im.y, i3 = im.z;
        }
        sh[2] = i1;
        sh[3] = (i2 & 0xffff) | (i3 << 16);
    }
    __syncthreads();
    int culled = 0;
    if (checkOri) {
        const int ne = sh[1], i1 = sh[2], i2 = (short)(sh[3] & 0xffff), i3 = sh[3] >> 16;
        for (int k = lane; k < ne; k += 64) {
            const int v = ent[k], bin = v >> 24, idx = v & 0xffffff;
            if (bin != i1 && bin != i2 && bin != i3) {
                owner[idx] = -1;  // all writes are NULL: order-free
                if (owner_obs) owner_obs[idx] = 0;
                culled++;
            }
        }
    }
    culled = og_wave_sum(culled);
    if (lane == 0) *nmatches = sh[0] - culled;
}

void og_launch_last_count(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                          OgLastFrameDev LF, float th, int mode, int* cnt, int* off)
{
    const int blocks = (LF.n + 255) / 256;
    if (blocks > 0)
        hipLaunchKernelGGL(og_last_count_kernel, dim3(blocks), dim3(256), 0, s, F, G, sf, cam, LF, th, mode, cnt);
    hipLaunchKernelGGL(og_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, LF.n, off);
}

void og_launch_last_resolve(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                            OgLastFrameDev LF, float th, int mode, int checkOri, const int* off, OgLastCand* cands,
                            int* ent, int* owner, int* owner_obs, int* nmatches)
{
    const int blocks = (LF.n + 255) / 256;
    if (blocks > 0)
        hipLaunchKernelGGL(og_last_fill_kernel, dim3(blocks), dim3(256), 0, s, F, G, sf, cam, LF, th, mode, off,
                           cands);
    hipLaunchKernelGGL(og_last_resolve_kernel, dim3(1), dim3(64), 0, s, F, LF, checkOri, 0, TH_HIGH, off, cands, ent,
                       owner, owner_obs, nmatches);
}

// ------------------------------------------------------------------------------------------------
// ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
// th, ORBdist) (src/ORBmatcher.cc:1472-1599): the keyframe's map points projected into the frame (no depth
// sign test), PredictScale on ||X - Ow|| picks the level window; any claim blocks; accept <= ORBdist.
// ------------------------------------------------------------------------------------------------
template <bool FILL>
__device__ int og_kf_enum(const OgFrameDev& F, const OgGridGeom& G, const float* sf, const OgCameraDev& cam,
                          const float* Ow, const OgLastFrameDev& KF, const float* max_dist, const float* min_dist,
                          const int* pred_level, int i, float th, OgLastCand* out)
{
    if (!KF.has_mp[i]) return 0;
    const float X[3] = {KF.pos[3 * i], KF.pos[3 * i + 1], KF.pos[3 * i + 2]};
    float x3[3];
    og_rx_t(cam.R, X, cam.t, x3);
    const float invzc = (float)__ddiv_rn(1.0, (double)x3[2]);
    const float u = __fmaf_rn(__fmul_rn(cam.fx, x3[0]), invzc, cam.cx);
    const float v = __fmaf_rn(__fmul_rn(cam.fy, x3[1]), invzc, cam.cy);
    if (u < G.minX || u > G.maxX) return 0;
    if (v < G.minY || v > G.maxY) return 0;
    if (u != u || v != v) return 0;
    int lvl;
    if (pred_level) {  // the caller's PredictScale (orbgpu_search_by_projection_keyframe_levels); -1: out of range
        lvl = pred_level[i];
        if (lvl < 0) return 0;
        lvl = lvl >= cam.nlevels ? cam.nlevels - 1 : lvl;
    } else {
        const float PO[3] = {__fsub_rn(X[0], Ow[0]), __fsub_rn(X[1], Ow[1]), __fsub_rn(X[2], Ow[2])};
        double ss = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) ss = __dadd_rn(ss, __dmul_rn((double)PO[k], (double)PO[k]));
        const float dist3D = (float)__dsqrt_rn(ss);
        const float maxD = __fmul_rn(1.2f, max_dist[i]), minD = __fmul_rn(0.8f, min_dist[i]);
        if (dist3D < minD || dist3D > maxD) return 0;
        lvl = (int)ceilf(__fdiv_rn(og_logf(__fdiv_rn(max_dist[i], dist3D)), og_logf(cam.scale_factor)));
        lvl = lvl < 0 ? 0 : (lvl >= cam.nlevels ? cam.nlevels - 1 : lvl);
    }
    const float radius = __fmul_rn(th, sf[lvl]);
    const int minLevel = lvl - 1, maxLevel = lvl + 1;
    const OgCellRange cr = og_cell_range(G, u, v, radius);
    if (cr.x0 > cr.x1) return 0;
    uint4 da, db;
    if (FILL) og_load_desc(KF.desc + (long long)i * 32, da, db);
    int n = 0;
    for (int ix = cr.x0; ix <= cr.x1; ix++)
        for (int iy = cr.y0; iy <= cr.y1; iy++) {
            const int cell = ix * OG_GRID_ROWS + iy;
            for (int j = F.cell_start[cell]; j < F.cell_start[cell + 1]; j++) {
                const int idx = F.cell_items[j];
                const orbgpu_kp_dev kp = F.kps[idx];
                if (kp.octave < minLevel || kp.octave > maxLevel) continue;  // bCheckLevels (maxLevel >= 0)
                const float distx = __fsub_rn(kp.x, u), disty = __fsub_rn(kp.y, v);
                if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
                if (FILL) {
                    uint4 ea, eb;
                    og_load_desc(F.desc + (long long)idx * 32, ea, eb);
                    out[n] = OgLastCand{idx, og_hamming(da, db, ea, eb)};
                }
                n++;
            }
        }
    return n;
}

__global__ __launch_bounds__(256) void og_kf_count_kernel(OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                                                          OgLastFrameDev KF, const float* max_dist,
                                                          const float* min_dist, const int* pred_level, float th,
                                                          int* cnt)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= KF.n) return;
    cnt[i] = og_kf_enum<false>(F, G, sf, cam, cam.Ow, KF, max_dist, min_dist, pred_level, i, th, nullptr);
}

__global__ __launch_bounds__(256) void og_kf_fill_kernel(OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                                                         OgLastFrameDev KF, const float* max_dist,
                                                         const float* min_dist, const int* pred_level, float th,
                                                         const int* off, OgLastCand* cands)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= KF.n) return;
    og_kf_enum<true>(F, G, sf, cam, cam.Ow, KF, max_dist, min_dist, pred_level, i, th, cands + off[i]);
}

void og_launch_kf_count(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                        OgLastFrameDev KF, const float* max_dist, const float* min_dist, const int* pred_level,
                        float th, int* cnt, int* off)
{
    const int blocks = (KF.n + 255) / 256;
    if (blocks > 0)
        hipLaunchKernelGGL(og_kf_count_kernel, dim3(blocks), dim3(256), 0, s, F, G, sf, cam, KF, max_dist, min_dist,
                           pred_level, th, cnt);
    hipLaunchKernelGGL(og_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, KF.n, off);
}

void og_launch_kf_resolve(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                          OgLastFrameDev KF, const float* max_dist, const float* min_dist, const int* pred_level,
                          float th, int ORBdist, int checkOri, const int* off, OgLastCand* cands, int* ent, int* owner,
                          int* nmatches)
{
    const int blocks = (KF.n + 255) / 256;
    if (blocks > 0)
        hipLaunchKernelGGL(og_kf_fill_kernel, dim3(blocks), dim3(256), 0, s, F, G, sf, cam, KF, max_dist, min_dist,
                           pred_level, th, off, cands);
    hipLaunchKernelGGL(og_last_resolve_kernel, dim3(1), dim3(64), 0, s, F, KF, checkOri, 1, ORBdist, off, cands, ent,
                       owner, (int*)nullptr, nmatches);
}

// dynamic-LDS attributes (more than the default per workgroup): per device, set from og_prepare_device
hipError_t og_prepare_device_match()
{
    hipError_t e = hipFuncSetAttribute((const void*)og_init_resolve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       OG_INIT_LDS_MAX);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)og_projb_resolve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, OG_PJ_LDS);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute((const void*)og_projb_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, OG_PJ_LDS);
}
