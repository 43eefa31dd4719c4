// orb_bow.hip -- gfx950 kernels of Frame::ComputeBoW (src/Frame.cc:395-402) =
// ORBVocabulary::transform(descriptors, mBowVec, mFeatVec, 4), DBoW2 TemplatedVocabulary<FORB>
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1256, BowVector.cpp:34-84, FeatureVector.cpp:31-45).
//
//   og_bow_descend_kernel : one wave per descriptor; at every level the node's children (k <= 20 in
//                           DBoW2 files) are scored by the 64 lanes (FORB Hamming distance), the strict-<
//                           first minimum is a DPP min over (distance, child position); the node at level
//                           L - levelsup is kept for the FeatureVector.
//   og_bow_reduce_kernel  : one workgroup per frame; bitonic sorts of (word, feature) and (node, feature) in
//                           LDS give the BowVector map (per-word weights summed in feature order, like
//                           std::map::operator+= in feature order) and the FeatureVector lists; the norm is
//                           accumulated in ascending word order as BowVector::normalize does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_math_dev.h"
#include "orbgpu_internal.h"
#include "orbgpu_launch.h"

typedef unsigned long long u64;

__device__ __forceinline__ uint32_t og_bow_wave_min(uint32_t v)
{
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false));
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return min(min(a, b), min(c, d));
}

__global__ __launch_bounds__(256) void og_bow_descend_kernel(OgVocDev V, const uint8_t* __restrict__ desc,
                                                            const int* counts, int n_fixed, int frame_cap,
                                                            int levelsup, int* __restrict__ word, double* __restrict__ wt,
                                                            int* __restrict__ nidOut)
{
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n = counts ? counts[b] : n_fixed;
    if (i >= n) return;
    const long long o = (long long)b * frame_cap + i;
    const uint4* fp = (const uint4*)(desc + o * 32);
    const uint4 fa = fp[0], fb = fp[1];
    const int nid_level = V.L - levelsup;
    int nid = 0, node = 0, level = 0;
    for (;;) {
        ++level;
        const int cs = V.child_start[node], nc = V.child_cnt[node];
        int child = 0;
        uint32_t key = 0xffffffffu;
        if (lane < nc) {
            child = V.children[cs + lane];
            const uint4* cp = (const uint4*)(V.desc + (long long)child * 32);
            key = ((uint32_t)og_hamming(fa, fb, cp[0], cp[1]) << 8) | (uint32_t)lane;
        }
        const uint32_t kmin = og_bow_wave_min(key);
        node = __builtin_amdgcn_readlane(child, (int)(kmin & 0xff));
        if (level == nid_level) nid = node;
        if (V.child_cnt[node] == 0) break;
    }
    if (lane == 0) {
        word[o] = V.word_id[node];
        wt[o] = V.weight[node];
        nidOut[o] = nid;
    }
}

#define BOW_NT 1024
#define BOW_MAXN 8192

// ascending bitonic sort of P (power of two) u64 keys in LDS
__device__ void og_bitonic_sort(u64* a, int P)
{
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P; t += BOW_NT) {
                const int u = t ^ j;
                if (u > t) {
                    const u64 x = a[t], y = a[u];
                    const bool up = (t & k) == 0;
                    if ((x > y) == up) {
                        a[t] = y;
                        a[u] = x;
                    }
                }
            }
            __syncthreads();
        }
}

__global__ __launch_bounds__(BOW_NT) void og_bow_reduce_kernel(OgVocDev V, const int* counts, int n_fixed, int frame_cap,
                                                              const int* __restrict__ word,
                                                              const double* __restrict__ wt,
                                                              const int* __restrict__ nidIn, int* __restrict__ words,
                                                              double* __restrict__ values, int* __restrict__ nwords,
                                                              int* __restrict__ nodes, int* __restrict__ node_off,
                                                              int* __restrict__ feats, int* __restrict__ nnodes)
{
    extern __shared__ __attribute__((aligned(16))) u64 keys[];  // [P]
    __shared__ int wsum[BOW_NT / 64];
    __shared__ double sh_norm;
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = counts ? counts[b] : n_fixed;
    int P = 2;
    while (P < n) P <<= 1;
    const long long base = (long long)b * frame_cap;
    int* W = words + base;
    double* Vv = values + base;
    int* ND = nodes + base;
    int* NO = node_off + (long long)b * (frame_cap + 1);
    int* FT = feats + base;
    const bool tf = V.weighting == 0 || V.weighting == 1;  // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    // ---- BowVector
    for (int t = tid; t < P; t += BOW_NT)
        keys[t] = (t < n && wt[base + t] > 0) ? (((u64)(uint32_t)word[base + t] << 32) | (u64)t) : ~0ull;
    __syncthreads();
    og_bitonic_sort(keys, P);
    // segment starts -> compacted word index (block scan over P elements, chunks of BOW_NT)
    int carry = 0;
    for (int t0 = 0; t0 < P; t0 += BOW_NT) {
        const int t = t0 + tid;
        const u64 k = t < P ? keys[t] : ~0ull;
        const bool valid = k != ~0ull;
        const bool start = valid && (t == 0 || (uint32_t)(keys[t - 1] >> 32) != (uint32_t)(k >> 32));
        const u64 m = __ballot(start);
        if (lane == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int before = carry;
        for (int q = 0; q < wv; q++) before += wsum[q];
        int tot = 0;
        for (int q = 0; q < BOW_NT / 64; q++) tot += wsum[q];
        if (start) {
            const int pos = before + __popcll(m & ((1ull << lane) - 1ull));
            double acc = wt[base + (int)(k & 0xffffffffu)];
            if (tf)  // the word's weights in feature order (keys sorted by (word, feature))
                for (int u = t + 1; u < P && keys[u] != ~0ull && (uint32_t)(keys[u] >> 32) == (uint32_t)(k >> 32); u++)
                    acc += wt[base + (int)(keys[u] & 0xffffffffu)];
            W[pos] = (int)(k >> 32);
            Vv[pos] = acc;
        }
        __syncthreads();
        carry += tot;
    }
    const int nw = carry;
    __threadfence_block();
    __syncthreads();
    const bool must = V.scoring != 5;  // mustNormalize: DOT_PRODUCT does not
    if (tid == 0) {
        double norm = 0.0;
        if (must) {
            if (V.scoring == 1) {
                for (int j = 0; j < nw; j++) norm += Vv[j] * Vv[j];
                norm = sqrt(norm);
            } else {
                for (int j = 0; j < nw; j++) norm += fabs(Vv[j]);
            }
        }
        sh_norm = norm;
    }
    __syncthreads();
    if (tf && nw > 0 && !must) {
        const double nd = nw;
        for (int j = tid; j < nw; j += BOW_NT) Vv[j] = Vv[j] / nd;
    }
    if (must && sh_norm > 0.0)
        for (int j = tid; j < nw; j += BOW_NT) Vv[j] = Vv[j] / sh_norm;
    // ---- FeatureVector
    for (int t = tid; t < P; t += BOW_NT)
        keys[t] = (t < n && wt[base + t] > 0) ? (((u64)(uint32_t)nidIn[base + t] << 32) | (u64)t) : ~0ull;
    __syncthreads();
    og_bitonic_sort(keys, P);
    carry = 0;
    int m_total = 0;
    for (int t0 = 0; t0 < P; t0 += BOW_NT) {
        const int t = t0 + tid;
        const u64 k = t < P ? keys[t] : ~0ull;
        const bool valid = k != ~0ull;
        const bool start = valid && (t == 0 || (uint32_t)(keys[t - 1] >> 32) != (uint32_t)(k >> 32));
        const u64 m = __ballot(start);
        const u64 mv = __ballot(valid);
        if (lane == 0) wsum[wv] = __popcll(m) | (__popcll(mv) << 16);
        __syncthreads();
        int before = carry;
        for (int q = 0; q < wv; q++) before += wsum[q] & 0xffff;
        int tot = 0, vt = 0;
        for (int q = 0; q < BOW_NT / 64; q++) tot += wsum[q] & 0xffff, vt += wsum[q] >> 16;
        if (valid) FT[t] = (int)(k & 0xffffffffu);
        if (start) {
            const int pos = before + __popcll(m & ((1ull << lane) - 1ull));
            ND[pos] = (int)(k >> 32);
            NO[pos] = t;
        }
        __syncthreads();
        carry += tot;
        m_total += vt;
    }
    if (tid == 0) {
        NO[carry] = m_total;
        nwords[b] = nw;
        nnodes[b] = carry;
    }
}

void og_launch_bow(hipStream_t s, const OgVocDev& V, const uint8_t* desc, const int* counts, int n_fixed,
                   int frame_cap, int levelsup, int* word, double* wt, int* nid, int* words, double* values,
                   int* nwords, int* nodes, int* node_off, int* feats, int* nnodes, int B)
{
    const int nmax = counts ? frame_cap : n_fixed;
    if (nmax > 0)
        hipLaunchKernelGGL(og_bow_descend_kernel, dim3((nmax + 3) / 4, B), dim3(256), 0, s, V, desc, counts, n_fixed,
                           frame_cap, levelsup, word, wt, nid);
    int P = 2;
    while (P < nmax) P <<= 1;
    hipLaunchKernelGGL(og_bow_reduce_kernel, dim3(B), dim3(BOW_NT), (size_t)P * 8, s, V, counts, n_fixed, frame_cap,
                       word, wt, nid, words, values, nwords, nodes, node_off, feats, nnodes);
}

// dynamic-LDS attribute of the reduce kernel: per device, set from og_prepare_device (orbgpu_create)
hipError_t og_prepare_device_bow()
{
    return hipFuncSetAttribute((const void*)og_bow_reduce_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               BOW_MAXN * 8);
}
