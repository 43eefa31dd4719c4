// orbgpu_launch.h -- host-side launchers of the gfx950 kernels (implemented in the .hip files).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbgpu_internal.h"

struct orbgpu_kp_dev {  // == orbgpu_keypoint == cv::KeyPoint (28 B)
    float x, y, size, angle, response;
    int octave, class_id;
};

struct OgGridGeom {
    float minX, minY, maxX, maxY, invW, invH;
};

hipError_t og_upload_pattern(int device);
// exhaustive pins of og_sincosf / og_logf (orb_pins.hip): chunked order-free hashes over a float bit range
hipError_t og_math_hash(int fn, unsigned long long begin, unsigned long long end, int chunk_log2,
                        unsigned long long* d_out, hipStream_t s);

// two chained levels per launch (og_resize2_kernel): A = level l from S = level l-1, B = level l+1 from A
struct OgRz2Geom {
    int sw, sh, aw, ah, bw, bh;
    const int4* xtabA;
    const int4* ytabA;
    int xmaxA;
    const int4* xtabB;
    const int4* ytabB;
    int xmaxB;
    int SR, SC, AR, AC;  // LDS capacities: staged S rows x row stride, A rows x row stride (host-computed maxima)
    const int4* tiles;   // per tile (row-major over B's 16 x 256 tiles): {ar0, ar1, own_r1, ac0}, {ac1, own_c1, sr0, sr1}, {sc0, sc1}
};
// og_resize2_kernel tiles: RZ2_TH rows x 256 columns of the coarser level per workgroup of 16 * RZ2_TH threads
// (4 output rows x 4 columns per thread in its last pass)
#define RZ2_TH 16  // (32-row tiles measured +7 % pyramid time)
#define RZ2_NT (16 * RZ2_TH)
// dynamic LDS of og_resize2_kernel: the A pass's y-table rows of the tile (AR int4), S, A, row misalignments
static inline size_t og_rz2_lds_bytes(int SR, int SC, int AR, int AC)
{
    return 16 * (size_t)AR + (size_t)SR * SC + (size_t)AR * AC + 4 * (size_t)SR;
}
void og_launch_resize2(hipStream_t s, const uint8_t* src, long long src_pitch, long long src_fstride, uint8_t* dstA,
                       long long pitchA, uint8_t* dstB, long long pitchB, long long dst_fstride, const OgRz2Geom& g,
                       int* status, int B, int sem);
void og_launch_resize(hipStream_t s, const uint8_t* src, long long src_pitch, long long src_fstride, uint8_t* dst,
                      long long dst_pitch, long long dst_fstride, int sw, int sh, int dw, int dh, const int4* xtab,
                      const int4* ytab, int xmax, int* status, int B, int sem);
hipError_t og_prepare_device();  // per-device kernel attributes (call after hipSetDevice)
hipError_t og_prepare_device_match();  // (called by og_prepare_device)
hipError_t og_prepare_device_bow();
// FAST of levels [lb, le) for each of B frames (table = the whole block table)
void og_launch_fast(hipStream_t s, const OgPlan& P, int lb, int le, const OgFastBlk* table, const uint8_t* img0,
                    long long pitch0, long long fstride0, const uint8_t* pyr, unsigned long long* cand, int* cand_count,
                    int* status, int B);
hipError_t og_read_fast_prof(unsigned long long* out, int n);  // OG_FAST_PROFILE builds only
hipError_t og_read_oct_prof(unsigned long long* out, int n);  // OG_OCT_PROFILE builds only
// ORBGPU_SEM_SCORE_HARRIS option: rewrite the response key of each candidate of levels [lb, le) with its Harris key
void og_launch_harris(hipStream_t s, const OgPlan& P, int lb, int le, const uint8_t* img0, long long pitch0,
                      long long fstride0, const uint8_t* pyr, unsigned long long* cand, const int* cand_count, int B);
// octree of levels [lb, le); oct_best: OG_OCT_BEST_CELLS u32 per (frame, level) of scratch (the cell-best table)
void og_launch_octree(hipStream_t s, const OgPlan& P, int lb, int le, const unsigned long long* cand,
                      const int* cand_count, uint16_t* node_of, unsigned* oct_best, uint32_t* oct_xy, uint32_t* oct_resp,
                      int* oct_count, int* status, int B);
void og_launch_describe(hipStream_t s, const OgPlan& P, const uint8_t* img0, long long pitch0, long long fstride0,
                        const uint8_t* pyr, const uint32_t* oct_xy, const uint32_t* oct_resp, const int* oct_count,
                        orbgpu_kp_dev* kps, uint8_t* desc, int* counts, int B);
// n ints at p to zero (one small kernel; the batch's candidate counters)
void og_launch_zero(hipStream_t s, int* p, int n);
// record_refused: non-null when the frames are a fresh extraction (clears the context's refused-record word)
void og_launch_grid(hipStream_t s, const orbgpu_kp_dev* kps, const int* counts, int frame_cap, OgGridGeom G,
                    int* cell_start, int* cell_items, int* status, int B, int* record_refused = nullptr);

// matchers (orb_match.hip)
// Ordering invariant of every writer of a context's keypoint slots (kps / kps_un): a frame's keypoints are in
// extraction order, levels nondecreasing (src/ORBextractor.cc:1076-1104), so its octave-0 keypoints are the first
// ones and number at most kcap_0 = plan.lv[0].kcap.  The batched SearchForInitialization queries F1's keypoints
// [0, qcap = kcap_0) only (og_init_resolve_kernel skips i >= qcap).  The writers today: the describe kernel
// (extraction, in order by construction) and og_record_unpack_kernel (refuses a record that breaks the order, status
// bit 128).  A future writer (host-supplied frames into a context's batch, reordering) must keep it or pass qcap = 0.
struct OgFrameDev {        // device view of one or many frames (batch stride frame_cap)
    const orbgpu_kp_dev* kps;
    const uint8_t* desc;
    const int* counts;     // per frame
    const int* cell_start; // per frame OG_GRID_CELLS+1
    const int* cell_items; // per frame frame_cap
    const float* uright;   // per frame frame_cap, or nullptr
    int frame_cap;
};

void og_launch_search_init(hipStream_t s, OgFrameDev F1, int ref, OgFrameDev F2, OgGridGeom G, float nnratio,
                           int checkOri, int windowSize, float* prev_xy, int prev_stride, int* matches12,
                           int match_stride, int* nmatches, uint32_t* lists, int list_cap, int* list_n, int* status,
                           int B, const int* ref_status = nullptr, int qcap = 0);

// LDS bytes of the ordered SearchForInitialization pass for frame capacities cap1/cap2 and `ecap` staged
// candidate entries; the pass needs og_init_resolve_lds(cap1, cap2, list_cap) <= OG_INIT_LDS_MAX
#define OG_INIT_LDS_MAX (150 * 1024)
size_t og_init_resolve_lds(int cap1, int cap2, int ecap);

void og_launch_prev_from_frame(hipStream_t s, OgFrameDev F1, int ref, float* prev_xy, int prev_stride, int B);

struct OgMapPointsDev {
    int m;
    const uint8_t* track_in_view;
    const uint8_t* is_bad;
    const int* level;
    const float* view_cos;
    const float* proj_x;
    const float* proj_y;
    const float* proj_xr;
    const int* n_obs;
    const uint8_t* desc;
    int shared_map = 0;  // batched forms: 1 = is_bad / n_obs / desc are one map shared by every frame (stride 0)
};

// batched SearchByProjection (B frames, map point j of frame b at b*stride + j of every mp array; mp.m points per
// frame): one enumeration pass writes each point's first OG_PJ_K kept candidates (dword entries, k-major slots of
// B * OG_PJ_K * stride) and its kept count (B * stride ints); then one workgroup per frame stages the lists in LDS
// and runs the parallel fixed-point resolve.  No host synchronisation.
#define OG_PJ_K 16
#define OG_PJ_LDS (159 * 1024)  // dynamic LDS of the resolve (its static LDS is < 1 KB)
int og_proj_keep_bound(float nnratio);
void og_launch_projb(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgMapPointsDev mp, int stride,
                     float nnratio, float th, int B, uint32_t* slots, int* kept, int* res, int* owner, int* owner_obs,
                     int* nmatches, int* status, int dbg);

// stereo (orb_stereo.hip): Frame::ComputeStereoMatches over frame pairs b of two extractor batches
struct OgStereoDev {
    OgFrameDev L, R;                 // left / right keypoints + descriptors (level-0 coordinates)
    const uint8_t* L0;               // level-0 images (the extractors' inputs)
    const uint8_t* R0;
    long long L0_pitch, L0_fstride, R0_pitch, R0_fstride;
    const uint8_t* Lpyr;             // levels >= 1 (same plan on both sides)
    const uint8_t* Rpyr;
    long long pyr_fstride;
    long long lvl_off[OG_MAXLEVELS];
    int lvl_pitch[OG_MAXLEVELS];
    int lvl_w[OG_MAXLEVELS];
    float sf[OG_MAXLEVELS], isf[OG_MAXLEVELS];
    float mbf, mb;
    int nRows;                       // level-0 image rows
    int row_cap;                     // per-frame capacity of row_items
    int* row_start;                  // per frame nRows+1
    int* row_items;                  // per frame row_cap
    float* uright;                   // per frame L.frame_cap
    float* depth;
    int* sad;                        // per frame L.frame_cap: SAD distance of a match, -1 otherwise
    int* nmatches;                   // per frame
};
void og_launch_stereo(hipStream_t s, const OgStereoDev& S, int B);

// projection matchers (orb_match.hip): Frame::isInFrustum (A17) and SearchByProjection(F, LastFrame) (A16)
struct OgCameraDev {          // Frame pose / intrinsics snapshot
    float R[9], t[3], Ow[3];  // mRcw (row-major), mtcw, mOw
    float fx, fy, cx, cy, mbf, mb;
    float scale_factor;       // mfScaleFactor (mfLogScaleFactor = logf of it, taken on the device)
    int nlevels;              // mnScaleLevels
    float minX, maxX, minY, maxY;
};
struct OgMapGeomDev {
    int m;
    const float* pos;      // m x 3
    const float* normal;   // m x 3
    const float* max_dist; // mfMaxDistance
    const float* min_dist; // mfMinDistance
};
// Frame::isInFrustum for B cameras (device array of orbgpu_camera's layout, the OgCameraDev prefix) against one shared
// map; outputs of camera b at b*stride + j
void og_launch_frustum_batch(hipStream_t s, const void* d_cams, int B, float minX, float maxX, float minY, float maxY,
                             struct OgMapGeomDev mp, float viewingCosLimit, struct OgFrustumOut out, int stride);
struct OgFrustumOut {
    uint8_t* in_view;
    float* proj_x;
    float* proj_y;
    float* proj_xr;
    int* level;
    float* view_cos;
    int* n_in_view;        // optional counter (nullptr = skip)
};
void og_launch_frustum(hipStream_t s, OgCameraDev cam, OgMapGeomDev mp, float viewingCosLimit, OgFrustumOut out);

struct OgLastFrameDev {
    int n;
    const orbgpu_kp_dev* kps;  // mvKeysUn (octave, angle)
    const uint8_t* has_mp;
    const uint8_t* outlier;
    const float* pos;          // n x 3
    const int* n_obs;
    const uint8_t* desc;       // n x 32
};
struct OgLastCand {
    int idx;
    int dist;
};
// mode: 0 = levels [o-1, o+1], 1 = forward [o, any), 2 = backward [0, o]
void og_launch_last_count(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                          OgLastFrameDev LF, float th, int mode, int* cnt, int* off);
void og_launch_last_resolve(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                            OgLastFrameDev LF, float th, int mode, int checkOri, const int* off, OgLastCand* cands,
                            int* ent, int* owner, int* owner_obs, int* nmatches);

// relocalisation SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist): KF.has_mp = valid flag, KF.outlier and
// KF.n_obs unused; cam.Ow = -Rcw^T tcw of the current frame as the reference computes it (:1478)
// pred_level (may be NULL): per KF point the caller's PredictScale level, -1 = outside the scale range; when given,
// max_dist / min_dist are not read
void og_launch_kf_count(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                        OgLastFrameDev KF, const float* max_dist, const float* min_dist, const int* pred_level,
                        float th, int* cnt, int* off);
void og_launch_kf_resolve(hipStream_t s, OgFrameDev F, OgGridGeom G, const float* sf, OgCameraDev cam,
                          OgLastFrameDev KF, const float* max_dist, const float* min_dist, const int* pred_level,
                          float th, int ORBdist, int checkOri, const int* off, OgLastCand* cands, int* ent, int* owner,
                          int* nmatches);

// Frame post-processing (orb_frame.hip): cv::undistortPoints of Frame::UndistortKeyPoints
struct OgUndistort {
    float K[4];  // fx, fy, cx, cy (mK)
    float d[5];  // k1, k2, p1, p2, k3 (mDistCoef, k3 = 0 when absent)
};
// counts == nullptr: n_fixed keypoints in one frame
void og_launch_undistort(hipStream_t s, const orbgpu_kp_dev* in, orbgpu_kp_dev* out, const int* counts, int n_fixed,
                         int frame_cap, const OgUndistort& U, int B);
void og_launch_undistort_points(hipStream_t s, const float* xy, float* out, int n, const OgUndistort& U);
// single-frame download: status, count, keypoints and descriptors of frame 0 into a pinned host block
// {status, count, 0, 0, frame_cap x 28 B, frame_cap x 32 B} (host_dev: its device-side address)
void og_launch_pack_host(hipStream_t s, const int* status, const int* counts, const orbgpu_kp_dev* kps,
                         const uint8_t* desc, int frame_cap, void* host_dev);
// frame-record unpack into frame 0, header and keypoint level order validated on the device (levels nondecreasing,
// octave-0 keypoints within the first kcap0 slots; otherwise count 0 and status bit 128)
void og_launch_record_unpack(hipStream_t s, const void* rec, int frame_cap, int undist, int kcap0, int* counts,
                             orbgpu_kp_dev* kps, uint8_t* desc, orbgpu_kp_dev* kps_un, int* status);
// Frame::ComputeStereoFromRGBD over B frames (counts == nullptr: one frame of n_fixed keypoints); depth rows
// are `pitch` bytes apart, frames `fstride` bytes; is_u16: raw CV_16U scaled by `factor`, else CV_32F
void og_launch_gray(hipStream_t s, const uint8_t* src, int cols, int rows, int cn, int bidx, long long spitch,
                    long long sfstride, uint8_t* dst, long long dpitch, long long dfstride, int B);
void og_launch_rgbd(hipStream_t s, const orbgpu_kp_dev* kps, const orbgpu_kp_dev* kps_un, const int* counts,
                    int n_fixed, int frame_cap, const uint8_t* depth, int is_u16, float factor, long long pitch,
                    long long fstride, float mbf, float* uright, float* dout, int B);

// DBoW2 transform (orb_bow.hip): device vocabulary, children in CSR (insertion order of loadFromTextFile)
struct OgVocDev {
    int n, L, scoring, weighting;
    const uint8_t* desc;      // n x 32
    const int* child_start;   // n
    const int* child_cnt;     // n
    const int* children;      // n
    const int* word_id;       // n (-1 for inner nodes)
    const double* weight;     // n
};
#define OG_BOW_MAXN 8192  // features per frame the LDS sort of og_bow_reduce_kernel holds
// counts == nullptr: one frame of n_fixed descriptors; word/wt/nid scratch and outputs at stride frame_cap
// (node_off: frame_cap + 1)
void og_launch_bow(hipStream_t s, const OgVocDev& V, const uint8_t* desc, const int* counts, int n_fixed,
                   int frame_cap, int levelsup, int* word, double* wt, int* nid, int* words, double* values,
                   int* nwords, int* nodes, int* node_off, int* feats, int* nnodes, int B);
