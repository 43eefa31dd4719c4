/*
 * orbgpu.h -- C ABI of the MI355X (gfx950) ORB extract + match hot path.
 *
 * This is the drop-in boundary for yxqc/ORBSLAM2_with_quadrics's per-frame feature path.  Every entry
 * point names the reference interface it replaces.  Plain pointers and sizes only; no OpenCV or torch
 * types.  All functions return an int status (ORBGPU_OK == 0) unless documented otherwise.
 *
 * Threading: one orbgpu_ctx == one ORBextractor instance (its own HIP stream, device buffers and
 * pinned staging).  A context is not re-entrant (as ORB_SLAM2::ORBextractor is not: mvImagePyramid is
 * mutable state); distinct contexts may be used concurrently from different host threads
 * (src/Frame.cc:78-81 runs the left/right extractors on two std::threads).
 */
#ifndef ORBGPU_H
#define ORBGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBGPU_OK 0
#define ORBGPU_ERR_ARG (-1)         /* bad argument (NULL, wrong size, out of range) */
#define ORBGPU_ERR_HIP (-2)         /* HIP runtime error (no device, launch failure, OOM) */
#define ORBGPU_ERR_CAPACITY (-3)    /* caller capacity too small; *n holds the required count */
#define ORBGPU_ERR_UNSUPPORTED (-4) /* geometry the reference itself cannot handle (e.g. a pyramid
                                       level narrower than one 30-px FAST cell) */
#define ORBGPU_ERR_INTERNAL (-5)    /* a device-side capacity guard tripped (reported, never silent) */

/* Same 28-byte layout as cv::KeyPoint {Point2f pt; float size, angle, response; int octave,
 * class_id;} so a std::vector<cv::KeyPoint> can be filled in place. */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbgpu_keypoint;

typedef struct orbgpu_ctx orbgpu_ctx;

/* ---- ORBextractor -------------------------------------------------------------------------- */

/* Replaces ORBextractor::ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 * int minThFAST) -- include/ORBextractor.h:51-52, src/ORBextractor.cc:410-470.  `device` is the HIP
 * device ordinal.  Returns NULL on failure. */
orbgpu_ctx* orbgpu_create(int device, int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
                          int minThFAST);
/* Replaces ORBextractor::~ORBextractor (include/ORBextractor.h:54). */
void orbgpu_destroy(orbgpu_ctx* ctx);

/* ---- OpenCV / compiler semantics switch -----------------------------------------
 * The reference takes three pixel-level behaviours from outside its own source, and they differ between
 * OpenCV versions/ISAs and compiler flags.  Each context reproduces one choice per behaviour:
 *  - cv::resize INTER_LINEAR 8U vertical pass (src/ORBextractor.cc:1120):
 *      default  OpenCV's VResizeLinear 8U specialisation ((b0*(D0>>4))>>16 + (b1*(D1>>4))>>16 + 2) >> 2
 *               (OpenCV 2.4-4.x; its SSE2 mulhi body and its scalar tail compute the same form);
 *      ORBGPU_SEM_RESIZE_FIXEDPT  the generic FixedPtCast form (b0*D0 + b1*D1 + 2^21) >> 22;
 *  - GaussianBlur 7x7 sigma 2 on CV_8U (src/ORBextractor.cc:1086), ORBGPU_SEM_BLUR_*:
 *      SSE2_257     OpenCV 3.0-3.4.1 on x86-64 without IPP: kernel [18,34,49,55,49,34,18], column sums
 *                   rounded half-to-even (float SIMD) in columns x < 4*floor(w/4), half-up in the tail;
 *      SCALAR_257   the same kernel rounded half-up everywhere (no SIMD);
 *      BITEXACT_256 the bit-exact fixed-point GaussianBlur, kernel [18,34,49,54,49,34,18];
 *      BITEXACT_ED  the bit-exact GaussianBlur with the error-diffused kernel [18,34,48,56,48,34,18];
 *  - rBRIEF rotation (src/ORBextractor.cc:118-120): default fma(x, b, y*a) as GCC -O3 -march=native
 *    contracts it on an FMA host (the reference's CMakeLists.txt:11 flags); ORBGPU_SEM_BRIEF_NOFMA rounds
 *    both products.
 * ORBGPU_SEM_DEFAULT (0) = OpenCV 3.x (< 3.4.2) on x86-64 without IPP, reference built with its own flags. */
#define ORBGPU_SEM_DEFAULT 0x00
#define ORBGPU_SEM_RESIZE_FIXEDPT 0x01
#define ORBGPU_SEM_BLUR_SHIFT 2
#define ORBGPU_SEM_BLUR_SSE2_257 (0 << ORBGPU_SEM_BLUR_SHIFT)
#define ORBGPU_SEM_BLUR_SCALAR_257 (1 << ORBGPU_SEM_BLUR_SHIFT)
#define ORBGPU_SEM_BLUR_BITEXACT_256 (2 << ORBGPU_SEM_BLUR_SHIFT)
#define ORBGPU_SEM_BLUR_BITEXACT_ED (3 << ORBGPU_SEM_BLUR_SHIFT)
#define ORBGPU_SEM_BLUR_MASK (7 << ORBGPU_SEM_BLUR_SHIFT)
#define ORBGPU_SEM_BRIEF_NOFMA 0x20
/* Option, not a reference behaviour (off by default; set only through orbgpu_set_semantics, never by the environment):
 * the octree ranks candidates by the Harris response of OpenCV's ORB HARRIS_SCORE (features2d orb.cpp
 * HarrisResponses: 7x7 block, 3x3 Sobel-form gradients, k = 0.04, scale (1/(4*7*255))^4) at the FAST
 * candidate's level pixel instead of by the FAST score, and the keypoint response is that float.
 * ORB-SLAM2 itself always uses the FAST score (src/ORBextractor.cc:795-806, :621-632).  Parity of this
 * option is unpinned: no reference fixture holds a Harris-ranked extraction. */
#define ORBGPU_SEM_SCORE_HARRIS 0x40
#define ORBGPU_SEM_ALL (ORBGPU_SEM_RESIZE_FIXEDPT | ORBGPU_SEM_BLUR_MASK | ORBGPU_SEM_BRIEF_NOFMA | ORBGPU_SEM_SCORE_HARRIS)
/* the round-1 semantics of this build: generic resize form, 257-kernel rounded half-up, FMA rotation */
#define ORBGPU_SEM_ROUND1 (ORBGPU_SEM_RESIZE_FIXEDPT | ORBGPU_SEM_BLUR_SCALAR_257)
/* Select the semantics of later extractions on ctx.  ORBGPU_ERR_ARG for unknown bits or blur variants. */
int orbgpu_set_semantics(orbgpu_ctx* ctx, int flags);
int orbgpu_get_semantics(const orbgpu_ctx* ctx);

/* Inline getters of include/ORBextractor.h:63-83.  Vector getters write nlevels floats. */
int orbgpu_get_levels(const orbgpu_ctx* ctx);
float orbgpu_get_scale_factor(const orbgpu_ctx* ctx);
int orbgpu_get_scale_factors(const orbgpu_ctx* ctx, float* out);
int orbgpu_get_inverse_scale_factors(const orbgpu_ctx* ctx, float* out);
int orbgpu_get_scale_sigma_squares(const orbgpu_ctx* ctx, float* out);
int orbgpu_get_inverse_scale_sigma_squares(const orbgpu_ctx* ctx, float* out);
/* mnFeaturesPerLevel (src/ORBextractor.cc:435-446); nlevels ints. */
int orbgpu_get_features_per_level(const orbgpu_ctx* ctx, int* out);

/* Replaces void ORBextractor::operator()(InputArray image, InputArray mask, vector<KeyPoint>& kps,
 * OutputArray descriptors) -- include/ORBextractor.h:59-61, src/ORBextractor.cc:1043-1105.
 * img: host u8 grey image, `step` bytes per row.  Keypoints (level-0 coordinates, levels 0..n-1
 * concatenated) go to kps[0..*n), descriptors to desc (row-major *n x 32 bytes).  The mask is ignored
 * by the reference and therefore absent here.  cols==0 || rows==0 mirrors `_image.empty()`: returns OK
 * with *n = -1 and the outputs untouched.  If cap < required, returns ORBGPU_ERR_CAPACITY with *n set.
 * A capacity of orbgpu_max_keypoints(ctx) is always sufficient. */
int orbgpu_extract(orbgpu_ctx* ctx, const uint8_t* img, int cols, int rows, size_t step,
                   orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n);
int orbgpu_max_keypoints(const orbgpu_ctx* ctx);

/* Backs the public member std::vector<cv::Mat> mvImagePyramid (include/ORBextractor.h:85), read by
 * Frame::ComputeStereoMatches (src/Frame.cc:473,563,575,580): lazy download of level `level` of the
 * LAST frame processed (frame 0 of the last batch).  dst==NULL only queries the level size. */
int orbgpu_get_level(orbgpu_ctx* ctx, int level, uint8_t* dst, size_t dst_step, int* cols, int* rows);

/* ---- batched, device-resident extraction (MI355X-native extension; same per-frame result) --- */

/* Extract B frames that already live in HBM: frame b starts at d_imgs + b*frame_stride, rows are
 * `pitch` bytes apart (pitch < 16 MiB, else ORBGPU_ERR_UNSUPPORTED).  Enqueued on the context stream;
 * returns without synchronising.  Results stay on the device (orbgpu_batch_outputs) until
 * orbgpu_batch_download. */
int orbgpu_extract_batch_device(orbgpu_ctx* ctx, const uint8_t* d_imgs, int B, int cols, int rows,
                                size_t pitch, size_t frame_stride);
/* Device pointers of the last batch: kps[b*frame_cap + i], desc[(b*frame_cap + i)*32],
 * counts[b] (final keypoint count of frame b).  Valid until the next batch call. */
int orbgpu_batch_outputs(orbgpu_ctx* ctx, orbgpu_keypoint** d_kps, uint8_t** d_desc, int** d_counts,
                         int* frame_cap);
/* Frame::mGrid of the last batch (Frame::AssignFeaturesToGrid, src/Frame.cc:230-245) as CSR per frame b:
 * cell (ix, iy) -> items cell_items[b*frame_cap + cell_start[b*3073 + ix*48 + iy] .. + cell_start[.. + 1]),
 * keypoint indices in ascending order (the reference's push_back order). */
int orbgpu_batch_grid(orbgpu_ctx* ctx, int** d_cell_start, int** d_cell_items);
/* Synchronise and copy frame b of the last batch to the host. */
int orbgpu_batch_download(orbgpu_ctx* ctx, int b, orbgpu_keypoint* kps, uint8_t* desc, int cap,
                          int* n);

/* One extracted frame as a flat device record: count, keypoints, descriptors (and mvKeysUn with an
 * undistortion model) at the context's frame capacity.  A multi-GPU run extracts the initial frame of
 * Tracking::MonocularInitialization (src/Tracking.cc:563-635) on one rank and broadcasts this record (RCCL)
 * to the others, which unpack it as frame 0 of a one-frame batch and match their frames against it
 * (SURVEY §8(e)).  Both calls are enqueued on the context stream; unpack requires a context planned for the
 * same image size and parameters, and records the event the matchers of other contexts wait for.  The record's
 * 16-byte header holds the count, a magic word, frame_cap and the undistortion flag.  Unpack never blocks the host:
 * the header is checked on the device, in stream order.  A record that does not match the context's plan, whose
 * count exceeds frame_cap, or whose keypoints are not in extraction order (pyramid levels nondecreasing, as pack
 * writes them), leaves frame 0 with count 0, and the next call that checks the context's status
 * (orbgpu_synchronize, orbgpu_batch_download, or any other call that returns results to the host) returns
 * ORBGPU_ERR_ARG.  A batched SearchForInitialization on another context that matches against such a frame raises the
 * same condition in its own context (its next status check returns ORBGPU_ERR_ARG), so a refused record never passes
 * as "zero matches".  Without a planned context, unpack itself returns ORBGPU_ERR_ARG. */
long long orbgpu_frame_record_bytes(const orbgpu_ctx* ctx);
int orbgpu_frame_record_pack(orbgpu_ctx* ctx, int b, void* d_dst);
int orbgpu_frame_record_unpack(orbgpu_ctx* ctx, const void* d_src);

/* ---- Frame grid (src/Frame.cc:230-245, 327-392) ----------------------------------------------- */

/* Grid geometry of ComputeImageBounds + grid scales (src/Frame.cc:207-223, 436-464) for an
 * undistorted image: mnMinX=0, mnMaxX=cols, mnMinY=0, mnMaxY=rows, inv = 64/W, 48/H. */
typedef struct {
    float minX, minY, maxX, maxY, invW, invH;
} orbgpu_grid_geom;
int orbgpu_grid_geom_for_image(int cols, int rows, orbgpu_grid_geom* g);

/* ---- ORBmatcher ------------------------------------------------------------------------------- */

/* Replaces int ORBmatcher::DescriptorDistance(const Mat&, const Mat&) -- src/ORBmatcher.cc:1647-1663
 * (host-side, 32-byte rows). */
int orbgpu_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* A host snapshot of the Frame fields the matchers read: mvKeysUn, mDescriptors, mvuRight and the
 * grid geometry (static members of Frame in the reference). */
typedef struct {
    int n;
    const orbgpu_keypoint* kps;
    const uint8_t* desc;   /* n x 32 */
    const float* uright;   /* n floats, or NULL (monocular: all -1) */
    orbgpu_grid_geom grid;
    const float* scale_factors; /* mvScaleFactors, nlevels */
    int nlevels;
} orbgpu_frame_view;

/* Replaces int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<Point2f>&
 * vbPrevMatched, vector<int>& vnMatches12, int windowSize) with ORBmatcher(nnratio, checkOri) --
 * src/ORBmatcher.cc:405-520, include/ORBmatcher.h:69.  prev_xy: 2*F1.n floats (in/out),
 * matches12: F1.n ints (out).  *nmatches receives the return value of the reference. */
int orbgpu_search_for_initialization(orbgpu_ctx* ctx, const orbgpu_frame_view* F1,
                                     const orbgpu_frame_view* F2, float nnratio, int checkOri,
                                     float* prev_xy, int* matches12, int windowSize, int* nmatches);

/* Device-resident batch form: frame `ref` of ctx_ref's last batch is F1 for every frame b of ctx's last
 * batch (F2 = frame b), as Tracking::MonocularInitialization matches each new frame against the
 * initial frame (src/Tracking.cc:563-635).  d_prev_xy: B x ref_cap x 2 floats (in/out, device),
 * d_matches12: B x ref_cap ints (device), d_nmatches: B ints (device).  Enqueued on ctx's stream.  F1's keypoints
 * are in extraction order (pyramid levels ascending, as every extracted frame and every accepted frame record has
 * them), so its octave-0 queries (:419-421) are its first keypoints, at most the level-0 capacity. */
int orbgpu_search_for_initialization_batch(orbgpu_ctx* ctx_ref, int ref, orbgpu_ctx* ctx,
                                           orbgpu_grid_geom grid, float nnratio, int checkOri,
                                           int windowSize, float* d_prev_xy, int* d_matches12,
                                           int* d_nmatches);

/* vbPrevMatched[i] = F1.mvKeysUn[i].pt for every frame of ctx's last batch (src/Tracking.cc:573-575),
 * device-side, into d_prev_xy laid out as in orbgpu_search_for_initialization_batch. */
int orbgpu_prev_matched_from_frame(orbgpu_ctx* ctx_ref, int ref, orbgpu_ctx* ctx, float* d_prev_xy);

/* Map points as seen by SearchByProjection (MapPoint fields, include/MapPoint.h:91-99, snapshot
 * gathered under the reference's per-point mutexes). */
typedef struct {
    int m;
    const uint8_t* track_in_view; /* mbTrackInView */
    const uint8_t* is_bad;        /* isBad() */
    const int32_t* level;         /* mnTrackScaleLevel */
    const float* view_cos;        /* mTrackViewCos */
    const float* proj_x;          /* mTrackProjX */
    const float* proj_y;          /* mTrackProjY */
    const float* proj_xr;         /* mTrackProjXR */
    const int32_t* n_obs;         /* Observations() */
    const uint8_t* desc;          /* GetDescriptor(), m x 32 */
} orbgpu_mappoints_view;

/* Replaces int ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints,
 * const float th) with ORBmatcher(nnratio) -- src/ORBmatcher.cc:45-137, include/ORBmatcher.h:48.
 * owner (F.n ints, in/out) = F.mvpMapPoints as map-point indices (-1 == NULL); owner_obs (F.n ints,
 * in/out) = mvpMapPoints[i]->Observations()>0 for the current owner. */
int orbgpu_search_by_projection(orbgpu_ctx* ctx, const orbgpu_frame_view* F,
                                const orbgpu_mappoints_view* mp, float nnratio, float th,
                                int32_t* owner, int32_t* owner_obs, int* nmatches);

/* Device-resident batch form of SearchByProjection(Frame&, vpMapPoints, th) (src/ORBmatcher.cc:45-137), as
 * Tracking::SearchLocalPoints runs it for every camera of a rig (src/Tracking.cc:1184-1191): frame b of ctx's
 * last batch against its own map-point snapshot, whose point j is element b*mp_stride + j of every array of
 * *d_mp (device pointers; d_mp->m points per frame, desc rows 32 B).  d_uright: B x frame_cap mvuRight
 * (device) or NULL for monocular frames.  d_owner / d_owner_obs: B x frame_cap ints (in/out, device; owner =
 * map-point index j, -1 == NULL, indices >= d_mp->m = claims made before the call), d_nmatches: B ints.
 * Enqueued on the context stream (one int is read back to size the candidate lists). */
int orbgpu_search_by_projection_batch(orbgpu_ctx* ctx, const orbgpu_mappoints_view* d_mp, int mp_stride,
                                      float nnratio, float th, const float* d_uright, int32_t* d_owner,
                                      int32_t* d_owner_obs, int* d_nmatches);

/* orbgpu_search_by_projection_batch with one local map shared by every frame of the batch: the track fields
 * (track_in_view, level, view_cos, proj_x/y/xr) of frame b at element b*mp_stride + j, the map's own fields
 * (is_bad, n_obs, desc) at element j for every frame (as orbgpu_is_in_frustum_batch produces them). */
int orbgpu_search_by_projection_batch_shared_map(orbgpu_ctx* ctx, const orbgpu_mappoints_view* d_mp, int mp_stride,
                                                 float nnratio, float th, const float* d_uright, int32_t* d_owner,
                                                 int32_t* d_owner_obs, int* d_nmatches);

/* ---- Frame post-processing: UndistortKeyPoints / ComputeImageBounds ---------------------------- */

/* Replaces void Frame::UndistortKeyPoints() -- src/Frame.cc:404-434: mvKeysUn from mvKeys through
 * cv::undistortPoints(mat, mat, mK, mDistCoef, Mat(), mK) (OpenCV 3.4, 5 iterations).  K4 = fx, fy, cx, cy;
 * dist = k1, k2, p1, p2[, k3], ndist 0..5.  When k1 == 0 the keypoints are copied (the reference's
 * `mDistCoef.at<float>(0)==0.0` shortcut).  in/out may alias. */
int orbgpu_undistort_keypoints(orbgpu_ctx* ctx, const float* K4, const float* dist, int ndist,
                               const orbgpu_keypoint* in, orbgpu_keypoint* out, int n);

/* Replaces void Frame::ComputeImageBounds(const cv::Mat&) -- src/Frame.cc:436-461 -- and fills the grid
 * scales mfGridElementWidthInv/HeightInv (src/Frame.cc:103-104). */
int orbgpu_compute_image_bounds(orbgpu_ctx* ctx, const float* K4, const float* dist, int ndist, int cols,
                                int rows, orbgpu_grid_geom* g);

/* Device-resident Frame post-processing for batches: from the next batch on, every extracted frame also
 * gets mvKeysUn on the device, and the batch grid, orbgpu_prev_matched_from_frame and the batched
 * SearchForInitialization use mvKeysUn with the undistorted image bounds (as Frame does, src/Frame.cc:
 * 180-207).  ndist == 0 or k1 == 0 switches it off (mvKeysUn == mvKeys). */
int orbgpu_set_undistortion(orbgpu_ctx* ctx, const float* K4, const float* dist, int ndist);
/* Device pointer of the last batch's mvKeysUn (== the keypoints when undistortion is off; stride
 * frame_cap per frame) and the image bounds/grid scales in use. */
int orbgpu_batch_outputs_undistorted(orbgpu_ctx* ctx, orbgpu_keypoint** d_kps_un, orbgpu_grid_geom* bounds);

/* ---- projection matchers: isInFrustum (A17) and SearchByProjection(Frame&, const Frame&) (A16) ---- */

/* Pose / intrinsics snapshot of a Frame: mRcw (row-major 3x3), mtcw, mOw (= -Rcw^T tcw, the camera
 * centre), fx, fy, cx, cy, mbf, mb, mfScaleFactor, mnScaleLevels (src/Frame.cc:253-266, include/Frame.h). */
typedef struct {
    float Rcw[9];
    float tcw[3];
    float Ow[3];
    float fx, fy, cx, cy, mbf, mb;
    float scale_factor;
    int nlevels;
} orbgpu_camera;

/* MapPoint geometry Frame::isInFrustum reads (under the per-point mutexes): GetWorldPos(), GetNormal(),
 * mfMaxDistance, mfMinDistance (src/MapPoint.cc:373-383). */
typedef struct {
    int m;
    const float* pos;       /* m x 3 */
    const float* normal;    /* m x 3 */
    const float* max_dist;  /* m */
    const float* min_dist;  /* m */
} orbgpu_mappoint_geom_view;

/* Replaces the per-point bool Frame::isInFrustum(MapPoint*, float viewingCosLimit) -- src/Frame.cc:269-325,
 * with MapPoint::PredictScale(dist, Frame*) src/MapPoint.cc:402-417 -- for all m points at once, as
 * Tracking::SearchLocalPoints calls it (src/Tracking.cc:1167-1180).  `bounds` = mnMinX/mnMaxX/mnMinY/
 * mnMaxY (grid fields ignored).  Writes mbTrackInView (track_in_view) and, for points in view,
 * mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos; those arrays feed orbgpu_mappoints_view
 * directly.  *n_in_view (optional) = number of points in view. */
int orbgpu_is_in_frustum(orbgpu_ctx* ctx, const orbgpu_camera* cam, orbgpu_grid_geom bounds,
                         const orbgpu_mappoint_geom_view* mp, float viewingCosLimit, uint8_t* track_in_view,
                         float* proj_x, float* proj_y, float* proj_xr, int32_t* level, float* view_cos,
                         int* n_in_view);

/* Device-resident batch form for frames sharing one local map (Tracking::SearchLocalPoints of a camera rig or of a
 * frame batch, src/Tracking.cc:1143-1195): camera b = d_cams[b] (a DEVICE array of B orbgpu_camera) against the m
 * points of *d_mp (device pointers, shared by all frames).  The five outputs of frame b go to element b*m_stride + j
 * of each device array -- the track fields orbgpu_search_by_projection_batch_shared_map reads.  Enqueued on the
 * context stream. */
int orbgpu_is_in_frustum_batch(orbgpu_ctx* ctx, const orbgpu_camera* d_cams, int B, orbgpu_grid_geom bounds,
                               const orbgpu_mappoint_geom_view* d_mp, float viewingCosLimit, int m_stride,
                               uint8_t* d_in_view, float* d_px, float* d_py, float* d_pxr, int32_t* d_level,
                               float* d_vc);

/* LastFrame snapshot for the motion-model matcher. */
typedef struct {
    int n;                         /* LastFrame.N */
    const orbgpu_keypoint* kps;    /* mvKeysUn (octave and angle equal mvKeys') */
    const uint8_t* has_mp;         /* mvpMapPoints[i] != NULL */
    const uint8_t* outlier;        /* mvbOutlier[i] */
    const float* pos;              /* n x 3: mvpMapPoints[i]->GetWorldPos() */
    const int32_t* n_obs;          /* mvpMapPoints[i]->Observations() */
    const uint8_t* desc;           /* n x 32: mvpMapPoints[i]->GetDescriptor() */
} orbgpu_last_frame_view;

/* Replaces int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th,
 * const bool bMono) -- src/ORBmatcher.cc:1328-1470, include/ORBmatcher.h:56; called from
 * Tracking::TrackWithMotionModel (src/Tracking.cc:869-891).  F = CurrentFrame (kps, desc, uright,
 * bounds/grid, scale factors), cur/last = the two frames' poses (cur also gives K, mbf, mb).
 * owner (F.n ints, in/out) = CurrentFrame.mvpMapPoints as LastFrame keypoint indices (-1 == NULL,
 * values >= LF.n = claims from other map points); owner_obs (in/out) = Observations()>0 of the claimant.
 * checkOri = the matcher's mbCheckOrientation. */
int orbgpu_search_by_projection_last_frame(orbgpu_ctx* ctx, const orbgpu_frame_view* F,
                                           const orbgpu_camera* cur, const orbgpu_camera* last,
                                           const orbgpu_last_frame_view* LF, float th, int bMono, int checkOri,
                                           int32_t* owner, int32_t* owner_obs, int* nmatches);

/* KeyFrame snapshot for the relocalisation / loop matcher. */
typedef struct {
    int n;                         /* pKF->GetMapPointMatches().size() */
    const orbgpu_keypoint* kps;    /* pKF->mvKeysUn (angle) */
    const uint8_t* valid;          /* pMP && !pMP->isBad() && !sAlreadyFound.count(pMP) */
    const float* pos;              /* n x 3: GetWorldPos() */
    const float* max_dist;         /* mfMaxDistance */
    const float* min_dist;         /* mfMinDistance */
    const uint8_t* desc;           /* n x 32: GetDescriptor() */
} orbgpu_keyframe_view;

/* Replaces int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
 * sAlreadyFound, const float th, const int ORBdist) -- src/ORBmatcher.cc:1472-1599, include/ORBmatcher.h:59;
 * called from Tracking::Relocalization (src/Tracking.cc:1433,1467).  owner (F.n ints, in/out) =
 * CurrentFrame.mvpMapPoints as keyframe indices (-1 == NULL, values >= KF.n = other claims; any claim
 * blocks the keypoint).  `cur` gives the current pose (Tcw) and intrinsics; cur->Ow is not read (the
 * matcher recomputes Ow = -Rcw^T tcw, :1478). */
int orbgpu_search_by_projection_keyframe(orbgpu_ctx* ctx, const orbgpu_frame_view* F, const orbgpu_camera* cur,
                                         const orbgpu_keyframe_view* KF, float th, int ORBdist, int checkOri,
                                         int32_t* owner, int* nmatches);

/* The same matcher with the scale test done by the caller: pred_level[i] (KF.n ints) is
 * pMP->PredictScale(dist3D, &CurrentFrame) when GetMinDistanceInvariance() <= dist3D <=
 * GetMaxDistanceInvariance() and -1 otherwise (src/ORBmatcher.cc:1513-1523), computed by the binding with the
 * reference's own MapPoint methods -- mfMaxDistance / mfMinDistance are protected (include/MapPoint.h:141-142), so
 * a drop-in binding cannot snapshot them.  KF.max_dist / KF.min_dist are not read (may be NULL); everything else
 * is as orbgpu_search_by_projection_keyframe. */
int orbgpu_search_by_projection_keyframe_levels(orbgpu_ctx* ctx, const orbgpu_frame_view* F, const orbgpu_camera* cur,
                                                const orbgpu_keyframe_view* KF, const int32_t* pred_level, float th,
                                                int ORBdist, int checkOri, int32_t* owner, int* nmatches);

/* ---- stereo ------------------------------------------------------------------------------------- */

/* Replaces void Frame::ComputeStereoMatches() -- src/Frame.cc:466-640, called from the stereo Frame
 * constructor src/Frame.cc:88.  `left` and `right` are the two extractors (mpORBextractorLeft/Right)
 * right after orbgpu_extract on the rectified left and right images; both must share image size and
 * scale pyramid (as constructed in src/Tracking.cc:119-122).  Reads mvKeys/mvKeysRight, both
 * descriptor sets and both image pyramids from device memory; writes mvuRight (uright) and mvDepth
 * (depth) for the n left keypoints (-1 where unmatched).  mbf = fx * baseline, mb = baseline.
 * *nmatches (optional) = number of surviving matches after the 2.1 x median SAD filter.
 * ORBGPU_ERR_CAPACITY (with *n set) when n > cap. */
int orbgpu_compute_stereo_matches(orbgpu_ctx* left, orbgpu_ctx* right, float mbf, float mb,
                                  float* uright, float* depth, int cap, int* n, int* nmatches);

/* Batched device form: frame b of the left batch is paired with frame b of the right batch (both
 * from orbgpu_extract_batch_device with the same B; the input image buffers must still be alive).
 * d_uright/d_depth have stride = left frame_cap per frame; d_nmatches one int per frame.  Runs on
 * the left context's stream after the right context's last batch. */
int orbgpu_compute_stereo_matches_batch(orbgpu_ctx* left, orbgpu_ctx* right, float mbf, float mb,
                                        float* d_uright, float* d_depth, int* d_nmatches);

/* Experiment builds only (OG_OCT_PROFILE=1, tools/octree_profile.py): per-round clock64 stamps and list
 * sizes of the octree workgroup of (frame 0, level 0) of the last batch.  ORBGPU_ERR_UNSUPPORTED in the
 * product build. */
int orbgpu_debug_octree_profile(orbgpu_ctx* ctx, unsigned long long* out, int n);
/* Diagnostic builds only (OG_FAST_PROFILE=1, tools/fast_profile.py): per-phase s_memtime clocks of every FAST block
 * of the middle frame of the last launch, 8 per block (ROI, stage 1-3, counts, reservation, end, survivors | level
 * << 32).  ORBGPU_ERR_UNSUPPORTED in product builds. */
int orbgpu_debug_fast_profile(orbgpu_ctx* ctx, unsigned long long* out, int n);
/* Test hook: make the context's SearchByProjection launches (host and batch forms) take the paths of frames too large
 * for the LDS, so tests can pin them against the oracle on ordinary frames.  flags: ORBGPU_DEBUG_PROJ_FILL_HBM =
 * enumerate windows from the frame geometry in HBM instead of the LDS copy; ORBGPU_DEBUG_PROJ_RESOLVE_HBM = run the
 * claim rounds on the candidate slots in HBM instead of LDS-staged lists.  0 restores the default. */
#define ORBGPU_DEBUG_PROJ_FILL_HBM 1
#define ORBGPU_DEBUG_PROJ_RESOLVE_HBM 2
int orbgpu_debug_set_projection_paths(orbgpu_ctx* ctx, int flags);
/* Exhaustive pin of the device restatements of glibc sincosf (fn 0; src/ORBextractor.cc:113) and logf (fn 1;
 * src/MapPoint.cc:410): every float bit pattern u in [begin, end) is evaluated on `device` and folded into
 * out[(u >> chunk_log2) - (begin >> chunk_log2)] (nchunks entries) as the order-free hash of
 * tools/libm_chunk_hash.c, which computes the same hashes from the host libm. */
int orbgpu_debug_math_hash(int device, int fn, unsigned long long begin, unsigned long long end, int chunk_log2,
                           unsigned long long* out, int nchunks);

/* ---- Colour input: Tracking::GrabImage* -------------------------------------------------------------- */

/* cv::cvtColor codes accepted by the colour entry points (OpenCV's own values, so a caller passes what it
 * passed to cvtColor): 3-channel BGR / RGB, 4-channel BGRA / RGBA, 8 bits per channel. */
#define ORBGPU_COLOR_BGR2GRAY 6
#define ORBGPU_COLOR_RGB2GRAY 7
#define ORBGPU_COLOR_BGRA2GRAY 10
#define ORBGPU_COLOR_RGBA2GRAY 11

/* Replaces the cvtColor(mImGray, mImGray, CV_RGB2GRAY / CV_BGR2GRAY / CV_RGBA2GRAY / CV_BGRA2GRAY) of
 * Tracking::GrabImageStereo / GrabImageRGBD / GrabImageMonocular (src/Tracking.cc:169-198, 209-225, 240-255),
 * batched and device-resident: frame b at d_src + b*src_frame_stride (rows of cols*channels bytes at
 * src_pitch) -> 8-bit gray at d_dst + b*dst_frame_stride (dst_pitch).  OpenCV's integer RGB2Gray<uchar>:
 * Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14.  Runs on the context's stream. */
int orbgpu_cvt_color_to_gray_batch(orbgpu_ctx* ctx, const uint8_t* d_src, int B, int cols, int rows,
                                   size_t src_pitch, size_t src_frame_stride, int code, uint8_t* d_dst,
                                   size_t dst_pitch, size_t dst_frame_stride);

/* Tracking::GrabImage*'s colour conversion followed by Frame::ExtractORB -> ORBextractor::operator()
 * (src/Tracking.cc:209-230, src/Frame.cc:247-253) for one host colour image: the image goes to HBM once, is
 * converted there and extracted from the gray copy (which also backs orbgpu_get_level(0)).  Same outputs,
 * capacity and empty-image rules as orbgpu_extract; step = bytes per source row. */
int orbgpu_extract_color(orbgpu_ctx* ctx, const uint8_t* img, int cols, int rows, size_t step, int code,
                         orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n);

/* ---- RGB-D ------------------------------------------------------------------------------------------ */

/* Replaces void Frame::ComputeStereoFromRGBD(const cv::Mat& imDepth) -- src/Frame.cc:643-664, called from the
 * RGB-D Frame constructor (src/Frame.cc:161) -- for the frame the context extracted last (mvKeys for the
 * lookup, mvKeysUn when orbgpu_set_undistortion is active).  depth: CV_32F (is_u16 = 0) or the raw CV_16U
 * image with Tracking::GrabImageRGBD's convertTo(CV_32F, mDepthMapFactor) fused in (is_u16 = 1, factor =
 * mDepthMapFactor; src/Tracking.cc:227-228).  Writes mvuRight / mvDepth (-1 where the depth is <= 0). */
int orbgpu_compute_stereo_from_rgbd(orbgpu_ctx* ctx, const void* depth, int is_u16, float factor, size_t step_bytes,
                                    float mbf, float* uright, float* depth_out, int cap, int* n);
/* Batched device form over the context's last batch: depth frame b at d_depth + b*frame_stride_bytes;
 * outputs at stride frame_cap per frame. */
int orbgpu_compute_stereo_from_rgbd_batch(orbgpu_ctx* ctx, const void* d_depth, int is_u16, float factor,
                                          size_t pitch_bytes, size_t frame_stride_bytes, float mbf, float* d_uright,
                                          float* d_depth_out);

/* ---- Bag of words: Frame::ComputeBoW ---------------------------------------------------------------- */

/* A DBoW2 vocabulary (ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB>, include/ORBVocabulary.h)
 * resident on the context's device. */
typedef struct orbgpu_vocabulary orbgpu_vocabulary;

/* Replaces TemplatedVocabulary::loadFromTextFile (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1420, called
 * at src/System.cc:65): header "k L scoring weighting", then one line per node "parent isLeaf d0..d31 weight".
 * NULL on failure (message in orbgpu_last_error(ctx)). */
orbgpu_vocabulary* orbgpu_vocabulary_load_text(orbgpu_ctx* ctx, const char* path);
/* The same from arrays: nn nodes 1..nn in file order (node 0 is the root). */
orbgpu_vocabulary* orbgpu_vocabulary_create(orbgpu_ctx* ctx, int k, int L, int scoring, int weighting, int nn,
                                            const int* parent, const uint8_t* is_leaf, const uint8_t* desc,
                                            const double* weight);
void orbgpu_vocabulary_destroy(orbgpu_vocabulary* voc);
int orbgpu_vocabulary_info(const orbgpu_vocabulary* voc, int* k, int* L, int* nodes, int* words);

/* Replaces void Frame::ComputeBoW() -- src/Frame.cc:395-402 --
 * mpORBvocabulary->transform(Converter::toDescriptorVector(mDescriptors), mBowVec, mFeatVec, levelsup = 4).
 * mBowVec as (*nwords) ascending word ids + double values; mFeatVec as (*nnodes) ascending node ids, offsets
 * node_off[0..nnodes] into feats (feature indices in feature order).  Capacities: n each (n+1 for node_off). */
int orbgpu_compute_bow(orbgpu_ctx* ctx, const orbgpu_vocabulary* voc, const uint8_t* desc, int n, int levelsup,
                       int32_t* words, double* values, int* nwords, int32_t* nodes, int32_t* node_off,
                       int32_t* feats, int* nnodes);
/* Batched device form over the context's last batch (descriptors in HBM): per frame b, outputs at stride
 * frame_cap (node_off: frame_cap + 1), counts in d_nwords[b] / d_nnodes[b]. */
int orbgpu_compute_bow_batch(orbgpu_ctx* ctx, const orbgpu_vocabulary* voc, int levelsup, int32_t* d_words,
                             double* d_values, int32_t* d_nwords, int32_t* d_nodes, int32_t* d_node_off,
                             int32_t* d_feats, int32_t* d_nnodes);

/* ---- stream / timing helpers ------------------------------------------------------------------ */

/* The context's hipStream_t (as void*), e.g. for torch.cuda.ExternalStream. */
void* orbgpu_stream(orbgpu_ctx* ctx);
int orbgpu_synchronize(orbgpu_ctx* ctx);
/* Per-stage HIP-event timing of the batch pipeline (off by default).  When on, every stage of
 * orbgpu_extract_batch_device / *_batch is bracketed by events on the context stream;
 * orbgpu_stage_times writes up to cap (name, milliseconds) pairs of the last batch and returns the
 * number of stages. */
int orbgpu_set_stage_timing(orbgpu_ctx* ctx, int on);
int orbgpu_stage_times(orbgpu_ctx* ctx, const char** names, float* ms, int cap);
/* The same marks as absolute times: milliseconds from `ref`'s first mark of its last batch to each mark
 * of ctx's (both contexts on one device, timing on).  Lets a caller measure the union of a stage's
 * busy intervals across concurrently running contexts.  Returns the number of marks written. */
int orbgpu_stage_marks(orbgpu_ctx* ctx, orbgpu_ctx* ref, const char** names, float* t_ms, int cap);
/* Human-readable message for the last error on this context (static storage, never NULL). */
const char* orbgpu_last_error(const orbgpu_ctx* ctx);

/* Introspection of the last batch (parity tests): FAST candidates of (frame b, level) as packed u64
 * {x-16:16, y-16:16, response key:32} in arbitrary order, and the octree output of (b, level) in list
 * order as u32 {x:16, y:16} (level pixels) + u32 response key.  The key is the FAST score (0..255), or
 * under ORBGPU_SEM_SCORE_HARRIS the order-preserving image of the float Harris response (bits ^ 0x80000000
 * for >= +0, ~bits below).  Return the count (or < 0 on error). */
int orbgpu_debug_candidates(orbgpu_ctx* ctx, int b, int level, uint64_t* out, int cap);
int orbgpu_debug_octree(orbgpu_ctx* ctx, int b, int level, uint32_t* xy, uint32_t* resp, int cap);

/* Device memory helpers for callers without a HIP runtime of their own (tests, bench). */
void* orbgpu_device_alloc(orbgpu_ctx* ctx, size_t bytes);
int orbgpu_device_free(orbgpu_ctx* ctx, void* p);
int orbgpu_memcpy_h2d(orbgpu_ctx* ctx, void* dst, const void* src, size_t bytes);
int orbgpu_memcpy_d2h(orbgpu_ctx* ctx, void* dst, const void* src, size_t bytes);
int orbgpu_memset_d(orbgpu_ctx* ctx, void* dst, int value, size_t bytes);
/* Asynchronous copies on the context stream (host memory should be pinned for the H2D/D2H forms to overlap). */
int orbgpu_memcpy_h2d_async(orbgpu_ctx* ctx, void* dst, const void* src, size_t bytes);
int orbgpu_memcpy_d2h_async(orbgpu_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Asynchronous device-to-device copy on the context stream. */
int orbgpu_memcpy_d2d_async(orbgpu_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Total FAST candidates of the last batch (all frames, all levels); synchronises.  < 0 on error. */
long long orbgpu_batch_candidate_total(orbgpu_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
