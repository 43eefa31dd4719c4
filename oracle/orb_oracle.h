/*
 * oracle/orb_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference's ORB extraction + matching hot path
 * (yxqc/ORBSLAM2_with_quadrics src/ORBextractor.cc, src/ORBmatcher.cc, src/Frame.cc).  It is the
 * checker for the HIP product (orbslam2_with_quadrics_amd/csrc) and the CPU baseline ("port") in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * PARITY STATUS: parity with the reference *binary* is UNPINNED -- the reference needs OpenCV 3.x,
 * Eigen3 and Pangolin, none of which exist in this image, and the reference ships no tests or golden
 * vectors.  Individual pieces are pinned: glibc sincosf (exhaustive, tools/verify_sincosf.c), GCC's FMA
 * contraction of the rBRIEF rotation (tools/probe_contraction.sh), the FAST score against its
 * definition (tests/test_oracle_pins.py), the ORB sampling pattern against the reference source text.
 * The OpenCV primitives follow the semantics written down in DESIGN.md §3; the ones that differ between
 * OpenCV versions/ISAs and compiler flags are selectable per extractor (oo_set_semantics, OO_SEM_*).
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same 28-byte layout as cv::KeyPoint {Point2f pt; float size, angle, response; int octave, class_id;} */
typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} oo_keypoint;

typedef struct oo_extractor oo_extractor;

oo_extractor* oo_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);

/* OpenCV/compiler behaviours the pixels depend on; same bits as ORBGPU_SEM_* in the
 * product's include/orbgpu.h (tests/test_oracle_pins.py checks the values agree).  0 = the default:
 * OpenCV 3.0-3.4.1 on x86-64 (SSE2, no IPP) under the reference's -O3 -march=native on an FMA host. */
#define OO_SEM_RESIZE_FIXEDPT 0x01 /* cv::resize vertical pass: generic FixedPtCast form, not the 8U form */
#define OO_SEM_BLUR_SHIFT 2        /* GaussianBlur variant, 3 bits: 0 SSE2_257, 1 SCALAR_257, 2 BITEXACT_256, 3 ED */
#define OO_SEM_BRIEF_NOFMA 0x20    /* rBRIEF rotation without FMA contraction */
#define OO_SEM_SCORE_HARRIS 0x40   /* option (not ORB-SLAM2): octree ranks by the Harris response (oo_harris_response) */
#define OO_SEM_ALL (OO_SEM_RESIZE_FIXEDPT | (7 << OO_SEM_BLUR_SHIFT) | OO_SEM_BRIEF_NOFMA | OO_SEM_SCORE_HARRIS)
/* Returns 0, or -1 for an unknown flag combination (the extractor is unchanged then). */
int oo_set_semantics(oo_extractor* e, int sem);
/* Harris response of OpenCV's ORB HARRIS_SCORE at pixel (x, y) of an 8-bit image (blockSize 7, k 0.04); the
 * pixel must lie >= 4 px inside the image. */
float oo_harris_response(const uint8_t* img, int stride, int x, int y);
void oo_destroy(oo_extractor* e);
int oo_nlevels(const oo_extractor* e);
void oo_scale_tables(const oo_extractor* e, float* scale, float* inv_scale, float* sigma2,
                     float* inv_sigma2, int* features_per_level, int* umax16);

/* ORBextractor::operator() (src/ORBextractor.cc:1043-1105).  Writes at most cap keypoints / rows.
 * Returns the number of keypoints, or -1 if cap is too small (nothing is written in that case). */
int oo_extract(oo_extractor* e, const uint8_t* img, int cols, int rows, int step, oo_keypoint* kps,
               uint8_t* desc, int cap);

/* Debug/introspection of the last oo_extract call. */
int oo_level_size(const oo_extractor* e, int level, int* cols, int* rows);
const uint8_t* oo_level_image(const oo_extractor* e, int level);       /* unpadded, stride = cols */
/* FAST candidates of a level in the reference's vToDistributeKeys order (x, y relative to minBorder,
 * response).  Returns the count; writes at most cap. */
int oo_level_candidates(const oo_extractor* e, int level, float* xy, float* resp, int cap);

/* DistributeOctTree on an explicit candidate list (x,y relative to minBorder, in vToDistributeKeys
 * order).  out_xy/out_resp need room for max(N+3, 4*nIni, n) entries.  Returns the output count. */
int oo_distribute_octree(const float* xy, const float* resp, int n, int minX, int maxX, int minY, int maxY,
                         int N, float* out_xy, float* out_resp);

/* Single-primitive entry points (used by tests to pin pieces). */
void oo_resize_linear(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, int sem);
void oo_gaussian7(const uint8_t* src, int w, int h, uint8_t* dst, int sem);
int oo_fast_score(const uint8_t* img, int stride, int x, int y);      /* M-1 or -1 (see DESIGN) */
float oo_fastatan2(float y, float x);
void oo_sincos(float ang, float* s, float* c);
int oo_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* ---------------------------------------------------------------------------------------------
 * Frame grid (src/Frame.cc:230-245, 327-392) and matchers (src/ORBmatcher.cc).
 * A "frame view" is a plain SoA snapshot of what the reference reads from Frame.
 * --------------------------------------------------------------------------------------------- */
typedef struct {
    int n;                      /* N keypoints */
    const oo_keypoint* kps;     /* mvKeysUn */
    const uint8_t* desc;        /* mDescriptors, n x 32 */
    const float* uright;        /* mvuRight (may be NULL => all -1) */
    float minX, minY, maxX, maxY;         /* mnMinX.. (static in reference) */
    float gridInvW, gridInvH;             /* mfGridElementWidthInv/HeightInv */
    const float* scale_factors;           /* mvScaleFactors */
    int nlevels;
    /* grid CSR (64 x 48 cells, cell index = ix*48+iy), filled by oo_grid_build */
    int* cell_start;            /* 64*48+1 */
    int* cell_items;            /* n */
} oo_frame;

void oo_grid_params(int cols, int rows, float* minX, float* minY, float* maxX, float* maxY,
                    float* invW, float* invH);
void oo_grid_build(oo_frame* f);
/* Frame::GetFeaturesInArea; returns count written to out (cap >= n is always enough). */
int oo_features_in_area(const oo_frame* f, float x, float y, float r, int minLevel, int maxLevel,
                        int* out);

/* ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:405-520).  prev_xy: 2*n1 floats (in/out),
 * matches12: n1 ints (out).  Returns nmatches. */
int oo_search_for_initialization(const oo_frame* f1, const oo_frame* f2, float nnratio,
                                 int checkOri, float* prev_xy, int* matches12, int windowSize);

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:45-129).
 * Map points as SoA.  owner (n ints, in/out): map point index owning each keypoint, or -1;
 * owner_obs (n ints, in/out): Observations()>0 flag of the current owner.  Returns nmatches. */
typedef struct {
    int m;
    const uint8_t* track_in_view;  /* mbTrackInView */
    const uint8_t* is_bad;         /* isBad() */
    const int* level;              /* mnTrackScaleLevel */
    const float* view_cos;         /* mTrackViewCos */
    const float* proj_x;           /* mTrackProjX */
    const float* proj_y;           /* mTrackProjY */
    const float* proj_xr;          /* mTrackProjXR */
    const int* n_obs;              /* Observations() */
    const uint8_t* desc;           /* GetDescriptor(), m x 32 */
} oo_mappoints;

int oo_search_by_projection(const oo_frame* f, const oo_mappoints* mp, float nnratio, float th,
                            int* owner, int* owner_obs);

/* Frame::ComputeStereoMatches (src/Frame.cc:466-640) on two oracle extractors' last pyramids.
 * uright/depth: N floats out.  Returns the number of surviving stereo matches. */
int oo_stereo_matches(const oo_extractor* EL, const oo_extractor* ER, const oo_keypoint* kL, const uint8_t* dL,
                      int N, const oo_keypoint* kR, const uint8_t* dR, int Nr, float mbf, float mb,
                      float* uright, float* depth);

/* Camera / pose snapshot of a Frame: mRcw (row-major), mtcw, mOw, intrinsics, mbf, mb, mfScaleFactor,
 * mnScaleLevels, image bounds mnMinX.. (src/Frame.cc:253-266, include/Frame.h). */
typedef struct {
    float Rcw[9], tcw[3], Ow[3];
    float fx, fy, cx, cy, mbf, mb;
    float scale_factor;
    int nlevels;
    float minX, maxX, minY, maxY;
} oo_camera;

/* MapPoint geometry read by Frame::isInFrustum: GetWorldPos, GetNormal, mfMaxDistance, mfMinDistance */
typedef struct {
    int m;
    const float* pos;      /* m x 3 */
    const float* normal;   /* m x 3 */
    const float* max_dist; /* mfMaxDistance */
    const float* min_dist; /* mfMinDistance */
} oo_mappoint_geom;

/* Frame::isInFrustum (src/Frame.cc:269-325) + MapPoint::PredictScale (src/MapPoint.cc:402-417) for every
 * map point; writes the mTrack* fields (SoA, m entries each).  Returns the number in view. */
int oo_is_in_frustum(const oo_camera* cam, const oo_mappoint_geom* mp, float viewingCosLimit, uint8_t* in_view,
                     float* proj_x, float* proj_y, float* proj_xr, int* level, float* view_cos);

/* LastFrame snapshot for SearchByProjection(Frame&, const Frame&, th, bMono) */
typedef struct {
    int n;
    const oo_keypoint* kps;  /* mvKeysUn (octave, angle; octave == mvKeys[i].octave) */
    const uint8_t* has_mp;   /* mvpMapPoints[i] != NULL */
    const uint8_t* outlier;  /* mvbOutlier[i] */
    const float* pos;        /* n x 3, GetWorldPos() */
    const int* n_obs;        /* Observations() */
    const uint8_t* desc;     /* n x 32, GetDescriptor() */
} oo_last_frame;

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 * (src/ORBmatcher.cc:1328-1470).  owner (F.n ints, in/out): last-frame index whose map point claims
 * the keypoint, or -1 (values >= LF.n denote pre-existing claims); owner_obs: Observations()>0 of
 * the claimant.  Returns nmatches. */
int oo_search_by_projection_last(const oo_frame* F, const oo_camera* cur, const oo_camera* last,
                                 const oo_last_frame* LF, float th, int bMono, int checkOri, int* owner,
                                 int* owner_obs);

/* KeyFrame snapshot for the relocalisation matcher */
typedef struct {
    int n;                   /* pKF->GetMapPointMatches().size() */
    const oo_keypoint* kps;  /* pKF->mvKeysUn (angle) */
    const uint8_t* valid;    /* pMP && !pMP->isBad() && !sAlreadyFound.count(pMP) */
    const float* pos;        /* n x 3 */
    const float* max_dist;   /* mfMaxDistance */
    const float* min_dist;   /* mfMinDistance */
    const uint8_t* desc;     /* n x 32 */
} oo_keyframe;

/* ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 * (src/ORBmatcher.cc:1472-1599).  owner (F.n ints, in/out): keyframe index claiming the keypoint, -1 = NULL,
 * >= KF.n = other claims.  Returns nmatches. */
void oo_kf_predicted_levels(const oo_camera* cur, const oo_keyframe* KF, int* level);
int oo_search_by_projection_kf(const oo_frame* F, const oo_camera* cur, const oo_keyframe* KF, float th, int ORBdist,
                               int checkOri, int* owner);

/* Frame::ComputeStereoFromRGBD (src/Frame.cc:643-664): depth = float map (step in floats). */
void oo_stereo_from_rgbd(const oo_keypoint* kps, const oo_keypoint* kps_un, int n, const float* depth, int step,
                         float mbf, float* uright, float* depth_out);
void oo_depth_u16_to_f32(const uint16_t* src, int n, float factor, float* dst);
/* cvtColor(..., CV_xxx2GRAY) 8U of Tracking::GrabImage* (src/Tracking.cc:169-255); bidx = blue channel */
void oo_cvt_gray(const uint8_t* src, int cols, int rows, int step, int cn, int bidx, uint8_t* dst, int dstep);

/* DBoW2 vocabulary + transform (oracle/oo_bow.c): Frame::ComputeBoW, src/Frame.cc:395-402 */
typedef struct oo_vocab oo_vocab;
oo_vocab* oo_vocab_from_arrays(int k, int L, int scoring, int weighting, int nn, const int* parent,
                               const uint8_t* is_leaf, const uint8_t* desc, const double* weight);
oo_vocab* oo_vocab_load_text(const char* path);
void oo_vocab_free(oo_vocab* v);
int oo_vocab_nodes(const oo_vocab* v);
int oo_vocab_words(const oo_vocab* v);
int oo_bow_transform(const oo_vocab* v, const uint8_t* desc, int n, int levelsup, int* words, double* values,
                     int* nwords, int* nodes, int* node_off, int* feat_idx, int* nnodes);

/* cv::undistortPoints(src, dst, K, D, noArray(), K) (OpenCV 3.4, 5 iterations) on n points (x, y interleaved);
 * K4 = fx, fy, cx, cy; dist = k1, k2, p1, p2[, k3] (ndist 4 or 5). */
void oo_undistort_points(const float* K4, const float* dist, int ndist, const float* xy, float* out, int n);
/* Frame::UndistortKeyPoints (src/Frame.cc:404-434): copies when k1 == 0. */
void oo_undistort_keypoints(const float* K4, const float* dist, int ndist, const oo_keypoint* in, oo_keypoint* out,
                            int n);
/* Frame::ComputeImageBounds (src/Frame.cc:436-461) and mfGridElementWidthInv/HeightInv. */
void oo_compute_image_bounds(const float* K4, const float* dist, int ndist, int cols, int rows, float* minX,
                             float* maxX, float* minY, float* maxY, float* invW, float* invH);

#ifdef __cplusplus
}
#endif
#endif
