// tests/binding_run/run_matchers.cc -- executes the matcher and stereo drop-in bindings
// (integration/ORBmatcher_perframe.cc, integration/Frame_stereo.cc) together with the extractor binding
// (integration/ORBextractor.cc, built against the reference's unchanged include/ORBextractor.h), with the calls
// ORB-SLAM2 makes (tests/test_gpu_binding_matchers.py compares every output with the CPU oracle).  Test
// infrastructure: Frame / MapPoint / KeyFrame are the restated declarations of integration/refdecl with the
// test-only definitions of tests/binding_run/refstubs.cc.
//
//   run_matchers <mode> <in.blob> <out.blob>      mode: init | proj | last | kf | stereo
//
// A blob is a sequence of named arrays: u32 name length, name, u64 byte count, bytes (tests/test_gpu_binding_matchers.py
// writes and reads them).  Every mode extracts its frames through ORBextractor::operator() (Frame::ExtractORB,
// src/Frame.cc:247-253) and writes each frame's keypoints and descriptors, so the test can check them too.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "refstubs.h"

using namespace ORB_SLAM2;

typedef std::map<std::string, std::vector<char>> Blob;

static Blob read_blob(const char* path)
{
    std::ifstream in(path, std::ios::binary);
    if (!in) throw std::runtime_error(std::string("cannot open ") + path);
    Blob b;
    uint32_t nl;
    while (in.read(reinterpret_cast<char*>(&nl), 4)) {
        std::string name(nl, '\0');
        uint64_t nb;
        in.read(&name[0], nl);
        in.read(reinterpret_cast<char*>(&nb), 8);
        std::vector<char> v(nb);
        if (nb) in.read(v.data(), (std::streamsize)nb);
        if (!in) throw std::runtime_error("truncated blob");
        b[name] = std::move(v);
    }
    return b;
}

struct Out {
    std::ofstream f;
    explicit Out(const char* p) : f(p, std::ios::binary) {}
    void put(const std::string& name, const void* p, size_t n)
    {
        const uint32_t nl = (uint32_t)name.size();
        const uint64_t nb = n;
        f.write(reinterpret_cast<const char*>(&nl), 4);
        f.write(name.data(), nl);
        f.write(reinterpret_cast<const char*>(&nb), 8);
        if (n) f.write(static_cast<const char*>(p), (std::streamsize)n);
    }
    template <typename T>
    void vec(const std::string& name, const std::vector<T>& v)
    {
        put(name, v.data(), v.size() * sizeof(T));
    }
    void i32(const std::string& name, int v) { put(name, &v, 4); }
};

template <typename T>
static std::vector<T> arr(const Blob& b, const std::string& k)
{
    auto it = b.find(k);
    if (it == b.end()) throw std::runtime_error("blob lacks " + k);
    if (it->second.size() % sizeof(T)) throw std::runtime_error("bad size of " + k);
    std::vector<T> v(it->second.size() / sizeof(T));
    if (!v.empty()) std::memcpy(v.data(), it->second.data(), it->second.size());
    return v;
}
template <typename T>
static T scalar(const Blob& b, const std::string& k)
{
    const std::vector<T> v = arr<T>(b, k);
    if (v.size() != 1) throw std::runtime_error(k + " is not a scalar");
    return v[0];
}

// image `name` (H x W bytes) through the extractor binding; fills the Frame fields Frame's constructor sets from it
// for an undistorted camera (src/Frame.cc:170-215: mvKeysUn = mvKeys when k1 == 0, src/Frame.cc:404-412)
static void extract(ORBextractor& ex, const Blob& b, const std::string& name, int W, int H, Frame& F, Out& out,
                    const std::string& tag)
{
    std::vector<uint8_t> img = arr<uint8_t>(b, name);
    if (img.size() != (size_t)W * H) throw std::runtime_error("image size");
    cv::Mat im(H, W, CV_8UC1, img.data(), (size_t)W);
    std::vector<cv::KeyPoint> keys;
    cv::Mat desc;
    ex(im, cv::Mat(), keys, desc);  // Frame::ExtractORB (src/Frame.cc:247-253)
    F.N = (int)keys.size();
    F.mvKeysUn = keys;
    F.mDescriptors = desc;
    F.mpORBextractorLeft = &ex;
    F.mpORBextractorRight = nullptr;
    F.mnScaleLevels = ex.GetLevels();
    F.mfScaleFactor = ex.GetScaleFactor();
    F.mfLogScaleFactor = std::log(F.mfScaleFactor);  // src/Frame.cc:184
    F.mvScaleFactors = ex.GetScaleFactors();
    F.mvpMapPoints.assign(F.N, nullptr);
    F.mvbOutlier.assign(F.N, false);
    out.vec(tag + "_kps", keys);
    std::vector<uint8_t> d((size_t)F.N * 32);
    for (int r = 0; r < desc.rows; r++) std::memcpy(&d[32 * (size_t)r], desc.data + r * desc.step, 32);
    out.vec(tag + "_desc", d);
}

// Frame::ComputeImageBounds for an undistorted camera (src/Frame.cc:457-463) and the grid constants (:155-156)
static void set_static_geometry(const Blob& b, int W, int H)
{
    Frame::mnMinX = 0.0f;
    Frame::mnMaxX = (float)W;
    Frame::mnMinY = 0.0f;
    Frame::mnMaxY = (float)H;
    Frame::mfGridElementWidthInv = 64.0f / (Frame::mnMaxX - Frame::mnMinX);
    Frame::mfGridElementHeightInv = 48.0f / (Frame::mnMaxY - Frame::mnMinY);
    if (b.count("K")) {
        const std::vector<float> K = arr<float>(b, "K");  // fx, fy, cx, cy
        Frame::fx = K[0];
        Frame::fy = K[1];
        Frame::cx = K[2];
        Frame::cy = K[3];
    }
}

static cv::Mat pose(const Blob& b, const std::string& k)
{
    const std::vector<float> T = arr<float>(b, k);
    if (T.size() != 16) throw std::runtime_error(k + ": 4x4 pose expected");
    cv::Mat m(4, 4, CV_32F);
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) m.at<float>(r, c) = T[4 * r + c];
    return m;
}

static MapPoint* new_point(const float* pos, const uint8_t* desc, int nobs)
{
    MapPoint* p = new MapPoint();
    MapPointState& s = state_of(p);
    if (pos) std::memcpy(s.pos, pos, 12);
    if (desc) std::memcpy(s.desc, desc, 32);
    s.nobs = nobs;
    return p;
}

// CurrentFrame.mvpMapPoints claims made before a matcher call: claim[i] = -1 none, 0 a point with no observations,
// 1 a point with observations (those block the keypoint, src/ORBmatcher.cc:87-89)
static void preclaim(Frame& F, const std::vector<int32_t>& claim, MapPoint* obs0, MapPoint* obs1)
{
    if ((int)claim.size() != F.N) throw std::runtime_error("claims do not match the extracted keypoint count");
    for (int i = 0; i < F.N; i++) F.mvpMapPoints[i] = claim[i] < 0 ? nullptr : (claim[i] ? obs1 : obs0);
}

// owner per keypoint: index of the matched point in `pts`, `npts` for a pre-claiming point, -1 for none
static std::vector<int32_t> owners(const Frame& F, const std::vector<MapPoint*>& pts, MapPoint* c0, MapPoint* c1)
{
    std::map<const MapPoint*, int> idx;
    for (size_t m = 0; m < pts.size(); m++)
        if (pts[m]) idx[pts[m]] = (int)m;
    std::vector<int32_t> o(F.N, -1);
    for (int i = 0; i < F.N; i++) {
        const MapPoint* p = F.mvpMapPoints[i];
        if (!p) continue;
        if (p == c0 || p == c1) o[i] = (int)pts.size();
        else if (idx.count(p)) o[i] = idx[p];
        else throw std::runtime_error("unknown map point in mvpMapPoints");
    }
    return o;
}

int main(int argc, char** argv)
{
    if (argc != 4) {
        std::cerr << "usage: run_matchers <init|proj|last|kf|stereo> <in.blob> <out.blob>\n";
        return 2;
    }
    try {
        const std::string mode = argv[1];
        const Blob b = read_blob(argv[2]);
        Out out(argv[3]);
        const std::vector<int32_t> P = arr<int32_t>(b, "params");  // W, H, nfeatures, ...
        const int W = P[0], H = P[1], nfeat = P[2];
        set_static_geometry(b, W, H);
        ORBextractor ex(nfeat, 1.2f, 8, 20, 7);
        if (mode == "init") {
            // Tracking::MonocularInitialization (src/Tracking.cc:563-610): ORBmatcher matcher(0.9, true) and
            // SearchForInitialization(mInitialFrame, mCurrentFrame, mvbPrevMatched, mvIniMatches, 100)
            Frame F1, F2;
            extract(ex, b, "img1", W, H, F1, out, "f1");
            extract(ex, b, "img2", W, H, F2, out, "f2");
            const std::vector<float> ratio = arr<float>(b, "ratio");
            const std::vector<int32_t> window = arr<int32_t>(b, "window"), ori = arr<int32_t>(b, "check_ori");
            for (size_t c = 0; c < ratio.size(); c++) {
                std::vector<cv::Point2f> prev(F1.mvKeysUn.size());
                for (size_t i = 0; i < prev.size(); i++) prev[i] = F1.mvKeysUn[i].pt;  // src/Tracking.cc:573-575
                std::vector<int> m12(F1.mvKeysUn.size(), -1);                            // :577
                ORBmatcher matcher(ratio[c], ori[c] != 0);
                const int n = matcher.SearchForInitialization(F1, F2, prev, m12, window[c]);
                const std::string t = std::to_string(c);
                out.i32("n" + t, n);
                out.vec("m12_" + t, m12);
                out.vec("prev_" + t, prev);
            }
        } else if (mode == "proj") {
            // Tracking::SearchLocalPoints (src/Tracking.cc:1184-1191): ORBmatcher matcher(0.8);
            // SearchByProjection(mCurrentFrame, mvpLocalMapPoints, th) with th 1 / 3 / 5
            Frame F;
            extract(ex, b, "img", W, H, F, out, "f");
            if (b.count("uright")) F.mvuRight = arr<float>(b, "uright");
            const std::vector<uint8_t> inview = arr<uint8_t>(b, "track_in_view"), bad = arr<uint8_t>(b, "is_bad"),
                                       desc = arr<uint8_t>(b, "desc");
            const std::vector<int32_t> level = arr<int32_t>(b, "level"), nobs = arr<int32_t>(b, "n_obs");
            const std::vector<float> vc = arr<float>(b, "view_cos"), px = arr<float>(b, "proj_x"),
                                     py = arr<float>(b, "proj_y"), pxr = arr<float>(b, "proj_xr");
            const std::vector<float> ths = arr<float>(b, "th");
            const int M = (int)level.size();
            std::vector<MapPoint*> pts(M);
            for (int m = 0; m < M; m++) {
                MapPoint* p = new_point(nullptr, &desc[32 * (size_t)m], nobs[m]);
                state_of(p).bad = bad[m] != 0;
                p->mbTrackInView = inview[m] != 0;
                p->mnTrackScaleLevel = level[m];
                p->mTrackViewCos = vc[m];
                p->mTrackProjX = px[m];
                p->mTrackProjY = py[m];
                p->mTrackProjXR = pxr[m];
                pts[m] = p;
            }
            MapPoint* c0 = new_point(nullptr, nullptr, 0);
            MapPoint* c1 = new_point(nullptr, nullptr, 3);
            const std::vector<int32_t> claim = arr<int32_t>(b, "claim");
            for (size_t c = 0; c < ths.size(); c++) {
                preclaim(F, claim, c0, c1);
                ORBmatcher matcher(0.8f);
                const int n = matcher.SearchByProjection(F, pts, ths[c]);
                const std::string t = std::to_string(c);
                out.i32("n" + t, n);
                out.vec("owner_" + t, owners(F, pts, c0, c1));
            }
        } else if (mode == "last") {
            // Tracking::TrackWithMotionModel (src/Tracking.cc:869-891): ORBmatcher matcher(0.9, true);
            // SearchByProjection(mCurrentFrame, mLastFrame, th, bMono), th = 15 (stereo) or 7, then 2 th
            Frame Last, Cur;
            extract(ex, b, "img_last", W, H, Last, out, "last");
            extract(ex, b, "img_cur", W, H, Cur, out, "cur");
            const int mono = P[3], ori = P[4];
            Last.mTcw = pose(b, "Tcw_last");
            Cur.mTcw = pose(b, "Tcw_cur");
            const std::vector<float> bf = arr<float>(b, "mbf_mb");
            Last.mbf = Cur.mbf = bf[0];
            Last.mb = Cur.mb = bf[1];
            if (b.count("uright")) Cur.mvuRight = arr<float>(b, "uright");
            const std::vector<uint8_t> has = arr<uint8_t>(b, "has_mp"), outl = arr<uint8_t>(b, "outlier"),
                                       desc = arr<uint8_t>(b, "desc");
            const std::vector<float> pos = arr<float>(b, "pos");
            const std::vector<int32_t> nobs = arr<int32_t>(b, "n_obs");
            if ((int)has.size() != Last.N) throw std::runtime_error("last-frame points do not match its keypoints");
            for (int i = 0; i < Last.N; i++) {
                Last.mvbOutlier[i] = outl[i] != 0;
                Last.mvpMapPoints[i] = has[i] ? new_point(&pos[3 * (size_t)i], &desc[32 * (size_t)i], nobs[i]) : nullptr;
            }
            MapPoint* c0 = new_point(nullptr, nullptr, 0);
            MapPoint* c1 = new_point(nullptr, nullptr, 2);
            const std::vector<int32_t> claim = arr<int32_t>(b, "claim");
            const std::vector<float> ths = arr<float>(b, "th");
            for (size_t c = 0; c < ths.size(); c++) {
                preclaim(Cur, claim, c0, c1);
                ORBmatcher matcher(0.9f, ori != 0);
                const int n = matcher.SearchByProjection(Cur, Last, ths[c], mono != 0);
                const std::string t = std::to_string(c);
                out.i32("n" + t, n);
                out.vec("owner_" + t, owners(Cur, Last.mvpMapPoints, c0, c1));
            }
        } else if (mode == "kf") {
            // Tracking::Relocalization (src/Tracking.cc:1433,1467): SearchByProjection(mCurrentFrame,
            // vpCandidateKFs[i], sFound, 10, 100) and (.., 3, 64)
            Frame KFF, Cur;
            extract(ex, b, "img_kf", W, H, KFF, out, "kf");
            extract(ex, b, "img_cur", W, H, Cur, out, "cur");
            const int ori = P[3];
            Cur.mTcw = pose(b, "Tcw_cur");
            const std::vector<float> bf = arr<float>(b, "mbf_mb");
            Cur.mbf = bf[0];
            Cur.mb = bf[1];
            const std::vector<uint8_t> valid = arr<uint8_t>(b, "valid"), desc = arr<uint8_t>(b, "desc");
            const std::vector<float> pos = arr<float>(b, "pos"), mx = arr<float>(b, "max_dist"),
                                     mn = arr<float>(b, "min_dist");
            if ((int)valid.size() != KFF.N) throw std::runtime_error("keyframe points do not match its keypoints");
            KeyFrame kf{KFF.mvKeysUn};
            std::vector<MapPoint*> vp(KFF.N, nullptr);
            std::set<MapPoint*> found;
            for (int i = 0; i < KFF.N; i++) {
                // an invalid point takes one of the three forms the reference skips (:1490): no point, a bad one, or
                // one already found
                const int form = i % 3;
                if (!valid[i] && form == 0) continue;
                MapPoint* p = new_point(&pos[3 * (size_t)i], &desc[32 * (size_t)i], 2);
                state_of(p).max_dist = mx[i];
                state_of(p).min_dist = mn[i];
                if (!valid[i] && form == 1) state_of(p).bad = true;
                if (!valid[i] && form == 2) found.insert(p);
                vp[i] = p;
            }
            set_map_point_matches(&kf, vp);
            MapPoint* c0 = new_point(nullptr, nullptr, 1);
            const std::vector<int32_t> claim = arr<int32_t>(b, "claim");
            const std::vector<float> ths = arr<float>(b, "th");
            const std::vector<int32_t> orbd = arr<int32_t>(b, "orbdist");
            for (size_t c = 0; c < ths.size(); c++) {
                preclaim(Cur, claim, c0, c0);
                ORBmatcher matcher(0.9f, ori != 0);
                const int n = matcher.SearchByProjection(Cur, &kf, found, ths[c], orbd[c]);
                const std::string t = std::to_string(c);
                out.i32("n" + t, n);
                out.vec("owner_" + t, owners(Cur, vp, c0, c0));
            }
        } else if (mode == "stereo") {
            // Frame's stereo constructor (src/Frame.cc:78-81 extracts left and right with their own extractors, then
            // ComputeStereoMatches, :105)
            ORBextractor exR(nfeat, 1.2f, 8, 20, 7);
            Frame L, R;
            extract(ex, b, "left", W, H, L, out, "left");
            extract(exR, b, "right", W, H, R, out, "right");
            const std::vector<float> bf = arr<float>(b, "mbf_mb");
            L.mpORBextractorRight = &exR;
            L.mDescriptorsRight = R.mDescriptors;
            L.mbf = bf[0];
            L.mb = bf[1];
            L.ComputeStereoMatches();
            out.vec("uright", L.mvuRight);
            out.vec("depth", L.mvDepth);
        } else {
            std::cerr << "unknown mode " << mode << "\n";
            return 2;
        }
        return out.f.good() ? 0 : 1;
    } catch (const std::exception& e) {
        std::cerr << "run_matchers: " << e.what() << "\n";
        return 1;
    }
}
