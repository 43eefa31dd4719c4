// host_parity -- drives the C++ host layer (ORB_SLAM2::ORBextractor / Frame / ORBmatcher / ORBVocabulary
// over liborbgpu.so) the way Tracking.cc drives the reference classes, for the parity tests in
// tests/test_gpu_host_cpp.py.  Inputs and outputs are raw little-endian arrays in a case directory that
// the Python test writes and then compares against the CPU oracle.
//
//   host_parity probe                      -> constructs an ORBextractor; exit 3 with the GpuError text
//                                             when no device is visible (no CPU fallback)
//   host_parity <mode> <case_dir>          -> mode in {mono_init, stereo, rgbd, projection, frustum, bow,
//                                             last_frame, keyframe}
//
// params.txt in the case dir: whitespace-separated `key value` pairs (rows cols nfeatures fx fy cx cy bf
// ndist d0..d4 th nnratio ...).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <algorithm>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "orbslam2_gpu/Frame.h"
#include "orbslam2_gpu/ORBVocabulary.h"
#include "orbslam2_gpu/ORBextractor.h"
#include "orbslam2_gpu/ORBmatcher.h"

using namespace ORB_SLAM2;

namespace
{
std::string gDir;

std::vector<uint8_t> read_bytes(const std::string& name)
{
    std::ifstream f(gDir + "/" + name, std::ios::binary);
    if (!f) throw std::runtime_error("missing input " + name);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

template <class T>
std::vector<T> read_arr(const std::string& name)
{
    const std::vector<uint8_t> b = read_bytes(name);
    std::vector<T> v(b.size() / sizeof(T));
    if (!v.empty()) std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}

template <class T>
void write_arr(const std::string& name, const T* p, size_t n)
{
    std::ofstream f(gDir + "/" + name, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

template <class T>
void write_vec(const std::string& name, const std::vector<T>& v)
{
    write_arr(name, v.data(), v.size());
}

std::map<std::string, double> read_params()
{
    std::ifstream f(gDir + "/params.txt");
    std::map<std::string, double> p;
    std::string k;
    double v;
    while (f >> k >> v) p[k] = v;
    return p;
}

struct Setup {
    std::map<std::string, double> p;
    int rows, cols, nf;
    CameraMatrix K;
    DistCoef dist;
    float bf;
    double get(const char* k, double d) const
    {
        auto it = p.find(k);
        return it == p.end() ? d : it->second;
    }
};

Setup setup()
{
    Setup s;
    s.p = read_params();
    s.rows = (int)s.get("rows", 0);
    s.cols = (int)s.get("cols", 0);
    s.nf = (int)s.get("nfeatures", 1000);
    s.K.fx = (float)s.get("fx", 500);
    s.K.fy = (float)s.get("fy", 500);
    s.K.cx = (float)s.get("cx", s.cols / 2.0);
    s.K.cy = (float)s.get("cy", s.rows / 2.0);
    const int nd = (int)s.get("ndist", 0);
    for (int i = 0; i < nd; ++i) s.dist.push_back((float)s.get(("d" + std::to_string(i)).c_str(), 0));
    s.bf = (float)s.get("bf", 0);
    Frame::mbInitialComputations = true;  // each case is its own calibration
    return s;
}

ImageU8 load_image(const std::string& name, std::vector<uint8_t>& keep, int rows, int cols)
{
    keep = read_bytes(name);
    if ((int)keep.size() != rows * cols) throw std::runtime_error("image size mismatch: " + name);
    return ImageU8::view(keep.data(), rows, cols, (size_t)cols);
}

void write_frame(const std::string& tag, const Frame& F)
{
    write_vec(tag + "_kps.bin", F.mvKeys);
    write_vec(tag + "_kpsun.bin", F.mvKeysUn);
    write_arr(tag + "_desc.bin", F.mDescriptors.data(), F.mDescriptors.buf.size());
    write_vec(tag + "_uright.bin", F.mvuRight);
    write_vec(tag + "_depth.bin", F.mvDepth);
    const float b[6] = {Frame::mnMinX, Frame::mnMinY, Frame::mnMaxX, Frame::mnMaxY, Frame::mfGridElementWidthInv,
                        Frame::mfGridElementHeightInv};
    write_arr(tag + "_bounds.bin", b, 6);
}

int mode_mono_init()
{
    Setup s = setup();
    ORBextractor ex(s.nf, 1.2f, 8, 20, 7);
    // Tracking::MonocularInitialization matches against the initial frame with a 2x-feature extractor
    // (src/Tracking.cc:125); one extractor serves both frames here, as the test sets nfeatures itself.
    std::vector<uint8_t> b1, b2;
    ImageU8 im1 = load_image("img1.u8", b1, s.rows, s.cols), im2 = load_image("img2.u8", b2, s.rows, s.cols);
    Frame F1(im1, 0.0, &ex, nullptr, s.K, s.dist, s.bf, 40.f);
    write_frame("f1", F1);
    Frame F2(im2, 0.033, &ex, nullptr, s.K, s.dist, s.bf, 40.f);
    write_frame("f2", F2);
    // pyramid of the last call (mvImagePyramid), level by level
    for (int l = 0; l < ex.GetLevels(); ++l) {
        const ImageU8& L = ex.mvImagePyramid[l];
        const int dims[2] = {L.rows, L.cols};
        write_arr("pyr" + std::to_string(l) + "_dims.bin", dims, 2);
        write_arr("pyr" + std::to_string(l) + ".u8", L.data, (size_t)L.rows * L.cols);
    }
    std::vector<Point2f> prev(F1.mvKeysUn.size());  // src/Tracking.cc:573-575
    for (size_t i = 0; i < F1.mvKeysUn.size(); ++i) prev[i] = F1.mvKeysUn[i].pt;
    std::vector<int> m12;
    ORBmatcher matcher(0.9f, true);
    const int nm = matcher.SearchForInitialization(F1, F2, prev, m12, (int)s.get("window", 100));
    write_vec("m12.bin", m12);
    write_vec("prev.bin", prev);
    write_arr("nmatches.bin", &nm, 1);
    return 0;
}

int mode_stereo()
{
    Setup s = setup();
    ORBextractor exL(s.nf, 1.2f, 8, 20, 7), exR(s.nf, 1.2f, 8, 20, 7);
    exL.SetPyramidDownload(false);  // the GPU stereo matcher reads the device pyramids
    exR.SetPyramidDownload(false);
    std::vector<uint8_t> bl, br;
    ImageU8 L = load_image("left.u8", bl, s.rows, s.cols), R = load_image("right.u8", br, s.rows, s.cols);
    Frame F(L, R, 0.0, &exL, &exR, nullptr, s.K, s.dist, s.bf, 40.f);
    write_frame("f", F);
    write_vec("f_kpsright.bin", F.mvKeysRight);
    return 0;
}

int mode_rgbd()
{
    Setup s = setup();
    ORBextractor ex(s.nf, 1.2f, 8, 20, 7);
    std::vector<uint8_t> bg;
    ImageU8 G = load_image("gray.u8", bg, s.rows, s.cols);
    const std::vector<uint16_t> dep = read_arr<uint16_t>("depth.u16");
    DepthImage D;
    D.data = dep.data();
    D.rows = s.rows;
    D.cols = s.cols;
    D.step = (size_t)s.cols * 2;
    D.is_u16 = true;
    D.factor = (float)s.get("depth_factor", 1.0 / 5000.0);
    Frame F(G, D, 0.0, &ex, nullptr, s.K, s.dist, s.bf, 40.f);
    write_frame("f", F);
    return 0;
}

// map points: SoA files written by the test (mp_*.bin)
std::vector<MapPoint*> load_mappoints(std::vector<std::unique_ptr<MapPoint>>& own)
{
    const auto inView = read_arr<uint8_t>("mp_track_in_view.bin");
    const auto bad = read_arr<uint8_t>("mp_is_bad.bin");
    const auto level = read_arr<int32_t>("mp_level.bin");
    const auto vc = read_arr<float>("mp_view_cos.bin");
    const auto px = read_arr<float>("mp_proj_x.bin");
    const auto py = read_arr<float>("mp_proj_y.bin");
    const auto pxr = read_arr<float>("mp_proj_xr.bin");
    const auto nobs = read_arr<int32_t>("mp_n_obs.bin");
    const auto desc = read_arr<uint8_t>("mp_desc.bin");
    std::vector<MapPoint*> v;
    for (size_t m = 0; m < level.size(); ++m) {
        own.emplace_back(new MapPoint());
        MapPoint* p = own.back().get();
        p->mbTrackInView = inView[m] != 0;
        p->SetBadFlag(bad[m] != 0);
        p->mnTrackScaleLevel = level[m];
        p->mTrackViewCos = vc[m];
        p->mTrackProjX = px[m];
        p->mTrackProjY = py[m];
        p->mTrackProjXR = pxr[m];
        p->SetObservations(nobs[m]);
        p->SetDescriptor(&desc[32 * m]);
        v.push_back(p);
    }
    return v;
}

int mode_projection()
{
    Setup s = setup();
    ORBextractor ex(s.nf, 1.2f, 8, 20, 7);
    ex.SetPyramidDownload(false);
    std::vector<uint8_t> bi;
    ImageU8 im = load_image("img.u8", bi, s.rows, s.cols);
    Frame F(im, 0.0, &ex, nullptr, s.K, s.dist, s.bf, 40.f);
    write_frame("f", F);
    std::vector<std::unique_ptr<MapPoint>> own;
    std::vector<MapPoint*> mps = load_mappoints(own);
    std::map<MapPoint*, int> index;
    for (size_t m = 0; m < mps.size(); ++m) index[mps[m]] = (int)m;
    ORBmatcher matcher((float)s.get("nnratio", 0.8), true);
    const int nm = matcher.SearchByProjection(F, mps, (float)s.get("th", 3.0));
    std::vector<int32_t> owner(F.N, -1);
    for (int i = 0; i < F.N; ++i)
        if (F.mvpMapPoints[i]) owner[i] = index[F.mvpMapPoints[i]];
    write_vec("owner.bin", owner);
    write_arr("nmatches.bin", &nm, 1);
    return 0;
}

int mode_frustum()
{
    Setup s = setup();
    ORBextractor ex(s.nf, 1.2f, 8, 20, 7);
    ex.SetPyramidDownload(false);
    std::vector<uint8_t> bi;
    ImageU8 im = load_image("img.u8", bi, s.rows, s.cols);
    Frame F(im, 0.0, &ex, nullptr, s.K, s.dist, s.bf, 40.f);
    Pose T;
    const auto Tcw = read_arr<float>("pose.f32");
    std::memcpy(T.T, Tcw.data(), sizeof(T.T));
    F.SetPose(T);
    const auto Ow = F.GetCameraCenter();
    write_arr("ow.bin", Ow.data(), 3);
    const auto pos = read_arr<float>("geom_pos.bin");
    const auto nrm = read_arr<float>("geom_normal.bin");
    const auto mx = read_arr<float>("geom_max.bin");
    const auto mn = read_arr<float>("geom_min.bin");
    std::vector<std::unique_ptr<MapPoint>> own;
    std::vector<MapPoint*> mps;
    for (size_t m = 0; m < mx.size(); ++m) {
        own.emplace_back(new MapPoint());
        own.back()->SetWorldPos(&pos[3 * m]);
        own.back()->SetNormal(&nrm[3 * m]);
        own.back()->SetDistances(mn[m], mx[m]);
        mps.push_back(own.back().get());
    }
    const float cosLimit = (float)s.get("cos_limit", 0.5);
    const int nin = F.isInFrustum(mps, cosLimit);
    // the per-point form on the first few points must agree with the batched form
    for (size_t m = 0; m < std::min<size_t>(mps.size(), 8); ++m) {
        const bool was = mps[m]->mbTrackInView;
        const float u = mps[m]->mTrackProjX;
        if (F.isInFrustum(mps[m], cosLimit) != was || (was && mps[m]->mTrackProjX != u)) {
            std::cerr << "per-point isInFrustum disagrees with the batched form at " << m << "\n";
            return 4;
        }
    }
    std::vector<uint8_t> inView(mps.size());
    std::vector<float> px(mps.size()), py(mps.size()), pxr(mps.size()), vc(mps.size());
    std::vector<int32_t> level(mps.size());
    for (size_t m = 0; m < mps.size(); ++m) {
        inView[m] = mps[m]->mbTrackInView;
        px[m] = mps[m]->mTrackProjX;
        py[m] = mps[m]->mTrackProjY;
        pxr[m] = mps[m]->mTrackProjXR;
        vc[m] = mps[m]->mTrackViewCos;
        level[m] = mps[m]->mnTrackScaleLevel;
    }
    write_vec("in_view.bin", inView);
    write_vec("proj_x.bin", px);
    write_vec("proj_y.bin", py);
    write_vec("proj_xr.bin", pxr);
    write_vec("view_cos.bin", vc);
    write_vec("level.bin", level);
    write_arr("nin.bin", &nin, 1);
    return 0;
}

int mode_bow()
{
    Setup s = setup();
    ORBextractor ex(s.nf, 1.2f, 8, 20, 7);
    ex.SetPyramidDownload(false);
    ORBVocabulary voc;
    if (!voc.loadFromTextFile(gDir + "/voc.txt")) {
        std::cerr << "vocabulary load failed\n";
        return 5;
    }
    std::vector<uint8_t> bi;
    ImageU8 im = load_image("img.u8", bi, s.rows, s.cols);
    Frame F(im, 0.0, &ex, &voc, s.K, s.dist, s.bf, 40.f);
    write_frame("f", F);
    F.ComputeBoW();
    std::vector<int32_t> words;
    std::vector<double> values;
    for (const auto& kv : F.mBowVec) {
        words.push_back((int32_t)kv.first);
        values.push_back(kv.second);
    }
    std::vector<int32_t> nodes, off{0}, feats;
    for (const auto& kv : F.mFeatVec) {
        nodes.push_back((int32_t)kv.first);
        for (unsigned f : kv.second) feats.push_back((int32_t)f);
        off.push_back((int32_t)feats.size());
    }
    write_vec("bow_words.bin", words);
    write_vec("bow_values.bin", values);
    write_vec("fv_nodes.bin", nodes);
    write_vec("fv_off.bin", off);
    write_vec("fv_feats.bin", feats);
    return 0;
}
// two mono frames (last, current) with poses; LastFrame map points from lf_* files; optional current-frame
// mvuRight and pre-existing claims (claim.u8: 1 = claimed by a foreign point, claim_obs.i32: its Observations())
struct TwoFrames {
    std::unique_ptr<ORBextractor> ex;
    std::unique_ptr<Frame> last, cur;
    std::vector<uint8_t> b1, b2;
    std::vector<std::unique_ptr<MapPoint>> own;
};

void load_two_frames(TwoFrames& t, const Setup& s)
{
    t.ex.reset(new ORBextractor(s.nf, 1.2f, 8, 20, 7));
    t.ex->SetPyramidDownload(false);
    ImageU8 i1 = load_image("img_last.u8", t.b1, s.rows, s.cols), i2 = load_image("img_cur.u8", t.b2, s.rows, s.cols);
    t.last.reset(new Frame(i1, 0.0, t.ex.get(), nullptr, s.K, s.dist, s.bf, 40.f));
    t.cur.reset(new Frame(i2, 0.033, t.ex.get(), nullptr, s.K, s.dist, s.bf, 40.f));
    Pose P;
    const auto Tl = read_arr<float>("pose_last.f32");
    std::memcpy(P.T, Tl.data(), sizeof(P.T));
    t.last->SetPose(P);
    const auto Tc = read_arr<float>("pose_cur.f32");
    std::memcpy(P.T, Tc.data(), sizeof(P.T));
    t.cur->SetPose(P);
    const auto ow = t.cur->GetCameraCenter();
    write_arr("ow_cur.bin", ow.data(), 3);
    const auto owl = t.last->GetCameraCenter();
    write_arr("ow_last.bin", owl.data(), 3);
    write_frame("last", *t.last);
    write_frame("cur", *t.cur);
    std::ifstream ur(gDir + "/uright.f32", std::ios::binary);
    if (ur) t.cur->mvuRight = read_arr<float>("uright.f32");
    const auto claim = read_arr<uint8_t>("claim.u8");
    const auto claimObs = read_arr<int32_t>("claim_obs.i32");
    for (int i = 0; i < t.cur->N && i < (int)claim.size(); ++i)
        if (claim[i]) {
            t.own.emplace_back(new MapPoint());
            t.own.back()->SetObservations(claimObs[i]);
            t.cur->mvpMapPoints[i] = t.own.back().get();
        }
}

// current-frame ownership as indices: -1 NULL, j for the j-th candidate point, `foreign` for a pre-claim
void write_owner(const Frame& F, const std::vector<MapPoint*>& cands, int foreign)
{
    std::map<MapPoint*, int> index;
    for (size_t j = 0; j < cands.size(); ++j)
        if (cands[j]) index[cands[j]] = (int)j;
    std::vector<int32_t> owner(F.N, -1);
    for (int i = 0; i < F.N; ++i) {
        MapPoint* p = F.mvpMapPoints[i];
        if (!p) continue;
        auto it = index.find(p);
        owner[i] = it == index.end() ? foreign : it->second;
    }
    write_vec("owner.bin", owner);
}

int mode_last_frame()
{
    Setup s = setup();
    TwoFrames t;
    load_two_frames(t, s);
    Frame& L = *t.last;
    const auto hasMp = read_arr<uint8_t>("lf_has_mp.bin");
    const auto outl = read_arr<uint8_t>("lf_outlier.bin");
    const auto pos = read_arr<float>("lf_pos.bin");
    const auto nobs = read_arr<int32_t>("lf_n_obs.bin");
    const auto desc = read_arr<uint8_t>("lf_desc.bin");
    if ((int)hasMp.size() != L.N) throw std::runtime_error("lf arrays do not match LastFrame.N");
    for (int i = 0; i < L.N; ++i) {
        L.mvbOutlier[i] = outl[i] != 0;
        if (!hasMp[i]) continue;
        t.own.emplace_back(new MapPoint());
        MapPoint* p = t.own.back().get();
        p->SetWorldPos(&pos[3 * i]);
        p->SetObservations(nobs[i]);
        p->SetDescriptor(&desc[32 * i]);
        L.mvpMapPoints[i] = p;
    }
    ORBmatcher matcher(0.9f, s.get("check_ori", 1) != 0);
    const int nm = matcher.SearchByProjection(*t.cur, L, (float)s.get("th", 7.0), s.get("mono", 1) != 0);
    write_owner(*t.cur, L.mvpMapPoints, L.N);
    write_arr("nmatches.bin", &nm, 1);
    return 0;
}

int mode_keyframe()
{
    Setup s = setup();
    TwoFrames t;
    load_two_frames(t, s);
    const auto valid = read_arr<uint8_t>("kf_valid.bin");  // 0 = NULL, 1 = valid, 2 = bad, 3 = already found
    const auto pos = read_arr<float>("kf_pos.bin");
    const auto mx = read_arr<float>("kf_max.bin");
    const auto mn = read_arr<float>("kf_min.bin");
    const auto desc = read_arr<uint8_t>("kf_desc.bin");
    std::vector<MapPoint*> mps(valid.size(), nullptr);
    std::set<MapPoint*> already;
    for (size_t i = 0; i < valid.size(); ++i) {
        if (valid[i] == 0) continue;
        t.own.emplace_back(new MapPoint());
        MapPoint* p = t.own.back().get();
        p->SetWorldPos(&pos[3 * i]);
        p->SetDistances(mn[i], mx[i]);
        p->SetDescriptor(&desc[32 * i]);
        p->SetObservations(2);
        if (valid[i] == 2) p->SetBadFlag();
        if (valid[i] == 3) already.insert(p);
        mps[i] = p;
    }
    KeyFrame kf(t.last->mvKeysUn, mps);
    ORBmatcher matcher(0.9f, s.get("check_ori", 1) != 0);
    const int nm = matcher.SearchByProjection(*t.cur, &kf, already, (float)s.get("th", 10.0),
                                              (int)s.get("orbdist", 100));
    write_owner(*t.cur, mps, (int)mps.size());
    write_arr("nmatches.bin", &nm, 1);
    return 0;
}
}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::cerr << "usage: host_parity probe | <mode> <case_dir>\n";
        return 2;
    }
    const std::string mode = argv[1];
    try {
        if (mode == "probe") {
            ORBextractor ex(1000, 1.2f, 8, 20, 7);
            std::cout << "device ok, levels " << ex.GetLevels() << "\n";
            return 0;
        }
        if (argc < 3) return 2;
        gDir = argv[2];
        if (mode == "mono_init") return mode_mono_init();
        if (mode == "stereo") return mode_stereo();
        if (mode == "rgbd") return mode_rgbd();
        if (mode == "projection") return mode_projection();
        if (mode == "frustum") return mode_frustum();
        if (mode == "bow") return mode_bow();
        if (mode == "last_frame") return mode_last_frame();
        if (mode == "keyframe") return mode_keyframe();
        std::cerr << "unknown mode " << mode << "\n";
        return 2;
    } catch (const GpuError& e) {
        std::cerr << "GpuError: " << e.what() << "\n";
        return 3;
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
}
