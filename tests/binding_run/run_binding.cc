// tests/binding_run/run_binding.cc -- executes the drop-in integration/ORBextractor.cc (built against the
// reference's unchanged include/ORBextractor.h and tests/binding_run/cvmini.cc) the way ORB-SLAM2 calls it:
// Frame::ExtractORB -> (*mpORBextractorLeft)(im, cv::Mat(), mvKeys, mDescriptors) (src/Frame.cc:247-253), one frame
// at a time with one long-lived extractor (src/Tracking.cc:119-125).  Test infrastructure
// (tests/test_gpu_binding_run.py compares its output with the CPU oracle).
//
//   run_binding <frames.u8> <W> <H> <pitch> <nframes> <nfeatures> <scaleFactor> <nlevels> <iniTh> <minTh> <out.bin>
//
// frames.u8 holds nframes images of H rows x pitch bytes (W used).  out.bin: the getters (GetLevels,
// GetScaleFactor, then the four per-level tables as float32), then per frame int32 n, n x 28-byte cv::KeyPoint,
// int32 descriptor rows/cols and the rows x 32 descriptor bytes, then the last frame's mvImagePyramid (per level
// int32 rows, cols and the rows x cols bytes).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <vector>

#include "ORBextractor.h"

int main(int argc, char** argv)
{
    if (argc != 12) {
        std::cerr << "usage: run_binding frames W H pitch nframes nfeatures scale nlevels iniTh minTh out\n";
        return 2;
    }
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), pitch = std::atoi(argv[4]), nf = std::atoi(argv[5]);
    std::ifstream in(argv[1], std::ios::binary);
    std::vector<unsigned char> buf((size_t)nf * H * pitch);
    if (!in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)buf.size())) {
        std::cerr << "short input\n";
        return 2;
    }
    ORB_SLAM2::ORBextractor ex(std::atoi(argv[6]), (float)std::atof(argv[7]), std::atoi(argv[8]), std::atoi(argv[9]),
                               std::atoi(argv[10]));
    std::ofstream out(argv[11], std::ios::binary);
    auto put_i = [&](int v) { out.write(reinterpret_cast<const char*>(&v), 4); };
    auto put_fv = [&](const std::vector<float>& v) { out.write(reinterpret_cast<const char*>(v.data()), 4 * v.size()); };
    const int nl = ex.GetLevels();
    const float sf = ex.GetScaleFactor();
    put_i(nl);
    out.write(reinterpret_cast<const char*>(&sf), 4);
    put_fv(ex.GetScaleFactors());
    put_fv(ex.GetInverseScaleFactors());
    put_fv(ex.GetScaleSigmaSquares());
    put_fv(ex.GetInverseScaleSigmaSquares());
    for (int f = 0; f < nf; f++) {
        cv::Mat im(H, W, CV_8UC1, buf.data() + (size_t)f * H * pitch, (size_t)pitch);
        std::vector<cv::KeyPoint> keys;
        cv::Mat desc;
        ex(im, cv::Mat(), keys, desc);  // Frame::ExtractORB (src/Frame.cc:247-253)
        put_i((int)keys.size());
        out.write(reinterpret_cast<const char*>(keys.data()), (std::streamsize)(sizeof(cv::KeyPoint) * keys.size()));
        put_i(desc.rows);
        put_i(desc.cols);
        for (int r = 0; r < desc.rows; r++) out.write(reinterpret_cast<const char*>(desc.data + r * desc.step), desc.cols);
    }
    for (int l = 0; l < nl; l++) {
        const cv::Mat& m = ex.mvImagePyramid[l];
        put_i(m.rows);
        put_i(m.cols);
        for (int r = 0; r < m.rows; r++) out.write(reinterpret_cast<const char*>(m.data + r * m.step), m.cols);
    }
    return out.good() ? 0 : 1;
}
