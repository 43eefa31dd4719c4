// ORB_SLAM2::ORBVocabulary (DBoW2 TemplatedVocabulary<FORB>) in HBM -- include/orbslam2_gpu/ORBVocabulary.h.
// Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1256 (transform), :1338-1420 (loadFromTextFile),
// src/Frame.cc:395-402 (Frame::ComputeBoW).
#include "orbslam2_gpu/ORBVocabulary.h"

#include "orbslam2_gpu/ORBextractor.h"

namespace ORB_SLAM2
{

ORBVocabulary::ORBVocabulary(int device)
{
    // a small context of its own: the vocabulary's device memory and the stream that uploads it
    mCtx = orbgpu_create(device, 1000, 1.2f, 8, 20, 7);
    if (!mCtx) throw GpuError("ORBVocabulary: orbgpu_create failed (no gfx950 HIP device)");
}

ORBVocabulary::~ORBVocabulary()
{
    if (mVoc) orbgpu_vocabulary_destroy(mVoc);
    if (mCtx) orbgpu_destroy(mCtx);
}

bool ORBVocabulary::loadFromTextFile(const std::string& filename)
{
    orbgpu_vocabulary* v = orbgpu_vocabulary_load_text(mCtx, filename.c_str());
    if (!v) return false;
    if (mVoc) orbgpu_vocabulary_destroy(mVoc);
    mVoc = v;
    return true;
}

void ORBVocabulary::create(int k, int L, int scoring, int weighting, const std::vector<int>& parent,
                           const std::vector<uint8_t>& isLeaf, const std::vector<uint8_t>& desc,
                           const std::vector<double>& weight)
{
    const int nn = (int)parent.size();
    if ((int)isLeaf.size() != nn || (int)weight.size() != nn || (int)desc.size() != 32 * nn)
        throw GpuError("ORBVocabulary::create: inconsistent node arrays");
    orbgpu_vocabulary* v =
        orbgpu_vocabulary_create(mCtx, k, L, scoring, weighting, nn, parent.data(), isLeaf.data(), desc.data(),
                                 weight.data());
    if (!v) throw GpuError(std::string("orbgpu_vocabulary_create failed: ") + orbgpu_last_error(mCtx));
    if (mVoc) orbgpu_vocabulary_destroy(mVoc);
    mVoc = v;
}

int ORBVocabulary::size() const
{
    int k = 0, L = 0, nodes = 0, words = 0;
    if (!mVoc || orbgpu_vocabulary_info(mVoc, &k, &L, &nodes, &words) != ORBGPU_OK) return 0;
    return words;
}

void ORBVocabulary::transform(orbgpu_ctx* ctx, const Descriptors& desc, DBoW2::BowVector& v,
                              DBoW2::FeatureVector& fv, int levelsup) const
{
    v.clear();
    fv.clear();
    if (!mVoc) throw GpuError("ORBVocabulary::transform: vocabulary not loaded");
    const int n = desc.rows;
    if (n == 0) return;  // TemplatedVocabulary::transform on an empty feature vector leaves both empty
    std::vector<int32_t> words(n), nodes(n), nodeOff(n + 1), feats(n);
    std::vector<double> values(n);
    int nw = 0, nnodes = 0;
    orbgpu_throw_if(ctx,
                    orbgpu_compute_bow(ctx, mVoc, desc.data(), n, levelsup, words.data(), values.data(), &nw,
                                       nodes.data(), nodeOff.data(), feats.data(), &nnodes),
                    "orbgpu_compute_bow");
    for (int i = 0; i < nw; ++i) v.emplace_hint(v.end(), (DBoW2::WordId)words[i], values[i]);
    for (int j = 0; j < nnodes; ++j) {
        std::vector<unsigned int>& f = fv[(DBoW2::NodeId)nodes[j]];
        for (int q = nodeOff[j]; q < nodeOff[j + 1]; ++q) f.push_back((unsigned int)feats[q]);
    }
}

}  // namespace ORB_SLAM2
