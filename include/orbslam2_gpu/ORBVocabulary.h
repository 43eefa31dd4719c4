/*
 * ORBVocabulary.h -- ORB_SLAM2::ORBVocabulary (= DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>,
 * include/ORBVocabulary.h) resident in HBM, with the two DBoW2 containers Frame::ComputeBoW fills.
 *
 * loadFromTextFile follows TemplatedVocabulary::loadFromTextFile (Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h:1338-1420, called at src/System.cc:65); transform follows
 * TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup) (:1127-1256) on the GPU.
 */
#ifndef ORBSLAM2_GPU_ORBVOCABULARY_H
#define ORBSLAM2_GPU_ORBVOCABULARY_H

#include <map>
#include <string>
#include <vector>

#include "Types.h"

namespace DBoW2
{
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
/* Thirdparty/DBoW2/DBoW2/BowVector.h: std::map<WordId, WordValue>. */
class BowVector : public std::map<WordId, WordValue>
{
};
/* Thirdparty/DBoW2/DBoW2/FeatureVector.h: std::map<NodeId, std::vector<unsigned int>>. */
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>>
{
};
}  // namespace DBoW2

namespace ORB_SLAM2
{

class ORBVocabulary
{
public:
    explicit ORBVocabulary(int device = 0);
    ~ORBVocabulary();
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;

    /* false on a malformed or missing file (the reference returns false too, src/System.cc:66-71). */
    bool loadFromTextFile(const std::string& filename);
    /* The same tree from arrays: nodes 1..nn in file order (node 0 is the root). */
    void create(int k, int L, int scoring, int weighting, const std::vector<int>& parent,
                const std::vector<uint8_t>& isLeaf, const std::vector<uint8_t>& desc,
                const std::vector<double>& weight);

    bool empty() const { return mVoc == nullptr; }
    int size() const;  // number of words

    /* transform(features, v, fv, levelsup) for the N x 32 descriptors of a frame, on `ctx`'s stream. */
    void transform(orbgpu_ctx* ctx, const Descriptors& desc, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                   int levelsup) const;

    orbgpu_vocabulary* handle() const { return mVoc; }

private:
    orbgpu_ctx* mCtx = nullptr;  // device + stream the vocabulary lives on
    orbgpu_vocabulary* mVoc = nullptr;
};

}  // namespace ORB_SLAM2

#endif
