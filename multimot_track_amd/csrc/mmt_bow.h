// multimot_track_amd/csrc/mmt_bow.h -- the vocabulary-driven part of the path:
// DBoW2's ORB vocabulary (loadFromTextFile, transform, L1 / L2 score), and the device records of
// the BoW matchers that need it.
//
// Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259 (transform), 1338-1424
// (loadFromTextFile); BowVector.cpp:34-84; FeatureVector.cpp:31-45; ScoringObject.cpp (L1 / L2);
// ORBmatcher.cc:1032-1198 (SearchForTriangulation), 2104-2231 (SearchByProjection(Frame&,
// KeyFrame*, set<MapPoint*>, th, ORBdist)).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mmt.h"
#include "mmt_match.h"

namespace mmt {

// DBoW2::BowVector (std::map<WordId, WordValue>) and FeatureVector (std::map<NodeId,
// std::vector<unsigned int>>) as flat arrays (words / nodes ascending)
struct BowVecH {
  std::vector<uint32_t> word;
  std::vector<double> value;
};
struct FeatVecH {
  std::vector<uint32_t> node;
  std::vector<int> start{0};
  std::vector<int> feat;
};

// The vocabulary tree on the device: node descriptors and the children in CSR (file order)
struct VocDev {
  const uint8_t* desc;      // n_nodes x 32
  const int* child_start;   // n_nodes + 1
  const int* child;         // n_nodes - 1
  const int* word_of;       // n_nodes (-1: inner node)
  const double* weight;     // n_nodes
  int n_nodes;
  int L;
};

class Vocabulary {
 public:
  ~Vocabulary();
  // TemplatedVocabulary::loadFromTextFile; throws ArgError with the reason
  void load_text(const char* path);
  // the tree on the device (once, on the first transform)
  void upload();
  bool empty() const { return words_ == 0; }
  int k = 0, L = 0, scoring = 0, weighting = 0;
  int n_nodes() const { return (int)word_of_.size(); }
  int n_words() const { return words_; }
  // transform(features, BowVector, FeatureVector, levelsup) from the per-feature outputs of
  // k_bow_transform (word, weight, node at level L - levelsup), in feature order
  void build(const uint32_t* word, const double* w, const uint32_t* node, int n, BowVecH& v,
             FeatVecH& fv) const;
  // score(v1, v2): L1Scoring / L2Scoring
  double score(const BowVecH& a, const BowVecH& b) const;
  VocDev dev{};

 private:
  std::vector<uint8_t> desc_;
  std::vector<int> child_start_, child_, word_of_;
  std::vector<double> weight_;
  int words_ = 0;
  void* d_block_ = nullptr;
};

// k_bow_transform: per descriptor (n x 32, device) its word, weight and node id at level
// L - levelsup (TemplatedVocabulary::transform(feature, id, w, &nid, levelsup))
void launch_bow_transform(const VocDev& v, const uint8_t* desc, int n, int levelsup,
                          uint32_t* word, double* weight, uint32_t* node, hipStream_t st);

// SearchForTriangulation (ORBmatcher(0.6, false), bOnlyStereo false): one query per keyframe-1
// feature without a MapPoint in a vocabulary node both keyframes hold; the query scans keyframe
// 2's features of that node (list [b0, b1) of its pair's feature table).  vbMatched2 is never set
// in the reference, so the queries are independent.
struct SftPair {
  const mmt_kp* k2;
  const uint8_t* d2;
  const float* uR2;
  const int* feat2;        // keyframe 2's FeatureVector features, node by node
  const uint8_t* taken2;   // keyframe 2 key holds a MapPoint
  float F12[9];
  float ex, ey;            // epipole of keyframe 1 in keyframe 2
};
struct SftQuery {
  int pair, idx1, b0, b1;
};
struct SftArgs {
  const mmt_kp* k1;
  const uint8_t* d1;
  const float* uR1;
  const SftPair* pairs;
  const SftQuery* q;
  int nq;
  float scale[kMaxLevels], sigma2[kMaxLevels];
  int* out;  // per query: idx2 or -1
};
void launch_sft(const SftArgs& a, hipStream_t st);

// SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist): per keyframe map point its
// projection, scale prediction and window, then the window's candidates (keys not bound when the
// call starts, level in [predicted - 1, predicted + 1]) as sorted (distance << 20 | position)
// keys; the order-dependent binding, the ORBdist test and the rotation histogram are the host's.
constexpr int kSbpKfCand = 32;
struct alignas(16) SbpKfPoint {
  float Xw[3];
  float min_dist, max_dist;
  int pad[3];
  uint8_t desc[32];  // offset 32: two 16-byte loads
};
struct SbpKfArgs {
  GridFrame C;
  float Tcw[16];
  float th;
  const SbpKfPoint* pts;
  int m;
  const uint8_t* bound;  // C.n: mvpMapPoints[i2] set when the call starts
  uint32_t* cand_key;    // m x kSbpKfCand
  int* cand_idx;
  int* n_cand;           // -1: not projected into the image / outside the distance range
  PointWin* win;         // the window (the host's rescan when every listed key got bound)
};
void launch_sbp_kf(const SbpKfArgs& a, hipStream_t st);

}  // namespace mmt
