// multimot_track_amd/csrc/mmt_bow.hip -- DBoW2 vocabulary (host tree + device transform) and
// the SearchForTriangulation kernel (see mmt_bow.h).
//
// k_bow_transform: one thread per descriptor walks the tree from the root, level after level:
// the Hamming distances to the node's children (their descriptors in a node-major table, two
// 16-byte loads each, v_bcnt on the XOR), the first smallest kept (DBoW2's strict `<`), until a
// node without children.  The tree of a 10^6-word ORBvoc.txt is 1.1 M nodes x 32 B = 35 MB: the
// upper levels stay in L2, the leaf level is one scattered 32-byte read per level per feature.
// Every branch depends on the previous one, so the kernel is latency-bound (a 6-level descent).
//
// k_sft: one thread per SearchForTriangulation query (a keyframe-1 feature against the features of
// its vocabulary node in keyframe 2): the descriptor distances, the epipole test for mono pairs
// and CheckDistEpipolarLine in float in the reference's operation order (-ffp-contract=off).

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

#include "mmt_bow.h"
#include "mmt_internal.h"

namespace mmt {

// ------------------------------------------------------------------ vocabulary (host)
Vocabulary::~Vocabulary() {
  if (d_block_) (void)hipFree(d_block_);
}

void Vocabulary::load_text(const char* path) {
  std::ifstream f(path);
  if (!f.is_open()) throw ArgError(std::string("cannot open vocabulary ") + path);
  std::string s;
  std::getline(f, s);
  std::stringstream ss;
  ss << s;
  int n1 = -1, n2 = -1;
  k = -1;
  L = -1;
  ss >> k;
  ss >> L;
  ss >> n1;
  ss >> n2;
  // TemplatedVocabulary.h:1359
  if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3)
    throw ArgError("Vocabulary loading failure: This is not a correct text file!");
  if (n1 > 1) throw ArgError("vocabulary: only the L1 / L2 norm scorings are supported");
  scoring = n1;
  weighting = n2;
  std::vector<int> parent{-1};
  std::vector<std::vector<int>> children(1);
  std::vector<uint8_t> leaf{0};
  desc_.assign(32, 0);
  word_of_.assign(1, -1);
  weight_.assign(1, 0.0);
  words_ = 0;
  while (!f.eof()) {
    std::string snode;
    std::getline(f, snode);
    // an empty line (the one after a trailing newline) is skipped: the reference links it to an
    // uninitialised parent (pinned, oracle/oracle_bow.h)
    if (snode.find_first_not_of(" \t\r") == std::string::npos) continue;
    std::stringstream ssnode;
    ssnode << snode;
    const int nid = (int)parent.size();
    int pid = -1;
    ssnode >> pid;
    if (pid < 0 || pid >= nid) throw ArgError("vocabulary node " + std::to_string(nid) + ": bad parent");
    parent.push_back(pid);
    children[pid].push_back(nid);
    children.emplace_back();
    int nIsLeaf = 0;
    ssnode >> nIsLeaf;
    std::stringstream ssd;
    for (int iD = 0; iD < 32; iD++) {
      std::string e;
      ssnode >> e;
      ssd << e << " ";
    }
    uint8_t d[32] = {0};  // FORB::fromString: a byte is written only when its integer parses
    {
      std::stringstream sd(ssd.str());
      for (int i = 0; i < 32; i++) {
        int n;
        sd >> n;
        if (!sd.fail()) d[i] = (uint8_t)n;
      }
    }
    desc_.insert(desc_.end(), d, d + 32);
    double w = 0;
    ssnode >> w;
    weight_.push_back(w);
    leaf.push_back(nIsLeaf > 0);
    word_of_.push_back(nIsLeaf > 0 ? words_++ : -1);
  }
  for (size_t n = 1; n < parent.size(); n++)
    if (children[n].empty() != (leaf[n] != 0))
      throw ArgError("vocabulary node " + std::to_string(n) + ": leaf flag and children disagree");
  child_start_.assign(1, 0);
  child_.clear();
  for (const auto& c : children) {
    child_.insert(child_.end(), c.begin(), c.end());
    child_start_.push_back((int)child_.size());
  }
  if (d_block_) {
    (void)hipFree(d_block_);
    d_block_ = nullptr;
  }
}

void Vocabulary::upload() {
  if (d_block_) return;
  const size_t nn = word_of_.size();
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_desc = 0, o_cs = al(32 * nn), o_c = o_cs + al(4 * (nn + 1)),
               o_w = o_c + al(4 * std::max<size_t>(child_.size(), 1)), o_wt = o_w + al(4 * nn),
               tot = o_wt + al(8 * nn);
  MMT_HIP(hipMalloc(&d_block_, tot));
  uint8_t* b = (uint8_t*)d_block_;
  MMT_HIP(hipMemcpy(b + o_desc, desc_.data(), 32 * nn, hipMemcpyHostToDevice));
  MMT_HIP(hipMemcpy(b + o_cs, child_start_.data(), 4 * (nn + 1), hipMemcpyHostToDevice));
  if (!child_.empty())
    MMT_HIP(hipMemcpy(b + o_c, child_.data(), 4 * child_.size(), hipMemcpyHostToDevice));
  MMT_HIP(hipMemcpy(b + o_w, word_of_.data(), 4 * nn, hipMemcpyHostToDevice));
  MMT_HIP(hipMemcpy(b + o_wt, weight_.data(), 8 * nn, hipMemcpyHostToDevice));
  dev.desc = b + o_desc;
  dev.child_start = (const int*)(b + o_cs);
  dev.child = (const int*)(b + o_c);
  dev.word_of = (const int*)(b + o_w);
  dev.weight = (const double*)(b + o_wt);
  dev.n_nodes = (int)nn;
  dev.L = L;
}

// transform(features, v, fv, levelsup) (TemplatedVocabulary.h:1127-1194) from the per-feature
// results, in feature order: the weights summed in that order (addWeight) or kept once
// (addIfNotExist), then BowVector::normalize (every scoring kept here normalises: L1 or L2)
void Vocabulary::build(const uint32_t* word, const double* w, const uint32_t* node, int n,
                       BowVecH& v, FeatVecH& fv) const {
  v.word.clear();
  v.value.clear();
  fv.node.clear();
  fv.start.assign(1, 0);
  fv.feat.clear();
  if (empty()) return;
  const bool add = weighting == 0 || weighting == 1;
  // features by (word, feature) and by (node, feature): a word's weights are then added in feature
  // order and a node's features listed in feature order, as the map insertions of the reference do
  std::vector<uint64_t> kw, kn;
  kw.reserve(n);
  kn.reserve(n);
  for (int i = 0; i < n; i++) {
    if (!(w[i] > 0)) continue;
    kw.push_back(((uint64_t)word[i] << 32) | (uint32_t)i);
    kn.push_back(((uint64_t)node[i] << 32) | (uint32_t)i);
  }
  std::sort(kw.begin(), kw.end());
  std::sort(kn.begin(), kn.end());
  for (size_t k = 0; k < kw.size(); k++) {
    const uint32_t id = (uint32_t)(kw[k] >> 32);
    const double x = w[(uint32_t)kw[k]];
    if (!v.word.empty() && v.word.back() == id) {
      if (add) v.value.back() += x;
    } else {
      v.word.push_back(id);
      v.value.push_back(x);
    }
  }
  for (size_t k = 0; k < kn.size(); k++) {
    const uint32_t nid = (uint32_t)(kn[k] >> 32);
    if (fv.node.empty() || fv.node.back() != nid) {
      if (!fv.node.empty()) fv.start.push_back((int)fv.feat.size());
      fv.node.push_back(nid);
    }
    fv.feat.push_back((int)(uint32_t)kn[k]);
  }
  if (!fv.node.empty()) fv.start.push_back((int)fv.feat.size());
  double norm = 0.0;
  if (scoring != 1) {
    for (double x : v.value) norm += std::fabs(x);
  } else {
    for (double x : v.value) norm += x * x;
    norm = std::sqrt(norm);
  }
  if (norm > 0.0)
    for (double& x : v.value) x /= norm;
}

double Vocabulary::score(const BowVecH& a, const BowVecH& b) const {
  size_t i = 0, j = 0;
  double s = 0;
  auto jump = [](const std::vector<uint32_t>& v, uint32_t id) {
    return (size_t)(std::lower_bound(v.begin(), v.end(), id) - v.begin());
  };
  if (scoring == 1) {  // L2Scoring
    while (i < a.word.size() && j < b.word.size()) {
      if (a.word[i] == b.word[j]) {
        s += a.value[i] * b.value[j];
        i++;
        j++;
      } else if (a.word[i] < b.word[j]) {
        i = jump(a.word, b.word[j]);
      } else {
        j = jump(b.word, a.word[i]);
      }
    }
    if (s >= 1) return 1.0;
    return 1.0 - std::sqrt(1.0 - s);
  }
  while (i < a.word.size() && j < b.word.size()) {  // L1Scoring
    const double vi = a.value[i], wi = b.value[j];
    if (a.word[i] == b.word[j]) {
      s += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
      i++;
      j++;
    } else if (a.word[i] < b.word[j]) {
      i = jump(a.word, b.word[j]);
    } else {
      j = jump(b.word, a.word[i]);
    }
  }
  return -s / 2.0;
}

// ------------------------------------------------------------------ device
__device__ __forceinline__ int hamming32(const uint4 a, const uint4 b, const uint32_t (&d)[8]) {
  return __popc(a.x ^ d[0]) + __popc(a.y ^ d[1]) + __popc(a.z ^ d[2]) + __popc(a.w ^ d[3]) +
         __popc(b.x ^ d[4]) + __popc(b.y ^ d[5]) + __popc(b.z ^ d[6]) + __popc(b.w ^ d[7]);
}

__global__ __launch_bounds__(256) void k_bow_transform(VocDev v, const uint8_t* __restrict__ desc,
                                                       int n, int levelsup, uint32_t* word,
                                                       double* weight, uint32_t* node) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t d[8];
  {
    const uint4* p = reinterpret_cast<const uint4*>(desc + 32 * (size_t)i);
    const uint4 a = p[0], b = p[1];
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
    d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
  }
  const int nid_level = v.L - levelsup;
  uint32_t nid = 0;
  int final_id = 0, level = 0;
  do {
    ++level;
    const int c0 = v.child_start[final_id], c1 = v.child_start[final_id + 1];
    int best_id = v.child[c0];
    const uint4* q = reinterpret_cast<const uint4*>(v.desc + 32 * (size_t)best_id);
    int best_d = hamming32(q[0], q[1], d);
    for (int c = c0 + 1; c < c1; c++) {
      const int id = v.child[c];
      const uint4* r = reinterpret_cast<const uint4*>(v.desc + 32 * (size_t)id);
      const int dd = hamming32(r[0], r[1], d);
      if (dd < best_d) {
        best_d = dd;
        best_id = id;
      }
    }
    final_id = best_id;
    if (level == nid_level) nid = (uint32_t)final_id;
  } while (v.child_start[final_id + 1] > v.child_start[final_id]);
  word[i] = (uint32_t)v.word_of[final_id];
  weight[i] = v.weight[final_id];
  node[i] = nid;
}

void launch_bow_transform(const VocDev& v, const uint8_t* desc, int n, int levelsup,
                          uint32_t* word, double* weight, uint32_t* node, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_bow_transform, dim3((n + 255) / 256), dim3(256), 0, st, v, desc, n,
                     levelsup, word, weight, node);
  MMT_HIP(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_sft(SftArgs a) {
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= a.nq) return;
  const SftQuery q = a.q[qi];
  const SftPair& P = a.pairs[q.pair];
  const mmt_kp kp1 = a.k1[q.idx1];
  const bool bStereo1 = a.uR1[q.idx1] >= 0;
  uint32_t d[8];
  {
    const uint4* p = reinterpret_cast<const uint4*>(a.d1 + 32 * (size_t)q.idx1);
    const uint4 x = p[0], y = p[1];
    d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
    d[4] = y.x; d[5] = y.y; d[6] = y.z; d[7] = y.w;
  }
  // the epipolar line of kp1 in keyframe 2 (CheckDistEpipolarLine, float)
  const float la = kp1.x * P.F12[0] + kp1.y * P.F12[3] + P.F12[6];
  const float lb = kp1.x * P.F12[1] + kp1.y * P.F12[4] + P.F12[7];
  const float lc = kp1.x * P.F12[2] + kp1.y * P.F12[5] + P.F12[8];
  const float den = la * la + lb * lb;
  int bestDist = 50, bestIdx2 = -1;  // TH_LOW
  for (int b = q.b0; b < q.b1; b++) {
    const int idx2 = P.feat2[b];
    if (P.taken2[idx2]) continue;
    const bool bStereo2 = P.uR2[idx2] >= 0;
    const uint4* r = reinterpret_cast<const uint4*>(P.d2 + 32 * (size_t)idx2);
    const int dist = hamming32(r[0], r[1], d);
    if (dist > 50 || dist > bestDist) continue;
    const mmt_kp kp2 = P.k2[idx2];
    if (!bStereo1 && !bStereo2) {
      const float distex = P.ex - kp2.x, distey = P.ey - kp2.y;
      if (distex * distex + distey * distey < 100 * a.scale[kp2.octave]) continue;
    }
    if (den == 0) continue;
    const float num = la * kp2.x + lb * kp2.y + lc;
    const float dsqr = num * num / den;
    if ((double)dsqr < 3.84 * (double)a.sigma2[kp2.octave]) {
      bestIdx2 = idx2;
      bestDist = dist;
    }
  }
  a.out[qi] = bestIdx2;
}

void launch_sft(const SftArgs& a, hipStream_t st) {
  if (a.nq <= 0) return;
  hipLaunchKernelGGL(k_sft, dim3((a.nq + 255) / 256), dim3(256), 0, st, a);
  MMT_HIP(hipGetLastError());
}

}  // namespace mmt
