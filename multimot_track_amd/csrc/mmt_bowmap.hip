// multimot_track_amd/csrc/mmt_bowmap.hip -- the reference's vocabulary-driven map steps, run when
// the context is given a vocabulary (mmt_load_vocabulary; System.cc:67):
//   Frame::ComputeBoW / KeyFrame::ComputeBoW           Frame.cc:778-786, KeyFrame.cc:59-68
//   KeyFrameDatabase::add / erase / DetectRelocalizationCandidates  KeyFrameDatabase.cc:40-67, 199-309
//   Tracking::TrackReferenceKeyFrame                    Tracking.cc:2836-2892
//   Tracking::Relocalization                            Tracking.cc:3614-3776
//   ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>&, th, ORBdist)  ORBmatcher.cc:2104-2231
//   LocalMapping::CreateNewMapPoints (+ ComputeF12)     LocalMapping.cc:210-456, 540-557
//   ORBmatcher::SearchForTriangulation                  ORBmatcher.cc:1032-1198
// The data-parallel parts run on the GPU: DBoW2's transform (k_bow_transform, one descent per
// feature), SearchByBoW (C4, k_bow_nodes / k_bow_rot), PnPsolver's hypotheses and refits (D6),
// PoseOptimization (D1), the relocalisation's projection search (k_sbp_kf's candidate lists) and
// SearchForTriangulation (k_sft, one query per keyframe feature and neighbour).  The bookkeeping
// (BoW / feature vectors, the database, the order-dependent binding of the projection search, the
// per-match triangulation with its libm calls) is host C++ where the reference keeps it.
// Pinned choices: as oracle/bowmap_ref.cpp.

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>

#include "mmt_internal.h"
#include "mmt_map.h"
#include "mmt_mat4.h"
#include "mmt_pnp.h"

namespace mmt {

namespace {
constexpr int TH_LOW = 50, HISTO_LENGTH = 30;

void cam_centre(const float* T, float* Ow) {  // -Rcw^T tcw
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    Ow[r] = -(float)s;
  }
}
void xform(const float* T, const float* x, float* y) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * r + k] * (double)x[k];
    y[r] = (float)s + T[4 * r + 3];
  }
}
float norm3(const float* v) {
  double s = 0;
  for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
  return (float)std::sqrt(s);
}
// KeyFrame::UnprojectStereo: Rwc * ((u - cx) z / fx, (v - cy) z / fy, z) + Ow
void unproject(const MapCamH& c, const float* T, float u, float v, float z, float* out) {
  const float x = (u - c.cx) * z * c.invfx, y = (v - c.cy) * z * c.invfy;
  const float xc[3] = {x, y, z};
  float Ow[3];
  cam_centre(T, Ow);
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)xc[k];
    out[r] = (float)s + Ow[r];
  }
}
void three_max(const std::vector<int>* histo, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < HISTO_LENGTH; i++) {
    const int s = (int)histo[i].size();
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}
int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 4; i++) {
    uint64_t x, y;
    memcpy(&x, a + 8 * i, 8);
    memcpy(&y, b + 8 * i, 8);
    d += __builtin_popcountll(x ^ y);
  }
  return d;
}
// the null vector of the linear triangulation's 4x4 A (cv::SVD::compute's vt.row(3), pinned:
// the eigenvector of A^T A for its smallest eigenvalue by cyclic Jacobi in double)
void null_vector4(const float A[16], float v_out[4]) {
  double M[4][4], V[4][4];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      double s = 0;
      for (int r = 0; r < 4; r++) s += (double)A[4 * r + i] * (double)A[4 * r + j];
      M[i][j] = s;
      V[i][j] = i == j ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 50; sweep++) {
    double off = 0, tr = 0;
    for (int i = 0; i < 4; i++) {
      tr += M[i][i] * M[i][i];
      for (int j = i + 1; j < 4; j++) off += M[i][j] * M[i][j];
    }
    if (off <= 1e-30 * tr) break;
    for (int p = 0; p < 3; p++)
      for (int q = p + 1; q < 4; q++) {
        if (M[p][q] == 0.0) continue;
        const double theta = (M[q][q] - M[p][p]) / (2.0 * M[p][q]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; k++) {
          const double mkp = M[k][p], mkq = M[k][q];
          M[k][p] = c * mkp - s * mkq;
          M[k][q] = s * mkp + c * mkq;
        }
        for (int k = 0; k < 4; k++) {
          const double mpk = M[p][k], mqk = M[q][k];
          M[p][k] = c * mpk - s * mqk;
          M[q][k] = s * mpk + c * mqk;
        }
        for (int k = 0; k < 4; k++) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int m = 0;
  for (int i = 1; i < 4; i++)
    if (M[i][i] < M[m][m]) m = i;
  double n = 0;
  for (int k = 0; k < 4; k++) n += V[k][m] * V[k][m];
  n = std::sqrt(n);
  for (int k = 0; k < 4; k++) v_out[k] = (float)(V[k][m] / n);
}
// LocalMapping::ComputeF12 = K1^-T [t12]x R12 K2^-1 (pinned: double from the float poses and K,
// one float rounding)
void compute_f12(const float* T1, const float* T2, const MapCamH& cam, float F[9]) {
  double R12[3][3], t12[3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += (double)T1[4 * r + k] * (double)T2[4 * c + k];
      R12[r][c] = s;
    }
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int c = 0; c < 3; c++) s += R12[r][c] * (double)T2[4 * c + 3];
    t12[r] = -s + (double)T1[4 * r + 3];
  }
  const double tx[3][3] = {{0, -t12[2], t12[1]}, {t12[2], 0, -t12[0]}, {-t12[1], t12[0], 0}};
  const double fx = cam.fx, fy = cam.fy, cx = cam.cx, cy = cam.cy;
  const double Ki[3][3] = {{1 / fx, 0, -cx / fx}, {0, 1 / fy, -cy / fy}, {0, 0, 1}};
  double A[3][3], B[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += Ki[k][r] * tx[k][c];
      A[r][c] = s;
    }
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += A[r][k] * R12[k][c];
      B[r][c] = s;
    }
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += B[r][k] * Ki[k][c];
      F[3 * r + c] = (float)s;
    }
}
size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
}  // namespace

// ------------------------------------------------------------------ glibc rand()
GlibcRandH::GlibcRandH() {
  r_.resize(34);
  r_[0] = 1;  // srand(1): an unseeded process
  for (int i = 1; i < 31; i++) {
    const int64_t hi = r_[i - 1] / 127773, lo = r_[i - 1] % 127773;
    int64_t word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r_[i] = (int32_t)word;
  }
  for (int i = 31; i < 34; i++) r_[i] = r_[i - 31];
  for (int i = 0; i < 310; i++) next();
}
int GlibcRandH::next() {
  const size_t i = r_.size();
  const uint32_t v = (uint32_t)r_[i - 31] + (uint32_t)r_[i - 3];
  r_.push_back((int32_t)v);
  if (r_.size() > 4096) r_.erase(r_.begin(), r_.end() - 34);
  return (int)(v >> 1);
}
int GlibcRandH::random_int(int min, int max) {  // DUtils::Random::RandomInt
  const int d = max - min + 1;
  return int(((double)next() / ((double)2147483647 + 1.0)) * d) + min;
}

// ------------------------------------------------------------------ BoW
void MapEngine::set_vocabulary(Vocabulary* v) {
  voc_ = v;
  invfile_.assign(v ? (size_t)v->n_words() : 0, std::vector<int>());
  if (v) v->upload();
}

void MapEngine::bw_grow(size_t need) {
  if (need <= bw_cap_ && d_bw_) return;
  if (s_) MMT_HIP(hipStreamSynchronize(s_));
  grow_dev(d_bw_, h_bw_, bw_cap_, need);
}

// transform(descriptors, BowVector, FeatureVector, 4): the descent on the GPU, the vectors built
// on the host in feature order (Vocabulary::build).  bow_launch queues the descent and the copy
// back on st; bow_finish waits for them and builds (nothing may touch d_bw_ / h_bw_ between)
void MapEngine::bow_launch(const uint8_t* d_desc, int n, hipStream_t st) {
  const size_t bytes = 16 * (size_t)std::max(n, 1);
  bw_grow(bytes);
  uint32_t* dw = (uint32_t*)d_bw_;
  uint32_t* dn = dw + n;
  double* dx = (double*)(d_bw_ + 8 * (size_t)n);
  launch_bow_transform(voc_->dev, d_desc, n, 4, dw, dx, dn, st);
  if (n > 0) MMT_HIP(hipMemcpyAsync(h_bw_, d_bw_, 16 * (size_t)n, hipMemcpyDeviceToHost, st));
}

void MapEngine::bow_finish(int n, hipStream_t st, BowVecH& v, FeatVecH& fv) {
  MMT_HIP(hipStreamSynchronize(st));
  const uint32_t* hw = (const uint32_t*)h_bw_;
  voc_->build(hw, (const double*)(h_bw_ + 8 * (size_t)n), hw + n, n, v, fv);
}

void MapEngine::frame_bow(MapFrameH& C, const GridFrame& G) {  // Frame::ComputeBoW
  if (C.hasBow) return;
  bow_launch(G.desc, C.n, s_);
  bow_finish(C.n, s_, C.bow, C.fv);
  C.hasBow = true;
  bstats_.n_bow_frames++;
}

// KeyFrame::ComputeBoW on the keyframe-store copy (lm_s_), in two halves: ProcessNewKeyFrame's
// host work runs between them (it does not read the vectors)
void MapEngine::kf_bow_launch(int kf) {
  const KFrame& K = kfs_[kf];
  if (!K.hasBow) bow_launch(K.dev.desc, (int)K.keys.size(), lm_s_);
}

void MapEngine::kf_bow_finish(int kf) {
  KFrame& K = kfs_[kf];
  if (K.hasBow) return;
  bow_finish((int)K.keys.size(), lm_s_, K.bow, K.fv);
  K.hasBow = true;
}

void MapEngine::kfdb_add(int kf) {  // KeyFrameDatabase::add
  for (uint32_t w : kfs_[kf].bow.word) invfile_[w].push_back(kf);
  bstats_.n_kfdb++;
}

void MapEngine::kfdb_erase(int kf) {  // KeyFrameDatabase::erase
  if (!voc_) return;
  for (uint32_t w : kfs_[kf].bow.word) {
    std::vector<int>& l = invfile_[w];
    auto it = std::find(l.begin(), l.end(), kf);
    if (it != l.end()) l.erase(it);
  }
}

// KeyFrameDatabase::DetectRelocalizationCandidates (KeyFrameDatabase.cc:199-309)
std::vector<int> MapEngine::detect_relocalization_candidates(const MapFrameH& C) {
  std::vector<int> shared;
  for (uint32_t w : C.bow.word)
    for (int k : invfile_[w]) {
      KFrame& K = kfs_[k];
      if (K.relocQuery != C.id) {
        K.relocWords = 0;
        K.relocQuery = C.id;
        shared.push_back(k);
      }
      K.relocWords++;
    }
  if (shared.empty()) return {};
  int maxCommonWords = 0;
  for (int k : shared) maxCommonWords = std::max(maxCommonWords, kfs_[k].relocWords);
  const int minCommonWords = (int)(maxCommonWords * 0.8f);
  std::vector<std::pair<float, int>> scored;
  for (int k : shared) {
    KFrame& K = kfs_[k];
    if (K.relocWords > minCommonWords) {
      const float si = (float)voc_->score(C.bow, K.bow);
      K.relocScore = si;
      scored.push_back({si, k});
    }
  }
  if (scored.empty()) return {};
  std::vector<std::pair<float, int>> acc;
  float bestAccScore = 0;
  for (const auto& sk : scored) {
    float bestScore = sk.first, accScore = bestScore;
    int bestKF = sk.second;
    const std::vector<int>& o = kfs_[sk.second].ordered;  // GetBestCovisibilityKeyFrames(10)
    for (size_t q = 0; q < o.size() && q < 10; q++) {
      const KFrame& K2 = kfs_[o[q]];
      if (K2.relocQuery != C.id) continue;
      accScore += K2.relocScore;
      if (K2.relocScore > bestScore) {
        bestKF = o[q];
        bestScore = K2.relocScore;
      }
    }
    acc.push_back({accScore, bestKF});
    if (accScore > bestAccScore) bestAccScore = accScore;
  }
  const float minScoreToRetain = 0.75f * bestAccScore;
  std::vector<int> out;
  std::set<int> added;
  for (const auto& a : acc)
    if (a.first > minScoreToRetain && !added.count(a.second)) {
      out.push_back(a.second);
      added.insert(a.second);
    }
  return out;
}

// C4: ORBmatcher(nnratio, true)::SearchByBoW(pKF, F, vpMapPointMatches) on the GPU: match[i] =
// the keyframe key whose MapPoint now matches frame key i (-1); returns nmatches
int MapEngine::search_by_bow_kf(int kf, const MapFrameH& C, const GridFrame& G, float nnratio,
                                std::vector<int>& match) {
  const KFrame& K = kfs_[kf];
  const int nk = (int)K.keys.size(), nF = C.n;
  const int nn1 = (int)K.fv.node.size(), nf1 = (int)K.fv.feat.size();
  const int nn2 = (int)C.fv.node.size(), nf2 = (int)C.fv.feat.size();
  for (int q = 0; q < nn2; q++)
    if (C.fv.start[q + 1] - C.fv.start[q] > kBowMaxNodeFeatures)
      throw ArgError("SearchByBoW: a vocabulary node holds more than 2048 frame features");
  const size_t o_ok = 0, o_n1 = al16(nk), o_s1 = o_n1 + al16(4 * (size_t)nn1),
               o_f1 = o_s1 + al16(4 * (size_t)(nn1 + 1)), o_n2 = o_f1 + al16(4 * (size_t)nf1),
               o_s2 = o_n2 + al16(4 * (size_t)nn2), o_f2 = o_s2 + al16(4 * (size_t)(nn2 + 1)),
               o_up = o_f2 + al16(4 * (size_t)nf2), o_m = o_up, o_h = o_m + al16(4 * (size_t)nF),
               o_c = o_h + al16(4 * 32), tot = o_c + 16;
  bw_grow(tot);
  uint8_t* h = h_bw_;
  for (int i = 0; i < nk; i++) h[o_ok + i] = K.mps[i] >= 0 && !pts_[K.mps[i]].bad;
  memcpy(h + o_n1, K.fv.node.data(), 4 * (size_t)nn1);
  memcpy(h + o_s1, K.fv.start.data(), 4 * (size_t)(nn1 + 1));
  memcpy(h + o_f1, K.fv.feat.data(), 4 * (size_t)nf1);
  memcpy(h + o_n2, C.fv.node.data(), 4 * (size_t)nn2);
  memcpy(h + o_s2, C.fv.start.data(), 4 * (size_t)(nn2 + 1));
  memcpy(h + o_f2, C.fv.feat.data(), 4 * (size_t)nf2);
  MMT_HIP(hipMemcpyAsync(d_bw_, h_bw_, o_up, hipMemcpyHostToDevice, s_));
  uint8_t* d = d_bw_;
  const BowFeatVec a{nn1, (const uint32_t*)(d + o_n1), (const int*)(d + o_s1),
                     (const int*)(d + o_f1)};
  const BowFeatVec b{nn2, (const uint32_t*)(d + o_n2), (const int*)(d + o_s2),
                     (const int*)(d + o_f2)};
  launch_search_by_bow(a, K.dev.keys, K.dev.desc, d + o_ok, b, G.keys, G.desc, nF, nnratio, 1,
                       (int*)(d + o_m), (int*)(d + o_h), (int*)(d + o_c), s_);
  MMT_HIP(hipMemcpyAsync(h + o_m, d + o_m, tot - o_m, hipMemcpyDeviceToHost, s_));
  MMT_HIP(hipStreamSynchronize(s_));
  match.assign((int*)(h + o_m), (int*)(h + o_m) + nF);
  return ((int*)(h + o_c))[1];
}

// Optimizer::PoseOptimization(&mCurrentFrame) on the GPU (D1) over the frame's MapPoints in key
// order; the pose and mvbOutlier applied; returns nInitialCorrespondences - nBad (0 below 3)
int MapEngine::gpu_pose_optimization(MapFrameH& C, float* Tcw) {
  float* X = h_edges_;
  float* ob = h_edges_ + 3 * (size_t)kcap_;
  float* s2 = h_edges_ + 6 * (size_t)kcap_;
  int n = 0;
  for (int i = 0; i < C.n; i++) {
    if (C.mps[i] < 0) continue;
    const MPoint& p = mp(C.mps[i]);
    memcpy(X + 3 * (size_t)n, p.pos, 12);
    ob[3 * (size_t)n] = C.kps[i].x;
    ob[3 * (size_t)n + 1] = C.kps[i].y;
    ob[3 * (size_t)n + 2] = C.uR[i];
    s2[n] = cam_.invSigma2[C.kps[i].octave];
    n++;
  }
  pose_desc_fill(h_last_, d_last_, Tcw);
  h_pod_->n = n;
  MMT_HIP(hipMemcpyAsync(d_last_, h_last_, kDescBytes, hipMemcpyHostToDevice, s_));
  if (n > 0) {
    MMT_HIP(hipMemcpyAsync(d_edges_, X, 12 * (size_t)n, hipMemcpyHostToDevice, s_));
    MMT_HIP(hipMemcpyAsync(d_edges_ + 3 * (size_t)kcap_, ob, 12 * (size_t)n,
                           hipMemcpyHostToDevice, s_));
    MMT_HIP(hipMemcpyAsync(d_edges_ + 6 * (size_t)kcap_, s2, 4 * (size_t)n,
                           hipMemcpyHostToDevice, s_));
  }
  launch_pose_opt(d_pod_, 1, n, s_);
  MMT_HIP(hipMemcpyAsync(h_out_, d_out_, out_bytes(C.n), hipMemcpyDeviceToHost, s_));
  MMT_HIP(hipStreamSynchronize(s_));
  apply_pose_opt(C, Tcw);
  return n < 3 ? 0 : *h_ninl_;
}

// Tracking::TrackReferenceKeyFrame (Tracking.cc:2836-2892)
bool MapEngine::track_reference_kf(MapFrameH& C, const GridFrame& G, float* Tcw,
                                   const float* Tlast) {
  bstats_.n_trk++;
  frame_bow(C, G);
  std::vector<int> match;
  int nmatches = search_by_bow_kf(refKF_, C, G, 0.7f, match);
  if (nmatches < 15) return false;
  const KFrame& K = kfs_[refKF_];
  for (int i = 0; i < C.n; i++) C.mps[i] = match[i] >= 0 ? K.mps[match[i]] : -1;
  memcpy(Tcw, Tlast, 64);
  gpu_pose_optimization(C, Tcw);
  int nmatchesMap = 0;
  discard_outliers(C, nmatches, &nmatchesMap);
  if (nmatchesMap >= 10) bstats_.n_trk_ok++;
  return nmatchesMap >= 10;
}

// ORBmatcher(0.9, true)::SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist): k_sbp_kf's
// candidate lists, then the binding in the keyframe's map-point order (a key bound by an earlier
// point is skipped), the ORBdist test and the rotation histogram
int MapEngine::search_by_projection_kf(MapFrameH& C, const GridFrame& G, const float* Tcw, int kf,
                                       const std::set<int>& found, float th, int orbDist) {
  const KFrame& K = kfs_[kf];
  std::vector<int> slot, hnd;
  for (size_t i = 0; i < K.mps.size(); i++) {
    const int h = K.mps[i];
    if (h < 0 || pts_[h].bad || found.count(h)) continue;
    slot.push_back((int)i);
    hnd.push_back(h);
  }
  const int m = (int)slot.size();
  const size_t o_p = 0, o_b = al16(sizeof(SbpKfPoint) * (size_t)m),
               o_up = o_b + al16((size_t)C.n), o_k = o_up,
               o_i = o_k + al16(4 * (size_t)m * kSbpKfCand),
               o_n = o_i + al16(4 * (size_t)m * kSbpKfCand),
               o_w = o_n + al16(4 * (size_t)m), tot = o_w + sizeof(PointWin) * (size_t)m + 16;
  bw_grow(tot);
  uint8_t* h = h_bw_;
  SbpKfPoint* P = (SbpKfPoint*)(h + o_p);
  for (int j = 0; j < m; j++) {
    const MPoint& p = pts_[hnd[j]];
    memcpy(P[j].Xw, p.pos, 12);
    P[j].min_dist = p.minDist;
    P[j].max_dist = p.maxDist;
    P[j].pad[0] = P[j].pad[1] = P[j].pad[2] = 0;
    memcpy(P[j].desc, p.desc, 32);
  }
  for (int i = 0; i < C.n; i++) h[o_b + i] = C.mps[i] >= 0;
  int nmatches = 0;
  if (m > 0) {
    MMT_HIP(hipMemcpyAsync(d_bw_, h_bw_, o_up, hipMemcpyHostToDevice, s_));
    SbpKfArgs a;
    a.C = G;
    memcpy(a.Tcw, Tcw, 64);
    a.th = th;
    a.pts = (const SbpKfPoint*)(d_bw_ + o_p);
    a.m = m;
    a.bound = d_bw_ + o_b;
    a.cand_key = (uint32_t*)(d_bw_ + o_k);
    a.cand_idx = (int*)(d_bw_ + o_i);
    a.n_cand = (int*)(d_bw_ + o_n);
    a.win = (PointWin*)(d_bw_ + o_w);
    launch_sbp_kf(a, s_);
    MMT_HIP(hipMemcpyAsync(h + o_k, d_bw_ + o_k, tot - o_k, hipMemcpyDeviceToHost, s_));
    MMT_HIP(hipStreamSynchronize(s_));
  }
  const uint32_t* ck = (const uint32_t*)(h + o_k);
  const int* ci = (const int*)(h + o_i);
  const int* nc = (const int*)(h + o_n);
  const PointWin* win = (const PointWin*)(h + o_w);
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  for (int j = 0; j < m; j++) {
    if (nc[j] <= 0) continue;
    int best = -1, bestDist = 256;
    const int nk = std::min(nc[j], kSbpKfCand);
    for (int c = 0; c < nk; c++) {
      const int k = ci[(size_t)j * kSbpKfCand + c];
      if (C.mps[k] >= 0) continue;  // bound by an earlier point of this call
      best = k;
      bestDist = (int)(ck[(size_t)j * kSbpKfCand + c] >> 20);
      break;
    }
    if (best < 0 && nc[j] > kSbpKfCand) {
      // every listed candidate was taken by earlier points: rescan the window on the host in
      // GetFeaturesInArea order (cells ix, iy ascending, keys ascending in a cell)
      const PointWin& w = win[j];
      const int cx0 = std::max(0, (int)std::floor((w.x - G.minX - w.r) * G.invW));
      const int cx1 = std::min(kGridCols - 1, (int)std::ceil((w.x - G.minX + w.r) * G.invW));
      const int cy0 = std::max(0, (int)std::floor((w.y - G.minY - w.r) * G.invH));
      const int cy1 = std::min(kGridRows - 1, (int)std::ceil((w.y - G.minY + w.r) * G.invH));
      long bestKey = LONG_MAX;
      for (int k = 0; k < C.n; k++) {
        const mmt_kp& kp = C.kps[k];
        const int px = (int)std::round((kp.x - 0.0f) * G.invW);
        const int py = (int)std::round((kp.y - 0.0f) * G.invH);
        if (px < cx0 || px > cx1 || py < cy0 || py > cy1) continue;
        if (kp.octave < w.minLevel || (w.maxLevel >= 0 && kp.octave > w.maxLevel)) continue;
        if (!(std::fabs(kp.x - w.x) < w.r && std::fabs(kp.y - w.y) < w.r)) continue;
        if (C.mps[k] >= 0) continue;
        const int dist = hamming(pts_[hnd[j]].desc, C.desc + 32 * (size_t)k);
        const long key = ((long)dist << 40) | ((long)(px * kGridRows + py) << 20) | k;
        if (key < bestKey) {
          bestKey = key;
          best = k;
          bestDist = dist;
        }
      }
    }
    if (best < 0 || bestDist > orbDist) continue;
    C.mps[best] = hnd[j];
    nmatches++;
    float rot = K.keys[slot[j]].angle - C.kps[best].angle;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    rotHist[bin].push_back(best);
  }
  int ind1 = -1, ind2 = -1, ind3 = -1;
  three_max(rotHist, ind1, ind2, ind3);
  for (int i = 0; i < HISTO_LENGTH; i++) {
    if (i == ind1 || i == ind2 || i == ind3) continue;
    for (int j : rotHist[i]) {
      C.mps[j] = -1;
      nmatches--;
    }
  }
  return nmatches;
}

// Tracking::Relocalization (Tracking.cc:3614-3776)
bool MapEngine::relocalization(MapFrameH& C, const GridFrame& G, float* Tcw) {
  bstats_.n_reloc++;
  frame_bow(C, G);
  const std::vector<int> cands = detect_relocalization_candidates(C);
  if (cands.empty()) return false;
  bstats_.n_reloc_cands += (long)cands.size();
  const int nKFs = (int)cands.size(), N = C.n;
  struct Solver {  // PnPsolver(F, vvpMapPointMatches[i]), SetRansacParameters(0.99, 10, 300, 4, 0.5, 5.991)
    std::vector<float> p3, p2, s2;
    std::vector<int> kpIdx;
    std::vector<uint8_t> best_mask;
    mmt_pnpsolver_state st{};
  };
  std::vector<Solver> solvers(nKFs);
  std::vector<std::vector<int>> matches(nKFs);
  std::vector<uint8_t> discarded(nKFs, 0);
  int nCandidates = 0;
  for (int i = 0; i < nKFs; i++) {
    const KFrame& K = kfs_[cands[i]];
    if (K.bad) {
      discarded[i] = 1;
      continue;
    }
    std::vector<int> match;
    const int nm = search_by_bow_kf(cands[i], C, G, 0.75f, match);
    matches[i].assign(N, -1);
    for (int j = 0; j < N; j++)
      if (match[j] >= 0) matches[i][j] = K.mps[match[j]];
    if (nm < 15) {
      discarded[i] = 1;
      continue;
    }
    Solver& S = solvers[i];
    for (int j = 0; j < N; j++) {
      const int h = matches[i][j];
      if (h < 0 || pts_[h].bad) continue;
      S.p2.push_back(C.kps[j].x);
      S.p2.push_back(C.kps[j].y);
      const float sc = cam_.scale[C.kps[j].octave];
      S.s2.push_back(sc * sc);
      S.p3.insert(S.p3.end(), pts_[h].pos, pts_[h].pos + 3);
      S.kpIdx.push_back(j);
    }
    S.best_mask.assign(std::max<size_t>(S.kpIdx.size(), 1), 0);
    S.st.best_mask = S.best_mask.data();
    nCandidates++;
  }
  bool bMatch = false;
  while (nCandidates > 0 && !bMatch) {
    for (int i = 0; i < nKFs; i++) {
      if (discarded[i]) continue;
      Solver& S = solvers[i];
      const int n = (int)S.kpIdx.size();
      mmt_pnpsolver_problem pr;
      pr.n = n;
      pr.pts3 = S.p3.data();
      pr.pts2 = S.p2.data();
      pr.sigma2 = S.s2.data();
      pr.fx = cam_.fx; pr.fy = cam_.fy; pr.cx = cam_.cx; pr.cy = cam_.cy;
      pr.probability = 0.99;
      pr.min_inliers = 10;
      pr.max_iterations = 300;
      pr.min_set = 4;
      pr.epsilon = 0.5f;
      pr.th2 = 5.991f;
      // iterate(5): the draws of as many iterations as the call can run, from a copy of the
      // process's rand() stream; the stream then advances by the draws the call used
      const int maxIts = 300 + 5;
      std::vector<int32_t> randi(4 * (size_t)maxIts, 0);
      {
        GlibcRandH g = rand_;
        for (int k = 0; k < maxIts; k++)
          for (int j = 0; j < 4; j++) randi[4 * k + j] = n - 1 - j >= 0 ? g.random_int(0, n - 1 - j) : 0;
      }
      const int it0 = S.st.iterations;
      float T[16];
      std::vector<uint8_t> inl(std::max(n, 1), 0);
      int ninl = 0, found = 0, no_more = 0;
      pnpsolver_iterate_gpu(s_, &pr, randi.data(), maxIts, 5, &S.st, T, inl.data(), &ninl,
                            &found, &no_more);
      for (int k = 0; k < 4 * (S.st.iterations - it0); k++) rand_.next();
      if (no_more) {
        discarded[i] = 1;
        nCandidates--;
      }
      if (!found) continue;
      bstats_.n_pnp_found++;
      memcpy(Tcw, T, 64);
      std::set<int> sFound;
      std::vector<uint8_t> inF(N, 0);
      for (int q = 0; q < n; q++)
        if (inl[q]) inF[S.kpIdx[q]] = 1;
      for (int j = 0; j < N; j++) {
        if (inF[j]) {
          C.mps[j] = matches[i][j];
          sFound.insert(matches[i][j]);
        } else {
          C.mps[j] = -1;
        }
      }
      int nGood = gpu_pose_optimization(C, Tcw);
      if (nGood < 10) continue;
      for (int io = 0; io < N; io++)
        if (C.outlier[io]) C.mps[io] = -1;
      if (nGood < 50) {
        bstats_.n_sbp_rounds++;
        int nadditional = search_by_projection_kf(C, G, Tcw, cands[i], sFound, 10, 100);
        if (nadditional + nGood >= 50) {
          nGood = gpu_pose_optimization(C, Tcw);
          if (nGood > 30 && nGood < 50) {
            sFound.clear();
            for (int ip = 0; ip < N; ip++)
              if (C.mps[ip] >= 0) sFound.insert(C.mps[ip]);
            bstats_.n_sbp_rounds++;
            nadditional = search_by_projection_kf(C, G, Tcw, cands[i], sFound, 3, 64);
            if (nGood + nadditional >= 50) {
              nGood = gpu_pose_optimization(C, Tcw);
              for (int io = 0; io < N; io++)
                if (C.outlier[io]) C.mps[io] = -1;
            }
          }
        }
      }
      if (nGood >= 50) {
        bMatch = true;
        break;
      }
    }
  }
  if (bMatch) bstats_.n_reloc_ok++;
  return bMatch;
}

// LocalMapping::CreateNewMapPoints (LocalMapping.cc:210-456), RGB-D branch: SearchForTriangulation
// of every neighbour in one k_sft launch (the queries of neighbour i whose keyframe-1 feature got
// a point from an earlier neighbour are dropped, as the reference skips them; neighbour i's own
// keyframe is touched by no earlier neighbour), then the triangulation on the host
void MapEngine::create_new_map_points(int kf) {
  std::vector<int> neigh;
  {
    const std::vector<int>& o = kfs_[kf].ordered;
    for (size_t q = 0; q < o.size() && q < 10; q++) neigh.push_back(o[q]);
  }
  const float ratioFactor = 1.5f * cam_.scale[1];
  const float mb = cam_.bf / cam_.fx;
  struct PairH {
    int k2;
    float F12[9];
    float ex, ey;
  };
  std::vector<PairH> pairs;
  for (int k2 : neigh) {
    const KFrame& K1 = kfs_[kf];
    const KFrame& K2 = kfs_[k2];
    const float vB[3] = {K2.Ow[0] - K1.Ow[0], K2.Ow[1] - K1.Ow[1], K2.Ow[2] - K1.Ow[2]};
    if (norm3(vB) < mb) continue;
    PairH p;
    p.k2 = k2;
    compute_f12(K1.Tcw, K2.Tcw, cam_, p.F12);
    float C2[3];
    xform(K2.Tcw, K1.Ow, C2);
    const float invz = 1.0f / C2[2];
    p.ex = cam_.fx * C2[0] * invz + cam_.cx;
    p.ey = cam_.fy * C2[1] * invz + cam_.cy;
    pairs.push_back(p);
  }
  if (pairs.empty()) return;
  const KFrame& K1 = kfs_[kf];
  const int np = (int)pairs.size();
  std::vector<SftQuery> q;
  std::vector<size_t> o_feat(np), o_tak(np);
  size_t off = al16(sizeof(SftPair) * (size_t)np);
  for (int p = 0; p < np; p++) {
    const KFrame& K2 = kfs_[pairs[p].k2];
    o_feat[p] = off;
    off += al16(4 * K2.fv.feat.size() + 4);
    o_tak[p] = off;
    off += al16(K2.keys.size() + 1);
    size_t a = 0, b = 0;
    const FeatVecH& f1 = K1.fv;
    const FeatVecH& f2 = K2.fv;
    while (a < f1.node.size() && b < f2.node.size()) {
      if (f1.node[a] == f2.node[b]) {
        for (int i = f1.start[a]; i < f1.start[a + 1]; i++) {
          const int idx1 = f1.feat[i];
          if (K1.mps[idx1] >= 0) continue;
          q.push_back(SftQuery{p, idx1, f2.start[b], f2.start[b + 1]});
        }
        a++;
        b++;
      } else if (f1.node[a] < f2.node[b]) {
        a = (size_t)(std::lower_bound(f1.node.begin(), f1.node.end(), f2.node[b]) - f1.node.begin());
      } else {
        b = (size_t)(std::lower_bound(f2.node.begin(), f2.node.end(), f1.node[a]) - f2.node.begin());
      }
    }
  }
  const int nq = (int)q.size();
  const size_t o_q = off, o_up = o_q + al16(sizeof(SftQuery) * (size_t)std::max(nq, 1)),
               o_out = o_up, tot = o_out + 4 * (size_t)std::max(nq, 1);
  bw_grow(tot);
  uint8_t* h = h_bw_;
  SftPair* P = (SftPair*)h;
  for (int p = 0; p < np; p++) {
    const KFrame& K2 = kfs_[pairs[p].k2];
    P[p].k2 = K2.dev.keys;
    P[p].d2 = K2.dev.desc;
    P[p].uR2 = K2.dev.uR;
    P[p].feat2 = (const int*)(d_bw_ + o_feat[p]);
    P[p].taken2 = d_bw_ + o_tak[p];
    memcpy(P[p].F12, pairs[p].F12, sizeof(P[p].F12));
    P[p].ex = pairs[p].ex;
    P[p].ey = pairs[p].ey;
    memcpy(h + o_feat[p], K2.fv.feat.data(), 4 * K2.fv.feat.size());
    for (size_t i = 0; i < K2.keys.size(); i++) h[o_tak[p] + i] = K2.mps[i] >= 0;
  }
  memcpy(h + o_q, q.data(), sizeof(SftQuery) * (size_t)nq);
  std::vector<int> best(std::max(nq, 1), -1);
  if (nq > 0) {
    MMT_HIP(hipMemcpyAsync(d_bw_, h_bw_, o_up, hipMemcpyHostToDevice, lm_s_));
    SftArgs a;
    a.k1 = K1.dev.keys;
    a.d1 = K1.dev.desc;
    a.uR1 = K1.dev.uR;
    a.pairs = (const SftPair*)d_bw_;
    a.q = (const SftQuery*)(d_bw_ + o_q);
    a.nq = nq;
    for (int l = 0; l < cam_.nlevels && l < kMaxLevels; l++) {
      a.scale[l] = cam_.scale[l];
      a.sigma2[l] = cam_.scale[l] * cam_.scale[l];
    }
    a.out = (int*)(d_bw_ + o_out);
    launch_sft(a, lm_s_);
    MMT_HIP(hipMemcpyAsync(best.data(), d_bw_ + o_out, 4 * (size_t)nq, hipMemcpyDeviceToHost, lm_s_));
    MMT_HIP(hipStreamSynchronize(lm_s_));
  }
  size_t qi = 0;
  for (int p = 0; p < np; p++) {
    const int k2 = pairs[p].k2;
    // vMatchedPairs in keyframe-1 key order, over the features still without a MapPoint
    std::vector<std::pair<int, int>> mp12;
    for (; qi < q.size() && q[qi].pair == p; qi++)
      if (best[qi] >= 0 && kfs_[kf].mps[q[qi].idx1] < 0) mp12.push_back({q[qi].idx1, best[qi]});
    std::sort(mp12.begin(), mp12.end());
    bstats_.n_sft_matches += (long)mp12.size();
    const float* T1 = kfs_[kf].Tcw;
    const float* T2 = kfs_[k2].Tcw;
    for (const auto& pr : mp12) {
      const int idx1 = pr.first, idx2 = pr.second;
      const mmt_kp& kp1 = kfs_[kf].keys[idx1];
      const float kp1_ur = kfs_[kf].uR[idx1];
      const bool bStereo1 = kp1_ur >= 0;
      const mmt_kp& kp2 = kfs_[k2].keys[idx2];
      const float kp2_ur = kfs_[k2].uR[idx2];
      const bool bStereo2 = kp2_ur >= 0;
      const float xn1[3] = {(kp1.x - cam_.cx) * cam_.invfx, (kp1.y - cam_.cy) * cam_.invfy, 1.0f};
      const float xn2[3] = {(kp2.x - cam_.cx) * cam_.invfx, (kp2.y - cam_.cy) * cam_.invfy, 1.0f};
      float ray1[3], ray2[3];
      for (int r = 0; r < 3; r++) {
        double s1 = 0, s2 = 0;
        for (int c = 0; c < 3; c++) {
          s1 += (double)T1[4 * c + r] * (double)xn1[c];
          s2 += (double)T2[4 * c + r] * (double)xn2[c];
        }
        ray1[r] = (float)s1;
        ray2[r] = (float)s2;
      }
      double dot = 0, n1 = 0, n2 = 0;
      for (int r = 0; r < 3; r++) {
        dot += (double)ray1[r] * (double)ray2[r];
        n1 += (double)ray1[r] * (double)ray1[r];
        n2 += (double)ray2[r] * (double)ray2[r];
      }
      const float cosParallaxRays = (float)(dot / (std::sqrt(n1) * std::sqrt(n2)));
      float cosParallaxStereo = cosParallaxRays + 1;
      float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
      if (bStereo1)
        cosParallaxStereo1 = std::cos(2 * std::atan2(mb / 2, kfs_[kf].depth[idx1]));
      else if (bStereo2)
        cosParallaxStereo2 = std::cos(2 * std::atan2(mb / 2, kfs_[k2].depth[idx2]));
      cosParallaxStereo = std::min(cosParallaxStereo1, cosParallaxStereo2);
      float x3D[3];
      if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
          (bStereo1 || bStereo2 || cosParallaxRays < 0.9998)) {
        float A[16];
        for (int c = 0; c < 4; c++) {
          A[0 * 4 + c] = xn1[0] * T1[8 + c] - T1[0 + c];
          A[1 * 4 + c] = xn1[1] * T1[8 + c] - T1[4 + c];
          A[2 * 4 + c] = xn2[0] * T2[8 + c] - T2[0 + c];
          A[3 * 4 + c] = xn2[1] * T2[8 + c] - T2[4 + c];
        }
        float v4[4];
        null_vector4(A, v4);
        if (v4[3] == 0) continue;
        for (int r = 0; r < 3; r++) x3D[r] = (float)((double)v4[r] * (1.0 / (double)v4[3]));
      } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
        unproject(cam_, T1, kp1.x, kp1.y, kfs_[kf].depth[idx1], x3D);
      } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
        unproject(cam_, T2, kp2.x, kp2.y, kfs_[k2].depth[idx2], x3D);
      } else {
        continue;
      }
      auto row_dot = [&](const float* T, int r) {
        double s = 0;
        for (int c = 0; c < 3; c++) s += (double)T[4 * r + c] * (double)x3D[c];
        return (float)(s + (double)T[4 * r + 3]);
      };
      const float z1 = row_dot(T1, 2);
      if (z1 <= 0) continue;
      const float z2 = row_dot(T2, 2);
      if (z2 <= 0) continue;
      const float sc1 = cam_.scale[kp1.octave], sigmaSquare1 = sc1 * sc1;
      const float x1 = row_dot(T1, 0), y1 = row_dot(T1, 1);
      const float invz1 = (float)(1.0 / z1);
      if (!bStereo1) {
        const float u1 = cam_.fx * x1 * invz1 + cam_.cx, v1 = cam_.fy * y1 * invz1 + cam_.cy;
        const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y;
        if ((errX1 * errX1 + errY1 * errY1) > 5.991 * sigmaSquare1) continue;
      } else {
        const float u1 = cam_.fx * x1 * invz1 + cam_.cx;
        const float u1_r = u1 - cam_.bf * invz1;
        const float v1 = cam_.fy * y1 * invz1 + cam_.cy;
        const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y, errX1_r = u1_r - kp1_ur;
        if ((errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * sigmaSquare1) continue;
      }
      const float sc2 = cam_.scale[kp2.octave], sigmaSquare2 = sc2 * sc2;
      const float x2 = row_dot(T2, 0), y2 = row_dot(T2, 1);
      const float invz2 = (float)(1.0 / z2);
      if (!bStereo2) {
        const float u2 = cam_.fx * x2 * invz2 + cam_.cx, v2 = cam_.fy * y2 * invz2 + cam_.cy;
        const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y;
        if ((errX2 * errX2 + errY2 * errY2) > 5.991 * sigmaSquare2) continue;
      } else {
        const float u2 = cam_.fx * x2 * invz2 + cam_.cx;
        const float u2_r = u2 - cam_.bf * invz2;
        const float v2 = cam_.fy * y2 * invz2 + cam_.cy;
        const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y, errX2_r = u2_r - kp2_ur;
        if ((errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * sigmaSquare2) continue;
      }
      const float n1v[3] = {x3D[0] - kfs_[kf].Ow[0], x3D[1] - kfs_[kf].Ow[1], x3D[2] - kfs_[kf].Ow[2]};
      const float n2v[3] = {x3D[0] - kfs_[k2].Ow[0], x3D[1] - kfs_[k2].Ow[1], x3D[2] - kfs_[k2].Ow[2]};
      const float dist1 = norm3(n1v), dist2 = norm3(n2v);
      if (dist1 == 0 || dist2 == 0) continue;
      const float ratioDist = dist2 / dist1;
      const float ratioOctave = cam_.scale[kp1.octave] / cam_.scale[kp2.octave];
      if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) continue;
      const int hnew = new_point_kf(x3D, kf);  // MapPoint(x3D, mpCurrentKeyFrame, mpMap)
      add_observation(hnew, kf, idx1);
      add_observation(hnew, k2, idx2);
      kfs_[kf].mps[idx1] = hnew;
      kfs_[k2].mps[idx2] = hnew;
      compute_distinctive(hnew);
      update_normal_depth(hnew);
      recent_.push_back(hnew);
      bstats_.n_triangulated++;
    }
  }
}

}  // namespace mmt
