// oracle/bowmap_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// The reference's vocabulary-driven map steps, run when the tracker is given a vocabulary
// (System.cc:67; oracle_bow.h for DBoW2 itself):
//   Frame::ComputeBoW / KeyFrame::ComputeBoW        Frame.cc:778-786, KeyFrame.cc:59-68 (levelsup 4)
//   KeyFrameDatabase::add / erase / DetectRelocalizationCandidates  KeyFrameDatabase.cc:40-67,
//                                                   199-309 (add: LoopClosing::DetectLoop's
//                                                   insertion of every keyframe but the first,
//                                                   LoopClosing.cc:92-97, 116-121, 148, 217; erase:
//                                                   KeyFrame::SetBadFlag KeyFrame.cc:544)
//   Tracking::TrackReferenceKeyFrame               Tracking.cc:2836-2892
//   Tracking::Relocalization                       Tracking.cc:3614-3776 (SearchByBoW 0.75,
//                                                   PnPsolver, PoseOptimization, and the
//                                                   SearchByProjection(F, KF, sFound, 10 / 3,
//                                                   100 / 64) rounds below 50 inliers)
//   ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>&, th, ORBdist)
//                                                   ORBmatcher.cc:2104-2231
//   LocalMapping::CreateNewMapPoints + ComputeF12   LocalMapping.cc:210-456, 540-557
//   ORBmatcher::SearchForTriangulation + CheckDistEpipolarLine  ORBmatcher.cc:1032-1198, 513-530
// Pinned choices (the same in the product):
//  * the mapping thread's LoopClosing adds each processed keyframe (but keyframe 0, which
//    LoopClosing::InsertKeyFrame drops) to the database right after its LocalMapping;
//  * rand() (PnPsolver's RandomInt) is the process's unseeded glibc stream, drawn by nothing else;
//  * a relocalisation that computes no pose leaves the frame at the motion model's prediction
//    (the reference's mCurrentFrame.mTcw is empty there);
//  * cv::Mat expressions: products accumulate in double and round to float once, the translation
//    added in float (as elsewhere); ComputeF12 is evaluated in double from the float poses and K
//    and rounded to float once; the 4x4 cv::SVD of the linear triangulation is replaced by the
//    eigenvector of A^T A for the smallest eigenvalue, by cyclic Jacobi in double (OpenCV's
//    float JacobiSVD is not available; the null vector is the same up to rounding and sign, and
//    the sign cancels in x3D / x3D(3)).

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>

#include "oracle_map.h"

namespace oracle {

namespace {
const int TH_LOW = 50, HISTO_LENGTH = 30;

inline void xform(const float* T, const float* x, float* y) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * r + k] * (double)x[k];
    y[r] = (float)s + T[4 * r + 3];
  }
}
inline float logf_pinned(float x) { return (float)std::log((double)x); }

// MapPoint::PredictScale(currentDist, Frame*) MapPoint.cc:402-417
int predict_scale(float maxDist, float dist, const MapCam& cam) {
  const float ratio = maxDist / dist;
  const float ls = logf_pinned(ratio) / cam.logScale;
  int n = std::isfinite(ls) ? (int)std::ceil(ls) : INT_MIN;
  if (n < 0)
    n = 0;
  else if (n >= cam.nlevels)
    n = cam.nlevels - 1;
  return n;
}

// ORBmatcher::ComputeThreeMaxima
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

// the right singular vector of the 4x4 A for its smallest singular value (pinned, header)
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
        for (int k = 0; k < 4; k++) {  // M <- J^T M J
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

// LocalMapping::ComputeF12 (pinned: double from the float poses, one float rounding)
void compute_f12(const float* T1, const float* T2, const MapCam& cam, float F[9]) {
  double R12[3][3], t12[3];
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += (double)T1[4 * r + k] * (double)T2[4 * c + k];
      R12[r][c] = s;
    }
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
  for (int r = 0; r < 3; r++)  // K1^-T [t12]x
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += Ki[k][r] * tx[k][c];
      A[r][c] = s;
    }
  for (int r = 0; r < 3; r++)  // * R12
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += A[r][k] * R12[k][c];
      B[r][c] = s;
    }
  for (int r = 0; r < 3; r++)  // * K2^-1
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += B[r][k] * Ki[k][c];
      F[3 * r + c] = (float)s;
    }
}

// ORBmatcher::CheckDistEpipolarLine
bool check_epipolar(const Key& kp1, const Key& kp2, const float* F, const MapCam& cam) {
  const float a = kp1.x * F[0] + kp1.y * F[3] + F[6];
  const float b = kp1.x * F[1] + kp1.y * F[4] + F[7];
  const float c = kp1.x * F[2] + kp1.y * F[5] + F[8];
  const float num = a * kp2.x + b * kp2.y + c;
  const float den = a * a + b * b;
  if (den == 0) return false;
  const float dsqr = num * num / den;
  const float s = cam.scale[kp2.octave];
  return dsqr < 3.84 * (s * s);
}
}  // namespace

void MapTracker::set_vocabulary(const Vocabulary* v) {
  voc_ = v;
  invfile_.assign(v ? v->words.size() : 0, std::vector<int>());
}

// Frame::ComputeBoW (Frame.cc:778-786): transform(descriptors, mBowVec, mFeatVec, 4)
void MapTracker::compute_bow(const std::vector<uint8_t>& desc, MapFrame& C) {
  if (C.hasBow) return;
  voc_->transform(desc.data(), (int)(desc.size() / 32), 4, C.bow, C.fv);
  C.hasBow = true;
  bstats.n_bow_frames++;
}

void MapTracker::kf_compute_bow(int kf) {  // KeyFrame::ComputeBoW
  OKeyFrame& K = kfs[kf];
  if (K.hasBow) return;
  voc_->transform(K.desc.data(), (int)K.keys.size(), 4, K.bow, K.fv);
  K.hasBow = true;
}

void MapTracker::kfdb_add(int kf) {  // KeyFrameDatabase::add
  for (uint32_t w : kfs[kf].bow.word) invfile_[w].push_back(kf);
  bstats.n_kfdb++;
}

void MapTracker::kfdb_erase(int kf) {  // KeyFrameDatabase::erase
  if (!voc_) return;
  for (uint32_t w : kfs[kf].bow.word) {
    std::vector<int>& l = invfile_[w];
    auto it = std::find(l.begin(), l.end(), kf);
    if (it != l.end()) l.erase(it);
  }
}

// KeyFrameDatabase::DetectRelocalizationCandidates (KeyFrameDatabase.cc:199-309)
std::vector<int> MapTracker::detect_relocalization_candidates(const MapFrame& C) {
  std::vector<int> shared;
  for (uint32_t w : C.bow.word)
    for (int k : invfile_[w]) {
      OKeyFrame& K = kfs[k];
      if (K.relocQuery != C.id) {
        K.relocWords = 0;
        K.relocQuery = C.id;
        shared.push_back(k);
      }
      K.relocWords++;
    }
  if (shared.empty()) return {};
  int maxCommonWords = 0;
  for (int k : shared) maxCommonWords = std::max(maxCommonWords, kfs[k].relocWords);
  const int minCommonWords = (int)(maxCommonWords * 0.8f);
  std::vector<std::pair<float, int>> scored;
  for (int k : shared) {
    OKeyFrame& K = kfs[k];
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
    for (int k2 : best_covisibles(sk.second, 10)) {
      const OKeyFrame& K2 = kfs[k2];
      if (K2.relocQuery != C.id) continue;
      accScore += K2.relocScore;
      if (K2.relocScore > bestScore) {
        bestKF = k2;
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

// Tracking::TrackReferenceKeyFrame (Tracking.cc:2836-2892)
bool MapTracker::track_reference_kf(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                                    MapFrame& C, float* Tcw, const float* Tlast) {
  bstats.n_trk++;
  compute_bow(desc, C);
  const OKeyFrame& K = kfs[refKF_];
  std::vector<uint8_t> ok(K.keys.size());
  for (size_t i = 0; i < K.mps.size(); i++) ok[i] = K.mps[i] >= 0 && !mp(K.mps[i]).bad;
  std::vector<int> match(std::max<size_t>(keys.size(), 1), -1);
  int nmatches = search_by_bow(K.fv.view(), K.keys.data(), K.desc.data(), ok.data(), C.fv.view(),
                               keys.data(), desc.data(), (int)keys.size(), 0.7f, true,
                               match.data());
  if (nmatches < 15) return false;
  for (size_t i = 0; i < keys.size(); i++) C.mps[i] = match[i] >= 0 ? K.mps[match[i]] : -1;
  memcpy(Tcw, Tlast, 64);
  pose_optimization(keys, C, Tcw);
  int nmatchesMap = 0;
  for (size_t i = 0; i < C.mps.size(); i++) {
    if (C.mps[i] < 0) continue;
    if (C.outlier[i]) {
      OMapPoint& p = mp(C.mps[i]);
      C.mps[i] = -1;
      C.outlier[i] = 0;
      p.trackInView = false;
      p.lastFrameSeen = curId_;
      nmatches--;
    } else if (mp(C.mps[i]).nObs > 0) {
      nmatchesMap++;
    }
  }
  if (nmatchesMap >= 10) bstats.n_trk_ok++;
  return nmatchesMap >= 10;
}

// ORBmatcher(0.9, true)::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
// (ORBmatcher.cc:2104-2231)
int MapTracker::search_by_projection_kf(const std::vector<Key>& keys,
                                        const std::vector<uint8_t>& desc, MapFrame& C,
                                        const float* Tcw, int kf, const std::set<int>& found,
                                        float th, int orbDist) {
  MatchFrame G;
  build_grid(keys, desc, C, G);
  float Ow[3];
  cam_centre(Tcw, Ow);
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  const OKeyFrame& K = kfs[kf];
  int nmatches = 0;
  for (size_t i = 0; i < K.mps.size(); i++) {
    const int h = K.mps[i];
    if (h < 0) continue;
    const OMapPoint& p = mp(h);
    if (p.bad || found.count(h)) continue;
    float x3Dc[3];
    xform(Tcw, p.pos, x3Dc);
    const float invzc = (float)(1.0 / x3Dc[2]);
    const float u = cam.fx * x3Dc[0] * invzc + cam.cx;
    const float v = cam.fy * x3Dc[1] * invzc + cam.cy;
    if (u < G.minX || u > G.maxX) continue;
    if (v < G.minY || v > G.maxY) continue;
    const float PO[3] = {p.pos[0] - Ow[0], p.pos[1] - Ow[1], p.pos[2] - Ow[2]};
    const float dist3D = norm3(PO);
    const float maxDistance = 1.2f * p.maxDist, minDistance = 0.8f * p.minDist;
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    const int npl = predict_scale(p.maxDist, dist3D, cam);
    const float radius = th * cam.scale[npl];
    const std::vector<int> idx = features_in_area(G, u, v, radius, npl - 1, npl + 1);
    if (idx.empty()) continue;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : idx) {
      if (C.mps[i2] >= 0) continue;
      const int dist = descriptor_distance(p.desc, desc.data() + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= orbDist) {
      C.mps[bestIdx2] = h;
      nmatches++;
      float rot = K.keys[i].angle - keys[bestIdx2].angle;
      if (rot < 0.0) rot += 360.0f;
      int bin = (int)std::round(rot * factor);
      if (bin == HISTO_LENGTH) bin = 0;
      rotHist[bin].push_back(bestIdx2);
    }
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
bool MapTracker::relocalization(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                                MapFrame& C, float* Tcw) {
  bstats.n_reloc++;
  compute_bow(desc, C);
  const std::vector<int> cands = detect_relocalization_candidates(C);
  if (cands.empty()) return false;
  bstats.n_reloc_cands += (long)cands.size();
  const int nKFs = (int)cands.size();
  const int N = (int)keys.size();
  struct Solver {  // PnPsolver(F, vvpMapPointMatches[i]) with SetRansacParameters(0.99, 10, 300, 4, 0.5, 5.991)
    std::vector<float> p3, p2, s2;
    std::vector<int> kpIdx;
    P4PState st;
  };
  std::vector<Solver> solvers(nKFs);
  std::vector<std::vector<int>> matches(nKFs);
  std::vector<uint8_t> discarded(nKFs, 0);
  int nCandidates = 0;
  for (int i = 0; i < nKFs; i++) {
    const OKeyFrame& K = kfs[cands[i]];
    if (K.bad) {
      discarded[i] = 1;
      continue;
    }
    std::vector<uint8_t> ok(K.keys.size());
    for (size_t j = 0; j < K.mps.size(); j++) ok[j] = K.mps[j] >= 0 && !mp(K.mps[j]).bad;
    std::vector<int> match(std::max(N, 1), -1);
    const int nm = search_by_bow(K.fv.view(), K.keys.data(), K.desc.data(), ok.data(),
                                 C.fv.view(), keys.data(), desc.data(), N, 0.75f, true,
                                 match.data());
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
      if (h < 0 || mp(h).bad) continue;
      S.p2.push_back(keys[j].x);
      S.p2.push_back(keys[j].y);
      const float sc = cam.scale[keys[j].octave];
      S.s2.push_back(sc * sc);
      S.p3.insert(S.p3.end(), mp(h).pos, mp(h).pos + 3);
      S.kpIdx.push_back(j);
    }
    nCandidates++;
  }
  bool bMatch = false;
  while (nCandidates > 0 && !bMatch) {
    for (int i = 0; i < nKFs; i++) {
      if (discarded[i]) continue;
      Solver& S = solvers[i];
      const int n = (int)S.kpIdx.size();
      // iterate(5): the draws of as many iterations as the call can run, from a copy of the
      // stream; the stream then advances by the draws the call used
      const int maxIts = 300 + 5;
      std::vector<int> randi(4 * (size_t)maxIts, 0);
      {
        GlibcRand g = rand_;
        for (int k = 0; k < maxIts; k++)
          for (int j = 0; j < 4; j++) randi[4 * k + j] = n - 1 - j >= 0 ? g.random_int(0, n - 1 - j) : 0;
      }
      const int it0 = S.st.iterations;
      P4PResult r = pnpsolver_iterate(S.p3.data(), S.p2.data(), S.s2.data(), n, cam.fx, cam.fy,
                                      cam.cx, cam.cy, 0.99, 10, 300, 4, 0.5f, 5.991f,
                                      randi.data(), 5, &S.st);
      for (int k = 0; k < 4 * (S.st.iterations - it0); k++) rand_.next();
      if (r.no_more) {
        discarded[i] = 1;
        nCandidates--;
      }
      if (!r.found) continue;
      bstats.n_pnp_found++;
      memcpy(Tcw, r.Tcw, 64);
      std::set<int> sFound;
      std::vector<uint8_t> inl(N, 0);
      for (int q = 0; q < n; q++)
        if (r.mask[q]) inl[S.kpIdx[q]] = 1;
      for (int j = 0; j < N; j++) {
        if (inl[j]) {
          C.mps[j] = matches[i][j];
          sFound.insert(matches[i][j]);
        } else {
          C.mps[j] = -1;
        }
      }
      int nGood = pose_optimization(keys, C, Tcw);
      if (nGood < 10) continue;
      for (int io = 0; io < N; io++)
        if (C.outlier[io]) C.mps[io] = -1;
      if (nGood < 50) {
        bstats.n_sbp_rounds++;
        int nadditional = search_by_projection_kf(keys, desc, C, Tcw, cands[i], sFound, 10, 100);
        if (nadditional + nGood >= 50) {
          nGood = pose_optimization(keys, C, Tcw);
          if (nGood > 30 && nGood < 50) {
            sFound.clear();
            for (int ip = 0; ip < N; ip++)
              if (C.mps[ip] >= 0) sFound.insert(C.mps[ip]);
            bstats.n_sbp_rounds++;
            nadditional = search_by_projection_kf(keys, desc, C, Tcw, cands[i], sFound, 3, 64);
            if (nGood + nadditional >= 50) {
              nGood = pose_optimization(keys, C, Tcw);
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
  if (bMatch) bstats.n_reloc_ok++;
  return bMatch;
}

// ORBmatcher(0.6, false)::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, false)
int MapTracker::search_for_triangulation(int kf1, int kf2, const float* F12,
                                         std::vector<std::pair<int, int>>& pairs) {
  const OKeyFrame& K1 = kfs[kf1];
  const OKeyFrame& K2 = kfs[kf2];
  float C2[3];
  xform(K2.Tcw, K1.Ow, C2);
  const float invz = 1.0f / C2[2];
  const float ex = cam.fx * C2[0] * invz + cam.cx;
  const float ey = cam.fy * C2[1] * invz + cam.cy;
  std::vector<int> m12(K1.keys.size(), -1);
  int nmatches = 0;
  const FeatVecO& f1 = K1.fv;
  const FeatVecO& f2 = K2.fv;
  size_t a = 0, b = 0;
  while (a < f1.node.size() && b < f2.node.size()) {
    if (f1.node[a] == f2.node[b]) {
      for (int p = f1.start[a]; p < f1.start[a + 1]; p++) {
        const int idx1 = f1.feat[p];
        if (K1.mps[idx1] >= 0) continue;
        const bool bStereo1 = K1.uR[idx1] >= 0;
        const Key& kp1 = K1.keys[idx1];
        const uint8_t* d1 = K1.desc.data() + 32 * (size_t)idx1;
        int bestDist = TH_LOW, bestIdx2 = -1;
        for (int q = f2.start[b]; q < f2.start[b + 1]; q++) {
          const int idx2 = f2.feat[q];
          if (K2.mps[idx2] >= 0) continue;  // vbMatched2 is never set (ORBmatcher.cc:1100)
          const bool bStereo2 = K2.uR[idx2] >= 0;
          const int dist = descriptor_distance(d1, K2.desc.data() + 32 * (size_t)idx2);
          if (dist > TH_LOW || dist > bestDist) continue;
          const Key& kp2 = K2.keys[idx2];
          if (!bStereo1 && !bStereo2) {
            const float distex = ex - kp2.x, distey = ey - kp2.y;
            if (distex * distex + distey * distey < 100 * cam.scale[kp2.octave]) continue;
          }
          if (check_epipolar(kp1, kp2, F12, cam)) {
            bestIdx2 = idx2;
            bestDist = dist;
          }
        }
        if (bestIdx2 >= 0) {
          m12[idx1] = bestIdx2;
          nmatches++;
        }
      }
      a++;
      b++;
    } else if (f1.node[a] < f2.node[b]) {
      a = (size_t)(std::lower_bound(f1.node.begin(), f1.node.end(), f2.node[b]) - f1.node.begin());
    } else {
      b = (size_t)(std::lower_bound(f2.node.begin(), f2.node.end(), f1.node[a]) - f2.node.begin());
    }
  }
  pairs.clear();
  for (size_t i = 0; i < m12.size(); i++)
    if (m12[i] >= 0) pairs.push_back({(int)i, m12[i]});
  return nmatches;
}

// LocalMapping::CreateNewMapPoints (LocalMapping.cc:210-456), RGB-D branch
void MapTracker::create_new_map_points(int kf) {
  const std::vector<int> neigh = best_covisibles(kf, 10);
  const float ratioFactor = 1.5f * cam.scale[1];
  const float mb = cam.bf / cam.fx;  // Frame::mb = mbf / fx
  for (int k2 : neigh) {
    const OKeyFrame& K1 = kfs[kf];
    const OKeyFrame& K2 = kfs[k2];
    const float vB[3] = {K2.Ow[0] - K1.Ow[0], K2.Ow[1] - K1.Ow[1], K2.Ow[2] - K1.Ow[2]};
    const float baseline = norm3(vB);
    if (baseline < mb) continue;
    float F12[9];
    compute_f12(K1.Tcw, K2.Tcw, cam, F12);
    std::vector<std::pair<int, int>> pairs;
    bstats.n_sft_matches += search_for_triangulation(kf, k2, F12, pairs);
    const float* T1 = K1.Tcw;
    const float* T2 = K2.Tcw;
    for (const auto& pr : pairs) {
      const int idx1 = pr.first, idx2 = pr.second;
      const Key& kp1 = kfs[kf].keys[idx1];
      const float kp1_ur = kfs[kf].uR[idx1];
      const bool bStereo1 = kp1_ur >= 0;
      const Key& kp2 = kfs[k2].keys[idx2];
      const float kp2_ur = kfs[k2].uR[idx2];
      const bool bStereo2 = kp2_ur >= 0;
      const float xn1[3] = {(kp1.x - cam.cx) * cam.invfx, (kp1.y - cam.cy) * cam.invfy, 1.0f};
      const float xn2[3] = {(kp2.x - cam.cx) * cam.invfx, (kp2.y - cam.cy) * cam.invfy, 1.0f};
      float ray1[3], ray2[3];
      for (int r = 0; r < 3; r++) {  // Rwc * xn
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
        cosParallaxStereo1 = std::cos(2 * std::atan2(mb / 2, kfs[kf].depth[idx1]));
      else if (bStereo2)
        cosParallaxStereo2 = std::cos(2 * std::atan2(mb / 2, kfs[k2].depth[idx2]));
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
        unproject(cam, T1, kp1.x, kp1.y, kfs[kf].depth[idx1], x3D);
      } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
        unproject(cam, T2, kp2.x, kp2.y, kfs[k2].depth[idx2], x3D);
      } else {
        continue;
      }
      auto row_dot = [&](const float* T, int r) {  // Rcw.row(r).dot(x3D) + t(r), in double
        double s = 0;
        for (int c = 0; c < 3; c++) s += (double)T[4 * r + c] * (double)x3D[c];
        return (float)(s + (double)T[4 * r + 3]);
      };
      const float z1 = row_dot(T1, 2);
      if (z1 <= 0) continue;
      const float z2 = row_dot(T2, 2);
      if (z2 <= 0) continue;
      const float s1 = cam.scale[kp1.octave], sigmaSquare1 = s1 * s1;
      const float x1 = row_dot(T1, 0), y1 = row_dot(T1, 1);
      const float invz1 = (float)(1.0 / z1);
      if (!bStereo1) {
        const float u1 = cam.fx * x1 * invz1 + cam.cx, v1 = cam.fy * y1 * invz1 + cam.cy;
        const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y;
        if ((errX1 * errX1 + errY1 * errY1) > 5.991 * sigmaSquare1) continue;
      } else {
        const float u1 = cam.fx * x1 * invz1 + cam.cx;
        const float u1_r = u1 - cam.bf * invz1;
        const float v1 = cam.fy * y1 * invz1 + cam.cy;
        const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y, errX1_r = u1_r - kp1_ur;
        if ((errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * sigmaSquare1) continue;
      }
      const float s2 = cam.scale[kp2.octave], sigmaSquare2 = s2 * s2;
      const float x2 = row_dot(T2, 0), y2 = row_dot(T2, 1);
      const float invz2 = (float)(1.0 / z2);
      if (!bStereo2) {
        const float u2 = cam.fx * x2 * invz2 + cam.cx, v2 = cam.fy * y2 * invz2 + cam.cy;
        const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y;
        if ((errX2 * errX2 + errY2 * errY2) > 5.991 * sigmaSquare2) continue;
      } else {
        const float u2 = cam.fx * x2 * invz2 + cam.cx;
        const float u2_r = u2 - cam.bf * invz2;
        const float v2 = cam.fy * y2 * invz2 + cam.cy;
        const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y, errX2_r = u2_r - kp2_ur;
        if ((errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * sigmaSquare2) continue;
      }
      const float n1v[3] = {x3D[0] - kfs[kf].Ow[0], x3D[1] - kfs[kf].Ow[1], x3D[2] - kfs[kf].Ow[2]};
      const float n2v[3] = {x3D[0] - kfs[k2].Ow[0], x3D[1] - kfs[k2].Ow[1], x3D[2] - kfs[k2].Ow[2]};
      const float dist1 = norm3(n1v), dist2 = norm3(n2v);
      if (dist1 == 0 || dist2 == 0) continue;
      const float ratioDist = dist2 / dist1;
      const float ratioOctave = cam.scale[kp1.octave] / cam.scale[kp2.octave];
      if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) continue;
      // MapPoint(x3D, mpCurrentKeyFrame, mpMap)
      const int h = new_point_kf(x3D, kf);
      add_observation(h, kf, idx1);
      add_observation(h, k2, idx2);
      kfs[kf].mps[idx1] = h;
      kfs[k2].mps[idx2] = h;
      compute_distinctive(h);
      update_normal_depth(h);
      recent_.push_back(h);
      bstats.n_triangulated++;
    }
  }
}

}  // namespace oracle
