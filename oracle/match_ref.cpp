// oracle/match_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// Scalar restatement of the frame grid (B3) and the projection matchers (C1-C3) of the reference,
// written in the reference's own iteration order so that the order-dependent parts (a key bound to
// a MapPoint by an earlier point is skipped by later ones; the first of equal distances wins) are
// reproduced literally.  cv::Mat float products are pinned as elsewhere in the oracle (double
// accumulation rounded to float, the translation added in float); cv::norm / Mat::dot accumulate
// in double.  MapPoint::PredictScale's log() is pinned as log in double rounded to float (glibc's
// logf is within 0.52 ulp of that).

#include <algorithm>
#include <cstdlib>
#include <climits>
#include <cmath>
#include <cstring>

#include "oracle_match.h"

namespace oracle {

static const int TH_HIGH = 100;      // ORBmatcher.cc:41
static const int HISTO_LENGTH = 30;  // ORBmatcher.cc:43

static inline float logf_pinned(float x) { return (float)std::log((double)x); }

// Frame::ComputeStereoFromRGBD (Frame.cc:1041-1062), ComputeImageBounds without distortion
// (Frame.cc:841-846), grid element sizes (Frame.cc:581-584), AssignFeaturesToGrid + PosInGrid
// (Frame.cc:601-616, 765-775).
void frame_stereo_grid(MatchFrame& F, const float* depth, int W, int H) {
  F.uR.assign(F.n, -1.f);
  F.depth.assign(F.n, -1.f);
  // ORACLE_ABLATE bit 4 (diagnostics only, tools/drift_ablation.py): the depth at the nearest
  // pixel instead of the truncated one
  static const bool nearest = [] {
    const char* e = getenv("ORACLE_ABLATE");
    return e && (atoi(e) & 4);
  }();
  for (int i = 0; i < F.n; i++) {
    const float v = F.keys[i].y, u = F.keys[i].x;
    const int iv = nearest ? std::min(H - 1, (int)std::lround(v)) : (int)v;
    const int iu = nearest ? std::min(W - 1, (int)std::lround(u)) : (int)u;
    const float d = depth[(size_t)iv * W + iu];  // at<float>(v,u): float -> int truncation
    if (d > 0) {
      F.depth[i] = d;
      F.uR[i] = F.keys[i].x - F.bf / d;
    }
  }
  F.minX = 0.0f;
  F.maxX = (float)W;
  F.minY = 0.0f;
  F.maxY = (float)H;
  F.invW = static_cast<float>(kGridCols) / static_cast<float>(F.maxX - F.minX);
  F.invH = static_cast<float>(kGridRows) / static_cast<float>(F.maxY - F.minY);
  F.grid.assign(kGridCols * kGridRows, std::vector<int>());
  for (int i = 0; i < F.n; i++) {
    const int posX = (int)std::round((F.keys[i].x - F.minX) * F.invW);
    const int posY = (int)std::round((F.keys[i].y - F.minY) * F.invH);
    if (posX < 0 || posX >= kGridCols || posY < 0 || posY >= kGridRows) continue;
    F.grid[posX * kGridRows + posY].push_back(i);
  }
}

// Frame::GetFeaturesInArea (Frame.cc:711-758).
std::vector<int> features_in_area(const MatchFrame& F, float x, float y, float r, int minLevel,
                                  int maxLevel) {
  std::vector<int> out;
  // a non-finite window centre (a map point unprojected from depth +inf) gives no cell: the
  // reference's float -> int conversions are undefined there, x86 yields INT_MIN and an empty range
  if (!std::isfinite(x) || !std::isfinite(y)) return out;
  const int nMinCellX = std::max(0, (int)std::floor((x - F.minX - r) * F.invW));
  if (nMinCellX >= kGridCols) return out;
  const int nMaxCellX = std::min(kGridCols - 1, (int)std::ceil((x - F.minX + r) * F.invW));
  if (nMaxCellX < 0) return out;
  const int nMinCellY = std::max(0, (int)std::floor((y - F.minY - r) * F.invH));
  if (nMinCellY >= kGridRows) return out;
  const int nMaxCellY = std::min(kGridRows - 1, (int)std::ceil((y - F.minY + r) * F.invH));
  if (nMaxCellY < 0) return out;
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
      for (int k : F.grid[ix * kGridRows + iy]) {
        const Key& kp = F.keys[k];
        if (bCheckLevels) {
          if (kp.octave < minLevel) continue;
          if (maxLevel >= 0 && kp.octave > maxLevel) continue;
        }
        const float distx = kp.x - x, disty = kp.y - y;
        if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(k);
      }
    }
  return out;
}

// ORBmatcher::DescriptorDistance (ORBmatcher.cc:2279-2295): popcount of the XOR of 8 words.
int descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t wa, wb;
    memcpy(&wa, a + 4 * i, 4);
    memcpy(&wb, b + 4 * i, 4);
    uint32_t v = wa ^ wb;
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return dist;
}

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:2236-2275).
static void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
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

// R*x + t of a row-major 4x4 float pose (cv::Mat gemm pin, see header).
static inline void xform(const float* T, const float* x, float* y) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * r + k] * (double)x[k];
    y[r] = (float)s + T[4 * r + 3];
  }
}
// -R^T t (camera centre), Frame::UpdatePoseMatrices mOw (Frame.cc:644-650).
static inline void centre(const float* T, float* o) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    o[r] = (float)(-s);
  }
}

int search_by_projection_frame(const MatchFrame& C, const float* Tcw, const LastFrameView& L,
                               float th, bool mono, bool check_orientation, int* match) {
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  for (int i = 0; i < C.n; i++) match[i] = -1;
  std::vector<uint8_t> taken(C.n, 0);  // bound to a MapPoint with Observations() > 0
  float twc[3], tlc[3];
  centre(Tcw, twc);
  xform(L.Tcw, twc, tlc);
  const float mb = C.bf / C.fx;
  const bool bForward = tlc[2] > mb && !mono;
  const bool bBackward = -tlc[2] > mb && !mono;
  for (int i = 0; i < L.n; i++) {
    if (!L.active[i]) continue;
    float x3Dc[3];
    xform(Tcw, L.Xw + 3 * i, x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / (double)x3Dc[2]);
    if (invzc < 0) continue;
    const float u = C.fx * xc * invzc + C.cx;
    const float v = C.fy * yc * invzc + C.cy;
    if (u < C.minX || u > C.maxX) continue;
    if (v < C.minY || v > C.maxY) continue;
    const int nLastOctave = L.keys[i].octave;
    const float radius = th * C.scale[nLastOctave];
    std::vector<int> idx2;
    if (bForward)
      idx2 = features_in_area(C, u, v, radius, nLastOctave, -1);
    else if (bBackward)
      idx2 = features_in_area(C, u, v, radius, 0, nLastOctave);
    else
      idx2 = features_in_area(C, u, v, radius, nLastOctave - 1, nLastOctave + 1);
    if (idx2.empty()) continue;
    const uint8_t* dMP = L.mp_desc + 32 * (size_t)i;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : idx2) {
      if (taken[i2]) continue;  // mvpMapPoints[i2] with Observations() > 0
      if (C.uR[i2] > 0) {
        const float ur = u - C.bf * invzc;
        const float er = std::fabs(ur - C.uR[i2]);
        if (er > radius) continue;
      }
      const int dist = descriptor_distance(dMP, C.desc + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= TH_HIGH) {
      match[bestIdx2] = i;
      if (!L.obs || L.obs[i]) taken[bestIdx2] = 1;
      nmatches++;
      if (check_orientation) {
        float rot = L.keys[i].angle - C.keys[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rotHist[bin].push_back(bestIdx2);
      }
    }
  }
  if (check_orientation) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int k : rotHist[i]) {
        match[k] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

bool is_in_frustum(const MatchFrame& F, const float* Tcw, const LocalPoint& p,
                   float viewing_cos_limit, FrustumOut& o) {
  o.in_view = 0;
  float Pc[3];
  xform(Tcw, p.Xw, Pc);
  if (Pc[2] < 0.0f) return false;
  const float invz = 1.0f / Pc[2];
  const float u = F.fx * Pc[0] * invz + F.cx;
  const float v = F.fy * Pc[1] * invz + F.cy;
  if (u < F.minX || u > F.maxX) return false;
  if (v < F.minY || v > F.maxY) return false;
  const float maxDistance = 1.2f * p.max_dist;  // MapPoint::GetMaxDistanceInvariance
  const float minDistance = 0.8f * p.min_dist;  // MapPoint::GetMinDistanceInvariance
  float Ow[3], PO[3];
  centre(Tcw, Ow);
  double n2 = 0, dot = 0;
  for (int k = 0; k < 3; k++) {
    PO[k] = p.Xw[k] - Ow[k];
    n2 += (double)PO[k] * (double)PO[k];
  }
  const float dist = (float)std::sqrt(n2);
  if (dist < minDistance || dist > maxDistance) return false;
  for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)p.normal[k];
  const float viewCos = (float)(dot / (double)dist);
  if (viewCos < viewing_cos_limit) return false;
  // MapPoint::PredictScale (MapPoint.cc:402-417)
  const float ratio = p.max_dist / dist;
  // (int)ceil of a non-finite value (a NaN point): INT_MIN on x86, which clamps to level 0
  const float ls = logf_pinned(ratio) / F.logScale;
  int nScale = std::isfinite(ls) ? (int)std::ceil(ls) : INT_MIN;
  if (nScale < 0)
    nScale = 0;
  else if (nScale >= F.nlevels)
    nScale = F.nlevels - 1;
  o.in_view = 1;
  o.u = u;
  o.uR = u - F.bf * invz;
  o.v = v;
  o.level = nScale;
  o.view_cos = viewCos;
  return true;
}

int search_local_points(const MatchFrame& C, const float* Tcw, const LocalPoint* pts, int m,
                        float th, const uint8_t* taken, int* match, FrustumOut* fr) {
  std::vector<FrustumOut> own;
  if (!fr) {
    own.resize(m);
    fr = own.data();
  }
  std::vector<uint8_t> bound(taken, taken + C.n);
  for (int i = 0; i < C.n; i++) match[i] = -1;
  int nToMatch = 0;
  for (int j = 0; j < m; j++) {
    fr[j] = FrustumOut{0, 0, 0, 0, 0, 0};
    if (pts[j].skip) continue;
    if (is_in_frustum(C, Tcw, pts[j], 0.5f, fr[j])) nToMatch++;
  }
  if (nToMatch == 0) return 0;
  const bool bFactor = th != 1.0;
  const float nnratio = 0.8f;
  int nmatches = 0;
  for (int j = 0; j < m; j++) {
    const FrustumOut& o = fr[j];
    if (!o.in_view) continue;
    const int lvl = o.level;
    float r = ((double)o.view_cos > 0.998) ? 2.5f : 4.0f;  // RadiusByViewingCos
    if (bFactor) r *= th;
    const std::vector<int> idx = features_in_area(C, o.u, o.v, r * C.scale[lvl], lvl - 1, lvl);
    if (idx.empty()) continue;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int k : idx) {
      if (bound[k]) continue;
      if (C.uR[k] > 0) {
        const float er = std::fabs(o.uR - C.uR[k]);
        if (er > r * C.scale[lvl]) continue;
      }
      const int dist = descriptor_distance(pts[j].desc, C.desc + 32 * (size_t)k);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = C.keys[k].octave;
        bestIdx = k;
      } else if (dist < bestDist2) {
        bestLevel2 = C.keys[k].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_HIGH) {
      if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
      bound[bestIdx] = 1;
      match[bestIdx] = j;
      nmatches++;
    }
  }
  return nmatches;
}

// C4: ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) ORBmatcher.cc:532-663, literally: the two
// feature vectors are walked in node order (equal ids: match the node; otherwise lower_bound the
// lagging side), inside a node every keyframe feature with a good MapPoint takes the closest frame
// feature not matched yet (strict '<', so the first of equal distances), accepted at
// bestDist1 <= TH_LOW and bestDist1 < nnratio * bestDist2 (floats); then the rotation histogram.
static const int TH_LOW = 50;  // ORBmatcher.cc:42

static int fv_lower_bound(const FeatVec& v, uint32_t id) {
  return (int)(std::lower_bound(v.node, v.node + v.n_nodes, id) - v.node);
}

int search_by_bow(const FeatVec& kfv, const Key* kf_keys, const uint8_t* kf_desc,
                  const uint8_t* kf_mp_ok, const FeatVec& fv, const Key* f_keys,
                  const uint8_t* f_desc, int nF, float nnratio, bool check_orientation,
                  int* match) {
  for (int i = 0; i < nF; i++) match[i] = -1;  // vpMapPointMatches = vector(F.N, NULL)
  int nmatches = 0;
  std::vector<int> rotHist[HISTO_LENGTH];
  const float factor = 1.0f / HISTO_LENGTH;
  int ki = 0, fi = 0;
  while (ki < kfv.n_nodes && fi < fv.n_nodes) {
    if (kfv.node[ki] == fv.node[fi]) {
      for (int a = kfv.start[ki]; a < kfv.start[ki + 1]; a++) {
        const int realIdxKF = kfv.feat[a];
        if (!kf_mp_ok[realIdxKF]) continue;
        const uint8_t* dKF = kf_desc + 32 * (size_t)realIdxKF;
        int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
        for (int b = fv.start[fi]; b < fv.start[fi + 1]; b++) {
          const int realIdxF = fv.feat[b];
          if (match[realIdxF] >= 0) continue;
          const int dist = descriptor_distance(dKF, f_desc + 32 * (size_t)realIdxF);
          if (dist < bestDist1) {
            bestDist2 = bestDist1;
            bestDist1 = dist;
            bestIdxF = realIdxF;
          } else if (dist < bestDist2) {
            bestDist2 = dist;
          }
        }
        if (bestDist1 <= TH_LOW) {
          if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
            match[bestIdxF] = realIdxKF;
            if (check_orientation) {
              float rot = kf_keys[realIdxKF].angle - f_keys[bestIdxF].angle;
              if (rot < 0.0) rot += 360.0f;
              int bin = (int)std::round(rot * factor);
              if (bin == HISTO_LENGTH) bin = 0;
              rotHist[bin].push_back(bestIdxF);
            }
            nmatches++;
          }
        }
      }
      ki++;
      fi++;
    } else if (kfv.node[ki] < fv.node[fi]) {
      ki = fv_lower_bound(kfv, fv.node[fi]);
    } else {
      fi = fv_lower_bound(fv, kfv.node[ki]);
    }
  }
  if (check_orientation) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int j : rotHist[i]) {
        match[j] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

}  // namespace oracle
