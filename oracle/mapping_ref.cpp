// oracle/mapping_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// The steps of LocalMapping::Run that follow ProcessNewKeyFrame / MapPointCulling
// (src/LocalMapping.cc:68-87), run synchronously on every new keyframe:
//   SearchInNeighbors            LocalMapping.cc:458-538 with ORBmatcher::Fuse(pKF, vpMapPoints, 3)
//                                ORBmatcher.cc:1200-1350 and MapPoint::Replace MapPoint.cc:177-215
//   LocalBundleAdjustment        Optimizer.cc:3341-3666 (graph set-up, erase, recovery here; the
//                                solve in ba_ref.cpp) when the map holds more than 2 keyframes
//   KeyFrameCulling              LocalMapping.cc:636-700 with KeyFrame::SetBadFlag KeyFrame.cc:453-545
// and the bookkeeping they use: MapPoint::EraseObservation (MapPoint.cc:111-137),
// KeyFrame::EraseConnection / GetBestCovisibilityKeyFrames / GetFeaturesInArea / SetPose
// (KeyFrame.cc:553-608, 174-182, 70-84).  cv::Mat float arithmetic as in map_ref.cpp.  Containers
// keyed by KeyFrame* / MapPoint* iterate in creation order (oracle_map.h).

#include <cstdlib>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>

#include "oracle_map.h"

namespace oracle {

namespace {
// R * x + t of a row-major float pose (double accumulation rounded to float, t added in float)
inline void xform(const float* T, const float* x, float* y) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * r + k] * (double)x[k];
    y[r] = (float)s + T[4 * r + 3];
  }
}
inline float logf_pinned(float x) { return (float)std::log((double)x); }
}  // namespace

// ------------------------------------------------------------------ KeyFrame / MapPoint helpers
void MapTracker::set_pose(int kf, const float* T) {  // KeyFrame::SetPose
  OKeyFrame& K = kfs[kf];
  memcpy(K.Tcw, T, 64);
  cam_centre(T, K.Ow);
  for (int i = 0; i < 16; i++) K.Twc[i] = (i % 5 == 0) ? 1.f : 0.f;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) K.Twc[4 * r + c] = T[4 * c + r];
    K.Twc[4 * r + 3] = K.Ow[r];
  }
}

std::vector<int> MapTracker::best_covisibles(int kf, int n) const {
  const std::vector<int>& o = kfs[kf].ordered;
  return std::vector<int>(o.begin(), o.begin() + std::min<size_t>(o.size(), (size_t)n));
}

// KeyFrame::GetFeaturesInArea (KeyFrame.cc:569-608): no level filter
std::vector<int> kf_features_in_area(const OKeyFrame& K, const MapCam& cam, float x, float y,
                                     float r) {
  std::vector<int> out;
  if (!std::isfinite(x) || !std::isfinite(y)) return out;
  const float invW = (float)kGridCols / (float)cam.W, invH = (float)kGridRows / (float)cam.H;
  const int nMinCellX = std::max(0, (int)std::floor((x - 0.f - r) * invW));
  if (nMinCellX >= kGridCols) return out;
  const int nMaxCellX = std::min(kGridCols - 1, (int)std::ceil((x - 0.f + r) * invW));
  if (nMaxCellX < 0) return out;
  const int nMinCellY = std::max(0, (int)std::floor((y - 0.f - r) * invH));
  if (nMinCellY >= kGridRows) return out;
  const int nMaxCellY = std::min(kGridRows - 1, (int)std::ceil((y - 0.f + r) * invH));
  if (nMaxCellY < 0) return out;
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
      for (int k : K.grid[ix * kGridRows + iy]) {
        const float distx = K.keys[k].x - x, disty = K.keys[k].y - y;
        if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(k);
      }
  return out;
}

// ORBmatcher::Fuse's search for one point (ORBmatcher.cc:1227-1324): returns bestDist (256: none)
int fuse_candidate(const OKeyFrame& K, const MapCam& cam, const OMapPoint& p, float th,
                   int* bestIdxOut) {
  *bestIdxOut = -1;
  const float* Tcw = K.Tcw;
  const float* Ow = K.Ow;
  float p3Dc[3];
  xform(Tcw, p.pos, p3Dc);
  if (p3Dc[2] < 0.0f) return 256;
  const float invz = 1 / p3Dc[2];
  const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
  const float u = cam.fx * x + cam.cx, v = cam.fy * y + cam.cy;
  if (!(u >= 0.f && u < (float)cam.W && v >= 0.f && v < (float)cam.H)) return 256;  // IsInImage
  const float ur = u - cam.bf * invz;
  const float maxDistance = 1.2f * p.maxDist, minDistance = 0.8f * p.minDist;
  const float PO[3] = {p.pos[0] - Ow[0], p.pos[1] - Ow[1], p.pos[2] - Ow[2]};
  const float dist3D = norm3(PO);
  if (dist3D < minDistance || dist3D > maxDistance) return 256;
  double dot = 0;
  for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)p.normal[k];
  if (dot < 0.5 * dist3D) return 256;
  // MapPoint::PredictScale(dist3D, pKF)
  const float ratio = p.maxDist / dist3D;
  const float ls = logf_pinned(ratio) / cam.logScale;
  int npl = std::isfinite(ls) ? (int)std::ceil(ls) : INT_MIN;
  if (npl < 0)
    npl = 0;
  else if (npl >= cam.nlevels)
    npl = cam.nlevels - 1;
  const float radius = th * cam.scale[npl];
  const std::vector<int> idx = kf_features_in_area(K, cam, u, v, radius);
  int bestDist = 256, bestIdx = -1;
  for (int i : idx) {
    const Key& kp = K.keys[i];
    const int kpLevel = kp.octave;
    if (kpLevel < npl - 1 || kpLevel > npl) continue;
    const float ex = u - kp.x, ey = v - kp.y;
    if (K.uR[i] >= 0) {
      const float er = ur - K.uR[i];
      const float e2 = ex * ex + ey * ey + er * er;
      if (e2 * cam.invSigma2[kpLevel] > 7.8) continue;
    } else {
      const float e2 = ex * ex + ey * ey;
      if (e2 * cam.invSigma2[kpLevel] > 5.99) continue;
    }
    const int dist = descriptor_distance(p.desc, K.desc.data() + 32 * (size_t)i);
    if (dist < bestDist) {
      bestDist = dist;
      bestIdx = i;
    }
  }
  *bestIdxOut = bestIdx;
  return bestDist;
}

void MapTracker::erase_observation(int h, int kf) {  // MapPoint::EraseObservation
  OMapPoint& p = mp(h);
  auto it = p.obs.find(kf);
  if (it == p.obs.end()) return;
  const int idx = it->second;
  if (kfs[kf].uR[idx] >= 0)
    p.nObs -= 2;
  else
    p.nObs--;
  p.obs.erase(it);
  // mObservations.begin() of an emptied map is undefined in the reference; the point is set bad
  // right below in that case (nObs <= 2)
  if (p.refKF == kf) p.refKF = p.obs.empty() ? -1 : p.obs.begin()->first;
  if (p.nObs <= 2) set_bad(h);
}

void MapTracker::replace(int h, int by) {  // MapPoint::Replace (this = h, pMP = by)
  if (h == by) return;
  OMapPoint& p = mp(h);
  const std::map<int, int> obs = p.obs;
  p.obs.clear();
  p.bad = true;
  const int nvisible = p.visible, nfound = p.found;
  p.replaced = by;
  for (const auto& kv : obs) {
    if (!mp(by).obs.count(kv.first)) {
      kfs[kv.first].mps[kv.second] = by;  // KeyFrame::ReplaceMapPointMatch
      add_observation(by, kv.first, kv.second);
    } else {
      kfs[kv.first].mps[kv.second] = -1;  // KeyFrame::EraseMapPointMatch(idx)
    }
  }
  mp(by).found += nfound;
  mp(by).visible += nvisible;
  compute_distinctive(by);
}

void MapTracker::erase_connection(int kf, int other) {  // KeyFrame::EraseConnection
  OKeyFrame& K = kfs[kf];
  if (K.conn.erase(other)) update_best_covisibles(kf);
}

void MapTracker::kf_set_bad(int kf) {  // KeyFrame::SetBadFlag (mbNotErase is never set here)
  OKeyFrame& K = kfs[kf];
  if (K.id == 0) return;
  for (const auto& kv : std::map<int, int>(K.conn)) erase_connection(kv.first, kf);
  for (size_t i = 0; i < K.mps.size(); i++)
    if (K.mps[i] >= 0) erase_observation(K.mps[i], kf);
  K.conn.clear();
  K.ordered.clear();
  K.orderedW.clear();
  // spanning tree: each round re-parents the child with the strongest link to a candidate
  std::set<int> cand;
  cand.insert(K.parent);
  while (!K.children.empty()) {
    bool bContinue = false;
    int mx = -1, pC = -1, pP = -1;
    for (int ch : K.children) {
      if (kfs[ch].bad) continue;
      for (int c : kfs[ch].ordered)
        for (int q : cand)
          if (c == q) {
            auto it = kfs[ch].conn.find(c);  // GetWeight
            const int w = it == kfs[ch].conn.end() ? 0 : it->second;
            if (w > mx) {
              pC = ch;
              pP = c;
              mx = w;
              bContinue = true;
            }
          }
    }
    if (!bContinue) break;
    kfs[pC].parent = pP;  // ChangeParent
    kfs[pP].children.insert(pC);
    mstats.n_reparent++;
    cand.insert(pC);
    K.children.erase(pC);
  }
  if (K.parent >= 0) {
    for (int ch : K.children) {
      kfs[ch].parent = K.parent;
      kfs[K.parent].children.insert(ch);
      mstats.n_reparent++;
    }
    kfs[K.parent].children.erase(kf);
  }
  K.bad = true;
  kfdb_erase(kf);  // mpKeyFrameDB->erase(this) (KeyFrame.cc:544)
}

// ------------------------------------------------------------------ ORBmatcher::Fuse
int MapTracker::fuse(int kf, const std::vector<int>& P, float th) {
  OKeyFrame& K = kfs[kf];
  int nFused = 0;
  for (int h : P) {
    if (h < 0) continue;
    OMapPoint& p = mp(h);
    if (p.bad || p.obs.count(kf)) continue;
    int bestIdx;
    const int bestDist = fuse_candidate(K, cam, p, th, &bestIdx);
    if (bestDist <= 50) {  // TH_LOW
      const int pin = K.mps[bestIdx];
      if (pin >= 0) {
        if (!mp(pin).bad) {
          if (mp(pin).nObs > p.nObs)
            replace(h, pin);
          else
            replace(pin, h);
        }
      } else {
        add_observation(h, kf, bestIdx);
        K.mps[bestIdx] = h;
      }
      nFused++;
    }
  }
  return nFused;
}

// ------------------------------------------------------------------ LocalMapping
void MapTracker::search_in_neighbors(int kf) {  // LocalMapping::SearchInNeighbors (RGB-D: nn 10)
  const long cur = kfs[kf].id;
  std::vector<int> targets;
  for (int k : best_covisibles(kf, 10)) {
    OKeyFrame& Ki = kfs[k];
    if (Ki.bad || Ki.fuseTargetForKF == cur) continue;
    targets.push_back(k);
    Ki.fuseTargetForKF = cur;
    for (int k2 : best_covisibles(k, 5)) {
      const OKeyFrame& K2 = kfs[k2];
      if (K2.bad || K2.fuseTargetForKF == cur || K2.id == cur) continue;
      targets.push_back(k2);
    }
  }
  const std::vector<int> matches = kfs[kf].mps;
  for (int t : targets) mstats.n_fused += fuse(t, matches, 3.f);
  std::vector<int> cands;
  for (int t : targets) {
    const std::vector<int> mps = kfs[t].mps;
    for (int h : mps) {
      if (h < 0) continue;
      OMapPoint& p = mp(h);
      if (p.bad || p.fuseCandForKF == cur) continue;
      p.fuseCandForKF = cur;
      cands.push_back(h);
    }
  }
  mstats.n_fused += fuse(kf, cands, 3.f);
  const std::vector<int> now = kfs[kf].mps;
  for (int h : now) {
    if (h < 0 || mp(h).bad) continue;
    compute_distinctive(h);
    update_normal_depth(h);
  }
  update_connections(kf);
}

void MapTracker::local_bundle_adjustment(int kf) {  // Optimizer::LocalBundleAdjustment
  const long cur = kfs[kf].id;
  std::vector<int> local{kf};
  kfs[kf].baLocalForKF = cur;
  for (int k : kfs[kf].ordered) {  // GetVectorCovisibleKeyFrames
    kfs[k].baLocalForKF = cur;
    if (!kfs[k].bad) local.push_back(k);
  }
  std::vector<int> lpts;
  for (int k : local)
    for (int h : std::vector<int>(kfs[k].mps)) {
      if (h < 0) continue;
      OMapPoint& p = mp(h);
      if (p.bad || p.baLocalForKF == cur) continue;
      lpts.push_back(h);
      p.baLocalForKF = cur;
    }
  std::vector<int> fixedKFs;
  for (int h : lpts)
    for (const auto& kv : mp(h).obs) {
      OKeyFrame& Ki = kfs[kv.first];
      if (Ki.baLocalForKF != cur && Ki.baFixedForKF != cur) {
        Ki.baFixedForKF = cur;
        if (!Ki.bad) fixedKFs.push_back(kv.first);
      }
    }
  // the graph: local keyframes (KF 0 fixed), fixed keyframes, points, edges
  std::vector<int> verts = local;
  verts.insert(verts.end(), fixedKFs.begin(), fixedKFs.end());
  std::map<int, int> vIdx;
  std::vector<float> T(16 * verts.size());
  std::vector<uint8_t> fixed(verts.size());
  for (size_t v = 0; v < verts.size(); v++) {
    vIdx[verts[v]] = (int)v;
    memcpy(&T[16 * v], kfs[verts[v]].Tcw, 64);
    fixed[v] = v >= local.size() || kfs[verts[v]].id == 0;
  }
  std::vector<float> X(3 * lpts.size());
  std::vector<int> ept, ekf, ekfId;
  std::vector<float> eobs, es;
  for (size_t j = 0; j < lpts.size(); j++) {
    const OMapPoint& p = mp(lpts[j]);
    memcpy(&X[3 * j], p.pos, 12);
    for (const auto& kv : p.obs) {
      const OKeyFrame& Ki = kfs[kv.first];
      if (Ki.bad) continue;
      const Key& kp = Ki.keys[kv.second];
      ept.push_back((int)j);
      ekf.push_back(vIdx.at(kv.first));
      ekfId.push_back(kv.first);
      eobs.push_back(kp.x);
      eobs.push_back(kp.y);
      eobs.push_back(Ki.uR[kv.second] < 0 ? -1.f : Ki.uR[kv.second]);
      es.push_back(cam.invSigma2[kp.octave]);
    }
  }
  BAProblem P;
  P.n_kf = (int)verts.size();
  P.n_pt = (int)lpts.size();
  P.n_edge = (int)ept.size();
  P.Tcw = T.data();
  P.fixed = fixed.data();
  P.Xw = X.data();
  P.e_pt = ept.data();
  P.e_kf = ekf.data();
  P.e_obs = eobs.data();
  P.e_inv_sigma2 = es.data();
  P.fx = cam.fx; P.fy = cam.fy; P.cx = cam.cx; P.cy = cam.cy; P.bf = cam.bf;
  BAResult R;
  local_ba_solve(P, R);
  if (ba_hook) ba_hook(P, R);
  mstats.n_ba++;
  mstats.ba_trials += R.trials[0] + R.trials[1];
  mstats.ba_edges += P.n_edge;
  mstats.ba_kfs += P.n_kf;
  mstats.ba_pts += P.n_pt;
  long nopt = 0;
  for (uint8_t f : fixed) nopt += !f;
  mstats.ba_max_opt_kfs = std::max(mstats.ba_max_opt_kfs, nopt);
  // vToErase: the monocular edges, then the stereo edges, each in creation order
  for (int pass = 0; pass < 2; pass++)
    for (int i = 0; i < P.n_edge; i++) {
      const bool stereo = !(eobs[3 * i + 2] < 0);
      if (stereo != (pass == 1) || !R.erase[i]) continue;
      const int h = lpts[ept[i]], k = ekfId[i];
      auto it = mp(h).obs.find(k);  // KeyFrame::EraseMapPointMatch(pMP)
      if (it != mp(h).obs.end()) kfs[k].mps[it->second] = -1;
      erase_observation(h, k);
      mstats.n_ba_erased++;
    }
  for (size_t v = 0; v < local.size(); v++) set_pose(local[v], &R.Tcw[16 * v]);
  for (size_t j = 0; j < lpts.size(); j++) {
    memcpy(mp(lpts[j]).pos, &R.Xw[3 * j], 12);  // SetWorldPos
    update_normal_depth(lpts[j]);
  }
}

void MapTracker::keyframe_culling(int kf) {  // LocalMapping::KeyFrameCulling (RGB-D)
  const std::vector<int> local = kfs[kf].ordered;
  for (int k : local) {
    OKeyFrame& K = kfs[k];
    if (K.id == 0) continue;
    const int thObs = 3;
    int nRedundant = 0, nMPs = 0;
    for (size_t i = 0; i < K.mps.size(); i++) {
      const int h = K.mps[i];
      if (h < 0) continue;
      const OMapPoint& p = mp(h);
      if (p.bad) continue;
      if (K.depth[i] > cam.thDepth || K.depth[i] < 0) continue;
      nMPs++;
      if (p.nObs > thObs) {
        const int scaleLevel = K.keys[i].octave;
        int nObs = 0;
        for (const auto& kv : p.obs) {
          if (kv.first == k) continue;
          if (kfs[kv.first].keys[kv.second].octave <= scaleLevel + 1) {
            nObs++;
            if (nObs >= thObs) break;
          }
        }
        if (nObs >= thObs) nRedundant++;
      }
    }
    if (nRedundant > cullRatio * nMPs) {  // 0.9 (LocalMapping.cc:697) unless a test sets it
      kf_set_bad(k);
      mstats.n_culled++;
    }
  }
}

void MapTracker::local_mapping(int kf) {
  // ORACLE_LM_STEPS (diagnostics only, default 7): bit 1 SearchInNeighbors, 2 the local BA,
  // 4 KeyFrameCulling; bit 8 set skips CreateNewMapPoints
  static const int steps = [] {
    const char* e = getenv("ORACLE_LM_STEPS");
    return e ? atoi(e) : 7;
  }();
  // CreateNewMapPoints (with a vocabulary: SearchForTriangulation needs FeatureVectors;
  // bowmap_ref.cpp), then the rest of LocalMapping::Run (LocalMapping.cc:68-87)
  if (voc_ && (steps & 8) == 0) create_new_map_points(kf);
  if (steps & 1) search_in_neighbors(kf);
  if ((steps & 2) && n_keyframes() > 2) local_bundle_adjustment(kf);
  if (steps & 4) keyframe_culling(kf);
}

}  // namespace oracle
