// oracle/map_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// ORB-SLAM2 map tracking for RGB-D as the reference runs it (see oracle_map.h for the functions
// restated and the pinned choices).  cv::Mat float products follow the oracle's pin: double
// accumulation rounded to float, the translation added in float; Mat / scalar is * (1.0 / s) in
// double rounded to float; cv::norm is the double sqrt of the double sum of squares.

#include <algorithm>
#include <cstdlib>
#include <climits>
#include <cmath>
#include <cstring>

#include "oracle_map.h"
#include "oracle_solve.h"

namespace oracle {

// ------------------------------------------------------------------ setup
void MapTracker::init(const MapCam& c) {
  cam = c;
  frameNextId_ = 0;
  mbVO_ = false;
  matchesInliers_ = 0;
  lastRelocFrameId_ = 0;
  reset();
}

void MapTracker::reset() {
  pts.clear();
  temps.clear();
  kfs.clear();
  state_ = 0;
  frameNextId_ = 0;  // Frame::nNextId = 0 (Tracking.cc:3808)
  kfNextId_ = 0;
  lastKFFrameId_ = 0;
  lastKF_ = -1;
  pendingKF_ = -1;
  refKF_ = -1;
  localKFs_.clear();
  localPts_.clear();
  temporal_.clear();
  recent_.clear();
  hasTlr_ = false;
  for (auto& l : invfile_) l.clear();  // mpKeyFrameDB->clear() (Tracking.cc:3801)
}

int MapTracker::n_keyframes() const {
  int n = 0;
  for (const OKeyFrame& k : kfs) n += !k.bad;
  return n;
}

int MapTracker::n_mappoints() const {
  int n = 0;
  for (const OMapPoint& p : pts) n += !p.bad;
  return n;
}

void MapTracker::prepare_frame(const std::vector<Key>& keys, const float* depth, MapFrame& F) {
  MatchFrame G;
  G.n = (int)keys.size();
  G.keys = keys.data();
  G.fx = cam.fx; G.fy = cam.fy; G.cx = cam.cx; G.cy = cam.cy; G.bf = cam.bf;
  G.scale = cam.scale;
  G.nlevels = cam.nlevels;
  G.logScale = cam.logScale;
  frame_stereo_grid(G, depth, cam.W, cam.H);
  F.uR = G.uR;
  F.depth = G.depth;
  F.mps.assign(keys.size(), -1);
  F.outlier.assign(keys.size(), 0);
  F.refKF = -1;
  F.hasBow = false;
  F.bow = BowVec();
  F.fv = FeatVecO();
  depth_ = depth;
}

void MapTracker::build_grid(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                            const MapFrame& C, MatchFrame& G) {
  G.n = (int)keys.size();
  G.keys = keys.data();
  G.desc = desc.data();
  G.fx = cam.fx; G.fy = cam.fy; G.cx = cam.cx; G.cy = cam.cy; G.bf = cam.bf;
  G.scale = cam.scale;
  G.nlevels = cam.nlevels;
  G.logScale = cam.logScale;
  frame_stereo_grid(G, depth_, cam.W, cam.H);
  (void)C;
}

// ------------------------------------------------------------------ MapPoint
int MapTracker::new_point_kf(const float* pos, int kf) {  // MapPoint(Pos, pRefKF, pMap)
  OMapPoint p;
  memcpy(p.pos, pos, 12);
  p.firstKFid = kfs[kf].id;
  p.firstFrame = kfs[kf].frameId;
  p.refKF = kf;
  pts.push_back(p);
  return (int)pts.size() - 1;
}

void MapTracker::add_observation(int h, int kf, int idx) {  // MapPoint::AddObservation
  OMapPoint& p = mp(h);
  if (p.obs.count(kf)) return;
  p.obs[kf] = idx;
  if (kfs[kf].uR[idx] >= 0)
    p.nObs += 2;
  else
    p.nObs++;
}

void MapTracker::set_bad(int h) {  // MapPoint::SetBadFlag
  OMapPoint& p = mp(h);
  p.bad = true;
  std::map<int, int> o = p.obs;
  p.obs.clear();
  for (auto& kv : o) kfs[kv.first].mps[kv.second] = -1;  // KeyFrame::EraseMapPointMatch(idx)
}

void MapTracker::compute_distinctive(int h) {  // MapPoint::ComputeDistinctiveDescriptors
  OMapPoint& p = mp(h);
  if (p.bad || p.obs.empty()) return;
  std::vector<const uint8_t*> D;
  for (auto& kv : p.obs)
    if (!kfs[kv.first].bad) D.push_back(kfs[kv.first].desc.data() + 32 * (size_t)kv.second);
  if (D.empty()) return;
  const size_t N = D.size();
  std::vector<int> dist(N * N, 0);
  for (size_t i = 0; i < N; i++)
    for (size_t j = i + 1; j < N; j++) dist[i * N + j] = dist[j * N + i] = descriptor_distance(D[i], D[j]);
  int best = INT_MAX, bi = 0;
  for (size_t i = 0; i < N; i++) {
    std::vector<int> v(dist.begin() + i * N, dist.begin() + (i + 1) * N);
    std::sort(v.begin(), v.end());
    const int median = v[(size_t)(0.5 * (N - 1))];
    if (median < best) {
      best = median;
      bi = (int)i;
    }
  }
  memcpy(p.desc, D[bi], 32);
}

void MapTracker::update_normal_depth(int h) {  // MapPoint::UpdateNormalAndDepth
  OMapPoint& p = mp(h);
  if (p.bad || p.obs.empty()) return;
  float normal[3] = {0, 0, 0};
  int n = 0;
  for (auto& kv : p.obs) {
    const float* Ow = kfs[kv.first].Ow;
    float ni[3] = {p.pos[0] - Ow[0], p.pos[1] - Ow[1], p.pos[2] - Ow[2]};
    const double inv = 1.0 / (double)norm3(ni);
    for (int k = 0; k < 3; k++) normal[k] = normal[k] + (float)((double)ni[k] * inv);
    n++;
  }
  const OKeyFrame& R = kfs[p.refKF];
  const float PC[3] = {p.pos[0] - R.Ow[0], p.pos[1] - R.Ow[1], p.pos[2] - R.Ow[2]};
  const float dist = norm3(PC);
  const int level = R.keys[p.obs.at(p.refKF)].octave;
  p.maxDist = dist * cam.scale[level];
  p.minDist = p.maxDist / cam.scale[cam.nlevels - 1];
  for (int k = 0; k < 3; k++) p.normal[k] = (float)((double)normal[k] * (1.0 / n));
}

// ------------------------------------------------------------------ KeyFrame
int MapTracker::new_keyframe(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                             const MapFrame& C, const float* Tcw) {  // KeyFrame(F, pMap, pKFDB)
  OKeyFrame k;
  k.id = kfNextId_++;
  k.frameId = C.id;
  memcpy(k.Tcw, Tcw, 64);
  cam_centre(Tcw, k.Ow);
  for (int i = 0; i < 16; i++) k.Twc[i] = (i % 5 == 0) ? 1.f : 0.f;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) k.Twc[4 * r + c] = Tcw[4 * c + r];
    k.Twc[4 * r + 3] = k.Ow[r];
  }
  k.keys = keys;
  k.uR = C.uR;
  k.depth = C.depth;
  k.desc = desc;
  k.mps = C.mps;
  MatchFrame G;  // mGrid: the frame's grid, copied (KeyFrame.cc:48-54)
  build_grid(keys, desc, C, G);
  k.grid = std::move(G.grid);
  kfs.push_back(std::move(k));
  return (int)kfs.size() - 1;
}

void MapTracker::update_best_covisibles(int kf) {  // KeyFrame::UpdateBestCovisibles
  OKeyFrame& K = kfs[kf];
  std::vector<std::pair<int, int>> v;
  for (auto& kv : K.conn) v.push_back({kv.second, kv.first});
  std::sort(v.begin(), v.end());
  K.ordered.clear();
  K.orderedW.clear();
  for (auto it = v.rbegin(); it != v.rend(); ++it) {
    K.ordered.push_back(it->second);
    K.orderedW.push_back(it->first);
  }
}

void MapTracker::add_connection(int kf, int other, int w) {  // KeyFrame::AddConnection
  OKeyFrame& K = kfs[kf];
  auto it = K.conn.find(other);
  if (it == K.conn.end())
    K.conn[other] = w;
  else if (it->second != w)
    it->second = w;
  else
    return;
  update_best_covisibles(kf);
}

void MapTracker::update_connections(int kf) {  // KeyFrame::UpdateConnections
  std::map<int, int> counter;
  const std::vector<int> mps = kfs[kf].mps;
  for (int h : mps) {
    if (h < 0) continue;
    const OMapPoint& p = mp(h);
    if (p.bad) continue;
    for (auto& kv : p.obs) {
      if (kfs[kv.first].id == kfs[kf].id) continue;
      counter[kv.first]++;
    }
  }
  if (counter.empty()) return;
  int nmax = 0, kmax = -1;
  const int th = 15;
  std::vector<std::pair<int, int>> v;
  for (auto& kv : counter) {
    if (kv.second > nmax) {
      nmax = kv.second;
      kmax = kv.first;
    }
    if (kv.second >= th) {
      v.push_back({kv.second, kv.first});
      add_connection(kv.first, kf, kv.second);
    }
  }
  if (v.empty()) {
    v.push_back({nmax, kmax});
    add_connection(kmax, kf, nmax);
  }
  std::sort(v.begin(), v.end());
  OKeyFrame& K = kfs[kf];
  K.conn = counter;
  K.ordered.clear();
  K.orderedW.clear();
  for (auto it = v.rbegin(); it != v.rend(); ++it) {
    K.ordered.push_back(it->second);
    K.orderedW.push_back(it->first);
  }
  if (K.firstConnection && K.id != 0) {
    K.parent = K.ordered.front();
    kfs[K.parent].children.insert(kf);
    K.firstConnection = false;
  }
}

int MapTracker::tracked_map_points(int kf, int minObs) {  // KeyFrame::TrackedMapPoints
  int n = 0;
  for (int h : kfs[kf].mps) {
    if (h < 0) continue;
    const OMapPoint& p = mp(h);
    if (p.bad) continue;
    if (minObs > 0) {
      if (p.nObs >= minObs) n++;
    } else {
      n++;
    }
  }
  return n;
}

// ------------------------------------------------------------------ LocalMapping (synchronous)
void MapTracker::process_new_keyframe(int kf) {  // LocalMapping::ProcessNewKeyFrame
  if (voc_) kf_compute_bow(kf);  // mpCurrentKeyFrame->ComputeBoW() (without a vocabulary: none)
  const std::vector<int> mps = kfs[kf].mps;
  for (size_t i = 0; i < mps.size(); i++) {
    const int h = mps[i];
    if (h < 0 || mp(h).bad) continue;
    if (!mp(h).obs.count(kf)) {
      add_observation(h, kf, (int)i);
      update_normal_depth(h);
      compute_distinctive(h);
    } else {
      recent_.push_back(h);  // new stereo points inserted by the Tracking
    }
  }
  update_connections(kf);
}

void MapTracker::map_point_culling(int kf) {  // LocalMapping::MapPointCulling (RGB-D: 3 obs)
  const int cur = kfs[kf].id;
  const int thObs = 3;
  std::vector<int> keep;
  for (int h : recent_) {
    OMapPoint& p = mp(h);
    if (p.bad) continue;
    if ((float)p.found / p.visible < 0.25f) {
      set_bad(h);
    } else if (cur - p.firstKFid >= 2 && p.nObs <= thObs) {
      set_bad(h);
    } else if (cur - p.firstKFid >= 3) {
      // leaves the list
    } else {
      keep.push_back(h);
    }
  }
  recent_ = keep;
}

// ------------------------------------------------------------------ Tracking
void MapTracker::initialize(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                            MapFrame& C, const float* Tcw) {
  const int kf = new_keyframe(keys, desc, C, Tcw);
  for (size_t i = 0; i < keys.size(); i++) {
    const float z = C.depth[i];
    if (z > 0) {
      float x3D[3];
      unproject(cam, Tcw, keys[i].x, keys[i].y, z, x3D);
      const int h = new_point_kf(x3D, kf);
      add_observation(h, kf, (int)i);
      kfs[kf].mps[i] = h;
      compute_distinctive(h);
      update_normal_depth(h);
      C.mps[i] = h;
    }
  }
  insert_keyframe(kf);  // mpLocalMapper->InsertKeyFrame(pKFini)
  lastKFFrameId_ = C.id;
  lastKF_ = kf;
  localKFs_.assign(1, kf);
  localPts_.clear();
  for (size_t h = 0; h < pts.size(); h++)
    if (!pts[h].bad) localPts_.push_back((int)h);  // mpMap->GetAllMapPoints()
  refKF_ = kf;
  C.refKF = kf;
  state_ = 1;
}

// LocalMapping::InsertKeyFrame: the mapping thread's iteration for this keyframe runs in
// frame_done, after the frame's Track() (pinned, oracle_map.h)
void MapTracker::insert_keyframe(int kf) { pendingKF_ = kf; }

void MapTracker::frame_done(const MapFrame& C, const float* Tcw) {
  // ORACLE_ABLATE (diagnostics only, tools/drift_ablation.py; default 0): bit 1 skips
  // MapPointCulling, bit 2 computes Tlr after the keyframe's LocalMapping (round 4's order)
  static const int ablate = [] {
    const char* e = getenv("ORACLE_ABLATE");
    return e ? atoi(e) : 0;
  }();
  if (C.refKF >= 0 && !(ablate & 2)) {
    m4_mul(Tcw, kfs[C.refKF].Twc, Tlr_);  // Tcr = mTcw * mpReferenceKF->GetPoseInverse()
    hasTlr_ = true;
  }
  // the mapping thread's iteration for the keyframe this frame inserted (pinned: it runs to
  // completion after the frame's Track(), before the next frame is tracked)
  if (pendingKF_ >= 0) {
    const int kf = pendingKF_;
    pendingKF_ = -1;
    process_new_keyframe(kf);
    if (!(ablate & 1)) map_point_culling(kf);
    local_mapping(kf);
    // mpLoopCloser->InsertKeyFrame: LoopClosing::DetectLoop adds it to the database (but
    // keyframe 0, LoopClosing.cc:95); loop detection itself is out of scope
    if (voc_ && kfs[kf].id != 0 && !kfs[kf].bad) kfdb_add(kf);
  }
  if (C.refKF >= 0 && (ablate & 2)) {
    m4_mul(Tcw, kfs[C.refKF].Twc, Tlr_);
    hasTlr_ = true;
  }
}

void MapTracker::update_last_frame(const std::vector<Key>& lkeys,
                                   const std::vector<uint8_t>& ldesc, MapFrame& L, float* Tlast) {
  // Tracking::UpdateLastFrame (Tracking.cc:2894-2960)
  if (L.refKF >= 0 && hasTlr_) m4_mul(Tlr_, kfs[L.refKF].Tcw, Tlast);
  if (lastKFFrameId_ == L.id) return;
  std::vector<std::pair<float, int>> v;
  for (size_t i = 0; i < L.depth.size(); i++)
    if (L.depth[i] > 0) v.push_back({L.depth[i], (int)i});
  if (v.empty()) return;
  std::sort(v.begin(), v.end());
  int nPoints = 0;
  for (size_t j = 0; j < v.size(); j++) {
    const int i = v[j].second;
    const bool create = L.mps[i] < 0 || mp(L.mps[i]).nObs < 1;
    if (create) {
      OMapPoint p;  // MapPoint(x3D, mpMap, &mLastFrame, i): position and descriptor are read
      unproject(cam, Tlast, lkeys[i].x, lkeys[i].y, L.depth[i], p.pos);
      memcpy(p.desc, ldesc.data() + 32 * (size_t)i, 32);
      p.firstFrame = L.id;
      temps.push_back(p);
      const int h = kTemp + (int)temps.size() - 1;
      L.mps[i] = h;
      temporal_.push_back(h);
    }
    nPoints++;
    if (v[j].first > cam.thDepth && nPoints > 200) break;
  }
}

int MapTracker::search_frame(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                             MapFrame& C, const float* Tcw, const std::vector<Key>& lkeys,
                             const MapFrame& L, const float* Tlast, float th) {
  MatchFrame G;
  build_grid(keys, desc, C, G);
  const int n1 = (int)L.mps.size();
  std::vector<float> X(3 * (size_t)std::max(n1, 1));
  std::vector<uint8_t> D(32 * (size_t)std::max(n1, 1)), act(std::max(n1, 1)), obs(std::max(n1, 1));
  for (int i = 0; i < n1; i++) {
    const int h = L.mps[i];
    act[i] = h >= 0 && !L.outlier[i];
    obs[i] = 0;
    if (h >= 0) {
      const OMapPoint& p = mp(h);
      memcpy(&X[3 * (size_t)i], p.pos, 12);
      memcpy(&D[32 * (size_t)i], p.desc, 32);
      obs[i] = p.nObs > 0;
    }
  }
  LastFrameView V;
  V.n = n1;
  V.keys = lkeys.data();
  V.Xw = X.data();
  V.mp_desc = D.data();
  V.active = act.data();
  V.obs = obs.data();
  memcpy(V.Tcw, Tlast, 64);
  std::vector<int> match(std::max(G.n, 1), -1);
  const int nm = search_by_projection_frame(G, Tcw, V, th, false, true, match.data());
  for (int i2 = 0; i2 < G.n; i2++)
    if (match[i2] >= 0) C.mps[i2] = L.mps[match[i2]];
  return nm;
}

int MapTracker::pose_optimization(const std::vector<Key>& keys, MapFrame& C, float* Tcw) {
  // Optimizer::PoseOptimization(&mCurrentFrame): edges of the frame's MapPoints in key order
  std::vector<int> idx;
  std::vector<float> X, ob, s2;
  for (size_t i = 0; i < C.mps.size(); i++) {
    if (C.mps[i] < 0) continue;
    const OMapPoint& p = mp(C.mps[i]);
    idx.push_back((int)i);
    X.insert(X.end(), p.pos, p.pos + 3);
    ob.push_back(keys[i].x);
    ob.push_back(keys[i].y);
    ob.push_back(C.uR[i]);
    s2.push_back(cam.invSigma2[keys[i].octave]);
    C.outlier[i] = 0;
  }
  PoseOptProblem P;
  P.n = (int)idx.size();
  P.Xw = X.data();
  P.obs = ob.data();
  P.inv_sigma2 = s2.data();
  memcpy(P.Tcw, Tcw, 64);
  P.fx = cam.fx; P.fy = cam.fy; P.cx = cam.cx; P.cy = cam.cy; P.bf = cam.bf;
  std::vector<uint8_t> out(std::max(P.n, 1), 0);
  float pose[16];
  const int r = oracle::pose_optimization(P, pose, out.data());
  if (P.n >= 3) {
    memcpy(Tcw, pose, 64);
    for (int e = 0; e < P.n; e++) C.outlier[idx[e]] = out[e];
  }
  return r;
}

bool MapTracker::track_with_motion_model(const std::vector<Key>& keys,
                                         const std::vector<uint8_t>& desc, MapFrame& C,
                                         float* Tcw, const std::vector<Key>& lkeys,
                                         const std::vector<uint8_t>& ldesc, MapFrame& L,
                                         float* Tlast, const float* vel, MapStats& st) {
  update_last_frame(lkeys, ldesc, L, Tlast);
  m4_mul(vel, Tlast, Tcw);
  std::fill(C.mps.begin(), C.mps.end(), -1);
  const float th = 15;
  int nmatches = search_frame(keys, desc, C, Tcw, lkeys, L, Tlast, th);
  if (nmatches < 20) {
    std::fill(C.mps.begin(), C.mps.end(), -1);
    nmatches = search_frame(keys, desc, C, Tcw, lkeys, L, Tlast, 2 * th);
  }
  st.matches_mm = nmatches;
  if (nmatches < 20) return false;
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
  mbVO_ = nmatchesMap < 20;
  return nmatchesMap >= 10;
}

// TrackReferenceKeyFrame with SearchByProjection against the last frame in place of SearchByBoW
// (pinned deviation, oracle_map.h); the acceptance tests are the reference's.
bool MapTracker::track_reference_subst(const std::vector<Key>& keys,
                                       const std::vector<uint8_t>& desc, MapFrame& C, float* Tcw,
                                       const std::vector<Key>& lkeys, const MapFrame& L,
                                       const float* Tlast) {
  std::fill(C.mps.begin(), C.mps.end(), -1);
  memcpy(Tcw, Tlast, 64);
  int nmatches = search_frame(keys, desc, C, Tcw, lkeys, L, Tlast, 15);
  if (nmatches < 15) {
    std::fill(C.mps.begin(), C.mps.end(), -1);
    return false;
  }
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
  return nmatchesMap >= 10;
}

// Relocalization substitute (pinned deviation, oracle_map.h).  The reference (Tracking.cc:3614-3776)
// takes its candidate keyframes from the BoW database and its pose hypotheses from SearchByBoW +
// PnPsolver, neither possible without ORBvoc.txt.  Here the candidates are the reference keyframe
// and its best 10 covisibles in order (GetBestCovisibilityKeyFrames), the hypothesis is the pose
// the motion model predicts from the last frame (the flow-solved pose of every frame keeps being
// tracked while the map is lost), and each candidate's map points are searched as
// TrackWithMotionModel searches the last frame's (the keyframe as the last frame: th 15, again at
// 30 below 20 matches; below 15 the candidate is discarded, the reference's test after
// SearchByBoW).  Then the reference's acceptance: PoseOptimization, fewer than 10 inliers -> next
// candidate, outliers dropped, 50 inliers or more -> relocalised.  The reference's extra
// SearchByProjection(F, KF, sFound, 10 / 3, 100 / 64) rounds for 10-49 inliers are not restated
// (the candidate's points were already searched in a wide window at the predicted pose).
bool MapTracker::relocalization_subst(const std::vector<Key>& keys,
                                      const std::vector<uint8_t>& desc, MapFrame& C, float* Tcw,
                                      const float* Tlast, const float* vel) {
  std::vector<int> cand;
  if (refKF_ >= 0 && !kfs[refKF_].bad) cand.push_back(refKF_);
  if (refKF_ >= 0)
    for (int k : best_covisibles(refKF_, 10))
      if (!kfs[k].bad) cand.push_back(k);
  float Tpred[16];
  m4_mul(vel, Tlast, Tpred);
  for (int k : cand) {
    const OKeyFrame& K = kfs[k];
    MapFrame V;  // the keyframe as a last frame: its good map points, no outliers
    V.mps = K.mps;
    for (int& h : V.mps)
      if (h >= 0 && mp(h).bad) h = -1;
    V.outlier.assign(V.mps.size(), 0);
    std::fill(C.mps.begin(), C.mps.end(), -1);
    memcpy(Tcw, Tpred, 64);
    int nmatches = search_frame(keys, desc, C, Tcw, K.keys, V, K.Tcw, 15);
    if (nmatches < 20) {
      std::fill(C.mps.begin(), C.mps.end(), -1);
      nmatches = search_frame(keys, desc, C, Tcw, K.keys, V, K.Tcw, 30);
    }
    if (nmatches < 15) continue;
    const int nGood = pose_optimization(keys, C, Tcw);
    if (nGood < 10) continue;
    for (size_t i = 0; i < C.mps.size(); i++)
      if (C.mps[i] >= 0 && C.outlier[i]) {
        C.mps[i] = -1;
        C.outlier[i] = 0;
      }
    if (nGood >= 50) return true;
  }
  std::fill(C.mps.begin(), C.mps.end(), -1);
  memcpy(Tcw, Tpred, 64);
  return false;
}

void MapTracker::update_local_keyframes(MapFrame& C) {  // Tracking::UpdateLocalKeyFrames
  std::map<int, int> counter;
  for (size_t i = 0; i < C.mps.size(); i++) {
    if (C.mps[i] < 0) continue;
    const OMapPoint& p = mp(C.mps[i]);
    if (!p.bad) {
      for (auto& kv : p.obs) counter[kv.first]++;
    } else {
      C.mps[i] = -1;
    }
  }
  if (counter.empty()) return;
  int mx = 0, kmax = -1;
  localKFs_.clear();
  for (auto& kv : counter) {
    OKeyFrame& K = kfs[kv.first];
    if (K.bad) continue;
    if (kv.second > mx) {
      mx = kv.second;
      kmax = kv.first;
    }
    localKFs_.push_back(kv.first);
    K.trackRefForFrame = curId_;
  }
  const size_t n0 = localKFs_.size();
  for (size_t q = 0; q < n0; q++) {
    if (localKFs_.size() > 80) break;
    const OKeyFrame& K = kfs[localKFs_[q]];
    const size_t nn = std::min<size_t>(10, K.ordered.size());  // GetBestCovisibilityKeyFrames(10)
    for (size_t a = 0; a < nn; a++) {
      OKeyFrame& N = kfs[K.ordered[a]];
      if (!N.bad && N.trackRefForFrame != curId_) {
        localKFs_.push_back(K.ordered[a]);
        N.trackRefForFrame = curId_;
        break;
      }
    }
    for (int ch : K.children) {
      OKeyFrame& N = kfs[ch];
      if (!N.bad && N.trackRefForFrame != curId_) {
        localKFs_.push_back(ch);
        N.trackRefForFrame = curId_;
        break;
      }
    }
    if (K.parent >= 0) {
      OKeyFrame& Pa = kfs[K.parent];
      if (Pa.trackRefForFrame != curId_) {
        localKFs_.push_back(K.parent);
        Pa.trackRefForFrame = curId_;
        break;  // leaves the keyframe loop (Tracking.cc:3601)
      }
    }
  }
  if (kmax >= 0) {
    refKF_ = kmax;
    C.refKF = kmax;
  }
}

void MapTracker::update_local_points(const MapFrame& C) {  // Tracking::UpdateLocalPoints
  (void)C;
  localPts_.clear();
  for (int kf : localKFs_)
    for (int h : kfs[kf].mps) {
      if (h < 0) continue;
      OMapPoint& p = mp(h);
      if (p.trackRefForFrame == curId_) continue;
      if (!p.bad) {
        localPts_.push_back(h);
        p.trackRefForFrame = curId_;
      }
    }
}

void MapTracker::search_local_points(const std::vector<Key>& keys,
                                     const std::vector<uint8_t>& desc, MapFrame& C,
                                     const float* Tcw) {  // Tracking::SearchLocalPoints
  for (size_t i = 0; i < C.mps.size(); i++) {
    if (C.mps[i] < 0) continue;
    OMapPoint& p = mp(C.mps[i]);
    if (p.bad) {
      C.mps[i] = -1;
    } else {
      p.visible++;
      p.lastFrameSeen = curId_;
      p.trackInView = false;
    }
  }
  MatchFrame G;
  build_grid(keys, desc, C, G);
  const int m = (int)localPts_.size();
  std::vector<LocalPoint> lp(std::max(m, 1));
  for (int j = 0; j < m; j++) {
    const OMapPoint& p = mp(localPts_[j]);
    LocalPoint& q = lp[j];
    memcpy(q.Xw, p.pos, 12);
    memcpy(q.normal, p.normal, 12);
    q.min_dist = p.minDist;
    q.max_dist = p.maxDist;
    q.desc = p.desc;
    q.skip = (p.lastFrameSeen == curId_) || p.bad;
  }
  // isInFrustum(pMP, 0.5) of the points not matched yet, then ORBmatcher(0.8)::SearchByProjection
  // (its th: 3 for RGB-D, 5 right after a relocalisation); IncreaseVisible for those in view
  float th = 3;
  if (curId_ < lastRelocFrameId_ + 2) th = 5;
  std::vector<uint8_t> taken(std::max(G.n, 1), 0);
  for (int i = 0; i < G.n; i++) taken[i] = C.mps[i] >= 0 && mp(C.mps[i]).nObs > 0;
  std::vector<int> match(std::max(G.n, 1), -1);
  std::vector<FrustumOut> fr(std::max(m, 1));
  oracle::search_local_points(G, Tcw, lp.data(), m, th, taken.data(), match.data(), fr.data());
  for (int j = 0; j < m; j++) {
    if (lp[j].skip) continue;
    OMapPoint& p = mp(localPts_[j]);
    p.trackInView = fr[j].in_view != 0;
    if (p.trackInView) p.visible++;
  }
  for (int i = 0; i < G.n; i++)
    if (match[i] >= 0) C.mps[i] = localPts_[match[i]];
}

bool MapTracker::track_local_map(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                                 MapFrame& C, float* Tcw) {  // Tracking::TrackLocalMap
  update_local_keyframes(C);
  update_local_points(C);
  search_local_points(keys, desc, C, Tcw);
  pose_optimization(keys, C, Tcw);
  matchesInliers_ = 0;
  for (size_t i = 0; i < C.mps.size(); i++) {
    if (C.mps[i] < 0) continue;
    if (!C.outlier[i]) {
      OMapPoint& p = mp(C.mps[i]);
      p.found++;
      if (p.nObs > 0) matchesInliers_++;
    }
  }
  if (curId_ < lastRelocFrameId_ + cam.maxFrames && matchesInliers_ < 50) return false;
  return matchesInliers_ >= 30;
}

bool MapTracker::need_new_keyframe(const MapFrame& C) {  // Tracking::NeedNewKeyFrame (RGB-D)
  const int nKFs = n_keyframes();
  if (curId_ < lastRelocFrameId_ + cam.maxFrames && nKFs > cam.maxFrames) return false;
  int nMinObs = 3;
  if (nKFs <= 2) nMinObs = 2;
  const int nRefMatches = tracked_map_points(refKF_, nMinObs);
  const bool bLocalMappingIdle = true;  // synchronous LocalMapping (pinned)
  int nNonTrackedClose = 0, nTrackedClose = 0;
  for (size_t i = 0; i < C.mps.size(); i++) {
    if (C.depth[i] > 0 && C.depth[i] < cam.thDepth) {
      if (C.mps[i] >= 0 && !C.outlier[i])
        nTrackedClose++;
      else
        nNonTrackedClose++;
    }
  }
  const bool bNeedToInsertClose = (nTrackedClose < 100) && (nNonTrackedClose > 70);
  float thRefRatio = 0.75f;
  if (nKFs < 2) thRefRatio = 0.4f;
  const bool c1a = curId_ >= lastKFFrameId_ + cam.maxFrames;
  const bool c1b = (curId_ >= lastKFFrameId_ + 0 && bLocalMappingIdle);
  const bool c1c = (matchesInliers_ < nRefMatches * 0.25 || bNeedToInsertClose);
  const bool c2 = ((matchesInliers_ < nRefMatches * thRefRatio || bNeedToInsertClose) &&
                   matchesInliers_ > 15);
  return (c1a || c1b || c1c) && c2;
}

void MapTracker::create_new_keyframe(const std::vector<Key>& keys,
                                     const std::vector<uint8_t>& desc, MapFrame& C,
                                     const float* Tcw) {  // Tracking::CreateNewKeyFrame (RGB-D)
  const int kf = new_keyframe(keys, desc, C, Tcw);
  refKF_ = kf;
  C.refKF = kf;
  std::vector<std::pair<float, int>> v;
  for (size_t i = 0; i < keys.size(); i++)
    if (C.depth[i] > 0) v.push_back({C.depth[i], (int)i});
  if (!v.empty()) {
    std::sort(v.begin(), v.end());
    int nPoints = 0;
    for (size_t j = 0; j < v.size(); j++) {
      const int i = v[j].second;
      bool create = false;
      if (C.mps[i] < 0) {
        create = true;
      } else if (mp(C.mps[i]).nObs < 1) {
        create = true;
        C.mps[i] = -1;
      }
      if (create) {
        float x3D[3];
        unproject(cam, Tcw, keys[i].x, keys[i].y, C.depth[i], x3D);
        const int h = new_point_kf(x3D, kf);
        add_observation(h, kf, i);
        kfs[kf].mps[i] = h;
        compute_distinctive(h);
        update_normal_depth(h);
        C.mps[i] = h;
      }
      nPoints++;
      if (v[j].first > cam.thDepth && nPoints > 200) break;
    }
  }
  insert_keyframe(kf);  // mpLocalMapper->InsertKeyFrame(pKF)
  lastKFFrameId_ = C.id;
  lastKF_ = kf;
}

int MapTracker::track(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                      MapFrame& C, float* Tcw, const std::vector<Key>& lkeys,
                      const std::vector<uint8_t>& ldesc, MapFrame& L, float* Tlast, float* vel,
                      bool& has_vel, bool& bSecondFrame, MapStats& st) {
  curId_ = C.id;
  bool bOK;
  // A branch that computes no pose (TrackReferenceKeyFrame below 15 BoW matches, a relocalisation
  // without a hypothesis) leaves mCurrentFrame.mTcw empty in the reference, and the flow solve
  // then starts from it (undefined).  Pinned: the motion model's prediction, or the last pose.
  if (has_vel)
    m4_mul(vel, Tlast, Tcw);
  else
    memcpy(Tcw, Tlast, 64);
  if (state_ == 1) {
    // CheckReplacedInLastFrame (Tracking.cc:2766-2781): one level of MapPoint::GetReplaced
    for (size_t i = 0; i < L.mps.size(); i++)
      if (L.mps[i] >= 0 && L.mps[i] < kTemp && mp(L.mps[i]).replaced >= 0)
        L.mps[i] = mp(L.mps[i]).replaced;
    if (!has_vel || C.id < lastRelocFrameId_ + 2) {
      bSecondFrame = true;
      bOK = voc_ ? track_reference_kf(keys, desc, C, Tcw, Tlast)
                 : track_reference_subst(keys, desc, C, Tcw, lkeys, L, Tlast);
    } else {
      bSecondFrame = false;
      bOK = track_with_motion_model(keys, desc, C, Tcw, lkeys, ldesc, L, Tlast, vel, st);
      if (!bOK) {
        bSecondFrame = true;
        bOK = voc_ ? track_reference_kf(keys, desc, C, Tcw, Tlast)
                   : track_reference_subst(keys, desc, C, Tcw, lkeys, L, Tlast);
      }
    }
  } else if (voc_) {  // Relocalization (Tracking.cc:3614-3776)
    bOK = relocalization(keys, desc, C, Tcw);  // from the prediction set above
    if (bOK) lastRelocFrameId_ = C.id;
  } else {
    bOK = relocalization_subst(keys, desc, C, Tcw, Tlast, vel);  // Relocalization substitute
    if (bOK) lastRelocFrameId_ = C.id;
  }
  C.refKF = refKF_;
  if (bOK && !mbVO_) {
    bOK = track_local_map(keys, desc, C, Tcw);
    st.inliers_local = matchesInliers_;
  }
  state_ = bOK ? 1 : 2;
  if (bOK) {
    // motion model from the map pose (Tracking.cc:1117-1125)
    float LastTwc[16];
    for (int i = 0; i < 16; i++) LastTwc[i] = (i % 5 == 0) ? 1.f : 0.f;
    float Ow[3];
    cam_centre(Tlast, Ow);
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) LastTwc[4 * r + c] = Tlast[4 * c + r];
      LastTwc[4 * r + 3] = Ow[r];
    }
    m4_mul(Tcw, LastTwc, vel);
    has_vel = true;
    // clean VO matches
    for (size_t i = 0; i < C.mps.size(); i++)
      if (C.mps[i] >= 0 && mp(C.mps[i]).nObs < 1) {
        C.outlier[i] = 0;
        C.mps[i] = -1;
      }
    // delete temporal MapPoints
    temporal_.clear();
    for (size_t i = 0; i < L.mps.size(); i++)
      if (L.mps[i] >= kTemp) L.mps[i] = -1;  // dangling in the reference, never read again
    temps.clear();
    if (need_new_keyframe(C)) {
      create_new_keyframe(keys, desc, C, Tcw);
      st.new_keyframe = 1;
    }
    for (size_t i = 0; i < C.mps.size(); i++)
      if (C.mps[i] >= 0 && C.outlier[i]) C.mps[i] = -1;
  }
  if (state_ == 2 && n_keyframes() <= 5) return 1;  // mpSystem->Reset(); return
  if (C.refKF < 0) C.refKF = refKF_;
  return 0;
}

}  // namespace oracle
