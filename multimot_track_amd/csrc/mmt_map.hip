// multimot_track_amd/csrc/mmt_map.hip -- ORB-SLAM2 map tracking for RGB-D (see mmt_map.h).
//
// cv::Mat float arithmetic as elsewhere on the host side of this path: products accumulate in
// double and round to float, the translation is added in float; Mat / scalar is * (1.0 / s) in
// double; cv::norm is the double square root of the double sum of squares.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>

#include "mmt_map.h"
#include "mmt_mat4.h"

namespace mmt {

// ------------------------------------------------------------------ pose helpers
// Frame::UpdatePoseMatrices / KeyFrame::SetPose: Ow = -Rcw^T tcw
static void cam_centre(const float* T, float* Ow) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    Ow[r] = -(float)s;
  }
}

// Frame::UnprojectStereo (Frame.cc:1064-1079): Rwc * ((u - cx) z / fx, (v - cy) z / fy, z) + Ow
static void unproject(const MapCamH& c, const float* T, float u, float v, float z, float* out) {
  const float x = (u - c.cx) * z * c.invfx;
  const float y = (v - c.cy) * z * c.invfy;
  const float xc[3] = {x, y, z};
  float Ow[3];
  cam_centre(T, Ow);
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)xc[k];
    out[r] = (float)s + Ow[r];
  }
}

static float norm3(const float* v) {
  double s = 0;
  for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
  return (float)std::sqrt(s);
}

#define MAP_PROF(k, stmt)                       \
  do {                                          \
    const double _t0 = prof_on_ ? now_us() : 0; \
    stmt;                                       \
    if (prof_on_) prof_[k] += now_us() - _t0;   \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

double MapEngine::prof_now_us() { return now_us(); }

MapEngine::~MapEngine() {
  if (prof_on_ && prof_n_ > 0) {
    static const char* names[12] = {"C2 search", "D1 (motion model)", "local map update",
                                    "C3 search", "D1 (local map)", "keyframe + mapping",
                                    "other", "total", "UpdateLastFrame", "C2 pack",
                                    "C3 pack", "D1 pack"};
    fprintf(stderr, "[mmt map profile] %ld frames, host wall us per frame:", prof_n_);
    for (int k = 0; k < 12; k++) fprintf(stderr, " %s %.1f%s", names[k], prof_[k] / prof_n_,
                                         k < 11 ? "," : "\n");
    if (mstats_.n_lm > 0) {
      const double n = (double)mstats_.n_lm;
      fprintf(stderr, "[mmt localmapping profile] %ld keyframes, host wall us per keyframe: "
              "ProcessNewKeyFrame+MapPointCulling %.1f, CreateNewMapPoints + SearchInNeighbors %.1f "
              "(CreateNewMapPoints %.1f, Fuse launches "
              "%.1f), LocalBundleAdjustment %.1f (solve %.1f), KeyFrameCulling %.1f, final sync "
              "%.1f, LocalMapping total %.1f; CreateNewKeyFrame with all of it %.1f\n", mstats_.n_lm,
              mstats_.pnk_us / n,
              mstats_.sin_us / n, mstats_.cnmp_us / n, mstats_.fuse_us / n, mstats_.ba_us / n,
              mstats_.basolve_us / n, mstats_.cull_us / n, mstats_.lmsync_us / n,
              mstats_.lm_us / n, mstats_.kfnew_us / n);
      static const char* bn[MappingStats::kBlk] = {
          "new keyframe + store", "new points", "SIN targets", "SIN fuse 1", "SIN candidates",
          "SIN fuse 2", "SIN point updates", "SIN connections", "BA graph", "BA apply",
          "Fuse pool flush", "Fuse enqueue", "Fuse wait", "Fuse apply (+ relaunches)",
          "ComputeDistinctiveDescriptors (inside the others)", "PNK ComputeBoW",
          "PNK observations", "PNK UpdateConnections"};
      fprintf(stderr, "[mmt localmapping profile] per keyframe, us:");
      for (int k = 0; k < MappingStats::kBlk; k++)
        fprintf(stderr, " %s %.1f%s", bn[k], mstats_.blk_us[k] / n,
                k + 1 < MappingStats::kBlk ? "," : "\n");
    }
    fprintf(stderr, "[mmt map profile] per frame: %.1f local keyframes, %.1f local points, "
            "%.1f C3 edges; %zu map points allocated, %d keyframes at the end; local map "
            "speculated %ld times, taken %ld\n",
            prof_cnt_[0] / prof_n_, prof_cnt_[1] / prof_n_, prof_cnt_[2] / prof_n_, pts_.size(),
            n_keyframes(), spec_tries_, spec_hits_);
  }
  if (s_) (void)hipStreamSynchronize(s_);
  if (lm_s_) {
    (void)hipStreamSynchronize(lm_s_);
    (void)hipStreamDestroy(lm_s_);
  }
  if (ev_early_) (void)hipEventDestroy(ev_early_);
  for (void* p : dallocs_) (void)hipFree(p);
  for (void* p : hallocs_) (void)hipHostFree(p);
}

static size_t last_bytes(int n) { return (size_t)n * (sizeof(mmt_kp) + 12 + 32 + 2); }

// every chain (C2 -> D1, C3 -> D1) moves one block up and one block down
static_assert(sizeof(PoseOptDesc) <= kDescBytes, "PoseOptDesc outgrew its slot");
static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// C3's upload block for m local points and n keys: offsets of taken (after ids, skip), the base
// positions and their flags, and the total size
struct SelLayout {
  size_t ids, skip, taken, bX, bHas, total;
  SelLayout(int m, int n) {
    ids = kDescBytes;
    skip = ids + 4 * (size_t)m;
    taken = skip + m;
    bX = align16(taken + n);
    bHas = bX + 12 * (size_t)n;
    total = bHas + n;
  }
};

size_t MapEngine::out_bytes(int n) const { return kOutHdr + 4 * (size_t)kcap_ + n; }

void MapEngine::setup(const MapCamH& cam, int kcap) {
  cam_ = cam;
  kcap_ = kcap;
  d_last_ = dev<uint8_t>(kDescBytes + last_bytes(kcap));
  h_last_ = pinned<uint8_t>(kDescBytes + last_bytes(kcap));
  c2_ = CandSet{dev<uint32_t>((size_t)kcap * kCandK), dev<int>((size_t)kcap * kCandK),
                dev<int>(kcap), dev<PointWin>(kcap), dev<int>(kcap)};
  d_out_ = dev<uint8_t>(kOutHdr + 5 * (size_t)kcap);
  h_out_ = pinned<uint8_t>(kOutHdr + 5 * (size_t)kcap);
  d_nm_ = (int*)d_out_;
  d_ninl_ = (int*)(d_out_ + 4);
  d_pose_ = (float*)(d_out_ + 16);
  d_match_ = (int*)(d_out_ + kOutHdr);
  d_outl_ = d_out_ + kOutHdr + 4 * (size_t)kcap;
  h_nm_ = (int*)h_out_;
  h_ninl_ = (int*)(h_out_ + 4);
  h_pose_ = (float*)(h_out_ + 16);
  h_match_ = (int*)(h_out_ + kOutHdr);
  h_outl_ = h_out_ + kOutHdr + 4 * (size_t)kcap;
  d_edges_ = dev<float>(7 * (size_t)kcap);
  h_edges_ = pinned<float>(7 * (size_t)kcap);
  d_esc_ = dev<double>(3 * (size_t)kcap);
  d_fsc_ = dev<int>(kcap);
  prof_on_ = getenv("MMT_MAP_PROFILE") != nullptr;
  if (const char* e = getenv("MMT_LOCALMAP_SPEC")) spec_on_ = atoi(e) != 0;
  if (const char* e = getenv("MMT_OVERLAP_C3")) overlap_c3_ = atoi(e) != 0;
  h_early_ = pinned<uint8_t>(kOutHdr + 4 * (size_t)kcap);
  MMT_HIP(hipEventCreateWithFlags(&ev_early_, hipEventDisableTiming));
  // LocalMapping's stream, normal priority (high / low measured within noise / slower in round 5,
  // without the vocabulary): its kernels (keyframe store copies, the BoW transform, Fuse,
  // SearchForTriangulation, the local BA) need nothing of the frame's flow solve.  MMT_LM_PRIO=high
  // (A/B): the greatest priority
  int prio_lo = 0, prio_hi = 0;
  MMT_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  const char* lmp = getenv("MMT_LM_PRIO");
  const int lm_prio = lmp && strcmp(lmp, "high") == 0 ? prio_hi : 0;
  MMT_HIP(hipStreamCreateWithPriority(&lm_s_, hipStreamNonBlocking, lm_prio));
  // keyframe store record: keys, descriptors, mvuRight, grid (cell starts + key lists)
  kf_rec_bytes_ = align16(sizeof(mmt_kp) * (size_t)kcap) + 32 * (size_t)kcap +
                  align16(4 * (size_t)kcap) + align16(4 * (size_t)(kGridCells + 1)) +
                  align16(4 * (size_t)kcap);
  frameNextId_ = 0;
  mbVO_ = false;
  matchesInliers_ = 0;
  lastRelocFrameId_ = 0;
  reset();
}

// the local-map buffers grow with the local map; the point pool with the map
void MapEngine::grow_local(int m) {
  if (m <= local_cap_ && d_sel_) return;
  const int cap = std::max(m + 4096, 2 * local_cap_);
  void* old[] = {d_sel_, h_sel_, d_inview_, h_inview_, c3_.key, c3_.idx, c3_.n, c3_.win,
                 c3_.choice};
  if (s_) MMT_HIP(hipStreamSynchronize(s_));
  for (int i = 0; i < 9; i++) {
    if (!old[i]) continue;
    auto it = std::find(i == 1 || i == 3 ? hallocs_.begin() : dallocs_.begin(),
                        i == 1 || i == 3 ? hallocs_.end() : dallocs_.end(), old[i]);
    if (i == 1 || i == 3) {
      (void)hipHostFree(old[i]);
      hallocs_.erase(it);
    } else {
      (void)hipFree(old[i]);
      dallocs_.erase(it);
    }
  }
  const size_t sel_cap = SelLayout(cap, kcap_).total + 16;
  d_sel_ = dev<uint8_t>(sel_cap);
  h_sel_ = pinned<uint8_t>(sel_cap);
  d_inview_ = dev<uint8_t>(cap);
  h_inview_ = pinned<uint8_t>(cap);
  c3_ = CandSet{dev<uint32_t>((size_t)cap * kCandK), dev<int>((size_t)cap * kCandK), dev<int>(cap),
                dev<PointWin>(cap), dev<int>(cap)};
  local_cap_ = cap;
}

void MapEngine::reset() {
  pts_.clear();
  hot_.clear();
  dcache_.clear();
  spec_discard();
  temps_.clear();
  kfs_.clear();
  state_ = 0;
  frameNextId_ = 0;  // Frame::nNextId = 0 (Tracking.cc:3808)
  kfNextId_ = 0;
  lastKFFrameId_ = 0;
  refKF_ = -1;
  localKFs_.clear();
  localPts_.clear();
  recent_.clear();
  dirty_.clear();
  hasTlr_ = false;
  snapKF_ = -1;
  n_good_ = 0;
  for (auto& l : invfile_) l.clear();  // mpKeyFrameDB->clear() (Tracking.cc:3801)
}

int MapEngine::n_keyframes() const {
  int n = 0;
  for (const KFrame& k : kfs_) n += !k.bad;
  return n;
}

void MapEngine::prepare(MapFrameH& F) const {
  F.mps.assign(F.n, -1);
  F.outlier.assign(F.n, 0);
  F.refKF = -1;
  F.hasBow = false;
  F.bow.word.clear();
  F.bow.value.clear();
  F.fv = FeatVecH();
}

// ------------------------------------------------------------------ MapPoint
void MapEngine::mark_dirty(int h) {
  if (h >= kTemp) return;  // temporal points never enter the local map
  MPoint& p = pts_[h];
  if (!p.dirty) {
    p.dirty = true;
    dirty_.push_back(h);
  }
}

int MapEngine::new_point_kf(const float* pos, int kf) {  // MapPoint(Pos, pRefKF, pMap)
  MPoint p;
  memcpy(p.pos, pos, 12);
  p.firstKFid = kfs_[kf].id;
  p.refKF = kf;
  pts_.push_back(p);
  hot_.push_back(PtHot());
  n_good_++;
  const int h = (int)pts_.size() - 1;
  mark_dirty(h);
  return h;
}

void MapEngine::add_observation(int h, int kf, int idx) {  // MapPoint::AddObservation
  MPoint& p = mp(h);
  if (p.obs_index(kf) >= 0) return;
  auto it = std::lower_bound(p.obs.begin(), p.obs.end(), std::make_pair(kf, INT_MIN));
  p.obs.insert(it, {kf, idx});
  if (kfs_[kf].uR[idx] >= 0)
    p.nObs += 2;
  else
    p.nObs++;
}

void MapEngine::mark_bad(int h) {
  MPoint& p = mp(h);
  if (!p.bad && h < kTemp) n_good_--;
  p.bad = true;
  if (h < kTemp) hot_[h].bad = 1;
  if (!dcache_.empty()) dcache_.erase(h);  // a bad point's descriptor is never recomputed
}

void MapEngine::set_bad(int h) {  // MapPoint::SetBadFlag
  MPoint& p = mp(h);
  mark_bad(h);
  const std::vector<std::pair<int, int>> o = p.obs;
  p.obs.clear();
  for (const auto& kv : o) kfs_[kv.first].mps[kv.second] = -1;
  mark_dirty(h);
}

void MapEngine::compute_distinctive(int h) {  // MapPoint::ComputeDistinctiveDescriptors
  MPoint& p = mp(h);
  if (p.bad || p.obs.empty()) return;
  struct Timer {  // MMT_MAP_PROFILE: this function's share of the keyframe path
    MapEngine* m;
    double t;
    ~Timer() {
      if (m) m->mstats_.blk_us[14] += now_us() - t;
    }
  } timer{prof_on_ ? this : nullptr, prof_on_ ? now_us() : 0};
  // the descriptors of the good observing keyframes, their pairwise Hamming distances and each
  // one's median distance (the (N - 1) / 2-th smallest, MapPoint.cc:295-313); up to 32
  // observations on the stack (no allocation per call), beyond that on the heap with the
  // distances kept per point (dcache_: a new observation costs N distances, not N^2 / 2)
  constexpr int kStack = 32;
  const uint8_t* Ds[kStack];
  std::vector<const uint8_t*> Dh;
  std::vector<uint64_t> ids;
  int N = 0;
  for (const auto& kv : p.obs)
    if (!kfs_[kv.first].bad) {
      const uint8_t* d = kfs_[kv.first].desc.data() + 32 * (size_t)kv.second;
      if (N < kStack) Ds[N] = d;
      if (N == kStack) Dh.assign(Ds, Ds + kStack);
      if (N >= kStack) Dh.push_back(d);
      ids.push_back(((uint64_t)(uint32_t)kv.first << 32) | (uint32_t)kv.second);
      N++;
    }
  if (N == 0) return;
  const uint8_t* const* Dv = N <= kStack ? Ds : Dh.data();
  auto hamming = [](const uint8_t* x, const uint8_t* y) {
    int d = 0;
    for (int w = 0; w < 4; w++) {
      uint64_t a, b;
      memcpy(&a, x + 8 * w, 8);
      memcpy(&b, y + 8 * w, 8);
      d += __builtin_popcountll(a ^ b);
    }
    return d;
  };
  int dist_s[kStack * kStack], v_s[kStack];
  std::vector<int> dist_h, v_h;
  if (N > kStack) {
    dist_h.assign((size_t)N * N, 0);
    v_h.resize(N);
  }
  int* dist = N <= kStack ? dist_s : dist_h.data();
  int* v = N <= kStack ? v_s : v_h.data();
  if (N <= kStack) {
    dcache_.erase(h);
    for (int i = 0; i < N; i++) {
      dist[(size_t)i * N + i] = 0;
      for (int j = i + 1; j < N; j++)
        dist[(size_t)i * N + j] = dist[(size_t)j * N + i] = hamming(Dv[i], Dv[j]);
    }
  } else {
    // old index of every current observation (both lists in keyframe order), -1 for a new one
    DistCache& c = dcache_[h];
    std::vector<int> old(N, -1);
    for (size_t i = 0, o = 0; i < (size_t)N; i++) {
      while (o < c.ids.size() && c.ids[o] < ids[i]) o++;
      if (o < c.ids.size() && c.ids[o] == ids[i]) old[i] = (int)o;
    }
    const size_t M = c.ids.size();
    for (int i = 0; i < N; i++) {
      dist[(size_t)i * N + i] = 0;
      for (int j = i + 1; j < N; j++) {
        const int d = old[i] >= 0 && old[j] >= 0 ? (int)c.d[(size_t)old[i] * M + old[j]]
                                                  : hamming(Dv[i], Dv[j]);
        dist[(size_t)i * N + j] = dist[(size_t)j * N + i] = d;
      }
    }
    c.ids = ids;
    c.d.resize((size_t)N * N);
    for (size_t q = 0; q < (size_t)N * N; q++) c.d[q] = (uint16_t)dist[q];
  }
  // the row with the smallest median (the first on ties): a row's median is below the best so
  // far iff more than m of its distances are, so most rows cost one counting pass
  const int m = (int)(0.5 * (N - 1));
  int best = INT_MAX, bi = 0;
  for (int i = 0; i < N; i++) {
    const int* row = dist + (size_t)i * N;
    if (best != INT_MAX) {
      int below = 0;
      for (int k = 0; k < N; k++) below += row[k] < best;
      if (below <= m) continue;
    }
    std::copy(row, row + N, v);
    std::nth_element(v, v + m, v + N);
    if (v[m] < best) {
      best = v[m];
      bi = i;
    }
  }
  memcpy(p.desc, Dv[bi], 32);
  p.desc_ver++;
  mark_dirty(h);
}

void MapEngine::update_normal_depth(int h) {  // MapPoint::UpdateNormalAndDepth
  MPoint& p = mp(h);
  if (p.bad || p.obs.empty()) return;
  float normal[3] = {0, 0, 0};
  int n = 0;
  for (const auto& kv : p.obs) {
    const float* Ow = kfs_[kv.first].Ow;
    const float ni[3] = {p.pos[0] - Ow[0], p.pos[1] - Ow[1], p.pos[2] - Ow[2]};
    const double inv = 1.0 / (double)norm3(ni);
    for (int k = 0; k < 3; k++) normal[k] = normal[k] + (float)((double)ni[k] * inv);
    n++;
  }
  const KFrame& R = kfs_[p.refKF];
  const float PC[3] = {p.pos[0] - R.Ow[0], p.pos[1] - R.Ow[1], p.pos[2] - R.Ow[2]};
  const float dist = norm3(PC);
  const int level = R.keys[p.obs_index(p.refKF)].octave;
  p.maxDist = dist * cam_.scale[level];
  p.minDist = p.maxDist / cam_.scale[cam_.nlevels - 1];
  for (int k = 0; k < 3; k++) p.normal[k] = (float)((double)normal[k] * (1.0 / n));
  mark_dirty(h);
}

// ------------------------------------------------------------------ KeyFrame
int MapEngine::new_keyframe(const MapFrameH& C, const float* Tcw) {  // KeyFrame(F, ...)
  kfs_.emplace_back();
  KFrame& k = kfs_.back();
  k.id = kfNextId_++;
  k.frameId = C.id;
  memcpy(k.Tcw, Tcw, 64);
  cam_centre(Tcw, k.Ow);
  mat4_eye(k.Twc);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) k.Twc[4 * r + c] = Tcw[4 * c + r];
    k.Twc[4 * r + 3] = k.Ow[r];
  }
  k.keys.assign(C.kps, C.kps + C.n);
  k.uR.assign(C.uR, C.uR + C.n);
  k.depth.assign(C.depth, C.depth + C.n);
  k.desc.assign(C.desc, C.desc + 32 * (size_t)C.n);
  k.mps = C.mps;
  return (int)kfs_.size() - 1;
}

void MapEngine::update_best_covisibles(int kf) {  // KeyFrame::UpdateBestCovisibles
  KFrame& K = kfs_[kf];
  std::vector<std::pair<int, int>> v;
  for (const auto& kv : K.conn) v.push_back({kv.second, kv.first});
  std::sort(v.begin(), v.end());
  K.ordered.clear();
  for (auto it = v.rbegin(); it != v.rend(); ++it) K.ordered.push_back(it->second);
}

void MapEngine::add_connection(int kf, int other, int w) {  // KeyFrame::AddConnection
  KFrame& K = kfs_[kf];
  auto it = K.conn.find(other);
  if (it == K.conn.end())
    K.conn[other] = w;
  else if (it->second != w)
    it->second = w;
  else
    return;
  update_best_covisibles(kf);
}

void MapEngine::update_connections(int kf) {  // KeyFrame::UpdateConnections
  std::map<int, int> counter;
  for (int h : kfs_[kf].mps) {
    if (h < 0) continue;
    const MPoint& p = mp(h);
    if (p.bad) continue;
    for (const auto& kv : p.obs)
      if (kv.first != kf) counter[kv.first]++;
  }
  if (counter.empty()) return;
  int nmax = 0, kmax = -1;
  std::vector<std::pair<int, int>> v;
  for (const auto& kv : counter) {
    if (kv.second > nmax) {
      nmax = kv.second;
      kmax = kv.first;
    }
    if (kv.second >= 15) {
      v.push_back({kv.second, kv.first});
      add_connection(kv.first, kf, kv.second);
    }
  }
  if (v.empty()) {
    v.push_back({nmax, kmax});
    add_connection(kmax, kf, nmax);
  }
  std::sort(v.begin(), v.end());
  KFrame& K = kfs_[kf];
  K.conn = counter;
  K.ordered.clear();
  for (auto it = v.rbegin(); it != v.rend(); ++it) K.ordered.push_back(it->second);
  if (K.firstConnection && K.id != 0) {
    K.parent = K.ordered.front();
    kfs_[K.parent].children.insert(kf);
    K.firstConnection = false;
  }
}

int MapEngine::tracked_map_points(int kf, int minObs) {  // KeyFrame::TrackedMapPoints
  int n = 0;
  for (int h : kfs_[kf].mps) {
    if (h < 0) continue;
    const MPoint& p = mp(h);
    if (p.bad) continue;
    if (minObs > 0) {
      if (p.nObs >= minObs) n++;
    } else {
      n++;
    }
  }
  return n;
}

void MapEngine::process_new_keyframe(int kf) {  // LocalMapping::ProcessNewKeyFrame
  double tb = prof_on_ ? now_us() : 0;
  // mpCurrentKeyFrame->ComputeBoW() (without a vocabulary: none): the descent runs on the GPU
  // while the observations and connections below are updated on the host (they do not read it)
  if (voc_) kf_bow_launch(kf);
  blk_time(15, tb);
  const std::vector<int> mps = kfs_[kf].mps;
  for (size_t i = 0; i < mps.size(); i++) {
    const int h = mps[i];
    if (h < 0 || mp(h).bad) continue;
    if (mp(h).obs_index(kf) < 0) {
      add_observation(h, kf, (int)i);
      update_normal_depth(h);
      compute_distinctive(h);
    } else {
      recent_.push_back(h);
    }
  }
  blk_time(16, tb);
  update_connections(kf);
  blk_time(17, tb);
  if (voc_) kf_bow_finish(kf);
  blk_time(15, tb);
}

void MapEngine::map_point_culling(int kf) {  // LocalMapping::MapPointCulling (RGB-D: 3 obs)
  const int cur = kfs_[kf].id;
  std::vector<int> keep;
  keep.reserve(recent_.size());
  for (int h : recent_) {
    MPoint& p = mp(h);
    if (p.bad) continue;
    if ((float)p.found / p.visible < 0.25f) {
      set_bad(h);
    } else if (cur - p.firstKFid >= 2 && p.nObs <= 3) {
      set_bad(h);
    } else if (cur - p.firstKFid < 3) {
      keep.push_back(h);
    }
  }
  recent_.swap(keep);
}

// ------------------------------------------------------------------ GPU stages
// D1's descriptor for an edge list that k_map_edges builds on the device (it writes n): the edge
// arrays at a fixed capacity of kcap edges
void MapEngine::pose_desc_fill(uint8_t* h_blk, uint8_t* d_blk, const float* Tcw) {
  h_pod_ = (PoseOptDesc*)h_blk;
  d_pod_ = (PoseOptDesc*)d_blk;
  PoseOptDesc& d = *h_pod_;
  memset(&d, 0, sizeof(d));
  d.n = 0;
  d.Xw = d_edges_;
  d.obs = d_edges_ + 3 * (size_t)kcap_;
  d.inv_sigma2 = d_edges_ + 6 * (size_t)kcap_;
  memcpy(d.Tcw, Tcw, 64);
  d.fx = cam_.fx; d.fy = cam_.fy; d.cx = cam_.cx; d.cy = cam_.cy; d.bf = cam_.bf;
  d.pose_out = d_pose_;
  d.outlier = d_outl_;
  d.n_inliers = d_ninl_;
  d.e_scratch = d_esc_;
  d.f_scratch = d_fsc_;
}

MapEdgeArgs MapEngine::edge_args(const GridFrame& G) const {
  MapEdgeArgs e;
  memset(&e, 0, sizeof(e));
  e.n = G.n;
  e.keys = G.keys;
  e.uR = G.uR;
  e.match = d_match_;
  for (int l = 0; l < cam_.nlevels && l < kMaxLevels; l++) e.inv_sigma2[l] = cam_.invSigma2[l];
  e.X = d_edges_;
  e.obs = d_edges_ + 3 * (size_t)kcap_;
  e.s2 = d_edges_ + 6 * (size_t)kcap_;
  e.desc = d_pod_;
  return e;
}

// Optimizer::PoseOptimization's results for the frame's MapPoints (edges in key order): every
// edge's mvbOutlier is reset, and below 3 edges the pose stays (Optimizer.cc:3160-3253)
void MapEngine::apply_pose_opt(MapFrameH& C, float* Tcw) {
  int n = 0;
  for (int i = 0; i < C.n; i++)
    if (C.mps[i] >= 0) {
      C.outlier[i] = 0;
      n++;
    }
  if (n < 3) return;
  memcpy(Tcw, h_pose_, 64);
  int e = 0;
  for (int i = 0; i < C.n; i++)
    if (C.mps[i] >= 0) C.outlier[i] = h_outl_[e++];
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono=false) with mbCheckOrientation, retried at
// retry_th while it finds fewer than min_matches (retry_th 0: no retry), then PoseOptimization on
// its matches when there are at least min_matches -- the whole chain on the device, one sync.
// Returns nmatches; the pose and outliers are applied when D1 ran.
int MapEngine::gpu_frame_chain(MapFrameH& C, const GridFrame& G, float* Tcw, const MapFrameH& L,
                               const float* Tlast, float th, float retry_th, int min_matches,
                               int retry_below, bool spec) {
  if (retry_below < 0) retry_below = min_matches;
  const double t_pack = prof_on_ ? now_us() : 0;
  const int n1 = L.n;
  uint8_t* hk = h_last_ + kDescBytes;
  float* hX = (float*)(hk + (size_t)n1 * sizeof(mmt_kp));
  uint8_t* hD = (uint8_t*)(hX + 3 * (size_t)n1);
  uint8_t* hA = hD + 32 * (size_t)n1;
  uint8_t* hO = hA + n1;
  memcpy(hk, L.kps, sizeof(mmt_kp) * (size_t)n1);
  int nact = 0;
  for (int i = 0; i < n1; i++) {
    const int h = L.mps[i];
    hA[i] = h >= 0 && !L.outlier[i];
    nact += hA[i];
    hO[i] = 0;
    if (h >= 0) {
      const MPoint& p = mp(h);
      memcpy(hX + 3 * (size_t)i, p.pos, 12);
      memcpy(hD + 32 * (size_t)i, p.desc, 32);
      hO[i] = p.nObs > 0;
    }
  }
  if (prof_on_) prof_[9] += now_us() - t_pack;
  pose_desc_fill(h_last_, d_last_, Tcw);
  MMT_HIP(hipMemcpyAsync(d_last_, h_last_, kDescBytes + last_bytes(n1), hipMemcpyHostToDevice,
                         s_));
  LastFrameDev LD;
  LD.keys = (const mmt_kp*)(d_last_ + kDescBytes);
  LD.Xw = (const float*)(d_last_ + kDescBytes + (size_t)n1 * sizeof(mmt_kp));
  LD.mp_desc = (const uint8_t*)(LD.Xw + 3 * (size_t)n1);
  LD.active = LD.mp_desc + 32 * (size_t)n1;
  LD.obs = LD.active + n1;
  LD.n = n1;
  memcpy(LD.Tcw, Tlast, 64);
  // D1's edges are built by the matcher kernels from their final bindings
  MapEdgeArgs e = edge_args(G);
  e.nm = d_nm_;
  e.min_matches = min_matches;
  e.src_X = LD.Xw;
  launch_sbp_frame(G, Tcw, LD, th, 0, 1, c2_, d_match_, d_nm_, s_, nullptr, 0, &e);
  if (retry_th > 0)
    launch_sbp_frame(G, Tcw, LD, retry_th, 0, 1, c2_, d_match_, d_nm_, s_, d_nm_, retry_below, &e);
  spec = spec && spec_on_;
  if (spec) {  // the final matches (D1 does not change them) ahead of D1, for speculate_local_map
    MMT_HIP(hipMemcpyAsync(h_early_, d_out_, kOutHdr + 4 * (size_t)C.n, hipMemcpyDeviceToHost, s_));
    MMT_HIP(hipEventRecord(ev_early_, s_));
  }
  launch_pose_opt(d_pod_, 1, std::min(C.n, nact), s_);
  MMT_HIP(hipMemcpyAsync(h_out_, d_out_, out_bytes(C.n), hipMemcpyDeviceToHost, s_));
  if (!spec || !overlap_c3_) run_overlap();
  if (spec) {
    MMT_HIP(hipEventSynchronize(ev_early_));
    if (*(const int*)h_early_ >= min_matches) speculate_local_map(L, C.n);
  }
  MMT_HIP(hipStreamSynchronize(s_));
  std::fill(C.mps.begin(), C.mps.end(), -1);
  for (int i2 = 0; i2 < C.n; i2++)
    if (h_match_[i2] >= 0) C.mps[i2] = L.mps[h_match_[i2]];
  const int nm = *h_nm_;
  if (nm >= min_matches) apply_pose_opt(C, Tcw);
  return nm;
}

void MapEngine::gpu_flush_pool(hipStream_t st) {
  if (!st) st = s_;
  // grow the pool with the map, then scatter the changed records
  if ((int)pts_.size() > pool_cap_) {
    const int cap = std::max((int)pts_.size() + 8192, 2 * pool_cap_);
    LocalPointDev* np = nullptr;
    uint8_t* nd = nullptr;
    MMT_HIP(hipMalloc((void**)&np, sizeof(LocalPointDev) * (size_t)cap));
    MMT_HIP(hipMalloc((void**)&nd, 32 * (size_t)cap));
    if (pool_cap_ > 0) {
      MMT_HIP(hipMemcpyAsync(np, d_pool_, sizeof(LocalPointDev) * (size_t)pool_cap_,
                             hipMemcpyDeviceToDevice, st));
      MMT_HIP(hipMemcpyAsync(nd, d_pool_desc_, 32 * (size_t)pool_cap_, hipMemcpyDeviceToDevice,
                             st));
      MMT_HIP(hipStreamSynchronize(st));
      auto drop = [&](void* p) {
        dallocs_.erase(std::find(dallocs_.begin(), dallocs_.end(), p));
        (void)hipFree(p);
      };
      drop(d_pool_);
      drop(d_pool_desc_);
    }
    d_pool_ = np;
    d_pool_desc_ = nd;
    dallocs_.push_back(np);
    dallocs_.push_back(nd);
    pool_cap_ = cap;
  }
  const int nd = (int)dirty_.size();
  if (nd == 0) return;
  if (nd > up_cap_) {
    MMT_HIP(hipStreamSynchronize(st));
    if (d_up_) {
      dallocs_.erase(std::find(dallocs_.begin(), dallocs_.end(), (void*)d_up_));
      hallocs_.erase(std::find(hallocs_.begin(), hallocs_.end(), (void*)h_up_));
      (void)hipFree(d_up_);
      (void)hipHostFree(h_up_);
    }
    up_cap_ = std::max(nd + 4096, 2 * up_cap_);
    d_up_ = dev<PoolUpdate>(up_cap_);
    h_up_ = pinned<PoolUpdate>(up_cap_);
  }
  for (int q = 0; q < nd; q++) {
    if (q + 8 < nd) prefetch_point(dirty_[q + 8]);
    const int h = dirty_[q];
    MPoint& p = pts_[h];
    PoolUpdate& u = h_up_[q];
    u.h = h;
    memcpy(u.p.Xw, p.pos, 12);
    memcpy(u.p.normal, p.normal, 12);
    u.p.min_dist = p.minDist;
    u.p.max_dist = p.maxDist;
    u.p.skip = 0;
    memcpy(u.desc, p.desc, 32);
    p.dirty = false;
  }
  MMT_HIP(hipMemcpyAsync(d_up_, h_up_, sizeof(PoolUpdate) * (size_t)nd, hipMemcpyHostToDevice,
                         st));
  launch_pool_scatter(d_up_, nd, d_pool_, d_pool_desc_, st);
  dirty_.clear();
}

// ------------------------------------------------------------------ map dump (tests)
void MapEngine::dump(int32_t* sizes, const mmt_map_dump_arrays* out) const {
  long nobs = 0, nconn = 0, nord = 0, nchild = 0, nslots = 0;
  for (size_t j = 0; j < pts_.size(); j++) nobs += (long)pts_[j].obs.size();
  for (const KFrame& K : kfs_) {
    nconn += (long)K.conn.size();
    nord += (long)K.ordered.size();
    nchild += (long)K.children.size();
    nslots += (long)K.mps.size();
  }
  const long n[7] = {(long)kfs_.size(), (long)pts_.size(), nobs, nconn, nord, nchild, nslots};
  for (int i = 0; i < 7; i++) sizes[i] = (int32_t)n[i];
  if (!out) return;
  long c = 0, o = 0, ch = 0, sl = 0;
  for (size_t k = 0; k < kfs_.size(); k++) {
    const KFrame& K = kfs_[k];
    int64_t* ki = out->kf_i + 4 * k;
    ki[0] = K.id; ki[1] = K.frameId; ki[2] = K.bad; ki[3] = K.parent;
    memcpy(out->kf_T + 16 * k, K.Tcw, 64);
    out->kf_mps_start[k] = (int32_t)sl;
    for (int h : K.mps) out->kf_mps[sl++] = h;
    for (const auto& kv : K.conn) {
      int32_t* e = out->conn + 3 * c++;
      e[0] = (int32_t)k; e[1] = kv.first; e[2] = kv.second;
    }
    for (int q : K.ordered) {
      int32_t* e = out->ord + 3 * o++;
      const auto it = K.conn.find(q);
      e[0] = (int32_t)k; e[1] = q; e[2] = it == K.conn.end() ? -1 : it->second;
    }
    for (int q : K.children) {
      int32_t* e = out->child + 2 * ch++;
      e[0] = (int32_t)k; e[1] = q;
    }
  }
  out->kf_mps_start[kfs_.size()] = (int32_t)sl;
  long b = 0;
  for (size_t j = 0; j < pts_.size(); j++) {
    const MPoint& p = pts_[j];
    float* f = out->pt_f + 5 * j;
    memcpy(f, p.pos, 12);
    f[3] = p.minDist; f[4] = p.maxDist;
    int32_t* pi = out->pt_i + 5 * j;
    pi[0] = p.bad; pi[1] = p.nObs; pi[2] = p.refKF; pi[3] = p.firstKFid; pi[4] = p.replaced;
    out->obs_start[j] = (int32_t)b;
    for (const auto& ob : p.obs) {
      const KFrame& K = kfs_[ob.first];
      int32_t* oi = out->obs_i + 3 * b;
      float* of = out->obs_f + 4 * b;
      oi[0] = ob.first; oi[1] = ob.second; oi[2] = K.keys[ob.second].octave;
      of[0] = K.keys[ob.second].x; of[1] = K.keys[ob.second].y;
      of[2] = K.depth[ob.second]; of[3] = K.uR[ob.second];
      b++;
    }
  }
  out->obs_start[pts_.size()] = (int32_t)b;
}

// ------------------------------------------------------------------ Tracking
void MapEngine::initialize(MapFrameH& C, const float* Tcw) {
  const int kf = new_keyframe(C, Tcw);
  kf_store_add(kf);
  for (int i = 0; i < C.n; i++) {
    const float z = C.depth[i];
    if (z > 0) {
      float x3D[3];
      unproject(cam_, Tcw, C.kps[i].x, C.kps[i].y, z, x3D);
      const int h = new_point_kf(x3D, kf);
      add_observation(h, kf, i);
      kfs_[kf].mps[i] = h;
      compute_distinctive(h);
      update_normal_depth(h);
      C.mps[i] = h;
    }
  }
  process_new_keyframe(kf);
  map_point_culling(kf);
  local_mapping(kf);  // keyframe 0 never enters the database (LoopClosing.cc:95)
  lastKFFrameId_ = C.id;
  localKFs_.assign(1, kf);
  localPts_.clear();
  for (size_t h = 0; h < pts_.size(); h++)
    if (!pts_[h].bad) localPts_.push_back((int)h);  // mpMap->GetAllMapPoints()
  refKF_ = kf;
  C.refKF = kf;
  state_ = 1;
}

void MapEngine::frame_done(const MapFrameH& C, const float* Tcw) {
  const int snap = snapKF_;
  snapKF_ = -1;
  if (C.refKF < 0) return;
  // Tcr = mTcw * mpReferenceKF->GetPoseInverse(), with the keyframe's pose as Track() leaves it
  // (before the mapping thread's local BA of a keyframe this frame inserted)
  mat4_mul(Tcw, C.refKF == snap ? snapTwc_ : kfs_[C.refKF].Twc, Tlr_);
  hasTlr_ = true;
}

void MapEngine::update_last_frame(MapFrameH& L, float* Tlast) {  // Tracking.cc:2894-2960
  if (L.refKF >= 0 && hasTlr_) mat4_mul(Tlr_, kfs_[L.refKF].Tcw, Tlast);
  if (lastKFFrameId_ == L.id) return;
  // The reference sorts (depth, index) and walks the prefix up to the first point that is both
  // beyond thDepth and past the 200th: that prefix is every close point plus the nearest far one,
  // or the 201 nearest points when fewer than 200 are close.  The temporary points are identities
  // only (C2 reads them by key index, they die with the frame), so the set is selected in O(n)
  // instead of sorting the keys.
  auto make = [&](int i) {
    if (L.mps[i] < 0 || mp(L.mps[i]).nObs < 1) {
      MPoint p;  // MapPoint(x3D, mpMap, &mLastFrame, i): C2 reads its position and descriptor
      unproject(cam_, Tlast, L.kps[i].x, L.kps[i].y, L.depth[i], p.pos);
      memcpy(p.desc, L.desc + 32 * (size_t)i, 32);
      temps_.push_back(p);
      L.mps[i] = kTemp + (int)temps_.size() - 1;
    }
  };
  temps_.reserve(L.n);
  far_.clear();
  int nclose = 0;
  for (int i = 0; i < L.n; i++) {
    const float z = L.depth[i];
    if (!(z > 0)) continue;
    if (z > cam_.thDepth) {
      far_.push_back({z, i});
    } else {
      make(i);
      nclose++;
    }
  }
  const size_t need = std::min(far_.size(), (size_t)(nclose >= 200 ? 1 : 201 - nclose));
  if (need == 0) return;
  std::nth_element(far_.begin(), far_.begin() + (need - 1), far_.end());
  for (size_t j = 0; j < need; j++) make(far_[j].second);
}

// TrackWithMotionModel / TrackReferenceKeyFrame's outlier discard: returns nmatches
int MapEngine::discard_outliers(MapFrameH& C, int nmatches, int* nmatchesMap) {
  *nmatchesMap = 0;
  for (int i = 0; i < C.n; i++) {
    if (C.mps[i] < 0) continue;
    if (C.outlier[i]) {
      const int h = C.mps[i];
      MPoint& p = mp(h);
      C.mps[i] = -1;
      C.outlier[i] = 0;
      p.trackInView = false;
      p.lastSeen = curId_;
      if (h < kTemp) hot_[h].lastSeen = (int)curId_;
      nmatches--;
    } else if (mp(C.mps[i]).nObs > 0) {
      (*nmatchesMap)++;
    }
  }
  return nmatches;
}

bool MapEngine::track_with_motion_model(MapFrameH& C, const GridFrame& G, float* Tcw,
                                        MapFrameH& L, float* Tlast, const float* vel,
                                        MapStatsH& st) {
  MAP_PROF(8, update_last_frame(L, Tlast));
  mat4_mul(vel, Tlast, Tcw);
  std::fill(C.mps.begin(), C.mps.end(), -1);
  const float th = 15;
  int nmatches;
  // C2 at th, again at 2 th below 20 matches, then D1 at 20 or more (Tracking.cc:2962-2990)
  MAP_PROF(0, nmatches = gpu_frame_chain(C, G, Tcw, L, Tlast, th, 2 * th, 20, -1, true));
  st.matches_mm = nmatches;
  if (nmatches < 20) return false;
  int nmatchesMap = 0;
  discard_outliers(C, nmatches, &nmatchesMap);
  mbVO_ = nmatchesMap < 20;
  return nmatchesMap >= 10;
}

bool MapEngine::track_reference_subst(MapFrameH& C, const GridFrame& G, float* Tcw,
                                      const MapFrameH& L, const float* Tlast) {
  std::fill(C.mps.begin(), C.mps.end(), -1);
  memcpy(Tcw, Tlast, 64);
  const int nmatches = gpu_frame_chain(C, G, Tcw, L, Tlast, 15, 0, 15);
  if (nmatches < 15) {
    std::fill(C.mps.begin(), C.mps.end(), -1);
    return false;
  }
  int nmatchesMap = 0;
  discard_outliers(C, nmatches, &nmatchesMap);
  return nmatchesMap >= 10;
}

// Relocalization substitute (pinned deviation, as oracle/map_ref.cpp relocalization_subst): the
// reference keyframe and its best 10 covisibles as candidates, each searched as TrackWithMotionModel
// searches the last frame (the keyframe as the last frame, th 15, again at 30 below 20 matches, at
// the pose the motion model predicts from the last, flow-tracked, frame), then the reference's
// acceptance of Tracking.cc:3700-3770 (PoseOptimization: fewer than 10 inliers -> next candidate;
// outliers dropped; 50 inliers or more -> relocalised).
bool MapEngine::relocalization_subst(MapFrameH& C, const GridFrame& G, float* Tcw,
                                     const float* Tlast, const float* vel) {
  std::vector<int> cand;
  if (refKF_ >= 0 && !kfs_[refKF_].bad) cand.push_back(refKF_);
  if (refKF_ >= 0) {
    const std::vector<int>& o = kfs_[refKF_].ordered;
    for (size_t q = 0; q < o.size() && q < 10; q++)
      if (!kfs_[o[q]].bad) cand.push_back(o[q]);
  }
  float Tpred[16];
  mat4_mul(vel, Tlast, Tpred);
  for (int k : cand) {
    const KFrame& K = kfs_[k];
    MapFrameH V;  // the keyframe as a last frame: its good map points, no outliers
    V.id = K.frameId;
    V.n = (int)K.keys.size();
    V.kps = K.keys.data();
    V.desc = K.desc.data();
    V.uR = K.uR.data();
    V.depth = K.depth.data();
    V.mps = K.mps;
    for (int& h : V.mps)
      if (h >= 0 && pts_[h].bad) h = -1;
    V.outlier.assign(V.mps.size(), 0);
    memcpy(Tcw, Tpred, 64);
    const int nm = gpu_frame_chain(C, G, Tcw, V, K.Tcw, 15, 30, 15, 20);
    if (nm < 15) continue;
    int nGood = 0;
    for (int i = 0; i < C.n; i++) nGood += C.mps[i] >= 0 && !C.outlier[i];
    if (nGood < 10) continue;
    for (int i = 0; i < C.n; i++)
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

// UpdateLocalKeyFrames' second part (Tracking.cc:3555-3604): per keyframe of the counted set, its
// first unmarked good covisible among the best 10, its first unmarked good child, and its parent
// (which ends the loop), up to 80 keyframes
template <class Marked, class Mark>
void MapEngine::expand_local_kfs(std::vector<int>& kfl, Marked marked, Mark mark) {
  const size_t n0 = kfl.size();
  for (size_t q = 0; q < n0; q++) {
    if (kfl.size() > 80) break;
    const KFrame& K = kfs_[kfl[q]];
    const size_t nn = std::min<size_t>(10, K.ordered.size());
    for (size_t a = 0; a < nn; a++) {
      const int id = K.ordered[a];
      if (!kfs_[id].bad && !marked(id)) {
        kfl.push_back(id);
        mark(id);
        break;
      }
    }
    for (int ch : K.children) {
      if (!kfs_[ch].bad && !marked(ch)) {
        kfl.push_back(ch);
        mark(ch);
        break;
      }
    }
    if (K.parent >= 0 && !marked(K.parent)) {
      kfl.push_back(K.parent);
      mark(K.parent);
      break;  // leaves the keyframe loop (Tracking.cc:3601)
    }
  }
}

void MapEngine::update_local_keyframes(MapFrameH& C) {  // Tracking::UpdateLocalKeyFrames
  // keyframeCounter (a std::map keyed by KeyFrame*, here by keyframe id): counts in a flat array,
  // then the touched ids in ascending order, as the map would iterate them
  if (kf_count_.size() < kfs_.size()) kf_count_.resize(kfs_.size(), 0);
  kf_touched_.clear();
  for (int i = 0; i < C.n; i++) {
    if (C.mps[i] < 0) continue;
    const MPoint& p = mp(C.mps[i]);
    if (!p.bad) {
      for (const auto& kv : p.obs)
        if (kf_count_[kv.first]++ == 0) kf_touched_.push_back(kv.first);
    } else {
      C.mps[i] = -1;
    }
  }
  if (kf_touched_.empty()) return;
  std::sort(kf_touched_.begin(), kf_touched_.end());
  int mx = 0, kmax = -1;
  localKFs_.clear();
  for (const int id : kf_touched_) {
    const int cnt = kf_count_[id];
    kf_count_[id] = 0;
    KFrame& K = kfs_[id];
    if (K.bad) continue;
    if (cnt > mx) {
      mx = cnt;
      kmax = id;
    }
    localKFs_.push_back(id);
    K.trackRef = curId_;
  }
  expand_local_kfs(
      localKFs_, [&](int id) { return kfs_[id].trackRef == curId_; },
      [&](int id) { kfs_[id].trackRef = curId_; });
  if (kmax >= 0) {
    refKF_ = kmax;
    C.refKF = kmax;
  }
}

void MapEngine::update_local_points() { collect_local_points(localKFs_, localPts_); }

void MapEngine::collect_local_points(const std::vector<int>& kfl, std::vector<int>& out) {
  // Tracking::UpdateLocalPoints over the keyframes kfl
  out.clear();
  // a keyframe's slots are about half empty (-1) in no predictable pattern: its handles are first
  // compacted without a branch, then visited in slot order (the same points in the same order).
  // mnTrackReferenceForFrame is a bit per point here (lp_seen_, tens of kB: the 70k slot visits
  // of a dense local map stay in cache), cleared again for the points this call marked; the one
  // call per frame (TrackLocalMap) makes it equal to the per-point frame id.
  std::vector<int>& buf = lp_buf_;
  const size_t words = (hot_.size() + 63) / 64;
  if (lp_seen_.size() < words) lp_seen_.resize(words, 0);
  for (int kf : kfl) {
    const std::vector<int>& mps = kfs_[kf].mps;
    buf.resize(mps.size());
    size_t n = 0;
    for (int h : mps) {
      buf[n] = h;
      // keyframes hold real points only (Track clears the VO points before a keyframe is made)
      n += (unsigned)h < (unsigned)kTemp;
    }
    for (size_t i = 0; i < n; i++) {
      const int h = buf[i];
      uint64_t& wd = lp_seen_[(size_t)h >> 6];
      const uint64_t bit = 1ull << (h & 63);
      if (wd & bit) continue;
      if (!hot_[h].bad) {  // a bad point stays unmarked and is skipped again, as the reference
        out.push_back(h);
        wd |= bit;
      }
    }
  }
  for (int h : out) lp_seen_[(size_t)h >> 6] &= ~(1ull << (h & 63));
}

// UpdateLocalMap from C2's final matches while D1 runs (track_with_motion_model; L: the last frame
// whose points the matches index).  Nothing of the map changes between here and TrackLocalMap but
// the frame's bindings, which D1's outliers can only remove: commit_local_map checks that every
// counted keyframe keeps a count (the same keyframe set, so the same expansion and points) and
// recomputes the best-counted keyframe.  Marks are private (spec_mark_), so a speculation that is
// never taken leaves no trace.
void MapEngine::speculate_local_map(const MapFrameH& L, int n) {
  spec_discard();
  const int* match = (const int*)(h_early_ + kOutHdr);
  if (spec_cnt_.size() < kfs_.size()) spec_cnt_.resize(kfs_.size(), 0);
  if (spec_mark_.size() < kfs_.size()) spec_mark_.resize(kfs_.size(), 0);
  spec_mps_.assign(n, -1);
  spec_touched_.clear();
  for (int i = 0; i < n; i++) {
    if (match[i] < 0) continue;
    const int h = L.mps[match[i]];
    spec_mps_[i] = h;
    if (h < 0) continue;
    const MPoint& p = mp(h);
    if (p.bad) continue;
    for (const auto& kv : p.obs)
      if (spec_cnt_[kv.first]++ == 0) spec_touched_.push_back(kv.first);
  }
  std::sort(spec_touched_.begin(), spec_touched_.end());
  const long stamp = ++spec_stamp_;
  spec_kfs_.clear();
  for (const int id : spec_touched_)
    if (!kfs_[id].bad) {
      spec_kfs_.push_back(id);
      spec_mark_[id] = stamp;
    }
  spec_frame_ = curId_;
  if (spec_kfs_.empty()) return;  // (the reference's early return keeps the last local map)
  expand_local_kfs(
      spec_kfs_, [&](int id) { return spec_mark_[id] == stamp; },
      [&](int id) { spec_mark_[id] = stamp; });
  collect_local_points(spec_kfs_, spec_pts_);
  spec_valid_ = true;
  spec_tries_++;
}

void MapEngine::spec_discard() {
  for (const int id : spec_touched_) spec_cnt_[id] = 0;
  spec_touched_.clear();
  spec_valid_ = false;
}

bool MapEngine::commit_local_map(MapFrameH& C) {
  if (!spec_valid_ || spec_frame_ != curId_ || (int)spec_mps_.size() != C.n) {
    spec_discard();
    return false;
  }
  // the bindings now: a subset of the speculated ones; the dropped ones' counts come off
  bool ok = true;
  for (int i = 0; i < C.n && ok; i++) {
    const int h = C.mps[i], s0 = spec_mps_[i];
    if (h >= 0 && h != s0) {
      ok = false;
    } else if (s0 >= 0 && h < 0) {
      const MPoint& p = mp(s0);
      if (!p.bad)
        for (const auto& kv : p.obs) spec_cnt_[kv.first]--;
    }
  }
  for (size_t q = 0; q < spec_touched_.size() && ok; q++) {
    const int id = spec_touched_[q];
    ok = kfs_[id].bad || spec_cnt_[id] > 0;
  }
  if (!ok) {
    spec_discard();
    return false;
  }
  for (int i = 0; i < C.n; i++)
    if (C.mps[i] >= 0 && mp(C.mps[i]).bad) C.mps[i] = -1;
  int mx = 0, kmax = -1;
  for (const int id : spec_touched_) {
    const int cnt = spec_cnt_[id];
    spec_cnt_[id] = 0;
    if (kfs_[id].bad) continue;
    if (cnt > mx) {
      mx = cnt;
      kmax = id;
    }
  }
  spec_touched_.clear();
  spec_valid_ = false;
  for (const int id : spec_kfs_) kfs_[id].trackRef = curId_;
  localKFs_.swap(spec_kfs_);
  localPts_.swap(spec_pts_);
  if (kmax >= 0) {
    refKF_ = kmax;
    C.refKF = kmax;
  }
  spec_hits_++;
  return true;
}

void MapEngine::search_local_points(MapFrameH& C, const GridFrame& G, const float* Tcw) {
  const double t_pack = prof_on_ ? now_us() : 0;
  // Tracking::SearchLocalPoints (Tracking.cc:3416-3466)
  for (int i = 0; i < C.n; i++) {
    if (C.mps[i] < 0) continue;
    const int h = C.mps[i];
    MPoint& p = mp(h);
    if (p.bad) {
      C.mps[i] = -1;
    } else {
      p.visible++;
      p.lastSeen = curId_;
      if (h < kTemp) hot_[h].lastSeen = (int)curId_;
      p.trackInView = false;
    }
  }
  const int m = (int)localPts_.size();
  grow_local(m);
  gpu_flush_pool();
  const SelLayout sl(m, C.n);
  int* ids = (int*)(h_sel_ + sl.ids);
  uint8_t* skip = h_sel_ + sl.skip;
  uint8_t* taken = h_sel_ + sl.taken;
  for (int j = 0; j < m; j++) {
    const int h = localPts_[j];
    const PtHot& q = hot_[h];
    ids[j] = h;
    skip[j] = q.lastSeen == (int)curId_ || q.bad;
  }
  // the keys bound before the search: taken (Observations() > 0) and, for D1's edge list, their
  // points' positions
  float* bX = (float*)(h_sel_ + sl.bX);
  uint8_t* bHas = h_sel_ + sl.bHas;
  int nbase = 0;
  for (int i = 0; i < C.n; i++) {
    const int h = C.mps[i];
    taken[i] = 0;
    bHas[i] = h >= 0;
    if (h >= 0) {
      const MPoint& p = mp(h);
      taken[i] = p.nObs > 0;
      memcpy(bX + 3 * (size_t)i, p.pos, 12);
      nbase++;
    }
  }
  if (prof_on_) prof_[10] += now_us() - t_pack;
  pose_desc_fill(h_sel_, d_sel_, Tcw);
  MMT_HIP(hipMemcpyAsync(d_sel_, h_sel_, sl.total, hipMemcpyHostToDevice, s_));
  // ORBmatcher(0.8)::SearchByProjection's th: 3 for RGB-D, 5 right after a relocalisation
  const float th = curId_ < lastRelocFrameId_ + 2 ? 5.f : 3.f;
  LocalSel sel{(const int*)(d_sel_ + sl.ids), d_sel_ + sl.skip, d_inview_};
  // D1 over every key bound after the search (Tracking.cc:3189-3200), chained on the device: the
  // matcher kernel builds its edge list from the final bindings
  MapEdgeArgs e = edge_args(G);
  e.pool = d_pool_;
  e.ids = (const int*)(d_sel_ + sl.ids);
  e.has_base = d_sel_ + sl.bHas;
  e.base_X = (const float*)(d_sel_ + sl.bX);
  launch_search_local(G, Tcw, d_pool_, d_pool_desc_, m, th, d_sel_ + sl.taken, nullptr, c3_,
                      d_match_, d_nm_, s_, &sel, &e);
  launch_pose_opt(d_pod_, 1, std::min(C.n, nbase + m), s_);
  MMT_HIP(hipMemcpyAsync(h_out_, d_out_, out_bytes(C.n), hipMemcpyDeviceToHost, s_));
  if (m > 0) MMT_HIP(hipMemcpyAsync(h_inview_, d_inview_, (size_t)m, hipMemcpyDeviceToHost, s_));
  run_overlap();
  MMT_HIP(hipStreamSynchronize(s_));
  // IncreaseVisible for the points in view (mbTrackInView itself is read by the GPU search only,
  // from h_inview_: the host's copy of the flag is not kept, so only the points in view are touched)
  for (int j = 0; j < m; j++)
    if (!skip[j] && h_inview_[j]) mp(localPts_[j]).visible++;
  for (int i = 0; i < C.n; i++)
    if (h_match_[i] >= 0) C.mps[i] = localPts_[h_match_[i]];
}

bool MapEngine::track_local_map(MapFrameH& C, const GridFrame& G, float* Tcw) {
  MAP_PROF(2, if (!commit_local_map(C)) {
    update_local_keyframes(C);
    update_local_points();
  });
  if (prof_on_) {
    prof_cnt_[0] += localKFs_.size();
    prof_cnt_[1] += localPts_.size();
  }
  MAP_PROF(3, search_local_points(C, G, Tcw));  // C3, then D1 on the device
  MAP_PROF(4, apply_pose_opt(C, Tcw));
  matchesInliers_ = 0;
  for (int i = 0; i < C.n; i++) {
    if (C.mps[i] < 0 || C.outlier[i]) continue;
    MPoint& p = mp(C.mps[i]);
    p.found++;
    if (p.nObs > 0) matchesInliers_++;
  }
  if (curId_ < lastRelocFrameId_ + cam_.maxFrames && matchesInliers_ < 50) return false;
  return matchesInliers_ >= 30;
}

bool MapEngine::need_new_keyframe(const MapFrameH& C) {  // Tracking::NeedNewKeyFrame (RGB-D)
  const int nKFs = n_keyframes();
  if (curId_ < lastRelocFrameId_ + cam_.maxFrames && nKFs > cam_.maxFrames) return false;
  const int nMinObs = nKFs <= 2 ? 2 : 3;
  const int nRefMatches = tracked_map_points(refKF_, nMinObs);
  const bool bLocalMappingIdle = true;  // synchronous LocalMapping (pinned)
  int nNonTrackedClose = 0, nTrackedClose = 0;
  for (int i = 0; i < C.n; i++)
    if (C.depth[i] > 0 && C.depth[i] < cam_.thDepth) {
      if (C.mps[i] >= 0 && !C.outlier[i])
        nTrackedClose++;
      else
        nNonTrackedClose++;
    }
  const bool bNeedToInsertClose = (nTrackedClose < 100) && (nNonTrackedClose > 70);
  const float thRefRatio = nKFs < 2 ? 0.4f : 0.75f;
  const bool c1a = curId_ >= lastKFFrameId_ + cam_.maxFrames;
  const bool c1b = curId_ >= lastKFFrameId_ && bLocalMappingIdle;
  const bool c1c = matchesInliers_ < nRefMatches * 0.25 || bNeedToInsertClose;
  const bool c2 = (matchesInliers_ < nRefMatches * thRefRatio || bNeedToInsertClose) &&
                  matchesInliers_ > 15;
  return (c1a || c1b || c1c) && c2;
}

void MapEngine::create_new_keyframe(MapFrameH& C, const float* Tcw) {  // Tracking.cc:3333-3414
  double tb = prof_on_ ? now_us() : 0;
  const int kf = new_keyframe(C, Tcw);
  kf_store_add(kf);
  blk_time(0, tb);
  refKF_ = kf;
  C.refKF = kf;
  // the keys with depth sorted by (depth, index): a stable LSD radix sort on the depths' bits
  // (positive floats order as their bit patterns) over the keys in index order, 3 x 11 bits
  std::vector<uint32_t>& key = sort_key_;
  std::vector<int>& v = sort_idx_;
  std::vector<int>& tmp = sort_tmp_;
  key.clear();
  v.clear();
  for (int i = 0; i < C.n; i++)
    if (C.depth[i] > 0) {
      uint32_t b;
      memcpy(&b, &C.depth[i], 4);
      key.push_back(b);
      v.push_back(i);
    }
  if (!v.empty()) {
    const int nv = (int)v.size();
    std::vector<int> pos(nv);  // position of each entry's key
    for (int k = 0; k < nv; k++) pos[k] = k;
    tmp.resize(nv);
    for (int pass = 0; pass < 3; pass++) {
      uint32_t cnt[2049];
      memset(cnt, 0, sizeof(cnt));
      const int sh = 11 * pass;
      for (int k = 0; k < nv; k++) cnt[((key[pos[k]] >> sh) & 0x7FF) + 1]++;
      for (int b = 0; b < 2048; b++) cnt[b + 1] += cnt[b];
      for (int k = 0; k < nv; k++) tmp[cnt[(key[pos[k]] >> sh) & 0x7FF]++] = pos[k];
      pos.swap(tmp);
    }
    int nPoints = 0;
    for (int j = 0; j < nv; j++) {
      const int i = v[pos[j]];
      const float depth_i = C.depth[i];
      bool create = false;
      if (C.mps[i] < 0) {
        create = true;
      } else if (mp(C.mps[i]).nObs < 1) {
        create = true;
        C.mps[i] = -1;
      }
      if (create) {
        float x3D[3];
        unproject(cam_, Tcw, C.kps[i].x, C.kps[i].y, C.depth[i], x3D);
        const int h = new_point_kf(x3D, kf);
        add_observation(h, kf, i);
        kfs_[kf].mps[i] = h;
        compute_distinctive(h);
        update_normal_depth(h);
        C.mps[i] = h;
      }
      nPoints++;
      if (depth_i > cam_.thDepth && nPoints > 200) break;
    }
  }
  blk_time(1, tb);
  snapKF_ = kf;
  memcpy(snapTwc_, kfs_[kf].Twc, sizeof(snapTwc_));
  const double tp = prof_on_ ? now_us() : 0;
  process_new_keyframe(kf);  // mpLocalMapper->InsertKeyFrame(pKF), processed at once
  map_point_culling(kf);
  if (prof_on_) mstats_.pnk_us += now_us() - tp;
  local_mapping(kf);
  // mpLoopCloser->InsertKeyFrame: LoopClosing::DetectLoop adds every keyframe but the first to
  // the database (LoopClosing.cc:92-121); loop detection itself is out of scope
  if (voc_ && kfs_[kf].id != 0 && !kfs_[kf].bad) kfdb_add(kf);
  lastKFFrameId_ = C.id;
}

int MapEngine::track(MapFrameH& C, const GridFrame& G, float* Tcw, MapFrameH& L, float* Tlast,
                     float* vel, bool& has_vel, bool& bSecondFrame, MapStatsH& st,
                     hipStream_t s) {
  s_ = s;
  curId_ = C.id;
  const double t_track = prof_on_ ? now_us() : 0;
  bool bOK;
  // a branch that computes no pose leaves the motion model's prediction, or the last pose
  // (pinned as in the oracle: the reference's mCurrentFrame.mTcw stays empty there)
  if (has_vel)
    mat4_mul(vel, Tlast, Tcw);
  else
    memcpy(Tcw, Tlast, 64);
  if (state_ == 1) {
    // CheckReplacedInLastFrame (Tracking.cc:2766-2781): one level of MapPoint::GetReplaced
    for (int i = 0; i < L.n; i++)
      if (L.mps[i] >= 0 && L.mps[i] < kTemp && pts_[L.mps[i]].replaced >= 0)
        L.mps[i] = pts_[L.mps[i]].replaced;
    if (!has_vel || C.id < lastRelocFrameId_ + 2) {
      bSecondFrame = true;
      bOK = voc_ ? track_reference_kf(C, G, Tcw, Tlast) : track_reference_subst(C, G, Tcw, L, Tlast);
    } else {
      bSecondFrame = false;
      bOK = track_with_motion_model(C, G, Tcw, L, Tlast, vel, st);
      if (!bOK) {
        bSecondFrame = true;
        bOK = voc_ ? track_reference_kf(C, G, Tcw, Tlast)
                   : track_reference_subst(C, G, Tcw, L, Tlast);
      }
    }
  } else if (voc_) {  // Relocalization (Tracking.cc:3614-3776)
    bOK = relocalization(C, G, Tcw);  // from the prediction set above
    if (bOK) lastRelocFrameId_ = C.id;
  } else {
    bOK = relocalization_subst(C, G, Tcw, Tlast, vel);  // Relocalization (substitute)
    if (bOK) lastRelocFrameId_ = C.id;
  }
  C.refKF = refKF_;
  if (bOK && !mbVO_) {
    bOK = track_local_map(C, G, Tcw);
    st.inliers_local = matchesInliers_;
  }
  state_ = bOK ? 1 : 2;
  if (bOK) {
    // motion model from the map pose (Tracking.cc:1117-1125): LastTwc = [Rwc, Ow] of mLastFrame
    float LastTwc[16], Ow[3];
    mat4_eye(LastTwc);
    cam_centre(Tlast, Ow);
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) LastTwc[4 * r + c] = Tlast[4 * c + r];
      LastTwc[4 * r + 3] = Ow[r];
    }
    mat4_mul(Tcw, LastTwc, vel);
    has_vel = true;
  }
  pending_ok_ = bOK;
  if (prof_on_) {
    prof_[7] += now_us() - t_track;
    prof_n_++;
  }
  if (state_ == 2 && n_keyframes() <= 5) return 1;  // mpSystem->Reset(); return
  return 0;
}

void MapEngine::track_finish(MapFrameH& C, MapFrameH& L, const float* Tcw, MapStatsH& st) {
  const double t0 = prof_on_ ? now_us() : 0;
  if (pending_ok_) {
    for (int i = 0; i < C.n; i++)  // clean VO matches
      if (C.mps[i] >= 0 && mp(C.mps[i]).nObs < 1) {
        C.outlier[i] = 0;
        C.mps[i] = -1;
      }
    for (int i = 0; i < L.n; i++)  // delete temporal MapPoints (mLastFrame's become dangling)
      if (L.mps[i] >= kTemp) L.mps[i] = -1;
    temps_.clear();
    MAP_PROF(5, if (need_new_keyframe(C)) {
      const double tk = prof_on_ ? now_us() : 0;
      create_new_keyframe(C, Tcw);
      if (prof_on_) mstats_.kfnew_us += now_us() - tk;
      st.new_keyframe = 1;
    });
    for (int i = 0; i < C.n; i++)
      if (C.mps[i] >= 0 && C.outlier[i]) C.mps[i] = -1;
  }
  pending_ok_ = false;
  if (C.refKF < 0) C.refKF = refKF_;
  if (prof_on_) {
    prof_[7] += now_us() - t0;
    prof_[6] = prof_[7];
    for (int k = 0; k < 6; k++) prof_[6] -= prof_[k];
    prof_[6] -= prof_[8];
  }
}

}  // namespace mmt
