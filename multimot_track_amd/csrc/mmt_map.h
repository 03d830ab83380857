// multimot_track_amd/csrc/mmt_map.h -- ORB-SLAM2 map tracking for RGB-D: the
// MapPoint / KeyFrame state and Tracking's map branch that produce the ego pose the flow solve
// (PoseOptimizationFlow2Cam, D2) starts from.
//
// Reference: MapPoint.cc, KeyFrame.cc, Map.cc; Tracking.cc:985-1176 (Track's map branch),
// 2531-2575 (StereoInitialization), 2766-3612 (CheckReplacedInLastFrame, UpdateLastFrame,
// TrackWithMotionModel, TrackReferenceKeyFrame, TrackLocalMap, NeedNewKeyFrame, CreateNewKeyFrame,
// SearchLocalPoints, UpdateLocalMap); LocalMapping.cc:61-87, 131-208, 458-538, 636-700
// (ProcessNewKeyFrame, MapPointCulling, SearchInNeighbors with ORBmatcher::Fuse,
// LocalBundleAdjustment (Optimizer.cc:3341-3666), KeyFrameCulling, run synchronously after each new
// keyframe; mmt_localmap.hip).
//
// The bookkeeping (observations, covisibility graph, spanning tree, local map, keyframe policy)
// is host C++ where the reference keeps it; the data-parallel parts run on the GPU through the
// C1-C3 / D1 kernels: SearchByProjection frame-to-frame (k_sbp_frame + k_match_greedy),
// SearchLocalPoints (k_local_cand + k_match_greedy over a device-resident pool of the map points,
// updated by scatter as points are created or refined) and PoseOptimization (k_pose_opt).
// Pinned choices and deviations (the same in oracle/oracle_map.h):
//  * maps and sets keyed by KeyFrame* iterate in keyframe creation order;
//  * LocalMapping runs synchronously (always idle for NeedNewKeyFrame, never aborted) and does
//    ProcessNewKeyFrame without the BoW conversion, MapPointCulling, SearchInNeighbors, the local
//    BA (GPU, mmt_ba.hip) and KeyFrameCulling; CreateNewMapPoints needs the missing vocabulary;
//  * TrackReferenceKeyFrame's SearchByBoW becomes SearchByProjection against the last frame at the
//    last frame's pose (th 15) + the reference's PoseOptimization and acceptance tests;
//  * Relocalization (BoW database + PnPsolver) becomes a search of the reference keyframe's and
//    its best covisibles' map points at the motion model's prediction from the last frame, with
//    the reference's acceptance tests (relocalization_subst).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <map>
#include <set>
#include <unordered_map>
#include <utility>
#include <memory>
#include <vector>

#include "mmt_ba.h"
#include "mmt_bow.h"
#include "mmt_internal.h"
#include "mmt_match.h"
#include "mmt_track.h"

namespace mmt {

struct MapCamH {
  int W = 0, H = 0;
  float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, bf = 0;
  float thDepth = 0;  // mThDepth = mbf * ThDepth / fx (Tracking.cc:225)
  int maxFrames = 0;  // mMaxFrames = fps (Tracking.cc:176)
  int nlevels = 0;
  float logScale = 0;
  std::vector<float> scale, invSigma2;
};

// An array in chunks of 2^kShift elements: indexing as a vector's (one more load), push_back never
// moves the elements already stored (references stay valid)
template <class T, int kShift = 13>
class ChunkArray {
 public:
  T& operator[](size_t i) { return chunks_[i >> kShift][i & kMask]; }
  const T& operator[](size_t i) const { return chunks_[i >> kShift][i & kMask]; }
  size_t size() const { return n_; }
  void push_back(const T& v) {
    if ((n_ >> kShift) >= chunks_.size()) chunks_.emplace_back(new T[kChunk]);
    (*this)[n_++] = v;
  }
  void clear() {
    chunks_.clear();
    n_ = 0;
  }

 private:
  static constexpr size_t kChunk = (size_t)1 << kShift, kMask = kChunk - 1;
  std::vector<std::unique_ptr<T[]>> chunks_;
  size_t n_ = 0;
};

struct MPoint {
  float pos[3] = {0, 0, 0};
  float normal[3] = {0, 0, 0};
  float minDist = 0, maxDist = 0;
  uint8_t desc[32] = {0};
  std::vector<std::pair<int, int>> obs;  // mObservations (keyframe id, key index), id-ascending
  int nObs = 0;
  int refKF = -1;
  int firstKFid = -1;
  int visible = 1, found = 1;
  bool bad = false;
  bool trackInView = false;
  bool dirty = false;  // pool record out of date
  long lastSeen = 0;  // real points: mirrored in MapEngine::hot_ (the per-frame scans read that)
  int replaced = -1;  // mpReplaced
  long fuseCand = 0, baLocal = 0;  // mnFuseCandidateForKF, mnBALocalForKF
  int desc_ver = 0;   // bumped by ComputeDistinctiveDescriptors (Fuse results read it)
  int obs_index(int kf) const {
    for (const auto& o : obs)
      if (o.first == kf) return o.second;
    return -1;
  }
};

struct KFrame {
  int id = 0;
  long frameId = 0;
  float Tcw[16], Twc[16], Ow[3];
  std::vector<mmt_kp> keys;
  std::vector<float> uR, depth;
  std::vector<uint8_t> desc;
  std::vector<int> mps;
  std::map<int, int> conn;  // mConnectedKeyFrameWeights
  std::vector<int> ordered;
  bool firstConnection = true;
  int parent = -1;
  std::set<int> children;
  long trackRef = 0;
  bool bad = false;
  long fuseTarget = 0, baLocal = 0, baFixed = 0;  // mnFuseTargetForKF, mnBALocalForKF, mnBAFixedForKF
  FuseKF dev{};  // the keyframe's keys, descriptors, mvuRight and grid on the device (KF store)
  // with a vocabulary: mBowVec, mFeatVec, and the KeyFrameDatabase query fields (KeyFrame.h:146-149;
  // mRelocScore uninitialised in the reference: pinned 0)
  BowVecH bow;
  FeatVecH fv;
  bool hasBow = false;
  long relocQuery = 0;
  int relocWords = 0;
  float relocScore = 0;
};

// glibc's rand() (random_r TYPE_3, srand(1) for an unseeded process): the stream
// DUtils::Random::RandomInt draws PnPsolver's minimal sets from (Random.cpp:47-50)
class GlibcRandH {
 public:
  GlibcRandH();
  int next();
  int random_int(int min, int max);

 private:
  std::vector<int32_t> r_;
};

// LocalMapping counters (tests, profiling)
struct MappingStats {
  long n_ba = 0, n_fused = 0, n_culled = 0, n_ba_erased = 0, ba_trials = 0, ba_edges = 0,
       ba_kfs = 0, ba_pts = 0, ba_max_opt = 0, fuse_launches = 0, fuse_queries = 0,
       fuse_relaunches = 0, n_reparent = 0;
  double lm_us = 0, ba_us = 0, fuse_us = 0;  // host wall time (MMT_MAP_PROFILE)
  // finer host wall times of the keyframe path (MMT_MAP_PROFILE; printed at destruction)
  double kfnew_us = 0, pnk_us = 0, sin_us = 0, basolve_us = 0, cull_us = 0, lmsync_us = 0;
  double cnmp_us = 0;  // CreateNewMapPoints (vocabulary path), inside sin_us
  static constexpr int kBlk = 18;  // finer blocks of the keyframe path (names in ~MapEngine)
  double blk_us[kBlk] = {};
  long n_lm = 0;
};

// The map-path view of one Frame: its ORB output and B3 arrays (host copies of the device ones)
// and its map state.
struct MapFrameH {
  long id = 0;
  int n = 0;
  const mmt_kp* kps = nullptr;
  const uint8_t* desc = nullptr;
  const float* uR = nullptr;     // mvuRight
  const float* depth = nullptr;  // mvDepth
  std::vector<int> mps;          // mvpMapPoints (point handle or -1)
  std::vector<uint8_t> outlier;  // mvbOutlier
  int refKF = -1;                // mpReferenceKF
  BowVecH bow;                   // mBowVec / mFeatVec (Frame::ComputeBoW, with a vocabulary)
  FeatVecH fv;
  bool hasBow = false;
};

// counters of the vocabulary path (tests, mmt_map_counters)
struct BowStatsH {
  long n_bow_frames = 0, n_trk = 0, n_trk_ok = 0, n_reloc = 0, n_reloc_ok = 0, n_reloc_cands = 0,
       n_pnp_found = 0, n_sbp_rounds = 0, n_triangulated = 0, n_sft_matches = 0, n_kfdb = 0;
};

struct MapStatsH {
  int state = 0;           // 0 not initialised, 1 OK, 2 LOST
  int matches_mm = -1;     // TrackWithMotionModel's nmatches before PoseOptimization (-1: not run)
  int inliers_local = -1;  // mnMatchesInliers after TrackLocalMap (-1: not run)
  int n_keyframes = 0, n_mappoints = 0;
  int new_keyframe = 0;
  float Tcw_map[16];       // the map branch's pose: PoseOptimizationFlow2Cam's initial estimate
};

constexpr size_t kDescBytes = 256;  // D1's descriptor at the head of an upload block
constexpr size_t kOutHdr = 128;     // [nm][ninl][pad][pose] at the head of the download block

class MapEngine {
 public:
  ~MapEngine();
  void setup(const MapCamH& cam, int kcap);
  void reset();  // Tracking::Reset (map part)
  long next_frame_id() { return frameNextId_++; }
  void prepare(MapFrameH& F) const;  // mvpMapPoints / mvbOutlier of a new frame
  // StereoInitialization's map part (Tracking.cc:2531-2575)
  void initialize(MapFrameH& C, const float* Tcw);
  // Track()'s map branch (Tracking.cc:985-1176) up to the pose: TrackWithMotionModel (or its
  // substitute) and TrackLocalMap; G: the current frame on the device.  Returns 1 when the
  // reference resets the system (LOST with <= 5 keyframes, Tracking.cc:1165-1172).
  int track(MapFrameH& C, const GridFrame& G, float* Tcw, MapFrameH& L, float* Tlast, float* vel,
            bool& has_vel, bool& bSecondFrame, MapStatsH& st, hipStream_t s);
  // the rest of the branch, which the pose does not depend on: VO-match and temporal-point
  // cleanup, NeedNewKeyFrame / CreateNewKeyFrame (Tracking.cc:1127-1160); host only, so it runs
  // while the flow solve that starts from the pose is on the GPU
  void track_finish(MapFrameH& C, MapFrameH& L, const float* Tcw, MapStatsH& st);
  // host work to run while the next device chain (C2 or C3 + D1) of track() executes, once: the
  // tracker hands the previous frame's object path here, which would otherwise wait for the GPU
  // beside the ego solve.  Returns whether it is still pending (track() ran no chain).
  void set_overlap(std::function<void()> fn) { overlap_ = std::move(fn); }
  bool overlap_pending() const { return (bool)overlap_; }
  // end of Track: mlRelativeFramePoses.push_back(Tcw * Tref^-1) (Tracking.cc:2481-2489)
  void frame_done(const MapFrameH& C, const float* Tcw);
  int state() const { return state_; }
  int n_keyframes() const;
  int n_mappoints() const { return n_good_; }
  // the current frame on the device (B3 grid, keys, descriptors): the keyframe made from it copies
  // them into the keyframe store, where Fuse reads them
  void set_frame_grid(const GridFrame& G) { G_ = G; }
  const MappingStats& mapping_stats() const { return mstats_; }
  // MMT_MAP_PROFILE: adds the time since t to block k and restarts t
  void blk_time(int k, double& t) {
    if (!prof_on_) return;
    const double n = prof_now_us();
    mstats_.blk_us[k] += n - t;
    t = n;
  }
  static double prof_now_us();
  // host prefetch of map point h's record (loops over point lists walk a 100k-point map in
  // random order: one cache miss per record otherwise); MMT_NO_PREFETCH builds without it (A/B)
  void prefetch_point(int h) const {
#ifndef MMT_NO_PREFETCH
    if (h >= 0 && h < kTemp && (size_t)h < pts_.size()) __builtin_prefetch(&pts_[h]);
#else
    (void)h;
#endif
  }
  // test knob: KeyFrameCulling's redundancy ratio (0.9 in the reference, LocalMapping.cc:697)
  void set_cull_ratio(double r) { cull_ratio_ = r; }
  // the map as flat arrays (mmt_map_dump, include/mmt.h): sizes[7]; arrays written when out != 0
  void dump(int32_t* sizes, const mmt_map_dump_arrays* out) const;
  // System's vocabulary (System.cc:67): with one, TrackReferenceKeyFrame, Relocalization and
  // CreateNewMapPoints run as the reference's (mmt_bowmap.hip); without, the substitutes above
  void set_vocabulary(Vocabulary* v);
  const BowStatsH& bow_stats() const { return bstats_; }

 private:
  std::function<void()> overlap_;
  std::vector<int> kf_count_, kf_touched_;  // update_local_keyframes' counter
  std::vector<int> lp_buf_;                  // update_local_points' compacted slots
  std::vector<uint64_t> lp_seen_;            // update_local_points' per-point marks (bits)
  // TrackLocalMap's local keyframes and points, computed from C2's matches while D1 runs on the
  // GPU (speculate_local_map) and taken by track_local_map when D1's outliers leave every counted
  // keyframe with a count (commit_local_map); MMT_LOCALMAP_SPEC=0 turns it off (A/B)
  bool spec_on_ = true, spec_valid_ = false;
  // the overlap work runs while the C3 chain executes when the C2 chain's wait holds the local
  // map speculation (MMT_OVERLAP_C3=0: in the C2 chain as before, A/B)
  bool overlap_c3_ = true;
  long spec_frame_ = -1, spec_stamp_ = 0, spec_hits_ = 0, spec_tries_ = 0;
  std::vector<int> spec_mps_, spec_cnt_, spec_touched_, spec_kfs_, spec_pts_;
  std::vector<long> spec_mark_;
  uint8_t* h_early_ = nullptr;  // C2's match count and matches, copied before D1
  hipEvent_t ev_early_ = nullptr;
  void speculate_local_map(const MapFrameH& L, int n);
  bool commit_local_map(MapFrameH& C);
  void spec_discard();
  template <class Marked, class Mark>
  void expand_local_kfs(std::vector<int>& kfl, Marked marked, Mark mark);
  void collect_local_points(const std::vector<int>& kfl, std::vector<int>& out);
  // compute_distinctive's pairwise descriptor distances of points with more than 32 good
  // observations, by observation ((keyframe << 32) | key, keyframe order)
  struct DistCache {
    std::vector<uint64_t> ids;
    std::vector<uint16_t> d;
  };
  std::unordered_map<int, DistCache> dcache_;
  void run_overlap() {
    if (!overlap_) return;
    std::function<void()> fn = std::move(overlap_);
    overlap_ = nullptr;
    fn();
  }
  static constexpr int kTemp = 1 << 29;
  MPoint& mp(int h) { return h >= kTemp ? temps_[h - kTemp] : pts_[h]; }
  bool track_with_motion_model(MapFrameH& C, const GridFrame& G, float* Tcw, MapFrameH& L,
                               float* Tlast, const float* vel, MapStatsH& st);
  bool track_reference_subst(MapFrameH& C, const GridFrame& G, float* Tcw, const MapFrameH& L,
                             const float* Tlast);
  bool relocalization_subst(MapFrameH& C, const GridFrame& G, float* Tcw, const float* Tlast,
                            const float* vel);
  bool track_local_map(MapFrameH& C, const GridFrame& G, float* Tcw);
  int discard_outliers(MapFrameH& C, int nmatches, int* nmatchesMap);
  void update_last_frame(MapFrameH& L, float* Tlast);
  void update_local_keyframes(MapFrameH& C);
  void update_local_points();
  void search_local_points(MapFrameH& C, const GridFrame& G, const float* Tcw);
  bool need_new_keyframe(const MapFrameH& C);
  void create_new_keyframe(MapFrameH& C, const float* Tcw);
  int new_keyframe(const MapFrameH& C, const float* Tcw);
  int new_point_kf(const float* pos, int kf);
  void add_observation(int h, int kf, int idx);
  void set_bad(int h);
  void compute_distinctive(int h);
  void update_normal_depth(int h);
  void update_connections(int kf);
  void add_connection(int kf, int other, int w);
  void update_best_covisibles(int kf);
  int tracked_map_points(int kf, int minObs);
  void process_new_keyframe(int kf);
  void map_point_culling(int kf);
  void mark_dirty(int h);
  void mark_bad(int h);  // mbBad, the map's point count, the per-frame scan record
  // ---- LocalMapping after ProcessNewKeyFrame / MapPointCulling (mmt_localmap.hip)
  void local_mapping(int kf);
  void search_in_neighbors(int kf);
  // ORBmatcher::Fuse(kfl[i], pts, 3) for every i in order; candidates from the GPU
  void fuse_sequence(const std::vector<int>& kfl, const std::vector<int>& pts);
  void fuse_apply(int kf, int h, int bestIdx, int bestDist);
  void local_bundle_adjustment(int kf);
  void keyframe_culling(int kf);
  void replace(int h, int by);
  void erase_observation(int h, int kf);
  void kf_set_bad(int kf);
  void erase_connection(int kf, int other);
  void set_pose(int kf, const float* Tcw);
  void kf_store_add(int kf);
  // ---- vocabulary path (mmt_bowmap.hip)
  void bow_launch(const uint8_t* d_desc, int n, hipStream_t st);
  void bow_finish(int n, hipStream_t st, BowVecH& v, FeatVecH& fv);
  void frame_bow(MapFrameH& C, const GridFrame& G);
  void kf_bow_launch(int kf);
  void kf_bow_finish(int kf);
  void kfdb_add(int kf);
  void kfdb_erase(int kf);
  std::vector<int> detect_relocalization_candidates(const MapFrameH& C);
  int search_by_bow_kf(int kf, const MapFrameH& C, const GridFrame& G, float nnratio,
                       std::vector<int>& match);
  int gpu_pose_optimization(MapFrameH& C, float* Tcw);
  bool track_reference_kf(MapFrameH& C, const GridFrame& G, float* Tcw, const float* Tlast);
  bool relocalization(MapFrameH& C, const GridFrame& G, float* Tcw);
  int search_by_projection_kf(MapFrameH& C, const GridFrame& G, const float* Tcw, int kf,
                              const std::set<int>& found, float th, int orbDist);
  void create_new_map_points(int kf);
  void bw_grow(size_t need);
  Vocabulary* voc_ = nullptr;
  std::vector<std::vector<int>> invfile_;  // KeyFrameDatabase::mvInvertedFile
  GlibcRandH rand_;
  BowStatsH bstats_;
  uint8_t* d_bw_ = nullptr;  // the vocabulary path's upload / download scratch
  uint8_t* h_bw_ = nullptr;
  size_t bw_cap_ = 0;
  void fuse_launch(const std::vector<int>& kft_kf, const std::vector<FuseQuery>& q, int2* res);
  // GPU stages (synchronous on s_)
  // retry_below (-1: min_matches): the retry at retry_th runs below this many matches
  int gpu_frame_chain(MapFrameH& C, const GridFrame& G, float* Tcw, const MapFrameH& L,
                      const float* Tlast, float th, float retry_th, int min_matches,
                      int retry_below = -1, bool spec = false);
  void pose_desc_fill(uint8_t* h_blk, uint8_t* d_blk, const float* Tcw);
  size_t out_bytes(int n) const;
  MapEdgeArgs edge_args(const GridFrame& G) const;
  void apply_pose_opt(MapFrameH& C, float* Tcw);
  void gpu_flush_pool(hipStream_t st = nullptr);
  template <typename T>
  T* dev(size_t n);
  template <typename T>
  T* pinned(size_t n);
  void grow_local(int m);

  MapCamH cam_;
  int kcap_ = 0;
  // map points in fixed chunks: growing the array never moves the existing points (a vector's
  // reallocation moved all of them, 100k points at a time, inside a keyframe's point creation)
#ifdef MMT_PTS_VECTOR  // A/B build (tools/build_prof_lib.sh)
  std::vector<MPoint> pts_;
#else
  ChunkArray<MPoint> pts_;
#endif
  std::vector<MPoint> temps_;
  // the fields the per-frame local-map scans read, one compact record per real point (pts_ index):
  // UpdateLocalPoints walks ~13k point references and SearchLocalPoints ~4.4k, at random, and a
  // 12-byte record keeps them in cache where the 136-byte MPoint does not
  struct PtHot {
    int trackRef = 0;  // mnTrackReferenceForFrame
    int lastSeen = 0;  // mnLastFrameSeen
    uint8_t bad = 0;
  };
  std::vector<PtHot> hot_;
  std::vector<KFrame> kfs_;
  int state_ = 0;
  long frameNextId_ = 0;
  int kfNextId_ = 0;
  long lastKFFrameId_ = 0;
  int refKF_ = -1;
  std::vector<int> localKFs_, localPts_, recent_, dirty_;
  std::vector<std::pair<float, int>> far_;  // UpdateLastFrame's far keys (scratch)
  std::vector<uint32_t> sort_key_;  // CreateNewKeyFrame's depth sort (scratch)
  std::vector<int> sort_idx_, sort_tmp_;
  float Tlr_[16];
  bool hasTlr_ = false;
  // the keyframe this frame created and its pose before its LocalMapping ran: the reference's
  // mapping thread adjusts the keyframe after Track() has stored mlRelativeFramePoses against it,
  // so frame_done reads this pose (the LocalMapping itself overlaps the flow solve here)
  int snapKF_ = -1;
  float snapTwc_[16];
  int matchesInliers_ = 0;
  bool mbVO_ = false;
  bool pending_ok_ = false;  // track() succeeded, track_finish() pending
  long lastRelocFrameId_ = 0;
  long curId_ = 0;
  int n_good_ = 0;  // non-bad map points
  hipStream_t s_ = nullptr;
  // MMT_MAP_PROFILE=1: host wall time per stage of track(), printed to stderr at destruction
  bool prof_on_ = false;
  double prof_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  long prof_n_ = 0;
  double prof_cnt_[4] = {0, 0, 0, 0};

  // device / pinned buffers
  std::vector<void*> dallocs_, hallocs_;
  // C2's one upload: D1's descriptor (kDescBytes), then the last frame, packed
  // [kps][Xw][desc][active][obs]
  uint8_t* d_last_ = nullptr;
  uint8_t* h_last_ = nullptr;
  CandSet c2_{};
  // the one download of a C2 / C3 chain: [nm][ninl][pad][pose 16 floats] (kOutHdr bytes), then
  // match[kcap] and D1's outlier flags[kcap]; the pointers below point into it
  uint8_t* d_out_ = nullptr;
  uint8_t* h_out_ = nullptr;
  int* d_match_ = nullptr;
  int* d_nm_ = nullptr;
  int* h_match_ = nullptr;
  int* h_nm_ = nullptr;
  // D1
  float* d_edges_ = nullptr;
  float* h_edges_ = nullptr;
  PoseOptDesc* d_pod_ = nullptr;  // the current chain's descriptor (in its upload block)
  PoseOptDesc* h_pod_ = nullptr;
  float* d_pose_ = nullptr;
  uint8_t* d_outl_ = nullptr;
  int* d_ninl_ = nullptr;
  double* d_esc_ = nullptr;
  int* d_fsc_ = nullptr;
  float* h_pose_ = nullptr;
  uint8_t* h_outl_ = nullptr;
  int* h_ninl_ = nullptr;
  // C3: point pool, local selection, candidates
  LocalPointDev* d_pool_ = nullptr;
  uint8_t* d_pool_desc_ = nullptr;
  int pool_cap_ = 0;
  PoolUpdate* d_up_ = nullptr;
  PoolUpdate* h_up_ = nullptr;
  int up_cap_ = 0;
  // C3's one upload: [D1 descriptor][ids m][skip m][taken n] and, for D1's edge list, the keys
  // bound before the search: [positions 3n floats][flags n] (sel_layout)
  uint8_t* d_sel_ = nullptr;
  uint8_t* h_sel_ = nullptr;
  uint8_t* d_inview_ = nullptr;
  uint8_t* h_inview_ = nullptr;
  CandSet c3_{};
  int local_cap_ = 0;
  // ---- LocalMapping
  GridFrame G_{};
  MappingStats mstats_;
  double cull_ratio_ = 0.9;
  hipStream_t lm_s_ = nullptr;  // LocalMapping's stream (beside the ego solve)
  std::vector<uint8_t*> kf_blocks_;  // keyframe store: blocks of kKFBlock records
  size_t kf_rec_bytes_ = 0;
  static constexpr int kKFBlock = 64;
  uint8_t* d_fup_ = nullptr;  // Fuse upload: [FuseKF table][queries]
  uint8_t* h_fup_ = nullptr;
  size_t fup_cap_ = 0;
  int2* d_fres_ = nullptr;
  int2* h_fres_ = nullptr;
  size_t fres_cap_ = 0;
  BARunner ba_;  // the local BA's buffers and launch
  std::vector<int> ba_vidx_;  // keyframe -> BA vertex while a local BA's graph is built
  void grow_dev(uint8_t*& d, uint8_t*& h, size_t& cap, size_t need);
};

// ------------------------------------------------------------------ buffers
template <typename T>
inline T* MapEngine::dev(size_t n) {
  T* p = nullptr;
  MMT_HIP(hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T)));
  dallocs_.push_back(p);
  return p;
}

template <typename T>
inline T* MapEngine::pinned(size_t n) {
  T* p = nullptr;
  MMT_HIP(hipHostMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault));
  hallocs_.push_back(p);
  return p;
}

}  // namespace mmt
