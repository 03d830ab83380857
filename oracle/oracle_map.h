// oracle/oracle_map.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
//
// CPU restatement of ORB-SLAM2's map tracking as the reference runs it for RGB-D (the ego initial
// pose that PoseOptimizationFlow2Cam starts from):
//   MapPoint / KeyFrame / Map                    src/MapPoint.cc, src/KeyFrame.cc, src/Map.cc
//   Tracking::StereoInitialization (map part)    src/Tracking.cc:2531-2575
//   Tracking::Track, map branch                  src/Tracking.cc:985-1176
//   CheckReplacedInLastFrame / UpdateLastFrame   src/Tracking.cc:2766-2781, 2894-2960
//   TrackWithMotionModel / TrackReferenceKeyFrame src/Tracking.cc:2962-3187, 2836-2892
//   TrackLocalMap / SearchLocalPoints / UpdateLocalMap / UpdateLocalKeyFrames / UpdateLocalPoints
//                                                src/Tracking.cc:3189-3240, 3416-3612
//   NeedNewKeyFrame / CreateNewKeyFrame          src/Tracking.cc:3243-3414
//   LocalMapping::ProcessNewKeyFrame / MapPointCulling  src/LocalMapping.cc:131-208, SearchInNeighbors
//   (+ ORBmatcher::Fuse, MapPoint::Replace)     src/LocalMapping.cc:458-538, ORBmatcher.cc:1200-1350,
//                                                MapPoint.cc:111-215
//   Optimizer::LocalBundleAdjustment             src/Optimizer.cc:3341-3666 (solve: ba_ref.cpp)
//   LocalMapping::KeyFrameCulling + KeyFrame::SetBadFlag  src/LocalMapping.cc:636-700,
//                                                KeyFrame.cc:453-567 (all run synchronously after
//                                                every new keyframe, LocalMapping.cc:61-87)
// Pinned choices:
//  * std::map / std::set keyed by KeyFrame* iterate in keyframe creation order (the reference's
//    order is the heap's);
//  * LocalMapping runs synchronously and is always idle when Tracking asks (AcceptKeyFrames):
//    ProcessNewKeyFrame (without the BoW conversion), MapPointCulling, SearchInNeighbors,
//    LocalBundleAdjustment (no abort: mbAbortBA stays false) and KeyFrameCulling run to completion
//    for every new keyframe once the frame that inserted it has finished Track() (its flow solve
//    and the mlRelativeFramePoses entry against the keyframe's pose as Track left it,
//    Tracking.cc:2481-2489), before the next frame: the mapping thread only receives the keyframe
//    in CreateNewKeyFrame (InsertKeyFrame, Tracking.cc:3408), so the local BA's correction of the
//    keyframe reaches the last frame through Tlr in UpdateLastFrame, as in the reference;
//    CreateNewMapPoints needs SearchForTriangulation, i.e. the BoW vocabulary (missing), and is
//    skipped;
//  * TrackReferenceKeyFrame's SearchByBoW needs the missing vocabulary: it is replaced by
//    SearchByProjection against the last frame at the last frame's pose (th 15, orientation
//    check), then PoseOptimization and the reference's own acceptance tests;
//  * Relocalization (candidates from the BoW database, hypotheses from SearchByBoW + PnPsolver)
//    likewise: the candidates are the reference keyframe and its best 10 covisibles, the
//    hypothesis the motion model's prediction from the last (flow-tracked) frame, each
//    candidate's map points searched as TrackWithMotionModel searches the last frame's, then
//    the reference's acceptance (PoseOptimization, >= 10 inliers, outliers dropped, >= 50);
//  * map points whose unprojection is not finite (depth +inf where the disparity is 0) project to
//    no pixel (the reference would index the grid with an undefined float -> int conversion).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <vector>

#include "oracle_bow.h"
#include "oracle_common.h"
#include "oracle_match.h"
#include "oracle_solve.h"

namespace oracle {

struct MapCam {
  int W = 0, H = 0;
  float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, bf = 0;
  float thDepth = 0;  // mThDepth = mbf * ThDepth / fx (Tracking.cc:225)
  int maxFrames = 0;  // mMaxFrames = fps (Tracking.cc:176)
  int nlevels = 0;
  float logScale = 0;
  std::vector<float> scale, invSigma2;
};

struct OMapPoint {
  float pos[3] = {0, 0, 0};
  float normal[3] = {0, 0, 0};
  uint8_t desc[32] = {0};
  std::map<int, int> obs;  // mObservations: keyframe id -> key index
  int nObs = 0;
  int refKF = -1;
  int firstKFid = -1;
  long firstFrame = 0;
  int visible = 1, found = 1;
  bool bad = false;
  float minDist = 0, maxDist = 0;
  long trackRefForFrame = 0, lastFrameSeen = 0;
  bool trackInView = false;
  int replaced = -1;                 // mpReplaced
  long fuseCandForKF = 0, baLocalForKF = 0;  // mnFuseCandidateForKF, mnBALocalForKF
};

struct OKeyFrame {
  int id = 0;
  long frameId = 0;
  float Tcw[16], Twc[16], Ow[3];
  std::vector<Key> keys;
  std::vector<float> uR, depth;
  std::vector<uint8_t> desc;
  std::vector<int> mps;  // mvpMapPoints (point handle or -1)
  std::map<int, int> conn;  // mConnectedKeyFrameWeights
  std::vector<int> ordered, orderedW;
  bool firstConnection = true;
  int parent = -1;
  std::set<int> children;
  long trackRefForFrame = 0;
  bool bad = false;
  long fuseTargetForKF = 0, baLocalForKF = 0, baFixedForKF = 0;
  std::vector<std::vector<int>> grid;  // mGrid (the frame's, copied), [ix * kGridRows + iy]
  // BoW (with a vocabulary): mBowVec, mFeatVec; KeyFrameDatabase query fields (KeyFrame.h:146-149;
  // mRelocScore is uninitialised in the reference: pinned 0)
  BowVec bow;
  FeatVecO fv;
  bool hasBow = false;
  long relocQuery = 0;
  int relocWords = 0;
  float relocScore = 0;
};

// Map-path fields of one Frame (Frame.h): its keys and descriptors live in OFrame.
struct MapFrame {
  long id = 0;
  std::vector<float> uR, depth;  // mvuRight, mvDepth (ComputeStereoFromRGBD)
  std::vector<int> mps;          // mvpMapPoints
  std::vector<uint8_t> outlier;  // mvbOutlier
  int refKF = -1;                // mpReferenceKF
  BowVec bow;                    // mBowVec / mFeatVec (Frame::ComputeBoW, with a vocabulary)
  FeatVecO fv;
  bool hasBow = false;
};

// What the parity tests compare besides the poses.
struct MapStats {
  int state = 0;            // 0 not initialised, 1 OK, 2 LOST
  int matches_mm = -1;      // TrackWithMotionModel's nmatches before PoseOptimization (-1: not run)
  int inliers_local = -1;   // mnMatchesInliers after TrackLocalMap (-1: not run)
  int n_keyframes = 0, n_mappoints = 0;
  int new_keyframe = 0;
  float Tcw_map[16];        // pose after the map branch (the initial estimate of PoseOptimizationFlow2Cam)
};

// ------------------------------------------------------------------ pose helpers
inline void m4_mul(const float* A, const float* B, float* C) {
  float R[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = 0;
      for (int k = 0; k < 4; k++) s += (double)A[4 * r + k] * (double)B[4 * k + c];
      R[4 * r + c] = (float)s;
    }
  memcpy(C, R, sizeof(R));
}

// Frame::UpdatePoseMatrices / KeyFrame::SetPose: Ow = -Rcw^T tcw
inline void cam_centre(const float* T, float* Ow) {
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    Ow[r] = -(float)s;
  }
}

// Frame::UnprojectStereo (Frame.cc:1064-1079) / KeyFrame::UnprojectStereo: Rwc * x3Dc + Ow
inline void unproject(const MapCam& c, const float* T, float u, float v, float z, float* out) {
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

inline float norm3(const float* v) {
  double s = 0;
  for (int k = 0; k < 3; k++) s += (double)v[k] * (double)v[k];
  return (float)std::sqrt(s);
}


// KeyFrame::GetFeaturesInArea and ORBmatcher::Fuse's per-point search (mapping_ref.cpp)
std::vector<int> kf_features_in_area(const OKeyFrame& K, const MapCam& cam, float x, float y,
                                     float r);
int fuse_candidate(const OKeyFrame& K, const MapCam& cam, const OMapPoint& p, float th,
                   int* bestIdx);

class MapTracker {
 public:
  void init(const MapCam& cam);
  // Tracking::Reset (map part): clears the map, keyframe and frame ids restart
  void reset();
  long next_frame_id() { return frameNextId_++; }
  // mCurrentFrame's ComputeStereoFromRGBD + grid (Frame.cc:1041-1062, 601-616)
  void prepare_frame(const std::vector<Key>& keys, const float* depth, MapFrame& F);
  // StereoInitialization, map part (Tracking.cc:2531-2575): C has pose identity
  void initialize(const std::vector<Key>& keys, const std::vector<uint8_t>& desc, MapFrame& C,
                  const float* Tcw);
  // Track()'s map branch (Tracking.cc:985-1176) for current frame C against last frame L.
  // Tcw (in/out): the current pose; Tlast (in/out): mLastFrame.mTcw (UpdateLastFrame resets it).
  // vel / has_vel: mVelocity (read; line 1122's update written).  bSecondFrame: the reference's
  // flag (TrackReferenceKeyFrame sets it, TrackWithMotionModel clears it).  Returns 1 when the
  // reference resets the system here (LOST with <= 5 keyframes: Track returns at line 1171).
  int track(const std::vector<Key>& keys, const std::vector<uint8_t>& desc, MapFrame& C,
            float* Tcw, const std::vector<Key>& lkeys, const std::vector<uint8_t>& ldesc,
            MapFrame& L, float* Tlast, float* vel, bool& has_vel, bool& bSecondFrame,
            MapStats& st);
  // end of Track (Tracking.cc:2481-2489): mlRelativeFramePoses.push_back(Tcw * Tref^-1)
  void frame_done(const MapFrame& C, const float* Tcw);
  int state() const { return state_; }
  int n_keyframes() const;
  int n_mappoints() const;

  // ---- everything below is the reference's state (public for the product parity probes)
  MapCam cam;
  std::vector<OMapPoint> pts;    // map points (handles 0..)
  std::vector<OMapPoint> temps;  // temporal VO points (handles kTemp + i)
  std::vector<OKeyFrame> kfs;
  static constexpr int kTemp = 1 << 29;
  // test hook: called with each LocalBundleAdjustment problem and its result (probe fixtures)
  std::function<void(const BAProblem&, const BAResult&)> ba_hook;
  struct MappingStats {
    long n_ba = 0, n_fused = 0, n_culled = 0, n_ba_erased = 0, n_reparent = 0;
    long ba_trials = 0, ba_edges = 0, ba_kfs = 0, ba_pts = 0, ba_max_opt_kfs = 0;
  } mstats;
  OMapPoint& mp(int h) { return h >= kTemp ? temps[h - kTemp] : pts[h]; }
  double cullRatio = 0.9;  // KeyFrameCulling's redundancy ratio (test knob; LocalMapping.cc:697)
  // the vocabulary System is given (System.cc:67): with one, TrackReferenceKeyFrame,
  // Relocalization and CreateNewMapPoints run as the reference's (bowmap_ref.cpp); without, the
  // substitutes of the header comment
  void set_vocabulary(const Vocabulary* v);
  const Vocabulary* voc() const { return voc_; }
  struct BowStats {
    long n_bow_frames = 0, n_trk = 0, n_trk_ok = 0, n_reloc = 0, n_reloc_ok = 0,
         n_reloc_cands = 0, n_pnp_found = 0, n_sbp_rounds = 0, n_triangulated = 0,
         n_sft_matches = 0, n_kfdb = 0;
  } bstats;

 private:
  bool track_with_motion_model(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                               MapFrame& C, float* Tcw, const std::vector<Key>& lkeys,
                               const std::vector<uint8_t>& ldesc, MapFrame& L, float* Tlast,
                               const float* vel, MapStats& st);
  bool track_reference_subst(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                             MapFrame& C, float* Tcw, const std::vector<Key>& lkeys,
                             const MapFrame& L, const float* Tlast);
  bool relocalization_subst(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                            MapFrame& C, float* Tcw, const float* Tlast, const float* vel);
  bool track_local_map(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                       MapFrame& C, float* Tcw);
  int search_frame(const std::vector<Key>& keys, const std::vector<uint8_t>& desc, MapFrame& C,
                   const float* Tcw, const std::vector<Key>& lkeys, const MapFrame& L,
                   const float* Tlast, float th);
  int pose_optimization(const std::vector<Key>& keys, MapFrame& C, float* Tcw);
  void update_local_keyframes(MapFrame& C);
  void update_local_points(const MapFrame& C);
  void search_local_points(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                           MapFrame& C, const float* Tcw);
  bool need_new_keyframe(const MapFrame& C);
  void create_new_keyframe(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                           MapFrame& C, const float* Tcw);
  void insert_keyframe(int kf);  // LocalMapping::InsertKeyFrame: processed in frame_done
  void process_new_keyframe(int kf);
  void map_point_culling(int kf);
  // the rest of LocalMapping::Run's iteration (LocalMapping.cc:68-87)
  void local_mapping(int kf);
  void search_in_neighbors(int kf);
  int fuse(int kf, const std::vector<int>& pts, float th);
  void local_bundle_adjustment(int kf);
  void keyframe_culling(int kf);
  void replace(int h, int by);
  void erase_observation(int h, int kf);
  void kf_set_bad(int kf);
  void erase_connection(int kf, int other);
  void set_pose(int kf, const float* Tcw);
  std::vector<int> best_covisibles(int kf, int n) const;
  void update_last_frame(const std::vector<Key>& lkeys, const std::vector<uint8_t>& ldesc,
                         MapFrame& L, float* Tlast);
  int new_keyframe(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                   const MapFrame& C, const float* Tcw);
  int new_point_kf(const float* pos, int kf);
  void add_observation(int h, int kf, int idx);
  void set_bad(int h);
  void compute_distinctive(int h);
  void update_normal_depth(int h);
  void update_connections(int kf);
  void add_connection(int kf, int other, int w);
  void update_best_covisibles(int kf);
  int tracked_map_points(int kf, int minObs);
  void build_grid(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                  const MapFrame& C, MatchFrame& G);
  // ---- vocabulary path (bowmap_ref.cpp)
  void compute_bow(const std::vector<uint8_t>& desc, MapFrame& C);
  void kf_compute_bow(int kf);
  void kfdb_add(int kf);
  void kfdb_erase(int kf);
  std::vector<int> detect_relocalization_candidates(const MapFrame& C);
  bool track_reference_kf(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                          MapFrame& C, float* Tcw, const float* Tlast);
  bool relocalization(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                      MapFrame& C, float* Tcw);
  int search_by_projection_kf(const std::vector<Key>& keys, const std::vector<uint8_t>& desc,
                              MapFrame& C, const float* Tcw, int kf, const std::set<int>& found,
                              float th, int orbDist);
  void create_new_map_points(int kf);
  int search_for_triangulation(int kf1, int kf2, const float* F12,
                               std::vector<std::pair<int, int>>& pairs);
  const Vocabulary* voc_ = nullptr;
  std::vector<std::vector<int>> invfile_;  // KeyFrameDatabase::mvInvertedFile
  GlibcRand rand_{1};                      // the process's rand() (PnPsolver's draws)

  int state_ = 0;
  long frameNextId_ = 0;
  int kfNextId_ = 0;
  long lastKFFrameId_ = 0;  // mnLastKeyFrameId
  int lastKF_ = -1;
  int pendingKF_ = -1;      // inserted keyframe whose LocalMapping runs in frame_done
  int refKF_ = -1;          // mpReferenceKF
  std::vector<int> localKFs_, localPts_;
  std::vector<int> temporal_;  // mlpTemporalPoints
  std::vector<int> recent_;    // LocalMapping::mlpRecentAddedMapPoints
  float Tlr_[16];
  bool hasTlr_ = false;
  int matchesInliers_ = 0;     // mnMatchesInliers
  bool mbVO_ = false;
  long lastRelocFrameId_ = 0;
  long curId_ = 0;
  const float* depth_ = nullptr;
};

}  // namespace oracle
