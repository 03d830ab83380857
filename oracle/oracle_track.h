// oracle/oracle_track.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
#pragma once
#include <memory>
#include <array>
#include <cstdint>
#include <functional>
#include <vector>

#include "oracle_common.h"
#include "oracle_map.h"
#include "oracle_solve.h"

namespace oracle {

struct P2 {
  float x, y;
};

struct TrackParams {
  int width = 0, height = 0;
  float fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
  uint64_t noise_seed = 0;
  float th_depth = 65.2f;  // ThDepth (kitti03.yaml:32)
  float fps = 10.f;        // Camera.fps (kitti03.yaml:23)
};

// The parts of ORB_SLAM2::Frame this path reads (Frame.h of the reference).
struct OFrame {
  std::vector<float> depth;
  std::vector<Key> keys;
  std::vector<uint8_t> desc;
  std::vector<P2> siftTmp, corres, flowNext;  // mvSiftKeysTmp, mvCorres, mvFlowNext
  std::vector<float> siftDepthTmp;            // mvSiftDepthTmp
  std::vector<P2> siftKeys;                   // mvSiftKeys
  std::vector<float> siftDepth;               // mvSiftDepth
  std::vector<P2> objKeys, objCorres, objFlow;  // mvObjKeys, mvObjCorres, mvObjFlowNext
  std::vector<float> objDepth;                // mvObjDepth
  std::vector<int> semObjLabel, objLabel;     // vSemObjLabel, vObjLabel
  std::vector<std::array<float, 3>> flow3d;   // vFlow_3d
  float Tcw[16] = {0};
  bool hasPose = false;
  std::vector<int> nModLabel, nSemPosition;
  std::vector<std::vector<float>> vObjMod;
  MapFrame m;  // mnId, mvuRight, mvDepth, mvpMapPoints, mvbOutlier, mpReferenceKF
};

struct ObjectResult {
  int label = 0, sem_label = 0, n_points = 0, n_ransac_inliers = 0, n_mm_inliers = -1;
  int n_solve = 0, n_inliers = 0, iterations = 0;
  float init[16], X[16], motion[16];
  float centre_pre[3] = {0, 0, 0};  // ObjCentre3D_pre (Tracking.cc:2032-2049)
  std::vector<int> ids, sub;
};

struct FrameResult {
  bool initialized = false;
  float Tcw[16] = {0};
  int n_keys = 0, n_static = 0, n_obj_samples = 0, ego_iterations = 0, ego_inliers = 0;
  std::vector<ObjectResult> objects;
  MapStats map;  // the ORB-SLAM2 map branch that sets PoseOptimizationFlow2Cam's initial pose
};

void build_frame(const TrackParams& P, const OrbConfig& orb, const uint8_t* bgr,
                 const uint16_t* disp, const float* flow, const int32_t* mask, OFrame& F);

class OTracker {
 public:
  void init(const TrackParams& p, const OrbConfig& orb);
  int track(const uint8_t* bgr, const uint16_t* disp, const float* flow, const int32_t* mask,
            FrameResult& out);
  TrackParams P;
  OrbConfig orbc;
  int state = 0;
  bool bFirstFrame = false, bSecondFrame = false, hasVelocity = false;
  bool reset_pending = false;  // System::Reset requested (LOST with <= 5 keyframes)
  MapTracker map;
  std::unique_ptr<Vocabulary> voc;  // System's vocabulary (null: the substitutes, oracle_map.h)
  float V[16] = {0};
  float g0 = 0;
  OFrame L;  // mLastFrame
  long n_tracked = 0;  // track() calls (test hook below)
  // test hook: every D3 problem (frame = track() call index, object index) before its solve
  std::function<void(const FlowProblem&, long frame, int obj)> d3_hook;
};

}  // namespace oracle
