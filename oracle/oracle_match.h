// oracle/oracle_match.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
//
// CPU restatement of the ORB-SLAM2 frame grid (B3) and projection matching (C1-C3) of the
// reference: Frame::ComputeStereoFromRGBD / AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea /
// isInFrustum (Frame.cc), MapPoint::PredictScale (MapPoint.cc:402-417) and
// ORBmatcher::DescriptorDistance / SearchByProjection (ORBmatcher.cc).
#pragma once
#include <cstdint>
#include <vector>

#include "oracle_common.h"

namespace oracle {

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS, Frame.h:37-38

// The parts of Frame the matcher reads.
struct MatchFrame {
  int n = 0;
  const Key* keys = nullptr;      // mvKeysUn (== mvKeys: zero distortion on this path)
  const uint8_t* desc = nullptr;  // n x 32
  std::vector<float> uR, depth;   // mvuRight, mvDepth
  float minX = 0, maxX = 0, minY = 0, maxY = 0, invW = 0, invH = 0;
  std::vector<std::vector<int>> grid;  // [ix * kGridRows + iy]
  float fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
  std::vector<float> scale;  // mvScaleFactors
  float logScale = 0;        // mfLogScaleFactor
  int nlevels = 0;
};

// B3: ComputeStereoFromRGBD (Frame.cc:1041-1062) + ComputeImageBounds (no distortion,
// Frame.cc:841-846) + AssignFeaturesToGrid (Frame.cc:601-616).
void frame_stereo_grid(MatchFrame& F, const float* depth, int W, int H);
std::vector<int> features_in_area(const MatchFrame& F, float x, float y, float r, int minLevel,
                                  int maxLevel);
int descriptor_distance(const uint8_t* a, const uint8_t* b);

// Last-frame side of SearchByProjection(Frame&, const Frame&, ...): one entry per last-frame key.
struct LastFrameView {
  int n = 0;
  const Key* keys = nullptr;       // mvKeysUn (octave, angle)
  const float* Xw = nullptr;       // n x 3 world position of mvpMapPoints[i]
  const uint8_t* mp_desc = nullptr;  // n x 32 descriptor of mvpMapPoints[i]
  const uint8_t* active = nullptr;   // mvpMapPoints[i] && !mvbOutlier[i]
  // mvpMapPoints[i]->Observations() > 0 (null: every point has observations).  A current key
  // bound to a point without observations (a temporal "visual odometry" point of UpdateLastFrame)
  // stays open: a later point may bind it again (ORBmatcher.cc:2033-2035, 2058).
  const uint8_t* obs = nullptr;
  float Tcw[16];
};

// C2: ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) ORBmatcher.cc:1958-2102.
// match[i2] = last-frame index bound to current key i2, or -1.  Returns nmatches.
int search_by_projection_frame(const MatchFrame& C, const float* Tcw, const LastFrameView& L,
                               float th, bool mono, bool check_orientation, int* match);

// A local map point as SearchLocalPoints sees it.
struct LocalPoint {
  float Xw[3];
  float normal[3];         // mNormalVector
  float min_dist, max_dist;  // mfMinDistance, mfMaxDistance
  const uint8_t* desc;     // mDescriptor
  int skip;                // mnLastFrameSeen == current frame (already matched) or isBad()
};
struct FrustumOut {
  int in_view, level;
  float u, v, uR, view_cos;
};

// Frame::isInFrustum(pMP, viewingCosLimit) Frame.cc:652-708 (+ PredictScale).
bool is_in_frustum(const MatchFrame& F, const float* Tcw, const LocalPoint& p,
                   float viewing_cos_limit, FrustumOut& o);
// C3: Tracking::SearchLocalPoints (Tracking.cc:3416-3466) projection + ORBmatcher::
// SearchByProjection(Frame&, vector<MapPoint*>, th) ORBmatcher.cc:418-502.  `taken[i]` marks
// current keys already bound to a MapPoint (Observations() > 0); match[i] receives the local point
// index for newly bound keys (-1 otherwise).  Returns nmatches; fr (optional) the frustum records.
int search_local_points(const MatchFrame& C, const float* Tcw, const LocalPoint* pts, int m,
                        float th, const uint8_t* taken, int* match, FrustumOut* fr);

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>) as flat arrays: node ids
// ascending; the features of node k are feat[start[k] .. start[k + 1]) in insertion order.
struct FeatVec {
  int n_nodes = 0;
  const uint32_t* node = nullptr;
  const int* start = nullptr;
  const int* feat = nullptr;
};

// C4: ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches, ...) ORBmatcher.cc:532-663
// with ORBmatcher(nnratio, check_orientation).  kf_mp_ok[i]: pKF->mvpMapPoints[i] && !isBad().
// match[iF] = the keyframe key whose MapPoint is matched to frame key iF, or -1.  Returns nmatches.
int search_by_bow(const FeatVec& kfv, const Key* kf_keys, const uint8_t* kf_desc,
                  const uint8_t* kf_mp_ok, const FeatVec& fv, const Key* f_keys,
                  const uint8_t* f_desc, int nF, float nnratio, bool check_orientation,
                  int* match);

}  // namespace oracle
