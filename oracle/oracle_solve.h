// oracle/oracle_solve.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
#pragma once
#include <cstdint>
#include <vector>

#include "oracle_common.h"

namespace oracle {

// One flow-refined pose solve (Optimizer::PoseOptimizationFlow2Cam / PoseOptimizationFlow2).
struct FlowProblem {
  int n = 0;
  const float* obs = nullptr;    // n x (u, v): last-frame sample pixel (edge measurement)
  const float* flow = nullptr;   // n x (fu, fv): flow init = prior measurement
  const float* depth = nullptr;  // n: last-frame depth (noisy for the ego solve)
  float Tcw_last[16];            // row-major last-frame camera pose (Twl = inverse)
  float init[16];                // row-major initial estimate of the solved pose
  float rp_thres = 0.04f;        // Huber delta^2 and outlier threshold (0.04 ego / 0.01 object)
  double prior_info = 0.3;       // EdgeFlowPrior information (0.3 ego / 0.5 object)
  int max_iters = 100;           // 100 ego / 200 object
  float fx = 0, fy = 0, cx = 0, cy = 0;
};
struct FlowSolveStats {
  int iterations = 0, inliers = 0, status = 0;
  // test statistics: rejected trials, those on a system without Huber-active edges (where the GPU
  // serves the next trials from its lambda candidate table) and the longest rejection run
  int rejections = 0, clean_rejections = 0, max_reject_run = 0;
};
int flow_pose_solve(const FlowProblem& p, float pose_out[16], FlowSolveStats* st);

// Optimizer::PoseOptimization (Optimizer.cc:3121-3339): pose-only LM over the frame's MapPoint
// observations, mono (uR < 0) and stereo edges, 4 rounds x 10 iterations with re-classification.
struct PoseOptProblem {
  int n = 0;
  const float* Xw = nullptr;      // n x 3 MapPoint world positions
  const float* obs = nullptr;     // n x (u, v, uR): undistorted keypoint, right u (< 0: mono)
  const float* inv_sigma2 = nullptr;  // n: mvInvLevelSigma2[octave]
  float Tcw[16];                  // row-major initial pose (pFrame->mTcw)
  float fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
};
// returns nInitialCorrespondences - nBad (0 and pose untouched below 3 edges); outlier[i] = mvbOutlier
int pose_optimization(const PoseOptProblem& p, float pose_out[16], uint8_t* outlier);

// Optimizer::LocalBundleAdjustment's solve (Optimizer.cc:3394-3665): keyframe poses (VertexSE3Expmap,
// fixed or not) and map points (VertexSBAPointXYZ, marginalised) joined by EdgeSE3ProjectXYZ (uR < 0)
// / EdgeStereoSE3ProjectXYZ edges.  The caller lists the edges point by point, each point's
// observations in keyframe order (the reference's edge creation order, mono and stereo mixed).
struct BAProblem {
  int n_kf = 0, n_pt = 0, n_edge = 0;
  const float* Tcw = nullptr;        // n_kf x 16 row-major
  const uint8_t* fixed = nullptr;    // n_kf
  const float* Xw = nullptr;         // n_pt x 3
  const int* e_pt = nullptr;         // n_edge
  const int* e_kf = nullptr;         // n_edge
  const float* e_obs = nullptr;      // n_edge x (u, v, uR)
  const float* e_inv_sigma2 = nullptr;  // n_edge: mvInvLevelSigma2[octave]
  float fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
};
struct BAResult {
  std::vector<float> Tcw, Xw;   // Converter::toCvMat of every vertex's final estimate
  std::vector<uint8_t> erase;   // the final inlier check failed (vToErase)
  int n_erase = 0;
  int iterations[2] = {0, 0}, trials[2] = {0, 0};  // optimize(5), optimize(10)
};
int local_ba_solve(const BAProblem& p, BAResult& out);

float cv_rng_first_gaussian(uint64_t seed);
float noisy_depth(float z, float g0);

// cv::solvePnPRansac(pre_3d, cur_2d, K, 0, rvec, tvec, false, iters, reproj, conf, inliers,
// SOLVEPNP_AP3P) as called by Tracking::GetInitModelObj (Tracking.cc:4362-4365).
struct PnPResult {
  bool ok = false;
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  double t[3] = {0, 0, 0};
  std::vector<int> inliers;
  int iterations = 0;
  int best_iter = -1;
};
PnPResult pnp_ransac(const float* pts3, const float* pts2, int n, double fx, double fy, double cx,
                     double cy, int max_iters, double reproj, double confidence);
// RANSAC subset indices exactly as RANSACPointSetRegistrator::getSubset draws them.
void ransac_subsets(int count, int model_points, int iters, std::vector<int>& idx);
// EPnP on n >= 4 correspondences (epnp.cpp / PnPsolver.cc:342-1022), pixel inputs.
void epnp_pose(const float* pts3, const float* pts2, const int* sel, int n, double fx, double fy,
               double cx, double cy, double R[9], double t[3], bool f64_points);
void epnp_pose_raw(const float* pts3, const float* pts2, const int* sel, int n, double fx,
                   double fy, double cx, double cy, double R[9], double t[3]);
void rodrigues_r2v(const double R[9], double r[3]);

// D6: glibc rand() (the stream DUtils::Random::RandomInt draws from) and PnPsolver.
struct GlibcRand {
  std::vector<int32_t> r;
  explicit GlibcRand(unsigned seed = 1);
  int next();
  int random_int(int min, int max);
};
struct P4PState {
  int iterations = 0, best_inliers = 0;
  float best_Tcw[16] = {0};
  std::vector<uint8_t> best_mask;
};
struct P4PResult {
  bool found = false, no_more = false;
  int n_inliers = 0;
  float Tcw[16] = {0};
  std::vector<uint8_t> mask;
};
// PnPsolver::SetRansacParameters + iterate(nIterations) on a solver in state *st; randi[4 k + j]
// = RandomInt(0, N - 1 - j) of draw j in iteration k of this call.
P4PResult pnpsolver_iterate(const float* pts3, const float* pts2, const float* sigma2, int N,
                            double fu, double fv, double uc, double vc, double probability,
                            int minInliers, int maxIterations, int minSet, float epsilon,
                            float th2, const int* randi, int nIterations, P4PState* st);
void rodrigues_v2r(const double r[3], double R[9]);

}  // namespace oracle
