// oracle/solve_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// CPU restatement of the flow-refined pose solves Optimizer::PoseOptimizationFlow2Cam
// (reference src/Optimizer.cc:396-601) and Optimizer::PoseOptimizationFlow2 (:2170-2377) as
// executed by the vendored, modified g2o:
//   SparseOptimizer::optimize         Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:354-400
//   OptimizationAlgorithmLevenberg    core/optimization_algorithm_levenberg.cpp:60-185
//   BlockSolver_6_3 (Schur)           core/block_solver.hpp:354-489, 502-604
//   LinearSolverDense (LDLT)          solvers/linear_solver_dense.h:65-113
//   EdgeSE3ProjectFlow2 / EdgeFlowPrior / VertexSBAFlow / SE3Quat   types/*
// including the 2-D "landmark" in a 3x3 block quirk, restated with the
// closed forms of its block algebra:
//   D_i   = [[h+l, h, 0], [0, l, 0], [0, 0, l]]       (2x2 column-major map onto a 3x3 block,
//                                                      setLambda on all 3 diagonal entries)
//   Dinv  = [[1/(h+l), -h/((h+l)l), 0], [0, 1/l, 0], [0, 0, 1/l]]
//   Hs    = lower(Hpp + l I - sum_i B_i Dinv2_i B_i^T)   (LDLT reads the lower triangle)
//   x_i   = (c0/(h+l) - h c1/((h+l)l) + [i>0] c0/l,  c1/l)   (stride-2 axpy spill)
// Double precision throughout, like g2o/Eigen.  Also: the cv::RNG gaussian that
// Frame::ObtainFlowDepthCamera draws from a freshly seeded RNG (Frame.cc:1241-1251).

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle_se3.h"
#include "oracle_solve.h"

namespace oracle {

// ------------------------------------------------------------------ cv::RNG (Appendix A.8)
static inline uint64_t rng_next(uint64_t x) {
  return (uint64_t)(unsigned)x * 4164903690ULL + (x >> 32);
}

float cv_rng_first_gaussian(uint64_t seed) {
  // randn_0_1_32f ziggurat tables (OpenCV core/src/rand.cpp)
  static unsigned kn[128];
  static float wn[128], fn[128];
  static bool init = false;
  if (!init) {
    const double m1 = 2147483648.0;
    double dn = 3.442619855899, tn = dn, vn = 9.91256303526217e-3;
    double q = vn / std::exp(-.5 * dn * dn);
    kn[0] = (unsigned)((dn / q) * m1);
    kn[1] = 0;
    wn[0] = (float)(q / m1);
    wn[127] = (float)(dn / m1);
    fn[0] = 1.f;
    fn[127] = (float)std::exp(-.5 * dn * dn);
    for (int i = 126; i >= 1; i--) {
      dn = std::sqrt(-2. * std::log(vn / dn + std::exp(-.5 * dn * dn)));
      kn[i + 1] = (unsigned)((dn / tn) * m1);
      tn = dn;
      fn[i] = (float)std::exp(-.5 * dn * dn);
      wn[i] = (float)(dn / m1);
    }
    init = true;
  }
  const float r = 3.442620f;
  const float rng_flt = 2.3283064365386962890625e-10f;
  uint64_t temp = seed ? seed : 0xffffffffULL;
  float x, y;
  for (;;) {
    int hz = (int)temp;
    temp = rng_next(temp);
    int iz = hz & 127;
    x = hz * wn[iz];
    if ((unsigned)std::abs(hz) < kn[iz]) break;
    if (iz == 0) {
      do {
        x = (unsigned)temp * rng_flt;
        temp = rng_next(temp);
        y = (unsigned)temp * rng_flt;
        temp = rng_next(temp);
        x = (float)(-std::log(x + FLT_MIN) * 0.2904764);
        y = (float)-std::log(y + FLT_MIN);
      } while (y + y < x * x);
      x = hz > 0 ? r + x : -r - x;
      break;
    }
    y = (unsigned)temp * rng_flt;
    temp = rng_next(temp);
    if (fn[iz] + y * (fn[iz - 1] - fn[iz]) < std::exp(-.5 * x * x)) break;
  }
  return x;
}

// Frame::ObtainFlowDepthCamera(i, addnoise=1): z + RNG(seed).gaussian(z*z/(725*0.5)*0.15)
float noisy_depth(float z, float g0) {
  const double sigma = (double)(z * z) / (725 * 0.5) * 0.15;
  return (float)((double)z + (double)g0 * sigma);
}

// ------------------------------------------------------------------ 6x6 LDLT (Eigen LDLT<MatrixXd>)
// Reads the lower triangle; diagonal pivoting as Eigen's ldlt_inplace<Lower>.  Returns false when
// the factorisation is not positive (LDLT::isPositive()).
static bool ldlt_solve6(const double Hin[6][6], const double b[6], double x[6]) {
  double A[6][6];
  for (int r = 0; r < 6; r++)
    for (int c = 0; c < 6; c++) A[r][c] = (c <= r) ? Hin[r][c] : Hin[c][r];
  int perm[6] = {0, 1, 2, 3, 4, 5};
  bool positive = true;
  double D[6];
  double L[6][6] = {{0}};
  // symmetric pivoting: at step k choose the largest remaining |diag|
  for (int k = 0; k < 6; k++) {
    int p = k;
    double best = std::fabs(A[k][k]);
    for (int i = k + 1; i < 6; i++)
      if (std::fabs(A[i][i]) > best) {
        best = std::fabs(A[i][i]);
        p = i;
      }
    if (p != k) {
      for (int c = 0; c < 6; c++) std::swap(A[k][c], A[p][c]);
      for (int r = 0; r < 6; r++) std::swap(A[r][k], A[r][p]);
      for (int c = 0; c < k; c++) std::swap(L[k][c], L[p][c]);
      std::swap(perm[k], perm[p]);
    }
    double d = A[k][k];
    for (int c = 0; c < k; c++) d -= L[k][c] * L[k][c] * D[c];
    D[k] = d;
    if (d < 0) positive = false;
    for (int i = k + 1; i < 6; i++) {
      double s = A[i][k];
      for (int c = 0; c < k; c++) s -= L[i][c] * L[k][c] * D[c];
      L[i][k] = (d != 0) ? s / d : 0.0;
    }
    L[k][k] = 1.0;
  }
  if (!positive) return false;
  double y[6];
  for (int i = 0; i < 6; i++) y[i] = b[perm[i]];
  for (int i = 0; i < 6; i++)
    for (int c = 0; c < i; c++) y[i] -= L[i][c] * y[c];
  for (int i = 0; i < 6; i++) y[i] = (D[i] != 0) ? y[i] / D[i] : 0.0;
  for (int i = 5; i >= 0; i--)
    for (int r = i + 1; r < 6; r++) y[i] -= L[r][i] * y[r];
  for (int i = 0; i < 6; i++) x[perm[i]] = y[i];
  return true;
}

// ------------------------------------------------------------------ the LM
struct EdgeState {
  double Xw[3];  // Twl * back-projected observation (constant per edge)
  double obs[2], prior[2];
};

static inline void huber(double e, double dsqr, double delta, double& rho0, double& rho1) {
  if (e <= dsqr) {
    rho0 = e;
    rho1 = 1.;
  } else {
    const double s = std::sqrt(e);
    rho0 = 2 * s * delta - dsqr;
    rho1 = delta / s;
  }
}

int flow_pose_solve(const FlowProblem& P, float pose_out[16], FlowSolveStats* st) {
  const int N = P.n;
  const double fx = P.fx, fy = P.fy, cx = P.cx, cy = P.cy;
  const double kInfo = 0.1;  // info_flow (Optimizer.cc:466 / 2241)
  const double pinfo = P.prior_info;
  const float deltaF = std::sqrt(P.rp_thres);  // const float deltaMono = sqrt(rp_thres)
  const double delta = (double)deltaF, dsqr = delta * delta;
  if (N < 3) {
    if (st) {
      st->iterations = 0;
      st->inliers = 0;
      st->status = 1;
    }
    return 1;  // caller keeps its pose (Flow2Cam) / identity (Flow2)
  }
  // Twl = inverse(last Tcw) built as in Optimizer.cc:473-479 (float Mat ops, then double)
  const float* T = P.Tcw_last;
  float Rwl[3][3], twl[3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Rwl[r][c] = T[4 * c + r];
  for (int r = 0; r < 3; r++) {  // -R^T * t via cv::gemm (double accumulation for CV_32F)
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)Rwl[r][k] * (double)T[4 * k + 3];
    twl[r] = (float)(-s);
  }
  std::vector<EdgeState> E(N);
  for (int i = 0; i < N; i++) {
    const double u = P.obs[2 * i], v = P.obs[2 * i + 1], depth = P.depth[i];
    const double Xc[3] = {(u - cx) * depth / fx, (v - cy) * depth / fy, depth};
    for (int r = 0; r < 3; r++)
      E[i].Xw[r] = (double)Rwl[r][0] * Xc[0] + (double)Rwl[r][1] * Xc[1] +
                   (double)Rwl[r][2] * Xc[2] + (double)twl[r];
    E[i].obs[0] = u;
    E[i].obs[1] = v;
    E[i].prior[0] = P.flow[2 * i];
    E[i].prior[1] = P.flow[2 * i + 1];
  }
  SE3 pose = se3_from_float(P.init);
  std::vector<double> f(2 * N), fb(2 * N);
  for (int i = 0; i < 2 * N; i++) f[i] = E[i / 2].prior[i % 2];  // vFlo->setEstimate(FloD.head(2))

  // error state (g2o keeps the errors of the LAST evaluated state, accepted or not)
  std::vector<double> err(2 * N), perr(2 * N);
  auto compute_errors = [&](const SE3& ps, const std::vector<double>& fl) {
    for (int i = 0; i < N; i++) {
      double pc[3];
      se3_map(ps, E[i].Xw, pc);
      const double pu = pc[0] / pc[2] * fx + cx, pv = pc[1] / pc[2] * fy + cy;
      err[2 * i] = (E[i].obs[0] + fl[2 * i]) - pu;
      err[2 * i + 1] = (E[i].obs[1] + fl[2 * i + 1]) - pv;
      perr[2 * i] = fl[2 * i] - E[i].prior[0];
      perr[2 * i + 1] = fl[2 * i + 1] - E[i].prior[1];
    }
  };
  auto robust_chi2 = [&]() {
    double chi = 0;
    for (int i = 0; i < N; i++) {
      const double e2 = kInfo * (err[2 * i] * err[2 * i] + err[2 * i + 1] * err[2 * i + 1]);
      double r0, r1;
      huber(e2, dsqr, delta, r0, r1);
      chi += r0;
      chi += pinfo * (perr[2 * i] * perr[2 * i] + perr[2 * i + 1] * perr[2 * i + 1]);
    }
    return chi;
  };

  double lambda = 0, ni = 2;
  int nBad = 0;
  double xbuf[6] = {0, 0, 0, 0, 0, 0};  // g2o's persistent _x (stale on a failed solve)
  std::vector<double> xl(2 * N, 0.0);
  std::vector<double> Bm(12 * N), h(N), bl(2 * N);
  double chi2_check = 0;
  int it_done = 0;
  for (int iter = 0; iter < P.max_iters; iter++) {
    // ---- OptimizationAlgorithmLevenberg::solve
    compute_errors(pose, f);
    double currentChi = robust_chi2();
    const double iniChi = currentChi;
    // buildSystem at the current state
    double Hpp[6][6] = {{0}}, bp[6] = {0};
    bool clean = true;  // no Huber-active edge at this linearisation (test statistic)
    for (int i = 0; i < N; i++) {
      double pc[3];
      se3_map(pose, E[i].Xw, pc);
      const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
      const double J[2][6] = {
          {x * y / z2 * fx, -(1 + (x * x / z2)) * fx, y / z * fx, -1. / z * fx, 0, x / z2 * fx},
          {(1 + y * y / z2) * fy, -x * y / z2 * fy, -x / z * fy, 0, -1. / z * fy, y / z2 * fy}};
      const double e2 = kInfo * (err[2 * i] * err[2 * i] + err[2 * i + 1] * err[2 * i + 1]);
      double r0, r1;
      huber(e2, dsqr, delta, r0, r1);
      const double w = kInfo * r1;
      if (e2 > dsqr) clean = false;
      const double om[2] = {-w * err[2 * i], -w * err[2 * i + 1]};  // rho' * (-Omega e)
      for (int a = 0; a < 6; a++) {
        for (int b = 0; b < 6; b++) Hpp[a][b] += J[0][a] * w * J[0][b] + J[1][a] * w * J[1][b];
        bp[a] += J[0][a] * om[0] + J[1][a] * om[1];
        Bm[12 * i + 2 * a] = w * J[0][a];  // B_i (6x2) = J^T * (rho' Omega) * I
        Bm[12 * i + 2 * a + 1] = w * J[1][a];
      }
      h[i] = w + pinfo;
      bl[2 * i] = om[0] - pinfo * perr[2 * i];
      bl[2 * i + 1] = om[1] - pinfo * perr[2 * i + 1];
    }
    if (iter == 0) {  // computeLambdaInit: tau * max |hessian diagonal| over all vertices
      double maxd = 0;
      for (int a = 0; a < 6; a++) maxd = std::max(maxd, std::fabs(Hpp[a][a]));
      for (int i = 0; i < N; i++) maxd = std::max(maxd, std::fabs(h[i]));
      lambda = 1e-5 * maxd;
      ni = 2;
      nBad = 0;
    }
    double rho = 0;
    int qmax = 0, run = 0;
    double lastTrialChi = 0;
    do {
      const SE3 pose_b = pose;
      fb = f;
      // ---- BlockSolver::solve with the lambda-augmented diagonals
      double Hs[6][6], bs[6];
      for (int a = 0; a < 6; a++) {
        for (int b = 0; b < 6; b++) Hs[a][b] = Hpp[a][b] + (a == b ? lambda : 0.0);
        bs[a] = bp[a];
      }
      for (int i = 0; i < N; i++) {
        const double hi = h[i];
        const double d00 = 1.0 / (hi + lambda), d01 = -hi / ((hi + lambda) * lambda),
                     d11 = 1.0 / lambda;
        const double* B = &Bm[12 * i];
        const double db0 = d00 * bl[2 * i] + d01 * bl[2 * i + 1], db1 = d11 * bl[2 * i + 1];
        for (int a = 0; a < 6; a++) {
          const double BD0 = B[2 * a] * d00, BD1 = B[2 * a] * d01 + B[2 * a + 1] * d11;
          for (int b = 0; b < 6; b++) Hs[a][b] -= BD0 * B[2 * b] + BD1 * B[2 * b + 1];
          bs[a] -= B[2 * a] * db0 + B[2 * a + 1] * db1;
        }
      }
      double xp[6];
      const bool ok2 = ldlt_solve6(Hs, bs, xp);
      if (ok2) {
        memcpy(xbuf, xp, sizeof(xp));
        for (int i = 0; i < N; i++) {
          const double* B = &Bm[12 * i];
          double c0 = bl[2 * i], c1 = bl[2 * i + 1];
          for (int a = 0; a < 6; a++) {
            c0 -= B[2 * a] * xp[a];
            c1 -= B[2 * a + 1] * xp[a];
          }
          const double hi = h[i];
          double x0 = c0 / (hi + lambda) - hi * c1 / ((hi + lambda) * lambda);
          if (i > 0) x0 += c0 / lambda;  // landmark i-1's third Dinv row lands here
          xl[2 * i] = x0;
          xl[2 * i + 1] = c1 / lambda;
        }
      }
      // SparseOptimizer::update(x) -- applied even when the solve failed (stale _x)
      pose = se3_mul(se3_exp(xbuf), pose);
      for (int i = 0; i < 2 * N; i++) f[i] += xl[i];
      compute_errors(pose, f);
      double tempChi = robust_chi2();
      lastTrialChi = tempChi;
      if (!ok2) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      double scale = 0;
      for (int a = 0; a < 6; a++) scale += xbuf[a] * (lambda * xbuf[a] + bp[a]);
      for (int i = 0; i < 2 * N; i++) scale += xl[i] * (lambda * xl[i] + bl[i]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi)) {
        double alpha = 1. - std::pow((2 * rho - 1), 3);
        alpha = std::min(alpha, 2. / 3.);
        const double sf = std::max(1. / 3., alpha);
        lambda *= sf;
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        pose = pose_b;
        f = fb;
        if (st) {
          st->rejections++;
          if (clean) st->clean_rejections++;  // the next trial's solve differs only in lambda
          st->max_reject_run = std::max(st->max_reject_run, ++run);
        }
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    bool ok = true;
    if (qmax == 10 || rho == 0) ok = false;  // Terminate
    if (ok) {
      if ((iniChi - currentChi) * 1e3 < iniChi)
        nBad++;
      else
        nBad = 0;
      if (nBad >= 3) ok = false;
    }
    // sparse_optimizer.cpp:393-396 (modified g2o): stop when the robust chi2 increased
    if (chi2_check < lastTrialChi && iter > 0) ok = false;
    chi2_check = lastTrialChi;
    it_done = iter + 1;
    if (!ok) break;
  }
  se3_to_float(pose, pose_out);
  // outlier count from the edges' last computed errors (Optimizer.cc:536-566)
  int nBadEdges = 0;
  for (int i = 0; i < N; i++) {
    const float chi2 = (float)(kInfo * (err[2 * i] * err[2 * i] + err[2 * i + 1] * err[2 * i + 1]));
    if (chi2 > P.rp_thres) nBadEdges++;
  }
  if (st) {
    st->iterations = it_done;
    st->inliers = N - nBadEdges;
    st->status = 0;
  }
  return 0;
}

// ------------------------------------------------------------------ D1: PoseOptimization
// Optimizer::PoseOptimization (Optimizer.cc:3121-3339) with the g2o machinery it runs:
//   EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.cpp:266-364;
//   the stereo cam_project takes invz as a float, .cpp:296-303), RobustKernelHuber, the
//   rho'-weighted quadratic form (base_unary_edge.hpp:56-63), OptimizationAlgorithmLevenberg::solve
//   and the modified SparseOptimizer::optimize (chi2-increase stop) as in flow_pose_solve above.
// Every round restarts from pFrame->mTcw (Optimizer.cc:3263), optimises the level-0 edges for 10
// iterations, then re-classifies every edge by its (non-robust) chi2 (3266-3322); the robust kernel
// is dropped after round 2's classification; fewer than 10 edges stop after one round (3324).
namespace {
struct PoEdge {
  double X[3], obs[3], s;  // world point, measurement, information scale
  bool stereo, outlier, robust;
  double e[3];             // last computed error
};

void po_error(const PoEdge& E, const SE3& T, double fx, double fy, double cx, double cy, double bf,
              double e[3]) {
  double pc[3];
  se3_map(T, E.X, pc);
  if (!E.stereo) {  // obs - cam_project(project2d(Xc))
    const double px = pc[0] / pc[2], py = pc[1] / pc[2];
    e[0] = E.obs[0] - (px * fx + cx);
    e[1] = E.obs[1] - (py * fy + cy);
    e[2] = 0;
  } else {
    const float invz = 1.0 / pc[2];  // const float invz = 1.0f/trans_xyz[2]
    const double u = pc[0] * invz * fx + cx, v = pc[1] * invz * fy + cy;
    e[0] = E.obs[0] - u;
    e[1] = E.obs[1] - v;
    e[2] = E.obs[2] - (u - bf * invz);
  }
}

double po_chi2(const PoEdge& E, const double e[3]) {
  return E.stereo ? E.s * (e[0] * e[0] + e[1] * e[1] + e[2] * e[2]) : E.s * (e[0] * e[0] + e[1] * e[1]);
}
}  // namespace

int pose_optimization(const PoseOptProblem& P, float pose_out[16], uint8_t* outlier) {
  const int N = P.n;
  const double fx = P.fx, fy = P.fy, cx = P.cx, cy = P.cy, bf = P.bf;
  const float deltaMono = std::sqrt(5.991), deltaStereo = std::sqrt(7.815);
  const double dM = deltaMono, dS = deltaStereo;
  std::vector<PoEdge> E(N);
  for (int i = 0; i < N; i++) {
    for (int k = 0; k < 3; k++) E[i].X[k] = P.Xw[3 * i + k];
    E[i].obs[0] = P.obs[3 * i];
    E[i].obs[1] = P.obs[3 * i + 1];
    E[i].obs[2] = P.obs[3 * i + 2];
    E[i].stereo = !(P.obs[3 * i + 2] < 0);
    E[i].s = P.inv_sigma2[i];
    E[i].outlier = false;
    E[i].robust = true;
    E[i].e[0] = E[i].e[1] = E[i].e[2] = 0;
  }
  if (N < 3) {
    for (int i = 0; i < N; i++) outlier[i] = 0;
    memcpy(pose_out, P.Tcw, 64);
    return 0;
  }
  const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
  auto robust_chi2 = [&]() {  // activeRobustChi2 over the level-0 edges, in edge order
    double chi = 0;
    for (int i = 0; i < N; i++) {
      if (E[i].outlier) continue;
      const double c = po_chi2(E[i], E[i].e);
      if (E[i].robust) {
        const double d = E[i].stereo ? dS : dM;
        double r0, r1;
        huber(c, d * d, d, r0, r1);
        chi += r0;
      } else {
        chi += c;
      }
    }
    return chi;
  };
  SE3 pose = se3_from_float(P.Tcw);
  int nBad = 0;
  for (int it = 0; it < 4; it++) {
    pose = se3_from_float(P.Tcw);  // vSE3->setEstimate(toSE3Quat(pFrame->mTcw))
    double lambda = 0, ni = 2, chk = 0;
    int nRaul = 0;
    double xbuf[6] = {0, 0, 0, 0, 0, 0};
    for (int iter = 0; iter < 10; iter++) {
      for (int i = 0; i < N; i++)
        if (!E[i].outlier) po_error(E[i], pose, fx, fy, cx, cy, bf, E[i].e);
      double currentChi = robust_chi2();
      const double iniChi = currentChi;
      double H[6][6] = {{0}}, b[6] = {0};
      for (int i = 0; i < N; i++) {
        if (E[i].outlier) continue;
        double pc[3];
        se3_map(pose, E[i].X, pc);
        const double x = pc[0], y = pc[1], invz = 1.0 / pc[2], invz_2 = invz * invz;
        double J[3][6] = {{x * y * invz_2 * fx, -(1 + (x * x * invz_2)) * fx, y * invz * fx,
                           -invz * fx, 0, x * invz_2 * fx},
                          {(1 + y * y * invz_2) * fy, -x * y * invz_2 * fy, -x * invz * fy, 0,
                           -invz * fy, y * invz_2 * fy},
                          {0, 0, 0, 0, 0, 0}};
        if (E[i].stereo) {
          J[2][0] = J[0][0] - bf * y * invz_2;
          J[2][1] = J[0][1] + bf * x * invz_2;
          J[2][2] = J[0][2];
          J[2][3] = J[0][3];
          J[2][4] = 0;
          J[2][5] = J[0][5] - bf * invz_2;
        }
        const int rows = E[i].stereo ? 3 : 2;
        double r1 = 1.0;
        if (E[i].robust) {
          const double d = E[i].stereo ? dS : dM;
          double r0;
          huber(po_chi2(E[i], E[i].e), d * d, d, r0, r1);
        }
        const double w = r1 * E[i].s;  // rho' Omega (Omega = s I)
        for (int a = 0; a < 6; a++) {
          for (int c = 0; c < 6; c++) {
            double acc = 0;
            for (int r = 0; r < rows; r++) acc += J[r][a] * w * J[r][c];
            H[a][c] += acc;
          }
          double g = 0;
          for (int r = 0; r < rows; r++) g += J[r][a] * (E[i].s * E[i].e[r]);
          b[a] -= r1 * g;  // b -= rho' A^T Omega e
        }
      }
      if (iter == 0) {
        double maxd = 0;
        for (int a = 0; a < 6; a++) maxd = std::max(maxd, std::fabs(H[a][a]));
        lambda = 1e-5 * maxd;
        ni = 2;
        nRaul = 0;
      }
      // g2o accumulates b -= rho' J^T Omega e and solves (H + lambda I) dx = b
      double rhs[6];
      for (int a = 0; a < 6; a++) rhs[a] = b[a];
      double rho = 0, lastTrialChi = 0;
      int qmax = 0;
      do {
        const SE3 pose_b = pose;
        double Hs[6][6];
        for (int a = 0; a < 6; a++)
          for (int c = 0; c < 6; c++) Hs[a][c] = H[a][c] + (a == c ? lambda : 0.0);
        double xp[6];
        const bool ok2 = ldlt_solve6(Hs, rhs, xp);
        if (ok2) memcpy(xbuf, xp, sizeof(xp));
        pose = se3_mul(se3_exp(xbuf), pose);
        for (int i = 0; i < N; i++)
          if (!E[i].outlier) po_error(E[i], pose, fx, fy, cx, cy, bf, E[i].e);
        double tempChi = robust_chi2();
        lastTrialChi = tempChi;
        if (!ok2) tempChi = DBL_MAX;
        rho = currentChi - tempChi;
        double scale = 0;
        for (int a = 0; a < 6; a++) scale += xbuf[a] * (lambda * xbuf[a] + rhs[a]);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && std::isfinite(tempChi)) {
          double alpha = 1. - std::pow((2 * rho - 1), 3);
          alpha = std::min(alpha, 2. / 3.);
          lambda *= std::max(1. / 3., alpha);
          ni = 2;
          currentChi = tempChi;
        } else {
          lambda *= ni;
          ni *= 2;
          pose = pose_b;
        }
        qmax++;
      } while (rho < 0 && qmax < 10);
      bool ok = true;
      if (qmax == 10 || rho == 0) ok = false;
      if (ok) {
        if ((iniChi - currentChi) * 1e3 < iniChi)
          nRaul++;
        else
          nRaul = 0;
        if (nRaul >= 3) ok = false;
      }
      if (chk < lastTrialChi && iter > 0) ok = false;
      chk = lastTrialChi;
      if (!ok) break;
    }
    // re-classification (Optimizer.cc:3266-3322): edges that sat this round out get their error
    // at the optimised pose; the others keep the last computed one
    nBad = 0;
    for (int i = 0; i < N; i++) {
      if (E[i].outlier) po_error(E[i], pose, fx, fy, cx, cy, bf, E[i].e);
      const double c = po_chi2(E[i], E[i].e);
      const float thr = E[i].stereo ? chi2Stereo : chi2Mono;
      if (c > thr) {
        E[i].outlier = true;
        nBad++;
      } else {
        E[i].outlier = false;
      }
      if (it == 2) E[i].robust = false;
    }
    if (N < 10) break;  // optimizer.edges().size() < 10
  }
  se3_to_float(pose, pose_out);
  for (int i = 0; i < N; i++) outlier[i] = E[i].outlier ? 1 : 0;
  return N - nBad;
}

}  // namespace oracle
