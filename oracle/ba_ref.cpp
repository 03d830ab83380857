// oracle/ba_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// CPU restatement of the solve inside Optimizer::LocalBundleAdjustment (src/Optimizer.cc:3394-3665)
// as the vendored, modified g2o executes it:
//   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ        types/types_six_dof_expmap.{h:91-141,cpp:103-234}
//   VertexSE3Expmap (left-multiplied exp), VertexSBAPointXYZ (additive)
//   BaseBinaryEdge::constructQuadraticForm             core/base_binary_edge.hpp:55-115
//   BlockSolver_6_3: buildSystem, setLambda, Schur     core/block_solver.hpp:354-489, 502-604
//   LinearSolverEigen (SimplicialLDLT<Upper>)          solvers/linear_solver_eigen.h:94-121
//   OptimizationAlgorithmLevenberg::solve + Raul stop  core/optimization_algorithm_levenberg.cpp:60-159
//   SparseOptimizer::optimize (chi2-increase stop)     core/sparse_optimizer.cpp:354-400
//   initializeOptimization(level): vertices without an edge of the level sit out
// and the two rounds of LocalBundleAdjustment: optimize(5) with Huber kernels, edges with
// chi2 > 5.991 / 7.815 (or behind a camera) moved to level 1, kernels dropped, optimize(10) over
// level 0, then the erase test over every edge (Optimizer.cc:3547-3631).
//
// Pinned choices:
//  * the reduced camera system is solved by a dense LDL^T in keyframe order without pivoting; the
//    reference's sparse SimplicialLDLT with an AMD ordering is the same factorisation in another
//    elimination order (results agree to rounding).  A zero pivot fails the solve, as Eigen's
//    (the solver's x then stays at its previous value, and g2o applies it anyway);
//  * sums run in edge order (points in the caller's order, each point's observations in keyframe
//    order); g2o's own order follows its hash maps and is not reproducible;
//  * the 3x3 landmark inverse is Eigen's cofactor formula (Inverse.h, compute_inverse_size3).
// pbStopFlag (mbAbortBA) is never raised: LocalMapping runs synchronously.

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "oracle_se3.h"
#include "oracle_solve.h"

namespace oracle {

namespace {

struct BAEdge {
  int pt, kf;
  double obs[3], s;
  bool stereo;
  int level;     // 1: set aside after round 1 (setLevel(1))
  bool robust;   // Huber kernel attached
  double e[3];   // _error of the last computeActiveErrors that included the edge
};

struct Cam {
  double fx, fy, cx, cy, bf;
};

// EdgeSE3ProjectXYZ::computeError / EdgeStereoSE3ProjectXYZ::computeError
void edge_error(const BAEdge& E, const SE3& T, const double* X, const Cam& c, double e[3]) {
  double pc[3];
  se3_map(T, X, pc);
  if (!E.stereo) {
    const double px = pc[0] / pc[2], py = pc[1] / pc[2];  // project2d
    e[0] = E.obs[0] - (px * c.fx + c.cx);
    e[1] = E.obs[1] - (py * c.fy + c.cy);
    e[2] = 0;
  } else {
    const float invz = 1.0f / pc[2];  // cam_project's float invz
    const double u = pc[0] * invz * c.fx + c.cx, v = pc[1] * invz * c.fy + c.cy;
    e[0] = E.obs[0] - u;
    e[1] = E.obs[1] - v;
    e[2] = E.obs[2] - (u - c.bf * invz);
  }
}

inline double edge_chi2(const BAEdge& E) {  // _error^T Omega _error, Omega = s I
  return E.stereo ? E.s * (E.e[0] * E.e[0] + E.e[1] * E.e[1] + E.e[2] * E.e[2])
                  : E.s * (E.e[0] * E.e[0] + E.e[1] * E.e[1]);
}

inline void huber_rho(double e, double delta, double& r0, double& r1) {  // RobustKernelHuber
  const double dsqr = delta * delta;
  if (e <= dsqr) {
    r0 = e;
    r1 = 1.;
  } else {
    const double s = std::sqrt(e);
    r0 = 2 * s * delta - dsqr;
    r1 = delta / s;
  }
}

// linearizeOplus: Jl (rows x 3, the point) and Jp (rows x 6, the pose)
void edge_jacobians(const BAEdge& E, const SE3& T, const double* X, const Cam& c, double Jl[3][3],
                    double Jp[3][6]) {
  double pc[3], R[3][3];
  se3_map(T, X, pc);
  quat_to_R(T.q, R);
  const double x = pc[0], y = pc[1], z = pc[2], z_2 = z * z;
  if (!E.stereo) {
    const double tmp[2][3] = {{c.fx, 0, -x / z * c.fx}, {0, c.fy, -y / z * c.fy}};
    const double s = -1. / z;
    for (int r = 0; r < 2; r++)
      for (int k = 0; k < 3; k++) {
        double a = 0;
        for (int m = 0; m < 3; m++) a += (s * tmp[r][m]) * R[m][k];
        Jl[r][k] = a;
      }
  } else {
    for (int k = 0; k < 3; k++) {
      Jl[0][k] = -c.fx * R[0][k] / z + c.fx * x * R[2][k] / z_2;
      Jl[1][k] = -c.fy * R[1][k] / z + c.fy * y * R[2][k] / z_2;
      Jl[2][k] = Jl[0][k] - c.bf * R[2][k] / z_2;
    }
  }
  Jp[0][0] = x * y / z_2 * c.fx;
  Jp[0][1] = -(1 + (x * x / z_2)) * c.fx;
  Jp[0][2] = y / z * c.fx;
  Jp[0][3] = -1. / z * c.fx;
  Jp[0][4] = 0;
  Jp[0][5] = x / z_2 * c.fx;
  Jp[1][0] = (1 + y * y / z_2) * c.fy;
  Jp[1][1] = -x * y / z_2 * c.fy;
  Jp[1][2] = -x / z * c.fy;
  Jp[1][3] = 0;
  Jp[1][4] = -1. / z * c.fy;
  Jp[1][5] = y / z_2 * c.fy;
  if (E.stereo) {
    Jp[2][0] = Jp[0][0] - c.bf * y / z_2;
    Jp[2][1] = Jp[0][1] + c.bf * x / z_2;
    Jp[2][2] = Jp[0][2];
    Jp[2][3] = Jp[0][3];
    Jp[2][4] = 0;
    Jp[2][5] = Jp[0][5] - c.bf / z_2;
  }
}

// Eigen's fixed-size 3x3 inverse: cofactors of column 0, det, then the adjugate rows
void inverse3(const double m[3][3], double r[3][3]) {
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
  };
  const double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
  const double det = c0[0] * m[0][0] + c0[1] * m[1][0] + c0[2] * m[2][0];
  const double invdet = 1.0 / det;
  for (int k = 0; k < 3; k++) r[0][k] = c0[k] * invdet;
  r[1][0] = cof(0, 1) * invdet;
  r[1][1] = cof(1, 1) * invdet;
  r[1][2] = cof(2, 1) * invdet;
  r[2][0] = cof(0, 2) * invdet;
  r[2][1] = cof(1, 2) * invdet;
  r[2][2] = cof(2, 2) * invdet;
}

// dense LDL^T of the upper triangle of the n x n matrix A (row-major), natural order, no pivoting;
// false on a zero pivot (Eigen SimplicialLDLT's NumericalIssue)
bool ldlt_dense(std::vector<double>& A, int n, const std::vector<double>& b, std::vector<double>& x) {
  // L stored in the strict lower triangle of A (the upper triangle is read as the input)
  std::vector<double> D(n);
  std::vector<double> L((size_t)n * n, 0.0);
  for (int k = 0; k < n; k++) {
    double d = A[(size_t)k * n + k];
    for (int c = 0; c < k; c++) d -= L[(size_t)k * n + c] * L[(size_t)k * n + c] * D[c];
    if (d == 0) return false;
    D[k] = d;
    for (int i = k + 1; i < n; i++) {
      double s = A[(size_t)k * n + i];  // upper triangle: A(k, i) = A(i, k)
      for (int c = 0; c < k; c++) s -= L[(size_t)i * n + c] * L[(size_t)k * n + c] * D[c];
      L[(size_t)i * n + k] = s / d;
    }
  }
  std::vector<double> y(b);
  for (int i = 0; i < n; i++)
    for (int c = 0; c < i; c++) y[i] -= L[(size_t)i * n + c] * y[c];
  for (int i = 0; i < n; i++) y[i] /= D[i];
  for (int i = n - 1; i >= 0; i--)
    for (int r = i + 1; r < n; r++) y[i] -= L[(size_t)r * n + i] * y[r];
  x = y;
  return true;
}

struct BAState {
  std::vector<SE3> pose;
  std::vector<double> X;  // n_pt x 3
};

}  // namespace

// One SparseOptimizer::optimize(iters) over the edges of `level` (the round's active set).
static int optimize(const BAProblem& P, const Cam& cam, std::vector<BAEdge>& E, BAState& S,
                    int iters, int level, int* trials) {
  const int nK = P.n_kf, nP = P.n_pt;
  // the active graph: edges of the level with a non-fixed vertex; the vertices they touch
  std::vector<int> act;
  std::vector<uint8_t> kfUsed(nK, 0), ptUsed(nP, 0);
  for (int i = 0; i < (int)E.size(); i++) {
    if (E[i].level != level) continue;
    act.push_back(i);
    kfUsed[E[i].kf] = 1;
    ptUsed[E[i].pt] = 1;
  }
  // index mapping: non-fixed keyframes with an active edge (keyframe order), then the points
  std::vector<int> kIdx(nK, -1), kList;
  for (int k = 0; k < nK; k++)
    if (kfUsed[k] && !P.fixed[k]) {
      kIdx[k] = (int)kList.size();
      kList.push_back(k);
    }
  std::vector<int> pList;
  for (int j = 0; j < nP; j++)
    if (ptUsed[j]) pList.push_back(j);
  if (kList.empty() && pList.empty()) return 0;  // "0 vertices to optimize"
  const int nk = (int)kList.size(), n6 = 6 * nk;
  // each point's active edges, in edge order
  std::vector<std::vector<int>> ptEdges(nP);
  for (int i : act) ptEdges[E[i].pt].push_back(i);

  const float dMonoF = std::sqrt(5.991), dStereoF = std::sqrt(7.815);
  const double dMono = dMonoF, dStereo = dStereoF;
  auto compute_errors = [&]() {
    for (int i : act) edge_error(E[i], S.pose[E[i].kf], &S.X[3 * (size_t)E[i].pt], cam, E[i].e);
  };
  auto robust_chi2 = [&]() {
    double chi = 0;
    for (int i : act) {
      const double c = edge_chi2(E[i]);
      if (E[i].robust) {
        double r0, r1;
        huber_rho(c, E[i].stereo ? dStereo : dMono, r0, r1);
        chi += r0;
      } else {
        chi += c;
      }
    }
    return chi;
  };

  // per-edge Hpl blocks (6 x 3), the vertices' H and b
  std::vector<double> Hpl(18 * E.size(), 0.0);
  std::vector<double> Hpp(36 * (size_t)nK), bp(6 * (size_t)nK), Hll(9 * (size_t)nP),
      bl(3 * (size_t)nP);
  std::vector<double> xbuf(n6 + 3 * (size_t)nP, 0.0);  // g2o's persistent _x (poses, then points)
  double lambda = 0, ni = 2, chk = 0;
  int nBad = 0, it_done = 0;
  for (int iter = 0; iter < iters; iter++) {
    compute_errors();
    double currentChi = robust_chi2();
    const double iniChi = currentChi;
    // buildSystem
    std::fill(Hpp.begin(), Hpp.end(), 0.0);
    std::fill(bp.begin(), bp.end(), 0.0);
    std::fill(Hll.begin(), Hll.end(), 0.0);
    std::fill(bl.begin(), bl.end(), 0.0);
    for (int i : act) {
      BAEdge& e = E[i];
      const int k = e.kf, j = e.pt;
      double Jl[3][3], Jp[3][6];
      edge_jacobians(e, S.pose[k], &S.X[3 * (size_t)j], cam, Jl, Jp);
      const int rows = e.stereo ? 3 : 2;
      double r1 = 1.0;
      if (e.robust) {
        double r0;
        huber_rho(edge_chi2(e), e.stereo ? dStereo : dMono, r0, r1);
      }
      const double w = r1 * e.s;  // robustInformation: rho' Omega
      double om[3];
      for (int r = 0; r < rows; r++) om[r] = -(e.s * e.e[r]) * r1;  // omega_r = -Omega e (* rho')
      double* hl = &Hll[9 * (size_t)j];
      for (int a = 0; a < 3; a++) {
        for (int b = 0; b < 3; b++) {
          double acc = 0;
          for (int r = 0; r < rows; r++) acc += Jl[r][a] * w * Jl[r][b];
          hl[3 * a + b] += acc;
        }
        double g = 0;
        for (int r = 0; r < rows; r++) g += Jl[r][a] * om[r];
        bl[3 * (size_t)j + a] += g;
      }
      if (P.fixed[k]) continue;
      double* hp = &Hpp[36 * (size_t)k];
      double* hpl = &Hpl[18 * (size_t)i];
      for (int a = 0; a < 6; a++) {
        for (int b = 0; b < 6; b++) {
          double acc = 0;
          for (int r = 0; r < rows; r++) acc += Jp[r][a] * w * Jp[r][b];
          hp[6 * a + b] += acc;
        }
        for (int b = 0; b < 3; b++) {
          double acc = 0;
          for (int r = 0; r < rows; r++) acc += Jp[r][a] * w * Jl[r][b];
          hpl[3 * a + b] = acc;
        }
        double g = 0;
        for (int r = 0; r < rows; r++) g += Jp[r][a] * om[r];
        bp[6 * (size_t)k + a] += g;
      }
    }
    if (iter == 0) {  // computeLambdaInit over the index-mapped vertices
      double maxd = 0;
      for (int k : kList)
        for (int a = 0; a < 6; a++) maxd = std::max(maxd, std::fabs(Hpp[36 * (size_t)k + 7 * a]));
      for (int j : pList)
        for (int a = 0; a < 3; a++) maxd = std::max(maxd, std::fabs(Hll[9 * (size_t)j + 4 * a]));
      lambda = 1e-5 * maxd;
      ni = 2;
      nBad = 0;
    }
    double rho = 0, lastTrialChi = 0;
    int qmax = 0;
    do {
      const BAState backup = S;
      // Schur complement over the points (block_solver.hpp:406-489)
      std::vector<double> Sm((size_t)n6 * n6, 0.0), coef(n6, 0.0);
      for (int a = 0; a < nk; a++) {
        const double* hp = &Hpp[36 * (size_t)kList[a]];
        for (int r = 0; r < 6; r++)
          for (int c = 0; c < 6; c++)
            Sm[(size_t)(6 * a + r) * n6 + 6 * a + c] = hp[6 * r + c] + (r == c ? lambda : 0.0);
      }
      std::vector<double> Dinv(9 * (size_t)nP, 0.0);
      for (int j : pList) {
        double D[3][3], Di[3][3];
        for (int a = 0; a < 3; a++)
          for (int b = 0; b < 3; b++) D[a][b] = Hll[9 * (size_t)j + 3 * a + b] + (a == b ? lambda : 0.0);
        inverse3(D, Di);
        memcpy(&Dinv[9 * (size_t)j], Di, sizeof(Di));
        double db[3];
        for (int a = 0; a < 3; a++)
          db[a] = Di[a][0] * bl[3 * (size_t)j] + Di[a][1] * bl[3 * (size_t)j + 1] +
                  Di[a][2] * bl[3 * (size_t)j + 2];
        // this point's edges to optimised keyframes, in keyframe (= pose index) order
        std::vector<std::pair<int, int>> col;
        for (int i : ptEdges[j])
          if (kIdx[E[i].kf] >= 0) col.push_back({kIdx[E[i].kf], i});
        std::sort(col.begin(), col.end());
        for (size_t p1 = 0; p1 < col.size(); p1++) {
          const int a = col[p1].first;
          const double* B1 = &Hpl[18 * (size_t)col[p1].second];
          double BD[6][3];
          for (int r = 0; r < 6; r++) {
            for (int c = 0; c < 3; c++)
              BD[r][c] = B1[3 * r] * Di[0][c] + B1[3 * r + 1] * Di[1][c] + B1[3 * r + 2] * Di[2][c];
            coef[6 * a + r] += B1[3 * r] * db[0] + B1[3 * r + 1] * db[1] + B1[3 * r + 2] * db[2];
          }
          for (size_t p2 = p1; p2 < col.size(); p2++) {
            const int b = col[p2].first;
            const double* B2 = &Hpl[18 * (size_t)col[p2].second];
            for (int r = 0; r < 6; r++)
              for (int c = 0; c < 6; c++)
                Sm[(size_t)(6 * a + r) * n6 + 6 * b + c] -=
                    BD[r][0] * B2[3 * c] + BD[r][1] * B2[3 * c + 1] + BD[r][2] * B2[3 * c + 2];
          }
        }
      }
      std::vector<double> bs(n6), xp;
      for (int a = 0; a < nk; a++)
        for (int r = 0; r < 6; r++) bs[6 * a + r] = bp[6 * (size_t)kList[a] + r] - coef[6 * a + r];
      const bool ok2 = n6 == 0 ? true : ldlt_dense(Sm, n6, bs, xp);
      if (ok2) {
        for (int q = 0; q < n6; q++) xbuf[q] = xp[q];
        // landmark increments: xl = Dinv (bl - Hpl^T xp)
        for (int j : pList) {
          double cl[3] = {bl[3 * (size_t)j], bl[3 * (size_t)j + 1], bl[3 * (size_t)j + 2]};
          for (int i : ptEdges[j]) {
            const int a = kIdx[E[i].kf];
            if (a < 0) continue;
            const double* B = &Hpl[18 * (size_t)i];
            for (int c = 0; c < 3; c++)
              for (int r = 0; r < 6; r++) cl[c] += B[3 * r + c] * (-xp[6 * a + r]);
          }
          const double* Di = &Dinv[9 * (size_t)j];
          for (int a = 0; a < 3; a++)
            xbuf[n6 + 3 * (size_t)j + a] = Di[3 * a] * cl[0] + Di[3 * a + 1] * cl[1] + Di[3 * a + 2] * cl[2];
        }
      }
      // SparseOptimizer::update (applied even when the solve failed: stale _x)
      for (int a = 0; a < nk; a++) {
        const int k = kList[a];
        S.pose[k] = se3_mul(se3_exp(&xbuf[6 * a]), S.pose[k]);
      }
      for (int j : pList)
        for (int a = 0; a < 3; a++) S.X[3 * (size_t)j + a] += xbuf[n6 + 3 * (size_t)j + a];
      compute_errors();
      double tempChi = robust_chi2();
      lastTrialChi = tempChi;
      if (!ok2) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      double scale = 0;
      for (int a = 0; a < nk; a++)
        for (int r = 0; r < 6; r++)
          scale += xbuf[6 * a + r] * (lambda * xbuf[6 * a + r] + bp[6 * (size_t)kList[a] + r]);
      for (int j : pList)
        for (int a = 0; a < 3; a++)
          scale += xbuf[n6 + 3 * (size_t)j + a] *
                   (lambda * xbuf[n6 + 3 * (size_t)j + a] + bl[3 * (size_t)j + a]);
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
        S = backup;
      }
      qmax++;
      if (trials) (*trials)++;
    } while (rho < 0 && qmax < 10);
    bool ok = true;
    if (qmax == 10 || rho == 0) ok = false;
    if (ok) {
      if ((iniChi - currentChi) * 1e3 < iniChi)
        nBad++;
      else
        nBad = 0;
      if (nBad >= 3) ok = false;
    }
    if (chk < lastTrialChi && iter > 0) ok = false;  // sparse_optimizer.cpp:393-396
    chk = lastTrialChi;
    it_done = iter + 1;
    if (!ok) break;
  }
  return it_done;
}

int local_ba_solve(const BAProblem& P, BAResult& out) {
  const Cam cam{P.fx, P.fy, P.cx, P.cy, P.bf};
  std::vector<BAEdge> E(P.n_edge);
  for (int i = 0; i < P.n_edge; i++) {
    BAEdge& e = E[i];
    e.pt = P.e_pt[i];
    e.kf = P.e_kf[i];
    for (int k = 0; k < 3; k++) e.obs[k] = P.e_obs[3 * i + k];
    e.stereo = !(P.e_obs[3 * i + 2] < 0);  // mvuRight < 0: monocular observation
    e.s = P.e_inv_sigma2[i];               // Identity * invSigma2 (float)
    e.level = 0;
    e.robust = true;
    e.e[0] = e.e[1] = e.e[2] = 0;
  }
  BAState S;
  S.pose.resize(P.n_kf);
  for (int k = 0; k < P.n_kf; k++) S.pose[k] = se3_from_float(P.Tcw + 16 * (size_t)k);
  S.X.resize(3 * (size_t)P.n_pt);
  for (size_t q = 0; q < 3 * (size_t)P.n_pt; q++) S.X[q] = P.Xw[q];
  out = BAResult();
  out.iterations[0] = optimize(P, cam, E, S, 5, 0, &out.trials[0]);
  auto depth_positive = [&](const BAEdge& e) {
    double pc[3];
    se3_map(S.pose[e.kf], &S.X[3 * (size_t)e.pt], pc);
    return pc[2] > 0.0;
  };
  // check inlier observations (Optimizer.cc:3559-3590): chi2 of the last computed error
  for (BAEdge& e : E) {
    const double th = e.stereo ? 7.815 : 5.991;
    if (edge_chi2(e) > th || !depth_positive(e)) e.level = 1;
    e.robust = false;
  }
  out.iterations[1] = optimize(P, cam, E, S, 10, 0, &out.trials[1]);
  out.erase.assign(P.n_edge, 0);
  for (int i = 0; i < P.n_edge; i++) {
    const BAEdge& e = E[i];
    const double th = e.stereo ? 7.815 : 5.991;
    if (edge_chi2(e) > th || !depth_positive(e)) {
      out.erase[i] = 1;
      out.n_erase++;
    }
  }
  out.Tcw.resize(16 * (size_t)P.n_kf);
  for (int k = 0; k < P.n_kf; k++) se3_to_float(S.pose[k], &out.Tcw[16 * (size_t)k]);
  out.Xw.resize(3 * (size_t)P.n_pt);
  for (size_t q = 0; q < 3 * (size_t)P.n_pt; q++) out.Xw[q] = (float)S.X[q];
  return 0;
}

}  // namespace oracle
