// oracle/pnp_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// CPU restatement of the object-motion initialiser D5: Tracking::GetInitModelObj's
// cv::solvePnPRansac(..., 500, 0.3, 0.98, inliers, SOLVEPNP_AP3P) (reference
// src/Tracking.cc:4324-4443).  OpenCV is not vendored; the RANSAC
// registrator, RNG, undistortPoints/projectPoints with zero distortion and Rodrigues are restated
// from their public 3.x/4.x sources; EPnP follows the reference's own Lepetit EPnP,
// src/PnPsolver.cc:342-1022 (same lineage as OpenCV's epnp.cpp).  The SVDs are one-sided /
// cyclic Jacobi in double (OpenCV's cvSVD is Jacobi as well; only singular-vector signs may
// differ and those cancel through the beta signs and solve_for_sign).

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle_solve.h"

namespace oracle {

// ---------------------------------------------------------------- small dense linear algebra
// Symmetric eigen-decomposition by cyclic Jacobi; eigenvectors returned as ROWS of `vt`, sorted by
// descending eigenvalue (cvSVD(A, D, Ut, 0, MODIFY_A | U_T) of a symmetric PSD matrix).
static void jacobi_eig_sym(int n, const double* Ain, double* d, double* vt) {
  std::vector<double> A(Ain, Ain + n * n), V(n * n, 0.0);
  for (int i = 0; i < n; i++) V[i * n + i] = 1.0;
  for (int sweep = 0; sweep < 100; sweep++) {
    // converged when the off-diagonal mass is below (1e-13)^2 of the diagonal's: rotations leave
    // residues of order eps * |a_pp| behind, so an absolute threshold is never reached
    double off = 0, dsum = 0;
    for (int p = 0; p < n; p++) {
      dsum += A[p * n + p] * A[p * n + p];
      for (int q = p + 1; q < n; q++) off += A[p * n + q] * A[p * n + q];
    }
    if (off <= 1e-26 * dsum) break;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) {
        const double apq = A[p * n + q];
        if (std::fabs(apq) < 1e-300) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double theta = (aqq - app) / (2 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        const double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; k++) {
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; k++) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; k++) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
  std::vector<int> ord(n);
  for (int i = 0; i < n; i++) ord[i] = i;
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return A[a * n + a] > A[b * n + b]; });
  for (int r = 0; r < n; r++) {
    d[r] = A[ord[r] * n + ord[r]];
    for (int k = 0; k < n; k++) vt[r * n + k] = V[k * n + ord[r]];
  }
}

// EPnP's cvSVD(MtM, D, Ut, 0, MODIFY_A | U_T) (PnPsolver.cc:392-395 lineage) by one-sided
// (Hestenes) Jacobi in PARALLEL ORDER: each sweep is 11 rounds of 6 disjoint column pairs
// (round-robin schedule, column 11 fixed); a pair is rotated unless its columns are already
// orthogonal to 1e-15 relative; sweeps stop when a whole sweep rotates nothing.  Disjoint pairs
// touch disjoint columns, so the rounds equal sequential processing in schedule order; the GPU
// (mmt_pnp.hip: eig12_group) runs one column per lane and follows this loop operation for
// operation.  M^T M is symmetric PSD, so its singular vectors are its eigenvectors: `vt` rows are
// the accumulated right vectors (V columns), ordered by descending column norm (= singular value).
static inline void rr_partner(int r, int j, int& p, int& q) {
  const int k = j == 11 ? r : (j == r ? 11 : (2 * r - j + 22) % 11);
  p = std::min(j, k);
  q = std::max(j, k);
}

static void jacobi_eig12(const double* Ain, double* vt) {
  const int n = 12;
  double A[144], V[144];  // row-major: A[k * 12 + j] = row k, column j
  memcpy(A, Ain, sizeof(A));
  for (int i = 0; i < 144; i++) V[i] = (i % 13 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 100; sweep++) {
    bool rotated = false;
    for (int r = 0; r < 11; r++)
      for (int slot = 0; slot < 6; slot++) {
        const int a0 = slot == 0 ? r : (r + slot) % 11, b0 = slot == 0 ? 11 : (r - slot + 11) % 11;
        const int p = std::min(a0, b0), q = std::max(a0, b0);
        double al = 0, be = 0, ga = 0;
        for (int k = 0; k < n; k++) {
          al += A[k * n + p] * A[k * n + p];
          be += A[k * n + q] * A[k * n + q];
          ga += A[k * n + p] * A[k * n + q];
        }
        if (std::fabs(ga) <= 1e-15 * std::sqrt(al * be) || ga == 0) continue;
        rotated = true;
        const double zeta = (be - al) / (2 * ga);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (int k = 0; k < n; k++) {
          const double x = A[k * n + p], y = A[k * n + q];
          A[k * n + p] = c * x - s * y;
          A[k * n + q] = s * x + c * y;
          const double vx = V[k * n + p], vy = V[k * n + q];
          V[k * n + p] = c * vx - s * vy;
          V[k * n + q] = s * vx + c * vy;
        }
      }
    if (!rotated) break;
  }
  double sig[12];
  for (int j = 0; j < n; j++) {
    double ss = 0;
    for (int k = 0; k < n; k++) ss += A[k * n + j] * A[k * n + j];
    sig[j] = std::sqrt(ss);
  }
  for (int j = 0; j < n; j++) {  // stable descending order
    int rank = 0;
    for (int i = 0; i < n; i++) rank += (sig[i] > sig[j]) || (i < j && sig[i] == sig[j]);
    for (int k = 0; k < n; k++) vt[rank * n + k] = V[k * n + j];
  }
}

// Thin SVD of an m x n matrix (m >= n) by one-sided Jacobi: A = U diag(w) V^T.
static void jacobi_svd(int m, int n, const double* Ain, double* U, double* w, double* V) {
  std::vector<double> A(Ain, Ain + m * n);
  for (int i = 0; i < n * n; i++) V[i] = 0;
  for (int i = 0; i < n; i++) V[i * n + i] = 1;
  for (int sweep = 0; sweep < 100; sweep++) {
    bool changed = false;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) {
        double a = 0, b = 0, g = 0;
        for (int k = 0; k < m; k++) {
          a += A[k * n + p] * A[k * n + p];
          b += A[k * n + q] * A[k * n + q];
          g += A[k * n + p] * A[k * n + q];
        }
        if (std::fabs(g) <= 1e-15 * std::sqrt(a * b) || g == 0) continue;
        changed = true;
        const double zeta = (b - a) / (2 * g);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (int k = 0; k < m; k++) {
          const double x = A[k * n + p], y = A[k * n + q];
          A[k * n + p] = c * x - s * y;
          A[k * n + q] = s * x + c * y;
        }
        for (int k = 0; k < n; k++) {
          const double x = V[k * n + p], y = V[k * n + q];
          V[k * n + p] = c * x - s * y;
          V[k * n + q] = s * x + c * y;
        }
      }
    if (!changed) break;
  }
  for (int j = 0; j < n; j++) {
    double s = 0;
    for (int k = 0; k < m; k++) s += A[k * n + j] * A[k * n + j];
    w[j] = std::sqrt(s);
    for (int k = 0; k < m; k++) U[k * n + j] = w[j] > 0 ? A[k * n + j] / w[j] : 0.0;
  }
}

// x = pinv(A) b (cvSolve(..., CV_SVD)); A is m x n, m >= n.
static void svd_solve(int m, int n, const double* A, const double* b, double* x) {
  std::vector<double> U(m * n), w(n), V(n * n);
  jacobi_svd(m, n, A, U.data(), w.data(), V.data());
  double wmax = 0;
  for (int j = 0; j < n; j++) wmax = std::max(wmax, w[j]);
  const double thr = DBL_EPSILON * wmax * m;
  for (int i = 0; i < n; i++) x[i] = 0;
  for (int j = 0; j < n; j++) {
    if (w[j] <= thr) continue;
    double ub = 0;
    for (int k = 0; k < m; k++) ub += U[k * n + j] * b[k];
    ub /= w[j];
    for (int i = 0; i < n; i++) x[i] += V[i * n + j] * ub;
  }
}

// ---------------------------------------------------------------- EPnP (PnPsolver.cc:342-1022)
namespace {
struct EPnP {
  int n = 0;
  double fu, fv, uc, vc;
  std::vector<double> pws, us, alphas, pcs;
  double cws[4][3], ccs[4][3];

  void choose_control_points() {
    cws[0][0] = cws[0][1] = cws[0][2] = 0;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) cws[0][j] += pws[3 * i + j];
    for (int j = 0; j < 3; j++) cws[0][j] /= n;
    double m[9] = {0};
    for (int i = 0; i < n; i++) {
      double p[3];
      for (int j = 0; j < 3; j++) p[j] = pws[3 * i + j] - cws[0][j];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) m[3 * a + b] += p[a] * p[b];
    }
    double dc[3], uct[9];
    jacobi_eig_sym(3, m, dc, uct);
    for (int i = 1; i < 4; i++) {
      const double k = std::sqrt(std::max(dc[i - 1], 0.0) / n);
      for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
    }
  }
  void compute_barycentric_coordinates() {
    double cc[9];
    for (int i = 0; i < 3; i++)
      for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    // cvInvert(CC, CC_inv, CV_SVD): pseudo-inverse through the SVD
    double U[9], w[3], V[9], ci[9];
    jacobi_svd(3, 3, cc, U, w, V);
    double wmax = std::max(w[0], std::max(w[1], w[2]));
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        double s = 0;
        for (int k = 0; k < 3; k++)
          if (w[k] > DBL_EPSILON * wmax * 3) s += V[r * 3 + k] * U[c * 3 + k] / w[k];
        ci[3 * r + c] = s;
      }
    for (int i = 0; i < n; i++) {
      const double* pi = &pws[3 * i];
      double* a = &alphas[4 * i];
      for (int j = 0; j < 3; j++)
        a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) +
                   ci[3 * j + 2] * (pi[2] - cws[0][2]);
      a[0] = 1.0f - a[1] - a[2] - a[3];
    }
  }
  void compute_ccs(const double* betas, const double* ut) {
    for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
    for (int i = 0; i < 4; i++) {
      const double* v = ut + 12 * (11 - i);
      for (int j = 0; j < 4; j++)
        for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
    }
  }
  void compute_pcs() {
    for (int i = 0; i < n; i++) {
      const double* a = &alphas[4 * i];
      double* pc = &pcs[3 * i];
      for (int j = 0; j < 3; j++)
        pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }
  }
  static double dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
  static double dist2(const double* a, const double* b) {
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
  }
  double reprojection_error(const double R[3][3], const double t[3]) {
    double sum2 = 0.0;
    for (int i = 0; i < n; i++) {
      const double* pw = &pws[3 * i];
      const double Xc = dot(R[0], pw) + t[0], Yc = dot(R[1], pw) + t[1];
      const double inv_Zc = 1.0 / (dot(R[2], pw) + t[2]);
      const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
      const double u = us[2 * i], v = us[2 * i + 1];
      sum2 += std::sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / n;
  }
  void estimate_R_and_t(double R[3][3], double t[3]) {
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) {
        pc0[j] += pcs[3 * i + j];
        pw0[j] += pws[3 * i + j];
      }
    for (int j = 0; j < 3; j++) {
      pc0[j] /= n;
      pw0[j] /= n;
    }
    double abt[9] = {0};
    for (int i = 0; i < n; i++) {
      const double* pc = &pcs[3 * i];
      const double* pw = &pws[3 * i];
      for (int j = 0; j < 3; j++) {
        abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
        abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
        abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
      }
    }
    double U[9], w[3], V[9];
    jacobi_svd(3, 3, abt, U, w, V);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i][j] = dot(U + 3 * i, V + 3 * j);
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] +
                       R[0][2] * R[1][0] * R[2][1] - R[0][2] * R[1][1] * R[2][0] -
                       R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) {
      R[2][0] = -R[2][0];
      R[2][1] = -R[2][1];
      R[2][2] = -R[2][2];
    }
    t[0] = pc0[0] - dot(R[0], pw0);
    t[1] = pc0[1] - dot(R[1], pw0);
    t[2] = pc0[2] - dot(R[2], pw0);
  }
  void solve_for_sign() {
    if (pcs[2] < 0.0) {
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
      for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) pcs[3 * i + j] = -pcs[3 * i + j];
    }
  }
  double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {
    compute_ccs(betas, ut);
    compute_pcs();
    solve_for_sign();
    estimate_R_and_t(R, t);
    return reprojection_error(R, t);
  }
  static void compute_L_6x10(const double* ut, double* l) {
    const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; i++) {
      int a = 0, b = 1;
      for (int j = 0; j < 6; j++) {
        for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
        b++;
        if (b > 3) {
          a++;
          b = a + 1;
        }
      }
    }
    for (int i = 0; i < 6; i++) {
      double* row = l + 10 * i;
      row[0] = dot(dv[0][i], dv[0][i]);
      row[1] = 2.0f * dot(dv[0][i], dv[1][i]);
      row[2] = dot(dv[1][i], dv[1][i]);
      row[3] = 2.0f * dot(dv[0][i], dv[2][i]);
      row[4] = 2.0f * dot(dv[1][i], dv[2][i]);
      row[5] = dot(dv[2][i], dv[2][i]);
      row[6] = 2.0f * dot(dv[0][i], dv[3][i]);
      row[7] = 2.0f * dot(dv[1][i], dv[3][i]);
      row[8] = 2.0f * dot(dv[2][i], dv[3][i]);
      row[9] = dot(dv[3][i], dv[3][i]);
    }
  }
  void compute_rho(double* rho) {
    rho[0] = dist2(cws[0], cws[1]);
    rho[1] = dist2(cws[0], cws[2]);
    rho[2] = dist2(cws[0], cws[3]);
    rho[3] = dist2(cws[1], cws[2]);
    rho[4] = dist2(cws[1], cws[3]);
    rho[5] = dist2(cws[2], cws[3]);
  }
  static void betas_approx_1(const double* L, const double* rho, double* betas) {
    double A[24], b4[4];
    for (int i = 0; i < 6; i++) {
      A[4 * i] = L[10 * i];
      A[4 * i + 1] = L[10 * i + 1];
      A[4 * i + 2] = L[10 * i + 3];
      A[4 * i + 3] = L[10 * i + 6];
    }
    svd_solve(6, 4, A, rho, b4);
    if (b4[0] < 0) {
      betas[0] = std::sqrt(-b4[0]);
      betas[1] = -b4[1] / betas[0];
      betas[2] = -b4[2] / betas[0];
      betas[3] = -b4[3] / betas[0];
    } else {
      betas[0] = std::sqrt(b4[0]);
      betas[1] = b4[1] / betas[0];
      betas[2] = b4[2] / betas[0];
      betas[3] = b4[3] / betas[0];
    }
  }
  static void betas_approx_2(const double* L, const double* rho, double* betas) {
    double A[18], b3[3];
    for (int i = 0; i < 6; i++)
      for (int k = 0; k < 3; k++) A[3 * i + k] = L[10 * i + k];
    svd_solve(6, 3, A, rho, b3);
    if (b3[0] < 0) {
      betas[0] = std::sqrt(-b3[0]);
      betas[1] = (b3[2] < 0) ? std::sqrt(-b3[2]) : 0.0;
    } else {
      betas[0] = std::sqrt(b3[0]);
      betas[1] = (b3[2] > 0) ? std::sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
  }
  static void betas_approx_3(const double* L, const double* rho, double* betas) {
    double A[30], b5[5];
    for (int i = 0; i < 6; i++)
      for (int k = 0; k < 5; k++) A[5 * i + k] = L[10 * i + k];
    svd_solve(6, 5, A, rho, b5);
    if (b5[0] < 0) {
      betas[0] = std::sqrt(-b5[0]);
      betas[1] = (b5[2] < 0) ? std::sqrt(-b5[2]) : 0.0;
    } else {
      betas[0] = std::sqrt(b5[0]);
      betas[1] = (b5[2] > 0) ? std::sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
  }
  static void qr_solve(double* A, double* b, double* X) {  // PnPsolver.cc:840-950, 6x4
    const int nr = 6, nc = 4;
    double A1[6], A2[6];
    double *pA = A, *ppAkk = pA;
    for (int k = 0; k < nc; k++) {
      double *ppAik = ppAkk, eta = std::fabs(*ppAik);
      for (int i = k + 1; i < nr; i++) {
        double elt = std::fabs(*ppAik);
        if (eta < elt) eta = elt;
        ppAik += nc;
      }
      if (eta == 0) {
        A1[k] = A2[k] = 0.0;
        return;  // "A is singular" -- X left unchanged
      }
      double sum = 0.0, inv_eta = 1. / eta;
      ppAik = ppAkk;
      for (int i = k; i < nr; i++) {
        *ppAik *= inv_eta;
        sum += *ppAik * *ppAik;
        ppAik += nc;
      }
      double sigma = std::sqrt(sum);
      if (*ppAkk < 0) sigma = -sigma;
      *ppAkk += sigma;
      A1[k] = sigma * *ppAkk;
      A2[k] = -eta * sigma;
      for (int j = k + 1; j < nc; j++) {
        double* pp = ppAkk;
        double s = 0;
        for (int i = k; i < nr; i++) {
          s += *pp * pp[j - k];
          pp += nc;
        }
        const double tau = s / A1[k];
        pp = ppAkk;
        for (int i = k; i < nr; i++) {
          pp[j - k] -= tau * *pp;
          pp += nc;
        }
      }
      ppAkk += nc + 1;
    }
    double *ppAjj = pA, *pb = b;
    for (int j = 0; j < nc; j++) {
      double *ppAij = ppAjj, tau = 0;
      for (int i = j; i < nr; i++) {
        tau += *ppAij * pb[i];
        ppAij += nc;
      }
      tau /= A1[j];
      ppAij = ppAjj;
      for (int i = j; i < nr; i++) {
        pb[i] -= tau * *ppAij;
        ppAij += nc;
      }
      ppAjj += nc + 1;
    }
    X[nc - 1] = pb[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
      double *ppAij = pA + i * nc + (i + 1), s = 0;
      for (int j = i + 1; j < nc; j++) {
        s += *ppAij * X[j];
        ppAij++;
      }
      X[i] = (pb[i] - s) / A2[i];
    }
  }
  static void gauss_newton(const double* L, const double* rho, double betas[4]) {
    for (int k = 0; k < 5; k++) {
      double A[24], b[6], x[4] = {0, 0, 0, 0};
      for (int i = 0; i < 6; i++) {
        const double* r = L + i * 10;
        double* a = A + i * 4;
        a[0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
        a[1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
        a[2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
        a[3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
        b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] +
                         r[2] * betas[1] * betas[1] + r[3] * betas[0] * betas[2] +
                         r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                         r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] +
                         r[8] * betas[2] * betas[3] + r[9] * betas[3] * betas[3]);
      }
      qr_solve(A, b, x);
      for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
  }
  void compute_pose(double R[3][3], double t[3]) {
    choose_control_points();
    compute_barycentric_coordinates();
    double mtm[144] = {0};
    for (int i = 0; i < n; i++) {
      const double* as = &alphas[4 * i];
      const double u = us[2 * i], v = us[2 * i + 1];
      double M1[12], M2[12];
      for (int k = 0; k < 4; k++) {
        M1[3 * k] = as[k] * fu;
        M1[3 * k + 1] = 0.0;
        M1[3 * k + 2] = as[k] * (uc - u);
        M2[3 * k] = 0.0;
        M2[3 * k + 1] = as[k] * fv;
        M2[3 * k + 2] = as[k] * (vc - v);
      }
      for (int a = 0; a < 12; a++)
        for (int b = 0; b < 12; b++) mtm[12 * a + b] += M1[a] * M1[b] + M2[a] * M2[b];
    }
    double ut[144];
    jacobi_eig12(mtm, ut);
    double L[60], rho[6];
    compute_L_6x10(ut, L);
    compute_rho(rho);
    double Betas[4][4], rep[4], Rs[4][3][3], ts[4][3];
    betas_approx_1(L, rho, Betas[1]);
    gauss_newton(L, rho, Betas[1]);
    rep[1] = compute_R_and_t(ut, Betas[1], Rs[1], ts[1]);
    betas_approx_2(L, rho, Betas[2]);
    gauss_newton(L, rho, Betas[2]);
    rep[2] = compute_R_and_t(ut, Betas[2], Rs[2], ts[2]);
    betas_approx_3(L, rho, Betas[3]);
    gauss_newton(L, rho, Betas[3]);
    rep[3] = compute_R_and_t(ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (rep[2] < rep[1]) N = 2;
    if (rep[3] < rep[N]) N = 3;
    memcpy(R, Rs[N], sizeof(double) * 9);
    memcpy(t, ts[N], sizeof(double) * 3);
  }
};
}  // namespace

// solvePnP(..., SOLVEPNP_EPNP): undistortPoints (zero distortion, float output) then epnp with
// pixel coordinates re-formed as x * fu + uc.
void epnp_pose(const float* pts3, const float* pts2, const int* sel, int n, double fx, double fy,
               double cx, double cy, double R[9], double t[3], bool f64_points) {
  EPnP e;
  e.n = n;
  e.fu = fx;
  e.fv = fy;
  e.uc = cx;
  e.vc = cy;
  e.pws.resize(3 * n);
  e.us.resize(2 * n);
  e.alphas.resize(4 * n);
  e.pcs.resize(3 * n);
  const double ifx = 1. / fx, ify = 1. / fy;
  for (int i = 0; i < n; i++) {
    const int j = sel ? sel[i] : i;
    for (int k = 0; k < 3; k++) e.pws[3 * i + k] = pts3[3 * j + k];
    // undistortPoints keeps the input depth: CV_32F points round the normalised coordinates
    // to float, the CV_64F refit input (solvePnPRansac's convertTo) keeps them in double
    double xn = ((double)pts2[2 * j] - cx) * ifx;
    double yn = ((double)pts2[2 * j + 1] - cy) * ify;
    if (!f64_points) {
      xn = (double)(float)xn;
      yn = (double)(float)yn;
    }
    e.us[2 * i] = xn * fx + cx;
    e.us[2 * i + 1] = yn * fy + cy;
  }
  double Rm[3][3];
  e.compute_pose(Rm, t);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[3 * r + c] = Rm[r][c];
}

// EPnP as PnPsolver uses it (add_correspondence with the pixel coordinates as they are).
void epnp_pose_raw(const float* pts3, const float* pts2, const int* sel, int n, double fx,
                   double fy, double cx, double cy, double R[9], double t[3]) {
  EPnP e;
  e.n = n;
  e.fu = fx;
  e.fv = fy;
  e.uc = cx;
  e.vc = cy;
  e.pws.resize(3 * n);
  e.us.resize(2 * n);
  e.alphas.resize(4 * n);
  e.pcs.resize(3 * n);
  for (int i = 0; i < n; i++) {
    const int j = sel ? sel[i] : i;
    for (int k = 0; k < 3; k++) e.pws[3 * i + k] = pts3[3 * j + k];
    e.us[2 * i] = pts2[2 * j];
    e.us[2 * i + 1] = pts2[2 * j + 1];
  }
  double Rm[3][3];
  e.compute_pose(Rm, t);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[3 * r + c] = Rm[r][c];
}

// cv::Rodrigues matrix -> vector (orthonormalisation by SVD omitted: EPnP's R is orthonormal to
// rounding, the effect is below 1e-15).
void rodrigues_r2v(const double R[9], double r[3]) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  const double theta = std::acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      rx = ry = rz = 0;
    } else {
      double tt = (R[0] + 1) * 0.5;
      rx = std::sqrt(std::max(tt, 0.));
      tt = (R[4] + 1) * 0.5;
      ry = std::sqrt(std::max(tt, 0.)) * (R[1] < 0 ? -1. : 1.);
      tt = (R[8] + 1) * 0.5;
      rz = std::sqrt(std::max(tt, 0.)) * (R[2] < 0 ? -1. : 1.);
      if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0))
        rz = -rz;
      const double nr = std::sqrt(rx * rx + ry * ry + rz * rz);
      rx *= theta / nr;
      ry *= theta / nr;
      rz *= theta / nr;
    }
  } else {
    double vth = 1 / (2 * s);
    vth *= theta;
    rx *= vth;
    ry *= vth;
    rz *= vth;
  }
  r[0] = rx;
  r[1] = ry;
  r[2] = rz;
}

void rodrigues_v2r(const double rv[3], double R[9]) {
  const double theta = std::sqrt(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]);
  if (theta < DBL_EPSILON) {
    for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c;
  const double itheta = theta ? 1. / theta : 0.;
  const double x = rv[0] * itheta, y = rv[1] * itheta, z = rv[2] * itheta;
  const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  for (int i = 0; i < 9; i++) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

// ---------------------------------------------------------------- RANSAC (ptsetreg.cpp)
static inline unsigned rng_next_u(uint64_t& state) {
  state = (uint64_t)(unsigned)state * 4164903690ULL + (unsigned)(state >> 32);
  return (unsigned)state;
}

void ransac_subsets(int count, int model_points, int iters, std::vector<int>& idx) {
  uint64_t state = 0xFFFFFFFFFFFFFFFFULL;  // RNG((uint64)-1)
  idx.assign((size_t)iters * model_points, 0);
  for (int it = 0; it < iters; it++) {
    int* cur = &idx[(size_t)it * model_points];
    for (int i = 0; i < model_points; i++) {
      for (;;) {
        const int v = (int)(rng_next_u(state) % (unsigned)count);
        cur[i] = v;
        int j = 0;
        for (; j < i; j++)
          if (v == cur[j]) break;
        if (j == i) break;
      }
    }
  }
}

static int ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = std::max(p, 0.);
  p = std::min(p, 1.);
  ep = std::max(ep, 0.);
  ep = std::min(ep, 1.);
  double num = std::max(1. - p, DBL_MIN);
  double denom = 1. - std::pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = std::log(num);
  denom = std::log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

// PnPRansacCallback::computeError + findInliers for the model (rvec, tvec).
static int count_inliers(const float* pts3, const float* pts2, int n, const double rv[3],
                         const double tv[3], double fx, double fy, double cx, double cy,
                         double thresh, std::vector<uint8_t>* mask) {
  double R[9];
  rodrigues_v2r(rv, R);
  const float t = (float)(thresh * thresh);
  int nz = 0;
  if (mask) mask->assign(n, 0);
  for (int i = 0; i < n; i++) {
    const double X = pts3[3 * i], Y = pts3[3 * i + 1], Z = pts3[3 * i + 2];
    double x = R[0] * X + R[1] * Y + R[2] * Z + tv[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + tv[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + tv[2];
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    const float pu = (float)(x * fx + cx), pv = (float)(y * fy + cy);
    const float du = pts2[2 * i] - pu, dv = pts2[2 * i + 1] - pv;
    const float err = du * du + dv * dv;
    const int f = err <= t;
    if (mask) (*mask)[i] = (uint8_t)f;
    nz += f;
  }
  return nz;
}

PnPResult pnp_ransac(const float* pts3, const float* pts2, int n, double fx, double fy, double cx,
                     double cy, int max_iters, double reproj, double confidence) {
  PnPResult res;
  const int model_points = 5;
  if (n < model_points) return res;
  std::vector<int> subsets;
  ransac_subsets(n, model_points, max_iters, subsets);
  int niters = std::max(max_iters, 1), maxGood = 0;
  double bestR[9], bestT[3], bestRv[3];
  std::vector<uint8_t> mask, bestMask;
  if (n == model_points) {  // ptsetreg.cpp run(): one kernel call on all points, mask all ones
    niters = 0;
    bestMask.assign(n, 1);
    maxGood = n;
    res.best_iter = 0;
  }
  for (int it = 0; it < niters; it++) {
    double R[9], t[3], rv[3];
    epnp_pose(pts3, pts2, &subsets[(size_t)it * model_points], model_points, fx, fy, cx, cy, R, t,
              false);
    rodrigues_r2v(R, rv);
    const int good = count_inliers(pts3, pts2, n, rv, t, fx, fy, cx, cy, reproj, &mask);
    res.iterations = it + 1;
    if (good > std::max(maxGood, model_points - 1)) {
      bestMask = mask;
      memcpy(bestRv, rv, sizeof(rv));
      memcpy(bestT, t, sizeof(t));
      maxGood = good;
      res.best_iter = it;
      niters = ransac_update_num_iters(confidence, (double)(n - good) / n, model_points, niters);
    }
  }
  (void)bestR;
  if (maxGood <= 0) return res;
  // refit with EPnP on all RANSAC inliers; `inliers` = the best RANSAC mask (Appendix A.9)
  std::vector<int> sel;
  for (int i = 0; i < n; i++)
    if (bestMask[i]) sel.push_back(i);
  double R[9], t[3], rv[3];
  epnp_pose(pts3, pts2, sel.data(), (int)sel.size(), fx, fy, cx, cy, R, t, true);
  rodrigues_r2v(R, rv);
  rodrigues_v2r(rv, res.R);  // GetInitModelObj: cv::Rodrigues(Rvec, d) (Tracking.cc:4367)
  memcpy(res.t, t, sizeof(t));
  res.inliers = sel;
  res.ok = true;
  return res;
}

// ---------------------------------------------------------------- D6: PnPsolver (P4P RANSAC)
// glibc rand() (random_r TYPE_3: additive feedback r[i] = r[i-3] + r[i-31], seeded by srand) --
// the stream DUtils::Random::RandomInt draws from (Thirdparty/DBoW2/DUtils/Random.cpp:47-50).
GlibcRand::GlibcRand(unsigned seed) {
  if (seed == 0) seed = 1;
  r.resize(34);
  r[0] = (int32_t)seed;
  for (int i = 1; i < 31; i++) {
    const int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
    int64_t word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r[i] = (int32_t)word;
  }
  for (int i = 31; i < 34; i++) r[i] = r[i - 31];
  for (int i = 0; i < 310; i++) next();
}

int GlibcRand::next() {
  const size_t i = r.size();
  const uint32_t v = (uint32_t)r[i - 31] + (uint32_t)r[i - 3];
  r.push_back((int32_t)v);
  if (r.size() > 4096) r.erase(r.begin(), r.end() - 34);
  return (int)(v >> 1);
}

int GlibcRand::random_int(int min, int max) {  // DUtils::Random::RandomInt
  const int d = max - min + 1;
  return int(((double)next() / ((double)2147483647 + 1.0)) * d) + min;
}

// PnPsolver::CheckInliers (PnPsolver.cc:310-337)
static int p4p_check(const float* pts3, const float* pts2, const std::vector<float>& maxErr, int n,
                     const double R[9], const double t[3], double fu, double fv, double uc,
                     double vc, std::vector<uint8_t>& mask) {
  int good = 0;
  mask.assign(n, 0);
  for (int i = 0; i < n; i++) {
    const double X = pts3[3 * i], Y = pts3[3 * i + 1], Z = pts3[3 * i + 2];
    const float Xc = (float)(R[0] * X + R[1] * Y + R[2] * Z + t[0]);
    const float Yc = (float)(R[3] * X + R[4] * Y + R[5] * Z + t[1]);
    const float invZc = (float)(1 / (R[6] * X + R[7] * Y + R[8] * Z + t[2]));
    const double ue = uc + fu * Xc * invZc;
    const double ve = vc + fv * Yc * invZc;
    const float distX = (float)(pts2[2 * i] - ue), distY = (float)(pts2[2 * i + 1] - ve);
    const float error2 = distX * distX + distY * distY;
    if (error2 < maxErr[i]) {
      mask[i] = 1;
      good++;
    }
  }
  return good;
}

static void to_Tcw(const double R[9], const double t[3], float T[16]) {
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) T[4 * r + c] = r == c ? 1.f : 0.f;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[3 * r + c];
    T[4 * r + 3] = (float)t[r];
  }
}

// SetRansacParameters (PnPsolver.cc:119-152) + iterate (PnPsolver.cc:160-264) + Refine
// (PnPsolver.cc:266-308), state carried in *st.
P4PResult pnpsolver_iterate(const float* pts3, const float* pts2, const float* sigma2, int N,
                            double fu, double fv, double uc, double vc, double probability,
                            int minInliers, int maxIterations, int minSet, float epsilon,
                            float th2, const int* randi, int nIterations, P4PState* st) {
  P4PResult res;
  float eps = epsilon;
  int nMinInliers = (int)(N * eps);
  if (nMinInliers < minInliers) nMinInliers = minInliers;
  if (nMinInliers < minSet) nMinInliers = minSet;
  const int minInl = nMinInliers;
  if (N > 0 && eps < (float)minInl / N) eps = (float)minInl / N;
  int nIt;
  if (minInl == N)
    nIt = 1;
  else
    nIt = (int)std::ceil(std::log(1 - probability) / std::log(1 - std::pow(eps, 3)));
  const int maxIts = std::max(1, std::min(nIt, maxIterations));
  std::vector<float> maxErr(N);
  for (int i = 0; i < N; i++) maxErr[i] = sigma2[i] * th2;
  if (N < minInl) {
    res.no_more = true;
    return res;
  }
  if ((int)st->best_mask.size() != N) st->best_mask.assign(N, 0);
  int cur = 0, k = 0;
  std::vector<uint8_t> mask;
  while (st->iterations < maxIts || cur < nIterations) {
    cur++;
    st->iterations++;
    std::vector<int> avail(N);
    for (int i = 0; i < N; i++) avail[i] = i;
    int sel[4];
    for (int j = 0; j < 4; j++) {
      const int r = randi[4 * k + j];
      sel[j] = avail[r];
      avail[r] = avail.back();
      avail.pop_back();
    }
    k++;
    double R[9], t[3];
    epnp_pose_raw(pts3, pts2, sel, 4, fu, fv, uc, vc, R, t);
    const int good = p4p_check(pts3, pts2, maxErr, N, R, t, fu, fv, uc, vc, mask);
    if (good >= minInl) {
      if (good > st->best_inliers) {
        st->best_mask = mask;
        st->best_inliers = good;
        to_Tcw(R, t, st->best_Tcw);
      }
      // Refine: EPnP over the best inliers, CheckInliers
      std::vector<int> idx;
      for (int i = 0; i < N; i++)
        if (st->best_mask[i]) idx.push_back(i);
      double Rr[9], tr[3];
      epnp_pose_raw(pts3, pts2, idx.data(), (int)idx.size(), fu, fv, uc, vc, Rr, tr);
      std::vector<uint8_t> rmask;
      const int rgood = p4p_check(pts3, pts2, maxErr, N, Rr, tr, fu, fv, uc, vc, rmask);
      if (rgood > minInl) {
        res.found = true;
        res.n_inliers = rgood;
        res.mask = rmask;
        to_Tcw(Rr, tr, res.Tcw);
        return res;
      }
    }
  }
  if (st->iterations >= maxIts) {
    res.no_more = true;
    if (st->best_inliers >= minInl) {
      res.found = true;
      res.n_inliers = st->best_inliers;
      res.mask = st->best_mask;
      memcpy(res.Tcw, st->best_Tcw, sizeof(res.Tcw));
    }
  }
  return res;
}

}  // namespace oracle
