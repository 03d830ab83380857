// multimot_track_amd/csrc/mmt_pnp.hip -- object-motion initialiser D5 on the GPU:
// cv::solvePnPRansac(pre_3d, cur_2d, K, 0, ..., 500, 0.3, 0.98, inliers, SOLVEPNP_AP3P) as
// called by Tracking::GetInitModelObj (reference src/Tracking.cc:4324-4443).
//
//   k_pnp_gather   pre_3d = UnprojectStereoObject(last sample), cur_2d = current sample
//   k_pnp_hyp      one lane per RANSAC hypothesis: 5-point EPnP (PnPsolver.cc:342-1022 lineage)
//                  on the subset drawn by RNG((uint64)-1) (precomputed on the host: the draw
//                  sequence depends only on the point count), then Rodrigues -> model
//   k_pnp_score    one workgroup per hypothesis: projectPoints + squared-error test, inlier
//                  count by ballot/popcount, inlier bit mask
//   k_pnp_select   replay of RANSACPointSetRegistrator::run's best-so-far / niters logic
//   k_pnp_refit    one workgroup per object: EPnP over all RANSAC inliers (reductions over the
//                  points, 12x12 eigen-solve and beta estimation in one lane)
//   k_mm_inliers   motion-model check (Tracking.cc:4375-4405)
// The dense algebra (cyclic/one-sided Jacobi) follows oracle/pnp_ref.cpp operation for
// operation so hypothesis models agree to the last bit with the CPU checker.

#include <hip/hip_runtime.h>

#include <cfloat>

#include "mmt_internal.h"
#include "mmt_devmath.h"
#include "mmt_pnp.h"

namespace mmt {

// ---------------------------------------------------------------- dense helpers (one lane)
__device__ void d_jacobi_eig_sym(int n, double* A, double* d, double* vt, double* V, int* ord) {
  for (int i = 0; i < n * n; i++) V[i] = 0.0;
  for (int i = 0; i < n; i++) V[i * n + i] = 1.0;
  for (int sweep = 0; sweep < 100; sweep++) {
    double off = 0;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) off += A[p * n + q] * A[p * n + q];
    if (off < 1e-300) break;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) {
        const double apq = A[p * n + q];
        if (fabs(apq) < 1e-300) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double theta = (aqq - app) / (2 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
        const double c = 1 / sqrt(t * t + 1), s = t * c;
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
  // stable sort by descending eigenvalue (insertion sort == std::stable_sort order)
  for (int i = 0; i < n; i++) ord[i] = i;
  for (int i = 1; i < n; i++) {
    const int v = ord[i];
    int j = i - 1;
    while (j >= 0 && A[ord[j] * n + ord[j]] < A[v * n + v]) {
      ord[j + 1] = ord[j];
      j--;
    }
    ord[j + 1] = v;
  }
  for (int r = 0; r < n; r++) {
    d[r] = A[ord[r] * n + ord[r]];
    for (int k = 0; k < n; k++) vt[r * n + k] = V[k * n + ord[r]];
  }
}

// thin SVD (m >= n) by one-sided Jacobi; A is overwritten
__device__ void d_jacobi_svd(int m, int n, double* A, double* U, double* w, double* V) {
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
        if (fabs(g) <= 1e-15 * sqrt(a * b) || g == 0) continue;
        changed = true;
        const double zeta = (b - a) / (2 * g);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), s = c * t;
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
    w[j] = sqrt(s);
    for (int k = 0; k < m; k++) U[k * n + j] = w[j] > 0 ? A[k * n + j] / w[j] : 0.0;
  }
}

__device__ void d_svd_solve(int m, int n, const double* Ain, const double* b, double* x) {
  double A[30], U[30], w[5], V[25];
  for (int i = 0; i < m * n; i++) A[i] = Ain[i];
  d_jacobi_svd(m, n, A, U, w, V);
  double wmax = 0;
  for (int j = 0; j < n; j++) wmax = fmax(wmax, w[j]);
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

__device__ __forceinline__ double d_dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ double d_dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

__device__ void d_compute_L_6x10(const double* ut, double* l) {
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
    row[0] = d_dot3(dv[0][i], dv[0][i]);
    row[1] = 2.0f * d_dot3(dv[0][i], dv[1][i]);
    row[2] = d_dot3(dv[1][i], dv[1][i]);
    row[3] = 2.0f * d_dot3(dv[0][i], dv[2][i]);
    row[4] = 2.0f * d_dot3(dv[1][i], dv[2][i]);
    row[5] = d_dot3(dv[2][i], dv[2][i]);
    row[6] = 2.0f * d_dot3(dv[0][i], dv[3][i]);
    row[7] = 2.0f * d_dot3(dv[1][i], dv[3][i]);
    row[8] = 2.0f * d_dot3(dv[2][i], dv[3][i]);
    row[9] = d_dot3(dv[3][i], dv[3][i]);
  }
}

__device__ void d_betas(int which, const double* L, const double* rho, double* betas) {
  if (which == 1) {
    double A[24], b4[4];
    for (int i = 0; i < 6; i++) {
      A[4 * i] = L[10 * i];
      A[4 * i + 1] = L[10 * i + 1];
      A[4 * i + 2] = L[10 * i + 3];
      A[4 * i + 3] = L[10 * i + 6];
    }
    d_svd_solve(6, 4, A, rho, b4);
    if (b4[0] < 0) {
      betas[0] = sqrt(-b4[0]);
      betas[1] = -b4[1] / betas[0];
      betas[2] = -b4[2] / betas[0];
      betas[3] = -b4[3] / betas[0];
    } else {
      betas[0] = sqrt(b4[0]);
      betas[1] = b4[1] / betas[0];
      betas[2] = b4[2] / betas[0];
      betas[3] = b4[3] / betas[0];
    }
  } else if (which == 2) {
    double A[18], b3[3];
    for (int i = 0; i < 6; i++)
      for (int k = 0; k < 3; k++) A[3 * i + k] = L[10 * i + k];
    d_svd_solve(6, 3, A, rho, b3);
    if (b3[0] < 0) {
      betas[0] = sqrt(-b3[0]);
      betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
    } else {
      betas[0] = sqrt(b3[0]);
      betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
  } else {
    double A[30], b5[5];
    for (int i = 0; i < 6; i++)
      for (int k = 0; k < 5; k++) A[5 * i + k] = L[10 * i + k];
    d_svd_solve(6, 5, A, rho, b5);
    if (b5[0] < 0) {
      betas[0] = sqrt(-b5[0]);
      betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
    } else {
      betas[0] = sqrt(b5[0]);
      betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
  }
}

__device__ void d_qr_solve(double* A, double* b, double* X) {  // 6 x 4 (PnPsolver.cc:840-950)
  const int nr = 6, nc = 4;
  double A1[6], A2[6];
  double *pA = A, *ppAkk = pA;
  for (int k = 0; k < nc; k++) {
    double *ppAik = ppAkk, eta = fabs(*ppAik);
    for (int i = k + 1; i < nr; i++) {
      double elt = fabs(*ppAik);
      if (eta < elt) eta = elt;
      ppAik += nc;
    }
    if (eta == 0) return;
    double sum = 0.0, inv_eta = 1. / eta;
    ppAik = ppAkk;
    for (int i = k; i < nr; i++) {
      *ppAik *= inv_eta;
      sum += *ppAik * *ppAik;
      ppAik += nc;
    }
    double sigma = sqrt(sum);
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

__device__ void d_gauss_newton(const double* L, const double* rho, double* betas) {
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
    d_qr_solve(A, b, x);
    for (int i = 0; i < 4; i++) betas[i] += x[i];
  }
}

__device__ void d_rodrigues_r2v(const double R[9], double r[3]) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  const double theta = acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      rx = ry = rz = 0;
    } else {
      double tt = (R[0] + 1) * 0.5;
      rx = sqrt(fmax(tt, 0.));
      tt = (R[4] + 1) * 0.5;
      ry = sqrt(fmax(tt, 0.)) * (R[1] < 0 ? -1. : 1.);
      tt = (R[8] + 1) * 0.5;
      rz = sqrt(fmax(tt, 0.)) * (R[2] < 0 ? -1. : 1.);
      if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      const double nr = sqrt(rx * rx + ry * ry + rz * rz);
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

__device__ void d_rodrigues_v2r(const double rv[3], double R[9]) {
  const double theta = sqrt(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]);
  if (theta < DBL_EPSILON) {
    for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double c = cos(theta), s = sin(theta), c1 = 1. - c;
  const double itheta = theta ? 1. / theta : 0.;
  const double x = rv[0] * itheta, y = rv[1] * itheta, z = rv[2] * itheta;
  const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  for (int i = 0; i < 9; i++) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

// ---------------------------------------------------------------- EPnP over a point set
// Points are accessed through `pw(i)`/`us(i)` loaders so the same code serves the 5-point
// hypotheses (one lane) and, via reductions, the refit.
struct EPnPSmall {  // n <= 5, all in lane-private storage
  int n;
  double fu, fv, uc, vc;
  double pws[15], us[10], alphas[20], pcs[15];
  double cws[4][3], ccs[4][3];

  __device__ void choose_control_points() {
    cws[0][0] = cws[0][1] = cws[0][2] = 0;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) cws[0][j] += pws[3 * i + j];
    for (int j = 0; j < 3; j++) cws[0][j] /= n;
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
      double p[3];
      for (int j = 0; j < 3; j++) p[j] = pws[3 * i + j] - cws[0][j];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) m[3 * a + b] += p[a] * p[b];
    }
    double dc[3], uct[9], V[9];
    int ord[3];
    d_jacobi_eig_sym(3, m, dc, uct, V, ord);
    for (int i = 1; i < 4; i++) {
      const double k = sqrt(fmax(dc[i - 1], 0.0) / n);
      for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
    }
  }
  __device__ void compute_barycentric() {
    double cc[9];
    for (int i = 0; i < 3; i++)
      for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    double U[9], w[3], V[9], ci[9];
    d_jacobi_svd(3, 3, cc, U, w, V);
    const double wmax = fmax(w[0], fmax(w[1], w[2]));
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
  __device__ double compute_R_and_t(const double* ut, const double* betas, double R[3][3],
                                    double t[3]) {
    for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
    for (int i = 0; i < 4; i++) {
      const double* v = ut + 12 * (11 - i);
      for (int j = 0; j < 4; j++)
        for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
    }
    for (int i = 0; i < n; i++) {
      const double* a = &alphas[4 * i];
      for (int j = 0; j < 3; j++)
        pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }
    if (pcs[2] < 0.0) {
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
      for (int i = 0; i < 3 * n; i++) pcs[i] = -pcs[i];
    }
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
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
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
    d_jacobi_svd(3, 3, abt, U, w, V);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i][j] = d_dot3(U + 3 * i, V + 3 * j);
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] +
                       R[0][2] * R[1][0] * R[2][1] - R[0][2] * R[1][1] * R[2][0] -
                       R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) {
      R[2][0] = -R[2][0];
      R[2][1] = -R[2][1];
      R[2][2] = -R[2][2];
    }
    t[0] = pc0[0] - d_dot3(R[0], pw0);
    t[1] = pc0[1] - d_dot3(R[1], pw0);
    t[2] = pc0[2] - d_dot3(R[2], pw0);
    double sum2 = 0.0;
    for (int i = 0; i < n; i++) {
      const double* pw = &pws[3 * i];
      const double Xc = d_dot3(R[0], pw) + t[0], Yc = d_dot3(R[1], pw) + t[1];
      const double inv_Zc = 1.0 / (d_dot3(R[2], pw) + t[2]);
      const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
      const double u = us[2 * i], v = us[2 * i + 1];
      sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / n;
  }
};

// ---------------------------------------------------------------- kernels
__global__ __launch_bounds__(256) void k_pnp_gather(PnPObject* objs) {
  PnPObject& o = objs[blockIdx.x];
  const int n = *o.n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int s = o.members[i];
    const float2 kl = o.last_keys[s];
    const float z = o.last_depth[s];
    const float* T = o.Tlast;
    const float invfx = 1.0f / o.fx, invfy = 1.0f / o.fy;
    const float x = (kl.x - o.cx) * z * invfx, y = (kl.y - o.cy) * z * invfy;
    const float xc[3] = {x, y, z};
    for (int r = 0; r < 3; r++) {
      double s1 = 0, s2 = 0;
      for (int k = 0; k < 3; k++) {
        s1 += (double)T[4 * k + r] * (double)T[4 * k + 3];
        s2 += (double)T[4 * k + r] * (double)xc[k];
      }
      o.pts3[3 * i + r] = (float)s2 + (float)(-s1);
    }
    o.pts2[i] = o.cur_keys[s];
  }
}

// one lane per (object, hypothesis)
__global__ __launch_bounds__(64) void k_pnp_hyp(PnPObject* objs, int max_iters) {
  const int h = blockIdx.x * 64 + threadIdx.x;
  PnPObject& o = objs[blockIdx.y];
  const int n = *o.n;
  if (h >= max_iters || n < 5) return;
  EPnPSmall e;
  e.n = 5;
  e.fu = o.fx;
  e.fv = o.fy;
  e.uc = o.cx;
  e.vc = o.cy;
  const double ifx = 1. / (double)o.fx, ify = 1. / (double)o.fy;
  const int* sub = o.subsets + 5 * h;
  for (int i = 0; i < 5; i++) {
    const int j = n == 5 ? i : sub[i];  // count == modelPoints: the kernel runs on all points
    for (int k = 0; k < 3; k++) e.pws[3 * i + k] = o.pts3[3 * j + k];
    const float2 p = o.pts2[j];
    const float xn = (float)(((double)p.x - (double)o.cx) * ifx);
    const float yn = (float)(((double)p.y - (double)o.cy) * ify);
    e.us[2 * i] = (double)xn * (double)o.fx + (double)o.cx;
    e.us[2 * i + 1] = (double)yn * (double)o.fy + (double)o.cy;
  }
  e.choose_control_points();
  e.compute_barycentric();
  double mtm[144];
  for (int i = 0; i < 144; i++) mtm[i] = 0;
  for (int i = 0; i < 5; i++) {
    const double* as = &e.alphas[4 * i];
    const double u = e.us[2 * i], v = e.us[2 * i + 1];
    double M1[12], M2[12];
    for (int k = 0; k < 4; k++) {
      M1[3 * k] = as[k] * e.fu;
      M1[3 * k + 1] = 0.0;
      M1[3 * k + 2] = as[k] * (e.uc - u);
      M2[3 * k] = 0.0;
      M2[3 * k + 1] = as[k] * e.fv;
      M2[3 * k + 2] = as[k] * (e.vc - v);
    }
    for (int a = 0; a < 12; a++)
      for (int b = 0; b < 12; b++) mtm[12 * a + b] += M1[a] * M1[b] + M2[a] * M2[b];
  }
  double d[12], ut[144], V[144];
  int ord[12];
  d_jacobi_eig_sym(12, mtm, d, ut, V, ord);
  double L[60], rho[6];
  d_compute_L_6x10(ut, L);
  rho[0] = d_dist2(e.cws[0], e.cws[1]);
  rho[1] = d_dist2(e.cws[0], e.cws[2]);
  rho[2] = d_dist2(e.cws[0], e.cws[3]);
  rho[3] = d_dist2(e.cws[1], e.cws[2]);
  rho[4] = d_dist2(e.cws[1], e.cws[3]);
  rho[5] = d_dist2(e.cws[2], e.cws[3]);
  double best_err = 0, bR[3][3], bt[3];
  for (int which = 1; which <= 3; which++) {
    double betas[4], R[3][3], t[3];
    d_betas(which, L, rho, betas);
    d_gauss_newton(L, rho, betas);
    const double err = e.compute_R_and_t(ut, betas, R, t);
    if (which == 1 || err < best_err) {  // rep_errors[2] < [1]; [3] < [N]
      best_err = err;
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) bR[r][c] = R[r][c];
        bt[r] = t[r];
      }
    }
  }
  double Rf[9], rv[3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Rf[3 * r + c] = bR[r][c];
  d_rodrigues_r2v(Rf, rv);
  double* m = o.models + 6 * h;
  m[0] = rv[0];
  m[1] = rv[1];
  m[2] = rv[2];
  m[3] = bt[0];
  m[4] = bt[1];
  m[5] = bt[2];
}

// one workgroup per (hypothesis, object): inlier count + mask (PnPRansacCallback::computeError,
// RANSACPointSetRegistrator::findInliers with t = (float)(0.3 * 0.3))
__global__ __launch_bounds__(256) void k_pnp_score(PnPObject* objs, int max_iters) {
  __shared__ double sR[9];
  __shared__ int s_w[4];
  const int h = blockIdx.x;
  PnPObject& o = objs[blockIdx.y];
  const int n = *o.n;
  if (h >= max_iters || n < 5) return;
  const double* m = o.models + 6 * h;
  if (threadIdx.x == 0) d_rodrigues_v2r(m, sR);
  __syncthreads();
  const double tx = m[3], ty = m[4], tz = m[5];
  const float thr = (float)(o.reproj * o.reproj);
  const int words = (n + 63) / 64;
  int good = 0;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    bool in = false;
    if (i < n) {
      const double X = o.pts3[3 * i], Y = o.pts3[3 * i + 1], Z = o.pts3[3 * i + 2];
      double x = sR[0] * X + sR[1] * Y + sR[2] * Z + tx;
      double y = sR[3] * X + sR[4] * Y + sR[5] * Z + ty;
      double z = sR[6] * X + sR[7] * Y + sR[8] * Z + tz;
      z = z ? 1. / z : 1;
      x *= z;
      y *= z;
      const float pu = (float)(x * (double)o.fx + (double)o.cx);
      const float pv = (float)(y * (double)o.fy + (double)o.cy);
      const float2 q = o.pts2[i];
      const float du = q.x - pu, dv = q.y - pv;
      // count == modelPoints: run() returns the model with every point marked inlier
      in = n == 5 || (du * du + dv * dv) <= thr;
    }
    const unsigned long long bal = __ballot(in);
    if ((threadIdx.x & 63) == 0 && i0 + (threadIdx.x & ~63) < n)
      o.masks[(size_t)h * o.mask_words + (i0 + (threadIdx.x & ~63)) / 64] = bal;
    good += in ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) good += __shfl_xor(good, off, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = good;
  __syncthreads();
  if (threadIdx.x == 0) o.good[h] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  (void)words;
}

__device__ int d_update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = fmax(p, 0.);
  p = fmin(p, 1.);
  ep = fmax(ep, 0.);
  ep = fmin(ep, 1.);
  double num = fmax(1. - p, DBL_MIN);
  double denom = 1. - pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

__global__ void k_pnp_select(PnPObject* objs, int max_iters) {
  PnPObject& o = objs[blockIdx.x];
  if (threadIdx.x != 0) return;
  const int n = *o.n;
  int niters = max_iters, maxGood = 0, best = -1, it = 0;
  if (n == 5) {  // RANSACPointSetRegistrator::run: count == modelPoints, no iterations
    best = 0;
    maxGood = 5;
  } else if (n > 5) {
    for (it = 0; it < niters; it++) {
      const int good = o.good[it];
      if (good > max(maxGood, 4)) {
        best = it;
        maxGood = good;
        niters = d_update_num_iters(o.confidence, (double)(n - good) / n, 5, niters);
      }
    }
  }
  o.result[0] = best;
  o.result[1] = maxGood;
  o.result[2] = it;
}

// one workgroup per object: EPnP refit over the best hypothesis' inliers; also emits the
// inlier index list (ascending) used as ObjIdTest_in
__global__ __launch_bounds__(256) void k_pnp_refit(PnPObject* objs) {
  __shared__ double s_red[4 * 80];
  __shared__ double s_sum[80];
  __shared__ double s_cws[4][3], s_ci[9], s_ut[144], s_L[60], s_rho[6], s_ccs[4][3];
  __shared__ double s_R[3][3], s_t[3], s_pc0[3], s_pw0[3], s_bestR[9], s_bestT[3], s_best;
  __shared__ int s_w[4], s_n;
  PnPObject& o = objs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int best = o.result[0];
  if (best < 0) {
    if (tid == 0) {
      o.result[3] = 0;
      for (int i = 0; i < 9; i++) o.Rt[i] = (i % 4 == 0) ? 1.0 : 0.0;
      o.Rt[9] = o.Rt[10] = o.Rt[11] = 0.0;
    }
    return;
  }
  const int n = *o.n;
  const unsigned long long* mask = o.masks + (size_t)best * o.mask_words;
  // ordered inlier list
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + tid;
    const bool in = i < n && ((mask[i >> 6] >> (i & 63)) & 1ull);
    const unsigned long long bal = __ballot(in);
    if (lane == 0) s_w[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) off += s_w[w];
      tot += s_w[w];
    }
    if (in) o.inliers[base + off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    base += tot;
    __syncthreads();
  }
  if (tid == 0) s_n = base;
  __syncthreads();
  const int ni = s_n;
  const double fu = o.fx, fv = o.fy, uc = o.cx, vc = o.cy;
  const double ifx = 1. / fu, ify = 1. / fv;
  auto pw = [&](int k, double* p) {
    const int j = o.inliers[k];
    p[0] = o.pts3[3 * j];
    p[1] = o.pts3[3 * j + 1];
    p[2] = o.pts3[3 * j + 2];
  };
  auto usp = [&](int k, double& u, double& v) {
    // solvePnPRansac converts the inliers to CV_64F before the refit, so undistortPoints
    // keeps the normalised coordinates in double here (the hypotheses round them to float)
    const float2 q = o.pts2[o.inliers[k]];
    u = (((double)q.x - uc) * ifx) * fu + uc;
    v = (((double)q.y - vc) * ify) * fv + vc;
  };
  // control points: centroid, then PCA of the centred points
  {
    double v[3] = {0, 0, 0};
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3];
      pw(k, p);
      v[0] += p[0];
      v[1] += p[1];
      v[2] += p[2];
    }
    wg_sum<3>(v, s_red, s_sum);
    if (tid == 0)
      for (int j = 0; j < 3; j++) s_cws[0][j] = s_sum[j] / ni;
    __syncthreads();
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3];
      pw(k, p);
      for (int j = 0; j < 3; j++) p[j] -= s_cws[0][j];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) m[3 * a + b] += p[a] * p[b];
    }
    wg_sum<9>(m, s_red, s_sum);
    if (tid == 0) {
      double mm[9], dc[3], uct[9], V[9];
      int ord[3];
      for (int i = 0; i < 9; i++) mm[i] = s_sum[i];
      d_jacobi_eig_sym(3, mm, dc, uct, V, ord);
      for (int i = 1; i < 4; i++) {
        const double k = sqrt(fmax(dc[i - 1], 0.0) / ni);
        for (int j = 0; j < 3; j++) s_cws[i][j] = s_cws[0][j] + k * uct[3 * (i - 1) + j];
      }
      double cc[9], U[9], w[3];
      for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = s_cws[j][i] - s_cws[0][i];
      d_jacobi_svd(3, 3, cc, U, w, V);
      const double wmax = fmax(w[0], fmax(w[1], w[2]));
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
          double s = 0;
          for (int k = 0; k < 3; k++)
            if (w[k] > DBL_EPSILON * wmax * 3) s += V[r * 3 + k] * U[c * 3 + k] / w[k];
          s_ci[3 * r + c] = s;
        }
    }
    __syncthreads();
  }
  auto alphas = [&](int k, double* a) {
    double p[3];
    pw(k, p);
    for (int j = 0; j < 3; j++)
      a[1 + j] = s_ci[3 * j] * (p[0] - s_cws[0][0]) + s_ci[3 * j + 1] * (p[1] - s_cws[0][1]) +
                 s_ci[3 * j + 2] * (p[2] - s_cws[0][2]);
    a[0] = 1.0f - a[1] - a[2] - a[3];
  };
  // M^T M (upper triangle, 78 entries)
  {
    double v[78];
    for (int i = 0; i < 78; i++) v[i] = 0;
    for (int k = tid; k < ni; k += blockDim.x) {
      double a[4], u, vv;
      alphas(k, a);
      usp(k, u, vv);
      double M1[12], M2[12];
      for (int q = 0; q < 4; q++) {
        M1[3 * q] = a[q] * fu;
        M1[3 * q + 1] = 0.0;
        M1[3 * q + 2] = a[q] * (uc - u);
        M2[3 * q] = 0.0;
        M2[3 * q + 1] = a[q] * fv;
        M2[3 * q + 2] = a[q] * (vc - vv);
      }
      int t = 0;
      for (int r = 0; r < 12; r++)
        for (int c = r; c < 12; c++) v[t++] += M1[r] * M1[c] + M2[r] * M2[c];
    }
    wg_sum<78>(v, s_red, s_sum);
    if (tid == 0) {
      double mtm[144], d[12], V[144];
      int ord[12];
      int t = 0;
      for (int r = 0; r < 12; r++)
        for (int c = r; c < 12; c++) {
          mtm[12 * r + c] = s_sum[t];
          mtm[12 * c + r] = s_sum[t];
          t++;
        }
      d_jacobi_eig_sym(12, mtm, d, s_ut, V, ord);
      d_compute_L_6x10(s_ut, s_L);
      s_rho[0] = d_dist2(s_cws[0], s_cws[1]);
      s_rho[1] = d_dist2(s_cws[0], s_cws[2]);
      s_rho[2] = d_dist2(s_cws[0], s_cws[3]);
      s_rho[3] = d_dist2(s_cws[1], s_cws[2]);
      s_rho[4] = d_dist2(s_cws[1], s_cws[3]);
      s_rho[5] = d_dist2(s_cws[2], s_cws[3]);
    }
    __syncthreads();
  }
  for (int which = 1; which <= 3; which++) {
    if (tid == 0) {
      double betas[4];
      d_betas(which, s_L, s_rho, betas);
      d_gauss_newton(s_L, s_rho, betas);
      for (int i = 0; i < 4; i++) s_ccs[i][0] = s_ccs[i][1] = s_ccs[i][2] = 0.0f;
      for (int i = 0; i < 4; i++) {
        const double* v = s_ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
          for (int k = 0; k < 3; k++) s_ccs[j][k] += betas[i] * v[3 * j + k];
      }
      // solve_for_sign uses the first point's camera depth
      double a[4];
      alphas(0, a);
      const double pc2 = a[0] * s_ccs[0][2] + a[1] * s_ccs[1][2] + a[2] * s_ccs[2][2] + a[3] * s_ccs[3][2];
      if (pc2 < 0.0)
        for (int i = 0; i < 4; i++)
          for (int j = 0; j < 3; j++) s_ccs[i][j] = -s_ccs[i][j];
    }
    __syncthreads();
    auto pcs = [&](int k, double* pc) {
      double a[4];
      alphas(k, a);
      for (int j = 0; j < 3; j++)
        pc[j] = a[0] * s_ccs[0][j] + a[1] * s_ccs[1][j] + a[2] * s_ccs[2][j] + a[3] * s_ccs[3][j];
    };
    {
      double v[6] = {0, 0, 0, 0, 0, 0};
      for (int k = tid; k < ni; k += blockDim.x) {
        double pc[3], p[3];
        pcs(k, pc);
        pw(k, p);
        for (int j = 0; j < 3; j++) {
          v[j] += pc[j];
          v[3 + j] += p[j];
        }
      }
      wg_sum<6>(v, s_red, s_sum);
      if (tid == 0)
        for (int j = 0; j < 3; j++) {
          s_pc0[j] = s_sum[j] / ni;
          s_pw0[j] = s_sum[3 + j] / ni;
        }
      __syncthreads();
    }
    {
      double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = tid; k < ni; k += blockDim.x) {
        double pc[3], p[3];
        pcs(k, pc);
        pw(k, p);
        for (int j = 0; j < 3; j++)
          for (int q = 0; q < 3; q++) v[3 * j + q] += (pc[j] - s_pc0[j]) * (p[q] - s_pw0[q]);
      }
      wg_sum<9>(v, s_red, s_sum);
      if (tid == 0) {
        double abt[9], U[9], w[3], V[9];
        for (int i = 0; i < 9; i++) abt[i] = s_sum[i];
        d_jacobi_svd(3, 3, abt, U, w, V);
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++) s_R[i][j] = d_dot3(U + 3 * i, V + 3 * j);
        const double det = s_R[0][0] * s_R[1][1] * s_R[2][2] + s_R[0][1] * s_R[1][2] * s_R[2][0] +
                           s_R[0][2] * s_R[1][0] * s_R[2][1] - s_R[0][2] * s_R[1][1] * s_R[2][0] -
                           s_R[0][1] * s_R[1][0] * s_R[2][2] - s_R[0][0] * s_R[1][2] * s_R[2][1];
        if (det < 0)
          for (int j = 0; j < 3; j++) s_R[2][j] = -s_R[2][j];
        for (int r = 0; r < 3; r++) s_t[r] = s_pc0[r] - d_dot3(s_R[r], s_pw0);
      }
      __syncthreads();
    }
    {
      double v[1] = {0};
      for (int k = tid; k < ni; k += blockDim.x) {
        double p[3], u, vv;
        pw(k, p);
        usp(k, u, vv);
        const double Xc = d_dot3(s_R[0], p) + s_t[0], Yc = d_dot3(s_R[1], p) + s_t[1];
        const double inv_Zc = 1.0 / (d_dot3(s_R[2], p) + s_t[2]);
        const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
        v[0] += sqrt((u - ue) * (u - ue) + (vv - ve) * (vv - ve));
      }
      wg_sum<1>(v, s_red, s_sum);
      if (tid == 0) {
        const double err = s_sum[0] / ni;
        if (which == 1 || err < s_best) {
          s_best = err;
          for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) s_bestR[3 * r + c] = s_R[r][c];
            s_bestT[r] = s_t[r];
          }
        }
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    double rv[3], R[9];
    d_rodrigues_r2v(s_bestR, rv);
    d_rodrigues_v2r(rv, R);
    for (int i = 0; i < 9; i++) o.Rt[i] = R[i];
    for (int i = 0; i < 3; i++) o.Rt[9 + i] = s_bestT[i];
    o.result[3] = ni;
  }
}

// motion-model inliers, ascending (GetInitModelObj, Tracking.cc:4380-4399); MM row-major float
__global__ __launch_bounds__(256) void k_mm_inliers(PnPObject* objs) {
  __shared__ int s_w[4];
  PnPObject& o = objs[blockIdx.x];
  if (!o.use_mm) return;
  const int n = *o.n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    bool in = false;
    if (i < n) {
      float xc[3];
      for (int r = 0; r < 3; r++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += (double)o.MM[4 * r + k] * (double)o.pts3[3 * i + k];
        xc[r] = (float)s + o.MM[4 * r + 3];
      }
      const float invzc = (float)(1.0 / (double)xc[2]);
      const float u = o.fx * xc[0] * invzc + o.cx, v = o.fy * xc[1] * invzc + o.cy;
      const float2 q = o.pts2[i];
      const float u_ = q.x - u, v_ = q.y - v;
      const float Rpe = sqrtf(u_ * u_ + v_ * v_);
      in = (double)Rpe < o.reproj;
    }
    const unsigned long long bal = __ballot(in);
    if (lane == 0) s_w[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) off += s_w[w];
      tot += s_w[w];
    }
    if (in) o.mm_inliers[base + off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) o.result[4] = base;
}

// D3 edge index list: ObjId_sub[i] = ObjId[inliers[i]] (sample indices)
__global__ __launch_bounds__(256) void k_pnp_subset(PnPObject* objs) {
  PnPObject& o = objs[blockIdx.x];
  const int n = o.use_mm_choice ? o.result[4] : o.result[3];
  const int* src = o.use_mm_choice ? o.mm_inliers : o.inliers;
  for (int i = threadIdx.x; i < n; i += blockDim.x) o.subset[i] = o.members[src[i]];
  if (threadIdx.x == 0) *o.n_subset = n;
}

void launch_pnp(PnPObject* d_objs, int nobj, int max_iters, hipStream_t st, bool gather) {
  if (gather) hipLaunchKernelGGL(k_pnp_gather, dim3(nobj), dim3(256), 0, st, d_objs);
  hipLaunchKernelGGL(k_pnp_hyp, dim3((max_iters + 63) / 64, nobj), dim3(64), 0, st, d_objs, max_iters);
  hipLaunchKernelGGL(k_pnp_score, dim3(max_iters, nobj), dim3(256), 0, st, d_objs, max_iters);
  hipLaunchKernelGGL(k_pnp_select, dim3(nobj), dim3(64), 0, st, d_objs, max_iters);
  hipLaunchKernelGGL(k_pnp_refit, dim3(nobj), dim3(256), 0, st, d_objs);
  hipLaunchKernelGGL(k_mm_inliers, dim3(nobj), dim3(256), 0, st, d_objs);
}

void launch_pnp_subset(PnPObject* d_objs, int nobj, hipStream_t st) {
  hipLaunchKernelGGL(k_pnp_subset, dim3(nobj), dim3(256), 0, st, d_objs);
}

}  // namespace mmt
