// multimot_track_amd/csrc/mmt_pnp.hip -- object-motion initialiser D5 on the GPU:
// cv::solvePnPRansac(pre_3d, cur_2d, K, 0, ..., 500, 0.3, 0.98, inliers, SOLVEPNP_AP3P) as
// called by Tracking::GetInitModelObj (reference src/Tracking.cc:4324-4443).
//
//   k_pnp_gather   pre_3d = UnprojectStereoObject(last sample), cur_2d = current sample
//   k_pnp_hyp      one wave per RANSAC hypothesis: 5-point EPnP (PnPsolver.cc:342-1022 lineage)
//                  on the subset drawn by RNG((uint64)-1) (precomputed on the host: the draw
//                  sequence depends only on the point count) up to the null space of M^T M
//   k_pnp_beta<V>  one lane per hypothesis: beta estimate V, Gauss-Newton, R and t
//   k_pnp_score    picks the best estimate (Rodrigues -> model), then one workgroup per
//                  hypothesis scores it
//                  (projectPoints + squared-error test, inlier count by ballot/popcount,
//                  inlier bit mask)
//   k_pnp_select   replay of RANSACPointSetRegistrator::run's best-so-far / niters logic
//   k_refit_*      EPnP over all RANSAC inliers (reductions over the points, block-wide 12x12
//                  eigen-solve, beta estimates in lanes, one Procrustes solve per wave)
//   k_mm_inliers   motion-model check (Tracking.cc:4375-4405)
// The dense algebra (cyclic/one-sided Jacobi) follows oracle/pnp_ref.cpp operation for
// operation so hypothesis models agree to the last bit with the CPU checker.

#include <hip/hip_runtime.h>

#include <cfloat>

#include "mmt_internal.h"
#include "mmt_devmath.h"
#include "mmt_pnp.h"

namespace mmt {

// ---------------------------------------------------------------- register-resident dense algebra
// One lane, every array index a compile-time constant after unrolling, so the matrices live in
// VGPRs (dynamic indexing of private arrays would put them in scratch memory).  Operation order
// follows oracle/pnp_ref.cpp exactly.

// cyclic Jacobi eigen-decomposition of a small symmetric matrix; eigenvectors as rows of vt,
// stable descending order of the eigenvalues
template <int N>
__device__ __forceinline__ void eig_sym_small(double (&A)[N * N], double (&d)[N],
                                              double (&vt)[N * N]) {
  double V[N * N];
#pragma unroll
  for (int i = 0; i < N * N; i++) V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 100; sweep++) {
    double off = 0, dsum = 0;  // convergence test of oracle/pnp_ref.cpp
#pragma unroll
    for (int p = 0; p < N; p++) {
      dsum += A[p * N + p] * A[p * N + p];
#pragma unroll
      for (int q = p + 1; q < N; q++) off += A[p * N + q] * A[p * N + q];
    }
    if (off <= 1e-26 * dsum) break;
#pragma unroll
    for (int p = 0; p < N; p++)
#pragma unroll
      for (int q = p + 1; q < N; q++) {
        const double apq = A[p * N + q];
        if (fabs(apq) < 1e-300) continue;
        const double app = A[p * N + p], aqq = A[q * N + q];
        const double theta = (aqq - app) / (2 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
        const double c = 1 / sqrt(t * t + 1), s = t * c;
#pragma unroll
        for (int k = 0; k < N; k++) {
          const double akp = A[k * N + p], akq = A[k * N + q];
          A[k * N + p] = c * akp - s * akq;
          A[k * N + q] = s * akp + c * akq;
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
          const double apk = A[p * N + k], aqk = A[q * N + k];
          A[p * N + k] = c * apk - s * aqk;
          A[q * N + k] = s * apk + c * aqk;
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
          const double vkp = V[k * N + p], vkq = V[k * N + q];
          V[k * N + p] = c * vkp - s * vkq;
          V[k * N + q] = s * vkp + c * vkq;
        }
      }
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
    int rank = 0;
#pragma unroll
    for (int j = 0; j < N; j++)
      rank += (A[j * (N + 1)] > A[i * (N + 1)]) || (j < i && A[j * (N + 1)] == A[i * (N + 1)]);
#pragma unroll
    for (int r = 0; r < N; r++)
      if (rank == r) {
        d[r] = A[i * (N + 1)];
#pragma unroll
        for (int k = 0; k < N; k++) vt[r * N + k] = V[k * N + i];
      }
  }
}

// thin SVD (M >= N) by one-sided Jacobi; A is overwritten
template <int M, int N>
__device__ __forceinline__ void svd_small(double (&A)[M * N], double (&U)[M * N], double (&w)[N],
                                          double (&V)[N * N]) {
#pragma unroll
  for (int i = 0; i < N * N; i++) V[i] = (i % (N + 1) == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 100; sweep++) {
    bool changed = false;
#pragma unroll
    for (int p = 0; p < N; p++)
#pragma unroll
      for (int q = p + 1; q < N; q++) {
        double a = 0, b = 0, g = 0;
#pragma unroll
        for (int k = 0; k < M; k++) {
          a += A[k * N + p] * A[k * N + p];
          b += A[k * N + q] * A[k * N + q];
          g += A[k * N + p] * A[k * N + q];
        }
        if (fabs(g) <= 1e-15 * sqrt(a * b) || g == 0) continue;
        changed = true;
        const double zeta = (b - a) / (2 * g);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), s = c * t;
#pragma unroll
        for (int k = 0; k < M; k++) {
          const double x = A[k * N + p], y = A[k * N + q];
          A[k * N + p] = c * x - s * y;
          A[k * N + q] = s * x + c * y;
        }
#pragma unroll
        for (int k = 0; k < N; k++) {
          const double x = V[k * N + p], y = V[k * N + q];
          V[k * N + p] = c * x - s * y;
          V[k * N + q] = s * x + c * y;
        }
      }
    if (!changed) break;
  }
#pragma unroll
  for (int j = 0; j < N; j++) {
    double s = 0;
#pragma unroll
    for (int k = 0; k < M; k++) s += A[k * N + j] * A[k * N + j];
    w[j] = sqrt(s);
#pragma unroll
    for (int k = 0; k < M; k++) U[k * N + j] = w[j] > 0 ? A[k * N + j] / w[j] : 0.0;
  }
}

// x = pinv(A) b (cvSolve(..., CV_SVD)); A (M x N) is overwritten
template <int M, int N>
__device__ __forceinline__ void svd_solve_small(double (&A)[M * N], const double (&b)[M],
                                                double (&x)[N]) {
  double U[M * N], w[N], V[N * N];
  svd_small<M, N>(A, U, w, V);
  double wmax = 0;
#pragma unroll
  for (int j = 0; j < N; j++) wmax = fmax(wmax, w[j]);
  const double thr = DBL_EPSILON * wmax * M;
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = 0;
#pragma unroll
  for (int j = 0; j < N; j++) {
    if (w[j] <= thr) continue;
    double ub = 0;
#pragma unroll
    for (int k = 0; k < M; k++) ub += U[k * N + j] * b[k];
    ub /= w[j];
#pragma unroll
    for (int i = 0; i < N; i++) x[i] += V[i * N + j] * ub;
  }
}

// pseudo-inverse of the 3x3 control-point matrix (cvInvert(CC, CC_inv, CV_SVD))
__device__ __forceinline__ void pinv3(double (&cc)[9], double (&ci)[9]) {
  double U[9], w[3], V[9];
  svd_small<3, 3>(cc, U, w, V);
  const double wmax = fmax(w[0], fmax(w[1], w[2]));
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) {
      double s = 0;
#pragma unroll
      for (int k = 0; k < 3; k++)
        if (w[k] > DBL_EPSILON * wmax * 3) s += V[r * 3 + k] * U[c * 3 + k] / w[k];
      ci[3 * r + c] = s;
    }
}

// rotation from the cross-covariance abt (estimate_R_and_t)
__device__ __forceinline__ void procrustes_R(double (&abt)[9], double (&R)[9]) {
  double U[9], w[3], V[9];
  svd_small<3, 3>(abt, U, w, V);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      R[3 * i + j] = U[3 * i] * V[3 * j] + U[3 * i + 1] * V[3 * j + 1] + U[3 * i + 2] * V[3 * j + 2];
  const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] -
                     R[2] * R[4] * R[6] - R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
  if (det < 0) {
    R[6] = -R[6];
    R[7] = -R[7];
    R[8] = -R[8];
  }
}

__device__ __forceinline__ double d_dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ double d_dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

// L_6x10 from the four null-space vectors ut rows 11, 10, 9, 8 (`ut8` points at row 8)
__device__ __forceinline__ void compute_L_6x10(const double* ut8, double (&l)[60]) {
  double dv[4][6][3];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double* v = ut8 + 12 * (3 - i);
    int a = 0, b = 1;
#pragma unroll
    for (int j = 0; j < 6; j++) {
#pragma unroll
      for (int k = 0; k < 3; k++) dv[i][j][k] = v[3 * a + k] - v[3 * b + k];
      b++;
      if (b > 3) {
        a++;
        b = a + 1;
      }
    }
  }
#pragma unroll
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

__device__ __forceinline__ void betas_approx_1(const double (&L)[60], const double (&rho)[6],
                                               double (&betas)[4]) {
  double A[24], b4[4];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    A[4 * i] = L[10 * i];
    A[4 * i + 1] = L[10 * i + 1];
    A[4 * i + 2] = L[10 * i + 3];
    A[4 * i + 3] = L[10 * i + 6];
  }
  svd_solve_small<6, 4>(A, rho, b4);
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
}

__device__ __forceinline__ void betas_approx_2(const double (&L)[60], const double (&rho)[6],
                                               double (&betas)[4]) {
  double A[18], b3[3];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) A[3 * i + k] = L[10 * i + k];
  svd_solve_small<6, 3>(A, rho, b3);
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
}

__device__ __forceinline__ void betas_approx_3(const double (&L)[60], const double (&rho)[6],
                                               double (&betas)[4]) {
  double A[30], b5[5];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int k = 0; k < 5; k++) A[5 * i + k] = L[10 * i + k];
  svd_solve_small<6, 5>(A, rho, b5);
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

// Householder QR solve of the 6x4 Gauss-Newton system (PnPsolver.cc:840-950, including its
// column-max scan that starts one row early)
__device__ __forceinline__ void qr_solve_6x4(double (&A)[24], double (&b)[6], double (&X)[4]) {
  constexpr int nr = 6, nc = 4;
  double A1[4], A2[4];
#pragma unroll
  for (int k = 0; k < nc; k++) {
    double eta = fabs(A[k * nc + k]);
#pragma unroll
    for (int i = k + 1; i < nr; i++) {
      const double elt = fabs(A[(i - 1) * nc + k]);
      if (eta < elt) eta = elt;
    }
    if (eta == 0) return;  // "A is singular": X left unchanged
    double sum = 0.0;
    const double inv_eta = 1. / eta;
#pragma unroll
    for (int i = k; i < nr; i++) {
      A[i * nc + k] *= inv_eta;
      sum += A[i * nc + k] * A[i * nc + k];
    }
    double sigma = sqrt(sum);
    if (A[k * nc + k] < 0) sigma = -sigma;
    A[k * nc + k] += sigma;
    A1[k] = sigma * A[k * nc + k];
    A2[k] = -eta * sigma;
#pragma unroll
    for (int j = k + 1; j < nc; j++) {
      double s = 0;
#pragma unroll
      for (int i = k; i < nr; i++) s += A[i * nc + k] * A[i * nc + j];
      const double tau = s / A1[k];
#pragma unroll
      for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
    }
  }
#pragma unroll
  for (int j = 0; j < nc; j++) {
    double tau = 0;
#pragma unroll
    for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
    tau /= A1[j];
#pragma unroll
    for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
  }
  X[nc - 1] = b[nc - 1] / A2[nc - 1];
#pragma unroll
  for (int i = nc - 2; i >= 0; i--) {
    double s = 0;
#pragma unroll
    for (int j = i + 1; j < nc; j++) s += A[i * nc + j] * X[j];
    X[i] = (b[i] - s) / A2[i];
  }
}

__device__ __forceinline__ void gauss_newton(const double (&L)[60], const double (&rho)[6],
                                             double (&betas)[4]) {
  for (int k = 0; k < 5; k++) {
    double A[24], b[6], x[4] = {0, 0, 0, 0};
#pragma unroll
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
    qr_solve_6x4(A, b, x);
#pragma unroll
    for (int i = 0; i < 4; i++) betas[i] += x[i];
  }
}

// ccs = sum_i betas[i] * ut row (11 - i)  (compute_ccs)
__device__ __forceinline__ void compute_ccs(const double* ut, const double (&betas)[4],
                                            double (&ccs)[12]) {
#pragma unroll
  for (int i = 0; i < 12; i++) ccs[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double* v = ut + 12 * (11 - i);
#pragma unroll
    for (int j = 0; j < 12; j++) ccs[j] += betas[i] * v[j];
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

// ---------------------------------------------------------------- 12x12 eigen-solve, one lane per column
// One-sided parallel-order Jacobi of oracle/pnp_ref.cpp (jacobi_eig12): lane `gb + j` holds
// column j of the matrix (a) and of the accumulated rotation (v) in registers; per round it
// fetches its partner column with cross-lane shuffles, both lanes of a pair compute the same
// (alpha, beta, gamma) in the same order, hence the same rotation, and each updates its own
// column.  A 64-lane wave runs five independent solves (lanes 0-59).  On return `rank` is the
// column's position in descending singular-value order.
__device__ __forceinline__ void rr_partner(int r, int j, int& p, int& q) {
  const int k = j == 11 ? r : (j == r ? 11 : (2 * r - j + 22) % 11);
  p = min(j, k);
  q = max(j, k);
}

__device__ __forceinline__ int eig12_group(double (&a)[12], double (&v)[12], int gb, int j,
                                           bool active, int& rank) {
  const int lane = threadIdx.x & 63;
  const unsigned long long gmask = active ? (0xFFFull << gb) : 0ull;
  int sweep = 0;
  for (; sweep < 100; sweep++) {
    bool rotated = false;
    for (int r = 0; r < 11; r++) {
      int p, q;
      rr_partner(r, j, p, q);
      const int src = gb + (j == p ? q : p);
      const bool mine_p = (j == p);
      // the partner's column; both lanes of a pair form the same sums bit for bit (same terms,
      // same order; x*y == y*x), so they take the same decision and rotation
      double b[12];
#pragma unroll
      for (int k = 0; k < 12; k++) b[k] = __shfl(a[k], src, 64);
      double nm = 0, no = 0, ga = 0;
#pragma unroll
      for (int k = 0; k < 12; k++) {
        nm += a[k] * a[k];
        no += b[k] * b[k];
        ga += a[k] * b[k];
      }
      const double al = mine_p ? nm : no, be = mine_p ? no : nm;
      if (active && !(fabs(ga) <= 1e-15 * sqrt(al * be) || ga == 0)) {
        rotated = true;
        const double zeta = (be - al) / (2 * ga);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), s = c * t;
        // p: c x - s y, q: s x + c y (x, y the p and q columns) == c mine + (-/+ s) other
        const double sg = mine_p ? -s : s;
        double w[12];
#pragma unroll
        for (int k = 0; k < 12; k++) w[k] = __shfl(v[k], src, 64);
#pragma unroll
        for (int k = 0; k < 12; k++) {
          a[k] = c * a[k] + sg * b[k];
          v[k] = c * v[k] + sg * w[k];
        }
      }
    }
    const unsigned long long any = __ballot(rotated);
    // every group keeps shuffling until all groups of the wave have converged; a converged
    // group's pairs are orthogonal and stay untouched, so its results do not change
    if (!(any & 0x0FFFFFFFFFFFFFFFull)) break;
    (void)gmask;
  }
  double ss = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) ss += a[k] * a[k];
  const double sig = sqrt(ss);
  rank = 0;
  for (int i = 0; i < 12; i++) {
    const double si = __shfl(sig, gb + i, 64);
    rank += (si > sig) || (i < j && si == sig);
  }
  (void)lane;
  return sweep;
}

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

// Hypothesis record layout (doubles): the four null-space vectors ut rows 8..11, alphas, pws,
// us, L_6x10, rho
constexpr int R_UT = 0, R_AL = 48, R_PW = 68, R_US = 83, R_L = 93, R_RHO = 153;

// 64-lane workgroup = five hypotheses (lanes 12g..12g+11 for hypothesis g): 5-point EPnP up to
// the null space of M^T M.  Lane 12g does the control points in registers, every lane builds one
// column of M^T M and runs its column of the eigen-solve.
constexpr int kHypPerBlock = 5;

// NP = points per minimal set: 5 for D5 (solvePnPRansac's EPnP sets), 4 for D6 (PnPsolver's
// P4P sets).  D6 (o.raw_pixels) feeds the pixel coordinates to EPnP as they are
// (PnPsolver::add_correspondence); D5 round-trips them through undistortPoints.
template <int NP>
__global__ __launch_bounds__(64) void k_pnp_hyp(PnPObject* objs, int max_iters) {
  __shared__ double s_al[kHypPerBlock][20], s_us[kHypPerBlock][10], s_pws[kHypPerBlock][15];
  __shared__ double s_cws[kHypPerBlock][12], s_ut[kHypPerBlock][48];
  const int lane = threadIdx.x, g = lane / 12, j = lane - 12 * g, gb = 12 * g;
  PnPObject& o = objs[blockIdx.y];
  const int n = *o.n;
  if (n < NP) return;
  const int h = blockIdx.x * kHypPerBlock + g;
  const bool active = g < kHypPerBlock && h < max_iters;
  const double fu = o.fx, fv = o.fy, uc = o.cx, vc = o.cy;
  if (active && j == 0) {
    double pws[3 * NP], us[2 * NP], cws[12];
    const double ifx = 1. / fu, ify = 1. / fv;
    const int* sub = o.subsets + NP * h;
#pragma unroll
    for (int i = 0; i < NP; i++) {
      // D5 with count == modelPoints: the kernel runs on all points
      const int jj = (NP == 5 && n == 5) ? i : sub[i];
#pragma unroll
      for (int k = 0; k < 3; k++) pws[3 * i + k] = o.pts3[3 * jj + k];
      const float2 pt = o.pts2[jj];
      if (o.raw_pixels) {
        us[2 * i] = pt.x;
        us[2 * i + 1] = pt.y;
      } else {
        const float xn = (float)(((double)pt.x - uc) * ifx);
        const float yn = (float)(((double)pt.y - vc) * ify);
        us[2 * i] = (double)xn * fu + uc;
        us[2 * i + 1] = (double)yn * fv + vc;
      }
    }
    // choose_control_points
    cws[0] = cws[1] = cws[2] = 0;
#pragma unroll
    for (int i = 0; i < NP; i++)
#pragma unroll
      for (int k = 0; k < 3; k++) cws[k] += pws[3 * i + k];
#pragma unroll
    for (int k = 0; k < 3; k++) cws[k] /= NP;
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NP; i++) {
      double pp[3];
#pragma unroll
      for (int k = 0; k < 3; k++) pp[k] = pws[3 * i + k] - cws[k];
#pragma unroll
      for (int x = 0; x < 3; x++)
#pragma unroll
        for (int y = 0; y < 3; y++) m[3 * x + y] += pp[x] * pp[y];
    }
    double dc[3], uct[9];
    eig_sym_small<3>(m, dc, uct);
#pragma unroll
    for (int i = 1; i < 4; i++) {
      const double k = sqrt(fmax(dc[i - 1], 0.0) / NP);
#pragma unroll
      for (int x = 0; x < 3; x++) cws[3 * i + x] = cws[x] + k * uct[3 * (i - 1) + x];
    }
    // compute_barycentric_coordinates
    double cc[9], ci[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int x = 1; x < 4; x++) cc[3 * i + x - 1] = cws[3 * x + i] - cws[i];
    pinv3(cc, ci);
#pragma unroll
    for (int i = 0; i < NP; i++) {
      const double* pi = &pws[3 * i];
      double al[4];
#pragma unroll
      for (int x = 0; x < 3; x++)
        al[1 + x] = ci[3 * x] * (pi[0] - cws[0]) + ci[3 * x + 1] * (pi[1] - cws[1]) +
                    ci[3 * x + 2] * (pi[2] - cws[2]);
      al[0] = 1.0f - al[1] - al[2] - al[3];
#pragma unroll
      for (int x = 0; x < 4; x++) s_al[g][4 * i + x] = al[x];
    }
#pragma unroll
    for (int i = 0; i < 3 * NP; i++) s_pws[g][i] = pws[i];
#pragma unroll
    for (int i = 0; i < 2 * NP; i++) s_us[g][i] = us[i];
#pragma unroll
    for (int i = 0; i < 12; i++) s_cws[g][i] = cws[i];
  }
  __syncthreads();
  // column j of M^T M: entry (k, j) = sum_i M1[k] M1[j] + M2[k] M2[j], points in order
  double a[12], v[12];
  {
    const int qb = j / 3, cb = j - 3 * qb;
    const int gg = active ? g : 0;
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int qa = k / 3, ca = k - 3 * qa;
      double acc = 0;
      for (int i = 0; i < NP; i++) {
        const double u = s_us[gg][2 * i], vv = s_us[gg][2 * i + 1];
        const double aa = s_al[gg][4 * i + qa], ab = s_al[gg][4 * i + qb];
        const double m1a = ca == 0 ? aa * fu : (ca == 1 ? 0.0 : aa * (uc - u));
        const double m1b = cb == 0 ? ab * fu : (cb == 1 ? 0.0 : ab * (uc - u));
        const double m2a = ca == 0 ? 0.0 : (ca == 1 ? aa * fv : aa * (vc - vv));
        const double m2b = cb == 0 ? 0.0 : (cb == 1 ? ab * fv : ab * (vc - vv));
        acc += m1a * m1b + m2a * m2b;
      }
      a[k] = active ? acc : 0.0;
      v[k] = (k == j) ? 1.0 : 0.0;
    }
  }
  int rank;
  eig12_group(a, v, gb, j, active, rank);
  // ut rows 8..11 (the four smallest singular values) = V columns of ranks 8..11
  if (active && rank >= 8)
#pragma unroll
    for (int k = 0; k < 12; k++) s_ut[g][(rank - 8) * 12 + k] = v[k];
  __syncthreads();
  if (!active) return;
  double* rec = o.hrec + (size_t)kHypRec * h;
  for (int e = j; e < 48; e += 12) rec[R_UT + e] = s_ut[g][e];
  for (int e = j; e < 4 * NP; e += 12) rec[R_AL + e] = s_al[g][e];
  for (int e = j; e < 3 * NP; e += 12) rec[R_PW + e] = s_pws[g][e];
  if (j < 2 * NP) rec[R_US + j] = s_us[g][j];
  if (j == 0) {
    double L[60];
    compute_L_6x10(s_ut[g], L);
#pragma unroll
    for (int i = 0; i < 60; i++) rec[R_L + i] = L[i];
    const double* cws = s_cws[g];
    rec[R_RHO + 0] = d_dist2(cws + 0, cws + 3);
    rec[R_RHO + 1] = d_dist2(cws + 0, cws + 6);
    rec[R_RHO + 2] = d_dist2(cws + 0, cws + 9);
    rec[R_RHO + 3] = d_dist2(cws + 3, cws + 6);
    rec[R_RHO + 4] = d_dist2(cws + 3, cws + 9);
    rec[R_RHO + 5] = d_dist2(cws + 6, cws + 9);
  }
}

// one lane per (hypothesis, object) for beta estimate V (betas_approx_V + gauss_newton +
// compute_R_and_t); each variant is its own launch so a wave runs one code path
template <int V, int NP>
__device__ __forceinline__ void pnp_beta(PnPObject& o, int max_iters) {
  const int h = blockIdx.x * 64 + threadIdx.x;
  const int n = *o.n;
  if (h >= max_iters || n < NP) return;
  const double fu = o.fx, fv = o.fy, uc = o.cx, vc = o.cy;
  const double* rec = o.hrec + (size_t)kHypRec * h;
  double L[60], rho[6], betas[4];
#pragma unroll
  for (int i = 0; i < 60; i++) L[i] = rec[R_L + i];
#pragma unroll
  for (int i = 0; i < 6; i++) rho[i] = rec[R_RHO + i];
  if (V == 1)
    betas_approx_1(L, rho, betas);
  else if (V == 2)
    betas_approx_2(L, rho, betas);
  else
    betas_approx_3(L, rho, betas);
  gauss_newton(L, rho, betas);
  // compute_R_and_t: ccs, pcs, solve_for_sign, estimate_R_and_t, reprojection_error
  double ccs[12], pcs[3 * NP], pws[3 * NP], R[9], t[3];
#pragma unroll
  for (int i = 0; i < 12; i++) ccs[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double* v = rec + R_UT + 12 * (3 - i);  // ut row 11 - i
#pragma unroll
    for (int j = 0; j < 12; j++) ccs[j] += betas[i] * v[j];
  }
#pragma unroll
  for (int i = 0; i < NP; i++) {
    const double* a = rec + R_AL + 4 * i;
#pragma unroll
    for (int j = 0; j < 3; j++)
      pcs[3 * i + j] = a[0] * ccs[j] + a[1] * ccs[3 + j] + a[2] * ccs[6 + j] + a[3] * ccs[9 + j];
  }
  if (pcs[2] < 0.0) {
#pragma unroll
    for (int i = 0; i < 3 * NP; i++) pcs[i] = -pcs[i];
  }
#pragma unroll
  for (int i = 0; i < 3 * NP; i++) pws[i] = rec[R_PW + i];
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < NP; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      pc0[j] += pcs[3 * i + j];
      pw0[j] += pws[3 * i + j];
    }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    pc0[j] /= NP;
    pw0[j] /= NP;
  }
  double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < NP; i++) {
    const double* pc = &pcs[3 * i];
    const double* pw = &pws[3 * i];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
      abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
      abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
    }
  }
  procrustes_R(abt, R);
#pragma unroll
  for (int r = 0; r < 3; r++) t[r] = pc0[r] - d_dot3(R + 3 * r, pw0);
  double sum2 = 0.0;
#pragma unroll
  for (int i = 0; i < NP; i++) {
    const double* pw = &pws[3 * i];
    const double Xc = d_dot3(R, pw) + t[0], Yc = d_dot3(R + 3, pw) + t[1];
    const double inv_Zc = 1.0 / (d_dot3(R + 6, pw) + t[2]);
    const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
    const double u = rec[R_US + 2 * i], v = rec[R_US + 2 * i + 1];
    sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
  }
  double* out = o.hout + (size_t)kHypOut * (3 * h + V - 1);
  out[0] = sum2 / NP;
#pragma unroll
  for (int i = 0; i < 9; i++) out[1 + i] = R[i];
#pragma unroll
  for (int i = 0; i < 3; i++) out[10 + i] = t[i];
}

// the three estimates of every hypothesis run concurrently (blockIdx.z = estimate), each block on
// one code path
template <int NP>
__global__ __launch_bounds__(64) void k_pnp_beta(PnPObject* objs, int max_iters) {
  PnPObject& o = objs[blockIdx.y];
  if (blockIdx.z == 0)
    pnp_beta<1, NP>(o, max_iters);
  else if (blockIdx.z == 1)
    pnp_beta<2, NP>(o, max_iters);
  else
    pnp_beta<3, NP>(o, max_iters);
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
  double* m = o.models + 6 * h;
  if (threadIdx.x == 0) {
    // compute_pose's choice among the three beta estimates (rep_errors[2] < [1]; [3] < [N]),
    // then the model as PnPRansacCallback stores it (rvec via Rodrigues, tvec)
    const double* out = o.hout + (size_t)kHypOut * 3 * h;
    int best = 0;
    if (out[kHypOut] < out[0]) best = 1;
    if (out[2 * kHypOut] < out[best * kHypOut]) best = 2;
    const double* bo = out + best * kHypOut;
    double rv[3];
    d_rodrigues_r2v(bo + 1, rv);
    m[0] = rv[0];
    m[1] = rv[1];
    m[2] = rv[2];
    m[3] = bo[10];
    m[4] = bo[11];
    m[5] = bo[12];
    d_rodrigues_v2r(m, sR);
  }
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

// EPnP refit over the best hypothesis' inliers, in three steps per object:
//   k_refit_null    inlier index list (ascending; ObjIdTest_in), control points, M^T M
//                   (reductions over the inliers), block-wide 12x12 eigen-solve, L_6x10, rho
//   k_refit_beta<V> lane 0: beta estimate V + Gauss-Newton -> control points in camera frame
//   k_refit_rt      R, t and reprojection error of the three estimates (reductions over the
//                   inliers, one Procrustes solve per wave), best estimate -> Rodrigues round trip
// The refit is not bit-identical to the CPU checker (its sums over the inliers are reduced in a
// different order); RANSAC's decisions (inlier sets, iteration counts) do not depend on it.
// Record: the hypothesis-0 slot of hrec (free once the hypotheses are scored); R_AL holds cws,
// R_PW the pseudo-inverse ci; hout slots 0..2 hold ccs of the three estimates.
struct RefitSmem {
  double red[4 * 80], sum[80];
  double A[144], ut8[48];
  double cws[12], ci[9];
  int w[4], n;
};

__device__ __forceinline__ void refit_pw(const PnPObject& o, int k, double* p) {
  const int j = o.inliers[k];
  p[0] = o.pts3[3 * j];
  p[1] = o.pts3[3 * j + 1];
  p[2] = o.pts3[3 * j + 2];
}

// solvePnPRansac converts the inliers to CV_64F before the refit, so undistortPoints keeps the
// normalised coordinates in double here (the hypotheses round them to float)
__device__ __forceinline__ void refit_us(const PnPObject& o, int k, double& u, double& v) {
  const float2 q = o.pts2[o.inliers[k]];
  if (o.raw_pixels) {  // D6: PnPsolver::Refine adds the pixels as they are
    u = q.x;
    v = q.y;
    return;
  }
  const double fu = o.fx, fv = o.fy, uc = o.cx, vc = o.cy;
  u = (((double)q.x - uc) * (1. / fu)) * fu + uc;
  v = (((double)q.y - vc) * (1. / fv)) * fv + vc;
}

__device__ __forceinline__ void refit_alphas(const PnPObject& o, int k, const double* cws,
                                             const double* ci, double* a) {
  double p[3];
  refit_pw(o, k, p);
  for (int j = 0; j < 3; j++)
    a[1 + j] = ci[3 * j] * (p[0] - cws[0]) + ci[3 * j + 1] * (p[1] - cws[1]) +
               ci[3 * j + 2] * (p[2] - cws[2]);
  a[0] = 1.0f - a[1] - a[2] - a[3];
}

__global__ __launch_bounds__(256) void k_refit_null(PnPObject* objs) {
  __shared__ RefitSmem S;
  PnPObject& o = objs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef MMT_PNP_PROFILE
  long long tp[8];
  int np = 0;
  if (tid == 0) tp[np++] = clock64();
#define PNPPROF() do { if (tid == 0) tp[np++] = clock64(); } while (0)
#else
#define PNPPROF() do { } while (0)
#endif
  const int best = o.result[0];
  if (best < 0) {
    if (tid == 0) o.result[3] = 0;
    return;
  }
  const int n = *o.n;
  const unsigned long long* mask = o.masks + (size_t)best * o.mask_words;
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + tid;
    const bool in = i < n && ((mask[i >> 6] >> (i & 63)) & 1ull);
    const unsigned long long bal = __ballot(in);
    if (lane == 0) S.w[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) off += S.w[w];
      tot += S.w[w];
    }
    if (in) o.inliers[base + off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    base += tot;
    __syncthreads();
  }
  if (tid == 0) {
    S.n = base;
    o.result[3] = base;
  }
  __syncthreads();
  PNPPROF();
  const int ni = S.n;
  const double fu = o.fx, fv = o.fy, uc = o.cx, vc = o.cy;
  // control points: centroid, then PCA of the centred points
  {
    double v[3] = {0, 0, 0};
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3];
      refit_pw(o, k, p);
      v[0] += p[0];
      v[1] += p[1];
      v[2] += p[2];
    }
    wg_sum<3>(v, S.red, S.sum);
    if (tid == 0)
      for (int j = 0; j < 3; j++) S.cws[j] = S.sum[j] / ni;
    __syncthreads();
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3];
      refit_pw(o, k, p);
      for (int j = 0; j < 3; j++) p[j] -= S.cws[j];
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b < 3; b++) m[3 * a + b] += p[a] * p[b];
    }
    wg_sum<9>(m, S.red, S.sum);
    if (tid == 0) {
      double mm[9], dc[3], uct[9], cws[12], cc[9], ci[9];
#pragma unroll
      for (int i = 0; i < 9; i++) mm[i] = S.sum[i];
      eig_sym_small<3>(mm, dc, uct);
#pragma unroll
      for (int j = 0; j < 3; j++) cws[j] = S.cws[j];
#pragma unroll
      for (int i = 1; i < 4; i++) {
        const double k = sqrt(fmax(dc[i - 1], 0.0) / ni);
#pragma unroll
        for (int j = 0; j < 3; j++) cws[3 * i + j] = cws[j] + k * uct[3 * (i - 1) + j];
      }
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[3 * j + i] - cws[i];
      pinv3(cc, ci);
#pragma unroll
      for (int i = 0; i < 12; i++) S.cws[i] = cws[i];
#pragma unroll
      for (int i = 0; i < 9; i++) S.ci[i] = ci[i];
    }
    __syncthreads();
  }
  PNPPROF();
  // M^T M (upper triangle, 78 entries)
  {
    double v[78];
#pragma unroll
    for (int i = 0; i < 78; i++) v[i] = 0;
    for (int k = tid; k < ni; k += blockDim.x) {
      double a[4], u, vv;
      refit_alphas(o, k, S.cws, S.ci, a);
      refit_us(o, k, u, vv);
      double M1[12], M2[12];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        M1[3 * q] = a[q] * fu;
        M1[3 * q + 1] = 0.0;
        M1[3 * q + 2] = a[q] * (uc - u);
        M2[3 * q] = 0.0;
        M2[3 * q + 1] = a[q] * fv;
        M2[3 * q + 2] = a[q] * (vc - vv);
      }
      int t = 0;
#pragma unroll
      for (int r = 0; r < 12; r++)
#pragma unroll
        for (int c = r; c < 12; c++) v[t++] += M1[r] * M1[c] + M2[r] * M2[c];
    }
    wg_sum<78>(v, S.red, S.sum);
    for (int e = tid; e < 144; e += blockDim.x) {
      const int r = e / 12, c = e - 12 * r;
      const int lo = min(r, c), hi = max(r, c);
      S.A[e] = S.sum[lo * 12 - lo * (lo - 1) / 2 + (hi - lo)];
    }
    __syncthreads();
  }
  PNPPROF();
  if (wave == 0) {  // the eigen-solve runs on lanes 0..11 of wave 0
    const bool act = lane < 12;
    const int j = act ? lane : 0;
    double a[12], v[12];
#pragma unroll
    for (int k = 0; k < 12; k++) {
      a[k] = act ? S.A[12 * k + j] : 0.0;
      v[k] = (act && k == j) ? 1.0 : 0.0;
    }
    int rank;
    const int nsw = eig12_group(a, v, 0, act ? lane : 12 + (lane % 12), act, rank);
#ifdef MMT_PNP_PROFILE
    if (lane == 0) S.n = nsw;
#else
    (void)nsw;
#endif
    if (act && rank >= 8)
#pragma unroll
      for (int k = 0; k < 12; k++) S.ut8[(rank - 8) * 12 + k] = v[k];
  }
  __syncthreads();
  PNPPROF();
  double* rec = o.hrec;
  for (int e = tid; e < 48; e += blockDim.x) rec[R_UT + e] = S.ut8[e];
  if (tid < 12) rec[R_AL + tid] = S.cws[tid];
  if (tid < 9) rec[R_PW + tid] = S.ci[tid];
  if (tid == 0) {
    double L[60];
    compute_L_6x10(S.ut8, L);
#pragma unroll
    for (int i = 0; i < 60; i++) rec[R_L + i] = L[i];
    const double* cws = S.cws;
    rec[R_RHO + 0] = d_dist2(cws + 0, cws + 3);
    rec[R_RHO + 1] = d_dist2(cws + 0, cws + 6);
    rec[R_RHO + 2] = d_dist2(cws + 0, cws + 9);
    rec[R_RHO + 3] = d_dist2(cws + 3, cws + 6);
    rec[R_RHO + 4] = d_dist2(cws + 3, cws + 9);
    rec[R_RHO + 5] = d_dist2(cws + 6, cws + 9);
  }
#ifdef MMT_PNP_PROFILE
  if (tid == 0)
    printf("refitprof ni=%d compact=%lld ctrl=%lld mtm=%lld eig=%lld sweeps=%d\n", ni,
           tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3], S.n);
#endif
#undef PNPPROF
}

template <int V>
__device__ __forceinline__ void refit_beta(PnPObject& o) {
  if (threadIdx.x != 0 || o.result[0] < 0) return;
  const double* rec = o.hrec;
  double L[60], rho[6], betas[4], ccs[12];
#pragma unroll
  for (int i = 0; i < 60; i++) L[i] = rec[R_L + i];
#pragma unroll
  for (int i = 0; i < 6; i++) rho[i] = rec[R_RHO + i];
  if (V == 1)
    betas_approx_1(L, rho, betas);
  else if (V == 2)
    betas_approx_2(L, rho, betas);
  else
    betas_approx_3(L, rho, betas);
  gauss_newton(L, rho, betas);
#pragma unroll
  for (int i = 0; i < 12; i++) ccs[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double* v = rec + R_UT + 12 * (3 - i);  // ut row 11 - i
#pragma unroll
    for (int j = 0; j < 12; j++) ccs[j] += betas[i] * v[j];
  }
  // solve_for_sign on the first inlier's camera depth
  double a[4];
  refit_alphas(o, 0, rec + R_AL, rec + R_PW, a);
  const double pc2 = a[0] * ccs[2] + a[1] * ccs[5] + a[2] * ccs[8] + a[3] * ccs[11];
  double* out = o.hout + (size_t)kHypOut * (V - 1);
#pragma unroll
  for (int i = 0; i < 12; i++) out[i] = pc2 < 0.0 ? -ccs[i] : ccs[i];
}

__global__ __launch_bounds__(64) void k_refit_beta(PnPObject* objs) {
  PnPObject& o = objs[blockIdx.x];
  if (blockIdx.y == 0)
    refit_beta<1>(o);
  else if (blockIdx.y == 1)
    refit_beta<2>(o);
  else
    refit_beta<3>(o);
}

struct RefitRtSmem {
  double red[4 * 40], sum[40];
  double ccs[36], cws[12], ci[9], pc0[9], pw0[3], R[27], t[9];
};

__global__ __launch_bounds__(256) void k_refit_rt(PnPObject* objs) {
  __shared__ RefitRtSmem S;
  PnPObject& o = objs[blockIdx.x];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (o.result[0] < 0) {
    if (tid == 0) {
      for (int i = 0; i < 9; i++) o.Rt[i] = (i % 4 == 0) ? 1.0 : 0.0;
      o.Rt[9] = o.Rt[10] = o.Rt[11] = 0.0;
    }
    return;
  }
  const int ni = o.result[3];
  for (int i = tid; i < 36; i += blockDim.x) S.ccs[i] = o.hout[(size_t)kHypOut * (i / 12) + i % 12];
  if (tid < 12) S.cws[tid] = o.hrec[R_AL + tid];
  if (tid < 9) S.ci[tid] = o.hrec[R_PW + tid];
  __syncthreads();
  const double fu = o.fx, fv = o.fy, uc = o.cx, vc = o.cy;
  auto pcs = [&](int k, int var, double* pc) {
    double a[4];
    refit_alphas(o, k, S.cws, S.ci, a);
    const double* c = S.ccs + 12 * var;
    for (int j = 0; j < 3; j++) pc[j] = a[0] * c[j] + a[1] * c[3 + j] + a[2] * c[6 + j] + a[3] * c[9 + j];
  };
  {  // centroids of the three camera-frame point sets and of the world points
    double v[12];
#pragma unroll
    for (int i = 0; i < 12; i++) v[i] = 0;
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3];
      refit_pw(o, k, p);
#pragma unroll
      for (int var = 0; var < 3; var++) {
        double pc[3];
        pcs(k, var, pc);
#pragma unroll
        for (int j = 0; j < 3; j++) v[3 * var + j] += pc[j];
      }
#pragma unroll
      for (int j = 0; j < 3; j++) v[9 + j] += p[j];
    }
    wg_sum<12>(v, S.red, S.sum);
    if (tid < 9) S.pc0[tid] = S.sum[tid] / ni;
    if (tid < 3) S.pw0[tid] = S.sum[9 + tid] / ni;
    __syncthreads();
  }
  {  // cross-covariances, then one Procrustes solve per wave
    double v[27];
#pragma unroll
    for (int i = 0; i < 27; i++) v[i] = 0;
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3];
      refit_pw(o, k, p);
#pragma unroll
      for (int var = 0; var < 3; var++) {
        double pc[3];
        pcs(k, var, pc);
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
          for (int q = 0; q < 3; q++)
            v[9 * var + 3 * j + q] += (pc[j] - S.pc0[3 * var + j]) * (p[q] - S.pw0[q]);
      }
    }
    wg_sum<27>(v, S.red, S.sum);
    if (lane == 0 && wave < 3) {
      double abt[9], R[9];
#pragma unroll
      for (int i = 0; i < 9; i++) abt[i] = S.sum[9 * wave + i];
      procrustes_R(abt, R);
#pragma unroll
      for (int i = 0; i < 9; i++) S.R[9 * wave + i] = R[i];
#pragma unroll
      for (int r = 0; r < 3; r++) S.t[3 * wave + r] = S.pc0[3 * wave + r] - d_dot3(R + 3 * r, S.pw0);
    }
    __syncthreads();
  }
  {  // reprojection errors, best estimate
    double v[3] = {0, 0, 0};
    for (int k = tid; k < ni; k += blockDim.x) {
      double p[3], u, vv;
      refit_pw(o, k, p);
      refit_us(o, k, u, vv);
#pragma unroll
      for (int var = 0; var < 3; var++) {
        const double* R = S.R + 9 * var;
        const double* t = S.t + 3 * var;
        const double Xc = d_dot3(R, p) + t[0], Yc = d_dot3(R + 3, p) + t[1];
        const double inv_Zc = 1.0 / (d_dot3(R + 6, p) + t[2]);
        const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
        v[var] += sqrt((u - ue) * (u - ue) + (vv - ve) * (vv - ve));
      }
    }
    wg_sum<3>(v, S.red, S.sum);
    if (tid == 0) {
      int best = 0;
      if (S.sum[1] / ni < S.sum[0] / ni) best = 1;
      if (S.sum[2] / ni < S.sum[best] / ni) best = 2;
      double rv[3], R[9];
      if (o.rt_raw) {  // D6: compute_pose's R as it is (no Rodrigues round trip)
        for (int i = 0; i < 9; i++) R[i] = S.R[9 * best + i];
      } else {
        d_rodrigues_r2v(S.R + 9 * best, rv);
        d_rodrigues_v2r(rv, R);
      }
      for (int i = 0; i < 9; i++) o.Rt[i] = R[i];
      for (int i = 0; i < 3; i++) o.Rt[9 + i] = S.t[3 * best + i];
    }
  }
}

// motion-model inliers (pnp_mm_inliers_block, mmt_pnp.h), one workgroup per object
__global__ __launch_bounds__(256) void k_mm_inliers(PnPObject* objs) {
  pnp_mm_inliers_block(objs[blockIdx.x]);
}

// D3 edge index list (pnp_subset_block, mmt_pnp.h), one workgroup per object
__global__ __launch_bounds__(256) void k_pnp_subset(PnPObject* objs) {
  pnp_subset_block(objs[blockIdx.x]);
}

// ---------------------------------------------------------------- D6: PnPsolver (P4P RANSAC)
// PnPsolver::CheckInliers (PnPsolver.cc:310-337) for the pose R, t (double): camera coordinates
// and 1/Zc rounded to float, the projection in double, the squared error in float against
// mvMaxError (strict)
__device__ __forceinline__ bool p4p_inlier(const PnPObject& o, const double* R, const double* t,
                                           int i) {
  const double X = o.pts3[3 * i], Y = o.pts3[3 * i + 1], Z = o.pts3[3 * i + 2];
  const float Xc = (float)(R[0] * X + R[1] * Y + R[2] * Z + t[0]);
  const float Yc = (float)(R[3] * X + R[4] * Y + R[5] * Z + t[1]);
  const float invZc = (float)(1 / (R[6] * X + R[7] * Y + R[8] * Z + t[2]));
  const double ue = (double)o.cx + (double)o.fx * (double)Xc * (double)invZc;
  const double ve = (double)o.cy + (double)o.fy * (double)Yc * (double)invZc;
  const float2 q = o.pts2[i];
  const float distX = (float)((double)q.x - ue), distY = (float)((double)q.y - ve);
  const float error2 = distX * distX + distY * distY;
  return error2 < o.max_err[i];
}

// inlier count + mask of pose (R, t) into masks row `row`; block-wide, 256 threads
__device__ int p4p_check(PnPObject& o, const double* R, const double* t, int row, int* s_w) {
  const int n = *o.n;
  int good = 0;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const bool in = i < n && p4p_inlier(o, R, t, i);
    const unsigned long long bal = __ballot(in);
    if ((threadIdx.x & 63) == 0 && i0 + (threadIdx.x & ~63) < n)
      o.masks[(size_t)row * o.mask_words + (i0 + (threadIdx.x & ~63)) / 64] = bal;
    good += in ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) good += __shfl_xor(good, off, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = good;
  __syncthreads();
  return s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// one workgroup per hypothesis: compute_pose's choice among the three beta estimates
// (rep_errors[2] < [1]; [3] < [N]), then CheckInliers
__global__ __launch_bounds__(256) void k_p4p_check(PnPObject* objs, int K) {
  __shared__ double sRt[12];
  __shared__ int s_w[4];
  PnPObject& o = objs[0];
  const int h = blockIdx.x;
  if (h >= K || *o.n < 4) return;
  if (threadIdx.x == 0) {
    const double* out = o.hout + (size_t)kHypOut * 3 * h;
    int best = 0;
    if (out[kHypOut] < out[0]) best = 1;
    if (out[2 * kHypOut] < out[best * kHypOut]) best = 2;
    const double* bo = out + best * kHypOut;
    for (int i = 0; i < 12; i++) {
      sRt[i] = bo[1 + i];
      o.hrt[12 * h + i] = bo[1 + i];
    }
  }
  __syncthreads();
  const int good = p4p_check(o, sRt, sRt + 9, h, s_w);
  if (threadIdx.x == 0) o.good[h] = good;
}

// CheckInliers of the refined pose o.Rt
__global__ __launch_bounds__(256) void k_p4p_check_rt(PnPObject* objs, int row_out) {
  __shared__ double sRt[12];
  __shared__ int s_w[4];
  PnPObject& o = objs[0];
  if (threadIdx.x < 12) sRt[threadIdx.x] = o.Rt[threadIdx.x];
  __syncthreads();
  const int good = p4p_check(o, sRt, sRt + 9, row_out, s_w);
  if (threadIdx.x == 0) o.result[6] = good;
}

__global__ void k_p4p_set_row(PnPObject* objs, int row) {
  if (threadIdx.x == 0) objs[0].result[0] = row;
}

void launch_p4p_hypotheses(PnPObject* d_obj, int K, hipStream_t st) {
  hipLaunchKernelGGL(k_pnp_hyp<4>, dim3((K + kHypPerBlock - 1) / kHypPerBlock, 1), dim3(64), 0,
                     st, d_obj, K);
  hipLaunchKernelGGL(k_pnp_beta<4>, dim3((K + 63) / 64, 1, 3), dim3(64), 0, st, d_obj, K);
  hipLaunchKernelGGL(k_p4p_check, dim3(K), dim3(256), 0, st, d_obj, K);
}

void launch_p4p_refine(PnPObject* d_obj, int row, int row_out, hipStream_t st) {
  hipLaunchKernelGGL(k_p4p_set_row, dim3(1), dim3(64), 0, st, d_obj, row);
  hipLaunchKernelGGL(k_refit_null, dim3(1), dim3(256), 0, st, d_obj);
  hipLaunchKernelGGL(k_refit_beta, dim3(1, 3), dim3(64), 0, st, d_obj);
  hipLaunchKernelGGL(k_refit_rt, dim3(1), dim3(256), 0, st, d_obj);
  hipLaunchKernelGGL(k_p4p_check_rt, dim3(1), dim3(256), 0, st, d_obj, row_out);
}

void launch_pnp(PnPObject* d_objs, int nobj, int max_iters, hipStream_t st, bool gather) {
  if (gather) hipLaunchKernelGGL(k_pnp_gather, dim3(nobj), dim3(256), 0, st, d_objs);
  hipLaunchKernelGGL(k_pnp_hyp<5>, dim3((max_iters + kHypPerBlock - 1) / kHypPerBlock, nobj),
                     dim3(64), 0, st, d_objs, max_iters);
  hipLaunchKernelGGL(k_pnp_beta<5>, dim3((max_iters + 63) / 64, nobj, 3), dim3(64), 0, st, d_objs,
                     max_iters);
  hipLaunchKernelGGL(k_pnp_score, dim3(max_iters, nobj), dim3(256), 0, st, d_objs, max_iters);
  hipLaunchKernelGGL(k_pnp_select, dim3(nobj), dim3(64), 0, st, d_objs, max_iters);
  hipLaunchKernelGGL(k_refit_null, dim3(nobj), dim3(256), 0, st, d_objs);
  hipLaunchKernelGGL(k_refit_beta, dim3(nobj, 3), dim3(64), 0, st, d_objs);
  hipLaunchKernelGGL(k_refit_rt, dim3(nobj), dim3(256), 0, st, d_objs);
}

void launch_pnp_mm(PnPObject* d_objs, int nobj, hipStream_t st) {
  hipLaunchKernelGGL(k_mm_inliers, dim3(nobj), dim3(256), 0, st, d_objs);
}

void launch_pnp_subset(PnPObject* d_objs, int nobj, hipStream_t st) {
  hipLaunchKernelGGL(k_pnp_subset, dim3(nobj), dim3(256), 0, st, d_objs);
}

}  // namespace mmt
