// multimot_track_amd/csrc/mmt_devmath.h -- double-precision SE(3) / small dense algebra for the
// pose-solve kernels, written for one lane (uniform values held in LDS by the caller).
// Semantics follow g2o's SE3Quat (Thirdparty/g2o/g2o/types/se3quat.h) and Eigen's quaternion
// conversions, which the reference solves run on.
#pragma once
#include <hip/hip_runtime.h>

namespace mmt {

struct DQuat {
  double x, y, z, w;
};
struct DSE3 {
  DQuat q;
  double t[3];
};

__device__ __forceinline__ void dq_normalize_rot(DQuat& q) {
  if (q.w < 0) {
    q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
  }
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

// Eigen::Quaternion(const Matrix3&): trace branch, else largest-diagonal branch.
__device__ inline DQuat dq_from_R(const double R[3][3]) {
  DQuat q;
  const double t = R[0][0] + R[1][1] + R[2][2];
  if (t > 0) {
    double s = sqrt(t + 1.0);
    q.w = 0.5 * s;
    s = 0.5 / s;
    q.x = (R[2][1] - R[1][2]) * s;
    q.y = (R[0][2] - R[2][0]) * s;
    q.z = (R[1][0] - R[0][1]) * s;
  } else {
    int i = 0;
    if (R[1][1] > R[0][0]) i = 1;
    if (R[2][2] > R[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double s = sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
    double v[3];
    v[i] = 0.5 * s;
    s = 0.5 / s;
    q.w = (R[k][j] - R[j][k]) * s;
    v[j] = (R[j][i] + R[i][j]) * s;
    v[k] = (R[k][i] + R[i][k]) * s;
    q.x = v[0]; q.y = v[1]; q.z = v[2];
  }
  return q;
}

__device__ __forceinline__ void dq_to_R(const DQuat& q, double R[3][3]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz;       R[0][2] = txz + twy;
  R[1][0] = txy + twz;       R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy;       R[2][1] = tyz + twx;       R[2][2] = 1 - (txx + tyy);
}

// q * v, Eigen's _transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv
__device__ __forceinline__ void dq_rotate(const DQuat& q, double vx, double vy, double vz,
                                          double& ox, double& oy, double& oz) {
  double ux = q.y * vz - q.z * vy, uy = q.z * vx - q.x * vz, uz = q.x * vy - q.y * vx;
  ux += ux; uy += uy; uz += uz;
  const double cx = q.y * uz - q.z * uy, cy = q.z * ux - q.x * uz, cz = q.x * uy - q.y * ux;
  ox = vx + q.w * ux + cx;
  oy = vy + q.w * uy + cy;
  oz = vz + q.w * uz + cz;
}

__device__ __forceinline__ DQuat dq_mul(const DQuat& a, const DQuat& b) {
  DQuat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

__device__ inline DSE3 dse3_from_float(const float* T) {  // Converter::toSE3Quat
  double R[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[r][c] = (double)T[4 * r + c];
  DSE3 s;
  s.q = dq_from_R(R);
  dq_normalize_rot(s.q);
  s.t[0] = T[3]; s.t[1] = T[7]; s.t[2] = T[11];
  return s;
}

__device__ inline void dse3_to_float(const DSE3& s, float* T) {  // Converter::toCvMat
  double R[3][3];
  dq_to_R(s.q, R);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[r][c];
    T[4 * r + 3] = (float)s.t[r];
  }
  T[12] = 0.f; T[13] = 0.f; T[14] = 0.f; T[15] = 1.f;
}

__device__ inline DSE3 dse3_exp(const double u[6]) {  // SE3Quat::exp
  const double o0 = u[0], o1 = u[1], o2 = u[2];
  const double theta = sqrt(o0 * o0 + o1 * o1 + o2 * o2);
  const double O[3][3] = {{0, -o2, o1}, {o2, 0, -o0}, {-o1, o0, 0}};
  double O2[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) O2[r][c] = O[r][0] * O[0][c] + O[r][1] * O[1][c] + O[r][2] * O[2][c];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + O[r][c] + O2[r][c];
        V[r][c] = R[r][c];
      }
  } else {
    const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
    const double c2 = (theta - sin(theta)) / (theta * theta * theta);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + a * O[r][c] + b * O2[r][c];
        V[r][c] = (r == c ? 1.0 : 0.0) + b * O[r][c] + c2 * O2[r][c];
      }
  }
  DSE3 s;
  s.q = dq_from_R(R);
  for (int r = 0; r < 3; r++) s.t[r] = V[r][0] * u[3] + V[r][1] * u[4] + V[r][2] * u[5];
  dq_normalize_rot(s.q);
  return s;
}

__device__ inline DSE3 dse3_mul(const DSE3& a, const DSE3& b) {
  DSE3 r;
  double x, y, z;
  dq_rotate(a.q, b.t[0], b.t[1], b.t[2], x, y, z);
  r.t[0] = a.t[0] + x;
  r.t[1] = a.t[1] + y;
  r.t[2] = a.t[2] + z;
  r.q = dq_mul(a.q, b.q);
  dq_normalize_rot(r.q);
  return r;
}

// 6x6 LDLT with symmetric diagonal pivoting on the LOWER triangle (Eigen LDLT<MatrixXd>).
// Returns false when not positive (LDLT::isPositive()).
__device__ inline bool ldlt_solve6(const double* Hl /*row-major 6x6, lower used*/, const double* b,
                                   double* x) {
  double A[6][6];
  for (int r = 0; r < 6; r++)
    for (int c = 0; c < 6; c++) A[r][c] = (c <= r) ? Hl[6 * r + c] : Hl[6 * c + r];
  int perm[6] = {0, 1, 2, 3, 4, 5};
  double D[6];
  double L[6][6];
  for (int r = 0; r < 6; r++)
    for (int c = 0; c < 6; c++) L[r][c] = 0.0;
  bool positive = true;
  for (int k = 0; k < 6; k++) {
    int p = k;
    double best = fabs(A[k][k]);
    for (int i = k + 1; i < 6; i++)
      if (fabs(A[i][i]) > best) {
        best = fabs(A[i][i]);
        p = i;
      }
    if (p != k) {
      for (int c = 0; c < 6; c++) {
        const double t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t;
      }
      for (int r = 0; r < 6; r++) {
        const double t = A[r][k]; A[r][k] = A[r][p]; A[r][p] = t;
      }
      for (int c = 0; c < k; c++) {
        const double t = L[k][c]; L[k][c] = L[p][c]; L[p][c] = t;
      }
      const int t = perm[k]; perm[k] = perm[p]; perm[p] = t;
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

// Workgroup sum of K doubles held per thread; result broadcast in `out` (LDS, K entries).
// `scratch` holds (blockDim/64) * K doubles.
template <int K>
__device__ inline void wg_sum(double (&v)[K], double* scratch, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; k++) {
    double s = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    v[k] = s;
  }
  if (lane == 0)
    for (int k = 0; k < K; k++) scratch[wave * K + k] = v[k];
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    double s = 0;
    for (int w = 0; w < nw; w++) s += scratch[w * K + k];
    out[k] = s;
  }
  __syncthreads();
}

}  // namespace mmt
