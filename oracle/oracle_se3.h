// oracle/oracle_se3.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
//
// g2o::SE3Quat (Thirdparty/g2o/g2o/types/se3quat.h) and the Converter float <-> SE3Quat round
// trip (src/Converter.cc:37-69), shared by the pose solves (solve_ref.cpp) and the local bundle
// adjustment (ba_ref.cpp).  Double precision, as Eigen.
#pragma once
#include <cmath>
#include <cstring>

namespace oracle {

// ------------------------------------------------------------------ SE3Quat (se3quat.h)
struct Quat {
  double x, y, z, w;
};
struct SE3 {
  Quat q;
  double t[3];
};

static inline void quat_normalize_rot(Quat& q) {  // SE3Quat::normalizeRotation
  if (q.w < 0) {
    q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
  }
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

static inline Quat quat_from_R(const double R[3][3]) {  // Eigen::Quaternion(const Matrix3&)
  Quat q;
  const double t = R[0][0] + R[1][1] + R[2][2];
  if (t > 0) {
    double s = std::sqrt(t + 1.0);
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
    double s = std::sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
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

static inline void quat_to_R(const Quat& q, double R[3][3]) {  // Eigen toRotationMatrix
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz;       R[0][2] = txz + twy;
  R[1][0] = txy + twz;       R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy;       R[2][1] = tyz + twx;       R[2][2] = 1 - (txx + tyy);
}

static inline void quat_rotate(const Quat& q, const double v[3], double out[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  for (int k = 0; k < 3; k++) out[k] = v[k] + q.w * uv[k] + c[k];
}

static inline Quat quat_mul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

static inline SE3 se3_from_float(const float T[16]) {  // Converter::toSE3Quat
  double R[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[r][c] = (double)T[4 * r + c];
  SE3 s;
  s.q = quat_from_R(R);
  quat_normalize_rot(s.q);
  s.t[0] = T[3]; s.t[1] = T[7]; s.t[2] = T[11];
  return s;
}

static inline void se3_to_float(const SE3& s, float T[16]) {  // Converter::toCvMat(SE3Quat)
  double R[3][3];
  quat_to_R(s.q, R);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[r][c];
    T[4 * r + 3] = (float)s.t[r];
  }
  T[12] = T[13] = T[14] = 0.f;
  T[15] = 1.f;
}

static inline SE3 se3_exp(const double u[6]) {  // SE3Quat::exp
  const double om[3] = {u[0], u[1], u[2]};
  const double up[3] = {u[3], u[4], u[5]};
  const double theta = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
  double O[3][3] = {{0, -om[2], om[1]}, {om[2], 0, -om[0]}, {-om[1], om[0], 0}};
  double O2[3][3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += O[r][k] * O[k][c];
      O2[r][c] = s;
    }
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) R[r][c] = (r == c ? 1.0 : 0.0) + O[r][c] + O2[r][c];
    memcpy(V, R, sizeof(R));
  } else {
    const double a = std::sin(theta) / theta, b = (1 - std::cos(theta)) / (theta * theta);
    const double c2 = (theta - std::sin(theta)) / std::pow(theta, 3);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + a * O[r][c] + b * O2[r][c];
        V[r][c] = (r == c ? 1.0 : 0.0) + b * O[r][c] + c2 * O2[r][c];
      }
  }
  SE3 s;
  s.q = quat_from_R(R);
  for (int r = 0; r < 3; r++) s.t[r] = V[r][0] * up[0] + V[r][1] * up[1] + V[r][2] * up[2];
  quat_normalize_rot(s.q);  // SE3Quat(const Quaterniond&, const Vector3d&) normalises
  return s;
}

static inline SE3 se3_mul(const SE3& a, const SE3& b) {  // SE3Quat::operator*
  SE3 r;
  double rt[3];
  quat_rotate(a.q, b.t, rt);
  for (int k = 0; k < 3; k++) r.t[k] = a.t[k] + rt[k];
  r.q = quat_mul(a.q, b.q);
  quat_normalize_rot(r.q);
  return r;
}

static inline void se3_map(const SE3& s, const double X[3], double out[3]) {
  quat_rotate(s.q, X, out);
  for (int k = 0; k < 3; k++) out[k] += s.t[k];
}

}  // namespace oracle
