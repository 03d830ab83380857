// multimot_track_amd/csrc/mmt_lm.hip -- D2 / D3: the flow-refined pose solves.
//
// Optimizer::PoseOptimizationFlow2Cam (ego, reference src/Optimizer.cc:396-601) and
// Optimizer::PoseOptimizationFlow2 (objects, Optimizer.cc:2170-2377): one SE(3) vertex plus one
// 2-D "flow" vertex per correspondence, EdgeFlowCamera/EdgeFlowObj (Huber, information 0.1) and a
// flow prior per correspondence, solved by g2o's Levenberg-Marquardt with the Schur complement over
// the flow vertices.  The g2o behaviour reproduced here (CPU restatement in
// oracle/solve_ref.cpp): LM damping init 1e-5 * max diagonal, rho/alpha update with the 1e-3 scale
// term, ni doubling, 10 trials, stale-x update when the LDLT fails, "Raul" stop after three
// iterations with under 0.1 % gain, the chi2-increase stop on the last trial's chi2, the landmark
// back-substitution with the stride-2 spill term, inliers from the last evaluated errors.
//
// One workgroup per solve (ego + every object of a frame in one launch), fp64.  Per-correspondence
// state lives in registers (IR items per thread; items beyond IR * blockDim spill to the global
// scratch arrays).  An LM trial is
//   Schur pass   J^T W J terms of the Schur complement (27 sums; only when some edge is
//                Huber-active, otherwise closed form from the current system's sums)
//   6x6 solve    computed redundantly by every thread from the sums
//   pass 1       flow back-substitution and the trial's errors: chi2 and the scale term (2 sums)
//   pass 2       accepted trials only: the flow step and the linearisation at the new state
//                (H, b and the closed-form Schur sums: 63 sums), the next trial's system
// so a rejected trial costs one light pass and a DPP reduction of two sums.  The 63-sum reductions
// go through an LDS transpose tile (mmt_devmath.h: block_sum_tile_lanes).  Sums are reduced in a
// different order than the CPU checker's sequential loops, so poses agree to rounding (1e-4 bar),
// not bit for bit.

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdio>
#include <cstdlib>

#include <algorithm>

#include "mmt_devmath.h"
#include "mmt_internal.h"
#include "mmt_track.h"

namespace mmt {

namespace {

constexpr double kInfo = 0.1;  // info_flow (Optimizer.cc:466 / 2241)

struct LMItem {
  double X[3];      // world point of the last frame's sample (Twl * unprojection)
  double ob[2];     // measurement: last-frame pixel
  double pr[2];     // flow prior
  double f[2];      // flow vertex estimate
  double xl[2];     // last flow increment (reused when the 6x6 solve fails)
  double w, bl[2];  // robust weight, landmark gradient at the current state
  double e[2];      // errors of the last evaluated state
};

enum { G_X0 = 0, G_X1, G_X2, G_OB0, G_OB1, G_PR0, G_PR1, G_F0, G_F1, G_XL0, G_XL1, G_W, G_BL0,
       G_BL1, G_E0, G_E1, G_COUNT };

__device__ __forceinline__ void item_load(const double* S, int cap, int i, LMItem& it) {
  double* d = &it.X[0];
  const double* src = S + i;
#pragma unroll
  for (int k = 0; k < G_COUNT; k++) d[k] = src[(size_t)k * cap];
}

__device__ __forceinline__ void item_store(double* S, int cap, int i, const LMItem& it) {
  const double* d = &it.X[0];
  double* dst = S + i;
#pragma unroll
  for (int k = 0; k < G_COUNT; k++) dst[(size_t)k * cap] = d[k];
}

static_assert(sizeof(LMItem) == G_COUNT * sizeof(double), "LMItem layout");

// the fields a trial changes (xl, e)
__device__ __forceinline__ void item_store_trial(double* S, int cap, int i, const LMItem& it) {
  double* dst = S + i;
  dst[(size_t)G_XL0 * cap] = it.xl[0];
  dst[(size_t)G_XL1 * cap] = it.xl[1];
  dst[(size_t)G_E0 * cap] = it.e[0];
  dst[(size_t)G_E1 * cap] = it.e[1];
}

// the fields an accepted trial changes (f, w, bl)
__device__ __forceinline__ void item_store_accept(double* S, int cap, int i, const LMItem& it) {
  double* dst = S + i;
  dst[(size_t)G_F0 * cap] = it.f[0];
  dst[(size_t)G_F1 * cap] = it.f[1];
  dst[(size_t)G_W * cap] = it.w;
  dst[(size_t)G_BL0 * cap] = it.bl[0];
  dst[(size_t)G_BL1 * cap] = it.bl[1];
}

// 1/x and 1/sqrt(x) from the hardware estimates plus two Newton steps (within an ulp of the
// correctly rounded result; the LM path is compared to the checker within 1e-4, not bitwise).
// They replace fp64 division/sqrt sequences on the per-trial dependency chains.
__device__ __forceinline__ double drcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

__device__ __forceinline__ double drsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double h = 0.5 * x * y;
  double e = fma(-h, y, 0.5);
  y = fma(y, e, y);
  h = 0.5 * x * y;
  e = fma(-h, y, 0.5);
  return fma(y, e, y);
}

__device__ __forceinline__ void huber(double e, double dsqr, double delta, double& r0, double& r1) {
  if (e <= dsqr) {
    r0 = e;
    r1 = 1.;
  } else {
    const double rs = drsq(e);
    const double s = e * rs;
    r0 = 2 * s * delta - dsqr;
    r1 = delta * rs;
  }
}

__device__ __forceinline__ void normalize_rot(DQuat& q) {
  if (q.w < 0) {
    q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
  }
  const double in = drsq(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x *= in; q.y *= in; q.z *= in; q.w *= in;
}

// SE3Quat::exp (g2o, as mmt_devmath.h dse3_exp) times P, on the solve's critical path.  g2o
// builds R by Rodrigues and converts it to a quaternion; below the sincos regime this computes the
// same rotation directly as (cos(t/2), w sin(t/2)/t) and V u through two cross products, with the
// half-angle and V coefficients as truncated series for t < 0.05 (remainder < 1e-20): equal to the
// matrix route up to rounding.  g2o's t < 1e-5 quirk (R = I + O + O^2, V = R) and the sincos
// regime keep the matrix route.
__device__ __forceinline__ DSE3 exp_mul(const double (&u)[6], const DSE3& P) {
  const double o0 = u[0], o1 = u[1], o2 = u[2];
  const double th2 = o0 * o0 + o1 * o1 + o2 * o2;
  DSE3 s;
  if (th2 >= 1e-10 && th2 < 0.0025) {
    const double x = th2;
    constexpr double c8 = 1.0 / 8, c48 = 1.0 / 48, c6 = 1.0 / 6, c24 = 1.0 / 24;
    constexpr double k20 = 1.0 / 20, k42 = 1.0 / 42, k72 = 1.0 / 72, k30 = 1.0 / 30;
    constexpr double k56 = 1.0 / 56, k90 = 1.0 / 90, k120 = 1.0 / 120, k110 = 1.0 / 110;
    // cos(t/2) = 1 - x/8 (1 - x/48 (1 - x/120 (1 - x/224)))
    const double cw = 1.0 - x * c8 * (1.0 - x * c48 * (1.0 - x * k120 * (1.0 - x * (1.0 / 224))));
    // sin(t/2)/t = 1/2 (1 - x/24 (1 - x/80 (1 - x/168 (1 - x/288))))
    const double sh = 0.5 * (1.0 - x * c24 * (1.0 - x * (1.0 / 80) * (1.0 - x * (1.0 / 168) *
                                                                       (1.0 - x * (1.0 / 288)))));
    const double b = 0.5 - x * c24 * (1.0 - x * k30 * (1.0 - x * k56 * (1.0 - x * k90)));
    const double c2 = c6 - x * k120 * (1.0 - x * k42 * (1.0 - x * k72 * (1.0 - x * k110)));
    (void)k20;
    s.q.w = cw;
    s.q.x = o0 * sh;
    s.q.y = o1 * sh;
    s.q.z = o2 * sh;
    // V u = u + b (w x u) + c2 (w x (w x u))
    const double v0 = u[3], v1 = u[4], v2 = u[5];
    const double a0 = o1 * v2 - o2 * v1, a1 = o2 * v0 - o0 * v2, a2 = o0 * v1 - o1 * v0;
    const double e0 = o1 * a2 - o2 * a1, e1 = o2 * a0 - o0 * a2, e2 = o0 * a1 - o1 * a0;
    s.t[0] = v0 + b * a0 + c2 * e0;
    s.t[1] = v1 + b * a1 + c2 * e1;
    s.t[2] = v2 + b * a2 + c2 * e2;
  } else if (th2 < 1e-10) {
    // g2o's quirk: R = I + O + O^2 (O^2 = w w^T - t^2 I), V = R; Quaternion(R) on the trace
    // branch (tr = 3 - 2 t^2 > 0): w = sqrt(1 + tr) / 2, v = (R21 - R12, ...) / (4 w) = w_vec / (2 w)
    const double tr = 3.0 - 2.0 * th2;
    const double rs = drsq(tr + 1.0);
    s.q.w = 0.5 * (tr + 1.0) * rs;
    const double h = rs;  // 1 / (2 w) = 1 / sqrt(1 + tr)
    s.q.x = o0 * h;
    s.q.y = o1 * h;
    s.q.z = o2 * h;
    const double v0 = u[3], v1 = u[4], v2 = u[5];
    const double a0 = o1 * v2 - o2 * v1, a1 = o2 * v0 - o0 * v2, a2 = o0 * v1 - o1 * v0;
    const double e0 = o1 * a2 - o2 * a1, e1 = o2 * a0 - o0 * a2, e2 = o0 * a1 - o1 * a0;
    s.t[0] = v0 + a0 + e0;
    s.t[1] = v1 + a1 + e1;
    s.t[2] = v2 + a2 + e2;
    normalize_rot(s.q);
  } else {
    const double O[3][3] = {{0, -o2, o1}, {o2, 0, -o0}, {-o1, o0, 0}};
    double O2[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++)
        O2[r][c] = O[r][0] * O[0][c] + O[r][1] * O[1][c] + O[r][2] * O[2][c];
    double a, b, c2;
    if (th2 < 1e-10) {
      a = 1.0;
      b = 1.0;
      c2 = 1.0;
    } else {
      const double th = sqrt(th2);
      double st, ct;
      sincos(th, &st, &ct);
      const double it = drcp(th), it2 = it * it;
      a = st * it;
      b = (1 - ct) * it2;
      c2 = (th - st) * it2 * it;
    }
    double R[3][3], V[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + a * O[r][c] + b * O2[r][c];
        V[r][c] = th2 < 1e-10 ? R[r][c] : (r == c ? 1.0 : 0.0) + b * O[r][c] + c2 * O2[r][c];
      }
    const double tr = R[0][0] + R[1][1] + R[2][2];
    if (tr > 0) {
      const double rs = drsq(tr + 1.0);
      s.q.w = 0.5 * (tr + 1.0) * rs;
      const double h = 0.5 * rs;
      s.q.x = (R[2][1] - R[1][2]) * h;
      s.q.y = (R[0][2] - R[2][0]) * h;
      s.q.z = (R[1][0] - R[0][1]) * h;
    } else {
      s.q = dq_from_R(R);
    }
#pragma unroll
    for (int r = 0; r < 3; r++) s.t[r] = V[r][0] * u[3] + V[r][1] * u[4] + V[r][2] * u[5];
    normalize_rot(s.q);
  }
  // dse3_mul(s, P)
  DSE3 out;
  double x, y, z;
  dq_rotate(s.q, P.t[0], P.t[1], P.t[2], x, y, z);
  out.t[0] = s.t[0] + x;
  out.t[1] = s.t[1] + y;
  out.t[2] = s.t[2] + z;
  out.q = dq_mul(s.q, P.q);
  normalize_rot(out.q);
  return out;
}

// projection Jacobian of EdgeFlowCamera / EdgeFlowObj (g2o's EdgeSE3ProjectXYZ form) at the
// camera-frame point (x, y, z), written with one reciprocal of z instead of nine divisions
__device__ __forceinline__ void jac(double x, double y, double iz, double fx, double fy,
                                    double J[2][6]) {
  const double iz2 = iz * iz;
  const double xx = x * x * iz2, yy = y * y * iz2, xy = x * y * iz2;
  J[0][0] = xy * fx;
  J[0][1] = -(1 + xx) * fx;
  J[0][2] = y * iz * fx;
  J[0][3] = -iz * fx;
  J[0][4] = 0;
  J[0][5] = x * iz2 * fx;
  J[1][0] = (1 + yy) * fy;
  J[1][1] = -xy * fy;
  J[1][2] = -x * iz * fy;
  J[1][3] = 0;
  J[1][4] = -iz * fy;
  J[1][5] = y * iz2 * fy;
}

__device__ __forceinline__ void map(const DSE3& p, const double* X, double& x, double& y,
                                    double& z) {
  dq_rotate(p.q, X[0], X[1], X[2], x, y, z);
  x += p.t[0];
  y += p.t[1];
  z += p.t[2];
}

struct Cam {
  double fx, fy, cx, cy, pinfo, dsqr, delta;
};

// sums of one linearisation: [0] chi2, [1] scale term (trial only), [2..22] lower triangle of
// J^T W J, [23..28] J^T W (-e), [29] Huber-active edge count, [30..50] sum B0a (B0b + B1b),
// [51..56] sum B0a (bl0 + bl1), [57..62] sum (B1a - B0a) bl1 (B = w J)
constexpr int kSums = 63;
constexpr int kCandStride = 16;  // doubles per candidate solve in LMSmem::cand

// linearise at (P, flow fl): errors, robust weight and landmark gradient of the edge; its sums
// (layout at kSums) go straight into `row`, this thread's row of the LDS reduction tile
// (block_sum_tile): stored by the thread's first edge (FIRST), accumulated by the others.  No sum
// lives in registers, which keeps the kernel clear of spills.
template <bool FIRST>
__device__ __forceinline__ void put(double* row, int q, double v) {
  if (FIRST)
    row[q] = v;
  else
    row[q] += v;
}

template <bool FIRST>
__device__ __forceinline__ void linearise(const Cam& c, const DSE3& P, const LMItem& it,
                                          const double f0, const double f1, double* row,
                                          double scale_term, double& e0, double& e1, double& w,
                                          double& bl0, double& bl1, double& mh,
                                          double* Bout = nullptr) {
  double x, y, z;
  map(P, it.X, x, y, z);
  const double iz = drcp(z);
  const double pu = x * iz * c.fx + c.cx, pv = y * iz * c.fy + c.cy;
  e0 = (it.ob[0] + f0) - pu;
  e1 = (it.ob[1] + f1) - pv;
  const double p0 = f0 - it.pr[0], p1 = f1 - it.pr[1];
  const double e2 = kInfo * (e0 * e0 + e1 * e1);
  double r0, r1;
  huber(e2, c.dsqr, c.delta, r0, r1);
  put<FIRST>(row, 0, r0 + c.pinfo * (p0 * p0 + p1 * p1));
  put<FIRST>(row, 1, scale_term);
  w = kInfo * r1;
  put<FIRST>(row, 29, w < kInfo ? 1.0 : 0.0);  // Huber-active
  double J[2][6];
  jac(x, y, iz, c.fx, c.fy, J);
  const double o0 = -w * e0, o1 = -w * e1;
  bl0 = o0 - c.pinfo * p0;
  bl1 = o1 - c.pinfo * p1;
  mh = fmax(mh, w + c.pinfo);
  double B0[6], B1[6];
#pragma unroll
  for (int a = 0; a < 6; a++) {
    B0[a] = w * J[0][a];
    B1[a] = w * J[1][a];
  }
  if (Bout) {
#pragma unroll
    for (int a = 0; a < 6; a++) {
      Bout[a] = B0[a];
      Bout[6 + a] = B1[a];
    }
  }
  // [2..22] J^T W J, [23..28] J^T W (-e); closed-form Schur sums (valid when every edge has the
  // same weight, see flow_lm_body), B = w J: [30..50] B0a (B0b + B1b), [51..56] B0a (bl0 + bl1),
  // [57..62] (B1a - B0a) bl1
  int k = 0;
#pragma unroll
  for (int a = 0; a < 6; a++) {
#pragma unroll
    for (int b = 0; b <= a; b++) {
      put<FIRST>(row, 2 + k, J[0][a] * w * J[0][b] + J[1][a] * w * J[1][b]);
      put<FIRST>(row, 30 + k, B0[a] * (B0[b] + B1[b]));
      k++;
    }
    put<FIRST>(row, 23 + a, J[0][a] * o0 + J[1][a] * o1);
    put<FIRST>(row, 51 + a, B0[a] * (bl0 + bl1));
    put<FIRST>(row, 57 + a, (B1[a] - B0[a]) * bl1);
  }
}

// Schur complement contributions of one correspondence at pose P with damping lam
__device__ __forceinline__ void schur_terms(const Cam& c, const DSE3& P, const LMItem& it,
                                            double lam, double ilam, double* v) {
  double x, y, z;
  map(P, it.X, x, y, z);
  double J[2][6];
  jac(x, y, drcp(z), c.fx, c.fy, J);
  const double w = it.w, h = w + c.pinfo;
  const double d00 = drcp(h + lam), d01 = -h * d00 * ilam, d11 = ilam;
  const double bl0 = it.bl[0], bl1 = it.bl[1];
  const double db0 = d00 * bl0 + d01 * bl1, db1 = d11 * bl1;
  int k = 0;
#pragma unroll
  for (int a = 0; a < 6; a++) {
    const double B0a = w * J[0][a], B1a = w * J[1][a];
    const double BD0 = B0a * d00, BD1 = B0a * d01 + B1a * d11;
#pragma unroll
    for (int b = 0; b <= a; b++) v[k++] += BD0 * (w * J[0][b]) + BD1 * (w * J[1][b]);
    v[21 + a] += B0a * db0 + B1a * db1;
  }
}

// pass 1 of a trial: back-substitution of the flow increment (when the 6x6 solve succeeded) and
// the errors at the trial state (PN, f + xl), accumulated into s_chi (the trial chi2 term) and
// s_sc (the scale term)
__device__ __forceinline__ void trial_terms(const Cam& c, const DSE3& P, const DSE3& PN,
                                            LMItem& it, int i, bool ok2, double lam, double ilam,
                                            const double* xb, double& s_chi, double& s_sc,
                                            const double* Bcur = nullptr) {
  const double bl0 = it.bl[0], bl1 = it.bl[1];
  if (ok2) {
    const double w = it.w, h = w + c.pinfo;
    double c0 = bl0, c1 = bl1;
    if (Bcur) {  // w J at P, kept from the linearisation that built the current system
#pragma unroll
      for (int a = 0; a < 6; a++) {
        c0 -= Bcur[a] * xb[a];
        c1 -= Bcur[6 + a] * xb[a];
      }
    } else {
      double x, y, z;
      map(P, it.X, x, y, z);
      double J[2][6];
      jac(x, y, drcp(z), c.fx, c.fy, J);
#pragma unroll
      for (int a = 0; a < 6; a++) {
        c0 -= w * J[0][a] * xb[a];
        c1 -= w * J[1][a] * xb[a];
      }
    }
    const double ihl = drcp(h + lam);
    double xl0 = c0 * ihl - h * c1 * ihl * ilam;
    if (i > 0) xl0 += c0 * ilam;  // stride-2 spill of landmark i-1's third Dinv row
    it.xl[0] = xl0;
    it.xl[1] = c1 * ilam;
  }
  const double xl0 = it.xl[0], xl1 = it.xl[1];
  const double f0 = it.f[0] + xl0, f1 = it.f[1] + xl1;
  double x, y, z;
  map(PN, it.X, x, y, z);
  const double iz = drcp(z);
  const double pu = x * iz * c.fx + c.cx, pv = y * iz * c.fy + c.cy;
  const double e0 = (it.ob[0] + f0) - pu;
  const double e1 = (it.ob[1] + f1) - pv;
  it.e[0] = e0;
  it.e[1] = e1;
  const double p0 = f0 - it.pr[0], p1 = f1 - it.pr[1];
  const double e2 = kInfo * (e0 * e0 + e1 * e1);
  double r0, r1;
  huber(e2, c.dsqr, c.delta, r0, r1);
  s_chi += r0 + c.pinfo * (p0 * p0 + p1 * p1);
  s_sc += xl0 * (lam * xl0 + bl0) + xl1 * (lam * xl1 + bl1);
}

// pass 2 (accepted trials only): the flow step is taken and the edge linearised at the new state
// (PN, f + xl), which builds the next iteration's system
template <bool FIRST>
__device__ __forceinline__ void accept_terms(const Cam& c, const DSE3& PN, LMItem& it, double* row,
                                             double* Bnext = nullptr) {
  it.f[0] += it.xl[0];
  it.f[1] += it.xl[1];
  double mh = 0;
  linearise<FIRST>(c, PN, it, it.f[0], it.f[1], row, 0.0, it.e[0], it.e[1], it.w, it.bl[0],
                   it.bl[1], mh, Bnext);
}

// the split solve's fused trial pass: back-substitution and errors as trial_terms, and the
// linearisation at the trial state (PN, f + xl) as the accepted trial's pass 2 would compute it,
// into the tile row: [0] the trial's chi2 term, [1] its scale term, the rest the system the next
// trial uses if this one is accepted.  The new robust weight, landmark gradient and w J stay
// pending (pw, pb, Bnext) until the decision; f, w and bl of the item are untouched.
template <bool FIRST>
__device__ __forceinline__ void spec_terms(const Cam& c, const DSE3& P, const DSE3& PN, LMItem& it,
                                           int i, bool ok2, double lam, double ilam,
                                           const double* xb, double* row, double& pw,
                                           double& pb0, double& pb1, const double* Bcur,
                                           double* Bnext) {
  const double bl0 = it.bl[0], bl1 = it.bl[1];
  if (ok2) {
    const double w = it.w, h = w + c.pinfo;
    double c0 = bl0, c1 = bl1;
    if (Bcur) {
#pragma unroll
      for (int a = 0; a < 6; a++) {
        c0 -= Bcur[a] * xb[a];
        c1 -= Bcur[6 + a] * xb[a];
      }
    } else {
      double x, y, z;
      map(P, it.X, x, y, z);
      double J[2][6];
      jac(x, y, drcp(z), c.fx, c.fy, J);
#pragma unroll
      for (int a = 0; a < 6; a++) {
        c0 -= w * J[0][a] * xb[a];
        c1 -= w * J[1][a] * xb[a];
      }
    }
    const double ihl = drcp(h + lam);
    double xl0 = c0 * ihl - h * c1 * ihl * ilam;
    if (i > 0) xl0 += c0 * ilam;  // stride-2 spill of landmark i-1's third Dinv row
    it.xl[0] = xl0;
    it.xl[1] = c1 * ilam;
  }
  const double xl0 = it.xl[0], xl1 = it.xl[1];
  const double sc = xl0 * (lam * xl0 + bl0) + xl1 * (lam * xl1 + bl1);
  double mh = 0;
  linearise<FIRST>(c, PN, it, it.f[0] + xl0, it.f[1] + xl1, row, sc, it.e[0], it.e[1], pw, pb0,
                   pb1, mh, Bnext);
}

#ifdef MMT_LM_PROFILE
#define MMT_LMPROF(k)                  \
  do {                                 \
    if (tid == 0) {                    \
      const long long now = clock64(); \
      sm.prof[k] += now - prof_t;      \
      prof_t = now;                    \
    }                                  \
  } while (0)
#else
#define MMT_LMPROF(k) \
  do {                \
  } while (0)
#endif

// 6x6 LDL^T of the (symmetric positive definite) Schur complement, unpivoted, in place on the
// packed lower triangle A[i(i+1)/2 + j] (L below the diagonal, D on it); false when a pivot is
// negative.  The reduced camera system H_pp + lambda I - B D^-1 B^T is SPD whenever lambda > 0,
// so the pivoting of Eigen's LDLT only moves rounding.  b is overwritten by the solution.
__device__ __forceinline__ bool ldlt6_packed(double (&A)[21], double (&b)[6]) {
#define PK(i, j) A[(i) * ((i) + 1) / 2 + (j)]
  bool positive = true;
  double ID[6];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    double LD[6];  // L(k, c) D(c)
#pragma unroll
    for (int c = 0; c < k; c++) LD[c] = PK(k, c) * PK(c, c);
    double d = PK(k, k);
#pragma unroll
    for (int c = 0; c < k; c++) d -= PK(k, c) * LD[c];
    PK(k, k) = d;
    positive = positive && !(d < 0);
    const double id = d != 0 ? drcp(d) : 0.0;
    ID[k] = id;
#pragma unroll
    for (int i = k + 1; i < 6; i++) {
      double s = PK(i, k);
#pragma unroll
      for (int c = 0; c < k; c++) s -= PK(i, c) * LD[c];
      PK(i, k) = s * id;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
#pragma unroll
    for (int c = 0; c < i; c++) b[i] -= PK(i, c) * b[c];
  }
#pragma unroll
  for (int i = 0; i < 6; i++) b[i] *= ID[i];
#pragma unroll
  for (int i = 5; i >= 0; i--) {
#pragma unroll
    for (int r = i + 1; r < 6; r++) b[i] -= PK(r, i) * b[r];
  }
#undef PK
  return positive;
}

struct LMSmem {
  long long prof[12];
  double red[16 * 32];
  double tile[4 * 64 * kTileStride];  // block_sum_rows / block_sum_t tiles (blockDim <= 256)
  double part[2][4 * 64];  // double-buffered: waves read one while a fast wave fills the other
  double S27[32];
  double mh[16];
  double cand[4 * 4 * 16];  // per wave: 4 candidate solves (ok, x[6], pose[7])
};

// ---- split solve: the G workgroups of one solve meet at every reduction.  Each publishes its
// workgroup sums (identical in every wave) as 8-byte granules {tag, 32 bits of the value}, two per
// double, stored write-through by one relaxed agent-scope atomic store each; every wave then reads
// all G slices with relaxed agent-scope loads until every tag matches, and adds them in workgroup
// order (the same bits in every wave of every workgroup).  The data is its own flag: no fence, no
// barrier, no counter (cdna_hip_programming.md §6 G16, R2).  Slots alternate by exchange parity: a
// workgroup can only rewrite a slot after every workgroup has read it (it needs their next
// exchange first).  tag = launch salt << 16 | exchange index (from 1), so granules of an earlier
// launch never match.  Spins are bounded: a workgroup that waits 0.1 s marks itself failed and
// stops waiting; the solve then reports status 2 (stats[2]) and the host fails loudly.
struct GridX {
  unsigned long long* g;  // [2][kFlowSplitMax][128] granules
  unsigned seq;
  int b, G, epoch, ntot;
  bool dead;
  unsigned long long spin;  // wall-clock ticks a wait may last
};

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

// sums over the G workgroups of the values lanes 0..K-1 hold (lane MAXL: maximum instead);
// every wave calls it with the same values
__device__ __forceinline__ double gx_sum(GridX& x, double v, int K, int maxl = -1) {
  const int lane = threadIdx.x & 63;
  x.epoch++;
  const unsigned long long tag = (unsigned long long)(((x.seq & 0xFFFFu) << 16) | (x.epoch & 0xFFFF))
                                 << 32;
  gu64_t* slot = (gu64_t*)(x.g + (size_t)(x.epoch & 1) * kFlowSplitMax * 128);
  if (threadIdx.x < 64 && lane < K) {  // wave 0 publishes
    const unsigned long long bits = __double_as_longlong(v);
    gu64_t* mine = slot + (size_t)x.b * 128 + 2 * lane;
    __hip_atomic_store(mine, tag | (bits & 0xFFFFFFFFull), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  double s = 0;
  if (x.dead) return 0.0;
  const unsigned long long t0 = wall_clock64();
  for (int g = 0; g < x.G; g++) {
    const gu64_t* src = slot + (size_t)g * 128 + 2 * lane;
    unsigned long long lo = 0, hi = 0;
    for (;;) {
      bool ok = true;
      if (lane < K) {
        lo = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hi = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = (lo & 0xFFFFFFFF00000000ull) == tag && (hi & 0xFFFFFFFF00000000ull) == tag;
      }
      if (__all(ok)) break;
      if (wall_clock64() - t0 > x.spin) {  // 0.1 s of the 100 MHz wall clock by default
        x.dead = true;
        return 0.0;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const double t = __longlong_as_double((long long)((hi << 32) | (lo & 0xFFFFFFFFull)));
    s = lane == maxl ? fmax(s, t) : s + t;
  }
  return lane < K ? s : 0.0;
}

}  // namespace

// One last-frame sample of ObjCentre3D_pre (Tracking.cc:2032-2049): the world point of
// Frame::UnprojectStereoObject(j, 1) (Frame.cc:1118-1152) with the depth noise of the frame's
// first gaussian draw, as cv::Mat float products (double accumulation rounded to float).
__device__ __forceinline__ void centre_point(const FlowSolveDesc& D, int i, float p[3]) {
  const float ifx = 1.0f / D.fx, ify = 1.0f / D.fy;
  float twl[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {  // -Rlw^T tlw (cv::Mat float product)
    double s = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) s += (double)D.Tcw_last[4 * k + r] * (double)D.Tcw_last[4 * k + 3];
    twl[r] = -(float)s;
  }
  const int s = D.idx ? D.idx[i] : i;
  float z = D.depth[s];
  const float noise = (float)((double)D.g0 * ((double)(z * z) / (725 * 0.5) * 0.15));
  z = z + noise;
  const float2 ob = D.obs[s];
  const float x = (ob.x - D.cx) * z * ifx, y = (ob.y - D.cy) * z * ify;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const double s3 = (double)D.Tcw_last[r] * x + (double)D.Tcw_last[4 + r] * y +
                      (double)D.Tcw_last[8 + r] * z;
    p[r] = (float)s3 + twl[r];
  }
}

// ObjCentre3D_pre = (sum of the points, added in float in sample order, as the reference's
// cv::Mat accumulation) / n, the division as cv::Mat / size_t: * (1.0 / n) in double.  No points
// give 0 * (1 / 0) = NaN.  One wave: the lanes compute 64 points at a time, the sum walks them in
// order (three independent float chains).  Called by the lanes of wave 0 only.
__device__ __forceinline__ void centre_sum_wave(const FlowSolveDesc& D, int N) {
  const int lane = threadIdx.x & 63;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int b = 0; b < N; b += 64) {
    float p[3] = {0.f, 0.f, 0.f};
    if (b + lane < N) centre_point(D, b + lane, p);
    const int m = min(64, N - b);
    for (int k = 0; k < m; k++) {
      a0 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p[0]), k));
      a1 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p[1]), k));
      a2 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p[2]), k));
    }
  }
  if (lane == 0) {
    D.centre_out[0] = (float)((double)a0 * (1.0 / N));
    D.centre_out[1] = (float)((double)a1 * (1.0 / N));
    D.centre_out[2] = (float)((double)a2 * (1.0 / N));
  }
}

// N edges from edge `lo` on (a slice of the solve's edges when SPLIT, which then meets the other
// workgroups at every reduction through gx)
template <int IR, bool SPLIT>
__device__ __forceinline__ void flow_lm_body(const FlowSolveDesc& D, int N, int lo, int nt,
                                             LMSmem& sm, int max_cand, GridX& gx,
                                             bool spec_ok = false) {
  const int tid = threadIdx.x, nw = nt >> 6;
#ifdef MMT_LM_PROFILE
  long long prof_t = 0;
  if (tid == 0)
    for (int k = 0; k < 12; k++) sm.prof[k] = 0;
#endif
  double* G = D.scratch;  // items beyond IR * blockDim
  const int cap = D.cap;
  // split solve with every workgroup's edges in registers (at most 2 x 256 per slice, the same
  // answer in every workgroup): a trial is one fused pass (errors + the linearisation at the trial
  // state) and one exchange, instead of a light pass, an exchange, and for accepted trials a
  // second pass and exchange.  The ego solve accepts nearly every trial (22 of 24), so the
  // speculative linearisation is almost never wasted.
  // The one-workgroup solves (D3) take the same fused pass when they have one edge per thread
  // (spec_ok: MMT_LM_SPEC1, default on).
  const bool spec = spec_ok && (SPLIT ? (gx.ntot + gx.G - 1) / gx.G <= 2 * 256 : IR == 1 && N <= nt);
  // the one-workgroup solves (D3) reduce the accepted trial's 63 sums in registers
  // (the one-edge path: with two register edges the kernel would spill); max_cand bit 8 turns it
  // on (MMT_LM_REGSUM, A/B knob)
  const bool kRegSums = !SPLIT && IR == 1 && (max_cand & 256);
  const bool kSpecRegSums = IR == 1 && (max_cand & 256);  // the fused pass's sums in registers
  max_cand &= 255;
  const int rs_idx = (kRegSums || kSpecRegSums) ? wave_rs_index() : 0;
  Cam c;
  c.fx = D.fx;
  c.fy = D.fy;
  c.cx = D.cx;
  c.cy = D.cy;
  c.pinfo = D.prior_info;
  const float deltaF = sqrtf(D.rp_thres);
  c.delta = (double)deltaF;
  c.dsqr = c.delta * c.delta;
  // Twl = inverse(last Tcw): Rwl = R^T (float), twl = -R^T t via double-accumulated gemm
  float Rwl[9], twl[3];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int cc = 0; cc < 3; cc++) Rwl[3 * r + cc] = D.Tcw_last[4 * cc + r];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double s = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) s += (double)Rwl[3 * r + k] * (double)D.Tcw_last[4 * k + 3];
    twl[r] = (float)(-s);
  }
  auto init_item = [&](int i, LMItem& it) {
    const int s = D.idx ? D.idx[i] : i;
    const float2 ob = D.obs[s];
    float z = D.depth[s];
    if (D.use_noise) z = (float)((double)z + (double)D.g0 * ((double)(z * z) / (725 * 0.5) * 0.15));
    const double u = ob.x, v = ob.y, dz = z;
    const double Xc0 = (u - c.cx) * dz / c.fx, Xc1 = (v - c.cy) * dz / c.fy, Xc2 = dz;
    it.X[0] = (double)Rwl[0] * Xc0 + (double)Rwl[1] * Xc1 + (double)Rwl[2] * Xc2 + (double)twl[0];
    it.X[1] = (double)Rwl[3] * Xc0 + (double)Rwl[4] * Xc1 + (double)Rwl[5] * Xc2 + (double)twl[1];
    it.X[2] = (double)Rwl[6] * Xc0 + (double)Rwl[7] * Xc1 + (double)Rwl[8] * Xc2 + (double)twl[2];
    it.ob[0] = u;
    it.ob[1] = v;
    const float2 fl = D.flow[s];
    it.pr[0] = fl.x;
    it.pr[1] = fl.y;
    it.f[0] = fl.x;
    it.f[1] = fl.y;
    it.xl[0] = it.xl[1] = 0;
    it.e[0] = it.e[1] = 0;
  };
  LMItem R[IR];
  const int n_reg = IR * nt;
  // one edge per thread: keep w J of the current linearisation in registers, so the
  // back-substitution needs no projection
  constexpr bool kCacheB = true;  // register item 0 of every thread
  double RB[12];
  // The LM bookkeeping below is computed redundantly by every thread from the block sums in LDS
  // (identical inputs, identical results), so only the 6x6 solve needs a lane-0 section.
  DSE3 P = dse3_from_float(D.init);
  const double hin = kInfo + c.pinfo;  // h of every edge when none is Huber-active
  // the sums of the current system (vc): sum k in lane k of every wave
  // ---- initial linearisation (computeActiveErrors + buildSystem at the initial estimate)
  double* row = tile_row(sm.tile);  // this thread's row of the reduction tile
  // every thread with an edge has one in register slot 0 (N > nt implies all do), so slot 0
  // stores the row and everything after accumulates; threads without edges zero it
  {
    double mh = 0;
#pragma unroll
    for (int k = 0; k < IR; k++) {
      const int i = tid + k * nt;
      if (i < N) {
        init_item(lo + i, R[k]);
        if (k == 0)
          linearise<true>(c, P, R[k], R[k].f[0], R[k].f[1], row, 0.0, R[k].e[0], R[k].e[1],
                          R[k].w, R[k].bl[0], R[k].bl[1], mh, kCacheB ? RB : nullptr);
        else
          linearise<false>(c, P, R[k], R[k].f[0], R[k].f[1], row, 0.0, R[k].e[0], R[k].e[1],
                           R[k].w, R[k].bl[0], R[k].bl[1], mh);
      }
    }
    for (int i = n_reg + tid; i < N; i += nt) {
      LMItem it;
      init_item(lo + i, it);
      linearise<false>(c, P, it, it.f[0], it.f[1], row, 0.0, it.e[0], it.e[1], it.w, it.bl[0],
                       it.bl[1], mh);
      item_store(G, cap, lo + i, it);
    }
    if (tid >= N)
      for (int q = 0; q < kSums; q++) row[q] = 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mh = fmax(mh, __shfl_xor(mh, o, 64));
    if ((tid & 63) == 0) sm.mh[tid >> 6] = mh;
  }
  int pb = 0;  // part buffer of the next reduction
  double vc = block_sum_tile_lanes<kSums>(sm.tile, sm.part[pb], nw);
  pb ^= 1;
  double mhw = 0;  // the largest flow-vertex diagonal of the workgroup's edges
  for (int w = 0; w < nw; w++) mhw = fmax(mhw, sm.mh[w]);
  if (SPLIT) {  // the solve's sums, and the largest diagonal in lane 63
    vc = gx_sum(gx, (tid & 63) == 63 ? mhw : vc, 64, 63);
    mhw = lane_value(vc, 63);
  }
  double cur = lane_value(vc, 0), lam, ni = 2, chk = 0;
  {
    double md = 0;
#pragma unroll
    for (int a = 0; a < 6; a++)
      md = fmax(md, fabs(lane_value(vc, 2 + a * (a + 3) / 2)));  // diagonal (a, a) of the lower triangle
    md = fmax(md, mhw);
    lam = 1e-5 * md;
  }
  int nbad = 0, iters = 0;
  double xb[6] = {0, 0, 0, 0, 0, 0};  // the last increment (reused when the LDLT fails)
  // candidate solves of the rejection chain (this wave's copy): [16 lanes][kCandStride]
  double* cand = sm.cand + (tid >> 6) * 4 * kCandStride;
  int ncand = 0, kc = 0;
  for (int iter = 0; iter < D.max_iters; iter++) {
    const double ini = cur;
    int qmax = 0;
    bool bad = false;
    for (;;) {
#ifdef MMT_LM_PROFILE
      if (tid == 0) prof_t = clock64();
#endif
      const double ilam = drcp(lam);
      // ---- Schur complement over the flow vertices.  Edge i contributes
      //   d00 B0 B0^T + d01 B0 B1^T + d11 B1 B1^T,  d00 = 1/(h_i + lam), d11 = 1/lam, d01 = d00 - d11
      // (h_i = w_i + prior).  With no Huber-active edge every w_i is the same, so the sum is
      // d00 SA + d11 SB with lam-independent sums the linearisation already reduced: no pass.
#ifdef MMT_LM_NO_CLOSED
      const bool clean = false;
#else
      const bool clean = lane_value(vc, 29) == 0;
#endif
      double s27 = 0;  // SPLIT: the solve's Schur sums, sum k in lane k
      if (!clean) {
        double v[27];
#pragma unroll
        for (int k = 0; k < 27; k++) v[k] = 0;
#pragma unroll
        for (int k = 0; k < IR; k++)
          if (tid + k * nt < N) schur_terms(c, P, R[k], lam, ilam, v);
        for (int i = n_reg + tid; i < N; i += nt) {
          LMItem it;
          item_load(G, cap, lo + i, it);
          schur_terms(c, P, it, lam, ilam, v);
        }
        MMT_LMPROF(4);
        block_sum_t<27>(v, sm.tile, sm.red, sm.S27, nw);
        if (SPLIT) s27 = gx_sum(gx, (tid & 63) < 27 ? sm.S27[tid & 63] : 0.0, 27);
      }
      MMT_LMPROF(0);
      // the 6x6 solve, computed redundantly by every wave from the sums (no lane-0 section, no
      // barrier).  A rejected trial changes only lambda (lam *= ni, ni *= 2), so on the
      // closed-form path the four 16-lane groups of a wave solve for the next four lambdas of the
      // rejection chain at once (the same instructions, a different lambda per lane): a trial
      // after a rejection takes its increment and pose from the wave's candidate table instead of
      // paying the solve's dependency chain again.  Each candidate is computed exactly as the
      // sequential solve for its lambda would be.
      if (!(clean && kc < ncand)) {
        double lg = lam, ilg = ilam;
        if (clean) {
          const double l1 = lam * ni, n1 = ni * 2, l2 = l1 * n1, n2 = n1 * 2, l3 = l2 * n2;
          const int g = (tid & 63) >> 4;
          lg = g == 0 ? lam : g == 1 ? l1 : g == 2 ? l2 : l3;
          ilg = drcp(lg);
        }
        double A[21], bs[6];
#pragma unroll
        for (int k = 0; k < 21; k++) A[k] = lane_value(vc, 2 + k);
#pragma unroll
        for (int a = 0; a < 6; a++) bs[a] = lane_value(vc, 23 + a);
        if (clean) {
          // SB = sum B1a B1b - B0a B1b = w H - SA (w = kInfo on every edge)
          const double d00 = drcp(hin + lg);
#pragma unroll
          for (int k = 0; k < 21; k++) {
            const double sa = lane_value(vc, 30 + k);
            A[k] -= d00 * sa + ilg * (kInfo * A[k] - sa);
          }
#pragma unroll
          for (int a = 0; a < 6; a++)
            bs[a] -= d00 * lane_value(vc, 51 + a) + ilg * lane_value(vc, 57 + a);
        } else {
#pragma unroll
          for (int k = 0; k < 21; k++) A[k] -= SPLIT ? lane_value(s27, k) : sm.S27[k];
#pragma unroll
          for (int a = 0; a < 6; a++) bs[a] -= SPLIT ? lane_value(s27, 21 + a) : sm.S27[21 + a];
        }
#pragma unroll
        for (int a = 0; a < 6; a++) A[a * (a + 3) / 2] += lg;  // diagonal (a, a)
#ifdef MMT_LM_PROFILE
        if (tid == 0) {  // force the loads to complete before the split point
          double chk = 0;
          for (int q = 0; q < 21; q++) chk += A[q];
          if (chk == 12345.678) sm.prof[11]++;
        }
#endif
        MMT_LMPROF(8);
        const bool okg = ldlt6_packed(A, bs);
#ifdef MMT_LM_PROFILE
        if (tid == 0 && bs[0] == 12345.678) sm.prof[11]++;
#endif
        MMT_LMPROF(9);
        double xg[6];
#pragma unroll
        for (int a = 0; a < 6; a++) xg[a] = okg ? bs[a] : xb[a];
        const DSE3 PG = exp_mul(xg, P);
        if ((tid & 15) == 0) {
          double* cw = cand + ((tid & 63) >> 4) * kCandStride;
          cw[0] = okg ? 1.0 : 0.0;
#pragma unroll
          for (int a = 0; a < 6; a++) cw[1 + a] = xg[a];
          cw[7] = PG.q.w;
          cw[8] = PG.q.x;
          cw[9] = PG.q.y;
          cw[10] = PG.q.z;
          cw[11] = PG.t[0];
          cw[12] = PG.t[1];
          cw[13] = PG.t[2];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ncand = clean ? max_cand : 1;
        kc = 0;
      }
      bool ok2;
      DSE3 PN;
      {
        const double* cw = cand + kc * kCandStride;
        ok2 = cw[0] != 0.0;
        if (ok2) {
#pragma unroll
          for (int a = 0; a < 6; a++) xb[a] = cw[1 + a];
          PN.q.w = cw[7];
          PN.q.x = cw[8];
          PN.q.y = cw[9];
          PN.q.z = cw[10];
          PN.t[0] = cw[11];
          PN.t[1] = cw[12];
          PN.t[2] = cw[13];
        } else {
          PN = exp_mul(xb, P);  // failed solve: the last increment (g2o's stale x)
        }
        kc++;
      }
      MMT_LMPROF(1);
      double lastTrialChi, scale;
      // split solve, every edge in registers: one fused pass and one exchange per trial (below)
      double vn = 0;                        // the trial's sums; the next system if accepted
      double pw[IR], pb0[IR], pb1[IR];      // pending w, bl of the register items
      double RBn[12];                       // pending w J of register item 0
      if (IR == 1 && spec && kSpecRegSums) {
        // the fused pass with its sums in registers (as D3's pass 2)
        double vals[64];
        if (tid < N)
          spec_terms<true>(c, P, PN, R[0], lo + tid, ok2, lam, ilam, xb, vals, pw[0], pb0[0],
                           pb1[0], kCacheB ? RB : nullptr, RBn);
        else
#pragma unroll
          for (int q = 0; q < 64; q++) vals[q] = 0;
        vals[63] = 0;
        MMT_LMPROF(5);
        vn = block_sum_regs64(vals, sm.part[pb], nw, rs_idx);
        pb ^= 1;
        if (SPLIT) vn = gx_sum(gx, vn, kSums);
        lastTrialChi = lane_value(vn, 0);
        scale = lane_value(vn, 1);
      } else if (spec) {
#pragma unroll
        for (int k = 0; k < IR; k++) {
          const int i = tid + k * nt;
          if (i < N) {
            if (k == 0)
              spec_terms<true>(c, P, PN, R[k], lo + i, ok2, lam, ilam, xb, row, pw[k], pb0[k],
                               pb1[k], kCacheB ? RB : nullptr, RBn);
            else
              spec_terms<false>(c, P, PN, R[k], lo + i, ok2, lam, ilam, xb, row, pw[k], pb0[k],
                                pb1[k], nullptr, nullptr);
          }
        }
        if (tid >= N)
          for (int q = 0; q < kSums; q++) row[q] = 0;
        MMT_LMPROF(5);
        vn = block_sum_tile_lanes<kSums>(sm.tile, sm.part[pb], nw);
        pb ^= 1;
        if (SPLIT) vn = gx_sum(gx, vn, kSums);
        lastTrialChi = lane_value(vn, 0);
        scale = lane_value(vn, 1);
      } else {
      // ---- pass 1: flow back-substitution and the trial's errors (chi2 and scale sums only)
        double s_chi = 0, s_sc = 0;
#pragma unroll
        for (int k = 0; k < IR; k++) {
          const int i = tid + k * nt;
          if (i < N)
            trial_terms(c, P, PN, R[k], lo + i, ok2, lam, ilam, xb, s_chi, s_sc,
                        (kCacheB && k == 0) ? RB : nullptr);
        }
        {  // global items: the next item's loads are in flight while this one computes
          int i = n_reg + tid;
          LMItem it, nx;
          if (i < N) item_load(G, cap, lo + i, it);
          for (; i < N; i += nt) {
            if (i + nt < N) item_load(G, cap, lo + i + nt, nx);
            trial_terms(c, P, PN, it, lo + i, ok2, lam, ilam, xb, s_chi, s_sc);
            item_store_trial(G, cap, lo + i, it);
            it = nx;
          }
        }
        MMT_LMPROF(5);
        block_sum2(s_chi, s_sc, sm.part[pb], nw, lastTrialChi, scale);
        pb ^= 1;
        if (SPLIT) {
          const int l = tid & 63;
          const double t = gx_sum(gx, l == 0 ? lastTrialChi : l == 1 ? scale : 0.0, 2);
          lastTrialChi = lane_value(t, 0);
          scale = lane_value(t, 1);
        }
      }
      MMT_LMPROF(2);
      // ---- g2o LM step acceptance and termination (every thread, same values)
      const double tempChi = ok2 ? lastTrialChi : DBL_MAX;
#pragma unroll
      for (int a = 0; a < 6; a++) scale += xb[a] * (lam * xb[a] + lane_value(vc, 23 + a));
      scale += 1e-3;
      const double rho = (cur - tempChi) / scale;
      const bool accept = rho > 0 && isfinite(tempChi);
      if (accept) {
        const double t = 2 * rho - 1;
        double alpha = 1. - t * t * t;
        alpha = fmin(alpha, 2. / 3.);
        lam = lam * fmax(1. / 3., alpha);
        ni = 2;
        cur = tempChi;
        P = PN;
        ncand = 0;  // the candidates belong to the old system
      } else {
        lam = lam * ni;
        ni = ni * 2;
      }
      qmax++;
      const bool again = (rho < 0 && qmax < 10);
      if (!again) {
        bool ok = true;
        if (qmax == 10 || rho == 0) ok = false;
        if (ok) {
          if ((ini - cur) * 1e3 < ini)
            nbad++;
          else
            nbad = 0;
          if (nbad >= 3) ok = false;
        }
        if (chk < lastTrialChi && iter > 0) ok = false;
        chk = lastTrialChi;
        iters = iter + 1;
        bad = !ok;
      }
      if (accept && spec) {
        // the fused pass already linearised at the accepted state: take the flow step and the
        // pending state, and the trial's sums become the current system
#pragma unroll
        for (int k = 0; k < IR; k++)
          if (tid + k * nt < N) {
            R[k].f[0] += R[k].xl[0];
            R[k].f[1] += R[k].xl[1];
            R[k].w = pw[k];
            R[k].bl[0] = pb0[k];
            R[k].bl[1] = pb1[k];
          }
        if (kCacheB && tid < N)
#pragma unroll
          for (int a = 0; a < 12; a++) RB[a] = RBn[a];
        vc = vn;
      } else if (IR == 1 && !SPLIT && accept && kRegSums) {
        // ---- pass 2 with its sums in registers: the thread's edges accumulate into vals, and a
        // register reduce-scatter (block_sum_regs64) replaces the LDS tile
        double vals[64];
#pragma unroll
        for (int k = 0; k < IR; k++)
          if (tid + k * nt < N) {
            if (k == 0)
              accept_terms<true>(c, P, R[k], vals, kCacheB ? RB : nullptr);
            else
              accept_terms<false>(c, P, R[k], vals);
          }
        {
          int i = n_reg + tid;
          LMItem it, nx;
          if (i < N) item_load(G, cap, lo + i, it);
          for (; i < N; i += nt) {
            if (i + nt < N) item_load(G, cap, lo + i + nt, nx);
            accept_terms<false>(c, P, it, vals);
            item_store_accept(G, cap, lo + i, it);
            it = nx;
          }
        }
        if (tid >= N)
#pragma unroll
          for (int q = 0; q < 64; q++) vals[q] = 0;
        vals[63] = 0;
        vc = block_sum_regs64(vals, sm.part[pb], nw, rs_idx);
        pb ^= 1;
      } else if (accept) {
        // ---- pass 2: take the flow step and linearise at the accepted state (the system of the
        // next trial); rejected trials skip it, so they cost the errors and two sums only
#pragma unroll
        for (int k = 0; k < IR; k++)
          if (tid + k * nt < N) {
            if (k == 0)
              accept_terms<true>(c, P, R[k], row, kCacheB ? RB : nullptr);
            else
              accept_terms<false>(c, P, R[k], row);
          }
        {
          int i = n_reg + tid;
          LMItem it, nx;
          if (i < N) item_load(G, cap, lo + i, it);
          for (; i < N; i += nt) {
            if (i + nt < N) item_load(G, cap, lo + i + nt, nx);
            accept_terms<false>(c, P, it, row);
            item_store_accept(G, cap, lo + i, it);
            it = nx;
          }
        }
        if (tid >= N)
          for (int q = 0; q < kSums; q++) row[q] = 0;
#ifdef MMT_LM_PROFILE
        if (tid == 0) {  // pass 2's edge work, apart from its reduction (decide keeps the rest)
          const long long now = clock64();
          sm.prof[10] += now - prof_t;
          prof_t = now;
        }
#endif
        vc = block_sum_tile_lanes<kSums>(sm.tile, sm.part[pb], nw);
        pb ^= 1;
        if (SPLIT) vc = gx_sum(gx, vc, kSums);
      }
      MMT_LMPROF(3);
#ifdef MMT_LM_PROFILE
      if (tid == 0) {
        sm.prof[6]++;
        if (lane_value(vc, 29) == 0) sm.prof[7]++;
      }
#endif
      if (!again) break;
    }
    if (bad) break;
  }
  // outputs: pose, iterations, inliers from the last computed edge errors (Optimizer.cc:536-566)
  double v[1] = {0};
  auto outlier = [&](const LMItem& it) {
    const float chi2 = (float)(kInfo * (it.e[0] * it.e[0] + it.e[1] * it.e[1]));
    return chi2 > D.rp_thres ? 1.0 : 0.0;
  };
#pragma unroll
  for (int k = 0; k < IR; k++)
    if (tid + k * nt < N) v[0] += outlier(R[k]);
  for (int i = n_reg + tid; i < N; i += nt) {
    LMItem it;
    item_load(G, cap, lo + i, it);
    v[0] += outlier(it);
  }
  block_sum<1>(v, sm.red, sm.S27, nw);
  int n_out = N - (int)sm.S27[0], status = 0;
  if (SPLIT) {  // the solve's outliers, and whether any workgroup gave up waiting
    const int l = tid & 63;
    const double t = gx_sum(gx, l == 0 ? sm.S27[0] : l == 1 ? (gx.dead ? 1.0 : 0.0) : 0.0, 2);
    n_out = gx.ntot - (int)lane_value(t, 0);
    status = (gx.dead || lane_value(t, 1) != 0) ? 2 : 0;
    if (gx.b != 0) return;
  }
  if (D.centre_out && tid < 64) centre_sum_wave(D, SPLIT ? gx.ntot : N);  // ObjCentre3D_pre, wave 0
  if (tid == 0) {
    dse3_to_float(P, D.pose_out);
    D.stats[0] = iters;
    D.stats[1] = n_out;
    D.stats[2] = status;
#ifdef MMT_LM_PROFILE
    printf("lmprof N=%d T=%d iters=%d trials=%lld clean=%lld schur_pass=%lld schur_red=%lld "
           "solve_ld=%lld solve_ldlt=%lld solve_exp=%lld upd_pass=%lld upd_red=%lld decide=%lld "
           "blk=%d stats=%p pass2=%lld\n",
           N, nt, iters, sm.prof[6], sm.prof[7], sm.prof[4], sm.prof[0], sm.prof[8], sm.prof[9],
           sm.prof[1], sm.prof[5], sm.prof[2], sm.prof[3], (int)blockIdx.x, (void*)D.stats,
           sm.prof[10]);
#endif
  }
}

// One workgroup per solve; each workgroup picks the register-item count its own edge count needs,
// so a small object solved in the same launch as a large one runs the short code path.
template <int MAXIR>
// max_cand (1..4): lambda candidates a clean system's solve provides (1: every trial solves for
// its own lambda, the sequential order; a test knob, candidates are bit-identical to it)
__global__ __launch_bounds__(256) void k_flow_lm(const FlowSolveDesc* __restrict__ descs,
                                                 int max_cand) {
  __shared__ LMSmem sm;
  const FlowSolveDesc& D = descs[blockIdx.x];
  const int N = D.d_n ? min(*D.d_n, D.cap) : min(D.n, D.cap);
  if (N < 3) {
    if (threadIdx.x == 0) {
      D.stats[0] = 0;
      D.stats[1] = 0;
      D.stats[2] = 1;
    }
    // the reference computes ObjCentre3D_pre before the solve whatever the count: 1-2 points
    // give their mean, none gives 0 * (1 / 0) = NaN (Tracking.cc:2032-2049)
    if (D.centre_out && threadIdx.x < 64) centre_sum_wave(D, N);
    return;
  }
  // Threads per solve: one edge per thread up to the block size (the passes are issue-bound:
  // a second register edge per thread doubles them, measured); a solve smaller than the block
  // uses only the waves it needs and the others leave at once (a finished wave no longer counts
  // at the barriers), which keeps the reductions' LDS traffic to the rows in use.
  const int nt = min((int)blockDim.x, max(64, (N + 63) / 64 * 64));
  if ((int)threadIdx.x >= nt) return;
  GridX gx{};
  const bool spec = (max_cand & 512) != 0;
  if (N <= nt || MAXIR == 1)
    flow_lm_body<1, false>(D, N, 0, nt, sm, max_cand, gx, spec);
  else
    flow_lm_body<2, false>(D, N, 0, nt, sm, max_cand, gx, spec);
}

// One large solve (descs[0]) over gridDim.x <= kFlowSplitMax workgroups, each on a contiguous slice
// of the edges (lo = b N / G); the LM bookkeeping runs in every workgroup on the exchanged sums.
// The workgroups must be resident together: one per CU, at most 8 (bounded spins otherwise).
__global__ __launch_bounds__(256) void k_flow_lm_split(const FlowSolveDesc* __restrict__ descs,
                                                       int max_cand, int spec) {
  __shared__ LMSmem sm;
  const FlowSolveDesc& D = descs[0];
  const int N = D.d_n ? min(*D.d_n, D.cap) : min(D.n, D.cap);
  const int G = gridDim.x, b = blockIdx.x;
  if (N < 3) {  // as k_flow_lm, by workgroup 0
    if (b == 0) {
      if (threadIdx.x == 0) {
        D.stats[0] = 0;
        D.stats[1] = 0;
        D.stats[2] = 1;
      }
      if (D.centre_out && threadIdx.x < 64) centre_sum_wave(D, N);
    }
    return;
  }
  const int lo = (int)((long long)b * N / G), hi = (int)((long long)(b + 1) * N / G);
  const int Nl = hi - lo;
  const int nt = min((int)blockDim.x, max(64, (Nl + 63) / 64 * 64));
  if ((int)threadIdx.x >= nt) return;
  GridX gx{D.gx, D.gx_seq, b, G, 0, N, false, D.gx_spin ? D.gx_spin : 10000000ull};
  if (Nl <= nt)
    flow_lm_body<1, true>(D, Nl, lo, nt, sm, max_cand, gx, spec != 0);
  else
    flow_lm_body<2, true>(D, Nl, lo, nt, sm, max_cand, gx, spec != 0);
}

void launch_flow_lm(const FlowSolveDesc* d_descs, int nsolves, int n_hint, hipStream_t st) {
  // Latency-bound: about one correspondence per thread where the block allows it (a trial's
  // passes cost about one correspondence's dependency chain), 64..256 threads, up to 2 register
  // items each (more register items spill: the 6x6 solve and the sums need the room); items
  // beyond go through the global item arrays.  Each workgroup picks its own item count
  // (k_flow_lm); n_hint (the largest edge count) only sizes the block.
  const int threads = std::min(256, std::max(64, (n_hint + 63) / 64 * 64));
  // MMT_LM_MAX_CAND=1..4 (read per launch; tests compare 1 against the default 4 bit for bit);
  // bit 256: the accepted trial's sums reduced in registers; bit 512: the fused trial pass
  int max_cand = 4;
  if (const char* e = getenv("MMT_LM_MAX_CAND")) max_cand = std::min(4, std::max(1, atoi(e)));
  max_cand |= 256 | 512;
  hipLaunchKernelGGL(k_flow_lm<2>, dim3(nsolves), dim3(threads), 0, st, d_descs, max_cand);
}

int flow_split_groups(int n_hint) {
  const char* e = getenv("MMT_LM_SPLIT");  // read per call (tests switch it)
  const int force = e ? atoi(e) : -1;
  if (force == 0) return 1;
  if (force > 0) return std::min(force, kFlowSplitMax);
  // about one edge per thread of 256-thread workgroups; small solves stay whole (each exchange
  // costs about a microsecond of latency)
  if (n_hint < 512) return 1;
  return std::min(kFlowSplitMax, (n_hint + 255) / 256);
}

void launch_flow_lm_split(const FlowSolveDesc* d_desc, int groups, hipStream_t st) {
  int max_cand = 4;
  if (const char* e = getenv("MMT_LM_MAX_CAND")) max_cand = std::min(4, std::max(1, atoi(e)));
  groups = std::max(1, std::min(groups, kFlowSplitMax));
  const int spec = 1;  // one fused pass and one exchange per trial
  max_cand |= 256;     // its sums reduced in registers
  hipLaunchKernelGGL(k_flow_lm_split, dim3(groups), dim3(256), 0, st, d_desc, max_cand, spec);
}

size_t flow_scratch_doubles(int cap) { return (size_t)G_COUNT * cap; }

// ============================================================================ D1
// Optimizer::PoseOptimization (reference src/Optimizer.cc:3121-3339; CPU checker:
// oracle/solve_ref.cpp pose_optimization): pose-only g2o LM over the frame's MapPoint
// observations.  Mono edges (uR < 0) EdgeSE3ProjectXYZOnlyPose, stereo edges
// EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.cpp:266-364, the stereo projection with a
// float 1/z), Huber delta^2 5.991 / 7.815, information 1/sigma^2 of the keypoint's octave.  Four
// rounds of at most 10 LM iterations, each restarting from the input pose on the edges classified
// inliers by the previous round; the robust kernel is dropped after round 2; fewer than 10 edges
// stop after one round.  One workgroup, up to 8 edges per thread in registers; per LM trial one
// pass over the edges (trial errors, robust chi2 and the speculative linearisation at the trial
// pose) and one block reduction of 28 sums.
namespace {

constexpr int kPoSums = 28;  // [0] robust chi2, [1..21] lower triangle of H, [22..27] b

struct PoEdgeR {  // constant inputs in registers; the last computed error lives in LDS
  float X[3], obs[3], s;
  int flags;  // bit 0 stereo, bit 1 outlier (level 1), bit 2 robust kernel
};
constexpr int kPoStereo = 1, kPoOutlier = 2, kPoRobust = 4;

struct PoSmem {
  double tile[4 * 64 * 33];
  double red[16 * 32];
  double H[2][32];  // current / trial sums
  double e[3][kPoseOptMaxEdges];
  int flags[kPoseOptMaxEdges];
};

__device__ __forceinline__ void po_err(const PoEdgeR& E, const DSE3& T, const PoseOptDesc& D,
                                       double e[3], double& x, double& y, double& z) {
  const double X[3] = {(double)E.X[0], (double)E.X[1], (double)E.X[2]};
  map(T, X, x, y, z);
  if (!(E.flags & kPoStereo)) {
    const double px = x / z, py = y / z;  // project2d
    e[0] = (double)E.obs[0] - (px * D.fx + D.cx);
    e[1] = (double)E.obs[1] - (py * D.fy + D.cy);
    e[2] = 0;
  } else {
    const float invz = 1.0 / z;  // const float invz = 1.0f/trans_xyz[2]
    const double u = x * invz * D.fx + D.cx, v = y * invz * D.fy + D.cy;
    e[0] = (double)E.obs[0] - u;
    e[1] = (double)E.obs[1] - v;
    e[2] = (double)E.obs[2] - (u - D.bf * invz);
  }
}

__device__ __forceinline__ double po_chi2(const PoEdgeR& E, const double e[3]) {
  return (E.flags & kPoStereo) ? E.s * (e[0] * e[0] + e[1] * e[1] + e[2] * e[2])
                               : E.s * (e[0] * e[0] + e[1] * e[1]);
}

// errors at T for an active edge (stored to LDS), robust chi2 and the rho'-weighted
// J^T Omega J / b terms
__device__ __forceinline__ void po_linearise(const PoEdgeR& E, const DSE3& T, const PoseOptDesc& D,
                                             double dM, double dS, double* eo, int stride,
                                             double* v) {
  double x, y, z, e[3];
  po_err(E, T, D, e, x, y, z);
  eo[0] = e[0];
  eo[stride] = e[1];
  eo[2 * stride] = e[2];
  const bool stereo = E.flags & kPoStereo;
  const double c = po_chi2(E, e);
  double r0 = c, r1 = 1.0;
  if (E.flags & kPoRobust) {
    const double d = stereo ? dS : dM;
    huber(c, d * d, d, r0, r1);
  }
  v[0] += r0;
  const double invz = 1.0 / z, invz_2 = invz * invz;
  double J[3][6];
  J[0][0] = x * y * invz_2 * D.fx;
  J[0][1] = -(1 + (x * x * invz_2)) * D.fx;
  J[0][2] = y * invz * D.fx;
  J[0][3] = -invz * D.fx;
  J[0][4] = 0;
  J[0][5] = x * invz_2 * D.fx;
  J[1][0] = (1 + y * y * invz_2) * D.fy;
  J[1][1] = -x * y * invz_2 * D.fy;
  J[1][2] = -x * invz * D.fy;
  J[1][3] = 0;
  J[1][4] = -invz * D.fy;
  J[1][5] = y * invz_2 * D.fy;
  J[2][0] = J[0][0] - D.bf * y * invz_2;
  J[2][1] = J[0][1] + D.bf * x * invz_2;
  J[2][2] = J[0][2];
  J[2][3] = J[0][3];
  J[2][4] = 0;
  J[2][5] = J[0][5] - D.bf * invz_2;
  const double w = r1 * (double)E.s;
  const double se0 = (double)E.s * e[0], se1 = (double)E.s * e[1], se2 = (double)E.s * e[2];
  int k = 1;
#pragma unroll
  for (int a = 0; a < 6; a++)
#pragma unroll
    for (int b = 0; b <= a; b++) {
      double acc = J[0][a] * w * J[0][b] + J[1][a] * w * J[1][b];
      if (stereo) acc += J[2][a] * w * J[2][b];
      v[k++] += acc;
    }
#pragma unroll
  for (int a = 0; a < 6; a++) {
    double g = J[0][a] * se0 + J[1][a] * se1;
    if (stereo) g += J[2][a] * se2;
    v[22 + a] -= r1 * g;
  }
}

__device__ __forceinline__ PoEdgeR po_load(const PoseOptDesc& D, const int* flags, int i,
                                           int fl = 0) {
  PoEdgeR E;
  E.X[0] = D.Xw[3 * i];
  E.X[1] = D.Xw[3 * i + 1];
  E.X[2] = D.Xw[3 * i + 2];
  E.obs[0] = D.obs[3 * i];
  E.obs[1] = D.obs[3 * i + 1];
  E.obs[2] = D.obs[3 * i + 2];
  E.s = D.inv_sigma2[i];
  E.flags = flags ? flags[i] : fl;
  return E;
}

// Edges are re-read from global memory (L2-resident, a few KB) on every pass and their flags and
// last errors live in LDS: no per-thread edge arrays, so the kernel stays clear of spills.
// GLOBAL: more edges than the LDS arrays hold (kPoseOptMaxEdges): the per-edge errors and flags
// live in the caller's scratch (D.e_scratch: 3 x N doubles, D.f_scratch: N ints) instead.
template <bool GLOBAL>
__device__ void pose_opt_body(const PoseOptDesc& D, int N, PoSmem& sm) {
  const int tid = threadIdx.x, nt = blockDim.x, nw = nt >> 6;
  // const float deltaMono = sqrt(5.991): double sqrt rounded to float, then setDelta(double)
  const double dM = (double)(float)sqrt(5.991), dS = (double)(float)sqrt(7.815);
  int* flags = GLOBAL ? D.f_scratch : sm.flags;
  double* const E = GLOBAL ? D.e_scratch : &sm.e[0][0];
  const int ES = GLOBAL ? N : kPoseOptMaxEdges;  // row stride of the three error rows
  for (int i = tid; i < N; i += nt) {
    flags[i] = (D.obs[3 * i + 2] < 0 ? 0 : kPoStereo) | kPoRobust;
    E[i] = E[ES + i] = E[2 * ES + i] = 0;
  }
  __syncthreads();
  const DSE3 P0 = dse3_from_float(D.Tcw);
  DSE3 P = P0;
  int nBad = 0;
  auto pass = [&](const DSE3& T, double* out) {
    double v[kPoSums];
#pragma unroll
    for (int q = 0; q < kPoSums; q++) v[q] = 0;
    for (int i = tid; i < N; i += nt) {
      const PoEdgeR Ed = po_load(D, flags, i);
      if (!(Ed.flags & kPoOutlier)) po_linearise(Ed, T, D, dM, dS, E + i, ES, v);
    }
    block_sum_t<kPoSums>(v, sm.tile, sm.red, out, nw);
  };
  for (int it = 0; it < 4; it++) {
    P = P0;
    int hs = 0;
    pass(P, sm.H[0]);  // computeActiveErrors + buildSystem at the round's start
    double cur = sm.H[0][0], lam, ni = 2, chk = 0;
    {
      double md = 0;
#pragma unroll
      for (int a = 0; a < 6; a++) md = fmax(md, fabs(sm.H[0][1 + a * (a + 3) / 2]));
      lam = 1e-5 * md;
    }
    int nRaul = 0;
    double xb[6] = {0, 0, 0, 0, 0, 0};
    for (int iter = 0; iter < 10; iter++) {
      const double ini = cur;
      int qmax = 0;
      bool bad = false;
      for (;;) {
        // ---- solve (H + lambda I) x = b (every thread, identical inputs)
        const double* Hc = sm.H[hs];
        double A[21], bs[6];
#pragma unroll
        for (int q = 0; q < 21; q++) A[q] = Hc[1 + q];
#pragma unroll
        for (int a = 0; a < 6; a++) {
          A[a * (a + 3) / 2] += lam;
          bs[a] = Hc[22 + a];
        }
        const bool ok2 = ldlt6_packed(A, bs);
#pragma unroll
        for (int a = 0; a < 6; a++) xb[a] = ok2 ? bs[a] : xb[a];
        const DSE3 PN = exp_mul(xb, P);
        pass(PN, sm.H[hs ^ 1]);  // trial errors, robust chi2, speculative linearisation
        const double* Ht = sm.H[hs ^ 1];
        const double lastTrialChi = Ht[0];
        const double tempChi = ok2 ? Ht[0] : DBL_MAX;
        double scale = 0;
#pragma unroll
        for (int a = 0; a < 6; a++) scale += xb[a] * (lam * xb[a] + Hc[22 + a]);
        scale += 1e-3;
        const double rho = (cur - tempChi) / scale;
        const bool accept = rho > 0 && isfinite(tempChi);
        if (accept) {
          const double t = 2 * rho - 1;
          double alpha = 1. - t * t * t;
          alpha = fmin(alpha, 2. / 3.);
          lam = lam * fmax(1. / 3., alpha);
          ni = 2;
          cur = tempChi;
          P = PN;
          hs ^= 1;
        } else {
          lam = lam * ni;
          ni = ni * 2;
        }
        qmax++;
        const bool again = (rho < 0 && qmax < 10);
        if (!again) {
          bool ok = true;
          if (qmax == 10 || rho == 0) ok = false;
          if (ok) {
            if ((ini - cur) * 1e3 < ini)
              nRaul++;
            else
              nRaul = 0;
            if (nRaul >= 3) ok = false;
          }
          if (chk < lastTrialChi && iter > 0) ok = false;
          chk = lastTrialChi;
          bad = !ok;
          break;
        }
      }
      if (bad) break;
    }
    // ---- re-classification (Optimizer.cc:3266-3322): edges that sat the round out get their
    // error at the optimised pose, the others keep the last computed one
    double nb[1] = {0};
    for (int i = tid; i < N; i += nt) {
      PoEdgeR Ed = po_load(D, flags, i);
      double e[3];
      if (Ed.flags & kPoOutlier) {
        double x, y, z;
        po_err(Ed, P, D, e, x, y, z);
        E[i] = e[0];
        E[ES + i] = e[1];
        E[2 * ES + i] = e[2];
      } else {
        e[0] = E[i];
        e[1] = E[ES + i];
        e[2] = E[2 * ES + i];
      }
      const double c = po_chi2(Ed, e);
      const float thr = (Ed.flags & kPoStereo) ? 7.815f : 5.991f;
      int f = c > (double)thr ? (Ed.flags | kPoOutlier) : (Ed.flags & ~kPoOutlier);
      nb[0] += (f & kPoOutlier) ? 1.0 : 0.0;
      if (it == 2) f &= ~kPoRobust;
      flags[i] = f;
    }
    block_sum<1>(nb, sm.red, sm.H[0], nw);  // ends with a barrier: flags visible to all
    nBad = (int)sm.H[0][0];
    __syncthreads();  // sm.H[0] is rewritten by the next round's first reduction
    if (N < 10) break;  // optimizer.edges().size() < 10
  }
  for (int i = tid; i < N; i += nt) D.outlier[i] = (flags[i] & kPoOutlier) ? 1 : 0;
  if (tid == 0) {
    dse3_to_float(P, D.pose_out);
    *D.n_inliers = N - nBad;
  }
}


// The same solve with the edges in registers: kPoThreads threads, IT edges per thread (edge
// tid + q * kPoThreads), their inputs, last errors and flags held for the whole solve, so a pass
// issues no memory operation but the reduction.  8 waves keep two per SIMD in flight to hide
// the FP64 dependency chains of one edge; the 28 sums meet by a butterfly reduce-scatter inside
// each wave and one LDS exchange (block_sum).
constexpr int kPoThreads = 512, kPoNone = 8;

constexpr int kPoStride = 29;  // odd row stride of the reduction tile (28 sums)


// po_linearise for the register path: the edge's contribution goes straight into the thread's
// row of the reduction tile (stored by its first edge, FIRST, accumulated by the others; an
// outlier edge contributes zeros), so the 28 sums never occupy registers.
template <bool FIRST>
__device__ __forceinline__ void po_linearise_row(const PoEdgeR& E, const DSE3& T,
                                                 const PoseOptDesc& D, double dM, double dS,
                                                 double* eo, double* row) {
  if (E.flags & kPoOutlier) {
    if (FIRST)
#pragma unroll
      for (int k = 0; k < kPoSums; k++) row[k] = 0;
    return;
  }
  double x, y, z, e[3];
  po_err(E, T, D, e, x, y, z);
  eo[0] = e[0];
  eo[1] = e[1];
  eo[2] = e[2];
  {  // J and the sums with FMA contraction (the errors and chi2 above keep the reference's rounding)
#pragma clang fp contract(fast)
  const bool stereo = E.flags & kPoStereo;
  const double c = po_chi2(E, e);
  double r0 = c, r1 = 1.0;
  if (E.flags & kPoRobust) {
    const double d = stereo ? dS : dM;
    huber(c, d * d, d, r0, r1);
  }
  row[0] = FIRST ? r0 : row[0] + r0;
  const double invz = 1.0 / z, invz_2 = invz * invz;
  double J[3][6];
  J[0][0] = x * y * invz_2 * D.fx;
  J[0][1] = -(1 + (x * x * invz_2)) * D.fx;
  J[0][2] = y * invz * D.fx;
  J[0][3] = -invz * D.fx;
  J[0][4] = 0;
  J[0][5] = x * invz_2 * D.fx;
  J[1][0] = (1 + y * y * invz_2) * D.fy;
  J[1][1] = -x * y * invz_2 * D.fy;
  J[1][2] = -x * invz * D.fy;
  J[1][3] = 0;
  J[1][4] = -invz * D.fy;
  J[1][5] = y * invz_2 * D.fy;
  J[2][0] = J[0][0] - D.bf * y * invz_2;
  J[2][1] = J[0][1] + D.bf * x * invz_2;
  J[2][2] = J[0][2];
  J[2][3] = J[0][3];
  J[2][4] = 0;
  J[2][5] = J[0][5] - D.bf * invz_2;
  const double w = r1 * (double)E.s;
  const double se0 = (double)E.s * e[0], se1 = (double)E.s * e[1], se2 = (double)E.s * e[2];
  int k = 1;
#pragma unroll
  for (int a = 0; a < 6; a++)
#pragma unroll
    for (int b = 0; b <= a; b++) {
      double acc = J[0][a] * w * J[0][b] + J[1][a] * w * J[1][b];
      if (stereo) acc += J[2][a] * w * J[2][b];
      row[k] = FIRST ? acc : row[k] + acc;
      k++;
    }
#pragma unroll
  for (int a = 0; a < 6; a++) {
    double g = J[0][a] * se0 + J[1][a] * se1;
    if (stereo) g += J[2][a] * se2;
    row[22 + a] = FIRST ? -(r1 * g) : row[22 + a] - r1 * g;
  }
  }
}

}  // namespace

// The same solve with light trial passes, as the flow LM does it: a trial first evaluates only
// its errors and robust chi2 (one DPP wave sum and one LDS exchange); the 28-sum linearisation
// runs only for an accepted trial, at its pose (g2o keeps the linearisation of the accepted
// state).  A rejected trial changes nothing but lambda (lam *= ni, ni *= 2), so the 6x6 solve runs
// for the next four lambdas of the rejection chain at once, one per 16-lane group (the same
// instructions, a different lambda per lane), and a trial after a rejection takes its increment
// and pose from the wave's candidate table.  Each candidate is computed exactly as the sequential
// solve for its lambda.  In the bench about 58 % of D1's trials are rejected.
struct PoSmemL {
  double tile[(kPoThreads / 64) * 64 * kPoStride];
  double part[2][(kPoThreads / 64) * 32];  // wave partials of the full pass, double-buffered
  double lpart[2][kPoThreads / 64];        // wave partials of the light pass, double-buffered
  double Hw[kPoThreads / 64][2][32];        // every wave's own copy of the current / trial sums
  double cand[kPoThreads / 64][4][16];      // every wave's lambda candidates (ok, x[6], pose[7])
  double red[16 * 32];
  double H[32];
};

template <int IT>
__device__ void pose_opt_light(const PoseOptDesc& D, int N, PoSmemL& sm) {
  const int tid = threadIdx.x, nw = kPoThreads >> 6;
  const int lane = tid & 63, wave = tid >> 6;
  const double dM = (double)(float)sqrt(5.991), dS = (double)(float)sqrt(7.815);
  PoEdgeR Ed[IT];
  double er[IT][3];
#pragma unroll
  for (int q = 0; q < IT; q++) {
    const int i = tid + q * kPoThreads;
    if (i < N) {
      Ed[q] = po_load(D, nullptr, i, (D.obs[3 * i + 2] < 0 ? 0 : kPoStereo) | kPoRobust);
    } else {
      Ed[q] = PoEdgeR{};
      Ed[q].flags = kPoNone | kPoOutlier;
    }
    er[q][0] = er[q][1] = er[q][2] = 0;
  }
  DSE3 P;
  int nBad = 0;
  double* row = tile_row<kPoStride>(sm.tile);
  int npass = 0, nlight = 0;
#ifdef MMT_PO_PROFILE
  int nrej = 0;
  long long pp[4] = {0, 0, 0, 0}, pt = clock64();
#define PL_T(k)                     \
  do {                              \
    const long long _n = clock64(); \
    pp[k] += _n - pt;               \
    pt = _n;                        \
  } while (0)
#else
#define PL_T(k) \
  do {          \
  } while (0)
#endif
  // full pass: errors and the 28 sums at T into the wave's copy `buf` of the sums
  auto full = [&](const DSE3& T, int buf) {
    PL_T(0);
    po_linearise_row<true>(Ed[0], T, D, dM, dS, er[0], row);
#pragma unroll
    for (int q = 1; q < IT; q++) po_linearise_row<false>(Ed[q], T, D, dM, dS, er[q], row);
    PL_T(1);
    const double* t = sm.tile + (size_t)wave * 64 * kPoStride;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double* part = sm.part[npass & 1];
    if (lane < kPoSums) {
      double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int r0 = 0; r0 < 64; r0 += 16) {
        double x[16];
#pragma unroll
        for (int j = 0; j < 16; j++) x[j] = t[(r0 + j) * kPoStride + lane];
#pragma unroll
        for (int j = 0; j < 16; j++) acc[j & 7] += x[j];
      }
      part[wave * 32 + lane] =
          ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    __syncthreads();
    if (lane < kPoSums) {
      double sum = 0;
#pragma unroll
      for (int w = 0; w < nw; w++) sum += part[w * 32 + lane];
      sm.Hw[wave][buf][lane] = sum;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    PL_T(2);
    npass++;
  };
  // light pass: errors and the robust chi2 at T (same per-edge arithmetic as the full pass)
  auto light = [&](const DSE3& T) {
    PL_T(0);
    double c = 0;
#pragma unroll
    for (int q = 0; q < IT; q++) {
      if (Ed[q].flags & kPoOutlier) continue;
      double x, y, z;
      po_err(Ed[q], T, D, er[q], x, y, z);
      const double ch = po_chi2(Ed[q], er[q]);
      double r0 = ch, r1 = 1.0;
      if (Ed[q].flags & kPoRobust) {
        const double d = (Ed[q].flags & kPoStereo) ? dS : dM;
        huber(ch, d * d, d, r0, r1);
      }
      c += r0;
    }
    PL_T(1);
    c = wave_sum_dpp(c);
    double* lp = sm.lpart[nlight & 1];
    if (lane == 0) lp[wave] = c;
    __syncthreads();
    double sum = 0;
#pragma unroll
    for (int w = 0; w < nw; w++) sum += lp[w];
    PL_T(2);
    nlight++;
    return sum;
  };
  double* cand = &sm.cand[wave][0][0];
  for (int it = 0; it < 4; it++) {
    P = dse3_from_float(D.Tcw);  // every round restarts from the input pose
    int hs = 0;
    full(P, 0);
    double cur = sm.Hw[wave][0][0], lam, ni = 2, chk = 0;
    {
      double md = 0;
#pragma unroll
      for (int a = 0; a < 6; a++) md = fmax(md, fabs(sm.Hw[wave][0][1 + a * (a + 3) / 2]));
      lam = 1e-5 * md;
    }
    int nRaul = 0;
    double xb[6] = {0, 0, 0, 0, 0, 0};
    int kc = 4, ncand = 0;  // candidate table empty
    for (int iter = 0; iter < 10; iter++) {
      const double ini = cur;
      int qmax = 0;
      bool bad = false;
      for (;;) {
        const double* Hc = sm.Hw[wave][hs];
        if (kc >= ncand) {
          // ---- the solves of the next four lambdas of the chain, one per 16-lane group
          const double l1 = lam * ni, n1 = ni * 2, l2 = l1 * n1, n2 = n1 * 2, l3 = l2 * n2;
          const int g = lane >> 4;
          const double lg = g == 0 ? lam : g == 1 ? l1 : g == 2 ? l2 : l3;
          double A[21], bs[6];
#pragma unroll
          for (int q = 0; q < 21; q++) A[q] = Hc[1 + q];
#pragma unroll
          for (int a = 0; a < 6; a++) {
            A[a * (a + 3) / 2] += lg;
            bs[a] = Hc[22 + a];
          }
          const bool okg = ldlt6_packed(A, bs);
          double xg[6];
#pragma unroll
          for (int a = 0; a < 6; a++) xg[a] = okg ? bs[a] : xb[a];
          const DSE3 PG = exp_mul(xg, P);
          if ((lane & 15) == 0) {
            double* cw = cand + g * 16;
            cw[0] = okg ? 1.0 : 0.0;
#pragma unroll
            for (int a = 0; a < 6; a++) cw[1 + a] = xg[a];
            cw[7] = PG.q.w;
            cw[8] = PG.q.x;
            cw[9] = PG.q.y;
            cw[10] = PG.q.z;
            cw[11] = PG.t[0];
            cw[12] = PG.t[1];
            cw[13] = PG.t[2];
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          ncand = 4;
          kc = 0;
        }
        bool ok2;
        DSE3 PN;
        {
          const double* cw = cand + kc * 16;
          ok2 = cw[0] != 0.0;
          if (ok2) {
#pragma unroll
            for (int a = 0; a < 6; a++) xb[a] = cw[1 + a];
            PN.q.w = cw[7];
            PN.q.x = cw[8];
            PN.q.y = cw[9];
            PN.q.z = cw[10];
            PN.t[0] = cw[11];
            PN.t[1] = cw[12];
            PN.t[2] = cw[13];
          } else {
            PN = exp_mul(xb, P);  // failed solve: the last increment (g2o's stale x)
          }
          kc++;
        }
        const double lastTrialChi = light(PN);
        const double tempChi = ok2 ? lastTrialChi : DBL_MAX;
        double scale = 0;
#pragma unroll
        for (int a = 0; a < 6; a++) scale += xb[a] * (lam * xb[a] + Hc[22 + a]);
        scale += 1e-3;
        const double rho = (cur - tempChi) / scale;
        const bool accept = rho > 0 && isfinite(tempChi);
        if (accept) {
          const double t = 2 * rho - 1;
          double alpha = 1. - t * t * t;
          alpha = fmin(alpha, 2. / 3.);
          lam = lam * fmax(1. / 3., alpha);
          ni = 2;
          cur = tempChi;
          P = PN;
          full(P, hs ^ 1);  // the accepted state's linearisation
          hs ^= 1;
          kc = ncand;  // the table belonged to the old system
        } else {
          lam = lam * ni;
          ni = ni * 2;
#ifdef MMT_PO_PROFILE
          nrej++;
#endif
        }
        qmax++;
        const bool again = (rho < 0 && qmax < 10);
        if (!again) {
          bool ok = true;
          if (qmax == 10 || rho == 0) ok = false;
          if (ok) {
            if ((ini - cur) * 1e3 < ini)
              nRaul++;
            else
              nRaul = 0;
            if (nRaul >= 3) ok = false;
          }
          if (chk < lastTrialChi && iter > 0) ok = false;
          chk = lastTrialChi;
          bad = !ok;
          break;
        }
      }
      if (bad) break;
    }
    // re-classification (Optimizer.cc:3266-3322): edges that sat the round out get their error at
    // the optimised pose, the others keep the last computed one (the last trial's)
    double nb[1] = {0};
#pragma unroll
    for (int q = 0; q < IT; q++) {
      if (Ed[q].flags & kPoNone) continue;
      if (Ed[q].flags & kPoOutlier) {
        double x, y, z;
        po_err(Ed[q], P, D, er[q], x, y, z);
      }
      const double c = po_chi2(Ed[q], er[q]);
      const float thr = (Ed[q].flags & kPoStereo) ? 7.815f : 5.991f;
      int f = c > (double)thr ? (Ed[q].flags | kPoOutlier) : (Ed[q].flags & ~kPoOutlier);
      nb[0] += (f & kPoOutlier) ? 1.0 : 0.0;
      if (it == 2) f &= ~kPoRobust;
      Ed[q].flags = f;
    }
    block_sum<1>(nb, sm.red, sm.H, nw);
    nBad = (int)sm.H[0];
    __syncthreads();  // sm.H is rewritten by the next round's count
    if (N < 10) break;
  }
#pragma unroll
  for (int q = 0; q < IT; q++) {
    const int i = tid + q * kPoThreads;
    if (i < N) D.outlier[i] = (Ed[q].flags & kPoOutlier) ? 1 : 0;
  }
  if (tid == 0) {
    dse3_to_float(P, D.pose_out);
    *D.n_inliers = N - nBad;
#ifdef MMT_PO_PROFILE
    printf("[po profile] N %d passes %d (rejected trials %d) cycles: solve+ctl %lld linearise "
           "%lld reduce %lld light %d\n", N, npass, nrej, pp[0], pp[1], pp[2], nlight);
#endif
  }
#undef PL_T
}

__device__ __forceinline__ bool pose_opt_trivial(const PoseOptDesc& D, int N) {
  if (N >= 3) return false;
  if (threadIdx.x == 0) {
    for (int k = 0; k < 16; k++) D.pose_out[k] = D.Tcw[k];
    *D.n_inliers = 0;
  }
  for (int i = threadIdx.x; i < N; i += blockDim.x) D.outlier[i] = 0;
  return true;
}

// n_lo: counts at or below it belong to another launch (-1: every count)
__global__ __launch_bounds__(256) void k_pose_opt(const PoseOptDesc* __restrict__ descs,
                                                  int n_lo) {
  __shared__ PoSmem sm;
  const PoseOptDesc& D = descs[blockIdx.x];
  const int N = D.n;
  if (N <= n_lo) return;
  if (pose_opt_trivial(D, N)) return;
  if (N <= kPoseOptMaxEdges)
    pose_opt_body<false>(D, N, sm);
  else
    pose_opt_body<true>(D, N, sm);
}

template <int IT>
__global__ __launch_bounds__(kPoThreads) void k_pose_opt_l(const PoseOptDesc* __restrict__ descs,
                                                           int n_lo) {
  __shared__ PoSmemL sm;
  const PoseOptDesc& D = descs[blockIdx.x];
  const int N = D.n;
  // edge counts outside (n_lo, IT * kPoThreads] belong to another launch (the host launches the
  // variants whose ranges cover its bound; the count is known on the device only)
  if (N <= n_lo || N > IT * kPoThreads) return;
  if (pose_opt_trivial(D, N)) return;
  pose_opt_light<IT>(D, N, sm);
}

void launch_pose_opt(const PoseOptDesc* d_descs, int nsolves, int n_max, hipStream_t st) {
  // The edge count is known on the device only: every variant whose range meets [0, n_max] is
  // launched and the ones outside the solve's count return at once (n_max is a bound).  Light
  // trial passes + lambda candidates, two edges per thread up to 2 * kPoThreads, four up to
  // 4 * kPoThreads, the LDS kernel beyond.  One kernel holding several variants spills (580 B per
  // lane), so each is a launch of its own.  The variants for the larger counts go first: a
  // 512-thread workgroup with 132 KB of LDS that queued behind the object path's RANSAC grids
  // waited for them to retire (the motion-model solve's no-op k_pose_opt_l<4> took 5-100 µs,
  // median 64, after its k_pose_opt_l<2>); ahead of it, it is placed before those grids.
  if (n_max > 2 * kPoThreads)
    hipLaunchKernelGGL(k_pose_opt_l<4>, dim3(nsolves), dim3(kPoThreads), 0, st, d_descs,
                       2 * kPoThreads);
  if (n_max > 4 * kPoThreads)
    hipLaunchKernelGGL(k_pose_opt, dim3(nsolves), dim3(256), 0, st, d_descs, 4 * kPoThreads);
  hipLaunchKernelGGL(k_pose_opt_l<2>, dim3(nsolves), dim3(kPoThreads), 0, st, d_descs, -1);
  MMT_HIP(hipGetLastError());
}


}  // namespace mmt
