// multimot_track_amd/csrc/mmt_ba.hip -- the solve of Optimizer::LocalBundleAdjustment (reference
// src/Optimizer.cc:3394-3665) as ONE persistent 512-thread workgroup: both rounds
// (optimize(5) with Huber kernels, the level-1 split of bad edges, optimize(10) without kernels),
// every LM iteration and trial, and the final erase test, with no host round trip.
//
// g2o semantics restated (the CPU checker is oracle/ba_ref.cpp):
//   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ computeError, linearizeOplus (types_six_dof_expmap
//   .h:91-141, .cpp:103-234); constructQuadraticForm with rho' Omega (base_binary_edge.hpp:55-115);
//   BlockSolver_6_3 Schur complement over the points (block_solver.hpp:406-489);
//   OptimizationAlgorithmLevenberg::solve (lambda init tau * max diagonal, rho, the 2/3 - 1/3 lambda
//   update, 10 trials, Raul's stop) and SparseOptimizer::optimize's chi2-increase stop; the solver's
//   x persists across trials (a failed solve re-applies the previous one); edges set to level 1
//   keep the error of their last evaluation.
//
// Work split (sizes of the synthetic C3 sequence: ~3,500 edges, ~3,000 points, ~6 keyframes):
//   * linearisation, point pass: one thread per point walks its edges (CSR, edge order) and keeps
//     the 3x3 H_ll / b_l in registers; it stores each edge's H_pl block (6x3);
//   * linearisation, keyframe pass: one wave per optimised keyframe sums J_p^T w J_p / J_p^T w e over
//     its edges (lanes strided, 27 register sums, DPP wave sums): fixed order, no atomics;
//   * Schur complement: per point D^-1 = (H_ll + lambda I)^-1 (Eigen's cofactor inverse), and per
//     edge Y = H_pl D^-1 and H_pl D^-1 b_l; then one wave per keyframe-pair block sums its
//     (edge, edge) triples (36 register sums per lane);
//   * the reduced camera system (6 x optimised keyframes) in LDS, LDL^T left-looking in the CPU
//     checker's operation order (one row per lane, one wave while it has at most 64 rows), the
//     substitutions on one lane;
//   * increments, update, errors, chi2 and the scale term per point / keyframe / edge.
// Every reduction runs in a fixed order, so the kernel is deterministic; it agrees with the CPU
// checker to rounding (sums in another association).  FP64 throughout; no MFMA (6x6 / 3x3 blocks).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <climits>
#include <cmath>
#include <cstring>
#include <map>

#include "mmt_ba.h"
#include "mmt_devmath.h"
#include "mmt_internal.h"

namespace mmt {

namespace {

constexpr int kBAThreads = 512;
constexpr int kBAWaves = kBAThreads / 64;
constexpr int kLdsRows = 96;  // reduced systems of up to 16 optimised keyframes live in LDS

struct BAWork {  // global scratch (doubles unless noted), carved from d.ws
  DSE3* pose;
  DSE3* pose_b;
  double* X;     // 3 n_pt
  double* Xb;
  double* Hll;   // 9 n_pt
  double* bl;    // 3 n_pt
  double* Dinv;  // 9 n_pt
  double* err;   // 3 n_edge
  double* Hpl;   // 18 n_edge
  double* Y;     // 18 n_edge
  double* cv;    // 6 n_edge
  double* Hpp;   // 36 n_opt
  double* bp;    // 6 n_opt
  double* x;     // 6 n_opt + 3 n_pt (g2o's _x: poses, then points)
  double* S;     // n6 x n6 (when the system does not fit in LDS)
  double* vec;   // 3 n6: bs, D, y (idem)
  uint8_t* level;  // n_edge
  uint8_t* kf_act; // n_kf: keyframe has an active edge this round
  uint8_t* pt_act; // n_pt
};

__device__ BAWork carve(const BADesc& d) {
  BAWork w;
  double* p = d.ws;
  const size_t n6 = 6 * (size_t)d.n_opt;
  w.pose = reinterpret_cast<DSE3*>(p); p += 7 * (size_t)d.n_kf;
  w.pose_b = reinterpret_cast<DSE3*>(p); p += 7 * (size_t)d.n_kf;
  w.X = p; p += 3 * (size_t)d.n_pt;
  w.Xb = p; p += 3 * (size_t)d.n_pt;
  w.Hll = p; p += 9 * (size_t)d.n_pt;
  w.bl = p; p += 3 * (size_t)d.n_pt;
  w.Dinv = p; p += 9 * (size_t)d.n_pt;
  w.err = p; p += 3 * (size_t)d.n_edge;
  w.Hpl = p; p += 18 * (size_t)d.n_edge;
  w.Y = p; p += 18 * (size_t)d.n_edge;
  w.cv = p; p += 6 * (size_t)d.n_edge;
  w.Hpp = p; p += 36 * (size_t)d.n_opt;
  w.bp = p; p += 6 * (size_t)d.n_opt;
  w.x = p; p += n6 + 3 * (size_t)d.n_pt;
  w.S = p; p += n6 * n6;
  w.vec = p; p += 3 * n6;
  uint8_t* b = reinterpret_cast<uint8_t*>(p);
  w.level = b; b += d.n_edge;
  w.kf_act = b; b += d.n_kf;
  w.pt_act = b;
  return w;
}

struct Cam {
  double fx, fy, cx, cy, bf;
};

__device__ __forceinline__ void se3_map(const DSE3& T, const double* X, double* pc) {
  dq_rotate(T.q, X[0], X[1], X[2], pc[0], pc[1], pc[2]);
  pc[0] += T.t[0];
  pc[1] += T.t[1];
  pc[2] += T.t[2];
}

// computeError; returns chi2 = e^T (s I) e
__device__ __forceinline__ double edge_error(const float* obs, double s, bool stereo,
                                             const DSE3& T, const double* X, const Cam& c,
                                             double* e) {
  double pc[3];
  se3_map(T, X, pc);
  if (!stereo) {
    const double px = pc[0] / pc[2], py = pc[1] / pc[2];
    e[0] = (double)obs[0] - (px * c.fx + c.cx);
    e[1] = (double)obs[1] - (py * c.fy + c.cy);
    e[2] = 0;
    return s * (e[0] * e[0] + e[1] * e[1]);
  }
  const float invz = 1.0f / pc[2];
  const double u = pc[0] * invz * c.fx + c.cx, v = pc[1] * invz * c.fy + c.cy;
  e[0] = (double)obs[0] - u;
  e[1] = (double)obs[1] - v;
  e[2] = (double)obs[2] - (u - c.bf * invz);
  return s * (e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
}

__device__ __forceinline__ double edge_chi2(const double* e, double s, bool stereo) {
  return stereo ? s * (e[0] * e[0] + e[1] * e[1] + e[2] * e[2]) : s * (e[0] * e[0] + e[1] * e[1]);
}

__device__ __forceinline__ void huber_rho(double e, double delta, double& r0, double& r1) {
  const double dsqr = delta * delta;
  if (e <= dsqr) {
    r0 = e;
    r1 = 1.;
  } else {
    const double s = sqrt(e);
    r0 = 2 * s * delta - dsqr;
    r1 = delta / s;
  }
}

// linearizeOplus: the pose Jacobian (rows x 6) always, the point Jacobian (rows x 3) on request
template <bool POINT>
__device__ __forceinline__ void edge_jac(bool stereo, const DSE3& T, const double* X, const Cam& c,
                                         double (&Jp)[3][6], double (&Jl)[3][3]) {
  double pc[3];
  se3_map(T, X, pc);
  const double x = pc[0], y = pc[1], z = pc[2], z_2 = z * z;
  if (POINT) {
    double R[3][3];
    dq_to_R(T.q, R);
    if (!stereo) {
      const double tmp[2][3] = {{c.fx, 0, -x / z * c.fx}, {0, c.fy, -y / z * c.fy}};
      const double s = -1. / z;
#pragma unroll
      for (int r = 0; r < 2; r++)
#pragma unroll
        for (int k = 0; k < 3; k++) {
          double a = 0;
#pragma unroll
          for (int m = 0; m < 3; m++) a += (s * tmp[r][m]) * R[m][k];
          Jl[r][k] = a;
        }
      Jl[2][0] = Jl[2][1] = Jl[2][2] = 0;
    } else {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        Jl[0][k] = -c.fx * R[0][k] / z + c.fx * x * R[2][k] / z_2;
        Jl[1][k] = -c.fy * R[1][k] / z + c.fy * y * R[2][k] / z_2;
        Jl[2][k] = Jl[0][k] - c.bf * R[2][k] / z_2;
      }
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
  if (stereo) {
    Jp[2][0] = Jp[0][0] - c.bf * y / z_2;
    Jp[2][1] = Jp[0][1] + c.bf * x / z_2;
    Jp[2][2] = Jp[0][2];
    Jp[2][3] = Jp[0][3];
    Jp[2][4] = 0;
    Jp[2][5] = Jp[0][5] - c.bf / z_2;
  } else {
#pragma unroll
    for (int k = 0; k < 6; k++) Jp[2][k] = 0;
  }
}

// Eigen's fixed-size 3x3 inverse (cofactors of column 0, det, adjugate rows)
__device__ __forceinline__ void inverse3(const double (&m)[9], double (&r)[9]) {
#define COF(i, j)                                                                           \
  (m[3 * (((i) + 1) % 3) + ((j) + 1) % 3] * m[3 * (((i) + 2) % 3) + ((j) + 2) % 3] -         \
   m[3 * (((i) + 1) % 3) + ((j) + 2) % 3] * m[3 * (((i) + 2) % 3) + ((j) + 1) % 3])
  const double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
  const double det = c0 * m[0] + c1 * m[3] + c2 * m[6];
  const double invdet = 1.0 / det;
  r[0] = c0 * invdet;
  r[1] = c1 * invdet;
  r[2] = c2 * invdet;
  r[3] = COF(0, 1) * invdet;
  r[4] = COF(1, 1) * invdet;
  r[5] = COF(2, 1) * invdet;
  r[6] = COF(0, 2) * invdet;
  r[7] = COF(1, 2) * invdet;
  r[8] = COF(2, 2) * invdet;
#undef COF
}

// workgroup sum / max of one double per thread, identical in every thread (fixed order)
__device__ __forceinline__ double wg_sum1(double v, double* part) {
  v = wave_sum_dpp(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = v;
  __syncthreads();
  double s = 0;
#pragma unroll
  for (int w = 0; w < kBAWaves; w++) s += part[w];
  __syncthreads();
  return s;
}

__device__ __forceinline__ double wg_max1(double v, double* part) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = v;
  __syncthreads();
  double m = 0;
#pragma unroll
  for (int w = 0; w < kBAWaves; w++) m = fmax(m, part[w]);
  __syncthreads();
  return m;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

namespace {
// ================================================================== multi-kernel solve
// The local BA's LM spread over the chip: one LM trial is a chain of short kernels on the
// caller's stream (points, keyframe-pair blocks and keyframes in parallel; the reduced camera
// system and the LM decision in one workgroup each), with the LM state in device memory.  The host
// enqueues trials in batches and reads the state's done flag after each batch; every kernel of a
// finished solve returns at once.  Round 4's first version ran the whole solve in one workgroup
// (10-11 ms per local BA of the C3 sequence); spread, a trial costs a few microseconds per kernel.
//   per iteration (need_lin):  k_ba2_lin   one thread per point: errors, robust chi2, H_ll, b_l,
//                                          H_pl and the edge's pose terms (J_p^T w J_p, J_p^T w e)
//                              k_ba2_kfsum one workgroup per optimised keyframe: H_pp, b_p
//   per trial:                 k_ba2_p1    one thread per point: (H_ll + lambda I)^-1, Y, H_pl D^-1 b_l
//                              k_ba2_p2    one workgroup per keyframe-pair block / keyframe: Schur sums
//                              k_ba2_p3    one workgroup: the reduced system, LDL^T, increments, trial poses
//                              k_ba2_p4    one thread per point: point increments, trial errors, chi2;
//                                          its last workgroup then takes the LM decision (rho,
//                                          lambda, Raul's stop, the chi2-increase stop) and the
//                                          iteration and round bookkeeping (ba2_decide)
// The estimates are double-buffered (current / trial, swapped on acceptance), so a rejected trial
// needs no restore.  Every reduction has a fixed order: the solve is deterministic.

constexpr int kMkThreads = 256;
constexpr int kMkWaves = kMkThreads / 64;
constexpr int kMkSolveThreads = 512;
constexpr int kMkDecideThreads = 1024;

struct BAState {
  int done, round, iter, qmax, need_lin, lam_init, cb, ok2, nBad, nact;
  int spec_ok;  // the last trial was accepted: k_ba2_p4 linearised at it, no k_ba2_lin needed
  int it_done[2], trials[2];
  double lambda, ni, chk, currentChi, iniChi, scale_p;
  long long prof[8];  // k_ba2_p3 phase times (wall clock ticks, 100 MHz), summed over trials
};

struct BAWork2 {
  BAState* st;
  DSE3* pose;       // [2][n_kf]: the current estimate (buffer st->cb) and the trial
  double* X;        // [2][3 n_pt]
  // the linearisation at the current estimate (buffer st->cb) and at the trial (k_ba2_p4)
  double* Hll;      // [2][9 n_pt]
  double* bl;       // [2][3 n_pt]
  double* Dinv;     // 9 n_pt
  double* err;      // 3 n_edge: the last computed errors
  double* Hpl;      // [2][18 n_edge]
  double* Hpe;      // [2][27 n_edge]: the edge's J_p^T w J_p (21, upper triangle), J_p^T w (-e) (6)
  double* Y;        // 18 n_edge
  double* cv;       // 6 n_edge
  double* Hpp;      // 36 n_opt
  double* bp;       // 6 n_opt
  double* cvs;      // 6 n_opt: the keyframe's sum of H_pl D^-1 b_l
  double* Sblk;     // 36 n_blk
  double* x;        // 6 n_opt + 3 n_pt (g2o's _x: poses, then points)
  double* S;        // n6 x n6 when the reduced system does not fit in LDS
  double* vec;      // 3 n6 (idem)
  const int4* kitem;        // keyframe items: (optimised keyframe, kf_edges range of <= 256)
  const int* kitem_start;   // n_opt + 1: each optimised keyframe's items
  const int4* bitem;        // block items: (block, trip range of <= 256)
  const int* bitem_start;   // n_blk + 1
  int n_kitem, n_bitem;
  double* Hpart;    // 27 per keyframe item: its edges' pose terms
  double* Spart;    // 36 per block item: its triples' sum of Y H_pl^T
  double* cvpart;   // 6 per keyframe item: its edges' H_pl D^-1 b_l
  double* linpart;  // 2 per point workgroup: chi2, largest active H_ll diagonal
  double* p4part;   // 2 per point workgroup: trial chi2, scale
  unsigned* p4cnt;  // k_ba2_p4's workgroups done with the trial (the last one decides, then resets)
  uint8_t* level;   // n_edge
  int* eopt;        // n_edge: the edge's optimised-keyframe index, -1 for a fixed keyframe
  uint8_t* kf_act;  // n_kf: optimised keyframe with an active edge this round
  uint8_t* pt_act;  // n_pt
  int gP;           // partial sums: one per point workgroup
  int gPp;          // point workgroups (one thread per point; k_ba2_p1's heavy waves follow them)
  const int* heavy; // the points with more than kBaHeavy edges, one wave each
  int n_heavy;
  double* hres;     // 2 n_pt: a heavy point's (chi2, H_ll diagonal max) or (trial chi2, scale)
  int spec;         // k_ba2_p4<true>: the trial kernel linearises at the trial state
};

// workgroup sums of K <= 64 values per thread, fixed order (DPP wave sums, then the waves in
// order); sum q lands in out[q] (LDS), visible to every thread on return
template <int K, int NW>
__device__ __forceinline__ void wg_sumK(const double (&v)[K], double* part, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double mine = 0;
#pragma unroll
  for (int q = 0; q < K; q++) {
    const double s = wave_sum_dpp(v[q]);
    if (lane == q) mine = s;
  }
  if (lane < K) part[wave * K + lane] = mine;
  __syncthreads();
  if ((int)threadIdx.x < K) {
    double s = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) s += part[w * K + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

template <int NW>
__device__ __forceinline__ double wg_maxN(double v, double* part) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = v;
  __syncthreads();
  double m = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) m = fmax(m, part[w]);
  __syncthreads();
  return m;
}

// computeLambdaInit over the round's vertices: 1e-5 x the largest diagonal entry of the active
// optimised keyframes' H_pp and the active points' H_ll (the latter from k_ba2_lin's partials)
// the upper-triangle index of H_pp entry (r, r) in the 21 pose terms (rows r0, columns c0 >= r0)
__device__ __forceinline__ int ba2_diag_q(int r) { return 6 * r - r * (r - 1) / 2; }

// keyframe a's sum of pose term q over its items, in item order (k_ba2_p1 and k_ba2_p3 both
// compute H_pp this way: the same bits)
// base[stride * b] + ... + base[stride * (e - 1)] added in index order from 0 (the scalar sum's
// rounding), the loads of U items issued together (clamped indices, no branch between them)
template <int U = 8>
__device__ __forceinline__ double ordered_sum(const double* base, size_t stride, int b, int e) {
  double s = 0;
  for (int it = b; it < e; it += U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = base[stride * (size_t)min(it + u, e - 1)];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (it + u < e) s += v[u];
  }
  return s;
}

__device__ __forceinline__ double ba2_hsum(const BAWork2& w, int a, int q) {
  return ordered_sum(w.Hpart + q, 27, w.kitem_start[a], w.kitem_start[a + 1]);
}

// computed by wave 0 (lanes over the point workgroups and the (keyframe, diagonal) pairs) and
// returned to every thread of the workgroup through `sh` (one barrier)
__device__ __forceinline__ double ba2_lambda_init(const BADesc& d, const BAWork2& w, double* sh) {
  if (threadIdx.x < 64) {
    double m = 0;
    for (int g = threadIdx.x; g < w.gP; g += 64) m = fmax(m, w.linpart[2 * g + 1]);
    for (int q = threadIdx.x; q < 6 * d.n_opt; q += 64) {
      const int a = q / 6;
      if (w.kf_act[d.opt_kf[a]]) m = fmax(m, fabs(ba2_hsum(w, a, ba2_diag_q(q % 6))));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if (threadIdx.x == 0) *sh = 1e-5 * m;
  }
  __syncthreads();
  return *sh;
}

__device__ __forceinline__ Cam ba_cam(const BADesc& d) { return Cam{d.fx, d.fy, d.cx, d.cy, d.bf}; }

// thHuberMono = sqrt(5.991) stored as a float (Optimizer.cc:3457-3458)
__device__ __forceinline__ double huber_mono() { return (double)(float)sqrt(5.991); }
__device__ __forceinline__ double huber_stereo() { return (double)(float)sqrt(7.815); }

__global__ __launch_bounds__(kMkThreads) void k_ba2_init(BADesc d, BAWork2 w) {
  const int gt = blockIdx.x * kMkThreads + threadIdx.x, gs = gridDim.x * kMkThreads;
  const size_t n6 = 6 * (size_t)d.n_opt;
  for (int j = gt; j < d.n_pt; j += gs) {
    for (int r = 0; r < 3; r++) {
      w.X[3 * (size_t)j + r] = (double)d.Xw[3 * (size_t)j + r];
      w.x[n6 + 3 * (size_t)j + r] = 0;
    }
    w.pt_act[j] = d.pt_start[j + 1] > d.pt_start[j] ? 1 : 0;
  }
  for (int e = gt; e < d.n_edge; e += gs) {
    w.level[e] = 0;
    w.eopt[e] = d.opt_of[d.e_kf[e]];
    w.err[3 * (size_t)e] = w.err[3 * (size_t)e + 1] = w.err[3 * (size_t)e + 2] = 0;
  }
  if (blockIdx.x == 0) {
    for (int k = threadIdx.x; k < d.n_kf; k += kMkThreads) {
      w.pose[k] = dse3_from_float(d.Tcw + 16 * (size_t)k);
      w.kf_act[k] = 0;
    }
    for (int q = threadIdx.x; q < (int)n6; q += kMkThreads) w.x[q] = 0;
    __syncthreads();
    for (int a = threadIdx.x; a < d.n_opt; a += kMkThreads)
      if (d.kf_start[a + 1] > d.kf_start[a]) w.kf_act[d.opt_kf[a]] = 1;
    if (threadIdx.x == 0) {
      *w.p4cnt = 0;
      BAState& s = *w.st;
      memset(&s, 0, sizeof(s));
      s.need_lin = 1;
      s.lam_init = 1;
      s.ni = 2;
      s.done = d.n_edge == 0 ? 1 : 0;
    }
  }
}

// Points with more edges than this are linearised, solved and tried by a wave each (lane = edge)
// instead of one thread: a point seen from far away by every keyframe (a key at disparity 0 has depth
// bf / 0 = inf, and CreateNewMapPoints triangulates such keys into far points) collects a hundred
// or more edges, and its thread's serial edge loop set k_ba2_lin / k_ba2_p4 at 100-160 us.
#ifndef MMT_BA_HEAVY
#define MMT_BA_HEAVY 2  // A/B builds: tools/ab_build.sh <tag> --src mmt_ba.hip -DMMT_BA_HEAVY=..
#endif
constexpr int kBaHeavy = MMT_BA_HEAVY;  // 2: BA 2,060 -> 1,800 us per keyframe against 8 (profiles/r06_ab_lmprio_baheavy.txt)

__device__ __forceinline__ bool ba2_heavy(const BADesc& d, int j) {
  return d.pt_start[j + 1] - d.pt_start[j] > kBaHeavy;
}

// one active edge e of the point at X: its error (stored), robust rho (returned: r0), H_pl and the
// pose terms (stored for an edge to an optimised keyframe), and its share of the point's H_ll
// (acc9) and b_l (g3)
__device__ __forceinline__ double ba2_lin_edge(const BADesc& d, const BAWork2& w, int e,
                                               const DSE3* pose, const double (&X)[3], bool robust,
                                               double* Hpl_b, double* Hpe_b, double (&acc9)[9],
                                               double (&g3)[3]) {
  const Cam cam = ba_cam(d);
  const double dMono = huber_mono(), dStereo = huber_stereo();
  const int k = d.e_kf[e];
  const bool stereo = !(d.e_obs[3 * (size_t)e + 2] < 0);
  const double s = (double)d.e_s[e];
  double er[3];
  const double c = edge_error(d.e_obs + 3 * (size_t)e, s, stereo, pose[k], X, cam, er);
#pragma unroll
  for (int r = 0; r < 3; r++) w.err[3 * (size_t)e + r] = er[r];
  double r0 = c, r1 = 1.0;
  if (robust) huber_rho(c, stereo ? dStereo : dMono, r0, r1);
  double Jp[3][6], Jl[3][3];
  edge_jac<true>(stereo, pose[k], X, cam, Jp, Jl);
  const int rows = stereo ? 3 : 2;
  const double wt = r1 * s;
  double om[3];
#pragma unroll
  for (int r = 0; r < 3; r++) om[r] = r < rows ? -(s * er[r]) * r1 : 0.0;
#pragma unroll
  for (int a = 0; a < 3; a++) {
#pragma unroll
    for (int b = 0; b < 3; b++) {
      double acc = 0;
      _Pragma("unroll") for (int r = 0; r < 3; r++) if (r < rows) acc += Jl[r][a] * wt * Jl[r][b];
      acc9[3 * a + b] = acc;
    }
    double g = 0;
    _Pragma("unroll") for (int r = 0; r < 3; r++) if (r < rows) g += Jl[r][a] * om[r];
    g3[a] = g;
  }
  if (d.opt_of[k] >= 0) {
    double* hpl = &Hpl_b[18 * (size_t)e];
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
      for (int b = 0; b < 3; b++) {
        double acc = 0;
        _Pragma("unroll") for (int r = 0; r < 3; r++) if (r < rows) acc += Jp[r][a] * wt * Jl[r][b];
        hpl[3 * a + b] = acc;
      }
    double* hpe = &Hpe_b[27 * (size_t)e];
    int q = 0;
#pragma unroll
    for (int r0i = 0; r0i < 6; r0i++)
#pragma unroll
      for (int c0 = r0i; c0 < 6; c0++) {
        double v = 0;
        _Pragma("unroll") for (int r = 0; r < 3; r++) if (r < rows) v += Jp[r][r0i] * wt * Jp[r][c0];
        hpe[q++] = v;
      }
#pragma unroll
    for (int r0i = 0; r0i < 6; r0i++) {
      double g = 0;
      _Pragma("unroll") for (int r = 0; r < 3; r++) if (r < rows) g += Jp[r][r0i] * (-(s * er[r]) * r1);
      hpe[21 + r0i] = g;
    }
  }
  return r0;
}

// the trial error of active edge e at (pose, X) (stored) and its robust rho
__device__ __forceinline__ double ba2_trial_edge(const BADesc& d, const BAWork2& w, int e,
                                                 const DSE3* tri, const double (&X)[3],
                                                 bool robust) {
  const Cam cam = ba_cam(d);
  const bool stereo = !(d.e_obs[3 * (size_t)e + 2] < 0);
  const double c = edge_error(d.e_obs + 3 * (size_t)e, (double)d.e_s[e], stereo, tri[d.e_kf[e]],
                              X, cam, &w.err[3 * (size_t)e]);
  double r0 = c, r1;
  if (robust) huber_rho(c, stereo ? huber_stereo() : huber_mono(), r0, r1);
  return r0;
}

// A heavy point's wave: lane l takes edge e0 + l of each 64-edge chunk, stages its shares in the
// wave's LDS rows, and every lane then adds them up in edge order (uniform broadcast reads): the
// point's H_ll, b_l and chi2 carry the one-thread loop's bits.  K values per edge.
template <int K>
__device__ __forceinline__ void ba2_wave_ordered_add(double* sh, int lane, int n, const bool valid,
                                                     const double (&v)[K], double (&sum)[K]) {
#pragma unroll
  for (int q = 0; q < K; q++) sh[K * lane + q] = valid ? v[q] : 0.0;
  const unsigned long long vb = __ballot(valid);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int k = 0; k < n; k++) {
    if (!((vb >> k) & 1ull)) continue;  // an inactive edge adds nothing (skipped, as the loop does)
#pragma unroll
    for (int q = 0; q < K; q++) sum[q] += sh[K * k + q];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// computeActiveErrors + activeRobustChi2 + buildSystem's point side for point j at (pose, X):
// its active edges' errors (stored), robust chi2 (returned), H_ll and b_l of the point, H_pl and
// the pose terms of each edge, into linearisation buffer `lb`; *mx = the largest H_ll diagonal
__device__ __forceinline__ double ba2_lin_point(const BADesc& d, const BAWork2& w, int j,
                                               const DSE3* pose, const double (&X)[3], bool robust,
                                               int lb, double* mx) {
  double* Hpl_b = w.Hpl + (size_t)lb * 18 * d.n_edge;
  double* Hpe_b = w.Hpe + (size_t)lb * 27 * d.n_edge;
  double chi = 0;
  {
    double hl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b3[3] = {0, 0, 0};
    for (int e = d.pt_start[j]; e < d.pt_start[j + 1]; e++) {
      if (w.level[e]) continue;
      double acc9[9], g3[3];
      chi += ba2_lin_edge(d, w, e, pose, X, robust, Hpl_b, Hpe_b, acc9, g3);
#pragma unroll
      for (int q = 0; q < 9; q++) hl[q] += acc9[q];
#pragma unroll
      for (int a = 0; a < 3; a++) b3[a] += g3[a];
    }
    double* Hll_b = w.Hll + (size_t)lb * 9 * d.n_pt;
    double* bl_b = w.bl + (size_t)lb * 3 * d.n_pt;
#pragma unroll
    for (int q = 0; q < 9; q++) Hll_b[9 * (size_t)j + q] = hl[q];
#pragma unroll
    for (int q = 0; q < 3; q++) bl_b[3 * (size_t)j + q] = b3[q];
    *mx = fmax(fabs(hl[0]), fmax(fabs(hl[4]), fabs(hl[8])));
  }
  return chi;
}

// ba2_lin_point by the wave of a heavy point (every lane returns the point's chi2 and *mx; sh: the
// wave's 64 x 13 LDS staging rows)
__device__ __forceinline__ double ba2_lin_point_wave(const BADesc& d, const BAWork2& w, int j,
                                                    const DSE3* pose, const double (&X)[3],
                                                    bool robust, int lb, double* mx, double* sh) {
  const int lane = threadIdx.x & 63;
  double* Hpl_b = w.Hpl + (size_t)lb * 18 * d.n_edge;
  double* Hpe_b = w.Hpe + (size_t)lb * 27 * d.n_edge;
  double sum[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // chi2, H_ll (9), b_l (3)
  const int e1 = d.pt_start[j + 1];
  for (int e0 = d.pt_start[j]; e0 < e1; e0 += 64) {
    const int e = e0 + lane;
    const bool valid = e < e1 && !w.level[e];
    double v[13];
    if (valid) {
      double acc9[9], g3[3];
      v[0] = ba2_lin_edge(d, w, e, pose, X, robust, Hpl_b, Hpe_b, acc9, g3);
#pragma unroll
      for (int q = 0; q < 9; q++) v[1 + q] = acc9[q];
#pragma unroll
      for (int q = 0; q < 3; q++) v[10 + q] = g3[q];
    }
    ba2_wave_ordered_add<13>(sh, lane, min(64, e1 - e0), valid, v, sum);
  }
  if (lane == 0) {
    double* Hll_b = w.Hll + (size_t)lb * 9 * d.n_pt;
    double* bl_b = w.bl + (size_t)lb * 3 * d.n_pt;
#pragma unroll
    for (int q = 0; q < 9; q++) Hll_b[9 * (size_t)j + q] = sum[1 + q];
#pragma unroll
    for (int q = 0; q < 3; q++) bl_b[3 * (size_t)j + q] = sum[10 + q];
  }
  *mx = fmax(fabs(sum[1]), fmax(fabs(sum[5]), fabs(sum[9])));
  return sum[0];
}

// the linearisation at the current estimate, one thread per point (the start of each round, and an
// iteration that follows a rejected trial; after an accepted one k_ba2_p4 has linearised already)
__global__ __launch_bounds__(kMkThreads) void k_ba2_lin(BADesc d, BAWork2 w) {
  __shared__ double s_part[2 * kMkWaves];
  const BAState* st = w.st;
  if (st->done || !st->need_lin || st->spec_ok) return;
  const bool robust = st->round == 0;
  const int cb = st->cb;
  const DSE3* pose = w.pose + (size_t)cb * d.n_kf;
  const double* Xc = w.X + (size_t)cb * 3 * d.n_pt;
  const int j = blockIdx.x * kMkThreads + threadIdx.x;
  double chi = 0, mx = 0;
  if (j < d.n_pt) {
    double m = 0;
    if (ba2_heavy(d, j)) {  // linearised by its wave in k_ba2_lin_heavy: its results
      chi = w.hres[2 * (size_t)j];
      m = w.hres[2 * (size_t)j + 1];
    } else {
      const double X[3] = {Xc[3 * (size_t)j], Xc[3 * (size_t)j + 1], Xc[3 * (size_t)j + 2]};
      chi = ba2_lin_point(d, w, j, pose, X, robust, cb, &m);
    }
    if (w.pt_act[j]) mx = m;
  }
  const double cs = wave_sum_dpp(chi);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) s_part[wave] = cs;
  const double m = wg_maxN<kMkWaves>(mx, s_part + kMkWaves);  // its barrier orders s_part too
  if (threadIdx.x == 0) {
    double t = 0;
#pragma unroll
    for (int q = 0; q < kMkWaves; q++) t += s_part[q];
    w.linpart[2 * blockIdx.x] = t;
    w.linpart[2 * blockIdx.x + 1] = m;
  }
}

// the heavy points' linearisation, a wave each, before k_ba2_lin (which takes their chi2 and
// H_ll diagonal maximum from hres into its sums at the point's own place: the sums' order is the
// one-thread-per-point kernel's)
__global__ __launch_bounds__(kMkThreads) void k_ba2_lin_heavy(BADesc d, BAWork2 w) {
  __shared__ double s_stage[kMkWaves][64 * 13];
  const BAState* st = w.st;
  if (st->done || !st->need_lin || st->spec_ok) return;
  const int wave = threadIdx.x >> 6;
  const int hi = (int)blockIdx.x * kMkWaves + wave;
  if (hi >= w.n_heavy) return;
  const int cb = st->cb;
  const DSE3* pose = w.pose + (size_t)cb * d.n_kf;
  const double* Xc = w.X + (size_t)cb * 3 * d.n_pt;
  const int j = w.heavy[hi];
  const double X[3] = {Xc[3 * (size_t)j], Xc[3 * (size_t)j + 1], Xc[3 * (size_t)j + 2]};
  double m = 0;
  const double c = ba2_lin_point_wave(d, w, j, pose, X, st->round == 0, cb, &m, s_stage[wave]);
  if ((threadIdx.x & 63) == 0) {
    w.hres[2 * (size_t)j] = c;
    w.hres[2 * (size_t)j + 1] = m;
  }
}

// buildSystem's keyframe side: one workgroup per keyframe item (<= 256 edges of one optimised
// keyframe, one per thread) sums its active edges' pose terms into Hpart
__global__ __launch_bounds__(kMkThreads) void k_ba2_kfsum(BADesc d, BAWork2 w) {
  __shared__ double s_part[27 * kMkWaves];
  __shared__ double s_out[32];
  const BAState* st = w.st;
  if (st->done || !st->need_lin) return;
  const int4 it = w.kitem[blockIdx.x];
  const int t = it.y + threadIdx.x;
  double acc[27];
#pragma unroll
  for (int q = 0; q < 27; q++) acc[q] = 0;
  if (t < it.z) {
    const int e = d.kf_edges[t];
    if (!w.level[e]) {
      const double* h = &w.Hpe[(size_t)st->cb * 27 * d.n_edge + 27 * (size_t)e];
#pragma unroll
      for (int q = 0; q < 27; q++) acc[q] = h[q];
    }
  }
  wg_sumK<27, kMkWaves>(acc, s_part, s_out);
  if (threadIdx.x < 27) w.Hpart[27 * (size_t)blockIdx.x + threadIdx.x] = s_out[threadIdx.x];
}

// trial step 1, one thread per active point: D^-1 = (H_ll + lambda I)^-1 (Eigen's cofactor
// inverse), and per active edge to an optimised keyframe Y = H_pl D^-1 and H_pl D^-1 b_l
__global__ __launch_bounds__(kMkThreads) void k_ba2_p1(BADesc d, BAWork2 w) {
  const BAState* st = w.st;
  if (st->done) return;
  __shared__ double s_lam;
  const double lambda = st->lam_init ? ba2_lambda_init(d, w, &s_lam) : st->lambda;
  const bool heavy_wg = (int)blockIdx.x >= w.gPp;
  const int lane = threadIdx.x & 63;
  int j = blockIdx.x * kMkThreads + threadIdx.x;
  if (heavy_wg) {  // a wave per heavy point, lanes over its edges (each edge's Y and cv alone)
    const int hi = ((int)blockIdx.x - w.gPp) * kMkWaves + (int)(threadIdx.x >> 6);
    j = hi < w.n_heavy ? w.heavy[hi] : d.n_pt;
  } else if (j < d.n_pt && ba2_heavy(d, j)) {
    return;
  }
  if (j >= d.n_pt || !w.pt_act[j]) return;
  const int cb = st->cb;
  const double* Hll_c = w.Hll + (size_t)cb * 9 * d.n_pt;
  const double* bl_c = w.bl + (size_t)cb * 3 * d.n_pt;
  const double* Hpl_c = w.Hpl + (size_t)cb * 18 * d.n_edge;
  double Dm[9], Di[9];
#pragma unroll
  for (int q = 0; q < 9; q++) Dm[q] = Hll_c[9 * (size_t)j + q] + ((q % 4) == 0 ? lambda : 0.0);
  inverse3(Dm, Di);
  if (!heavy_wg || lane == 0) {
#pragma unroll
    for (int q = 0; q < 9; q++) w.Dinv[9 * (size_t)j + q] = Di[q];
  }
  const double* b3 = &bl_c[3 * (size_t)j];
  double db[3];
#pragma unroll
  for (int a = 0; a < 3; a++) db[a] = Di[3 * a] * b3[0] + Di[3 * a + 1] * b3[1] + Di[3 * a + 2] * b3[2];
  const int eb = d.pt_start[j] + (heavy_wg ? lane : 0), es = heavy_wg ? 64 : 1;
  for (int e = eb; e < d.pt_start[j + 1]; e += es) {
    if (w.level[e] || w.eopt[e] < 0) continue;
    const double* B = &Hpl_c[18 * (size_t)e];
    double* Ye = &w.Y[18 * (size_t)e];
    double* ce = &w.cv[6 * (size_t)e];
#pragma unroll
    for (int r = 0; r < 6; r++) {
      const double b0 = B[3 * r], b1 = B[3 * r + 1], b2 = B[3 * r + 2];
#pragma unroll
      for (int c = 0; c < 3; c++) Ye[3 * r + c] = b0 * Di[c] + b1 * Di[3 + c] + b2 * Di[6 + c];
      ce[r] = b0 * db[0] + b1 * db[1] + b2 * db[2];
    }
  }
}

// trial step 2: the Schur sums, one workgroup per block item (<= 256 (edge, edge) triples of one
// keyframe-pair block, one per thread) and per keyframe item (its edges' H_pl D^-1 b_l)
__global__ __launch_bounds__(kMkThreads) void k_ba2_p2(BADesc d, BAWork2 w) {
  __shared__ double s_part[36 * kMkWaves];
  __shared__ double s_out[64];
  const BAState* st = w.st;
  if (st->done) return;
  if ((int)blockIdx.x < w.n_bitem) {
    const int4 it = w.bitem[blockIdx.x];
    const int t = it.y + threadIdx.x;
    double acc[36];
#pragma unroll
    for (int q = 0; q < 36; q++) acc[q] = 0;
    if (t < it.z) {
      const int2 tr = d.trip[t];
      if (!w.level[tr.x] && !w.level[tr.y]) {
        const double* Ye = &w.Y[18 * (size_t)tr.x];
        const double* B2 = &w.Hpl[(size_t)st->cb * 18 * d.n_edge + 18 * (size_t)tr.y];
        double h2[18], y[18];
#pragma unroll
        for (int q = 0; q < 18; q++) {
          h2[q] = B2[q];
          y[q] = Ye[q];
        }
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
          for (int c = 0; c < 6; c++)
            acc[6 * r + c] = y[3 * r] * h2[3 * c] + y[3 * r + 1] * h2[3 * c + 1] + y[3 * r + 2] * h2[3 * c + 2];
      }
    }
    wg_sumK<36, kMkWaves>(acc, s_part, s_out);
    if (threadIdx.x < 36) w.Spart[36 * (size_t)blockIdx.x + threadIdx.x] = s_out[threadIdx.x];
  } else {
    const int ki = blockIdx.x - w.n_bitem;
    const int4 it = w.kitem[ki];
    const int t = it.y + threadIdx.x;
    double cs[6] = {0, 0, 0, 0, 0, 0};
    if (t < it.z) {
      const int e = d.kf_edges[t];
      if (!w.level[e]) {
#pragma unroll
        for (int r = 0; r < 6; r++) cs[r] = w.cv[6 * (size_t)e + r];
      }
    }
    wg_sumK<6, kMkWaves>(cs, s_part, s_out);
    if (threadIdx.x < 6) w.cvpart[6 * (size_t)ki + threadIdx.x] = s_out[threadIdx.x];
  }
}

// trial step 3, one workgroup: the reduced camera system H_pp + lambda I - sum Y H_pl^T (upper
// triangle, mirrored), b_schur, LDL^T right-looking (for every entry the left-looking sequence of
// operations of the CPU checker), the substitutions on one wave, the increment (stale on a zero
// pivot, as g2o re-applies its _x), the trial poses and the poses' share of the LM scale term
__global__ __launch_bounds__(kMkSolveThreads) void k_ba2_p3(BADesc d, BAWork2 w) {
  __shared__ double s_S[kLdsRows * kLdsRows];
  __shared__ double s_vec[3 * kLdsRows];
  __shared__ double s_vec2[2];
  __shared__ int s_ok;
  BAState* stp = w.st;
  if (stp->done) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n6 = 6 * d.n_opt;
  long long pt[6];
  pt[0] = wall_clock64();
  const bool lam_init = stp->lam_init != 0, need_lin = stp->need_lin != 0;
  const bool lin_ran = need_lin && !stp->spec_ok;
  const int cb = stp->cb;
  __shared__ double s_lam;
  const double lambda = lam_init ? ba2_lambda_init(d, w, &s_lam) : stp->lambda;
  double* S = n6 <= kLdsRows ? s_S : w.S;
  double* bs = n6 <= kLdsRows ? s_vec : w.vec;
  double* Dg = bs + n6;
  double* yv = Dg + n6;
  // the item partials summed in item order: H_pp, b_p, sum of H_pl D^-1 b_l, the block sums
  for (int q = tid; q < d.n_opt * 27; q += kMkSolveThreads) {
    const int a = q / 27, k = q % 27;
    const double v = ba2_hsum(w, a, k);
    if (k < 21) {
      int r0 = 0, kk = k;
      while (kk >= 6 - r0) {
        kk -= 6 - r0;
        r0++;
      }
      const int c0 = r0 + kk;
      w.Hpp[36 * (size_t)a + 6 * r0 + c0] = v;
      w.Hpp[36 * (size_t)a + 6 * c0 + r0] = v;
    } else {
      w.bp[6 * (size_t)a + k - 21] = v;
    }
  }
  for (int q = tid; q < d.n_opt * 6; q += kMkSolveThreads) {
    const int a = q / 6, k = q % 6;
    w.cvs[q] = ordered_sum(w.cvpart + k, 6, w.kitem_start[a], w.kitem_start[a + 1]);
  }
  for (int q = tid; q < d.n_blk * 36; q += kMkSolveThreads) {
    const int bk = q / 36, k = q % 36;
    w.Sblk[q] = ordered_sum(w.Spart + k, 36, w.bitem_start[bk], w.bitem_start[bk + 1]);
  }
  for (int q = tid; q < n6 * n6; q += kMkSolveThreads) S[q] = 0;
  __syncthreads();
  pt[1] = wall_clock64();
  for (int q = tid; q < d.n_blk * 36; q += kMkSolveThreads) {
    const int bk = q / 36, k = q % 36, r = k / 6, c = k % 6;
    const int a = d.blk_ab[2 * bk], b = d.blk_ab[2 * bk + 1];
    double base = 0;
    if (a == b) base = w.Hpp[36 * (size_t)a + k] + (r == c ? lambda : 0.0);
    // the upper triangle's entry and its mirror in the lower triangle, which the factorisation reads
    if (a < b || r <= c) {
      const double v = base - w.Sblk[36 * (size_t)bk + k];
      const int i = 6 * a + r, j = 6 * b + c;
      S[(size_t)i * n6 + j] = v;
      S[(size_t)j * n6 + i] = v;
    }
  }
  for (int i = tid; i < n6; i += kMkSolveThreads) bs[i] = w.bp[i] - w.cvs[i];
  if (tid == 0) s_ok = 1;
  __syncthreads();
  // Right-looking LDL^T on the lower triangle (row-major), TWO columns per step (n6 is a multiple
  // of 6), one barrier per step.  At the step of the pair (a, a + 1) every thread has D(a), D(a + 1)
  // (Dg) and the columns L(., a), L(., a + 1) (pair slot (a / 2) & 1 of colbuf).  Wave 0 looks one
  // pair ahead: it applies the pair's updates to columns a + 2 and a + 3, takes their pivots,
  // divides them into the other slot (column a + 3 also receiving column a + 2's update first), and
  // carries the forward substitution y(i) -= L(i, c) y(c) for c = a, a + 1; waves 1.. apply the
  // pair's updates to the columns right of a + 3.  Every entry receives the scalar algorithm's
  // operations in the scalar order (the subtraction of (L(i, c) L(j, c)) D(c) for c ascending, then
  // the division by D(j)), as the CPU checker's left-looking loops, and so does y: the factors and
  // y are bit-identical to it.  Values every lane needs (pivots, L(a + 3, a + 2), y(a + 1)) are
  // computed redundantly by every lane from the same operands (no cross-lane traffic).  With no
  // optimised keyframe (n6 = 0, every keyframe fixed) nothing is factored and s_ok stays 1.
  __shared__ double s_col[4 * kLdsRows];
  double* colbuf = n6 <= kLdsRows ? s_col : w.vec + 3 * (size_t)n6;  // [2 slots][2 columns][n6]
  bool ok = true;
  pt[2] = wall_clock64();
  if (wave == 0 && n6 >= 2) {  // the first pair: columns 0 and 1, y = b (n6 = 0: nothing)
    double* l0 = colbuf;
    double* l1 = colbuf + n6;
    const double d0 = S[0];
    const double l10 = S[(size_t)n6] / d0;         // L(1, 0)
    const double d1 = S[(size_t)n6 + 1] - l10 * l10 * d0;  // D(1)
    for (int i = lane; i < n6; i += 64) {
      yv[i] = bs[i];
      if (i > 0) {
        const double l = S[(size_t)i * n6] / d0;
        l0[i] = l;
        S[(size_t)i * n6] = l;
        if (i > 1) {
          const double l_1 = (S[(size_t)i * n6 + 1] - l * l10 * d0) / d1;
          l1[i] = l_1;
          S[(size_t)i * n6 + 1] = l_1;
        }
      }
    }
    if (lane == 0) {
      Dg[0] = d0;
      Dg[1] = d1;
      S[(size_t)n6 + 1] = d1;
      if (d0 == 0 || d1 == 0) s_ok = 0;
    }
  }
  __syncthreads();
  if (s_ok == 0) ok = false;
  for (int a = 0; ok && a + 2 < n6; a += 2) {
    const double da = Dg[a], da1 = Dg[a + 1];
    const double* la = colbuf + (size_t)((a >> 1) & 1) * 2 * n6;  // L(., a)
    const double* la1 = la + n6;                                  // L(., a + 1)
    if (wave == 0) {
      double* lb = colbuf + (size_t)(((a >> 1) + 1) & 1) * 2 * n6;  // L(., a + 2)
      double* lb1 = lb + n6;                                        // L(., a + 3)
      const int b = a + 2, b1 = a + 3;
      // the uniform operands: the pair's entries in rows b, b1 and the two new pivots
      const double lba = la[b], lb1a = la[b1], lba1 = la1[b], lb1a1 = la1[b1];
      const double piv2 = (S[(size_t)b * n6 + b] - lba * lba * da) - lba1 * lba1 * da1;
      const double l32 = ((S[(size_t)b1 * n6 + b] - lb1a * lba * da) - lb1a1 * lba1 * da1) / piv2;
      const double piv3 =
          ((S[(size_t)b1 * n6 + b1] - lb1a * lb1a * da) - lb1a1 * lb1a1 * da1) - l32 * l32 * piv2;
      // forward substitution: y(a + 1) -= L(a + 1, a) y(a); rows > a + 1 take both columns
      const double ya = yv[a];
      const double ya1 = yv[a + 1] - la[a + 1] * ya;
      if (lane == 0) yv[a + 1] = ya1;
      for (int i = b + lane; i < n6; i += 64) {
        const double lia = la[i], lia1 = la1[i];
        yv[i] = (yv[i] - lia * ya) - lia1 * ya1;
        if (i > b) {
          const double l2 = ((S[(size_t)i * n6 + b] - lia * lba * da) - lia1 * lba1 * da1) / piv2;
          lb[i] = l2;
          S[(size_t)i * n6 + b] = l2;
          if (i > b1) {
            const double l3 =
                (((S[(size_t)i * n6 + b1] - lia * lb1a * da) - lia1 * lb1a1 * da1) - l2 * l32 * piv2) /
                piv3;
            lb1[i] = l3;
            S[(size_t)i * n6 + b1] = l3;
          }
        }
      }
      if (lane == 0) {
        S[(size_t)b * n6 + b] = piv2;
        S[(size_t)b1 * n6 + b1] = piv3;
        Dg[b] = piv2;
        Dg[b1] = piv3;
        if (piv2 == 0 || piv3 == 0) s_ok = 0;
      }
    } else {
      // the pair's update of the trailing triangle a + 4 <= j <= i < n6, one entry per thread
      const int m = n6 - a - 4, nq = m * (m + 1) / 2;
      for (int q = tid - 64; q < nq; q += kMkSolveThreads - 64) {
        int ii = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
        while (ii * (ii + 1) / 2 > q) ii--;
        while ((ii + 1) * (ii + 2) / 2 <= q) ii++;
        const int i = a + 4 + ii, j = a + 4 + (q - ii * (ii + 1) / 2);
        double v = S[(size_t)i * n6 + j];
        v -= la[i] * la[j] * da;
        v -= la1[i] * la1[j] * da1;
        S[(size_t)i * n6 + j] = v;
      }
    }
    __syncthreads();
    if (s_ok == 0) ok = false;
  }
  // the last pair's column n6 - 2 still owes y(n6 - 1) its term (the loop's last step carried
  // columns n6 - 4 and n6 - 3; no optimised keyframe: n6 = 0)
  const bool y_last = n6 >= 2;
  pt[3] = wall_clock64();
  if (!ok) {
    if (tid == 0) s_ok = 0;
  } else if (wave == 0) {
    // y / D and the backward substitution, y in registers (lane i: rows i, i + 64), y[r]
    // broadcast by readlane, L(r, i) read at (r, i): coalesced rows
    // (every lane computes the last row's final y, the lane of that row takes it)
    const double ylast = y_last ? yv[n6 - 1] - S[(size_t)(n6 - 1) * n6 + n6 - 2] * yv[n6 - 2] : 0.0;
    auto y_at = [&](int i) { return y_last && i == n6 - 1 ? ylast : yv[i]; };
    double y0 = lane < n6 ? y_at(lane) : 0.0, y1 = lane + 64 < n6 ? y_at(lane + 64) : 0.0;
    if (n6 <= 128) {
      if (lane < n6) y0 /= Dg[lane];
      if (lane + 64 < n6) y1 /= Dg[lane + 64];
      // rows in blocks of kSb: the block's L loads (clamped, unconditional) go out together ahead
      // of its dependent readlane + update steps
      constexpr int kSb = 4;  // 8 measured no faster
      const int c0 = min(lane, n6 - 1), c1 = min(lane + 64, n6 - 1);
      for (int r = n6 - 1; r > 0; r -= kSb) {
        double l0[kSb], l1[kSb];
#pragma unroll
        for (int k = 0; k < kSb; k++) {
          const int rr = max(r - k, 0);
          l0[k] = S[(size_t)rr * n6 + c0];
          l1[k] = S[(size_t)rr * n6 + c1];
        }
#pragma unroll
        for (int k = 0; k < kSb; k++) {
          const int rr = r - k;
          if (rr > 0) {
            const double yr = rr < 64 ? lane_value(y0, rr) : lane_value(y1, rr - 64);
            if (lane < rr) y0 -= l0[k] * yr;
            if (lane + 64 < rr) y1 -= l1[k] * yr;
          }
        }
      }
      if (lane < n6) w.x[lane] = y0;
      if (lane + 64 < n6) w.x[lane + 64] = y1;
    } else {
      for (int i = lane; i < n6; i += 64) yv[i] = y_at(i) / Dg[i];
      wave_sync_lds();
      for (int r = n6 - 1; r > 0; r--) {
        const double yr = yv[r];
        for (int i = lane; i < r; i += 64) yv[i] -= S[(size_t)r * n6 + i] * yr;
        wave_sync_lds();
      }
      for (int i = lane; i < n6; i += 64) w.x[i] = yv[i];
    }
  }
  __syncthreads();
  pt[4] = wall_clock64();
  const bool ok2 = s_ok != 0;
  // the trial poses: exp(x_p) * pose for the round's optimised keyframes, the others unchanged
  const DSE3* cur = w.pose + (size_t)cb * d.n_kf;
  DSE3* tri = w.pose + (size_t)(1 - cb) * d.n_kf;
  // (waves 1..: the exponentials run beside wave 0's sums below)
  for (int k = tid - 64; tid >= 64 && k < d.n_kf; k += kMkSolveThreads - 64) {
    const int a = d.opt_of[k];
    if (a >= 0 && w.kf_act[k]) {
      double u[6];
#pragma unroll
      for (int r = 0; r < 6; r++) u[r] = w.x[6 * a + r];
      tri[k] = dse3_mul(dse3_exp(u), cur[k]);
    } else {
      tri[k] = cur[k];
    }
  }
  // the poses' share of the scale term and the iteration's chi2, by wave 0 (fixed order)
  if (wave == 0) {
    double sp = 0, c = 0;
    for (int i = lane; i < n6; i += 64)
      if (w.kf_act[d.opt_kf[i / 6]]) {
        const double xv = w.x[i];
        sp += xv * (lambda * xv + w.bp[i]);
      }
    if (lin_ran)
      for (int g = lane; g < w.gP; g += 64) c += w.linpart[2 * g];
    sp = wave_sum_dpp(sp);
    c = wave_sum_dpp(c);
    if (lane == 0) {
      s_vec2[0] = sp;
      s_vec2[1] = c;
    }
  }
  __syncthreads();
  if (tid == 0) {
    const double sp = s_vec2[0];
    BAState& s = *stp;
    if (lin_ran) s.currentChi = s_vec2[1];
    if (need_lin) s.iniChi = s.currentChi;  // the iteration's start (after an accepted trial: its chi2)
    if (lam_init) {
      s.lam_init = 0;
      s.ni = 2;
      s.nBad = 0;
    }
    s.lambda = lambda;
    pt[5] = wall_clock64();
    for (int q = 0; q < 5; q++) s.prof[q] += pt[q + 1] - pt[q];
    s.ok2 = ok2 ? 1 : 0;
    s.scale_p = sp;
  }
}

// trial step 5, one workgroup: OptimizationAlgorithmLevenberg::solve's decision for the trial,
// the end of the iteration (SparseOptimizer::optimize's stops), the switch to the second round
// (the inlier check of Optimizer.cc:3559-3590 on the last computed errors) and the end of the solve
// (every thread of one workgroup of NT threads; k_ba2_p4's last workgroup runs it)
template <int NT>
__device__ void ba2_decide(const BADesc& d, const BAWork2& w) {
  __shared__ int s_round_end;
  __shared__ double s_part[NT / 64];
  __shared__ double s_sum[2];
  BAState* stp = w.st;
  const int tid = threadIdx.x;
  if (tid < 64) {  // the trial's chi2 and scale over the point workgroups (wave 0, fixed order)
    double a = 0, b = 0;
    for (int g = tid; g < w.gP; g += 64) {
      a += w.p4part[2 * g];
      b += w.p4part[2 * g + 1];
    }
    a = wave_sum_dpp(a);
    b = wave_sum_dpp(b);
    if (tid == 0) {
      s_sum[0] = a;
      s_sum[1] = b;
    }
  }
  __syncthreads();
  if (tid == 0) {
    BAState& s = *stp;
    const double tc = s_sum[0], sc = s_sum[1];
    double tempChi = tc;
    const double lastTrialChi = tempChi;
    if (!s.ok2) tempChi = DBL_MAX;
    double scale = s.scale_p + sc;
    double rho = s.currentChi - tempChi;
    scale += 1e-3;
    rho /= scale;
    if (rho > 0 && isfinite(tempChi)) {
      double alpha = 1. - pow((2 * rho - 1), 3);
      alpha = fmin(alpha, 2. / 3.);
      s.lambda *= fmax(1. / 3., alpha);
      s.ni = 2;
      s.currentChi = tempChi;
      s.cb = 1 - s.cb;  // the trial (and its linearisation, with SPEC) becomes the current estimate
      s.spec_ok = w.spec;
    } else {
      s.lambda *= s.ni;
      s.ni *= 2;
      s.spec_ok = 0;
    }
    s.qmax++;
    s.trials[s.round]++;
    int round_end = 0;
    if (rho < 0 && s.qmax < 10) {
      s.need_lin = 0;  // another trial of this iteration
    } else {
      bool ok = true;
      if (s.qmax == 10 || rho == 0) ok = false;
      if (ok) {
        if ((s.iniChi - s.currentChi) * 1e3 < s.iniChi)
          s.nBad++;
        else
          s.nBad = 0;
        if (s.nBad >= 3) ok = false;
      }
      if (s.chk < lastTrialChi && s.iter > 0) ok = false;
      s.chk = lastTrialChi;
      s.it_done[s.round] = s.iter + 1;
      s.iter++;
      s.qmax = 0;
      s.need_lin = 1;
      if (!ok || s.iter == (s.round == 0 ? 5 : 10)) round_end = 1;
    }
    if (round_end && s.round == 1) {
      s.done = 1;
      round_end = 0;
    }
    s_round_end = round_end;
  }
  __syncthreads();
  if (!s_round_end) return;
  // ---- round 2: the observations that fail the inlier test on the last computed errors (or sit
  // behind the camera) set aside (level 1), every kernel dropped, the solver's x reset
  const int cb = stp->cb;
  const Cam cam = ba_cam(d);
  (void)cam;
  const DSE3* pose = w.pose + (size_t)cb * d.n_kf;
  const double* Xc = w.X + (size_t)cb * 3 * d.n_pt;
  for (int e = tid; e < d.n_edge; e += NT) {
    const bool stereo = !(d.e_obs[3 * (size_t)e + 2] < 0);
    const double chi = edge_chi2(&w.err[3 * (size_t)e], (double)d.e_s[e], stereo);
    double pc[3];
    se3_map(pose[d.e_kf[e]], &Xc[3 * (size_t)d.e_pt[e]], pc);
    if (chi > (stereo ? 7.815 : 5.991) || !(pc[2] > 0.0)) w.level[e] = 1;
  }
  for (int k = tid; k < d.n_kf; k += NT) w.kf_act[k] = 0;
  const size_t n6 = 6 * (size_t)d.n_opt;
  for (size_t q = tid; q < n6 + 3 * (size_t)d.n_pt; q += NT) w.x[q] = 0;
  __syncthreads();
  int nact = 0;
  for (int j = tid; j < d.n_pt; j += NT) {
    uint8_t a = 0;
    for (int e = d.pt_start[j]; e < d.pt_start[j + 1]; e++)
      if (w.level[e] == 0) {
        a = 1;
        if (d.opt_of[d.e_kf[e]] >= 0) w.kf_act[d.e_kf[e]] = 1;  // every writer stores 1
      }
    w.pt_act[j] = a;
    nact += a;
  }
  double na = wave_sum_dpp((double)nact);
  if ((tid & 63) == 0) s_part[tid >> 6] = na;
  __syncthreads();
  if (tid == 0) {
    double t = 0;
    for (int q = 0; q < NT / 64; q++) t += s_part[q];
    BAState& s = *stp;
    s.round = 1;
    s.spec_ok = 0;
    s.iter = 0;
    s.qmax = 0;
    s.need_lin = 1;
    s.lam_init = 1;
    s.lambda = 0;
    s.ni = 2;
    s.chk = 0;
    s.nBad = 0;
    s.nact = (int)t;
    if (t == 0) s.done = 1;
  }
}

// trial step 4, one thread per point (a wave per heavy point): x_l = D^-1 (b_l - H_pl^T x_p) (stale
// on a failed solve), the trial point, the errors of its active edges at the trial state, chi2 and
// the scale term.  (Linearising at the trial state here as well, so that an accepted trial needs no
// k_ba2_lin, measured slower in round 5: its registers slowed every trial more than the launch it
// saved.)
// point j's trial: x_l, the trial point (stored to Xt), its active edges' trial errors (stored),
// chi2 and the scale term.  WAVE: the heavy point's wave (every lane returns the same values;
// edges 64 at a time, the chi2 added in edge order from the staging row sh)
template <bool WAVE>
__device__ __forceinline__ void ba2_trial_point(const BADesc& d, const BAWork2& w, int j,
                                                double* sh, double* chi_out, double* sc_out) {
  const BAState* st = w.st;
  const int cb = st->cb, nb = 1 - cb;
  const bool ok2 = st->ok2 != 0, robust = st->round == 0;
  const double lambda = st->lambda;
  const size_t n6 = 6 * (size_t)d.n_opt;
  const DSE3* tri = w.pose + (size_t)nb * d.n_kf;
  const double* Xc = w.X + (size_t)cb * 3 * d.n_pt;
  double* Xt = w.X + (size_t)nb * 3 * d.n_pt;
  const double* bl_c = w.bl + (size_t)cb * 3 * d.n_pt;
  const double* Hpl_c = w.Hpl + (size_t)cb * 18 * d.n_edge;
  const int lane = threadIdx.x & 63;
  double chi = 0, sc = 0;
  double X[3] = {Xc[3 * (size_t)j], Xc[3 * (size_t)j + 1], Xc[3 * (size_t)j + 2]};
  if (w.pt_act[j]) {
    double* xl = &w.x[n6 + 3 * (size_t)j];
    const double bl3[3] = {bl_c[3 * (size_t)j], bl_c[3 * (size_t)j + 1], bl_c[3 * (size_t)j + 2]};
    double xv3[3];  // the increment, kept in registers (no read-back of the store)
    if (ok2) {
      // the loads that depend on j alone first (D^-1); an edge's H_pl block only for the edges
      // of the level to an optimised keyframe (ba2_lin_point writes no block for the others)
      double Di[9];
#pragma unroll
      for (int q = 0; q < 9; q++) Di[q] = w.Dinv[9 * (size_t)j + q];
      double cl[3] = {bl3[0], bl3[1], bl3[2]};
      auto add_edge = [&](int e, int a) {
        double B[18];
#pragma unroll
        for (int q = 0; q < 18; q++) B[q] = Hpl_c[18 * (size_t)e + q];
#pragma unroll
        for (int c = 0; c < 3; c++)
#pragma unroll
          for (int r = 0; r < 6; r++) cl[c] += B[3 * r + c] * (-w.x[6 * a + r]);
      };
      if (!WAVE) {
        for (int e = d.pt_start[j]; e < d.pt_start[j + 1]; e++) {
          const int a = w.eopt[e];
          if (w.level[e] || a < 0) continue;
          add_edge(e, a);
        }
      } else {  // the active edges to optimised keyframes found 64 at a time, taken in edge order
        const int e1 = d.pt_start[j + 1];
        for (int e0 = d.pt_start[j]; e0 < e1; e0 += 64) {
          const int e = e0 + lane;
          const bool take = e < e1 && !w.level[e] && w.eopt[e] >= 0;
          unsigned long long m = __ballot(take);
          while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            add_edge(e0 + k, w.eopt[e0 + k]);
          }
        }
      }
#pragma unroll
      for (int a = 0; a < 3; a++)
        xv3[a] = Di[3 * a] * cl[0] + Di[3 * a + 1] * cl[1] + Di[3 * a + 2] * cl[2];
      if (!WAVE || lane == 0) {
#pragma unroll
        for (int a = 0; a < 3; a++) xl[a] = xv3[a];
      }
    } else {
#pragma unroll
      for (int a = 0; a < 3; a++) xv3[a] = xl[a];  // stale (g2o re-applies its _x)
    }
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const double xv = xv3[r];
      sc += xv * (lambda * xv + bl3[r]);
      X[r] += xv;
    }
    if (!WAVE) {  // the trial's errors and chi2
      for (int e = d.pt_start[j]; e < d.pt_start[j + 1]; e++)
        if (!w.level[e]) chi += ba2_trial_edge(d, w, e, tri, X, robust);
    } else {
      double sum[1] = {0};
      const int e1 = d.pt_start[j + 1];
      for (int e0 = d.pt_start[j]; e0 < e1; e0 += 64) {
        const int e = e0 + lane;
        const bool valid = e < e1 && !w.level[e];
        double v[1] = {0};
        if (valid) v[0] = ba2_trial_edge(d, w, e, tri, X, robust);
        ba2_wave_ordered_add<1>(sh, lane, min(64, e1 - e0), valid, v, sum);
      }
      chi = sum[0];
    }
  }
  if (!WAVE || lane == 0) {
#pragma unroll
    for (int r = 0; r < 3; r++) Xt[3 * (size_t)j + r] = X[r];
  }
  *chi_out = chi;
  *sc_out = sc;
}

// the heavy points' trials, a wave each, before k_ba2_p4 (which adds their chi2 and scale terms
// from hres at the point's own place)
__global__ __launch_bounds__(kMkThreads) void k_ba2_p4_heavy(BADesc d, BAWork2 w) {
  __shared__ double s_stage[kMkWaves][64];
  if (w.st->done) return;
  const int wave = threadIdx.x >> 6;
  const int hi = (int)blockIdx.x * kMkWaves + wave;
  if (hi >= w.n_heavy) return;
  const int j = w.heavy[hi];
  double chi, sc;
  ba2_trial_point<true>(d, w, j, s_stage[wave], &chi, &sc);
  if ((threadIdx.x & 63) == 0) {
    w.hres[2 * (size_t)j] = chi;
    w.hres[2 * (size_t)j + 1] = sc;
  }
}

__global__ __launch_bounds__(kMkThreads) void k_ba2_p4(BADesc d, BAWork2 w) {
  __shared__ double s_part[2 * kMkWaves];
  __shared__ int s_last;
  const BAState* st = w.st;
  if (st->done) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * kMkThreads + threadIdx.x;
  double chi = 0, sc = 0;
  if (j < d.n_pt) {
    if (ba2_heavy(d, j)) {  // tried by its wave in k_ba2_p4_heavy
      chi = w.hres[2 * (size_t)j];
      sc = w.hres[2 * (size_t)j + 1];
    } else {
      ba2_trial_point<false>(d, w, j, nullptr, &chi, &sc);
    }
  }
  const double a = wave_sum_dpp(chi), b = wave_sum_dpp(sc);
  if (lane == 0) {
    s_part[2 * wave] = a;
    s_part[2 * wave + 1] = b;
  }
  __threadfence();  // release this thread's err / Xt stores to the deciding workgroup
  __syncthreads();
  if (threadIdx.x == 0) {
    double t0 = 0, t1 = 0;
#pragma unroll
    for (int q = 0; q < kMkWaves; q++) {
      t0 += s_part[2 * q];
      t1 += s_part[2 * q + 1];
    }
    w.p4part[2 * blockIdx.x] = t0;
    w.p4part[2 * blockIdx.x + 1] = t1;
    // the last workgroup to finish takes the trial's decision (k_ba2_p5's work, one launch fewer
    // per trial): its partials published by an agent-scope release (every thread's err / Xt
    // stores were released by their own fence before the barrier above), the count, and the
    // last one's acquire before it reads every partial
    __threadfence();
    const unsigned done = atomicAdd(w.p4cnt, 1u);
    s_last = done == (unsigned)gridDim.x - 1;
    if (s_last) __threadfence();
  }
  __syncthreads();
  if (!s_last) return;
  ba2_decide<kMkThreads>(d, w);
  if (threadIdx.x == 0) *w.p4cnt = 0;
}

// the erase test (Optimizer.cc:3603-3631) and the recovered estimates
__global__ __launch_bounds__(kMkDecideThreads) void k_ba2_finish(BADesc d, BAWork2 w) {
  __shared__ double s_part[kMkDecideThreads / 64];
  const int tid = threadIdx.x;
  const int cb = w.st->cb;
  const DSE3* pose = w.pose + (size_t)cb * d.n_kf;
  const double* Xc = w.X + (size_t)cb * 3 * d.n_pt;
  int nerase = 0;
  for (int e = tid; e < d.n_edge; e += kMkDecideThreads) {
    const bool stereo = !(d.e_obs[3 * (size_t)e + 2] < 0);
    const double chi = edge_chi2(&w.err[3 * (size_t)e], (double)d.e_s[e], stereo);
    double pc[3];
    se3_map(pose[d.e_kf[e]], &Xc[3 * (size_t)d.e_pt[e]], pc);
    const bool er = chi > (stereo ? 7.815 : 5.991) || !(pc[2] > 0.0);
    d.erase[e] = er ? 1 : 0;
    nerase += er;
  }
  for (int k = tid; k < d.n_kf; k += kMkDecideThreads) dse3_to_float(pose[k], d.T_out + 16 * (size_t)k);
  for (int q = tid; q < 3 * d.n_pt; q += kMkDecideThreads) d.X_out[q] = (float)Xc[q];
  const double na = wave_sum_dpp((double)nerase);
  if ((tid & 63) == 0) s_part[tid >> 6] = na;
  __syncthreads();
  if (tid == 0) {
    double t = 0;
    for (int q = 0; q < kMkDecideThreads / 64; q++) t += s_part[q];
    const BAState& s = *w.st;
    d.stats[0] = s.it_done[0];
    d.stats[1] = s.it_done[1];
    d.stats[2] = s.trials[0];
    d.stats[3] = s.trials[1];
    d.stats[4] = (int)t;
  }
}

}  // namespace

size_t ba_workspace_bytes(int n_kf, int n_pt, int n_edge, int n_opt) {
  const size_t n6 = 6 * (size_t)n_opt;
  const size_t nd = 14 * (size_t)n_kf + (3 + 3 + 9 + 3 + 9) * (size_t)n_pt +
                    (3 + 18 + 18 + 6) * (size_t)n_edge + 42 * (size_t)n_opt + n6 + 3 * (size_t)n_pt +
                    n6 * n6 + 3 * n6;
  return 8 * nd + (size_t)n_edge + n_kf + n_pt + 64;
}

size_t ba2_workspace_bytes(int n_kf, int n_pt, int n_edge, int n_opt, int n_blk, int gP) {
  auto a = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t n6 = 6 * (size_t)n_opt;
  return a(sizeof(BAState)) + a(sizeof(DSE3) * 2 * (size_t)n_kf) + a(8 * 6 * (size_t)n_pt) +
         a(8 * 18 * (size_t)n_pt) + a(8 * 6 * (size_t)n_pt) + a(8 * 9 * (size_t)n_pt) +
         a(8 * 3 * (size_t)n_edge) + a(8 * 36 * (size_t)n_edge) + a(8 * 54 * (size_t)n_edge) +
         a(8 * 18 * (size_t)n_edge) + a(8 * 6 * (size_t)n_edge) + a(8 * 36 * (size_t)n_opt) +
         a(8 * 6 * (size_t)n_opt) + a(8 * 6 * (size_t)n_opt) + a(8 * 36 * (size_t)n_blk) +
         a(8 * (n6 + 3 * (size_t)n_pt)) + a(8 * n6 * n6) + a(8 * 7 * n6) + 2 * a(8 * 2 * (size_t)gP) +
         a((size_t)n_edge) + a(4 * (size_t)n_edge) + a((size_t)n_kf) + a((size_t)n_pt) + a(16) + 64;
}


// ------------------------------------------------------------------ host side
static size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

BARunner::~BARunner() {
  if (d_ws2_) (void)hipFree(d_ws2_);
  if (h_flag_) (void)hipHostFree(h_flag_);
  if (d_up_) (void)hipFree(d_up_);
  if (d_dn_) (void)hipFree(d_dn_);
  if (d_ws_) (void)hipFree(d_ws_);
  if (h_up_) (void)hipHostFree(h_up_);
  if (h_dn_) (void)hipHostFree(h_dn_);
}

void BARunner::grow(uint8_t*& d, uint8_t*& h, size_t& cap, size_t need, hipStream_t st) {
  if (need <= cap && d) return;
  MMT_HIP(hipStreamSynchronize(st));
  if (d) (void)hipFree(d);
  if (h) (void)hipHostFree(h);
  cap = std::max(need + (need >> 1), (size_t)1 << 16);
  MMT_HIP(hipMalloc((void**)&d, cap));
  MMT_HIP(hipHostMalloc((void**)&h, cap, hipHostMallocDefault));
}

namespace {
double ba_now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
// MMT_BA_PROFILE=1: host wall time of BARunner::run's phases, printed every 32 solves
struct BAHostProf {
  bool on = getenv("MMT_BA_PROFILE") != nullptr;
  double t[5] = {0, 0, 0, 0, 0};  // layout, launches, waits, finish, total
  long long p3[5] = {0, 0, 0, 0, 0};  // k_ba2_p3 phases (ticks of 10 ns)
  long n = 0, slots = 0;
};
BAHostProf g_ba_prof;
}  // namespace

void BARunner::run(const BAHostProblem& P, hipStream_t st, float* T_out, float* X_out,
                   uint8_t* erase, int* stats) {
  BAHostProf& hp = g_ba_prof;
  const double tp0 = hp.on ? ba_now_us() : 0;
  const int nK = P.n_kf, nP = P.n_pt, nE = P.n_edge;
  for (int i = 0; i < nE; i++)
    if (P.e_pt[i] < 0 || P.e_pt[i] >= nP || P.e_kf[i] < 0 || P.e_kf[i] >= nK ||
        (i > 0 && P.e_pt[i] < P.e_pt[i - 1]))
      throw ArgError("local BA: edges must be listed point by point with valid vertices");
  std::vector<int> opt_of(nK, -1), opt_kf;
  for (int v = 0; v < nK; v++)
    if (!P.fixed[v]) {
      opt_of[v] = (int)opt_kf.size();
      opt_kf.push_back(v);
    }
  const int nO = (int)opt_kf.size();
  std::vector<int> pt_start(nP + 1, 0), kf_start(nO + 1, 0), kf_edges;
  // the Schur triples grouped by keyframe-pair block (a <= b, blocks in (a, b) order, triples in
  // point order): counted, then placed; every diagonal block exists (it carries H_pp + lambda I)
  std::vector<int> bcnt((size_t)nO * nO, 0), kcnt(nO, 0);
  std::vector<std::pair<int, int>> col;
  auto point_col = [&](int& e, int j) {  // point j's edges to optimised keyframes, pose order
    col.clear();
    for (; e < nE && P.e_pt[e] == j; e++) {
      const int a = opt_of[P.e_kf[e]];
      if (a >= 0) col.push_back({a, e});
    }
    std::sort(col.begin(), col.end());  // pose-index order, as g2o's H_pl column
  };
  for (int j = 0, e = 0; j < nP; j++) {
    point_col(e, j);
    pt_start[j + 1] = e;
    for (size_t p1 = 0; p1 < col.size(); p1++) {
      kcnt[col[p1].first]++;
      for (size_t p2 = p1; p2 < col.size(); p2++) bcnt[(size_t)col[p1].first * nO + col[p2].first]++;
    }
  }
  std::vector<int> bid((size_t)nO * nO, -1), blk_ab, blk_start{0};
  for (int a = 0; a < nO; a++)
    for (int b = a; b < nO; b++)
      if (a == b || bcnt[(size_t)a * nO + b] > 0) {
        bid[(size_t)a * nO + b] = (int)blk_ab.size() / 2;
        blk_ab.push_back(a);
        blk_ab.push_back(b);
        blk_start.push_back(blk_start.back() + bcnt[(size_t)a * nO + b]);
      }
  const int nblocks = (int)blk_ab.size() / 2;
  for (int a = 0; a < nO; a++) kf_start[a + 1] = kf_start[a] + kcnt[a];
  std::vector<int2> trip(blk_start.back());
  kf_edges.resize(kf_start[nO]);
  std::vector<int> bfill(blk_start.begin(), blk_start.end() - 1), kfill(kf_start.begin(), kf_start.end() - 1);
  for (int j = 0, e = 0; j < nP; j++) {
    point_col(e, j);
    for (size_t p1 = 0; p1 < col.size(); p1++) {
      kf_edges[kfill[col[p1].first]++] = col[p1].second;
      for (size_t p2 = p1; p2 < col.size(); p2++)
        trip[bfill[bid[(size_t)col[p1].first * nO + col[p2].first]]++] =
            make_int2(col[p1].second, col[p2].second);
    }
  }
  // work items of the multi-kernel solve: <= 256 edges of one keyframe, <= 256 triples of one block
  std::vector<int4> kitem, bitem;
  std::vector<int> kitem_start{0}, bitem_start{0};
  for (int a = 0; a < nO; a++) {
    for (int t = kf_start[a]; t < kf_start[a + 1]; t += 256)
      kitem.push_back(make_int4(a, t, std::min(t + 256, kf_start[a + 1]), 0));
    kitem_start.push_back((int)kitem.size());
  }
  for (size_t bk = 0; bk + 1 < blk_start.size(); bk++) {
    for (int t = blk_start[bk]; t < blk_start[bk + 1]; t += 256)
      bitem.push_back(make_int4((int)bk, t, std::min(t + 256, blk_start[bk + 1]), 0));
    bitem_start.push_back((int)bitem.size());
  }
  // the heavy points (more than kBaHeavy edges): a wave each, in the point kernels' workgroups
  // after the thread-per-point ones
  std::vector<int> heavy;
  for (int j = 0; j < nP; j++)
    if (pt_start[j + 1] - pt_start[j] > kBaHeavy) heavy.push_back(j);
  struct Seg {
    size_t bytes;
    const void* src;
  };
  const Seg segs[] = {{64 * (size_t)nK, P.Tcw},           {4 * opt_of.size(), opt_of.data()},
                      {4 * opt_kf.size(), opt_kf.data()}, {12 * (size_t)nP, P.Xw},
                      {4 * pt_start.size(), pt_start.data()}, {4 * (size_t)nE, P.e_pt},
                      {4 * (size_t)nE, P.e_kf},           {12 * (size_t)nE, P.e_obs},
                      {4 * (size_t)nE, P.e_s},            {4 * kf_start.size(), kf_start.data()},
                      {4 * kf_edges.size(), kf_edges.data()}, {4 * blk_ab.size(), blk_ab.data()},
                      {4 * blk_start.size(), blk_start.data()}, {8 * trip.size(), trip.data()},
                      {16 * kitem.size(), kitem.data()}, {4 * kitem_start.size(), kitem_start.data()},
                      {16 * bitem.size(), bitem.data()}, {4 * bitem_start.size(), bitem_start.data()},
                      {4 * heavy.size(), heavy.data()}};
  constexpr int nseg = sizeof(segs) / sizeof(segs[0]);
  size_t off[nseg], tot = 0;
  for (int i = 0; i < nseg; i++) {
    off[i] = tot;
    tot += al16(segs[i].bytes);
  }
  grow(d_up_, h_up_, up_cap_, tot, st);
  for (int i = 0; i < nseg; i++)
    if (segs[i].bytes) memcpy(h_up_ + off[i], segs[i].src, segs[i].bytes);
  const size_t o_X = al16(64 * (size_t)nK), o_er = o_X + al16(12 * (size_t)nP),
               o_st = o_er + al16((size_t)nE), dn = o_st + 64;
  grow(d_dn_, h_dn_, dn_cap_, dn, st);
  const size_t wsb = ba_workspace_bytes(nK, nP, nE, nO);
  if (wsb > ws_cap_ || !d_ws_) {
    MMT_HIP(hipStreamSynchronize(st));
    if (d_ws_) (void)hipFree(d_ws_);
    ws_cap_ = wsb + (wsb >> 1);
    MMT_HIP(hipMalloc((void**)&d_ws_, ws_cap_));
  }
  MMT_HIP(hipMemcpyAsync(d_up_, h_up_, tot, hipMemcpyHostToDevice, st));
  BADesc d;
  memset(&d, 0, sizeof(d));
  d.n_kf = nK;
  d.n_pt = nP;
  d.n_edge = nE;
  d.n_opt = nO;
  d.n_blk = nblocks;
  const uint8_t* u = d_up_;
  d.Tcw = (const float*)(u + off[0]);
  d.opt_of = (const int*)(u + off[1]);
  d.opt_kf = (const int*)(u + off[2]);
  d.Xw = (const float*)(u + off[3]);
  d.pt_start = (const int*)(u + off[4]);
  d.e_pt = (const int*)(u + off[5]);
  d.e_kf = (const int*)(u + off[6]);
  d.e_obs = (const float*)(u + off[7]);
  d.e_s = (const float*)(u + off[8]);
  d.kf_start = (const int*)(u + off[9]);
  d.kf_edges = (const int*)(u + off[10]);
  d.blk_ab = (const int*)(u + off[11]);
  d.blk_start = (const int*)(u + off[12]);
  d.trip = (const int2*)(u + off[13]);
  d.fx = P.fx; d.fy = P.fy; d.cx = P.cx; d.cy = P.cy; d.bf = P.bf;
  d.ws = d_ws_;
  d.T_out = (float*)d_dn_;
  d.X_out = (float*)(d_dn_ + o_X);
  d.erase = d_dn_ + o_er;
  d.stats = (int*)(d_dn_ + o_st);
  {
    const int gPp = std::max(1, (nP + kMkThreads - 1) / kMkThreads);
    const int gH = ((int)heavy.size() + kMkWaves - 1) / kMkWaves;
    const int gP = gPp;  // the partial sums: one per point workgroup
    const int n6 = 6 * nO, nblk = nblocks;
    const size_t wsb2 = ba2_workspace_bytes(nK, nP, nE, nO, nblk, gP) +
                        8 * (27 + 6) * kitem.size() + 8 * 36 * bitem.size() + 16 * (size_t)nP +
                        64 * 4;
    if (wsb2 > ws2_cap_ || !d_ws2_) {
      MMT_HIP(hipStreamSynchronize(st));
      if (d_ws2_) (void)hipFree(d_ws2_);
      ws2_cap_ = wsb2 + (wsb2 >> 1);
      MMT_HIP(hipMalloc((void**)&d_ws2_, ws2_cap_));
    }
    if (!h_flag_) MMT_HIP(hipHostMalloc((void**)&h_flag_, 64, hipHostMallocDefault));
    BAWork2 w;
    uint8_t* p = d_ws2_;
    auto take = [&](size_t bytes) {
      uint8_t* r = p;
      p += al16(bytes);
      return r;
    };
    w.st = (BAState*)take(sizeof(BAState));
    w.pose = (DSE3*)take(sizeof(DSE3) * 2 * (size_t)nK);
    w.X = (double*)take(8 * 6 * (size_t)nP);
    w.Hll = (double*)take(8 * 2 * 9 * (size_t)nP);
    w.bl = (double*)take(8 * 2 * 3 * (size_t)nP);
    w.Dinv = (double*)take(8 * 9 * (size_t)nP);
    w.err = (double*)take(8 * 3 * (size_t)nE);
    w.Hpl = (double*)take(8 * 2 * 18 * (size_t)nE);
    w.Hpe = (double*)take(8 * 2 * 27 * (size_t)nE);
    w.Y = (double*)take(8 * 18 * (size_t)nE);
    w.cv = (double*)take(8 * 6 * (size_t)nE);
    w.Hpp = (double*)take(8 * 36 * (size_t)nO);
    w.bp = (double*)take(8 * 6 * (size_t)nO);
    w.cvs = (double*)take(8 * 6 * (size_t)nO);
    w.Sblk = (double*)take(8 * 36 * (size_t)nblk);
    w.kitem = (const int4*)(u + off[14]);
    w.kitem_start = (const int*)(u + off[15]);
    w.bitem = (const int4*)(u + off[16]);
    w.bitem_start = (const int*)(u + off[17]);
    w.n_kitem = (int)kitem.size();
    w.n_bitem = (int)bitem.size();
    w.Hpart = (double*)take(8 * 27 * kitem.size());
    w.Spart = (double*)take(8 * 36 * bitem.size());
    w.cvpart = (double*)take(8 * 6 * kitem.size());
    w.x = (double*)take(8 * ((size_t)n6 + 3 * (size_t)nP));
    w.S = (double*)take(8 * (size_t)n6 * n6);
    w.vec = (double*)take(8 * 7 * (size_t)n6);  // b, D, y, four L columns (p3)
    w.linpart = (double*)take(8 * 2 * (size_t)gP);
    w.p4part = (double*)take(8 * 2 * (size_t)gP);
    w.p4cnt = (unsigned*)take(16);
    w.level = take((size_t)nE);
    w.eopt = (int*)take(4 * (size_t)nE);
    w.kf_act = take((size_t)nK);
    w.pt_act = take((size_t)nP);
    w.gP = gP;
    w.gPp = gPp;
    w.heavy = (const int*)(u + off[18]);
    w.n_heavy = (int)heavy.size();
    w.hres = (double*)take(16 * (size_t)nP);
    w.spec = 0;  // k_ba2_lin linearises every trial (the trial kernel's own linearisation,
                 // k_ba2_p4<true>, measured 1,509 against 1,549 us per BA but spills)
    const double tp1 = hp.on ? ba_now_us() : 0;
    double t_launch = 0, t_wait = 0;
    hipLaunchKernelGGL(k_ba2_init, dim3(gPp), dim3(kMkThreads), 0, st, d, w);
    MMT_HIP(hipGetLastError());
    // A trial is at most 6 launches; a solve at most 5 x 10 + 10 x 10 trials.  The first batch
    // covers a typical solve (about 15 trials on the C3 sequence), later ones are short.
    int slots = 0;
    for (bool done = nE == 0; !done;) {
      // g2o runs 5 + 10 iterations; on the tracker's graphs every trial is accepted, so 15 slots
      // usually finish the solve (a slot left over costs its six launches, about 30 us)
      const int batch = slots == 0 ? 15 : 4;
      const double tl = hp.on ? ba_now_us() : 0;
      for (int b = 0; b < batch; b++) {
        if (gH > 0) hipLaunchKernelGGL(k_ba2_lin_heavy, dim3(gH), dim3(kMkThreads), 0, st, d, w);
        hipLaunchKernelGGL(k_ba2_lin, dim3(gPp), dim3(kMkThreads), 0, st, d, w);
        if (w.n_kitem > 0)
          hipLaunchKernelGGL(k_ba2_kfsum, dim3(w.n_kitem), dim3(kMkThreads), 0, st, d, w);
        hipLaunchKernelGGL(k_ba2_p1, dim3(gPp + gH), dim3(kMkThreads), 0, st, d, w);
        if (w.n_bitem + w.n_kitem > 0)
          hipLaunchKernelGGL(k_ba2_p2, dim3(w.n_bitem + w.n_kitem), dim3(kMkThreads), 0, st, d, w);
        hipLaunchKernelGGL(k_ba2_p3, dim3(1), dim3(kMkSolveThreads), 0, st, d, w);
        if (gH > 0) hipLaunchKernelGGL(k_ba2_p4_heavy, dim3(gH), dim3(kMkThreads), 0, st, d, w);
        hipLaunchKernelGGL(k_ba2_p4, dim3(gPp), dim3(kMkThreads), 0, st, d, w);
      }
      MMT_HIP(hipGetLastError());
      slots += batch;
      MMT_HIP(hipMemcpyAsync(h_flag_, &w.st->done, sizeof(int), hipMemcpyDeviceToHost, st));
      const double tw = hp.on ? ba_now_us() : 0;
      MMT_HIP(hipStreamSynchronize(st));
      if (hp.on) {
        t_launch += tw - tl;
        t_wait += ba_now_us() - tw;
      }
      done = *h_flag_ != 0;
      if (!done && slots >= 160) throw DeviceError("local BA: the LM did not finish in 150 trials");
    }
    hipLaunchKernelGGL(k_ba2_finish, dim3(1), dim3(kMkDecideThreads), 0, st, d, w);
    MMT_HIP(hipGetLastError());
    if (hp.on) {
      hp.t[0] += tp1 - tp0;
      hp.t[1] += t_launch;
      hp.t[2] += t_wait;
      hp.slots += slots;
      BAState hs;
      MMT_HIP(hipMemcpy(&hs, w.st, sizeof(hs), hipMemcpyDeviceToHost));
      for (int q = 0; q < 5; q++) hp.p3[q] += hs.prof[q];
    }
  }
  MMT_HIP(hipMemcpyAsync(h_dn_, d_dn_, dn, hipMemcpyDeviceToHost, st));
  MMT_HIP(hipStreamSynchronize(st));
  memcpy(T_out, h_dn_, 64 * (size_t)nK);
  memcpy(X_out, h_dn_ + o_X, 12 * (size_t)nP);
  memcpy(erase, h_dn_ + o_er, (size_t)nE);
  memcpy(stats, h_dn_ + o_st, 5 * sizeof(int));
  if (hp.on) {
    hp.t[4] += ba_now_us() - tp0;
    if (++hp.n % 32 == 0)
      fprintf(stderr, "[mmt ba profile] %ld solves, host us per solve: layout + upload %.1f, "
              "launches %.1f, waits %.1f, total %.1f; %.1f trial slots per solve\n", hp.n,
              hp.t[0] / hp.n, hp.t[1] / hp.n, hp.t[2] / hp.n, hp.t[4] / hp.n,
              (double)hp.slots / hp.n);
    if (hp.on && hp.n % 32 == 0)
      fprintf(stderr, "[mmt ba profile] k_ba2_p3 us per solve: partials %.1f, assembly %.1f, "
              "LDL^T %.1f, substitutions %.1f, poses + state %.1f\n", hp.p3[0] * 0.01 / hp.n,
              hp.p3[1] * 0.01 / hp.n, hp.p3[2] * 0.01 / hp.n, hp.p3[3] * 0.01 / hp.n,
              hp.p3[4] * 0.01 / hp.n);
  }
}

}  // namespace mmt
