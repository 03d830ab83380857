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
  const double in = 1.0 / sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x *= in; q.y *= in; q.z *= in; q.w *= in;
}

// Eigen::Quaternion(const Matrix3&): trace branch, else largest-diagonal branch (the three
// (i, j, k) cases written out so nothing is indexed at run time).
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
    if (R[2][2] > (i == 0 ? R[0][0] : R[1][1])) i = 2;
    if (i == 0) {  // j = 1, k = 2
      double s = sqrt(R[0][0] - R[1][1] - R[2][2] + 1.0);
      q.x = 0.5 * s;
      s = 0.5 / s;
      q.w = (R[2][1] - R[1][2]) * s;
      q.y = (R[1][0] + R[0][1]) * s;
      q.z = (R[2][0] + R[0][2]) * s;
    } else if (i == 1) {  // j = 2, k = 0
      double s = sqrt(R[1][1] - R[2][2] - R[0][0] + 1.0);
      q.y = 0.5 * s;
      s = 0.5 / s;
      q.w = (R[0][2] - R[2][0]) * s;
      q.z = (R[2][1] + R[1][2]) * s;
      q.x = (R[0][1] + R[1][0]) * s;
    } else {  // j = 0, k = 1
      double s = sqrt(R[2][2] - R[0][0] - R[1][1] + 1.0);
      q.z = 0.5 * s;
      s = 0.5 / s;
      q.w = (R[1][0] - R[0][1]) * s;
      q.x = (R[0][2] + R[2][0]) * s;
      q.y = (R[1][2] + R[2][1]) * s;
    }
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
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
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
#pragma unroll
  for (int r = 0; r < 3; r++) {
#pragma unroll
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
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) O2[r][c] = O[r][0] * O[0][c] + O[r][1] * O[1][c] + O[r][2] * O[2][c];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + O[r][c] + O2[r][c];
        V[r][c] = R[r][c];
      }
  } else {
    double st, ct;
    sincos(theta, &st, &ct);
    const double a = st / theta, b = (1 - ct) / (theta * theta);
    const double c2 = (theta - st) / (theta * theta * theta);
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) {
        R[r][c] = (r == c ? 1.0 : 0.0) + a * O[r][c] + b * O2[r][c];
        V[r][c] = (r == c ? 1.0 : 0.0) + b * O[r][c] + c2 * O2[r][c];
      }
  }
  DSE3 s;
  s.q = dq_from_R(R);
#pragma unroll
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

// 6x6 LDLT with symmetric diagonal pivoting on the LOWER triangle (Eigen LDLT<MatrixXd>); returns
// false when not positive (LDLT::isPositive()).  Every array index is a compile-time constant
// (pivot swaps by predicated unrolled blocks), so the factorisation stays in registers.
__device__ inline bool ldlt_solve6(const double (&Hl)[36], const double (&b)[6], double (&x)[6]) {
  double A[6][6], L[6][6], D[6];
  int perm[6] = {0, 1, 2, 3, 4, 5};
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int c = 0; c < 6; c++) {
      A[r][c] = (c <= r) ? Hl[6 * r + c] : Hl[6 * c + r];
      L[r][c] = 0.0;
    }
  bool positive = true;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    int p = k;
    double best = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < 6; i++)
      if (fabs(A[i][i]) > best) {
        best = fabs(A[i][i]);
        p = i;
      }
#pragma unroll
    for (int i = k + 1; i < 6; i++)
      if (p == i) {
#pragma unroll
        for (int c = 0; c < 6; c++) {
          const double t = A[k][c];
          A[k][c] = A[i][c];
          A[i][c] = t;
        }
#pragma unroll
        for (int r = 0; r < 6; r++) {
          const double t = A[r][k];
          A[r][k] = A[r][i];
          A[r][i] = t;
        }
#pragma unroll
        for (int c = 0; c < k; c++) {
          const double t = L[k][c];
          L[k][c] = L[i][c];
          L[i][c] = t;
        }
        const int t = perm[k];
        perm[k] = perm[i];
        perm[i] = t;
      }
    double d = A[k][k];
#pragma unroll
    for (int c = 0; c < k; c++) d -= L[k][c] * L[k][c] * D[c];
    D[k] = d;
    if (d < 0) positive = false;
#pragma unroll
    for (int i = k + 1; i < 6; i++) {
      double s = A[i][k];
#pragma unroll
      for (int c = 0; c < k; c++) s -= L[i][c] * L[k][c] * D[c];
      L[i][k] = (d != 0) ? s / d : 0.0;
    }
    L[k][k] = 1.0;
  }
  if (!positive) return false;
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double v = 0;
#pragma unroll
    for (int j = 0; j < 6; j++)
      if (perm[i] == j) v = b[j];
    y[i] = v;
  }
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int c = 0; c < i; c++) y[i] -= L[i][c] * y[c];
#pragma unroll
  for (int i = 0; i < 6; i++) y[i] = (D[i] != 0) ? y[i] / D[i] : 0.0;
#pragma unroll
  for (int i = 5; i >= 0; i--)
#pragma unroll
    for (int r = i + 1; r < 6; r++) y[i] -= L[r][i] * y[r];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 6; j++)
      if (perm[i] == j) x[j] = y[i];
  return true;
}

// Block sum of K <= 32 doubles held per thread (blockDim a multiple of 64): a butterfly
// reduce-scatter inside each wave (32 shuffles instead of 6 per value), then one LDS pass across
// waves.  `red` holds 32 doubles per wave; the sums land in out[0..K) (LDS), visible to every
// thread on return.
template <int K>
__device__ inline void block_sum(const double (&v)[K], double* red, double* out,
                                 int nw_active = 0) {
  static_assert(K <= 32, "block_sum: at most 32 values");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = nw_active > 0 ? nw_active : (int)(blockDim.x >> 6);
  double a[16];
  {
    const bool hi = lane & 32;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const double x0 = j < K ? v[j] : 0.0, x1 = (16 + j) < K ? v[16 + j] : 0.0;
      a[j] = (hi ? x1 : x0) + __shfl_xor(hi ? x0 : x1, 32, 64);
    }
  }
#pragma unroll
  for (int h = 8, bit = 16; h >= 1; h >>= 1, bit >>= 1) {
    const bool hi = lane & bit;
#pragma unroll
    for (int j = 0; j < h; j++) a[j] = (hi ? a[h + j] : a[j]) + __shfl_xor(hi ? a[j] : a[h + j], bit, 64);
  }
  a[0] += __shfl_xor(a[0], 1, 64);
  const int idx = lane >> 1;  // value index this lane pair holds
  if (nw == 1) {
    if (!(lane & 1) && idx < K) out[idx] = a[0];
    __syncthreads();
    return;
  }
  if (!(lane & 1) && idx < K) red[wave * 32 + idx] = a[0];
  __syncthreads();
  if (threadIdx.x < K) {
    double s = 0;
    for (int w = 0; w < nw; w++) s += red[w * 32 + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

// Block sum of K <= 32 doubles per thread by an LDS transpose: every lane stores its K partials
// in a row of a [64][33] tile per wave, lane k of each wave then sums column k (64 LDS reads,
// four interleaved chains), and the per-wave partials are added.  Fewer cross-lane operations
// than a shuffle tree when K is large.  `tile` holds 64 * 33 doubles per wave, `part` 32 per wave;
// out[0..K) is visible to every thread on return.  blockDim <= 256.
template <int K>
__device__ inline void block_sum_t(const double (&v)[K], double* tile, double* part, double* out,
                                   int nw_active = 0) {
  static_assert(K <= 32, "block_sum_t: at most 32 values");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = nw_active > 0 ? nw_active : (int)(blockDim.x >> 6);
  double* t = tile + (size_t)wave * 64 * 33;
#pragma unroll
  for (int k = 0; k < K; k++) t[lane * 33 + k] = v[k];
  // the tile is the wave's own: a wave-level LDS fence replaces the workgroup barrier
#ifdef MMT_DBG_BARRIER
  __syncthreads();
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
  if (lane < K) {
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll 4
    for (int r = 0; r < 64; r += 4) {
      s0 += t[(r + 0) * 33 + lane];
      s1 += t[(r + 1) * 33 + lane];
      s2 += t[(r + 2) * 33 + lane];
      s3 += t[(r + 3) * 33 + lane];
    }
    const double s = (s0 + s1) + (s2 + s3);
    if (nw == 1)
      out[lane] = s;
    else
      part[wave * 32 + lane] = s;
  }
  __syncthreads();
  if (nw > 1) {
    if (threadIdx.x < K) {
      double s = 0;
      for (int w = 0; w < nw; w++) s += part[w * 32 + threadIdx.x];
      out[threadIdx.x] = s;
    }
    __syncthreads();
  }
}

// Workgroup sum of K <= 64 values per thread that the threads have written into their rows of a
// [64][65] per-wave LDS tile (tile_row()) while computing them, so the sums never occupy
// registers.  Lane k of each wave sums column k, the wave partials meet in `part` (nw * K).
// out[0..K) is visible to every thread on return.
constexpr int kTileStride = 65;
template <int STRIDE = kTileStride>
__device__ __forceinline__ double* tile_row(double* tile) {
  return tile + (size_t)(threadIdx.x >> 6) * 64 * STRIDE + (threadIdx.x & 63) * STRIDE;
}

// STRIDE >= K: row stride of the tile in doubles (odd: conflict-free row stores)
template <int K, int STRIDE = kTileStride>
__device__ inline void block_sum_tile(double* tile, double* part, double* out, int nw_active = 0) {
  static_assert(K <= 64 && K <= STRIDE, "block_sum_tile: at most 64 values");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = nw_active > 0 ? nw_active : (int)(blockDim.x >> 6);
  const double* t = tile + (size_t)wave * 64 * STRIDE;
  // the rows are the wave's own: a wave-level LDS fence orders them before the column reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // column sum in batches of 16 independent loads, so the LDS latency is paid 4 times, not 64
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (lane < K) {
#pragma unroll
    for (int r0 = 0; r0 < 64; r0 += 16) {
      double x[16];
#pragma unroll
      for (int j = 0; j < 16; j++) x[j] = t[(r0 + j) * STRIDE + lane];
#pragma unroll
      for (int j = 0; j < 16; j++) acc[j & 7] += x[j];
    }
  }
  const double mine = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (nw == 1) {
    if (lane < K) out[lane] = mine;
    __syncthreads();
    return;
  }
  if (lane < K) part[wave * K + lane] = mine;
  __syncthreads();
  if (threadIdx.x < K) {
    double s = 0;
    for (int w = 0; w < nw; w++) s += part[w * K + threadIdx.x];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

// block_sum_tile whose result stays in registers: every wave adds the wave partials itself (same
// order everywhere, so every wave holds the same bits) and returns sum k in lane k.  One barrier,
// no broadcast through LDS; read single sums with lane_value().
template <int K>
__device__ inline double block_sum_tile_lanes(double* tile, double* part, int nw) {
  static_assert(K <= 64, "block_sum_tile_lanes: at most 64 values");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double* t = tile + (size_t)wave * 64 * kTileStride;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (lane < K) {
#pragma unroll
    for (int r0 = 0; r0 < 64; r0 += 16) {
      double x[16];
#pragma unroll
      for (int j = 0; j < 16; j++) x[j] = t[(r0 + j) * kTileStride + lane];
#pragma unroll
      for (int j = 0; j < 16; j++) acc[j & 7] += x[j];
    }
  }
  const double mine = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (nw == 1) return lane < K ? mine : 0.0;
  if (lane < K) part[wave * K + lane] = mine;
  __syncthreads();
  double s = 0;
  if (lane < K)
    for (int w = 0; w < nw; w++) s += part[w * K + lane];
  // the partials are read before anyone rewrites `part` (the next reduction is a full pass away,
  // with a barrier in between)
  return s;
}

// value held by lane `l` (a compile-time constant in unrolled code), as a wave-uniform scalar
__device__ __forceinline__ double lane_value(double v, int l) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// v + (v of the lane selected by the DPP control CTRL), both 32-bit halves moved by DPP
template <int CTRL>
__device__ __forceinline__ double dpp_add(double v) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
  return v + __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// ---- register reduce-scatter of 64 doubles per lane (gfx950 v_permlane32/16_swap + DPP): after
// six halving steps every lane holds the wave's sum of one value index, a permutation of 0..63
// that wave_rs_index() reads off once.  No LDS; the sums never leave registers.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// x, y swapped across the lane halves of 32 (W = 32) or of 16 within each 32 (W = 16), then added:
// one half of the lanes holds x's pair sums, the other y's
template <int W>
__device__ __forceinline__ double swap_add(double x, double y) {
  const unsigned long long bx = __double_as_longlong(x), by = __double_as_longlong(y);
  unsigned xl, yl, xh, yh;
  if (W == 32) {
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)bx, (unsigned)by, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(bx >> 32), (unsigned)(by >> 32),
                                                     false, false);
    xl = lo[0]; yl = lo[1]; xh = hi[0]; yh = hi[1];
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)bx, (unsigned)by, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(bx >> 32), (unsigned)(by >> 32),
                                                     false, false);
    xl = lo[0]; yl = lo[1]; xh = hi[0]; yh = hi[1];
  }
  return __longlong_as_double(((unsigned long long)xh << 32) | xl) +
         __longlong_as_double(((unsigned long long)yh << 32) | yl);
}

// a lane with BIT clear keeps x and sends y to its DPP partner (CTRL pairs it with a lane that
// has BIT set), which keeps y
template <int CTRL, int BIT>
__device__ __forceinline__ double pair_add(double x, double y, int lane) {
  const bool up = lane & BIT;
  return (up ? y : x) + dpp_mov<CTRL>(up ? x : y);
}

__device__ __forceinline__ double wave_reduce_scatter64(double (&v)[64]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 32; k++) v[k] = swap_add<32>(v[k], v[k + 32]);
#pragma unroll
  for (int k = 0; k < 16; k++) v[k] = swap_add<16>(v[k], v[k + 16]);
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = pair_add<0x128, 8>(v[k], v[k + 8], lane);  // row_ror:8
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = pair_add<0x141, 4>(v[k], v[k + 4], lane);  // row_half_mirror
#pragma unroll
  for (int k = 0; k < 2; k++) v[k] = pair_add<0x4E, 2>(v[k], v[k + 2], lane);   // quad [2,3,0,1]
  return pair_add<0xB1, 1>(v[0], v[1], lane);                                   // quad [1,0,3,2]
}

// the value index this lane ends with in wave_reduce_scatter64 (one-hot probe: lane 0 holds
// k + 1 at index k, every other lane zeros)
__device__ __forceinline__ int wave_rs_index() {
  const int lane = threadIdx.x & 63;
  double v[64];
#pragma unroll
  for (int k = 0; k < 64; k++) v[k] = lane == 0 ? (double)(k + 1) : 0.0;
  return (int)wave_reduce_scatter64(v) - 1;
}

// Workgroup sums of 64 doubles per thread held in registers (v[63] a pad), returned as
// block_sum_tile_lanes returns them: sum k in lane k, the same in every wave.  idx =
// wave_rs_index(); `part` holds 64 * nw doubles; one barrier.
__device__ inline double block_sum_regs64(double (&v)[64], double* part, int nw, int idx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  part[wave * 64 + idx] = wave_reduce_scatter64(v);
  __syncthreads();
  double t = 0;
  for (int w = 0; w < nw; w++) t += part[w * 64 + lane];
  return t;
}

// wave sum of a double, wave-uniform result: quad swaps (xor 1, xor 2), half-row and row mirrors
// give every lane its 16-lane row sum, then the four row sums are added from lanes 0/16/32/48 in
// a fixed order.  Inactive lanes must hold 0.
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v = dpp_add<0xB1>(v);   // quad_perm [1,0,3,2]
  v = dpp_add<0x4E>(v);   // quad_perm [2,3,0,1]
  v = dpp_add<0x141>(v);  // row_half_mirror
  v = dpp_add<0x140>(v);  // row_mirror
  return (lane_value(v, 0) + lane_value(v, 16)) + (lane_value(v, 32) + lane_value(v, 48));
}

// Workgroup sums of two doubles per thread, identical in every wave: DPP wave sums, one LDS
// exchange of the wave totals (`part`: 2 * nw doubles), one barrier.  For the light pass of an
// LM trial, whose two sums would otherwise pay a whole tile reduction's latency.
__device__ __forceinline__ void block_sum2(double a, double b, double* part, int nw, double& sa,
                                           double& sb) {
  a = wave_sum_dpp(a);
  b = wave_sum_dpp(b);
  if (nw == 1) {
    sa = a;
    sb = b;
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    part[2 * wave] = a;
    part[2 * wave + 1] = b;
  }
  __syncthreads();
  double s0 = 0, s1 = 0;
  for (int w = 0; w < nw; w++) {
    s0 += part[2 * w];
    s1 += part[2 * w + 1];
  }
  sa = s0;
  sb = s1;
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
