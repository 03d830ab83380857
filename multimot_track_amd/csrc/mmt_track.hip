// multimot_track_amd/csrc/mmt_track.hip -- per-frame association and pose-solve kernels.
//
//   k_gray_depth      cvtColor RGB2GRAY on BGR bytes + disparity -> depth   (Tracking.cc:447-465)
//   k_static_samples  B2: static ORB keys associated through the flow         (Frame.cc:228-324)
//   k_obj_samples     B1: semi-dense object samples, order-preserving         (Frame.cc:188-217)
//   k_handoff         B4: correspondences -> current keys + depth/label gathers (Tracking.cc:487-578)
//   k_obj_group       B6 + B7 statistics: scene flow, per-label counts, ordered depth sums,
//                     member lists, last-label histograms           (Tracking.cc:1389-1536, 4007-4093)
//   k_flow_lm         D2 / D3: the whole g2o Levenberg-Marquardt of PoseOptimizationFlow2Cam /
//                     PoseOptimizationFlow2 in one workgroup per solve, fp64 (Optimizer.cc:396-601,
//                     2170-2377; g2o quirks as SURVEY.md Appendix B, see oracle/solve_ref.cpp)

#include <hip/hip_runtime.h>

#include <cfloat>

#include "mmt_devmath.h"
#include "mmt_internal.h"
#include "mmt_track.h"

namespace mmt {

// ------------------------------------------------------------------ frame preparation
__global__ __launch_bounds__(256) void k_gray_depth(const uint8_t* __restrict__ bgr, size_t bgr_pitch,
                                                    const uint16_t* __restrict__ disp,
                                                    size_t disp_pitch, uint8_t* __restrict__ gray,
                                                    size_t gray_pitch, float* __restrict__ depth,
                                                    size_t depth_pitch, int npix, float bf) {
  const int f = blockIdx.y;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < npix; p += gridDim.x * 256) {
    const uint8_t* c = bgr + f * bgr_pitch + 3 * (size_t)p;
    gray[f * gray_pitch + p] = (uint8_t)((c[0] * 4899 + c[1] * 9617 + c[2] * 1868 + (1 << 13)) >> 14);
    const float dp = (float)((float)disp[f * disp_pitch + p] / 256.0);
    depth[f * depth_pitch + p] = bf / dp;
  }
}

// order-preserving workgroup compaction helper: returns this lane's slot (or -1) and advances
// `base` by the round's total.  blockDim = 1024.
__device__ __forceinline__ int wg_compact_slot(bool keep, int* s_w, int& base) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned long long bal = __ballot(keep);
  if (lane == 0) s_w[wave] = __popcll(bal);
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < nw; w++) {
    const int c = s_w[w];
    if (w < wave) off += c;
    tot += c;
  }
  const int slot = keep ? base + off + __popcll(bal & ((1ull << lane) - 1ull)) : -1;
  base += tot;
  __syncthreads();
  return slot;
}

// B2 (+ mvSiftDepthTmp) for one frame; single workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void k_static_samples(const mmt_kp* __restrict__ kps,
                                                         const int* __restrict__ nkp,
                                                         const float* __restrict__ depth,
                                                         const float2* __restrict__ flow,
                                                         const int32_t* __restrict__ mask, int W,
                                                         int H, SampleSet out) {
  __shared__ int s_w[16];
  const int n = *nkp;
  int base = 0;
  for (int r0 = 0; r0 < n; r0 += blockDim.x) {
    const int i = r0 + threadIdx.x;
    bool keep = false;
    float kx = 0, ky = 0, fxe = 0, fye = 0, d = 0;
    if (i < n) {
      kx = kps[i].x;
      ky = kps[i].y;
      const int x = (int)kx, y = (int)ky;
      const size_t p = (size_t)y * W + x;
      d = depth[p];
      if (mask[p] == 0 && !(d > 40 || d <= 0)) {
        const float2 fl = flow[p];
        fxe = fl.x;
        fye = fl.y;
        keep = fxe != 0 && fye != 0 && kx + fxe < W && ky + fye < H && kx < W && ky < H;
      }
    }
    const int slot = wg_compact_slot(keep, s_w, base);
    if (keep && slot < out.cap) {
      out.keys[slot] = make_float2(kx, ky);
      out.corres[slot] = make_float2(kx + fxe, ky + fye);
      out.flow[slot] = make_float2(fxe, fye);
      out.depth[slot] = d;  // > 0 here, mvSiftDepthTmp (Frame.cc:312-324)
    }
  }
  if (threadIdx.x == 0) *out.count = min(base, out.cap);
}

// B1 for one frame; single workgroup, grid positions in row-major order.
__global__ __launch_bounds__(1024) void k_obj_samples(const float* __restrict__ depth,
                                                      const float2* __restrict__ flow,
                                                      const int32_t* __restrict__ mask, int W,
                                                      int H, ObjSampleSet out) {
  __shared__ int s_w[16];
  const int gw = (W + 3) / 4, gh = (H + 3) / 4, n = gw * gh;
  int base = 0;
  for (int r0 = 0; r0 < n; r0 += blockDim.x) {
    const int g = r0 + threadIdx.x;
    bool keep = false;
    int i = 0, j = 0, lab = 0;
    float fx = 0, fy = 0, d = 0;
    if (g < n) {
      i = (g / gw) * 4;
      j = (g % gw) * 4;
      const size_t p = (size_t)i * W + j;
      lab = mask[p];
      d = depth[p];
      if (lab != 0 && d < 25 && d > 0) {
        const float2 fl = flow[p];
        fx = fl.x;
        fy = fl.y;
        keep = (float)j + fx < (float)W && (float)j + fx > 0 && (float)i + fy < (float)H &&
               (float)i + fy > 0;
      }
    }
    const int slot = wg_compact_slot(keep, s_w, base);
    if (keep && slot < out.cap) {
      out.keys[slot] = make_float2((float)j, (float)i);
      out.corres[slot] = make_float2((float)j + fx, (float)i + fy);
      out.flow[slot] = make_float2(fx, fy);
      out.depth[slot] = d;
      out.label[slot] = lab;
    }
  }
  if (threadIdx.x == 0) *out.count = min(base, out.cap);
}

// B4: current keys = last correspondences; depth (and label) at std::round coordinates.
__global__ __launch_bounds__(256) void k_handoff(const float2* __restrict__ last_corres,
                                                 const int* __restrict__ n_last,
                                                 const float2* __restrict__ last_ocorres,
                                                 const int* __restrict__ n_olast,
                                                 const float* __restrict__ depth,
                                                 const int32_t* __restrict__ mask, int W, int H,
                                                 HandoffSet cur) {
  const int ns = *n_last, no = *n_olast;
  const int tid = blockIdx.x * 256 + threadIdx.x, nt = gridDim.x * 256;
  for (int i = tid; i < ns; i += nt) {
    const float2 k = last_corres[i];
    cur.skeys[i] = k;
    const float ru = roundf(k.x), rv = roundf(k.y);
    float dd = -1.f;
    if (ru < W && ru > 0 && rv < H && rv > 0) {
      const float d = depth[(size_t)rv * W + (size_t)ru];
      if (d > 0) dd = d;
    }
    cur.sdepth[i] = dd;
  }
  for (int i = tid; i < no; i += nt) {
    const float2 k = last_ocorres[i];
    cur.okeys[i] = k;
    const float ru = roundf(k.x), rv = roundf(k.y);
    if (ru < W && ru > 0 && rv < H && rv > 0) {
      const size_t p = (size_t)rv * W + (size_t)ru;
      cur.odepth[i] = depth[p];
      cur.olabel[i] = mask[p];
    } else {
      cur.odepth[i] = 0.1f;
      cur.olabel[i] = 0;
    }
  }
  if (tid == 0) {
    *cur.ns = ns;
    *cur.no = no;
  }
}

// Frame::UnprojectStereoObject(i, 0) with cv::gemm's double accumulation (Frame.cc:1118-1152).
__device__ __forceinline__ void unproject_world(const float* T, float fx, float fy, float cx,
                                                float cy, float u, float v, float z, float out[3]) {
  const float invfx = 1.0f / fx, invfy = 1.0f / fy;
  const float x = (u - cx) * z * invfx, y = (v - cy) * z * invfy;
  const float xc[3] = {x, y, z};
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double s = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      s += (double)T[4 * k + r] * (double)T[4 * k + 3];
      s2 += (double)T[4 * k + r] * (double)xc[k];
    }
    out[r] = (float)s2 + (float)(-s);
  }
}

// B6 + B7 statistics for one frame; single workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void k_obj_group(GroupArgs a) {
  __shared__ int s_cnt[kMaxLabel], s_bcnt[kMaxLabel], s_sfcnt[kMaxLabel];
  __shared__ int s_wl[16 * kMaxLabel];
  __shared__ int s_hist[kMaxLabel * kMaxLabel];
  const int n = *a.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < kMaxLabel; i += blockDim.x) s_cnt[i] = s_bcnt[i] = s_sfcnt[i] = 0;
  for (int i = tid; i < kMaxLabel * kMaxLabel; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
  int base[kMaxLabel];
#pragma unroll
  for (int l = 0; l < kMaxLabel; l++) base[l] = 0;
  for (int r0 = 0; r0 < n; r0 += blockDim.x) {
    const int i = r0 + tid;
    int lab = -1;
    if (i < n) {
      const int cl = a.cur_label[i], ll = a.last_label[i];
      if (cl <= 0 || ll <= 0) {
        a.obj_label[i] = -1;  // vObjLabel (GetSceneFlowObj, Tracking.cc:4021-4025)
      } else {
        a.obj_label[i] = -2;
        float xp[3], xc[3];
        const float2 kl = a.last_keys[i], kc = a.cur_keys[i];
        unproject_world(a.Tlast, a.fx, a.fy, a.cx, a.cy, kl.x, kl.y, a.last_depth[i], xp);
        unproject_world(a.Tcur, a.fx, a.fy, a.cx, a.cy, kc.x, kc.y, a.cur_depth[i], xc);
        const float f0 = xc[0] - xp[0], f2 = xc[2] - xp[2];
        const float sf = sqrtf(f0 * f0 + f2 * f2);
        lab = cl < kMaxLabel ? cl : -1;
        if (lab < 0) atomicOr(a.err, 1);
        if (lab >= 0) {
          const float u = kc.x, v = kc.y;
          const bool bnd = v < 25 || v > (float)(a.H - 25) || u < 50 || u > (float)(a.W - 50);
          atomicAdd(&s_cnt[lab], 1);
          if (bnd) atomicAdd(&s_bcnt[lab], 1);
          if (sf < 0.12f) atomicAdd(&s_sfcnt[lab], 1);
          if (ll < kMaxLabel) atomicAdd(&s_hist[lab * kMaxLabel + ll], 1);
          else atomicOr(a.err, 1);
        }
      }
    }
    // ordered per-label member lists (Posi, ascending index)
    unsigned long long my_bal = 0;
#pragma unroll
    for (int l = 1; l < kMaxLabel; l++) {
      const unsigned long long bal = __ballot(lab == l);
      if (lane == 0) s_wl[wave * kMaxLabel + l] = __popcll(bal);
      if (lab == l) my_bal = bal;
    }
    __syncthreads();
    if (lab > 0) {
      int off = 0;
      for (int w = 0; w < wave; w++) off += s_wl[w * kMaxLabel + lab];
      const int rank = __popcll(my_bal & ((1ull << lane) - 1ull));
      const int slot = base[lab] + off + rank;
      if (slot < a.member_cap) a.members[lab * a.member_cap + slot] = i;
    }
    const int nw = blockDim.x >> 6;
#pragma unroll
    for (int l = 1; l < kMaxLabel; l++) {
      int tot = 0;
      for (int w = 0; w < nw; w++) tot += s_wl[w * kMaxLabel + l];
      base[l] += tot;
    }
    __syncthreads();
  }
  // ordered float depth sums (obj_center_depth accumulates in index order, Tracking.cc:1473)
  if (tid < kMaxLabel) {
    const int l = tid;
    const int m = min(base[l], a.member_cap);
    float s = 0;
    for (int k = 0; k < m; k++) s = s + a.cur_depth[a.members[l * a.member_cap + k]];
    a.stats[l].cnt = s_cnt[l];
    a.stats[l].bcnt = s_bcnt[l];
    a.stats[l].sfcnt = s_sfcnt[l];
    a.stats[l].depth_sum = s;
    a.stats[l].members = m;
  }
  for (int i = tid; i < kMaxLabel * kMaxLabel; i += blockDim.x) a.hist[i] = s_hist[i];
}

// ------------------------------------------------------------------ D2 / D3 Levenberg-Marquardt
// Edge scratch (SoA doubles, `cap` each): Xw0..2, OB0..1, PR0..1, F0..1, FS0..1, W, BL0..1,
// XL0..1, E0..1.
enum { S_X0 = 0, S_X1, S_X2, S_OB0, S_OB1, S_PR0, S_PR1, S_F0, S_F1, S_FS0, S_FS1, S_W, S_BL0,
       S_BL1, S_XL0, S_XL1, S_E0, S_E1, S_COUNT };

__device__ __forceinline__ void huber(double e, double dsqr, double delta, double& r0, double& r1) {
  if (e <= dsqr) {
    r0 = e;
    r1 = 1.;
  } else {
    const double s = sqrt(e);
    r0 = 2 * s * delta - dsqr;
    r1 = delta / s;
  }
}

__device__ __forceinline__ void jac(double x, double y, double z, double fx, double fy,
                                    double J[2][6]) {
  const double z2 = z * z;
  J[0][0] = x * y / z2 * fx;
  J[0][1] = -(1 + (x * x / z2)) * fx;
  J[0][2] = y / z * fx;
  J[0][3] = -1. / z * fx;
  J[0][4] = 0;
  J[0][5] = x / z2 * fx;
  J[1][0] = (1 + y * y / z2) * fy;
  J[1][1] = -x * y / z2 * fy;
  J[1][2] = -x / z * fy;
  J[1][3] = 0;
  J[1][4] = -1. / z * fy;
  J[1][5] = y / z2 * fy;
}

__device__ __forceinline__ void se3_map(const DSE3& p, const double* S, int cap, int i,
                                        double& x, double& y, double& z) {
  dq_rotate(p.q, S[S_X0 * cap + i], S[S_X1 * cap + i], S[S_X2 * cap + i], x, y, z);
  x += p.t[0];
  y += p.t[1];
  z += p.t[2];
}

__global__ __launch_bounds__(256) void k_flow_lm(const FlowSolveDesc* __restrict__ descs) {
  __shared__ double s_red[4 * 28];
  __shared__ double s_out[28];
  __shared__ double s_max[4];
  __shared__ DSE3 s_pose, s_pose_new;
  __shared__ double s_Hpp[36], s_bp[6], s_xbuf[6];
  __shared__ double s_lambda, s_ni, s_cur, s_ini, s_chk;
  __shared__ int s_ok2, s_accept, s_stop, s_qmax, s_nbad, s_iters, s_bad;
  const FlowSolveDesc D = descs[blockIdx.x];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int N = D.d_n ? min(*D.d_n, D.cap) : min(D.n, D.cap);
  if (N < 3) {
    if (tid == 0) {
      D.stats[0] = 0;
      D.stats[1] = 0;
      D.stats[2] = 1;
    }
    return;
  }
  double* S = D.scratch;
  const int cap = D.cap;
  const double fx = D.fx, fy = D.fy, cx = D.cx, cy = D.cy;
  const double kInfo = 0.1, pinfo = D.prior_info;
  const float deltaF = sqrtf(D.rp_thres);
  const double delta = (double)deltaF, dsqr = delta * delta;
  // Twl = inverse(last Tcw): Rwl = R^T (float), twl = -R^T t via double-accumulated gemm
  float Rwl[9], twl[3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Rwl[3 * r + c] = D.Tcw_last[4 * c + r];
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)Rwl[3 * r + k] * (double)D.Tcw_last[4 * k + 3];
    twl[r] = (float)(-s);
  }
  for (int i = tid; i < N; i += nt) {
    const int s = D.idx ? D.idx[i] : i;
    const float2 ob = D.obs[s];
    float z = D.depth[s];
    if (D.use_noise) z = (float)((double)z + (double)D.g0 * ((double)(z * z) / (725 * 0.5) * 0.15));
    const double u = ob.x, v = ob.y, dz = z;
    const double Xc0 = (u - cx) * dz / fx, Xc1 = (v - cy) * dz / fy, Xc2 = dz;
    S[S_X0 * cap + i] = (double)Rwl[0] * Xc0 + (double)Rwl[1] * Xc1 + (double)Rwl[2] * Xc2 + (double)twl[0];
    S[S_X1 * cap + i] = (double)Rwl[3] * Xc0 + (double)Rwl[4] * Xc1 + (double)Rwl[5] * Xc2 + (double)twl[1];
    S[S_X2 * cap + i] = (double)Rwl[6] * Xc0 + (double)Rwl[7] * Xc1 + (double)Rwl[8] * Xc2 + (double)twl[2];
    S[S_OB0 * cap + i] = u;
    S[S_OB1 * cap + i] = v;
    const float2 fl = D.flow[s];
    S[S_PR0 * cap + i] = fl.x;
    S[S_PR1 * cap + i] = fl.y;
    S[S_F0 * cap + i] = fl.x;
    S[S_F1 * cap + i] = fl.y;
    S[S_XL0 * cap + i] = 0;
    S[S_XL1 * cap + i] = 0;
  }
  if (tid == 0) {
    s_pose = dse3_from_float(D.init);
    for (int k = 0; k < 6; k++) s_xbuf[k] = 0;
    s_chk = 0;
    s_stop = 0;
    s_iters = 0;
  }
  __syncthreads();
  for (int iter = 0; iter < D.max_iters; iter++) {
    // ---- linearise at the current state (computeActiveErrors + buildSystem)
    {
      double v[28];
#pragma unroll
      for (int k = 0; k < 28; k++) v[k] = 0;
      double mh = 0;
      const DSE3 P = s_pose;
      for (int i = tid; i < N; i += nt) {
        double x, y, z;
        se3_map(P, S, cap, i, x, y, z);
        const double pu = x / z * fx + cx, pv = y / z * fy + cy;
        const double f0 = S[S_F0 * cap + i], f1 = S[S_F1 * cap + i];
        const double e0 = (S[S_OB0 * cap + i] + f0) - pu, e1 = (S[S_OB1 * cap + i] + f1) - pv;
        const double p0 = f0 - S[S_PR0 * cap + i], p1 = f1 - S[S_PR1 * cap + i];
        const double e2 = kInfo * (e0 * e0 + e1 * e1);
        double r0, r1;
        huber(e2, dsqr, delta, r0, r1);
        v[27] += r0 + pinfo * (p0 * p0 + p1 * p1);
        const double w = kInfo * r1;
        double J[2][6];
        jac(x, y, z, fx, fy, J);
        int k = 0;
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
          for (int b = 0; b <= a; b++) v[k++] += J[0][a] * w * J[0][b] + J[1][a] * w * J[1][b];
        const double o0 = -w * e0, o1 = -w * e1;
#pragma unroll
        for (int a = 0; a < 6; a++) v[21 + a] += J[0][a] * o0 + J[1][a] * o1;
        S[S_W * cap + i] = w;
        S[S_BL0 * cap + i] = o0 - pinfo * p0;
        S[S_BL1 * cap + i] = o1 - pinfo * p1;
        mh = fmax(mh, w + pinfo);
      }
      wg_sum<28>(v, s_red, s_out);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mh = fmax(mh, __shfl_xor(mh, o, 64));
      if ((tid & 63) == 0) s_max[tid >> 6] = mh;
      __syncthreads();
      if (tid == 0) {
        int k = 0;
        for (int a = 0; a < 6; a++)
          for (int b = 0; b <= a; b++) {
            s_Hpp[6 * a + b] = s_out[k];
            s_Hpp[6 * b + a] = s_out[k];
            k++;
          }
        for (int a = 0; a < 6; a++) s_bp[a] = s_out[21 + a];
        s_cur = s_out[27];
        s_ini = s_out[27];
        if (iter == 0) {
          double md = 0;
          for (int a = 0; a < 6; a++) md = fmax(md, fabs(s_Hpp[7 * a]));
          for (int w = 0; w < (nt >> 6); w++) md = fmax(md, s_max[w]);
          s_lambda = 1e-5 * md;
          s_ni = 2;
          s_nbad = 0;
        }
        s_qmax = 0;
      }
      __syncthreads();
    }
    // ---- Levenberg trials
    double lastTrialChi = 0, rho = 0;
    for (;;) {
      const DSE3 P = s_pose;
      const double lam = s_lambda;
      // Schur complement over the flow "landmarks"
      {
        double v[27];
#pragma unroll
        for (int k = 0; k < 27; k++) v[k] = 0;
        for (int i = tid; i < N; i += nt) {
          double x, y, z;
          se3_map(P, S, cap, i, x, y, z);
          double J[2][6];
          jac(x, y, z, fx, fy, J);
          const double w = S[S_W * cap + i], h = w + pinfo;
          const double d00 = 1.0 / (h + lam), d01 = -h / ((h + lam) * lam), d11 = 1.0 / lam;
          const double bl0 = S[S_BL0 * cap + i], bl1 = S[S_BL1 * cap + i];
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
        wg_sum<27>(v, s_red, s_out);
      }
      if (tid == 0) {
        double Hs[36], bs[6], xp[6];
        int k = 0;
        for (int a = 0; a < 6; a++)
          for (int b = 0; b <= a; b++) {
            Hs[6 * a + b] = s_Hpp[6 * a + b] + (a == b ? lam : 0.0) - s_out[k];
            k++;
          }
        for (int a = 0; a < 6; a++) bs[a] = s_bp[a] - s_out[21 + a];
        const bool ok2 = ldlt_solve6(Hs, bs, xp);
        if (ok2)
          for (int a = 0; a < 6; a++) s_xbuf[a] = xp[a];
        s_ok2 = ok2;
        s_pose_new = dse3_mul(dse3_exp(s_xbuf), s_pose);
      }
      __syncthreads();
      // landmark back-substitution, update, errors of the trial state
      {
        const bool ok2 = s_ok2;
        const DSE3 PN = s_pose_new;
        double v[2] = {0, 0};
        for (int i = tid; i < N; i += nt) {
          double xl0, xl1;
          const double bl0 = S[S_BL0 * cap + i], bl1 = S[S_BL1 * cap + i];
          if (ok2) {
            double x, y, z;
            se3_map(P, S, cap, i, x, y, z);
            double J[2][6];
            jac(x, y, z, fx, fy, J);
            const double w = S[S_W * cap + i], h = w + pinfo;
            double c0 = bl0, c1 = bl1;
#pragma unroll
            for (int a = 0; a < 6; a++) {
              c0 -= w * J[0][a] * s_xbuf[a];
              c1 -= w * J[1][a] * s_xbuf[a];
            }
            xl0 = c0 / (h + lam) - h * c1 / ((h + lam) * lam);
            if (i > 0) xl0 += c0 / lam;  // stride-2 spill of landmark i-1's third Dinv row
            xl1 = c1 / lam;
            S[S_XL0 * cap + i] = xl0;
            S[S_XL1 * cap + i] = xl1;
          } else {
            xl0 = S[S_XL0 * cap + i];
            xl1 = S[S_XL1 * cap + i];
          }
          const double f0o = S[S_F0 * cap + i], f1o = S[S_F1 * cap + i];
          S[S_FS0 * cap + i] = f0o;
          S[S_FS1 * cap + i] = f1o;
          const double f0 = f0o + xl0, f1 = f1o + xl1;
          S[S_F0 * cap + i] = f0;
          S[S_F1 * cap + i] = f1;
          double x, y, z;
          se3_map(PN, S, cap, i, x, y, z);
          const double pu = x / z * fx + cx, pv = y / z * fy + cy;
          const double e0 = (S[S_OB0 * cap + i] + f0) - pu, e1 = (S[S_OB1 * cap + i] + f1) - pv;
          const double p0 = f0 - S[S_PR0 * cap + i], p1 = f1 - S[S_PR1 * cap + i];
          S[S_E0 * cap + i] = e0;
          S[S_E1 * cap + i] = e1;
          const double e2 = kInfo * (e0 * e0 + e1 * e1);
          double r0, r1;
          huber(e2, dsqr, delta, r0, r1);
          v[0] += r0 + pinfo * (p0 * p0 + p1 * p1);
          v[1] += xl0 * (lam * xl0 + bl0) + xl1 * (lam * xl1 + bl1);
        }
        wg_sum<2>(v, s_red, s_out);
      }
      if (tid == 0) {
        lastTrialChi = s_out[0];
        double tempChi = s_ok2 ? s_out[0] : DBL_MAX;
        double scale = s_out[1];
        for (int a = 0; a < 6; a++) scale += s_xbuf[a] * (lam * s_xbuf[a] + s_bp[a]);
        scale += 1e-3;
        rho = (s_cur - tempChi) / scale;
        if (rho > 0 && isfinite(tempChi)) {
          double alpha = 1. - pow((2 * rho - 1), 3);
          alpha = fmin(alpha, 2. / 3.);
          const double sf = fmax(1. / 3., alpha);
          s_lambda = lam * sf;
          s_ni = 2;
          s_cur = tempChi;
          s_pose = s_pose_new;
          s_accept = 1;
        } else {
          s_lambda = lam * s_ni;
          s_ni = s_ni * 2;
          s_accept = 0;
        }
        s_qmax = s_qmax + 1;
        // loop condition (rho < 0 && qmax < 10) and termination bookkeeping
        const bool again = (rho < 0 && s_qmax < 10);
        s_stop = again ? 0 : 1;
        if (!again) {
          bool ok = true;
          if (s_qmax == 10 || rho == 0) ok = false;
          if (ok) {
            if ((s_ini - s_cur) * 1e3 < s_ini)
              s_nbad = s_nbad + 1;
            else
              s_nbad = 0;
            if (s_nbad >= 3) ok = false;
          }
          if (s_chk < lastTrialChi && iter > 0) ok = false;
          s_chk = lastTrialChi;
          s_iters = iter + 1;
          s_bad = ok ? 0 : 1;
        }
      }
      __syncthreads();
      if (!s_accept)
        for (int i = tid; i < N; i += nt) {
          S[S_F0 * cap + i] = S[S_FS0 * cap + i];
          S[S_F1 * cap + i] = S[S_FS1 * cap + i];
        }
      const int stop = s_stop;
      __syncthreads();
      if (stop) break;
    }
    if (s_bad) break;
  }
  // outputs: pose, iterations, inliers from the last computed edge errors (Optimizer.cc:536-566)
  double v[1] = {0};
  for (int i = tid; i < N; i += nt) {
    const double e0 = S[S_E0 * cap + i], e1 = S[S_E1 * cap + i];
    const float chi2 = (float)(kInfo * (e0 * e0 + e1 * e1));
    if (chi2 > D.rp_thres) v[0] += 1.0;
  }
  wg_sum<1>(v, s_red, s_out);
  if (tid == 0) {
    dse3_to_float(s_pose, D.pose_out);
    D.stats[0] = s_iters;
    D.stats[1] = N - (int)s_out[0];
    D.stats[2] = 0;
  }
}

// ------------------------------------------------------------------ launchers
void launch_gray_depth(const uint8_t* bgr, size_t bgr_pitch, const uint16_t* disp,
                       size_t disp_pitch, uint8_t* gray, size_t gray_pitch, float* depth,
                       size_t depth_pitch, int npix, int nframes, float bf, hipStream_t st) {
  const int blocks = std::min((npix + 255) / 256, 2048);
  hipLaunchKernelGGL(k_gray_depth, dim3(blocks, nframes), dim3(256), 0, st, bgr, bgr_pitch, disp,
                     disp_pitch, gray, gray_pitch, depth, depth_pitch, npix, bf);
}

void launch_static_samples(const mmt_kp* kps, const int* nkp, const float* depth,
                           const float2* flow, const int32_t* mask, int W, int H,
                           const SampleSet& out, hipStream_t st) {
  hipLaunchKernelGGL(k_static_samples, dim3(1), dim3(1024), 0, st, kps, nkp, depth, flow, mask, W,
                     H, out);
}

void launch_obj_samples(const float* depth, const float2* flow, const int32_t* mask, int W,
                        int H, const ObjSampleSet& out, hipStream_t st) {
  hipLaunchKernelGGL(k_obj_samples, dim3(1), dim3(1024), 0, st, depth, flow, mask, W, H, out);
}

void launch_handoff(const float2* last_corres, const int* n_last, const float2* last_ocorres,
                    const int* n_olast, const float* depth, const int32_t* mask, int W, int H,
                    const HandoffSet& cur, hipStream_t st) {
  hipLaunchKernelGGL(k_handoff, dim3(32), dim3(256), 0, st, last_corres, n_last, last_ocorres,
                     n_olast, depth, mask, W, H, cur);
}

void launch_obj_group(const GroupArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_obj_group, dim3(1), dim3(1024), 0, st, a);
}

void launch_flow_lm(const FlowSolveDesc* d_descs, int nsolves, hipStream_t st) {
  hipLaunchKernelGGL(k_flow_lm, dim3(nsolves), dim3(256), 0, st, d_descs);
}

size_t flow_scratch_doubles(int cap) { return (size_t)S_COUNT * cap; }

}  // namespace mmt
