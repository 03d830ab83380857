// multimot_track_amd/csrc/mmt_track.hip -- per-frame association and pose-solve kernels.
//
//   k_gray_depth      cvtColor RGB2GRAY on BGR bytes + disparity -> depth   (Tracking.cc:447-465)
//   k_static_samples  B2: static ORB keys associated through the flow         (Frame.cc:228-324)
//   k_obj_samples     B1: semi-dense object samples, order-preserving         (Frame.cc:188-217)
//   k_handoff         B4: correspondences -> current keys + depth/label gathers (Tracking.cc:487-578)
//   k_obj_group       B6 + B7 statistics: scene flow, per-label counts, ordered depth sums,
//                     member lists, last-label histograms           (Tracking.cc:1389-1536, 4007-4093)
// (D2 / D3, the flow-refined pose solves, are in mmt_lm.hip)

#include <hip/hip_runtime.h>

#include <cfloat>

#include "mmt_devmath.h"
#include "mmt_internal.h"
#include "mmt_track.h"

namespace mmt {

// ------------------------------------------------------------------ frame preparation
__device__ __forceinline__ void gray_depth_px(const uint8_t* c, uint16_t d, float bf, uint8_t* g,
                                              float* z) {
  *g = (uint8_t)((c[0] * 4899 + c[1] * 9617 + c[2] * 1868 + (1 << 13)) >> 14);
  const float dp = (float)((float)d / 256.0);
  *z = bf / dp;
}

// Four pixels per thread: 12 BGR bytes and four u16 disparities in, one gray dword and four
// depths out (unaligned vector accesses: frame pitches need not be multiples of 4).
__global__ __launch_bounds__(256) void k_gray_depth(const uint8_t* __restrict__ bgr, size_t bgr_pitch,
                                                    const uint16_t* __restrict__ disp,
                                                    size_t disp_pitch, uint8_t* __restrict__ gray,
                                                    size_t gray_pitch, float* __restrict__ depth,
                                                    size_t depth_pitch, int npix, float bf) {
  const int f = blockIdx.y;
  const uint8_t* B = bgr + f * bgr_pitch;
  const uint16_t* D = disp + f * disp_pitch;
  uint8_t* G = gray + f * gray_pitch;
  float* Z = depth + f * depth_pitch;
  const int nq = npix >> 2;
  for (int q = blockIdx.x * 256 + threadIdx.x; q < nq; q += gridDim.x * 256) {
    uint8_t c[12];
    __builtin_memcpy(c, B + 12 * (size_t)q, 12);
    uint16_t d[4];
    __builtin_memcpy(d, D + 4 * (size_t)q, 8);
    uint8_t g[4];
    float z[4];
#pragma unroll
    for (int k = 0; k < 4; k++) gray_depth_px(c + 3 * k, d[k], bf, g + k, z + k);
    __builtin_memcpy(G + 4 * (size_t)q, g, 4);
    __builtin_memcpy(Z + 4 * (size_t)q, z, 16);
  }
  const int p = 4 * nq + blockIdx.x * 256 + threadIdx.x;
  if (p < npix) gray_depth_px(B + 3 * (size_t)p, D[p], bf, G + p, Z + p);
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

// B2 (+ mvSiftDepthTmp) for one frame; single workgroup of 1024 threads.  Each thread takes up to
// kSsItems consecutive keys per round and issues all their key loads, then all their depth, label
// and flow gathers, before anything waits: two memory round trips per round (a key count up to
// 4,096 is one round), not three per 1,024 keys.  The flow is gathered for every key and used
// only where the label and depth keep it.
constexpr int kSsItems = 4;

__device__ __forceinline__ int block_scan_excl(int v, int* s_w, int& excl);

__global__ __launch_bounds__(1024) void k_static_samples(const mmt_kp* __restrict__ kps,
                                                         const int* __restrict__ nkp,
                                                         const float* __restrict__ depth,
                                                         const float2* __restrict__ flow,
                                                         const int32_t* __restrict__ mask, int W,
                                                         int H, SampleSet out) {
  __shared__ int s_w[16];
  const int n = *nkp;
  int base = 0;
  for (int r0 = 0; r0 < n; r0 += kSsItems * (int)blockDim.x) {
    const int i0 = r0 + kSsItems * (int)threadIdx.x;
    float kx[kSsItems], ky[kSsItems], d[kSsItems];
    int lab[kSsItems];
    float2 fl[kSsItems];
#pragma unroll
    for (int k = 0; k < kSsItems; k++) {
      kx[k] = ky[k] = 0;
      if (i0 + k < n) {
        kx[k] = kps[i0 + k].x;
        ky[k] = kps[i0 + k].y;
      }
    }
#pragma unroll
    for (int k = 0; k < kSsItems; k++) {
      d[k] = 0;
      lab[k] = 1;
      fl[k] = make_float2(0.f, 0.f);
      if (i0 + k < n) {
        const size_t p = (size_t)(int)ky[k] * W + (int)kx[k];
        d[k] = depth[p];
        lab[k] = mask[p];
        fl[k] = flow[p];
      }
    }
    int cnt = 0;
    bool keep[kSsItems];
#pragma unroll
    for (int k = 0; k < kSsItems; k++) {
      const float fxe = fl[k].x, fye = fl[k].y;
      keep[k] = i0 + k < n && lab[k] == 0 && !(d[k] > 40 || d[k] <= 0) && fxe != 0 && fye != 0 &&
                kx[k] + fxe < W && ky[k] + fye < H && kx[k] < W && ky[k] < H;
      cnt += keep[k] ? 1 : 0;
    }
    int excl;
    const int tot = block_scan_excl(cnt, s_w, excl);
    int slot = base + excl;
#pragma unroll
    for (int k = 0; k < kSsItems; k++) {
      if (!keep[k]) continue;
      if (slot < out.cap) {
        out.keys[slot] = make_float2(kx[k], ky[k]);
        out.corres[slot] = make_float2(kx[k] + fl[k].x, ky[k] + fl[k].y);
        out.flow[slot] = fl[k];
        out.depth[slot] = d[k];  // > 0 here, mvSiftDepthTmp (Frame.cc:312-324)
      }
      slot++;
    }
    base += tot;
  }
  if (threadIdx.x == 0) *out.count = min(base, out.cap);
}

// B1 for one frame; single workgroup, grid positions in row-major order.
// exclusive block-wide scan of one int per thread (thread order); returns the total
__device__ __forceinline__ int block_scan_excl(int v, int* s_w, int& excl) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < nw; w++) {
    const int c = s_w[w];
    if (w < wave) off += c;
    tot += c;
  }
  excl = off + x - v;
  __syncthreads();
  return tot;
}

// B1: every 4th row/column, order-preserving, over kObjBlocks workgroups (one CU cannot pull the
// ~2 MB of sampled rows fast enough).  Two passes: k_obj_count counts each workgroup's kept
// samples, k_obj_write recomputes its flags, offsets by the counts of the workgroups before it
// and writes in order.  Workgroup b owns grid positions [b*per, (b+1)*per).
constexpr int kObjBlocks = 64;

__device__ __forceinline__ bool obj_keep(const float* __restrict__ depth,
                                         const float2* __restrict__ flow,
                                         const int32_t* __restrict__ mask, int W, int H, int gw,
                                         int g, int& lab, float& d, float2& fl) {
  const int i = (g / gw) * 4, j = (g % gw) * 4;
  const size_t p = (size_t)i * W + j;
  lab = mask[p];
  d = depth[p];
  fl = flow[p];
  if (!(lab != 0 && d < 25 && d > 0)) return false;
  return (float)j + fl.x < (float)W && (float)j + fl.x > 0 && (float)i + fl.y < (float)H &&
         (float)i + fl.y > 0;
}

__global__ __launch_bounds__(256) void k_obj_count(const float* __restrict__ depth,
                                                   const float2* __restrict__ flow,
                                                   const int32_t* __restrict__ mask, int W, int H,
                                                   int* __restrict__ counts) {
  __shared__ int s_w[4];
  const int gw = (W + 3) / 4, n = gw * ((H + 3) / 4);
  const int per = (n + kObjBlocks - 1) / kObjBlocks;
  const int g0 = blockIdx.x * per, g1 = min(n, g0 + per);
  int c = 0;
  for (int g = g0 + (int)threadIdx.x; g < g1; g += blockDim.x) {
    int lab;
    float d;
    float2 fl;
    c += obj_keep(depth, flow, mask, W, H, gw, g, lab, d, fl) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(256) void k_obj_write(const float* __restrict__ depth,
                                                   const float2* __restrict__ flow,
                                                   const int32_t* __restrict__ mask, int W, int H,
                                                   const int* __restrict__ counts,
                                                   ObjSampleSet out) {
  __shared__ int s_w[4];
  __shared__ int s_base;
  const int gw = (W + 3) / 4, n = gw * ((H + 3) / 4);
  const int per = (n + kObjBlocks - 1) / kObjBlocks;
  const int g0 = blockIdx.x * per, g1 = min(n, g0 + per);
  if (threadIdx.x < 64) {
    int b = 0;
    for (int k = threadIdx.x; k < (int)blockIdx.x; k += 64) b += counts[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (threadIdx.x == 0) s_base = b;
  }
  __syncthreads();
  int base = s_base;
  for (int r0 = g0; r0 < g1; r0 += blockDim.x) {
    const int g = r0 + threadIdx.x;
    int lab = 0;
    float d = 0;
    float2 fl = make_float2(0.f, 0.f);
    const bool keep = g < g1 && obj_keep(depth, flow, mask, W, H, gw, g, lab, d, fl);
    const int slot = wg_compact_slot(keep, s_w, base);
    if (keep && slot < out.cap) {
      const int i = (g / gw) * 4, j = (g % gw) * 4;
      out.keys[slot] = make_float2((float)j, (float)i);
      out.corres[slot] = make_float2((float)j + fl.x, (float)i + fl.y);
      out.flow[slot] = fl;
      out.depth[slot] = d;
      out.label[slot] = lab;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *out.count = min(base, out.cap);
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
constexpr int kDepthChunk = 512;

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
  // ordered float depth sums (obj_center_depth accumulates in index order, Tracking.cc:1473):
  // float addition is not associative, so each label's sum stays sequential -- but over depths
  // gathered into LDS in parallel, chunk by chunk, instead of dependent global loads
  __shared__ float s_dep[kMaxLabel][kDepthChunk];
  __shared__ int s_m[kMaxLabel];
  if (tid < kMaxLabel) s_m[tid] = min(base[tid], a.member_cap);
  __syncthreads();
  int mmax = 0;
  for (int l = 0; l < kMaxLabel; l++) mmax = max(mmax, s_m[l]);
  float dsum = 0;
  for (int c0 = 0; c0 < mmax; c0 += kDepthChunk) {
    for (int e = tid; e < kMaxLabel * kDepthChunk; e += blockDim.x) {
      const int l = e / kDepthChunk, k = e - l * kDepthChunk;
      if (c0 + k < s_m[l]) s_dep[l][k] = a.cur_depth[a.members[l * a.member_cap + c0 + k]];
    }
    __syncthreads();
    if (tid < kMaxLabel) {
      const int m = min(s_m[tid] - c0, kDepthChunk);
      for (int k = 0; k < m; k++) dsum = dsum + s_dep[tid][k];
    }
    __syncthreads();
  }
  if (tid < kMaxLabel) {
    const int l = tid;
    a.stats[l].cnt = s_cnt[l];
    a.stats[l].bcnt = s_bcnt[l];
    a.stats[l].sfcnt = s_sfcnt[l];
    a.stats[l].depth_sum = dsum;
    a.stats[l].members = s_m[l];
  }
  for (int i = tid; i < kMaxLabel * kMaxLabel; i += blockDim.x) a.hist[i] = s_hist[i];
}

// ------------------------------------------------------------------ D2 / D3 Levenberg-Marquardt
// Edge scratch (SoA doubles, `cap` each): Xw0..2, OB0..1, PR0..1, F0..1, FS0..1, W, BL0..1,
// XL0..1, E0..1.
// ------------------------------------------------------------------ launchers
void launch_gray_depth(const uint8_t* bgr, size_t bgr_pitch, const uint16_t* disp,
                       size_t disp_pitch, uint8_t* gray, size_t gray_pitch, float* depth,
                       size_t depth_pitch, int npix, int nframes, float bf, hipStream_t st) {
  const int blocks = std::max(1, std::min((npix / 4 + 255) / 256, 2048));
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
  hipLaunchKernelGGL(k_obj_count, dim3(kObjBlocks), dim3(256), 0, st, depth, flow, mask, W, H,
                     out.block_counts);
  hipLaunchKernelGGL(k_obj_write, dim3(kObjBlocks), dim3(256), 0, st, depth, flow, mask, W, H,
                     out.block_counts, out);
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

}  // namespace mmt
