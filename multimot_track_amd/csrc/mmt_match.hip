// multimot_track_amd/csrc/mmt_match.hip -- frame grid (B3) and projection matching (C1-C3).
//
//   k_stereo_grid   B3: Frame::ComputeStereoFromRGBD (Frame.cc:1041-1062) and AssignFeaturesToGrid
//                   (Frame.cc:601-616, PosInGrid 765-775) as a per-frame counting sort: the grid
//                   is CSR over cells ix * 48 + iy, so GetFeaturesInArea's cell walk (x outer,
//                   y inner, key order inside a cell) is one contiguous index range per column.
//   k_sbp_frame     C2 candidates: ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
//                   ORBmatcher.cc:1958-2102, one wave per last-frame MapPoint.
//   k_local_cand    C3 candidates: Frame::isInFrustum (Frame.cc:652-708, PredictScale
//                   MapPoint.cc:402-417) + ORBmatcher::SearchByProjection(Frame&,
//                   vector<MapPoint*>, th) ORBmatcher.cc:418-502, one wave per local MapPoint.
//   k_match_fix     the order-dependent part of both matchers: a key bound by an earlier point is
//                   skipped by later ones (`mvpMapPoints[i2]->Observations() > 0`).  One
//                   1024-thread workgroup iterates "each point's choice given the choices before
//                   it" to its fixpoint, which is the sequential replay (see the kernel).  C2's
//                   rotation-consistency histogram (ComputeThreeMaxima, ORBmatcher.cc:2236-2275)
//                   runs at the end.
// C1 (DescriptorDistance, ORBmatcher.cc:2279-2295) is the XOR + popcount of eight dwords.
//
// Each candidate is ranked by (distance, position in GetFeaturesInArea's order): the reference's
// strict `dist < bestDist` keeps the first of equal distances, and its best/second-best tracker
// equals the two smallest of that ranking.  A wave keeps the kCandK smallest; a point whose unbound
// choices run past them is rescanned over the whole window against the current bindings.

#include <hip/hip_runtime.h>

#include <atomic>
#include <climits>
#include <cmath>

#include "mmt_bow.h"
#include "mmt_internal.h"
#include "mmt_match.h"
#include "mmt_track.h"

namespace mmt {

static constexpr int TH_HIGH = 100;      // ORBmatcher.cc:41
static constexpr int HISTO_LENGTH = 30;  // ORBmatcher.cc:43
static constexpr uint32_t kNoCand = 0xFFFFFFFFu;

// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ int grid_block_scan_excl(int v, int* s_w, int& excl) {
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

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// PosInGrid (Frame.cc:765-775): C round() of the float product; -1 outside the grid.
__device__ __forceinline__ int grid_cell(float x, float y, float invW, float invH) {
  const int px = (int)roundf((x - 0.0f) * invW);
  const int py = (int)roundf((y - 0.0f) * invH);
  if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) return -1;
  return px * kGridRows + py;
}

// R * x + t of a row-major float pose: cv::Mat gemm (double accumulation, rounded to float) and
// the translation added in float, as the CPU checker pins it.
__device__ __forceinline__ void pose_xform(const float* T, const float* x, float* y) {
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double s = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) s += (double)T[4 * r + k] * (double)x[k];
    y[r] = (float)s + T[4 * r + 3];
  }
}
__device__ __forceinline__ void pose_centre(const float* T, float* o) {  // -R^T t
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double s = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    o[r] = (float)(-s);
  }
}

// ------------------------------------------------------------------------------ B3
// One workgroup per frame.  LDS: the frame's cell counts, then (LDS variant) the cell lists, built
// and sorted in LDS and written out once, coalesced; the global variant (capacities above the LDS
// budget) sorts in place in HBM.  With `ho` set, the frame's keys, descriptors, uR and depths go
// straight into the caller's pinned host buffers (n valid entries, 16-byte stores), with its key
// count and the ORB error word: the host copies of the chunk need no copy launches of their own.
template <bool LDS>
__global__ __launch_bounds__(1024) void k_stereo_grid(const mmt_kp* __restrict__ keys,
                                                      const int* __restrict__ nkp, int cap,
                                                      const float* __restrict__ depth,
                                                      size_t depth_pitch, int W, float bf,
                                                      float invW, float invH, float* uR,
                                                      float* kdepth, int* cell_start,
                                                      int* cell_idx, B3HostOut ho) {
  __shared__ int s_cnt[kGridCells];
  __shared__ int s_w[16];
  extern __shared__ int s_idx[];  // LDS: cap entries
  const int f = blockIdx.x, t = threadIdx.x;
  keys += (size_t)f * cap;
  depth += (size_t)f * depth_pitch;
  uR += (size_t)f * cap;
  kdepth += (size_t)f * cap;
  cell_start += (size_t)f * (kGridCells + 1);
  cell_idx += (size_t)f * cap;
  const int n = min(nkp[f], cap);
  for (int c = t; c < kGridCells; c += blockDim.x) s_cnt[c] = 0;
  __syncthreads();
  for (int i = t; i < n; i += blockDim.x) {
    const float x = keys[i].x, y = keys[i].y;
    const float d = depth[(size_t)(int)y * W + (int)x];  // at<float>(v, u): truncation
    float dd = -1.f, ur = -1.f;
    if (d > 0) {
      dd = d;
      ur = x - bf / d;
    }
    kdepth[i] = dd;
    uR[i] = ur;
    if (ho.uR) {
      ho.uR[(size_t)f * cap + i] = ur;
      ho.kdepth[(size_t)f * cap + i] = dd;
    }
    const int c = grid_cell(x, y, invW, invH);
    if (c >= 0) atomicAdd(&s_cnt[c], 1);
  }
  if (ho.kps) {
    // keys (7 words each: one word per thread, consecutive lanes on consecutive words) and
    // descriptors (two 16-byte halves) of the valid entries
    static_assert(sizeof(mmt_kp) == 28, "mmt_kp layout");
    const uint32_t* k1 = (const uint32_t*)keys;
    uint32_t* hk = (uint32_t*)(ho.kps + (size_t)f * cap);
    for (int i = t; i < 7 * n; i += blockDim.x) hk[i] = k1[i];
    const uint4* d4 = (const uint4*)(ho.ddesc + (size_t)f * cap * 32);
    uint4* hd = (uint4*)(ho.desc + (size_t)f * cap * 32);
    for (int i = t; i < 2 * n; i += blockDim.x) hd[i] = d4[i];
    if (t == 0) {
      ho.nkp[f] = nkp[f];
      if (f == 0) ho.nkp[gridDim.x] = *ho.err_src;
    }
  }
  __syncthreads();
  // exclusive scan over the 3072 cells, three per thread (blockDim == 1024)
  const int a0 = s_cnt[3 * t], a1 = s_cnt[3 * t + 1], a2 = s_cnt[3 * t + 2];
  int excl = 0;
  const int tot = grid_block_scan_excl(a0 + a1 + a2, s_w, excl);
  s_cnt[3 * t] = excl;
  s_cnt[3 * t + 1] = excl + a0;
  s_cnt[3 * t + 2] = excl + a0 + a1;
  cell_start[3 * t] = excl;
  cell_start[3 * t + 1] = excl + a0;
  cell_start[3 * t + 2] = excl + a0 + a1;
  if (t == 0) cell_start[kGridCells] = tot;
  // cell c's list is [start(c), s_cnt[c]) once the scatter is done: keep the starts in registers
  const int b0 = excl, b1 = excl + a0, b2 = excl + a0 + a1;
  __syncthreads();
  int* list = LDS ? s_idx : cell_idx;
  for (int i = t; i < n; i += blockDim.x) {
    const int c = grid_cell(keys[i].x, keys[i].y, invW, invH);
    if (c >= 0) list[atomicAdd(&s_cnt[c], 1)] = i;
  }
  __threadfence_block();
  __syncthreads();
  // restore ascending key order inside each cell (cells hold a handful of keys)
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int b = k == 0 ? b0 : (k == 1 ? b1 : b2), e = s_cnt[3 * t + k];
    for (int p = b + 1; p < e; p++) {
      const int v = list[p];
      int q = p - 1;
      while (q >= b && list[q] > v) {
        list[q + 1] = list[q];
        q--;
      }
      list[q + 1] = v;
    }
  }
  if (LDS) {
    __syncthreads();
    for (int p = t; p < tot; p += blockDim.x) cell_idx[p] = s_idx[p];
  }
}

void launch_stereo_grid(const mmt_kp* keys, const int* nkp, int cap, const float* depth,
                        size_t depth_pitch, int W, int H, float bf, float invW, float invH,
                        float* uR, float* kdepth, int* cell_start, int* cell_idx, int nframes,
                        hipStream_t st, const B3HostOut* ho) {
  (void)H;
  if (nframes <= 0) return;
  B3HostOut h{};
  if (ho) h = *ho;
  const size_t lds = sizeof(int) * (size_t)cap;
  if (lds <= kStereoGridLds)
    hipLaunchKernelGGL(k_stereo_grid<true>, dim3(nframes), dim3(1024), lds, st, keys, nkp, cap,
                       depth, depth_pitch, W, bf, invW, invH, uR, kdepth, cell_start, cell_idx, h);
  else
    hipLaunchKernelGGL(k_stereo_grid<false>, dim3(nframes), dim3(1024), 0, st, keys, nkp, cap,
                       depth, depth_pitch, W, bf, invW, invH, uR, kdepth, cell_start, cell_idx, h);
  MMT_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------ windows
// GetFeaturesInArea's cell range (Frame.cc:711-729); false when the window is empty.
__device__ __forceinline__ bool window_cells(const GridFrame& G, float x, float y, float r,
                                             int& cx0, int& cx1, int& cy0, int& cy1) {
  // a non-finite centre (a map point unprojected from depth +inf) has no cells: the reference's
  // float -> int conversions are undefined there, x86 gives INT_MIN and an empty range
  if (!isfinite(x) || !isfinite(y)) return false;
  cx0 = max(0, (int)floorf((x - G.minX - r) * G.invW));
  if (cx0 >= kGridCols) return false;
  cx1 = min(kGridCols - 1, (int)ceilf((x - G.minX + r) * G.invW));
  if (cx1 < 0) return false;
  cy0 = max(0, (int)floorf((y - G.minY - r) * G.invH));
  if (cy0 >= kGridRows) return false;
  cy1 = min(kGridRows - 1, (int)ceilf((y - G.minY + r) * G.invH));
  if (cy1 < 0) return false;
  return true;
}

// Wave-cooperative candidate scan of one window (uniform arguments): enumerates the keys in
// GetFeaturesInArea order, applies the level / area / stereo filters (and `taken`, if given),
// computes the Hamming distance to `dmp` and keeps the K smallest (dist << 20 | order) keys.
// On return lanes 0..K-1 hold the sorted keys (kNoCand past the end) and key indices; the
// return value is the number of candidates that passed the filters.
struct NoneTaken {
  __device__ bool operator()(int) const { return false; }
};

template <int K, typename Taken>
__device__ int wave_topk(const GridFrame& G, const PointWin& w, const uint32_t (&dmp)[8],
                         const Taken& taken, uint32_t& top_key, int& top_idx) {
  const int lane = threadIdx.x & 63;
  top_key = kNoCand;
  top_idx = -1;
  int cx0, cx1, cy0, cy1;
  if (!window_cells(G, w.x, w.y, w.r, cx0, cx1, cy0, cy1)) return 0;
  const bool checkLevels = (w.minLevel > 0) || (w.maxLevel >= 0);
  // one column segment per lane: [cell_start[ix*48+cy0], cell_start[ix*48+cy1+1])
  const int nseg = cx1 - cx0 + 1;
  int sb = 0, sl = 0;
  if (lane < nseg) {
    const int base = (cx0 + lane) * kGridRows;
    sb = G.cell_start[base + cy0];
    sl = G.cell_start[base + cy1 + 1] - sb;
  }
  int pre = sl;  // inclusive prefix of the segment lengths
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(pre, o, 64);
    if (lane >= o) pre += y;
  }
  const int total = __shfl(pre, nseg - 1, 64);
  pre -= sl;  // exclusive
  int passed = 0;
  for (int p0 = 0; p0 < total; p0 += 64) {
    const int p = p0 + lane;
    uint32_t cv = kNoCand;
    int ci = -1;
    int s = 0;  // this position's column segment (shuffles with every lane active)
    for (int q = 1; q < nseg; q++) {
      const int pq = __shfl(pre, q, 64);
      if (pq <= p) s = q;
    }
    const int seg_b = __shfl(sb, s, 64), seg_p = __shfl(pre, s, 64);
    if (p < total) {
      const int k = G.cell_idx[seg_b + p - seg_p];
      const mmt_kp kp = G.keys[k];
      bool ok = true;
      if (checkLevels) {
        if (kp.octave < w.minLevel) ok = false;
        if (w.maxLevel >= 0 && kp.octave > w.maxLevel) ok = false;
      }
      if (ok) ok = fabsf(kp.x - w.x) < w.r && fabsf(kp.y - w.y) < w.r;
      if (ok) ok = !taken(k);
      if (ok) {
        const float ukr = G.uR[k];
        if (ukr > 0 && fabsf(w.ur - ukr) > w.er) ok = false;
      }
      if (ok) {
        const uint4* dk = reinterpret_cast<const uint4*>(G.desc + 32 * (size_t)k);
        const uint4 a = dk[0], b = dk[1];
        const int dist = __popc(a.x ^ dmp[0]) + __popc(a.y ^ dmp[1]) + __popc(a.z ^ dmp[2]) +
                         __popc(a.w ^ dmp[3]) + __popc(b.x ^ dmp[4]) + __popc(b.y ^ dmp[5]) +
                         __popc(b.z ^ dmp[6]) + __popc(b.w ^ dmp[7]);
        cv = ((uint32_t)dist << 20) | (uint32_t)p;
        ci = k;
      }
    }
    const unsigned long long vb = __ballot(cv != kNoCand);
    if (!vb) continue;
    passed += __popcll(vb);
    // merge the round into the running top-K (lanes 0..K-1)
    uint32_t a = cv, b = lane < K ? top_key : kNoCand;
    int ai = ci, bi = top_idx;
    uint32_t nk = kNoCand;
    int ni = -1;
    for (int r = 0; r < K; r++) {
      const uint32_t m = wave_min_u32(min(a, b));
      if (m == kNoCand) break;
      const bool own = (a == m) || (b == m);
      const int ol = __ffsll((long long)__ballot(own)) - 1;
      const int oi = __shfl(a == m ? ai : bi, ol, 64);
      if (own) {
        if (a == m) a = kNoCand;
        else b = kNoCand;
      }
      if (lane == r) {
        nk = m;
        ni = oi;
      }
    }
    top_key = nk;
    top_idx = ni;
  }
  return passed;
}

__device__ __forceinline__ void load_desc8(const uint8_t* d, uint32_t (&o)[8]) {
  const uint4* p = reinterpret_cast<const uint4*>(d);
  const uint4 a = p[0], b = p[1];
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

__device__ __forceinline__ void store_cands(const CandSet& cs, int i, int passed, uint32_t key,
                                            int idx, const PointWin& w) {
  const int lane = threadIdx.x & 63;
  if (lane < kCandK) {
    cs.key[(size_t)i * kCandK + lane] = key;
    cs.idx[(size_t)i * kCandK + lane] = idx;
  }
  if (lane == 0) {
    cs.n[i] = passed;
    cs.win[i] = w;
  }
}

// ------------------------------------------------------------------------------ C2 candidates
struct SbpArgs {
  GridFrame C;
  LastFrameDev L;
  float Tcw[16];
  float th;
  int mono;
  CandSet cs;
  const int* run_if;
  int run_lt;
};

__global__ __launch_bounds__(256) void k_sbp_frame(SbpArgs a) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= a.L.n) return;  // wave-uniform
  if (a.run_if && *a.run_if >= a.run_lt) return;
  const GridFrame& C = a.C;
  PointWin w = {};
  if (!a.L.active[i]) {
    store_cands(a.cs, i, -1, kNoCand, -1, w);
    return;
  }
  float twc[3], tlc[3], x3Dc[3];
  pose_centre(a.Tcw, twc);
  pose_xform(a.L.Tcw, twc, tlc);
  const float mb = C.bf / C.fx;
  const bool bForward = tlc[2] > mb && !a.mono;
  const bool bBackward = -tlc[2] > mb && !a.mono;
  pose_xform(a.Tcw, a.L.Xw + 3 * (size_t)i, x3Dc);
  const float invzc = (float)(1.0 / (double)x3Dc[2]);
  const float u = C.fx * x3Dc[0] * invzc + C.cx;
  const float v = C.fy * x3Dc[1] * invzc + C.cy;
  if (invzc < 0 || u < C.minX || u > C.maxX || v < C.minY || v > C.maxY) {
    store_cands(a.cs, i, 0, kNoCand, -1, w);
    return;
  }
  const int lo = a.L.keys[i].octave;
  w.x = u;
  w.y = v;
  w.r = a.th * C.scale[lo];
  w.ur = u - C.bf * invzc;
  w.er = w.r;
  if (bForward) {
    w.minLevel = lo;
    w.maxLevel = -1;
  } else if (bBackward) {
    w.minLevel = 0;
    w.maxLevel = lo;
  } else {
    w.minLevel = lo - 1;
    w.maxLevel = lo + 1;
  }
  uint32_t dmp[8];
  load_desc8(a.L.mp_desc + 32 * (size_t)i, dmp);
  uint32_t tk;
  int ti;
  const int passed = wave_topk<kCandK>(C, w, dmp, NoneTaken(), tk, ti);
  store_cands(a.cs, i, passed, tk, ti, w);
}

// ------------------------------------------------------------------------------ C3 candidates
struct LocalArgs {
  GridFrame C;
  float Tcw[16];
  const LocalPointDev* pts;
  const uint8_t* pdesc;
  int m;
  float th;
  FrustumRec* fr;
  CandSet cs;
  LocalSel sel;
};

__global__ __launch_bounds__(256) void k_local_cand(LocalArgs a) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= a.m) return;
  const int lane = threadIdx.x & 63;
  const GridFrame& C = a.C;
  const int pj = a.sel.ids ? a.sel.ids[j] : j;
  const LocalPointDev p = a.pts[pj];
  const bool skip = a.sel.skip ? a.sel.skip[j] != 0 : p.skip != 0;
  FrustumRec o = {0, 0, 0.f, 0.f, 0.f, 0.f};
  PointWin w = {};
  bool in = false;
  if (!skip) {
    // Frame::isInFrustum(pMP, 0.5)
    float Pc[3];
    pose_xform(a.Tcw, p.Xw, Pc);
    if (!(Pc[2] < 0.0f)) {
      const float invz = 1.0f / Pc[2];
      const float u = C.fx * Pc[0] * invz + C.cx;
      const float v = C.fy * Pc[1] * invz + C.cy;
      if (!(u < C.minX || u > C.maxX) && !(v < C.minY || v > C.maxY)) {
        const float maxDistance = 1.2f * p.max_dist;
        const float minDistance = 0.8f * p.min_dist;
        float Ow[3], PO[3];
        pose_centre(a.Tcw, Ow);
        double n2 = 0, dot = 0;
        for (int k = 0; k < 3; k++) {
          PO[k] = p.Xw[k] - Ow[k];
          n2 += (double)PO[k] * (double)PO[k];
        }
        const float dist = (float)sqrt(n2);
        if (!(dist < minDistance || dist > maxDistance)) {
          for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)p.normal[k];
          const float viewCos = (float)(dot / (double)dist);
          if (!(viewCos < 0.5f)) {
            const float ratio = p.max_dist / dist;
            // (int)ceil of a non-finite value (a NaN point): INT_MIN on x86 -> level 0
            const float ls = (float)log((double)ratio) / C.logScale;
            int nScale = isfinite(ls) ? (int)ceilf(ls) : INT_MIN;
            if (nScale < 0) nScale = 0;
            else if (nScale >= C.nlevels) nScale = C.nlevels - 1;
            o.in_view = 1;
            o.level = nScale;
            o.u = u;
            o.v = v;
            o.uR = u - C.bf * invz;
            o.view_cos = viewCos;
            in = true;
          }
        }
      }
    }
  }
  if (lane == 0) {
    if (a.fr) a.fr[j] = o;
    if (a.sel.inview) a.sel.inview[j] = (uint8_t)o.in_view;
  }
  if (!in) {
    store_cands(a.cs, j, -1, kNoCand, -1, w);
    return;
  }
  float r = ((double)o.view_cos > 0.998) ? 2.5f : 4.0f;  // RadiusByViewingCos
  if (a.th != 1.0f) r *= a.th;
  w.x = o.u;
  w.y = o.v;
  w.r = r * C.scale[o.level];
  w.ur = o.uR;
  w.er = w.r;
  w.minLevel = o.level - 1;
  w.maxLevel = o.level;
  uint32_t dmp[8];
  load_desc8(a.pdesc + 32 * (size_t)pj, dmp);
  uint32_t tk;
  int ti;
  const int passed = wave_topk<kCandK>(C, w, dmp, NoneTaken(), tk, ti);
  store_cands(a.cs, j, passed, tk, ti, w);
}

// ------------------------------------------------------------------------------ greedy replay
struct GreedyArgs {
  GridFrame C;
  int mode;  // 0: C2 (best only), 1: C3 (best + second-best ratio test)
  int npts;
  CandSet cs;
  const uint8_t* pdesc;      // npts x 32 point descriptors (rescans), or the pool with ids
  const int* ids;            // C3 pool indices (null: point j's descriptor is pdesc[j])
  const uint8_t* taken_in;   // C.n bytes or null
  const uint8_t* obs;        // C2: per point, its binding takes the key (null: all do)
  int check_orientation;
  const mmt_kp* lkeys;       // C2: last-frame keys (angles)
  int* match;                // C.n
  int* nmatches;
  const int* run_if;         // optional: run only while *run_if < run_lt
  int run_lt;
  int build_edges;           // D1's edge list from the final bindings (map_edges_body), in-kernel
  MapEdgeArgs edges;
};

// the decision of one point from its best / second-best unbound candidates
__device__ __forceinline__ int decide(const GreedyArgs& a, int best, int bestD, int sec,
                                      int secD) {
  if (best < 0 || bestD > TH_HIGH) return -1;
  if (a.mode == 0) return best;
  const int bestL = a.C.keys[best].octave;
  const int secL = sec >= 0 ? a.C.keys[sec].octave : -1;
  if (bestL == secL && (float)bestD > 0.8f * (float)secD) return -1;
  return best;
}

// C2's rotation bin of a binding event (ORBmatcher.cc:2064-2071): round() of the float product,
// only bins 0..12 are reachable (the reference's 1/30 factor on degrees)
__device__ __forceinline__ int rot_bin(float a_last, float a_cur) {
  float rot = a_last - a_cur;
  if (rot < 0.0f) rot += 360.0f;
  int bin = (int)roundf(rot * (1.0f / HISTO_LENGTH));
  if (bin == HISTO_LENGTH) bin = 0;
  return bin;
}

// Points bind in index order: point i takes its best (C3: best + second-best) candidate among
// the keys no earlier point has taken.  A binding by a point with observations takes its key for
// the points after it; one by a point without (a temporal VO point) leaves the key open, and a
// later point's binding replaces it (the key keeps the last binder).  Every binding is an event of
// C2's rotation histogram; an event in a rejected bin clears its key, whoever binds it last
// (ORBmatcher.cc:2087-2098).
//
// The sequential replay is the unique fixpoint of "every point's choice, given the choices of the
// points before it", so one 1024-thread workgroup iterates that map in parallel rounds:
//   1) owner[k] = the smallest index of a point whose current choice takes key k (LDS atomicMin;
//      -1 for keys bound before the call),
//   2) every point re-decides from its sorted candidates with "k taken" = owner[k] < i; a point
//      whose unbound choices run past its kCandK candidates is rescanned over its whole window by
//      a wave, with the same predicate,
// until a round changes nothing.  After round r the first r points hold their sequential choice
// (point 0 depends on nothing, point i only on points < i), so the loop ends within npts + 1
// rounds; conflicts between neighbouring points are short chains and it ends in a few.
constexpr int kFixThreads = 1024, kFixWaves = kFixThreads / 64, kFixResCap = 2048;

__device__ __forceinline__ int fix_decide_from_cands(const GreedyArgs& a, int i, const int* owner,
                                                     int cn, bool& resc) {
  int best = -1, bestD = 256, sec = -1, secD = 256;
  const int kk = min(cn, kCandK);
  for (int e = 0; e < kk; e++) {
    const int idx = a.cs.idx[(size_t)i * kCandK + e];
    if (owner[idx] < i) continue;
    const int d = (int)(a.cs.key[(size_t)i * kCandK + e] >> 20);
    if (best < 0) {
      best = idx;
      bestD = d;
      if (a.mode == 0) break;
    } else {
      sec = idx;
      secD = d;
      break;
    }
  }
  resc = cn > kCandK && (best < 0 || (a.mode == 1 && sec < 0));
  return resc ? -1 : decide(a, best, bestD, sec, secD);
}

struct OwnerTaken {
  const int* owner;
  int i;
  __device__ bool operator()(int k) const { return owner[k] < i; }
};

// A point with candidates, cached in LDS: its candidates packed (distance << 14 | key) in sorted
// order (0xFFFFFFFF past its count) and its index (bit 31: more candidates than cached, so it
// may need a rescan).  Rounds then read LDS only.
constexpr uint32_t kPackNone = 0xFFFFFFFFu;

// D1's edge list in key order (k_map_edges; also the tail of k_match_fix): a key with a new match
// takes its point's position, a key bound before the search its held position; nothing is built
// below min_matches (build false).  One 1024-thread workgroup; writes desc->n.
__device__ __forceinline__ void map_edges_body(const MapEdgeArgs& a, bool build, int* s_w) {
  const int t = threadIdx.x;
  int base = 0;
  for (int k0 = 0; k0 < (build ? a.n : 0); k0 += 1024) {
    const int i = k0 + t;
    int src = -1;  // 0: a new match, 1: a binding held before the search
    if (i < a.n) {
      if (a.match[i] >= 0)
        src = 0;
      else if (a.has_base && a.has_base[i])
        src = 1;
    }
    int excl = 0;
    const int tot = grid_block_scan_excl(src >= 0 ? 1 : 0, s_w, excl);
    if (src >= 0) {
      const int e = base + excl;
      const float* X;
      if (src == 1)
        X = a.base_X + 3 * (size_t)i;
      else if (a.pool)
        X = a.pool[a.ids[a.match[i]]].Xw;
      else
        X = a.src_X + 3 * (size_t)a.match[i];
      a.X[3 * e] = X[0];
      a.X[3 * e + 1] = X[1];
      a.X[3 * e + 2] = X[2];
      const mmt_kp kp = a.keys[i];
      a.obs[3 * e] = kp.x;
      a.obs[3 * e + 1] = kp.y;
      a.obs[3 * e + 2] = a.uR[i];
      a.s2[e] = a.inv_sigma2[kp.octave];
    }
    base += tot;
  }
  if (t == 0) a.desc->n = base;
}

__device__ __forceinline__ int fix_decide_packed(const GreedyArgs& a, int i, bool big,
                                                 const uint32_t* pc, const int* owner,
                                                 bool& resc) {
  int best = -1, bestD = 256, sec = -1, secD = 256;
#pragma unroll
  for (int e = 0; e < kCandK; e++) {
    const uint32_t v = pc[e];
    if (v == kPackNone) break;
    const int idx = (int)(v & 0x3FFFu);
    if (owner[idx] < i) continue;
    const int d = (int)(v >> 14);
    if (best < 0) {
      best = idx;
      bestD = d;
      if (a.mode == 0) break;
    } else {
      sec = idx;
      secD = d;
      break;
    }
  }
  resc = big && (best < 0 || (a.mode == 1 && sec < 0));
  return resc ? -1 : decide(a, best, bestD, sec, secD);
}

__global__ __launch_bounds__(kFixThreads) void k_match_fix(GreedyArgs a, int cache_cap) {
  extern __shared__ int s_owner[];  // C.n keys, then the cache of cache_cap points
  __shared__ int s_res[kFixResCap];
  __shared__ int s_hist[HISTO_LENGTH];
  __shared__ int s_ind[3];
  __shared__ int s_changed, s_nres, s_more, s_nm, s_removed, s_nact;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // every thread reads the condition before thread 0 may rewrite it (*nmatches, at the end)
  if (a.run_if && *a.run_if >= a.run_lt) return;
  const int n = a.C.n, np = a.npts;
  int* ch = a.cs.choice;
  int* s_pid = s_owner + ((n + 3) & ~3);
  uint32_t* s_cand = (uint32_t*)(s_pid + cache_cap);
  for (int k = tid; k < n; k += kFixThreads) {
    s_owner[k] = (a.taken_in && a.taken_in[k]) ? -1 : INT_MAX;
    a.match[k] = -1;
  }
  if (tid < HISTO_LENGTH) s_hist[tid] = 0;
  if (tid == 0) s_nact = 0;
  __syncthreads();
  // ---- the points with candidates go to the LDS cache (any order: every round decides every
  // point from the same owner table, so their order does not matter)
  for (int i = tid; i < np; i += kFixThreads) {
    ch[i] = -1;
    const int cn = a.cs.n[i];
    if (cn <= 0) continue;
    const int slot = atomicAdd(&s_nact, 1);
    if (slot >= cache_cap) continue;
    s_pid[slot] = cn > kCandK ? (int)((unsigned)i | 0x80000000u) : i;
    const int kk = min(cn, kCandK);
#pragma unroll
    for (int e = 0; e < kCandK; e++)
      s_cand[slot * kCandK + e] =
          e < kk ? ((a.cs.key[(size_t)i * kCandK + e] >> 20) << 14) |
                       (uint32_t)a.cs.idx[(size_t)i * kCandK + e]
                 : kPackNone;
  }
  __syncthreads();
  const bool cached = s_nact <= cache_cap;  // uniform: else every round reads the candidates
  const int nitems = cached ? s_nact : np;  // from global memory, point by point
#ifdef MMT_MATCH_PROFILE
  int prof_rounds = 0, prof_resc = 0;
  long long prof_t0 = clock64();
#endif
  for (int round = 0; round <= np + 1; round++) {
#ifdef MMT_MATCH_PROFILE
    prof_rounds++;
#endif
    if (tid == 0) {
      s_changed = 0;
      s_more = nitems;
    }
    if (round > 0) {
      for (int it = tid; it < nitems; it += kFixThreads) {
        const int i = cached ? (s_pid[it] & 0x7FFFFFFF) : it;
        const int c = ch[i];
        if (c >= 0 && (!a.obs || a.obs[i])) atomicMin(&s_owner[c], i);
      }
    }
    __syncthreads();
    // re-decide every point; rescans are queued (in passes of kFixResCap items)
    int from = 0;
    for (;;) {
      if (tid == 0) s_nres = 0;
      __syncthreads();
      int next = nitems;
      for (int it = from + tid; it < nitems; it += kFixThreads) {
        int i, t;
        bool resc;
        if (cached) {
          const int pid = s_pid[it];
          i = pid & 0x7FFFFFFF;
          t = fix_decide_packed(a, i, pid < 0, s_cand + it * kCandK, s_owner, resc);
        } else {
          i = it;
          const int cn = a.cs.n[i];
          if (cn <= 0) continue;
          t = fix_decide_from_cands(a, i, s_owner, cn, resc);
        }
        if (resc) {
          const int slot = atomicAdd(&s_nres, 1);
          if (slot < kFixResCap) {
            s_res[slot] = it;
          } else {
            next = min(next, it);  // no room: this item (and the ones after it) next pass
          }
          continue;
        }
        if (it >= next) continue;
        if (t != ch[i]) {
          ch[i] = t;
          s_changed = 1;
        }
      }
      // the pass covered items [from, cut): the smallest item that found no room starts the
      // next pass (items past it are re-decided then)
      if (next < nitems) atomicMin(&s_more, next);
      __syncthreads();
      const int cut = s_more;
      const int nres = min(s_nres, kFixResCap);
#ifdef MMT_MATCH_PROFILE
      prof_resc += nres;
#endif
      for (int r = wave; r < nres; r += kFixWaves) {
        const int it = s_res[r];
        if (it >= cut) continue;  // wave-uniform
        const int i = cached ? (s_pid[it] & 0x7FFFFFFF) : it;
        uint32_t dmp[8];
        load_desc8(a.pdesc + 32 * (size_t)(a.ids ? a.ids[i] : i), dmp);
        const PointWin w = a.cs.win[i];
        uint32_t tkey;
        int ti;
        wave_topk<2>(a.C, w, dmp, OwnerTaken{s_owner, i}, tkey, ti);
        const uint32_t k0 = __shfl((int)tkey, 0, 64), k1 = __shfl((int)tkey, 1, 64);
        const int i0 = __shfl(ti, 0, 64), i1 = __shfl(ti, 1, 64);
        const int t = decide(a, k0 != kNoCand ? i0 : -1, k0 != kNoCand ? (int)(k0 >> 20) : 256,
                             k1 != kNoCand ? i1 : -1, k1 != kNoCand ? (int)(k1 >> 20) : 256);
        if (lane == 0 && t != ch[i]) {
          ch[i] = t;
          s_changed = 1;
        }
      }
      __syncthreads();
      if (cut >= nitems) break;
      from = cut;
      __syncthreads();  // every thread has read s_more
      if (tid == 0) s_more = nitems;
    }
    if (!s_changed && round > 0) break;
    __syncthreads();  // every thread has read s_changed
    for (int k = tid; k < n; k += kFixThreads)
      if (s_owner[k] != -1) s_owner[k] = INT_MAX;
    __syncthreads();
  }
  // ---- bindings: the key keeps its last binder; nmatches counts every binding
  if (tid == 0) {
    s_nm = 0;
    s_removed = 0;
  }
  __syncthreads();
  int nm = 0;
  for (int i = tid; i < np; i += kFixThreads) {
    const int c = ch[i];
    if (c >= 0) {
      atomicMax(&a.match[c], i);
      nm++;
      if (a.mode == 0 && a.check_orientation)
        atomicAdd(&s_hist[rot_bin(a.lkeys[i].angle, a.C.keys[c].angle)], 1);
    }
  }
  atomicAdd(&s_nm, nm);
  __syncthreads();
  if (a.mode == 0 && a.check_orientation) {
    if (tid == 0) {
      int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
      for (int h = 0; h < HISTO_LENGTH; h++) {
        const int s = s_hist[h];
        if (s > max1) {
          max3 = max2; max2 = max1; max1 = s;
          ind3 = ind2; ind2 = ind1; ind1 = h;
        } else if (s > max2) {
          max3 = max2; max2 = s;
          ind3 = ind2; ind2 = h;
        } else if (s > max3) {
          max3 = s;
          ind3 = h;
        }
      }
      if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
      } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
      }
      s_ind[0] = ind1;
      s_ind[1] = ind2;
      s_ind[2] = ind3;
    }
    // s_owner becomes the flag of keys an event in a rejected bin clears
    for (int k = tid; k < n; k += kFixThreads) s_owner[k] = 0;
    __syncthreads();
    int removed = 0;
    for (int i = tid; i < np; i += kFixThreads) {
      const int k = ch[i];
      if (k >= 0) {
        const int bin = rot_bin(a.lkeys[i].angle, a.C.keys[k].angle);
        if (bin != s_ind[0] && bin != s_ind[1] && bin != s_ind[2]) {
          s_owner[k] = 1;
          removed++;
        }
      }
    }
    atomicAdd(&s_removed, removed);
    __syncthreads();
    for (int k = tid; k < n; k += kFixThreads)
      if (s_owner[k]) a.match[k] = -1;
  }
  if (tid == 0) *a.nmatches = s_nm - s_removed;
  if (a.build_edges) {
    __shared__ int s_we[16];
    __syncthreads();  // the final bindings (a.match) and the count
    map_edges_body(a.edges, s_nm - s_removed >= a.edges.min_matches, s_we);
  }
#ifdef MMT_MATCH_PROFILE
  if (tid == 0)
    printf("[match profile] mode %d npts %d keys %d rounds %d rescans %d cycles %lld\n", a.mode,
           np, n, prof_rounds, prof_resc, clock64() - prof_t0);
#endif
}

static void launch_match_fix(const GreedyArgs& g, hipStream_t st) {
  // dynamic LDS: the owner table (C.n keys, up to 64 KB) and the candidate cache (36 bytes per
  // point with candidates) in what is left of kFixLds
  constexpr int kFixLds = 150 * 1024;
  static std::atomic<uint64_t> attr_set{0};
  int dev = 0;
  MMT_HIP(hipGetDevice(&dev));
  const uint64_t bit = 1ull << (dev & 63);
  if (!(attr_set.load() & bit)) {
    MMT_HIP(hipFuncSetAttribute((const void*)k_match_fix,
                                hipFuncAttributeMaxDynamicSharedMemorySize, kFixLds));
    attr_set.fetch_or(bit);
  }
  const size_t owner = sizeof(int) * (size_t)((g.C.n + 3) & ~3);
  const int cap = std::min(g.npts, (int)((kFixLds - owner) / (sizeof(int) * (1 + kCandK))));
  const size_t lds = owner + sizeof(int) * (size_t)cap * (1 + kCandK);
  hipLaunchKernelGGL(k_match_fix, dim3(1), dim3(kFixThreads), lds, st, g, cap);
  MMT_HIP(hipGetLastError());
}

void launch_sbp_frame(const GridFrame& C, const float* Tcw, const LastFrameDev& L, float th,
                      int mono, int check_orientation, const CandSet& cs, int* match,
                      int* nmatches, hipStream_t st, const int* run_if, int run_lt,
                      const MapEdgeArgs* edges) {
  if (C.n > kMaxMatchKeys) throw ArgError("SearchByProjection: more than 16384 current keys");
  if (check_orientation && L.n > kMaxMatchKeys)
    throw ArgError("SearchByProjection: more than 16384 last-frame keys");
  SbpArgs a;
  a.C = C;
  a.L = L;
  for (int k = 0; k < 16; k++) a.Tcw[k] = Tcw[k];
  a.th = th;
  a.mono = mono;
  a.cs = cs;
  a.run_if = run_if;
  a.run_lt = run_lt;
  if (L.n > 0) {
    hipLaunchKernelGGL(k_sbp_frame, dim3((L.n + 3) / 4), dim3(256), 0, st, a);
    MMT_HIP(hipGetLastError());
  }
  GreedyArgs g;
  g.C = C;
  g.mode = 0;
  g.npts = L.n;
  g.cs = cs;
  g.pdesc = L.mp_desc;
  g.ids = nullptr;
  g.taken_in = nullptr;
  g.obs = L.obs;
  g.check_orientation = check_orientation;
  g.lkeys = L.keys;
  g.match = match;
  g.nmatches = nmatches;
  g.run_if = run_if;
  g.run_lt = run_lt;
  g.build_edges = edges != nullptr;
  if (edges) g.edges = *edges;
  launch_match_fix(g, st);
}

void launch_search_local(const GridFrame& C, const float* Tcw, const LocalPointDev* pts,
                         const uint8_t* pdesc, int m, float th, const uint8_t* taken,
                         FrustumRec* fr, const CandSet& cs, int* match, int* nmatches,
                         hipStream_t st, const LocalSel* sel, const MapEdgeArgs* edges) {
  if (C.n > kMaxMatchKeys) throw ArgError("SearchByProjection: more than 16384 current keys");
  LocalArgs a;
  a.C = C;
  for (int k = 0; k < 16; k++) a.Tcw[k] = Tcw[k];
  a.pts = pts;
  a.pdesc = pdesc;
  a.m = m;
  a.th = th;
  a.fr = fr;
  a.cs = cs;
  a.sel = sel ? *sel : LocalSel{nullptr, nullptr, nullptr};
  if (m > 0) {
    hipLaunchKernelGGL(k_local_cand, dim3((m + 3) / 4), dim3(256), 0, st, a);
    MMT_HIP(hipGetLastError());
  }
  GreedyArgs g;
  g.C = C;
  g.mode = 1;
  g.npts = m;
  g.cs = cs;
  g.pdesc = pdesc;
  g.ids = a.sel.ids;
  g.taken_in = taken;
  g.obs = nullptr;
  g.check_orientation = 0;
  g.lkeys = nullptr;
  g.match = match;
  g.nmatches = nmatches;
  g.run_if = nullptr;
  g.run_lt = 0;
  g.build_edges = edges != nullptr;
  if (edges) g.edges = *edges;
  launch_match_fix(g, st);
}

// ------------------------------------------------------------------------------ C4
// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) ORBmatcher.cc:532-663.  A frame feature belongs
// to one vocabulary node, so nodes never compete for features: one wave per keyframe node (its
// frame node found by binary search), the node's keyframe features replayed in list order.  Per
// keyframe feature the wave scores every unmatched frame feature of the node at once (lane =
// position, in chunks of 64), the best is the smallest (distance, position) key (the reference's
// strict '<' keeps the first of equal distances) and the second-best distance the smallest of the
// rest, accepted at TH_LOW and the ratio test; the winner's lane marks it matched.
static constexpr int TH_LOW = 50;  // ORBmatcher.cc:42

struct BowArgs {
  BowFeatVec kf, f;
  const mmt_kp* kf_keys;
  const uint8_t* kf_desc;
  const uint8_t* kf_ok;
  const mmt_kp* f_keys;
  const uint8_t* f_desc;
  int nF;
  float ratio;
  int check_orientation;
  int* match;
  int* hist;
  int* counters;
};

__global__ __launch_bounds__(256) void k_bow_nodes(BowArgs a) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= a.kf.n_nodes) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const uint32_t id = a.kf.node[k];
  int lo = 0, hi = a.f.n_nodes;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a.f.node[mid] < id)
      lo = mid + 1;
    else
      hi = mid;
  }
  if (lo >= a.f.n_nodes || a.f.node[lo] != id) return;
  const int fb = a.f.start[lo], fn = a.f.start[lo + 1] - fb;
  const int nch = (fn + 63) >> 6;  // <= 32 (host-checked)
  // this lane's frame features (positions lane + 64 c) and their descriptors stay in L1/L2; the
  // matched flags live in a register bitmask
  uint32_t taken = 0;
  int nm = 0;
  for (int q = a.kf.start[k]; q < a.kf.start[k + 1]; q++) {
    const int ikf = a.kf.feat[q];
    if (!a.kf_ok[ikf]) continue;  // pMP == NULL or isBad()
    uint32_t dk[8];
    load_desc8(a.kf_desc + 32 * (size_t)ikf, dk);
    uint32_t k1 = kNoCand;  // lane-local smallest (dist << 16 | position)
    int d2 = 256;           // lane-local second-smallest distance
    for (int c = 0; c < nch; c++) {
      const int p = lane + 64 * c;
      if (p >= fn || ((taken >> c) & 1u)) continue;
      uint32_t df[8];
      load_desc8(a.f_desc + 32 * (size_t)a.f.feat[fb + p], df);
      int dist = 0;
#pragma unroll
      for (int w = 0; w < 8; w++) dist += __popc(dk[w] ^ df[w]);
      const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)p;
      if (key < k1) {
        if (k1 != kNoCand) d2 = min(d2, (int)(k1 >> 16));
        k1 = key;
      } else {
        d2 = min(d2, dist);
      }
    }
    const uint32_t m1 = wave_min_u32(k1);
    if (m1 == kNoCand) continue;  // bestDist1 = 256 > TH_LOW
    const int c2 = k1 == m1 ? d2 : (k1 != kNoCand ? (int)(k1 >> 16) : 256);
    const int best2 = (int)wave_min_u32((uint32_t)c2);
    const int best1 = (int)(m1 >> 16);
    if (best1 > TH_LOW || !((float)best1 < a.ratio * (float)best2)) continue;
    const int p = (int)(m1 & 0xFFFFu);
    if (lane == (p & 63)) {
      taken |= 1u << (p >> 6);
      const int iF = a.f.feat[fb + p];
      a.match[iF] = ikf;
      if (a.check_orientation)
        atomicAdd(&a.hist[rot_bin(a.kf_keys[ikf].angle, a.f_keys[iF].angle)], 1);
    }
    nm++;
  }
  if (lane == 0 && nm) atomicAdd(&a.counters[0], nm);
}

// the rotation-consistency filter of SearchByBoW (ORBmatcher.cc:641-660) and nmatches
__global__ __launch_bounds__(256) void k_bow_rot(BowArgs a) {
  __shared__ int s_ind[3], s_removed;
  const int tid = threadIdx.x;
  if (tid == 0) {
    s_removed = 0;
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int h = 0; h < HISTO_LENGTH; h++) {
      const int s = a.check_orientation ? a.hist[h] : 0;
      if (s > max1) {
        max3 = max2; max2 = max1; max1 = s;
        ind3 = ind2; ind2 = ind1; ind1 = h;
      } else if (s > max2) {
        max3 = max2; max2 = s;
        ind3 = ind2; ind2 = h;
      } else if (s > max3) {
        max3 = s;
        ind3 = h;
      }
    }
    if (max2 < 0.1f * (float)max1) {
      ind2 = -1;
      ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
      ind3 = -1;
    }
    s_ind[0] = ind1;
    s_ind[1] = ind2;
    s_ind[2] = ind3;
  }
  __syncthreads();
  int removed = 0;
  if (a.check_orientation)
    for (int i = tid; i < a.nF; i += blockDim.x) {
      const int m = a.match[i];
      if (m < 0) continue;
      const int bin = rot_bin(a.kf_keys[m].angle, a.f_keys[i].angle);
      if (bin != s_ind[0] && bin != s_ind[1] && bin != s_ind[2]) {
        a.match[i] = -1;
        removed++;
      }
    }
  if (removed) atomicAdd(&s_removed, removed);
  __syncthreads();
  if (tid == 0) a.counters[1] = a.counters[0] - s_removed;
}

void launch_search_by_bow(const BowFeatVec& kf, const mmt_kp* kf_keys, const uint8_t* kf_desc,
                          const uint8_t* kf_ok, const BowFeatVec& f, const mmt_kp* f_keys,
                          const uint8_t* f_desc, int nF, float nnratio, int check_orientation,
                          int* match, int* hist, int* counters, hipStream_t st) {
  BowArgs a;
  a.kf = kf;
  a.f = f;
  a.kf_keys = kf_keys;
  a.kf_desc = kf_desc;
  a.kf_ok = kf_ok;
  a.f_keys = f_keys;
  a.f_desc = f_desc;
  a.nF = nF;
  a.ratio = nnratio;
  a.check_orientation = check_orientation;
  a.match = match;
  a.hist = hist;
  a.counters = counters;
  if (nF > 0) MMT_HIP(hipMemsetAsync(match, 0xFF, sizeof(int) * (size_t)nF, st));
  MMT_HIP(hipMemsetAsync(hist, 0, sizeof(int) * HISTO_LENGTH, st));
  MMT_HIP(hipMemsetAsync(counters, 0, sizeof(int) * 2, st));
  if (kf.n_nodes > 0 && f.n_nodes > 0) {
    hipLaunchKernelGGL(k_bow_nodes, dim3((kf.n_nodes + 3) / 4), dim3(256), 0, st, a);
    MMT_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_bow_rot, dim3(1), dim3(256), 0, st, a);
  MMT_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------ D1 edges
// One 1024-thread workgroup: order-preserving compaction of the bound keys, 1024 keys per step.
__global__ __launch_bounds__(1024) void k_map_edges(MapEdgeArgs a) {
  __shared__ int s_w[16];
  map_edges_body(a, !a.nm || *a.nm >= a.min_matches, s_w);
}

void launch_map_edges(const MapEdgeArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_map_edges, dim3(1), dim3(1024), 0, st, a);
  MMT_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------ pool
__global__ void k_pool_scatter(const PoolUpdate* __restrict__ up, int n, LocalPointDev* pool,
                               uint8_t* pool_desc) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const PoolUpdate u = up[t];
  pool[u.h] = u.p;
  uint4* d = reinterpret_cast<uint4*>(pool_desc + 32 * (size_t)u.h);
  const uint4* s = reinterpret_cast<const uint4*>(u.desc);
  d[0] = s[0];
  d[1] = s[1];
}

void launch_pool_scatter(const PoolUpdate* up, int n, LocalPointDev* pool, uint8_t* pool_desc,
                         hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pool_scatter, dim3((n + 255) / 256), dim3(256), 0, st, up, n, pool,
                     pool_desc);
  MMT_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------ Fuse candidates
// ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>, th) ORBmatcher.cc:1200-1324: the projection,
// image / distance / viewing-angle tests, PredictScale and the best key in the window (levels
// predicted - 1 .. predicted, the reprojection-error gate of stereo / monocular keys, the first of
// equal Hamming distances).  Everything here depends on the point and the keyframe only; what the
// match does to the map (AddObservation / MapPoint::Replace, order-dependent) is the host's.
// One wave per (keyframe, point) query.
struct FuseArgs {
  const FuseKF* kfs;
  const FuseQuery* q;
  int nq;
  const LocalPointDev* pool;
  const uint8_t* pool_desc;
  FuseCam cam;
  int2* out;
};

__global__ __launch_bounds__(256) void k_fuse_cand(FuseArgs a) {
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= a.nq) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const FuseQuery Q = a.q[qi];
  const FuseKF& K = a.kfs[Q.kft];
  const LocalPointDev p = a.pool[Q.h];
  const FuseCam& c = a.cam;
  int2 res = make_int2(-1, 256);
  float p3Dc[3];
  pose_xform(K.Tcw, p.Xw, p3Dc);
  bool ok = !(p3Dc[2] < 0.0f);
  float u = 0, v = 0, ur = 0, radius = 0;
  int npl = 0;
  if (ok) {
    const float invz = 1 / p3Dc[2];
    const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
    u = c.fx * x + c.cx;
    v = c.fy * y + c.cy;
    ok = u >= 0.f && u < c.W && v >= 0.f && v < c.H;  // KeyFrame::IsInImage
    if (ok) {
      ur = u - c.bf * invz;
      const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
      float PO[3];
      double n2 = 0;
      for (int k = 0; k < 3; k++) {
        PO[k] = p.Xw[k] - K.Ow[k];
        n2 += (double)PO[k] * (double)PO[k];
      }
      const float dist3D = (float)sqrt(n2);
      ok = !(dist3D < minDistance || dist3D > maxDistance);
      if (ok) {
        double dot = 0;
        for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)p.normal[k];
        ok = !(dot < 0.5 * (double)dist3D);  // viewing angle under 60 degrees
      }
      if (ok) {
        const float ratio = p.max_dist / dist3D;  // MapPoint::PredictScale(dist3D, pKF)
        const float ls = (float)log((double)ratio) / c.logScale;
        npl = isfinite(ls) ? (int)ceilf(ls) : INT_MIN;
        if (npl < 0) npl = 0;
        else if (npl >= c.nlevels) npl = c.nlevels - 1;
        radius = c.th * c.scale[npl];
      }
    }
  }
  int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
  if (ok && isfinite(u) && isfinite(v)) {  // KeyFrame::GetFeaturesInArea's cell range
    cx0 = max(0, (int)floorf((u - 0.f - radius) * c.invW));
    cx1 = min(kGridCols - 1, (int)ceilf((u - 0.f + radius) * c.invW));
    cy0 = max(0, (int)floorf((v - 0.f - radius) * c.invH));
    cy1 = min(kGridRows - 1, (int)ceilf((v - 0.f + radius) * c.invH));
    if (cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0) ok = false;
  } else {
    ok = false;
  }
  if (ok) {
    uint32_t dmp[8];
    load_desc8(a.pool_desc + 32 * (size_t)Q.h, dmp);
    const int nseg = cx1 - cx0 + 1;
    int sb = 0, sl = 0;
    if (lane < nseg) {
      const int base = (cx0 + lane) * kGridRows;
      sb = K.cell_start[base + cy0];
      sl = K.cell_start[base + cy1 + 1] - sb;
    }
    int pre = sl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(pre, o, 64);
      if (lane >= o) pre += y;
    }
    const int total = __shfl(pre, nseg - 1, 64);
    pre -= sl;
    uint32_t best = kNoCand;
    int bidx = -1;
    for (int p0 = 0; p0 < total; p0 += 64) {
      const int pp = p0 + lane;
      int s = 0;
      for (int q = 1; q < nseg; q++) {
        const int pq = __shfl(pre, q, 64);
        if (pq <= pp) s = q;
      }
      const int seg_b = __shfl(sb, s, 64), seg_p = __shfl(pre, s, 64);
      if (pp < total) {
        const int k = K.cell_idx[seg_b + pp - seg_p];
        const mmt_kp kp = K.keys[k];
        bool g = fabsf(kp.x - u) < radius && fabsf(kp.y - v) < radius;
        if (g) g = !(kp.octave < npl - 1 || kp.octave > npl);
        if (g) {
          const float ex = u - kp.x, ey = v - kp.y;
          const float kr = K.uR[k];
          if (kr >= 0) {
            const float er = ur - kr;
            const float e2 = ex * ex + ey * ey + er * er;
            g = !((double)(e2 * c.invSigma2[kp.octave]) > 7.8);
          } else {
            const float e2 = ex * ex + ey * ey;
            g = !((double)(e2 * c.invSigma2[kp.octave]) > 5.99);
          }
        }
        if (g) {
          const uint4* dk = reinterpret_cast<const uint4*>(K.desc + 32 * (size_t)k);
          const uint4 da = dk[0], db = dk[1];
          const int dist = __popc(da.x ^ dmp[0]) + __popc(da.y ^ dmp[1]) +
                           __popc(da.z ^ dmp[2]) + __popc(da.w ^ dmp[3]) +
                           __popc(db.x ^ dmp[4]) + __popc(db.y ^ dmp[5]) +
                           __popc(db.z ^ dmp[6]) + __popc(db.w ^ dmp[7]);
          const uint32_t key = ((uint32_t)dist << 20) | (uint32_t)pp;
          if (key < best) {
            best = key;
            bidx = k;
          }
        }
      }
    }
    const uint32_t m = wave_min_u32(best);
    if (m != kNoCand) {
      const int ol = __ffsll((long long)__ballot(best == m)) - 1;
      res = make_int2(__shfl(bidx, ol, 64), (int)(m >> 20));
    }
  }
  if (lane == 0) a.out[qi] = res;
}

void launch_fuse_cand(const FuseKF* kfs, const FuseQuery* q, int nq, const LocalPointDev* pool,
                      const uint8_t* pool_desc, const FuseCam& cam, int2* out, hipStream_t st) {
  if (nq <= 0) return;
  FuseArgs a{kfs, q, nq, pool, pool_desc, cam, out};
  hipLaunchKernelGGL(k_fuse_cand, dim3((nq + 3) / 4), dim3(256), 0, st, a);
  MMT_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------ relocalisation
// SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) (ORBmatcher.cc:2104-2231):
// one wave per keyframe map point (those not bad and not found, listed by the host): projection
// (no depth test, as the reference), image bounds, distance invariance, PredictScale, then the
// window's candidates in GetFeaturesInArea order with the level gate [p - 1, p + 1] and no stereo
// test (er = inf); keys bound when the call starts are skipped, the rest is the host's replay.
struct BoundKeys {
  const uint8_t* b;
  __device__ bool operator()(int k) const { return b[k] != 0; }
};

__global__ __launch_bounds__(256) void k_sbp_kf(SbpKfArgs a) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= a.m) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const GridFrame& C = a.C;
  const SbpKfPoint p = a.pts[j];
  float x3Dc[3];
  pose_xform(a.Tcw, p.Xw, x3Dc);
  const float invzc = (float)(1.0 / (double)x3Dc[2]);
  const float u = C.fx * x3Dc[0] * invzc + C.cx;
  const float v = C.fy * x3Dc[1] * invzc + C.cy;
  bool ok = !(u < C.minX || u > C.maxX) && !(v < C.minY || v > C.maxY);
  int npl = 0;
  if (ok) {
    float Ow[3];
    pose_centre(a.Tcw, Ow);
    double n2 = 0;
    for (int k = 0; k < 3; k++) {
      const float d = p.Xw[k] - Ow[k];
      n2 += (double)d * (double)d;
    }
    const float dist3D = (float)sqrt(n2);
    const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
    ok = !(dist3D < minDistance || dist3D > maxDistance);
    if (ok) {  // MapPoint::PredictScale(dist3D, &CurrentFrame)
      const float ratio = p.max_dist / dist3D;
      const float ls = (float)log((double)ratio) / C.logScale;
      npl = isfinite(ls) ? (int)ceilf(ls) : INT_MIN;
      if (npl < 0) npl = 0;
      else if (npl >= C.nlevels) npl = C.nlevels - 1;
    }
  }
  if (!ok) {
    if (lane < kSbpKfCand) {
      a.cand_key[(size_t)j * kSbpKfCand + lane] = kNoCand;
      a.cand_idx[(size_t)j * kSbpKfCand + lane] = -1;
    }
    if (lane == 0) a.n_cand[j] = -1;
    return;
  }
  PointWin w = {};
  w.x = u;
  w.y = v;
  w.r = a.th * C.scale[npl];
  w.ur = 0.f;
  w.er = INFINITY;
  w.minLevel = npl - 1;
  w.maxLevel = npl + 1;
  uint32_t dmp[8];
  load_desc8(p.desc, dmp);
  uint32_t tk;
  int ti;
  const int passed = wave_topk<kSbpKfCand>(C, w, dmp, BoundKeys{a.bound}, tk, ti);
  if (lane < kSbpKfCand) {
    a.cand_key[(size_t)j * kSbpKfCand + lane] = tk;
    a.cand_idx[(size_t)j * kSbpKfCand + lane] = ti;
  }
  if (lane == 0) {
    a.n_cand[j] = passed;
    a.win[j] = w;
  }
}

void launch_sbp_kf(const SbpKfArgs& a, hipStream_t st) {
  if (a.m <= 0) return;
  hipLaunchKernelGGL(k_sbp_kf, dim3((a.m + 3) / 4), dim3(256), 0, st, a);
  MMT_HIP(hipGetLastError());
}

}  // namespace mmt
