// multimot_track_amd/csrc/mmt_orb.hip -- batched, bit-exact ORB extraction for gfx950.
//
// Replaces ORBextractor::operator() (reference src/ORBextractor.cc:1046-1109).  Pipeline per
// batch of frames (every launch covers all frames of the batch):
//   k_resize x (nlevels-1)   ComputePyramid, cv::resize INTER_LINEAR fixed point   (:1111-1136)
//   k_fast                   per-cell FAST-9 + cell-local NMS + iniTh/minTh fallback (:765-829)
//   k_octree                 DistributeOctTree, data-parallel pass formulation      (:539-763)
//   k_blur                   GaussianBlur 7x7 sigma 2 bit-exact fixed point          (:1089-1090)
//   k_orient_desc            IC_Angle + rotated BRIEF + level-major assembly  (:77-147, :1079-1108)
// k_blur depends only on the pyramid; it is issued after k_octree on the same stream (a
// second stream would overlap it with FAST/octree).
//
// All arithmetic that feeds an output is integer, or fp32 with contraction disabled
// (-ffp-contract=off) and correctly rounded division, so results equal the CPU oracle bit for bit.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "mmt_internal.h"

namespace mmt {

static const int kEdge = 19;       // EDGE_THRESHOLD
static const int kMinBorder = 16;  // EDGE_THRESHOLD - 3

// bit_pattern_31_ (ORBextractor.cc:150-407), one int8 quadruple (x0, y0, x1, y1) per test
constexpr int kPatternRaw[1024] = {
#include "orb_pattern.inc"
};
struct PackedPattern {
  uint32_t t[256];
};
constexpr PackedPattern pack_pattern() {
  PackedPattern p{};
  for (int i = 0; i < 256; i++)
    p.t[i] = (uint32_t)(uint8_t)(int8_t)kPatternRaw[4 * i] |
             (uint32_t)(uint8_t)(int8_t)kPatternRaw[4 * i + 1] << 8 |
             (uint32_t)(uint8_t)(int8_t)kPatternRaw[4 * i + 2] << 16 |
             (uint32_t)(uint8_t)(int8_t)kPatternRaw[4 * i + 3] << 24;
  return p;
}
__constant__ PackedPattern c_pattern = pack_pattern();

static inline int host_round(float v) { return (int)lrintf(v); }
static inline int host_floor(float v) {
  int i = (int)v;
  return i - (i > v);
}
static inline int host_ceil(float v) {
  int i = (int)v;
  return i + (i < v);
}

void OrbTables::init(int nf, float scaleFactorF, int nl, int ini, int mn) {
  nfeatures = nf;
  nlevels = nl;
  iniTh = ini;
  minTh = mn;
  const double sf = (double)scaleFactorF;
  scale.assign(nl, 1.f);
  sigma2.assign(nl, 1.f);
  for (int i = 1; i < nl; i++) {
    scale[i] = (float)((double)scale[i - 1] * sf);
    sigma2[i] = scale[i] * scale[i];
  }
  invScale.resize(nl);
  invSigma2.resize(nl);
  for (int i = 0; i < nl; i++) {
    invScale[i] = 1.0f / scale[i];
    invSigma2[i] = 1.0f / sigma2[i];
  }
  nPerLevel.assign(nl, 0);
  const float factor = (float)(1.0f / sf);
  float nd = nf * (1 - factor) / (1 - (float)pow((double)factor, (double)nl));
  int sum = 0;
  for (int l = 0; l < nl - 1; l++) {
    nPerLevel[l] = host_round(nd);
    sum += nPerLevel[l];
    nd *= factor;
  }
  nPerLevel[nl - 1] = std::max(nf - sum, 0);
  umax.assign(16, 0);
  const int vmax = host_floor(15 * sqrtf(2.f) / 2 + 1), vmin = host_ceil(15 * sqrtf(2.f) / 2);
  const double hp2 = 225.0;
  int v, v0;
  for (v = 0; v <= vmax; ++v) umax[v] = (int)lrint(sqrt(hp2 - v * v));
  for (v = 15, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
}

// ======================================================================== kernels

// ---- pyramid level l from level l-1 (cv::resize INTER_LINEAR 8U, scalar fixed point) ----
// One workgroup per (band of kResizeRows output rows, 1024 output columns, frame).  The source
// rows and columns the band reads are staged once in LDS with coalesced dword loads; each thread
// then forms four adjacent outputs per row from LDS and stores them as one dword.
constexpr int kResizeRows = 8;
constexpr int kResizeCols = 1024;  // 256 threads x 4 columns
constexpr int kResizeStage = 16;   // staging dwords per thread issued together

__global__ __launch_bounds__(256) void k_resize(uint8_t* __restrict__ pyr, size_t pyr_stride,
                                                int src_off, int sw, int dst_off, int dw, int dh,
                                                const ResizeX* __restrict__ xt,
                                                const ResizeY* __restrict__ yt, int lds_pitch,
                                                int xcd_order) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rs_lds[];
  const int tid = threadIdx.x;
  // (column block, band, frame) from the workgroup index with contiguous runs per XCD (as
  // fast_job): vertically adjacent bands, which stage overlapping source rows, share an L2
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  {
    const int gx = gridDim.x, gy = gridDim.y, total = gx * gy * gridDim.z;
    if (xcd_order && (total & 7) == 0) {
      const int lin = (bz * gy + by) * gx + bx;
      const int j = (lin & 7) * (total >> 3) + (lin >> 3);
      bx = j % gx;
      by = (j / gx) % gy;
      bz = j / (gx * gy);
    }
  }
  uint8_t* base = pyr + (size_t)bz * pyr_stride;
  const uint8_t* src = base + src_off;
  const int dx0 = bx * kResizeCols, dx1 = min(dx0 + kResizeCols, dw);
  const int y0 = by * kResizeRows, y1 = min(y0 + kResizeRows, dh);
  // source window (sx and sy are non-decreasing in dx and dy)
  const int sx_lo = xt[dx0].sx, sx_hi = min(xt[dx1 - 1].sx + 1, sw - 1);
  const int sy_lo = yt[y0].sy0, sy_hi = yt[y1 - 1].sy1;
  const int nq = (sx_hi - sx_lo + 4) >> 2;  // dwords per staged row
  const int items = (sy_hi - sy_lo + 1) * nq;
  const float inv_nq = 1.0f / (float)nq;
  const uint8_t* s0 = src + (size_t)sy_lo * sw + sx_lo;
  // every staging load is issued before the first LDS store (one memory round trip per
  // workgroup; the source may be 3 bytes past a row end: next row, next level or slack)
  auto item_addr = [&](int i, int& lds_off) {
    int r = (int)((float)i * inv_nq);
    r -= (int)__umul24((unsigned)r, (unsigned)nq) > i ? 1 : 0;
    r += (int)__umul24((unsigned)(r + 1), (unsigned)nq) <= i ? 1 : 0;
    const int q = i - (int)__umul24((unsigned)r, (unsigned)nq);  // 24-bit multiplies: full rate
    lds_off = (int)__umul24((unsigned)r, (unsigned)lds_pitch) + 4 * q;
    return s0 + __umul24((unsigned)r, (unsigned)sw) + 4 * q;
  };
  uint32_t v[kResizeStage];
  int off[kResizeStage];
#pragma unroll
  for (int k = 0; k < kResizeStage; k++) {
    const int i = tid + 256 * k;
    if (i < items) __builtin_memcpy(&v[k], item_addr(i, off[k]), 4);
  }
  const int dx = dx0 + 4 * tid;
  ResizeX cx[4];
#pragma unroll
  for (int j = 0; j < 4; j++) cx[j] = xt[min(dx + j, dw - 1)];
  ResizeY cy[kResizeRows];
#pragma unroll
  for (int k = 0; k < kResizeRows; k++) cy[k] = yt[min(y0 + k, dh - 1)];
#pragma unroll
  for (int k = 0; k < kResizeStage; k++)
    if (tid + 256 * k < items) *(uint32_t*)(rs_lds + off[k]) = v[k];
  for (int i = tid + 256 * kResizeStage; i < items; i += 256) {  // wide windows only
    int o;
    uint32_t w;
    __builtin_memcpy(&w, item_addr(i, o), 4);
    *(uint32_t*)(rs_lds + o) = w;
  }
  __syncthreads();
  if (dx >= dx1) return;
  const int ncols = min(4, dx1 - dx);
  int lx[4];
#pragma unroll
  for (int j = 0; j < 4; j++) lx[j] = cx[j].sx - sx_lo;
#pragma unroll
  for (int k = 0; k < kResizeRows; k++) {
    const int y = y0 + k;
    if (y >= y1) break;
    const uint8_t* r0 = rs_lds + __umul24((unsigned)(cy[k].sy0 - sy_lo), (unsigned)lds_pitch);
    const uint8_t* r1 = rs_lds + __umul24((unsigned)(cy[k].sy1 - sy_lo), (unsigned)lds_pitch);
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      // a1 == 0 marks the clamped right edge (dx >= xmax): only S[sx]*2048 contributes (the
      // byte at sx+1 is then multiplied by 0; it lies inside the LDS row pitch)
      // 24-bit multiplies (full rate): |a|, |b| <= 2048, pixels <= 255, |h| < 2^20
      const int h0 = __mul24(r0[lx[j]], cx[j].a0) + __mul24(r0[lx[j] + 1], cx[j].a1);
      const int h1 = __mul24(r1[lx[j]], cx[j].a0) + __mul24(r1[lx[j] + 1], cx[j].a1);
      int v = (__mul24(cy[k].b0, h0) + __mul24(cy[k].b1, h1) + (1 << 21)) >> 22;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      packed |= (uint32_t)v << (8 * j);
    }
    uint8_t* dp = base + dst_off + (size_t)y * dw + dx;
    if (ncols == 4) {
      __builtin_memcpy(dp, &packed, 4);
    } else {
      for (int j = 0; j < ncols; j++) dp[j] = (uint8_t)(packed >> (8 * j));
    }
  }
}

// ---- the whole pyramid in one launch (levels 1.. from level 0, cv::resize as k_resize) ----
// One 1024-thread workgroup per (band of rows, frame): band b owns rows [h b / nb, h (b + 1) / nb)
// of every level and computes, level after level, its own rows plus the halo rows the next level's
// computed rows read (PyrBand, from the host's backward pass over the row tables), each level from
// the previous one in LDS (two alternating buffers), writing its own rows to the pyramid.  No
// workgroup waits for another, so the seven launches of the k_resize chain (each one memory round
// trip and a launch gap on the window's critical path) become one; halo rows are recomputed from
// the same bytes with the same arithmetic, so every level is bit-identical to the chain's.
constexpr int kPyrStage = 16;  // level-0 staging dwords per thread issued together

__global__ __launch_bounds__(1024) void k_pyramid(uint8_t* __restrict__ pyr, size_t pyr_stride,
                                                  const LevelInfo* __restrict__ lv,
                                                  const ResizeX* __restrict__ xt,
                                                  const ResizeY* __restrict__ yt,
                                                  const PyrBand* __restrict__ bands, PyrArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t py_lds[];
  const int tid = threadIdx.x, band = blockIdx.x, nb = gridDim.x;
  uint8_t* base = pyr + (size_t)blockIdx.y * pyr_stride;
  const PyrBand& B = bands[band];
  // the band's row coefficients of every level, staged in LDS after the two level buffers
  ResizeY* ylds = (ResizeY*)(py_lds + 2 * (size_t)a.buf_bytes);
  // thread -> (row offset, dword column) of a level whose rows hold nq dwords: rstep rows per pass
  auto lane_map = [&](int nq, int& q, int& rsub, int& rstep) {
    const float inv = 1.0f / (float)nq;
    rsub = (int)(((float)tid + 0.5f) * inv);  // exact: tid < 2^10, nq <= 1024
    q = tid - rsub * nq;
    rstep = (int)((1024.0f + 0.5f) * inv);
  };
  // this thread's four column coefficients of level l (issued a level ahead of their use)
  auto load_cx = [&](int l, ResizeX (&cx)[4]) {
    const LevelInfo D = lv[l];
    int q, rsub, rstep;
    lane_map((D.w + 3) >> 2, q, rsub, rstep);
    const ResizeX* X = xt + a.xoff[l];
#pragma unroll
    for (int j = 0; j < 4; j++) cx[j] = X[min(4 * q + j, D.w - 1)];
  };
  ResizeX cx[4];
  load_cx(1, cx);
  {  // level 0 rows of the band into buffer 0, the row coefficients into ylds: loads all in flight
    const LevelInfo L0 = lv[0];
    const int lo = B.lo[0], hi = B.hi[0], nq = (L0.w + 3) >> 2, pitch = a.pitch[0];
    int q, rsub, rstep;
    lane_map(nq, q, rsub, rstep);
    const bool act = rsub < rstep;
    // unconditional loads (rows clamped into the band): a load on a conditional path makes the
    // compiler drain every outstanding load where the paths join
    const int rs = act ? rsub : 0;
    const uint8_t* l0 = base + L0.off + 4 * q;
    uint32_t v[kPyrStage];
#pragma unroll
    for (int k = 0; k < kPyrStage; k++)  // may read <= 3 bytes past the row: next row / slack
      __builtin_memcpy(&v[k], l0 + (size_t)min(lo + rs + k * rstep, hi - 1) * L0.w, 4);
    int yo = 0;
    int ya[kPyrMaxLevels], yb[kPyrMaxLevels], yc[kPyrMaxLevels];  // ResizeY as three dwords
#pragma unroll
    for (int l = 1; l < kPyrMaxLevels; l++) {
      const int* yp = (const int*)(yt + a.yoff[l] + B.lo[l] +
                                   min(tid, max(B.hi[min(l, a.nl - 1)] - B.lo[l] - 1, 0)));
      ya[l] = l < a.nl ? yp[0] : 0;
      yb[l] = l < a.nl ? yp[1] : 0;
      yc[l] = l < a.nl ? yp[2] : 0;
    }
    uint8_t* lp = py_lds + rsub * pitch + 4 * q;
#pragma unroll
    for (int k = 0; k < kPyrStage; k++)
      if (act && lo + rsub + k * rstep < hi) *(uint32_t*)(lp + k * rstep * pitch) = v[k];
    for (int y = lo + rsub + kPyrStage * rstep; act && y < hi; y += rstep) {  // tall bands only
      uint32_t w;
      __builtin_memcpy(&w, base + L0.off + (size_t)y * L0.w + 4 * q, 4);
      *(uint32_t*)(py_lds + (y - lo) * pitch + 4 * q) = w;
    }
#pragma unroll
    for (int l = 1; l < kPyrMaxLevels; l++)
      if (l < a.nl) {
        const int n = B.hi[l] - B.lo[l];
        if (tid < n) {  // n <= 1024 (host)
          int* yd = (int*)(ylds + yo + tid);
          yd[0] = ya[l];
          yd[1] = yb[l];
          yd[2] = yc[l];
        }
        yo += n;
      }
  }
  __syncthreads();
  int ybase = 0;  // level l's rows start at ylds[ybase]
  for (int l = 1; l < a.nl; l++) {
    const LevelInfo D = lv[l];
    const uint8_t* src = py_lds + (size_t)((l - 1) & 1) * a.buf_bytes;
    uint8_t* dst = py_lds + (size_t)(l & 1) * a.buf_bytes;
    const int slo = B.lo[l - 1], spitch = a.pitch[l - 1], dpitch = a.pitch[l];
    const int lo = B.lo[l], hi = B.hi[l];
    const int own_lo = D.h * band / nb, own_hi = D.h * (band + 1) / nb;
    const bool keep = l + 1 < a.nl;  // the next level reads this one from LDS
    int q, rsub, rstep;
    lane_map((D.w + 3) >> 2, q, rsub, rstep);
    ResizeX cn[4];
    if (keep) load_cx(l + 1, cn);  // in flight during this level
    if (rsub < rstep && lo < hi) {
      const int dx = 4 * q, ncols = min(4, D.w - dx);
      const int sx0 = cx[0].sx;
      int lx[4];
#pragma unroll
      for (int j = 0; j < 4; j++) lx[j] = cx[j].sx - sx0;
      for (int y = lo + rsub; y < hi; y += rstep) {
        const ResizeY cy = ylds[ybase + y - lo];
        const uint8_t* r0 = src + __umul24((unsigned)(cy.sy0 - slo), (unsigned)spitch) + sx0;
        const uint8_t* r1 = src + __umul24((unsigned)(cy.sy1 - slo), (unsigned)spitch) + sx0;
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          // a1 == 0 marks the clamped right edge: the byte at sx + 1 (inside the row pitch) is
          // multiplied by 0.  24-bit multiplies as k_resize: |a|, |b| <= 2048, |h| < 2^20
          const int h0 = __mul24(r0[lx[j]], cx[j].a0) + __mul24(r0[lx[j] + 1], cx[j].a1);
          const int h1 = __mul24(r1[lx[j]], cx[j].a0) + __mul24(r1[lx[j] + 1], cx[j].a1);
          int v = (__mul24(cy.b0, h0) + __mul24(cy.b1, h1) + (1 << 21)) >> 22;
          v = v < 0 ? 0 : (v > 255 ? 255 : v);
          packed |= (uint32_t)v << (8 * j);
        }
        if (keep) *(uint32_t*)(dst + __umul24((unsigned)(y - lo), (unsigned)dpitch) + dx) = packed;
        if (y >= own_lo && y < own_hi) {
          uint8_t* dp = base + D.off + (size_t)y * D.w + dx;
          if (ncols == 4) {
            __builtin_memcpy(dp, &packed, 4);
          } else {
            for (int j = 0; j < ncols; j++) dp[j] = (uint8_t)(packed >> (8 * j));
          }
        }
      }
    }
    ybase += hi - lo;
    if (keep) {
#pragma unroll
      for (int j = 0; j < 4; j++) cx[j] = cn[j];
    }
    __syncthreads();
  }
}

// ---- FAST arc strength: max over 9-arcs of min(v - p) (dark) and min(p - v) (bright). ----
// A pixel is a FAST-9 corner at threshold t iff M > t, and OpenCV's cornerScore<16> returns
// M - 1 for every corner (derivation in DESIGN.md), so one M per pixel serves both thresholds.
typedef short short2v __attribute__((ext_vector_type(2)));

// LDS row stride of a FAST tile (template parameter FS): a compile-time constant, so every
// circle / compass / NMS neighbour read is one ds_read with an immediate offset from the pixel's
// address.  40 covers the ~31-pixel cells of any image (tile = cell + 6); 72 is the general case.
#ifndef MMT_FAST_FS
#define MMT_FAST_FS 40  // A/B builds: tools/ab_build.sh <tag> -DMMT_FAST_FS=..
#endif
constexpr int kFSSmall = MMT_FAST_FS, kFSMax = 72;
static_assert(kFSSmall % 4 == 0 && kFSSmall >= 40 && kFSSmall <= 128, "FAST tile stride");

// Circle differences as packed f16 pairs (v - q, q - v): every value is an integer of
// magnitude <= 255, exact in f16, and min / max are exact, so the result equals the integer
// formulation.  The pair comes from one v_pk_add_f16 (op_sel / neg modifiers on the scalar
// halves), the 9-arc minima from two rounds of 3-input v_pk_minimum3_f16 (arc k = d[k..k+2],
// d[k+3..k+5], d[k+6..k+8]) and the maximum over arcs from v_pk_maximum3_f16: about half the
// instructions of the 2-input integer min/max chain.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

template <int kFS>
__device__ __forceinline__ int arc_strength(const uint8_t* t) {
  const int off[16] = {3 * kFS,     3 * kFS + 1,  2 * kFS + 2,  kFS + 3,
                       3,           -kFS + 3,     -2 * kFS + 2, -3 * kFS + 1,
                       -3 * kFS,    -3 * kFS - 1, -2 * kFS - 2, -kFS - 3,
                       -3,          kFS - 3,      2 * kFS - 2,  3 * kFS - 1};
  const _Float16 v = (_Float16)(unsigned)t[0];
  h2v d[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const _Float16 q = (_Float16)(unsigned)t[off[k]];
    d[k] = (h2v){v, -v} + (h2v){-q, q};
  }
  h2v m3[16];
#pragma unroll
  for (int k = 0; k < 16; k++)
    m3[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(d[k], d[(k + 1) & 15]),
                                          d[(k + 2) & 15]);
  h2v mx[6];
#pragma unroll
  for (int j = 0; j < 6; j++) mx[j] = (h2v){(_Float16)-1000.f, (_Float16)-1000.f};
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const h2v mn9 = __builtin_elementwise_minimum(
        __builtin_elementwise_minimum(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
    mx[k % 6] = __builtin_elementwise_maximum(mx[k % 6], mn9);
  }
  const h2v b = __builtin_elementwise_maximum(
      __builtin_elementwise_maximum(__builtin_elementwise_maximum(mx[0], mx[1]), mx[2]),
      __builtin_elementwise_maximum(__builtin_elementwise_maximum(mx[3], mx[4]), mx[5]));
  return (int)(float)__builtin_elementwise_maximum(b.x, b.y);
}

// p -> (p / C, p % C) for p < 2^13, C <= 72: (p + 0.5) / C sits at least 0.5 / C away from an
// integer, far beyond the float error, so the truncation is exact
__device__ __forceinline__ int div_small(int p, float invC) {
  return (int)(((float)p + 0.5f) * invC);
}

__device__ __forceinline__ uint32_t ldg32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// Wave-level LDS ordering (no s_barrier): a wave's LDS writes are visible to its other lanes
// after this point.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP (row shifts within rows of 16, then
// the row broadcasts of GFX9): no LDS round trips.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Compass pre-test of four adjacent pixels at once (packed u16 halves, saturating arithmetic):
// is some pair of adjacent compass points (0/4/8/12) both darker or both brighter than the
// centre by more than th?  Adjacent pairs: (b0 && b4) || (b4 && b8) || (b8 && b12) || (b12 && b0)
// == (b0 || b8) && (b4 || b12).  sat(q - (v + th)) is nonzero iff q > v + th, sat((v - th) - q)
// nonzero iff q < v - th, so OR is bitwise or and AND is min of the saturated differences.
// c/dn/rt/up/lf hold the centre and the compass points 0 (down 3), 4 (right 3), 8 (up 3),
// 12 (left 3) of pixels 0..3 in bytes 0..3; returns the 4-bit mask of passing pixels.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

__device__ __forceinline__ uint32_t compass4(uint32_t c, uint32_t dn, uint32_t rt, uint32_t up,
                                             uint32_t lf, uint32_t th2) {
  uint32_t m = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t sel = h ? 0x0c030c01u : 0x0c020c00u;  // bytes (1, 3) or (0, 2) -> u16 halves
    const u16x2 v = as_u16x2(__builtin_amdgcn_perm(0u, c, sel));
    const u16x2 q0 = as_u16x2(__builtin_amdgcn_perm(0u, dn, sel));
    const u16x2 q4 = as_u16x2(__builtin_amdgcn_perm(0u, rt, sel));
    const u16x2 q8 = as_u16x2(__builtin_amdgcn_perm(0u, up, sel));
    const u16x2 q12 = as_u16x2(__builtin_amdgcn_perm(0u, lf, sel));
    const u16x2 t = as_u16x2(th2);
    const u16x2 hi = v + t, lo = __builtin_elementwise_sub_sat(v, t);
    const u16x2 br = __builtin_elementwise_min(
        __builtin_elementwise_sub_sat(q0, hi) | __builtin_elementwise_sub_sat(q8, hi),
        __builtin_elementwise_sub_sat(q4, hi) | __builtin_elementwise_sub_sat(q12, hi));
    const u16x2 dk = __builtin_elementwise_min(
        __builtin_elementwise_sub_sat(lo, q0) | __builtin_elementwise_sub_sat(lo, q8),
        __builtin_elementwise_sub_sat(lo, q4) | __builtin_elementwise_sub_sat(lo, q12));
    const u16x2 one = {1, 1};
    m |= __builtin_bit_cast(uint32_t, __builtin_elementwise_min(br | dk, one)) << h;
  }
  return (m & 3u) | ((m >> 14) & 0xCu);  // bits 0/1 (pixels 0, 1), 16/17 (pixels 2, 3)
}

// LDS bytes of one wave's FAST workspace: tile and arc-strength map (rows x kFS each) and the
// u16 candidate list (one entry per window pixel).
__host__ __device__ constexpr int fast_wave_lds(int kFS, int rows_max, int win_max) {
  return ((2 * rows_max * kFS + 2 * win_max) + 15) & ~15;
}

// Lane -> (row offset rsub, dword q) map of a cell's tile copy: one dword per lane per step, every
// step rps rows down, so the addresses advance by uniform strides (no per-item division and no
// quarter-rate 32-bit multiply).  src starts one byte before the tile (c0 >= 16; the pyramid
// allocation has slack for the <= 3 bytes read past the last row).
struct FastTileMap {
  const uint8_t* src;
  size_t sstep;
  int rps, rsub, q, act;  // act: the lane copies (an int: no padding bytes to move on a copy)
};

__device__ __forceinline__ FastTileMap fast_tile_map(const CellInfo& c, const LevelInfo& L,
                                                     const uint8_t* fbase, int lane) {
  FastTileMap m;
  const int nq = (c.cols + 4) >> 2;  // dwords per LDS row (tile shifted by 1)
  const float inv_nq = 1.0f / (float)nq;
  m.rps = __builtin_amdgcn_readfirstlane(div_small(64, inv_nq));  // rows per step
  m.rsub = div_small(lane, inv_nq);
  m.q = lane - (int)__umul24((unsigned)m.rsub, (unsigned)nq);
  m.act = m.rsub < m.rps;
  m.src = fbase + L.off + (size_t)c.r0 * L.w + c.c0 - 1 + 4 * m.q +
          __umul24((unsigned)m.rsub, (unsigned)L.w);
  m.sstep = (size_t)m.rps * L.w;
  return m;
}

constexpr int kFastStage = 6;  // tile row steps held in registers (36 rows of a <= 40-byte-wide tile)

__device__ __forceinline__ void fast_tile_fetch(const FastTileMap& m, int rows,
                                                uint32_t (&v)[kFastStage]) {
  const uint8_t* sp = m.src;
#pragma unroll
  for (int k = 0; k < kFastStage; k++, sp += m.sstep)
    if (m.act && m.rsub + k * m.rps < rows) v[k] = ldg32(sp);
}

template <int kFS>
__device__ __forceinline__ void fast_tile_store(const FastTileMap& m, int rows,
                                                const uint32_t (&v)[kFastStage], uint8_t* tile) {
  uint8_t* lp = tile + m.rsub * kFS + 4 * m.q;
  const int lstep = m.rps * kFS;
#pragma unroll
  for (int k = 0; k < kFastStage; k++, lp += lstep)
    if (m.act && m.rsub + k * m.rps < rows) *(uint32_t*)lp = v[k];
  // rows past the register stage (tall cells of wide tiles): copied here, synchronously
  const uint8_t* sp = m.src + kFastStage * m.sstep;
  for (int r = m.rsub + kFastStage * m.rps; m.act && r < rows; r += m.rps, sp += m.sstep, lp += lstep)
    *(uint32_t*)lp = ldg32(sp);
}

// Workgroup -> (cell group, frame): the hardware deals consecutive workgroups to the 8 XCDs in
// turn; this gives each XCD a contiguous run of (frame, cell group) jobs instead, so cells that
// share halo rows (vertical neighbours of one frame) meet in the same L2.
__device__ __forceinline__ void fast_job(int& xg, int& frame) {
  const int gx = gridDim.x, total = gx * gridDim.y;
  const int lin = blockIdx.y * gx + blockIdx.x;
  int j = lin;
  if ((total & 7) == 0) j = (lin & 7) * (total >> 3) + (lin >> 3);
  frame = j / gx;
  xg = j - frame * gx;
}

// One wave per cell at a time, four waves per workgroup; the grid's waves walk the cells of
// [cell_begin, cell_end) with a stride of one grid round (one cell per wave by default,
// MMT_FAST_CPW for more).  Cell = the submatrix the reference hands to cv::FAST (ORBextractor.cc:791-816).
// The wave stages the cell in its own LDS tile (row stride kFS, tile column c at LDS column c + 1
// so the detection window starts on a dword) and keeps an arc-strength map of the same shape, zero
// except at the candidates of the current pass, so out-of-window NMS neighbours read 0 without
// bounds checks.  With several cells per wave, the next cell's record and tile loads are issued
// before the current cell's passes and land in registers meanwhile.
// Per threshold (iniTh, then minTh if the cell came out empty, ORBextractor.cc:809-816):
//  1) compass pre-test at th over the window, four pixels per lane (one aligned dword of the
//     window row, packed u16 arithmetic): a 9-arc covers two adjacent compass points (0/4/8/12),
//     so a pixel whose pairs all fail has M <= th and is no corner; survivors are compacted in
//     row-major order (lanes are row-major groups of four pixels);
//  2) arc strength M of the candidates;
//  3) cell-local 3x3 strict NMS on scores s = (M > th ? M - 1 : 0) over the candidate list,
//     neighbours scored on the fly from the map; ballot compaction keeps row-major order.
// All wave-synchronous, so cells of different sizes never wait for each other.
template <int kFS>
__global__ __launch_bounds__(256) void k_fast(const uint8_t* __restrict__ pyr, size_t pyr_stride,
                                              const LevelInfo* __restrict__ lv,
                                              const CellInfo* __restrict__ cells, int ncells,
                                              uint32_t* __restrict__ keys, int total_slots,
                                              int* __restrict__ cellcnt, int iniTh, int minTh,
                                              int rows_max, int win_max, int cell_begin,
                                              int cell_end) {
  extern __shared__ __attribute__((aligned(16))) uint8_t fast_lds[];
#ifdef MMT_FAST_PROFILE
  long long fp_t = clock64(), fp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define FP_T(k) do { long long _n = clock64(); fp[k] += _n - fp_t; fp_t = _n; } while (0)
#else
#define FP_T(k) do {} while (0)
#endif
  const int lane = threadIdx.x & 63;
  // wave-uniform (readfirstlane): the cell record and everything derived from it live in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int xg, frame;
  fast_job(xg, frame);
  const int cstep = gridDim.x * 4;
  int cell = cell_begin + xg * 4 + wave;
  if (cell >= cell_end) return;
  uint8_t* tile = fast_lds + wave * fast_wave_lds(kFS, rows_max, win_max);
  uint8_t* arcm = tile + rows_max * kFS;
  uint16_t* cand_list = (uint16_t*)(arcm + rows_max * kFS);
  const uint8_t* fbase = pyr + (size_t)frame * pyr_stride;
  const uint32_t* t32 = (const uint32_t*)tile;
  constexpr int kRow32 = kFS / 4;  // dwords per LDS row
  const unsigned long long lt = (1ull << lane) - 1ull;
  CellInfo ci = cells[cell];
  FastTileMap tm = fast_tile_map(ci, lv[ci.level], fbase, lane);
  uint32_t v[kFastStage];
  fast_tile_fetch(tm, ci.rows, v);
  for (;;) {
    fast_tile_store<kFS>(tm, ci.rows, v, tile);
    for (int i = lane; i < ci.rows * (kFS / 4); i += 64) *(uint32_t*)(arcm + 4 * i) = 0u;
    wave_sync();
    // the next cell's record and tile: in flight during this cell's passes
    const int next = cell + cstep;
    const bool more = next < cell_end;
    CellInfo cn = ci;
    FastTileMap tn = tm;
    if (more) {
      cn = cells[next];
      tn = fast_tile_map(cn, lv[cn.level], fbase, lane);
      fast_tile_fetch(tn, cn.rows, v);
    }
    FP_T(0);
    const int R = ci.rows - 6, C = ci.cols - 6;  // detection window: tile rows 3..R+2, cols 3..C+2
    // pre-test lane mapping: gs groups of four pixels per row (power of two), 64 / gs rows per step
    const int G = (C + 3) >> 2, lgg = G <= 8 ? 3 : 4;
    const int grp = lane & ((1 << lgg) - 1), rsub = lane >> lgg, rstep = 64 >> lgg;
    const int nvalid = C - 4 * grp;  // window pixels of this lane's group
    const uint32_t colmask = grp < G ? (nvalid >= 4 ? 0xFu : (1u << nvalid) - 1u) : 0u;
    uint32_t* out = keys + (size_t)frame * total_slots + ci.slot_off;
    int count = 0, ncand = 0;
    for (int pass = 0; pass < 2; pass++) {
      const int th = min(max(pass == 0 ? iniTh : minTh, 0), 255);
      const uint32_t th2 = (uint32_t)th | ((uint32_t)th << 16);
      if (pass && minTh > iniTh) {  // pass 0's candidates are then no subset of pass 1's
        for (int i = lane; i < ci.rows * (kFS / 4); i += 64) *(uint32_t*)(arcm + 4 * i) = 0u;
        wave_sync();
      }
      // (with minTh <= iniTh, pass 0's candidates are pass 1's too and their arc strengths, which
      // do not depend on the threshold, stay valid in the map)
      ncand = 0;
      // two wave steps per iteration: the ten dword reads of both are in flight together
      for (int r0 = 0; r0 < R; r0 += 2 * rstep) {
        uint32_t m[2];
        int base[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const int wr = r0 + u * rstep + rsub;
          base[u] = (wr + 3) * kRow32 + 1 + grp;  // dword of window pixels 4 grp .. 4 grp + 3
          m[u] = 0;
          if (wr < R && colmask) {
            const int bb = base[u];
            const uint32_t c = t32[bb], cp = t32[bb - 1], cn4 = t32[bb + 1];
            const uint32_t up = t32[bb - 3 * kRow32], dn = t32[bb + 3 * kRow32];
            m[u] = compass4(c, dn, __builtin_amdgcn_alignbyte(cn4, c, 3), up,
                            __builtin_amdgcn_alignbyte(c, cp, 1), th2) & colmask;
          }
        }
        // candidates of step 0 precede those of step 1 (row-major): one scan of n0 + (n1 << 16)
        const int n0 = __popc(m[0]), n1 = __popc(m[1]);
        const int incl = wave_incl_scan(n0 | (n1 << 16));
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        int slot0 = ncand + (incl & 0xFFFF) - n0;
        int slot1 = ncand + (tot & 0xFFFF) + (incl >> 16) - n1;
        ncand += (tot & 0xFFFF) + (tot >> 16);
        uint32_t ma = m[0], mb = m[1];
        while (ma) {
          cand_list[slot0++] = (uint16_t)(4 * base[0] + __builtin_ctz(ma));
          ma &= ma - 1;
        }
        while (mb) {
          cand_list[slot1++] = (uint16_t)(4 * base[1] + __builtin_ctz(mb));
          mb &= mb - 1;
        }
      }
      wave_sync();
      FP_T(1 + 3 * pass);
      // arc strengths into the map; corners (M > th) are compacted in place at the front of the
      // candidate list (a write never passes the iteration's reads), keeping row-major order
      int ncorner = 0;
      for (int k0 = 0; k0 < ncand; k0 += 64) {
        const int k = k0 + lane;
        int p = 0, mm = 0;
        if (k < ncand) {
          p = cand_list[k];
          mm = arc_strength<kFS>(tile + p);
          arcm[p] = (uint8_t)(mm < 0 ? 0 : mm);
        }
        const bool corner = k < ncand && mm > th;
        const unsigned long long bc = __ballot(corner);
        if (corner) cand_list[ncorner + __popcll(bc & lt)] = (uint16_t)p;
        ncorner += __popcll(bc);
      }
      wave_sync();
      FP_T(2 + 3 * pass);
      int base = 0;
      for (int k0 = 0; k0 < ncorner; k0 += 64) {  // cell-local 3x3 NMS over the corners
        const int k = k0 + lane;
        bool keep = false;
        int sc = 0, p = 0;
        if (k < ncorner) {
          p = cand_list[k];
          const uint8_t* a = arcm + p;
          sc = a[0] - 1;
          const int n8[8] = {a[-kFS - 1], a[-kFS], a[-kFS + 1], a[-1],
                             a[1],        a[kFS - 1], a[kFS], a[kFS + 1]};
          int nmax = 0;
#pragma unroll
          for (int j = 0; j < 8; j++) nmax = max(nmax, n8[j] > th ? n8[j] - 1 : 0);
          keep = sc > nmax;
        }
        const unsigned long long bal = __ballot(keep);
        if (keep) {
          const int tr = p / kFS, tc = p - tr * kFS - 1;  // LDS column = tile column + 1
          const uint32_t x = (uint32_t)(ci.c0 - kMinBorder + tc);
          const uint32_t y = (uint32_t)(ci.r0 - kMinBorder + tr);
          const int slot = base + __popcll(bal & lt);
          if (slot < ci.slot_cap) out[slot] = (y << 20) | (x << 8) | (uint32_t)sc;
        }
        base += __popcll(bal);
      }
      count = base;
      FP_T(3 + 3 * pass);
#ifdef MMT_FAST_PROFILE
      fp[7] = ncand;
#endif
      if (count > 0) break;
      wave_sync();
    }
#ifdef MMT_FAST_PROFILE
    if (lane == 0 && frame == 0 && cell % 37 == 0)
      printf("fastprof cell %d lvl %d: copy %lld pre %lld arc %lld nms %lld | pass2 pre %lld arc %lld nms %lld | ncand %lld cnt %d\n",
             cell, ci.level, fp[0], fp[1], fp[2], fp[3], fp[4], fp[5], fp[6], fp[7], count);
    for (int k = 0; k < 8; k++) fp[k] = 0;
#endif
    if (lane == 0) cellcnt[(size_t)frame * ncells + cell] = min(count, ci.slot_cap);
    if (!more) break;
    // every lane is done with this cell's tile, map and candidates before the next store
    wave_sync();
    cell = next;
    ci = cn;
    tm = tn;
  }
}

// ---------------------------------------------------------------- octree helpers
// LDS arrays are typed as address-space-3 pointers so every access is a ds_* instruction, also
// through the double-buffered node arrays selected at run time.
#define LDS __attribute__((address_space(3)))
typedef LDS uint16_t lds_u16;
typedef LDS uint32_t lds_u32;
typedef LDS int lds_i32;
typedef LDS uint8_t lds_u8;
typedef LDS unsigned long long lds_u64;


// In-place exclusive scan of LDS ints a[0..n) by the whole workgroup; returns the total.  One
// barrier: wave totals go to one of two alternating LDS slots, every thread sums the ones before
// its wave.  Afterwards each thread has rewritten only its own items (the contiguous chunk
// [tid * per, tid * per + per)); with per == 1 these are the items a loop "for (i = tid; i < n;
// i += blockDim.x)" visits, so such a loop may read them without a barrier.  sync_after adds
// the barrier for callers that read other threads' items.
__device__ int wg_scan_excl(lds_i32* a, int n, lds_i32* s_tmp /*[2 * 16]*/, int& pp,
                            bool sync_after) {
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6;
  const int nw = nt >> 6;
  const int per = (n + nt - 1) / nt;
  const int b = min(tid * per, n), e = min(b + per, n);
  int local = 0;
  for (int i = b; i < e; i++) local += a[i];
  const int incl = wave_incl_scan(local);
  lds_i32* slot = s_tmp + 16 * pp;
  pp ^= 1;
  if (lane == 63) slot[wave] = incl;
  __syncthreads();
  int before = 0, total = 0;
  for (int w = 0; w < nw; w++) {
    const int t = slot[w];
    before += w < wave ? t : 0;
    total += t;
  }
  int run = before + incl - local;
  for (int i = b; i < e; i++) {
    const int t = a[i];
    a[i] = run;
    run += t;
  }
  if (sync_after || per > 1) __syncthreads();
  return total;
}

__device__ __forceinline__ uint32_t key_x(uint32_t k) { return (k >> 8) & 0xFFFu; }
__device__ __forceinline__ uint32_t key_y(uint32_t k) { return k >> 20; }
__device__ __forceinline__ uint32_t key_s(uint32_t k) { return k & 0xFFu; }

// Node arrays are double-buffered as two halves of one array (buffer c at offset c * nb): a
// run-time buffer index is then address arithmetic, not a pointer array in scratch memory.
struct OctLDS {
  lds_u16* x0;
  lds_u16* y0;
  lds_u16* x1;
  lds_u16* y1;
  lds_u32* cnt;
  lds_u32* seq;
  int nb;
  lds_i32* prank;
  lds_i32* order;
  lds_i32* gst;    // group start of processed rank r, later reused
  lds_i32* cumnc;  // exclusive prefix of child counts
  lds_u32* mid;    // aliases cumnc between steps A and B: split point (mx | my << 16) per rank
  lds_i32* krank;  // kept-node rank
  lds_u32* cc;     // 4 per processed rank (aliases sortkey / best / the gather's cell offsets)
  lds_u64* sortkey;
  lds_u32* best;
  lds_i32* s_tmp;  // [2 * 16] alternating wave-total slots of wg_scan_excl
  lds_i32* s_ctl;  // [4]
  int pp;          // next s_tmp slot (uniform across the workgroup)
};

// Per-key arrays of one (level, frame): gathered keys, key -> node, quadrant scratch.  In LDS
// when the level's keys fit, otherwise in global memory (KP/NP/QP are the pointer types).
template <typename KP, typename NP, typename QP>
struct OctKeys {
  KP lk;
  NP knode;
  QP kq;
};

// ---- division passes.  Node-level work (at most ncap nodes) runs on wave 0 alone, wave-
// synchronously (DPP scans, no barriers); key-level work (n keys) runs on every wave.  A pass is
//   [A: wave 0]   the nodes to divide, in processing order: order[r], prank[node] = r or -1
//   [B: all]      child counts per divided node (key quadrants, LDS atomics)
//   [C: wave 0]   children and the new node list (push_front order), the pass's results in ctl
//   [D: all]      key -> node in the new list
// with one barrier after each step.

// wave 0: in-place exclusive scan of a[0..n), lane-contiguous chunks; returns the total
__device__ int w0_scan_excl(lds_i32* a, int n) {
  const int lane = threadIdx.x & 63;
  const int per = (n + 63) >> 6;
  const int b = min(lane * per, n), e = min(b + per, n);
  int local = 0;
  for (int i = b; i < e; i++) local += a[i];
  const int incl = wave_incl_scan(local);
  const int total = __builtin_amdgcn_readlane(incl, 63);
  int run = incl - local;
  for (int i = b; i < e; i++) {
    const int t = a[i];
    a[i] = run;
    run += t;
  }
  wave_sync();
  return total;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

// atomicAdd(&a[key], 1) for every active lane with key != ~0u, one LDS atomic per run of equal
// keys in adjacent lanes: keys arrive in cell order, so equal nodes/quadrants sit next to each
// other, and the instruction count does not grow with the number of distinct keys (repeats of a
// key in separate runs just add separately).  Lanes outside the loop's exec mask count as ~0u.
__device__ __forceinline__ void wave_run_inc(lds_u32* a, uint32_t key) {
  const int lane = threadIdx.x & 63;
  // key of lane - 1 (wave_shr:1; lane 0 and lanes whose left neighbour is inactive read ~0u)
  const uint32_t prev =
      (uint32_t)__builtin_amdgcn_update_dpp((int)~0u, (int)key, 0x138, 0xF, 0xF, false);
  const bool valid = key != ~0u;
  const bool head = valid && (lane == 0 || prev != key);
  // run boundaries: heads and invalid lanes (inactive lanes read as set, ending every run)
  const unsigned long long bnd = __ballot(head || !valid) | ~__ballot(1);
  if (head) {
    const unsigned long long rest = lane < 63 ? bnd >> (lane + 1) : 0ull;
    const int len = rest ? __builtin_ctzll(rest) + 1 : 64 - lane;
    atomicAdd((uint32_t*)&a[key], (uint32_t)len);
  }
}

// split point of node nd of buffer c (ExtractorNode::DivideNode, ORBextractor.cc:481-486)
__device__ __forceinline__ uint32_t node_mid(const OctLDS& S, int c, int nd) {
  const int X0 = S.x0[(c) * S.nb + nd], Y0 = S.y0[(c) * S.nb + nd];
  const int mx = X0 + (int)ceilf((float)(S.x1[(c) * S.nb + nd] - X0) / 2.f);
  const int my = Y0 + (int)ceilf((float)(S.y1[(c) * S.nb + nd] - Y0) / 2.f);
  return (uint32_t)mx | ((uint32_t)my << 16);
}

// [A, phase 1, wave 0] nodes with cnt > 1 in list order into order[]; prank; zero their child
// counters.  Returns D.
__device__ int w0_expandable_in_order(OctLDS& S, int cur, int L) {
  const int lane = threadIdx.x & 63;
  for (int s = lane; s < L; s += 64) S.gst[s] = S.cnt[(cur) * S.nb + s] > 1 ? 1 : 0;
  wave_sync();
  const int D = w0_scan_excl(S.gst, L);
  for (int s = lane; s < L; s += 64) {
    if (S.cnt[(cur) * S.nb + s] > 1) {
      S.order[S.gst[s]] = s;
      S.prank[s] = S.gst[s];
      S.mid[S.gst[s]] = node_mid(S, cur, s);
    } else {
      S.prank[s] = -1;
    }
  }
  for (int i = lane; i < 4 * D; i += 64) S.cc[i] = 0;
  return D;
}

// [A, phase 2] expandable nodes sorted by (size, creation seq) descending (ORBextractor.cc:684
// sorts pair<size, ExtractorNode*> ascending and walks it backwards; pointer order is pinned to
// creation order).  Wave 0 compacts the keys, then every wave ranks them.
__device__ int oct_expandable_sorted(OctLDS& S, int cur, int L) {
  const int tid = threadIdx.x, nt = blockDim.x, wave = tid >> 6, lane = tid & 63;
  if (wave == 0) {
    for (int s = lane; s < L; s += 64) S.gst[s] = S.cnt[(cur) * S.nb + s] > 1 ? 1 : 0;
    wave_sync();
    const int D = w0_scan_excl(S.gst, L);
    for (int s = lane; s < L; s += 64) {
      if (S.cnt[(cur) * S.nb + s] > 1)
        S.sortkey[S.gst[s]] = ((unsigned long long)S.cnt[(cur) * S.nb + s] << 40) |
                              ((unsigned long long)(S.seq[(cur) * S.nb + s] & 0xFFFFFFu) << 16) |
                              (unsigned long long)s;
      S.prank[s] = -1;
    }
    if (lane == 0) {
      S.sortkey[D] = 0ull;  // pad to an even count (0 is below every key)
      S.s_ctl[3] = D;
    }
  }
  __syncthreads();
  const int D = S.s_ctl[3];
  // rank sort, descending: the keys are unique (node index in the low bits), so a key's rank is
  // the number of keys above it.  T adjacent lanes rank one key, each against an even-sized
  // slice of the keys (broadcast LDS reads, two keys per read), and add their counts with
  // shuffles: one barrier instead of a sorting network's log^2 steps, about D^2 / nt compares per
  // thread instead of D.
  int T = 1;
  while (T < 64 && D * (2 * T) <= nt) T *= 2;
  const int slice = (((D + 1) >> 1) + T - 1) / T * 2;  // keys per lane, even (sortkey[D] is 0)
  for (int base = tid; base < D * T; base += nt) {
    const int i = base / T, part = base & (T - 1);
    const unsigned long long k = S.sortkey[i];
    const int j0 = part * slice, j1 = min(j0 + slice, D + (D & 1));
    int rank = 0;
    for (int j = j0; j < j1; j += 2) rank += (S.sortkey[j] > k) + (S.sortkey[j + 1] > k);
    for (int o = T >> 1; o > 0; o >>= 1) rank += __shfl_xor(rank, o, 64);
    if (part == 0) {
      const int s = (int)(k & 0xFFFFull);
      S.order[rank] = s;
      S.prank[s] = rank;
      S.mid[rank] = node_mid(S, cur, s);
    }
  }
  __syncthreads();
  // cc aliases sortkey: zero the child counters only once every rank is done
  for (int i = tid; i < 4 * D; i += nt) S.cc[i] = 0;
  __syncthreads();
  return D;
}

// [B, all waves] child counts per divided node
template <typename KA>
__device__ __forceinline__ void oct_count_children(OctLDS& S, int c, const KA& kk, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t nd = kk.knode[i];
    const int r = S.prank[nd];
    uint32_t key = ~0u;
    if (r >= 0) {
      const uint32_t k = kk.lk[i], m = S.mid[r];
      const uint32_t mx = m & 0xFFFFu, my = m >> 16;
      const int q = (key_x(k) < mx) ? ((key_y(k) < my) ? 0 : 2) : ((key_y(k) < my) ? 1 : 3);
      kk.kq[i] = (uint8_t)q;
      key = (uint32_t)(r * 4 + q);
    }
    wave_run_inc(S.cc, key);
  }
}

// [C, wave 0] divide order[0..D) (children of the last processed node go to the front:
// std::list::push_front); every other node is kept.  With limitN > 0 (phase 2,
// ORBextractor.cc:730) the pass stops after the first node whose division makes the list size
// reach limitN.  Writes the new list into buffer c ^ 1 and ctl = {new size, nodes with more than
// one key, T = children created}.
__device__ void w0_divide(OctLDS& S, int c, int L, uint32_t seqBase, int D, int limitN) {
  const int lane = threadIdx.x & 63;
  for (int r = lane; r < D; r += 64) {
    int nc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) nc += S.cc[r * 4 + k] > 0;
    S.cumnc[r] = nc;
  }
  wave_sync();
  int Dt = D;
  if (limitN > 0) {
    for (int r = lane; r < D; r += 64) S.gst[r] = S.cumnc[r] - 1;
    wave_sync();
    w0_scan_excl(S.gst, D);
    int first = D;
    for (int r = lane; r < D; r += 64)
      if (L + S.gst[r] + S.cumnc[r] - 1 >= limitN) first = min(first, r + 1);
    Dt = wave_min(first);
  }
  for (int r = Dt + lane; r < D; r += 64) S.prank[S.order[r]] = -1;  // not divided this pass
  wave_sync();
  const int T = w0_scan_excl(S.cumnc, Dt);  // cumnc = sum_{q<r} nc
  for (int r = lane; r < Dt; r += 64) {
    int nc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) nc += S.cc[r * 4 + k] > 0;
    S.gst[r] = T - S.cumnc[r] - nc;  // sum_{q>r} nc
  }
  for (int s = lane; s < L; s += 64) S.krank[s] = S.prank[s] < 0 ? 1 : 0;
  wave_sync();
  const int K = w0_scan_excl(S.krank, L);
  const int o = c ^ 1;
  // new node list: processed children (n4..n1 per group, last group first), then kept nodes
  for (int r = lane; r < Dt; r += 64) {
    const int nd = S.order[r];
    const int X0 = S.x0[(c) * S.nb + nd], Y0 = S.y0[(c) * S.nb + nd], X1 = S.x1[(c) * S.nb + nd], Y1 = S.y1[(c) * S.nb + nd];
    const int mx = X0 + (int)ceilf((float)(X1 - X0) / 2.f);
    const int my = Y0 + (int)ceilf((float)(Y1 - Y0) / 2.f);
    const int rx0[4] = {X0, mx, X0, mx}, ry0[4] = {Y0, Y0, my, my};
    const int rx1[4] = {mx, X1, mx, X1}, ry1[4] = {my, my, Y1, Y1};
    uint32_t cnts[4];
#pragma unroll
    for (int k = 0; k < 4; k++) cnts[k] = S.cc[r * 4 + k];
    int before = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (!cnts[k]) continue;
      int after = 0;
#pragma unroll
      for (int k2 = k + 1; k2 < 4; k2++) after += cnts[k2] > 0;
      const int slot = S.gst[r] + after;
      S.cc[r * 4 + k] = (uint32_t)slot;  // child slot for step D (the counts are in cnts)
      S.x0[(o) * S.nb + slot] = (uint16_t)rx0[k];
      S.y0[(o) * S.nb + slot] = (uint16_t)ry0[k];
      S.x1[(o) * S.nb + slot] = (uint16_t)rx1[k];
      S.y1[(o) * S.nb + slot] = (uint16_t)ry1[k];
      S.cnt[(o) * S.nb + slot] = cnts[k];
      S.seq[(o) * S.nb + slot] = seqBase + (uint32_t)(S.cumnc[r] + before);
      before++;
    }
  }
  for (int s = lane; s < L; s += 64) {
    if (S.prank[s] < 0) {
      const int slot = T + S.krank[s];
      S.x0[(o) * S.nb + slot] = S.x0[(c) * S.nb + s];
      S.y0[(o) * S.nb + slot] = S.y0[(c) * S.nb + s];
      S.x1[(o) * S.nb + slot] = S.x1[(c) * S.nb + s];
      S.y1[(o) * S.nb + slot] = S.y1[(c) * S.nb + s];
      S.cnt[(o) * S.nb + slot] = S.cnt[(c) * S.nb + s];
      S.seq[(o) * S.nb + slot] = S.seq[(c) * S.nb + s];
    }
  }
  wave_sync();
  const int Ln = T + K;
  int e = 0;
  for (int s = lane; s < Ln; s += 64) e += S.cnt[(o) * S.nb + s] > 1 ? 1 : 0;
  e = wave_sum(e);
  if (lane == 0) {
    S.s_ctl[0] = Ln;
    S.s_ctl[1] = e;
    S.s_ctl[2] = T;
  }
}

// [D, all waves] key -> node in the new list
template <typename KA>
__device__ __forceinline__ void oct_relink_keys(OctLDS& S, const KA& kk, int n, int T) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t nd = kk.knode[i];
    const int r = S.prank[nd];
    if (r >= 0) {
      kk.knode[i] = (uint16_t)S.cc[r * 4 + kk.kq[i]];
    } else {
      kk.knode[i] = (uint16_t)(T + S.krank[nd]);
    }
  }
}

// One division pass over the D nodes selected by step A (already behind a barrier).  Updates the
// uniform list state of every thread; returns the number of nodes with more than one key.
#ifdef MMT_OCT_PROFILE
#define OP_T(k, t) do { long long _n = clock64(); g_op[k] += _n - t; t = _n; } while (0)
#define OP_PARAM , long long* g_op
#define OP_ARG , g_op
#else
#define OP_T(k, t) do {} while (0)
#define OP_PARAM
#define OP_ARG
#endif
#ifdef MMT_OCT_PROFILE
#define OP_DECL(t) long long t = clock64()
#define OP_SET(t) t = clock64()
#else
#define OP_DECL(t) do {} while (0)
#define OP_SET(t) do {} while (0)
#endif
template <typename KA>
__device__ __forceinline__ int oct_pass(OctLDS& S, int& cur, int& L, uint32_t& seqBase, int D,
                                        int limitN, const KA& kk, int n OP_PARAM) {
  OP_DECL(t);
  oct_count_children(S, cur, kk, n);
  __syncthreads();
  OP_T(0, t);
  if ((threadIdx.x >> 6) == 0) w0_divide(S, cur, L, seqBase, D, limitN);
  __syncthreads();
  OP_T(1, t);
  const int Ln = S.s_ctl[0], nexp = S.s_ctl[1], T = S.s_ctl[2];
  oct_relink_keys(S, kk, n, T);
  __syncthreads();
  OP_T(2, t);
  cur ^= 1;
  L = Ln;
  seqBase += (uint32_t)T;
  return nexp;
}

// LDS layout of k_octree: node arrays (ncap nodes, double-buffered where the passes alternate),
// then the per-key arrays of up to kcap keys.  The kernel carves exactly these offsets and the
// host sizes the launch from `end`, so the two cannot drift apart.
struct OctLayout {
  uint32_t x0, y0, x1, y1, cnt, seq, prank, order, gst, cumnc, krank, cc, tmp, lk, knode, kq, end;
};
__host__ __device__ inline OctLayout oct_layout(int ncap, int kcap) {
  OctLayout o{};
  uint32_t p = 0;
  auto take = [&](uint32_t bytes) {
    const uint32_t r = p;
    p += (bytes + 15u) & ~15u;
    return r;
  };
  o.x0 = take(2 * 2 * ncap);
  o.y0 = take(2 * 2 * ncap);
  o.x1 = take(2 * 2 * ncap);
  o.y1 = take(2 * 2 * ncap);
  o.cnt = take(2 * 4 * ncap);
  o.seq = take(2 * 4 * ncap);
  o.prank = take(4 * ncap);
  o.order = take(4 * ncap);
  o.gst = take(4 * ncap);
  o.cumnc = take(4 * ncap);
  o.krank = take(4 * ncap);
  o.cc = take(16 * ncap);
  o.tmp = take(4 * 36);  // s_tmp [2 * 16] + s_ctl [4]
  o.lk = take(4 * kcap);
  o.knode = take(2 * kcap);
  o.kq = take(kcap);
  o.end = p;
  return o;
}

// Gather of the level's FAST candidates in cell order (cells hold them row-major), then
// DistributeOctTree (ORBextractor.cc:539-763) and the best key per node.
template <typename KA>
__device__ __forceinline__ void oct_run(OctLDS& S, const KA& kk, const LevelInfo& L0,
                                        const CellInfo* __restrict__ cells, const int* cnt,
                                        int nc, const uint32_t* __restrict__ fk, int n,
                                        uint32_t* __restrict__ outp, int* __restrict__ ocount_p,
                                        int ncap, int* __restrict__ err) {
  const int tid = threadIdx.x, nt = blockDim.x;
  // thread per key: its cell is the last one whose offset is <= the key index
#ifdef MMT_OCT_PROFILE
  long long g_op[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  OP_DECL(tq);
  // cell of every key: one thread per cell marks its key range (knode as scratch), and the
  // cell's slot base minus its key offset goes next to the offsets when it fits
  lds_i32* coff = (lds_i32*)S.cc;
  const bool lds_base = 2 * nc <= 4 * ncap;
  for (int c = tid; c < nc; c += nt) {
    const int b = coff[c], e = c + 1 < nc ? coff[c + 1] : n;
    for (int i = b; i < e; i++) kk.knode[i] = (uint16_t)c;
    if (lds_base) coff[nc + c] = cells[L0.cell_begin + c].slot_off - b;
  }
  __syncthreads();
  for (int i0 = tid; i0 < n; i0 += 4 * nt) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = i0 + u * nt;
      if (i < n) {
        const int c = kk.knode[i];
        const int base = lds_base ? coff[nc + c] : cells[L0.cell_begin + c].slot_off - coff[c];
        v[u] = fk[base + i];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (i0 + u * nt < n) kk.lk[i0 + u * nt] = v[u];
  }
  __syncthreads();
  OP_T(3, tq);
#ifdef MMT_OCT_PROFILE
  long long tp0 = clock64(), tsort = 0, tpass = 0, tmain = 0;
  int npass1 = 0, npass2 = 0;
#endif
  // ---- initial nodes (ORBextractor.cc:552-585)
  const int nIni = L0.nIni;
  const float hX = L0.hX;
  const int H = (L0.h - kEdge + 3) - kMinBorder;  // maxBorderY - minBorderY
  for (int i = tid; i < nIni; i += nt) S.cnt[(0) * S.nb + i] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += nt) {
    const int idx = (int)((float)key_x(kk.lk[i]) / hX);
    kk.knode[i] = (uint16_t)idx;
    wave_run_inc(S.cnt, (uint32_t)idx);
  }
  __syncthreads();
  for (int i = tid; i < nIni; i += nt) S.krank[i] = S.cnt[(0) * S.nb + i] > 0 ? 1 : 0;
  __syncthreads();
  int Lsz = wg_scan_excl(S.krank, nIni, S.s_tmp, S.pp, false);
  for (int i = tid; i < nIni; i += nt) {
    if (S.cnt[(0) * S.nb + i] > 0) {
      const int s = S.krank[i];
      S.x0[(1) * S.nb + s] = (uint16_t)(int)(hX * (float)i);
      S.x1[(1) * S.nb + s] = (uint16_t)(int)(hX * (float)(i + 1));
      S.y0[(1) * S.nb + s] = 0;
      S.y1[(1) * S.nb + s] = (uint16_t)H;
      S.cnt[(1) * S.nb + s] = S.cnt[(0) * S.nb + i];
      S.seq[(1) * S.nb + s] = (uint32_t)i;
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += nt) kk.knode[i] = (uint16_t)S.krank[kk.knode[i]];
  __syncthreads();
  OP_T(4, tq);
  int cur = 1;
  uint32_t seqBase = (uint32_t)nIni;
  const int N = L0.N;
  // ---- main loop (ORBextractor.cc:594-739)
  bool finish = false;
  int guard = 0;
  while (!finish) {
    if (++guard > 4096) {
      if (tid == 0) atomicOr(err, 1);
      break;
    }
    const int prevSize = Lsz;
#ifdef MMT_OCT_PROFILE
    long long ta = clock64();
    npass1++;
#endif
    if ((tid >> 6) == 0) {
      const int D = w0_expandable_in_order(S, cur, Lsz);
      if ((tid & 63) == 0) S.s_ctl[3] = D;
    }
    __syncthreads();
    const int D = S.s_ctl[3];
    const int nToExpand = oct_pass(S, cur, Lsz, seqBase, D, 0, kk, n OP_ARG);
#ifdef MMT_OCT_PROFILE
    tmain += clock64() - ta;
#endif
    if (Lsz >= N || Lsz == prevSize) {
      finish = true;
    } else if (Lsz + nToExpand * 3 > N) {
      while (!finish) {
        if (++guard > 4096) {
          if (tid == 0) atomicOr(err, 1);
          finish = true;
          break;
        }
        const int prev2 = Lsz;
#ifdef MMT_OCT_PROFILE
        long long tb = clock64();
        npass2++;
#endif
        const int D2 = oct_expandable_sorted(S, cur, Lsz);
#ifdef MMT_OCT_PROFILE
        long long tc = clock64();
        tsort += tc - tb;
#endif
        oct_pass(S, cur, Lsz, seqBase, D2, N, kk, n OP_ARG);
#ifdef MMT_OCT_PROFILE
        tpass += clock64() - tc;
#endif
        if (Lsz >= N || Lsz == prev2) finish = true;
      }
    }
    if (Lsz + 4 > ncap) {  // capacity guard (cannot happen for N + 8 <= ncap)
      if (tid == 0) atomicOr(err, 2);
      finish = true;
    }
  }
  // ---- retain the best key per node: max response, first in key order (:744-760)
  OP_SET(tq);
  for (int s = tid; s < Lsz; s += nt) S.best[s] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += nt)
    atomicMax((uint32_t*)&S.best[kk.knode[i]], (key_s(kk.lk[i]) << 24) | (0xFFFFFFu - (uint32_t)i));
  __syncthreads();
  const int nout = min(Lsz, L0.out_cap);
  for (int s = tid; s < nout; s += nt) {
    const uint32_t i = 0xFFFFFFu - (S.best[s] & 0xFFFFFFu);
    const uint32_t k = kk.lk[i];
    const uint32_t x = key_x(k) + kMinBorder, y = key_y(k) + kMinBorder;
    outp[s] = (y << 20) | (x << 8) | key_s(k);
  }
  OP_T(5, tq);
#ifdef MMT_OCT_PROFILE
  if (tid == 0 && blockIdx.y == 0 && blockIdx.x == 0)
    printf("steps count=%lld divide=%lld relink=%lld gather=%lld init=%lld best=%lld\n", g_op[0], g_op[1], g_op[2], g_op[3], g_op[4], g_op[5]);
  if (tid == 0 && blockIdx.y == 0)
    printf("octprof level=%d n=%d N=%d L=%d total=%lld main=%lld (%d passes) sort=%lld pass2=%lld (%d)\n",
           L0.out_off, n, N, Lsz, clock64() - tp0, tmain, npass1, tsort, tpass, npass2);
#endif
  if (tid == 0) {
    *ocount_p = nout;
    if (Lsz > L0.out_cap) atomicOr(err, 4);
  }
}

// One workgroup per (frame, level), dispatched level-major.  Keys of the level live in LDS when at most kcap of them
// survived FAST (the usual case), in global scratch otherwise.
// kWaves: minimum waves per SIMD the register allocation must allow.  8 (at most 64 VGPRs) lets
// two 1024-thread workgroups share a CU when their LDS fits in half of it (the launch of levels
// 1.., whose key counts are small); 1 leaves the allocation unconstrained (level 0).
template <int kWaves>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(kWaves))) void k_octree(
                                                 const LevelInfo* __restrict__ lv,
                                                 const CellInfo* __restrict__ cells, int ncells,
                                                 const uint32_t* __restrict__ keys,
                                                 const int* __restrict__ cellcnt, int total_slots,
                                                 uint32_t* __restrict__ lkeys,
                                                 uint32_t* __restrict__ knode_g,
                                                 uint8_t* __restrict__ kq_g,
                                                 uint32_t* __restrict__ okeys, int out_slots,
                                                 int* __restrict__ ocount, int nlevels,
                                                 int ncap, int kcap, int level_begin,
                                                 int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_generic[];
  LDS unsigned char* smem = (LDS unsigned char*)smem_generic;
  // frames along x: workgroups are dispatched level-major, the heavy low levels first, so the
  // light levels fill in behind them instead of heavy workgroups trailing at the end
  const int level = level_begin + blockIdx.y, frame = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const LevelInfo L0 = lv[level];
  // ---- carve LDS (oct_layout: the same offsets the host sized the launch with)
  const OctLayout ly = oct_layout(ncap, kcap);
  OctLDS S;
  S.nb = ncap;
  S.x0 = (lds_u16*)(smem + ly.x0);
  S.y0 = (lds_u16*)(smem + ly.y0);
  S.x1 = (lds_u16*)(smem + ly.x1);
  S.y1 = (lds_u16*)(smem + ly.y1);
  S.cnt = (lds_u32*)(smem + ly.cnt);
  S.seq = (lds_u32*)(smem + ly.seq);
  S.prank = (lds_i32*)(smem + ly.prank);
  S.order = (lds_i32*)(smem + ly.order);
  S.gst = (lds_i32*)(smem + ly.gst);
  S.cumnc = (lds_i32*)(smem + ly.cumnc);
  S.mid = (lds_u32*)S.cumnc;
  S.krank = (lds_i32*)(smem + ly.krank);
  S.cc = (lds_u32*)(smem + ly.cc);
  S.sortkey = (lds_u64*)S.cc;
  S.best = S.cc;
  S.s_tmp = (lds_i32*)(smem + ly.tmp);
  S.s_ctl = S.s_tmp + 32;
  S.pp = 0;
  lds_u32* k_lk = (lds_u32*)(smem + ly.lk);
  lds_u16* k_node = (lds_u16*)(smem + ly.knode);
  lds_u8* k_q = (lds_u8*)(smem + ly.kq);

  // ---- cell offsets of this level's candidates
  const int nc = L0.cell_end - L0.cell_begin;
  const int* cnt = cellcnt + (size_t)frame * ncells + L0.cell_begin;
  lds_i32* coff = (lds_i32*)S.cc;  // scratch (nc <= 4 * ncap checked on host)
  for (int i = tid; i < nc; i += nt) coff[i] = cnt[i];
  __syncthreads();
  const int n = wg_scan_excl(coff, nc, S.s_tmp, S.pp, true);
  uint32_t* outp = okeys + (size_t)frame * out_slots + L0.out_off;
  int* ocount_p = ocount + frame * nlevels + level;
  if (n == 0) {
    if (tid == 0) *ocount_p = 0;
    return;
  }
  const uint32_t* fk = keys + (size_t)frame * total_slots;
  if (n <= kcap) {
    OctKeys<lds_u32*, lds_u16*, lds_u8*> kk{k_lk, k_node, k_q};
    oct_run(S, kk, L0, cells, cnt, nc, fk, n, outp, ocount_p, ncap, err);
  } else {
    // global scratch: knode as u16 in the u32 slots, quadrant bytes after all frames' knode
    uint32_t* lk = lkeys + (size_t)frame * total_slots + L0.key_off;
    uint16_t* knode = (uint16_t*)(knode_g + (size_t)frame * total_slots + L0.key_off);
    uint8_t* kq = kq_g + (size_t)frame * total_slots + L0.key_off;
    OctKeys<uint32_t*, uint16_t*, uint8_t*> kk{lk, knode, kq};
    oct_run(S, kk, L0, cells, cnt, nc, fk, n, outp, ocount_p, ncap, err);
  }
}

// ---- GaussianBlur 7x7 sigma 2, 8U bit-exact, BORDER_REFLECT_101 ---------------------------
__device__ __forceinline__ int reflect101(int p, int n) {
  p = p < 0 ? -p : p;
  p = p >= n ? 2 * n - 2 - p : p;
  return p;
}

// GaussianBlur(7x7, sigma 2, REFLECT_101) of every level (ORBextractor.cc:1089-1090), bit-exact
// 8U fixed point: horizontal Q8 taps -> 16-bit sums, vertical Q8 taps, (v + 2^15) >> 16.
// One wave per (stripe of 256 columns, band of kBlurBand rows); each lane owns four adjacent
// columns and walks the band: per row it loads the twelve source bytes around its columns as
// three (unaligned) dwords, forms the four 7-tap horizontal sums with byte-aligned extracts and
// two v_dot4_u32_u8 each, keeps the last seven rows of sums in a register ring (rows unrolled by
// seven, so the ring never moves), and stores its four outputs as one dword.  Source rows are
// loaded seven rows ahead into a register ring of their own.  No LDS, no barriers.  Lanes whose columns touch the level edge gather their bytes with REFLECT_101.
#ifndef MMT_BLUR_BAND
#define MMT_BLUR_BAND 32
#endif
constexpr int kBlurBand = MMT_BLUR_BAND;

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

typedef float f2x __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ pyr,
                                              uint8_t* __restrict__ blur, size_t pyr_stride,
                                              const LevelInfo* __restrict__ lv,
                                              const BlurTile* __restrict__ tiles, int ntiles, int xcd_order) {
  const uint32_t T0 = 18, T1 = 34, T2 = 48, T3 = 56;
  const uint32_t W1 = T0 | (T1 << 8) | (T2 << 16) | (T3 << 24);  // bytes x-3+j .. x+j
  const uint32_t W2 = T2 | (T1 << 8) | (T0 << 16);               // bytes x+1+j .. x+3+j, 0
  // wave-uniform (readfirstlane): the tile record, its level and the row arithmetic go to SALU
  // workgroups of one frame contiguous on one XCD (fast_job): vertically adjacent bands read the
  // same halo rows from one L2
  int xg = blockIdx.x, frame = blockIdx.y;
  if (xcd_order) fast_job(xg, frame);
  const int tile_id = __builtin_amdgcn_readfirstlane(xg * 4 + (threadIdx.x >> 6));
  if (tile_id >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const BlurTile t = tiles[tile_id];
  const LevelInfo L = lv[t.level];
  const size_t fo = (size_t)frame * pyr_stride + L.off;
  const uint8_t* img = pyr + fo;
  uint8_t* dst = blur + fo;
  // first of this lane's four columns; the lane that would hold the row's last 1-3 columns takes
  // the last four instead (it rewrites 1-3 outputs of its neighbour with the same values), so every
  // lane stores one dword and no store sits on a divergent path (levels are >= 62 columns wide)
  const int xl = t.x0 + 4 * lane;
  if (xl >= L.w) return;
  const int x = min(xl, L.w - 4);
  const int y_end = min(t.y0 + kBlurBand, L.h);
  const bool edge = x < 4 || x + 8 > L.w;  // the 12 loaded bytes x-4 .. x+7 leave the row
  // Every lane loads three dwords at `base`; edge lanes then pick their REFLECT_101 bytes out of
  // those 12 with v_perm (all reflected positions lie inside [base, base + 12)).
  const int base = min(max(x - 4, 0), max(L.w - 12, 0));
  uint32_t selA[3] = {0, 0, 0}, selB[3] = {0, 0, 0};
  if (edge) {
#pragma unroll
    for (int k = 0; k < 12; k++) {
      const int sidx = reflect101(min(max(x - 4 + k, -4), L.w + 3), L.w) - base;  // 0..11
      const uint32_t a = sidx < 8 ? (uint32_t)sidx : 0x0cu;
      const uint32_t b = sidx >= 8 ? (uint32_t)(sidx - 8) : 0x0cu;
      selA[k >> 2] |= a << (8 * (k & 3));
      selB[k >> 2] |= b << (8 * (k & 3));
    }
  }
  // raw row load (three aligned-or-clamped dwords at `base`); edge lanes pick their REFLECT_101
  // bytes when the row is consumed, so no instruction waits on a load at issue time
  auto load_row = [&](int r, uint32_t (&d)[3]) {
    const int sy = reflect101(min(r, L.h + 2), L.h);
    const uint8_t* srow = img + (size_t)sy * L.w + base;
    d[0] = ld32(srow);
    d[1] = ld32(srow + 4);
    d[2] = ld32(srow + 8);
  };
  auto fix_row = [&](uint32_t (&d)[3]) {
    if (edge) {
      const uint32_t s0 = d[0], s1 = d[1], s2 = d[2];
      d[0] = __builtin_amdgcn_perm(s1, s0, selA[0]) | __builtin_amdgcn_perm(s2, s2, selB[0]);
      d[1] = __builtin_amdgcn_perm(s1, s0, selA[1]) | __builtin_amdgcn_perm(s2, s2, selB[1]);
      d[2] = __builtin_amdgcn_perm(s1, s0, selA[2]) | __builtin_amdgcn_perm(s2, s2, selB[2]);
    }
  };
  // Horizontal sums w (<= 256 * 255) go into a 7-row ring as floats, two columns per packed
  // register; the vertical taps then run as packed fp32 FMA on integers: every product and partial
  // sum stays below 2^24 (the total is at most 256 * 65280), so the float arithmetic is exact and
  // equals the u32 formulation.
  f2x w[7][2];
#pragma unroll
  for (int i = 0; i < 7; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) w[i][j] = (f2x){0.f, 0.f};
  const f2x t0 = {(float)T0, (float)T0}, t1 = {(float)T1, (float)T1};
  const f2x t2 = {(float)T2, (float)T2}, t3 = {(float)T3, (float)T3};
  const f2x sc = {1.0f / 65536.0f, 1.0f / 65536.0f}, half = {0.5f, 0.5f};
  const int r_end = y_end + 3;
  // Source rows in a 7-slot register ring, loaded seven rows ahead: the load of row r + 7 is
  // issued as soon as row r has been consumed, so every row's load has six rows of work to hide
  // behind.  A full band (every band but a level's last) runs as straight-line code with
  // compile-time row bounds: the compiler's wait counts then stay exact from row to row (any
  // branch join or loop back edge in between makes it drain every outstanding load); a level's
  // last band takes the rolled loop.
  auto row = [&](uint32_t (&dg)[3], int g) {
    fix_row(dg);
    // horizontal sums of the four columns -> ring slot g (rows of this group: slots 0..6)
    uint32_t hs[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t a = j < 3 ? __builtin_amdgcn_alignbyte(dg[1], dg[0], 1 + j) : dg[1];
      const uint32_t bb = j < 3 ? __builtin_amdgcn_alignbyte(dg[2], dg[1], 1 + j) : dg[2];
      hs[j] = __builtin_amdgcn_udot4(bb, W2, __builtin_amdgcn_udot4(a, W1, 0u, false), false);
    }
    w[g][0] = (f2x){(float)hs[0], (float)hs[1]};
    w[g][1] = (f2x){(float)hs[2], (float)hs[3]};
  };
  auto emit = [&](int g, int yo) {
    // rows yo-3 .. yo+3 live in ring slots g+1 .. g+7 (mod 7)
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      f2x v = t3 * w[(g + 4) % 7][j];
      v = __builtin_elementwise_fma(t2, w[(g + 3) % 7][j] + w[(g + 5) % 7][j], v);
      v = __builtin_elementwise_fma(t1, w[(g + 2) % 7][j] + w[(g + 6) % 7][j], v);
      v = __builtin_elementwise_fma(t0, w[(g + 1) % 7][j] + w[g][j], v);
      // (v + 32768) >> 16 = floor(v / 65536 + 0.5): both steps exact in float
      const f2x q = __builtin_elementwise_fma(v, sc, half);
      o[2 * j] = min((uint32_t)q.x, 255u);
      o[2 * j + 1] = min((uint32_t)q.y, 255u);
    }
    const uint32_t packed = o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24);
    __builtin_memcpy(dst + (size_t)yo * L.w + x, &packed, 4);
  };
  uint32_t d[7][3];
  int r0 = t.y0 - 3;
  if (y_end - t.y0 == kBlurBand) {
    constexpr int kRows = kBlurBand + 6;  // source rows of a full band
#pragma unroll
    for (int g = 0; g < 7; g++) load_row(r0 + g, d[g]);
#pragma unroll
    for (int i = 0; i < kRows; i++) {
      const int g = i % 7;
      row(d[g], g);
      if (i + 7 < kRows) load_row(r0 + i + 7, d[g]);
      if (i >= 6) emit(g, r0 + i - 3);  // output row yo = r - 3 >= t.y0
    }
    return;
  }
#pragma unroll
  for (int g = 0; g < 7; g++) load_row(min(r0 + g, r_end - 1), d[g]);
  for (; r0 < r_end; r0 += 7) {
#pragma unroll
    for (int g = 0; g < 7; g++) {
      const int r = r0 + g;
      if (r >= r_end) break;
      row(d[g], g);
      load_row(min(r + 7, r_end - 1), d[g]);
      if (r - 3 >= t.y0) emit(g, r - 3);
    }
  }
}

// ---- fastAtan2 (OpenCV core), fp32 without contraction -------------------------------------
__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
  const float k = (float)(180.0 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
  const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
  const float eps = (float)2.220446049250313e-16;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// sin and cos of x in [0, 2pi] in double precision: Cody-Waite reduction by pi/2 (k <= 4, so
// k * PIO2_HI is exact) and the fdlibm kernels __kernel_sin / __kernel_cos (|r| <= pi/4, error
// < 1 ulp), evaluated without contraction like the C they come from.  Rounded to float this
// equals (float)cos((double)x) / (float)sin((double)x) of the host libm unless the double lies
// within an ulp of a float rounding boundary; it replaces OCML's general sin/cos (about 200
// FP64 instructions with the large-argument path) on the descriptor's critical chain.
__device__ __forceinline__ void sincos_small(double x, double* s_out, double* c_out) {
  const double PIO2_HI = 1.57079632673412561417e+00, PIO2_LO = 6.07710050650619224932e-11;
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double kd = __builtin_rint(x * 6.36619772367581382433e-01);  // x * 2/pi
  const int k = (int)kd;
  const double r = (x - kd * PIO2_HI) - kd * PIO2_LO;
  const double z = r * r;
  const double v = z * r;
  const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  const double sn = r + v * (S1 + z * ps);
  const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cs = w + (((1.0 - w) - hz) + z * pc);
  switch (k & 3) {
    case 0: *s_out = sn; *c_out = cs; break;
    case 1: *s_out = cs; *c_out = -sn; break;
    case 2: *s_out = -sn; *c_out = -cs; break;
    default: *s_out = -cs; *c_out = sn; break;
  }
}

// Four output keypoint slots per wave, 16 lanes each: IC_Angle on the level (:77-104),
// rotated BRIEF on the blurred level (:108-147), level-major assembly with coordinate scaling
// (:1079-1108). Every load of a slot is independent of the others (no dependent chains), so a
// wave keeps four keypoints' disc and pattern gathers in flight.
__device__ __forceinline__ uint32_t ld16(const uint8_t* p) {
  uint16_t v;
  __builtin_memcpy(&v, p, 2);
  return v;
}

// k_orient_desc LDS slot of one keypoint: the blurred window, kOdBRows rows of kOdBw bytes
// around the keypoint (radius kOdR)
constexpr int kOdR = 18, kOdBRows = 2 * kOdR + 1, kOdBw = 40;
constexpr int kOdSlot = kOdBRows * kOdBw;                      // 1480 (a multiple of 4)
constexpr int kOdBLoads = (kOdBRows * (kOdBw / 4) + 15) / 16;  // dwords per lane (24)
static_assert(kOdSlot % 4 == 0, "dword-aligned slots");

__global__ __launch_bounds__(256) void k_orient_desc(
    const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur, size_t pyr_stride,
    const LevelInfo* __restrict__ lv, int nlevels, const int* __restrict__ umax,
    const uint32_t* __restrict__ okeys, int out_slots, const int* __restrict__ ocount,
    mmt_kp* __restrict__ kps, uint8_t* __restrict__ desc, int cap_frame, int* __restrict__ nkp,
    int nframes, int slot_begin, int slot_end, int write_total) {
  // slots [slot_begin, slot_end) of every frame (a level range: level 0 runs as soon as its
  // octree and the blur are done); write_total: this launch stores the frame's keypoint count
  const int lane = threadIdx.x & 63;
  const int gl = lane & 15, grp = lane >> 4;
  __shared__ uint32_t od_pat[256];  // the packed test pattern, once per workgroup
  __shared__ __attribute__((aligned(16))) uint8_t od_lds[16 * kOdSlot];  // 16 keypoint slots
  od_pat[threadIdx.x] = c_pattern.t[threadIdx.x];
  __syncthreads();
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (b % 8 share one; speed
  // only, never correctness), so workgroup b serves frame (b % 8) + 8 * (b / 8 / wgf): the
  // slots of a frame run on one XCD, whose L2 then holds that frame's level and blurred level
  // rows across the overlapping patches of its keypoints
  const int wgf = (slot_end - slot_begin + 15) / 16;  // workgroups per frame (16 slots each)
  const int jx = blockIdx.x >> 3;
  const int frame = (blockIdx.x & 7) + 8 * (jx / wgf);
  if (frame >= nframes) return;  // whole 16-lane groups leave together
  const int local = slot_begin + (jx % wgf) * 16 + (threadIdx.x >> 6) * 4 + grp;
  if (local >= slot_end) return;
  // level lookup: lane gl of the group holds level gl's slot offset and count (nlevels <= 16);
  // the level is a ballot count within the group and the keys before it a group sum
  const uint32_t k = okeys[(size_t)frame * out_slots + local];
  int my_off = 0x7fffffff, my_cnt = 0, my_w = 0, my_loff = 0;
  float my_scale = 0.f, my_size = 0.f;
  if (gl < nlevels) {
    my_off = lv[gl].out_off;
    my_cnt = ocount[frame * nlevels + gl];
    my_w = lv[gl].w;
    my_loff = lv[gl].off;
    my_scale = lv[gl].scale;
    my_size = lv[gl].size;
  }
  const unsigned long long lb = __ballot(gl >= 1 && gl < nlevels && local >= my_off);
  const int level = __popcll((lb >> (16 * grp)) & 0xFFFFull);
  int before = gl < level ? my_cnt : 0, tot = my_cnt;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    before += __shfl_xor(before, o, 64);
    tot += __shfl_xor(tot, o, 64);
  }
  const int src = 16 * grp + level;
  const int lvl_off = __shfl(my_off, src, 64), lvl_cnt = __shfl(my_cnt, src, 64);
  const int Lw = __shfl(my_w, src, 64);
  const float Lscale = __shfl(my_scale, src, 64), Lsize = __shfl(my_size, src, 64);
  const size_t fo = (size_t)frame * pyr_stride + __shfl(my_loff, src, 64);
  if (write_total && local == slot_begin && gl == 0) nkp[frame] = min(tot, cap_frame);
  const int sidx = local - lvl_off;
  const int outi = before + sidx;
  if (sidx >= lvl_cnt || outi >= cap_frame) return;
  const int kx = (int)((k >> 8) & 0xFFFu), ky = (int)(k >> 20);
  const float response = (float)(k & 0xFFu);
  // The blurred 37 x 37 window the rotated tests can reach (|rotated offset| <= 13 sqrt 2 < 18.5;
  // rows of kOdBw bytes) goes to this group's LDS slot with coalesced dword loads, issued
  // together with the IC_Angle disc loads (two bytes per lane and row, into registers): one memory
  // round trip per keypoint.  Keypoints sit >= 19 px inside the level, so the windows stay inside
  // it (row tails may read a few bytes of the next row).
  uint8_t* slot_lds = od_lds + ((threadIdx.x >> 6) * 4 + grp) * kOdSlot;
  const int c0 = 2 * gl - 15, c1 = c0 + 1;
  uint32_t rows[31];
  {
    // item i = gl + 16 k is (row i / 10, dword i % 10): each step advances (1 row, 6 dwords)
    // with one carry, so the addresses are running pointers (no division, no 64-bit multiply)
    constexpr int kQ = kOdBw / 4, kDq = 16 % kQ, kDr = 16 / kQ;
    static_assert(kDr == 1 && kQ == 10, "step pattern of the staging loop");
    const uint8_t* bsrc = blur + fo + (size_t)(ky - kOdR) * Lw + (kx - kOdR);
    const uint8_t* bp = bsrc + (gl >= kQ ? Lw + 4 * (gl - kQ) : 4 * gl);
    int q = gl >= kQ ? gl - kQ : gl;
    uint32_t vb[kOdBLoads];
#pragma unroll
    for (int k = 0; k < kOdBLoads; k++) {
      if (gl + 16 * k < kOdBRows * kQ) vb[k] = ld32(bp);
      q += kDq;
      bp += Lw + 4 * kDq;
      if (q >= kQ) {
        q -= kQ;
        bp += Lw - 4 * kQ;
      }
    }
    // the whole 31 x 32 disc square is inside the level: load it unconditionally, mask later
    const uint8_t* col = pyr + fo + (size_t)(ky - 15) * Lw + kx + c0;
#pragma unroll
    for (int v = -15; v <= 15; v++, col += Lw) rows[v + 15] = ld16(col);
#pragma unroll
    for (int k = 0; k < kOdBLoads; k++) {
      const int i = gl + 16 * k;
      if (i < kOdBRows * (kOdBw / 4)) *(uint32_t*)(slot_lds + 4 * i) = vb[k];
    }
  }
  // BRIEF tests 16r + gl of this lane (r = 0..15)
  uint32_t pat[16];
#pragma unroll
  for (int r = 0; r < 16; r++) pat[r] = od_pat[16 * r + gl];
  // --- IC_Angle: lane gl owns disc columns c0 = 2gl-15 and c0+1 (column 16 does not exist; the
  // keypoint border, >= 19 px, keeps its byte inside the level)
  const int a0 = c0 < 0 ? -c0 : c0, a1 = c1 < 0 ? -c1 : c1;
  int vmax0 = 0, vmax1 = 0;
#pragma unroll
  for (int v = 1; v <= 15; v++) {
    const int um = umax[v];
    vmax0 += a0 <= um ? 1 : 0;
    vmax1 += a1 <= um ? 1 : 0;
  }
  if (c1 > 15) vmax1 = -1;
  int cs0 = 0, cs1 = 0, vs = 0;
#pragma unroll
  for (int v = -15; v <= 15; v++) {
    const int av = v < 0 ? -v : v;
    const int p0 = av <= vmax0 ? (int)(rows[v + 15] & 0xFFu) : 0;
    const int p1 = av <= vmax1 ? (int)(rows[v + 15] >> 8) : 0;
    cs0 += p0;
    cs1 += p1;
    vs += v * (p0 + p1);
  }
  int m10 = c0 * cs0 + c1 * cs1, m01 = vs;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    m10 += __shfl_xor(m10, o, 64);
    m01 += __shfl_xor(m01, o, 64);
  }
  const float angle = fast_atan2_deg((float)m01, (float)m10);
  // --- rotated BRIEF; cos/sin pinned to (float)cos((double)angle) (parity hazards)
  const float factorPI = (float)(3.14159265358979323846 / 180.0);
  const float ang = angle * factorPI;
  double sd, cd;
  sincos_small((double)ang, &sd, &cd);
  const float a = (float)cd, b = (float)sd;
  wave_sync();  // the staged window of every group of the wave
  const uint8_t* center = slot_lds + kOdR * kOdBw + kOdR;
  int bits[16];
  // the rotation as packed fp32 pairs, each product and sum rounded exactly as the scalar
  // x * a - y * b, x * b + y * a (no contraction): (x a, x b) + (-(y b), y a)
  const f2x ab = {a, b}, ba = {b, a};
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const float x0 = (float)(int8_t)(pat[r] & 0xFFu), y0 = (float)(int8_t)((pat[r] >> 8) & 0xFFu);
    const float x1 = (float)(int8_t)((pat[r] >> 16) & 0xFFu), y1 = (float)(int8_t)(pat[r] >> 24);
    const f2x p0 = (f2x){x0, x0} * ab, q0 = (f2x){y0, y0} * ba;
    const f2x p1 = (f2x){x1, x1} * ab, q1 = (f2x){y1, y1} * ba;
    const f2x rr0 = p0 + (f2x){-q0.x, q0.y}, rr1 = p1 + (f2x){-q1.x, q1.y};  // (rx, ry)
    const int v0 = center[__mul24(__float2int_rn(rr0.y), kOdBw) + __float2int_rn(rr0.x)];
    const int v1 = center[__mul24(__float2int_rn(rr1.y), kOdBw) + __float2int_rn(rr1.x)];
    bits[r] = v0 < v1;
  }
  // round r gives descriptor bytes 2r, 2r+1 (test 16r + gl -> byte 2r + gl/8, bit gl%8);
  // lane gl < 8 stores bytes 4gl..4gl+3
  uint32_t word = 0;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const uint32_t seg = (uint32_t)((__ballot(bits[r]) >> (16 * grp)) & 0xFFFFull);
    if ((r >> 1) == gl) word |= seg << (16 * (r & 1));
  }
  uint8_t* dout = desc + ((size_t)frame * cap_frame + outi) * 32;
  if (gl < 8) *(uint32_t*)(dout + 4 * gl) = word;
  if (gl == 0) {
    mmt_kp kp;
    kp.x = level == 0 ? (float)kx : (float)kx * Lscale;
    kp.y = level == 0 ? (float)ky : (float)ky * Lscale;
    kp.size = Lsize;
    kp.angle = angle;
    kp.response = response;
    kp.octave = level;
    kp.class_id = -1;
    kps[(size_t)frame * cap_frame + outi] = kp;
  }
}

// ======================================================================== host engine


OrbEngine::~OrbEngine() { release(); }

void OrbEngine::release() {
  void* ptrs[] = {d_lv_,    d_cells_,  d_xtab_,  d_ytab_,    d_tiles_,  d_umax_,   d_pyr_,
                  d_blur_,  d_keys_,   d_lkeys_, d_knode_,   d_cellcnt_, d_okeys_, d_ocount_,
                  d_err_,   d_pyr_bands_};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  d_lv_ = nullptr;
  d_cells_ = nullptr;
  d_xtab_ = nullptr;
  d_ytab_ = nullptr;
  d_tiles_ = nullptr;
  d_umax_ = nullptr;
  d_pyr_ = d_blur_ = nullptr;
  d_keys_ = d_lkeys_ = d_knode_ = d_okeys_ = nullptr;
  d_cellcnt_ = d_ocount_ = d_err_ = nullptr;
  d_pyr_bands_ = nullptr;
  pyr_bands_ = 0;
  for (hipEvent_t* e : {&ev_pyr_, &ev_blur_, &ev_gray_}) {
    if (*e) (void)hipEventDestroy(*e);
    *e = nullptr;
  }
  if (side_) (void)hipStreamDestroy(side_);
  side_ = nullptr;
}

template <typename T>
static void upload(T** dptr, const std::vector<T>& v) {
  MMT_HIP(hipMalloc((void**)dptr, std::max<size_t>(1, v.size()) * sizeof(T)));
  if (!v.empty()) MMT_HIP(hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
}

void OrbEngine::setup(int w, int h, const OrbTables& t, int max_batch) {
  release();
  if (w > 4000 || h > 4000) throw ArgError("image larger than 4000 px is not supported");
  w_ = w;
  h_ = h;
  nlevels_ = t.nlevels;
  max_batch_ = std::max(1, max_batch);
  iniTh_ = t.iniTh;
  minTh_ = t.minTh;
  lv_.assign(nlevels_, LevelInfo());
  cells_.clear();
  fast_rows_max_ = fast_cols_max_ = fast_win_max_ = 0;
  int off = 0, key_off = 0, out_off = 0, maxN = 0;
  std::vector<ResizeX> xt;
  std::vector<ResizeY> yt;
  xtab_off_.assign(nlevels_, 0);
  ytab_off_.assign(nlevels_, 0);
  rs_pitch_.assign(nlevels_, 0);
  rs_lds_.assign(nlevels_, 0);
  std::vector<BlurTile> tiles;
  for (int l = 0; l < nlevels_; l++) {
    LevelInfo& L = lv_[l];
    L.w = host_round((float)w * t.invScale[l]);
    L.h = host_round((float)h * t.invScale[l]);
    if (L.w - 2 * kMinBorder < 30 || L.h - 2 * kMinBorder < 30)
      throw ArgError("image too small for the requested pyramid (level " + std::to_string(l) + ")");
    L.off = off;
    off += L.w * L.h;
    // FAST cells (ORBextractor.cc:769-806)
    const int maxBorderX = L.w - kEdge + 3, maxBorderY = L.h - kEdge + 3;
    const float width = (float)(maxBorderX - kMinBorder), height = (float)(maxBorderY - kMinBorder);
    const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
    const int wCell = (int)ceil(width / nCols), hCell = (int)ceil(height / nRows);
    L.cell_begin = (int)cells_.size();
    L.key_off = key_off;
    for (int i = 0; i < nRows; i++) {
      const float iniY = (float)(kMinBorder + i * hCell);
      float maxY = iniY + hCell + 6;
      if (iniY >= maxBorderY - 3) continue;
      if (maxY > maxBorderY) maxY = (float)maxBorderY;
      for (int j = 0; j < nCols; j++) {
        const float iniX = (float)(kMinBorder + j * wCell);
        float maxX = iniX + wCell + 6;
        if (iniX >= maxBorderX - 6) continue;
        if (maxX > maxBorderX) maxX = (float)maxBorderX;
        CellInfo c;
        c.level = l;
        c.r0 = (int)iniY;
        c.c0 = (int)iniX;
        c.rows = (int)maxY - (int)iniY;
        c.cols = (int)maxX - (int)iniX;
        if (c.rows > kFSMax || ((c.cols + 4) & ~3) > kFSMax || c.cols - 6 > 64)
          throw ArgError("FAST cell larger than the LDS tile");
        fast_rows_max_ = std::max(fast_rows_max_, c.rows);
        fast_cols_max_ = std::max(fast_cols_max_, (c.cols + 4) & ~3);  // tile at LDS column 1
        fast_win_max_ = std::max(fast_win_max_, std::max(c.rows - 6, 0) * std::max(c.cols - 6, 0));
        const int R = std::max(c.rows - 6, 0), C = std::max(c.cols - 6, 0);
        c.slot_cap = ((R + 1) / 2) * ((C + 1) / 2);  // max strict-NMS survivors
        c.slot_off = key_off;
        c.pad = 0;
        key_off += c.slot_cap;
        cells_.push_back(c);
      }
    }
    L.cell_end = (int)cells_.size();
    L.key_cap = key_off - L.key_off;
    // octree geometry (ORBextractor.cc:543-545)
    const int minX = kMinBorder, maxX = maxBorderX, minY = kMinBorder, maxY = maxBorderY;
    L.nIni = (int)round(static_cast<float>(maxX - minX) / (maxY - minY));
    if (L.nIni < 1) throw ArgError("degenerate octree geometry (nIni < 1)");
    L.hX = static_cast<float>(maxX - minX) / L.nIni;
    L.N = t.nPerLevel[l];
    maxN = std::max(maxN, L.N);
    L.out_off = out_off;
    L.out_cap = L.N + 8;
    out_off += L.out_cap;
    L.scale = t.scale[l];
    L.size = (float)(int)(31 * t.scale[l]);
    // resize tables for level l (from l-1)
    if (l > 0) {
      const LevelInfo& S = lv_[l - 1];
      const int sw = S.w, sh = S.h, dw = L.w, dh = L.h;
      const double isx = (double)dw / sw, isy = (double)dh / sh;
      const double scx = 1. / isx, scy = 1. / isy;
      xtab_off_[l] = (int)xt.size();
      for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scx - 0.5);
        int sx = host_floor(fx);
        fx -= sx;
        bool clampR = false;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
          clampR = true;
          if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        ResizeX r;
        r.sx = sx;
        r.a0 = (short)std::min(std::max(host_round((1.f - fx) * 2048), -32768), 32767);
        r.a1 = (short)std::min(std::max(host_round(fx * 2048), -32768), 32767);
        if (clampR) { r.a0 = 2048; r.a1 = 0; }
        xt.push_back(r);
      }
      ytab_off_[l] = (int)yt.size();
      for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scy - 0.5);
        int sy = host_floor(fy);
        fy -= sy;
        auto clip = [&](int v) { return v >= 0 ? (v < sh ? v : sh - 1) : 0; };
        ResizeY r;
        r.sy0 = clip(sy);
        r.sy1 = clip(sy + 1);
        r.b0 = (short)std::min(std::max(host_round((1.f - fy) * 2048), -32768), 32767);
        r.b1 = (short)std::min(std::max(host_round(fy * 2048), -32768), 32767);
        yt.push_back(r);
      }
      // k_resize staging window: widest column block, tallest row band
      int pitch = 0, rows = 0;
      const ResizeX* X = xt.data() + xtab_off_[l];
      const ResizeY* Y = yt.data() + ytab_off_[l];
      for (int dx0 = 0; dx0 < dw; dx0 += kResizeCols) {
        const int dx1 = std::min(dx0 + kResizeCols, dw);
        const int lo = X[dx0].sx, hi = std::min(X[dx1 - 1].sx + 1, sw - 1);
        pitch = std::max(pitch, 4 * ((hi - lo + 4) >> 2) + 4);
      }
      for (int y0 = 0; y0 < dh; y0 += kResizeRows) {
        const int y1 = std::min(y0 + kResizeRows, dh);
        rows = std::max(rows, Y[y1 - 1].sy1 - Y[y0].sy0 + 1);
      }
      rs_pitch_[l] = pitch;
      rs_lds_[l] = pitch * rows;
      if (rs_lds_[l] > 64 * 1024) throw ArgError("resize staging window exceeds 64 KB of LDS");
    }
    for (int y0 = 0; y0 < L.h; y0 += kBlurBand)
      for (int x0 = 0; x0 < L.w; x0 += 256) tiles.push_back(BlurTile{l, x0, y0, 0});
  }
  ncells_ = (int)cells_.size();
  ntiles_ = (int)tiles.size();
  // MMT_ORB_SCHED=2 (profiling switch, tools/orb_sched.sh): every ORB launch on the caller's
  // stream, so a kernel trace gives standalone kernel times
  if (const char* e = getenv("MMT_ORB_SCHED")) sched_ = atoi(e);
  total_slots_ = key_off;
  out_slots_ = out_off;
  cap_frame_ = out_off;
  pyr_stride_ = ((size_t)off + 255) & ~(size_t)255;
  node_cap_ = 256;
  while (node_cap_ < maxN + 16) node_cap_ <<= 1;
  for (auto& L : lv_) {
    while (L.cell_end - L.cell_begin > 4 * node_cap_) node_cap_ <<= 1;  // gather scratch
    if (L.nIni > node_cap_) throw ArgError("too many initial octree nodes");
  }
  if (node_cap_ > 2048) throw ArgError("ORB nfeatures too large for the LDS octree (max ~9000)");
  for (int fs : {kFSSmall, kFSMax}) {
    const int lds = 4 * fast_wave_lds(fs, fast_rows_max_, fast_win_max_);
    if (lds > 160 * 1024) throw ArgError("FAST cells too large for LDS");
    MMT_HIP(hipFuncSetAttribute(fs == kFSSmall ? (const void*)k_fast<kFSSmall> : (const void*)k_fast<kFSMax>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  }
  // keys in LDS up to what the node arrays leave of the CU's 160 KB (global scratch beyond)
  const uint32_t lds_budget = 160 * 1024 - 1024;
  key_cap_ = 0;  // largest multiple of 16 keys (<= 16384) whose carved layout fits the budget
  for (int k = 16384; k >= 256; k -= 16)
    if (oct_layout(node_cap_, k).end <= lds_budget) {
      key_cap_ = k;
      break;
    }
  octree_lds_ = oct_layout(node_cap_, key_cap_).end;
  if (octree_lds_ > lds_budget) throw ArgError("octree node arrays exceed the LDS budget");
  MMT_HIP(hipFuncSetAttribute((const void*)k_octree<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)octree_lds_));
  // levels 1..: keys in LDS up to half a CU's LDS, so two workgroups share a CU and a batch's
  // (levels x frames) workgroups run in one round; the few (level, frame) pairs with more keys
  // take the global-scratch path
  const uint32_t half_budget = 80 * 1024 - 512;
  key_cap1_ = 0;
  for (int k = std::min(key_cap_, 16384); k >= 256; k -= 16)
    if (oct_layout(node_cap_, k).end <= half_budget) {
      key_cap1_ = k;
      break;
    }
  int max_key_cap1 = 0;  // keys any level 1.. can hold at most (its FAST slot capacity)
  for (int l = 1; l < nlevels_; l++) max_key_cap1 = std::max(max_key_cap1, lv_[l].key_cap);
  if (key_cap1_ < 256) {
    key_cap1_ = key_cap_;  // the node arrays alone fill half the LDS: one workgroup per CU
    octree_lds1_ = octree_lds_;
    oct_two_per_cu_ = false;
  } else {
    key_cap1_ = std::min(key_cap1_, (max_key_cap1 + 15) & ~15);
    octree_lds1_ = oct_layout(node_cap_, key_cap1_).end;
    oct_two_per_cu_ = true;
    MMT_HIP(hipFuncSetAttribute((const void*)k_octree<8>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)octree_lds1_));
  }
  // k_pyramid bands: the fewest (from 16) whose two level buffers fit 120 KB of LDS
  pyr_bands_ = 0;
  if (nlevels_ <= kPyrMaxLevels && nlevels_ > 1) {
    for (int nb = 16; nb <= 256 && pyr_bands_ == 0; nb *= 2) {
      std::vector<PyrBand> bands(nb);
      PyrArgs pa{};
      pa.nl = nlevels_;
      for (int l = 0; l < nlevels_; l++) {
        pa.pitch[l] = ((lv_[l].w + 3) & ~3) + 4;  // + the clamped edge's byte at sx + 1
        pa.xoff[l] = xtab_off_[l];
        pa.yoff[l] = ytab_off_[l];
      }
      bool fits = true;
      int buf = 0;
      for (int b = 0; b < nb && fits; b++) {
        PyrBand& B = bands[b];
        // backward from the last level: rows computed = own rows + the rows the next level reads
        for (int l = nlevels_ - 1; l >= 0; l--) {
          int lo = l > 0 ? lv_[l].h * b / nb : 0, hi = l > 0 ? lv_[l].h * (b + 1) / nb : 0;
          if (l + 1 < nlevels_ && B.lo[l + 1] < B.hi[l + 1]) {
            const ResizeY* Y = yt.data() + ytab_off_[l + 1];
            const int slo = Y[B.lo[l + 1]].sy0, shi = Y[B.hi[l + 1] - 1].sy1 + 1;
            if (lo < hi) {
              lo = std::min(lo, slo);
              hi = std::max(hi, shi);
            } else {
              lo = slo;
              hi = shi;
            }
          }
          B.lo[l] = lo;
          B.hi[l] = std::max(lo, hi);
          if (l + 1 < nlevels_) buf = std::max(buf, (B.hi[l] - B.lo[l]) * pa.pitch[l]);
        }
        fits = 2 * ((buf + 15) & ~15) <= 120 * 1024;
        for (int l = 0; l < nlevels_; l++) fits = fits && B.hi[l] - B.lo[l] <= 1024;
        // k_pyramid stages level-0 rows clamped to [lo, hi - 1]: an empty level-0 range would
        // read row -1, so such a band count is rejected (the k_resize chain takes over)
        fits = fits && B.lo[0] < B.hi[0];
      }
      if (!fits) continue;
      pa.buf_bytes = (buf + 15) & ~15;
      int yrows = 0;  // the largest band's row coefficients over levels 1..
      for (const PyrBand& B : bands) {
        int n = 0;
        for (int l = 1; l < nlevels_; l++) n += B.hi[l] - B.lo[l];
        yrows = std::max(yrows, n);
      }
      pyr_lds_ = 2 * pa.buf_bytes + (int)sizeof(ResizeY) * yrows;
      pyr_bands_ = nb;
      pyr_args_ = pa;
      upload(&d_pyr_bands_, bands);
      MMT_HIP(hipFuncSetAttribute((const void*)k_pyramid, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  pyr_lds_));
    }
  }
  upload(&d_lv_, lv_);
  upload(&d_cells_, cells_);
  upload(&d_xtab_, xt);
  upload(&d_ytab_, yt);
  upload(&d_tiles_, tiles);
  upload(&d_umax_, t.umax);
  const size_t B = (size_t)max_batch_;
  MMT_HIP(hipMalloc((void**)&d_pyr_, B * pyr_stride_ + 64));  // + dword over-read slack
  MMT_HIP(hipMalloc((void**)&d_blur_, B * pyr_stride_ + 64));  // + aligned over-read slack
  MMT_HIP(hipMalloc((void**)&d_keys_, B * total_slots_ * sizeof(uint32_t)));
  MMT_HIP(hipMalloc((void**)&d_lkeys_, B * total_slots_ * sizeof(uint32_t)));
  // knode (u32 per slot) followed by the per-key quadrant bytes (u8 per slot)
  MMT_HIP(hipMalloc((void**)&d_knode_, B * total_slots_ * (sizeof(uint32_t) + 1) + 16));
  MMT_HIP(hipMalloc((void**)&d_cellcnt_, B * ncells_ * sizeof(int)));
  MMT_HIP(hipMalloc((void**)&d_okeys_, B * out_slots_ * sizeof(uint32_t)));
  MMT_HIP(hipMalloc((void**)&d_ocount_, B * nlevels_ * sizeof(int)));
  MMT_HIP(hipMalloc((void**)&d_err_, sizeof(int)));
  MMT_HIP(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  for (hipEvent_t* e : {&ev_pyr_, &ev_blur_, &ev_gray_})
    MMT_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  MMT_HIP(hipMemset(d_err_, 0, sizeof(int)));
}

void OrbEngine::run(const uint8_t* d_gray, int nframes, size_t frame_pitch, mmt_kp* d_kps,
                    uint8_t* d_desc, int cap_per_frame, int* d_n, hipStream_t stream) {
  if (nframes < 1 || nframes > max_batch_) throw ArgError("nframes outside [1, max_batch]");
  if (cap_per_frame < cap_frame_) throw ArgError("cap_per_frame below mmt_orb_capacity()");
  const size_t lvl0 = (size_t)w_ * h_;
  // level 0: copy the gray frames into the pyramid buffer
  if (d_gray != d_pyr_ || frame_pitch != pyr_stride_)
    MMT_HIP(hipMemcpy2DAsync(d_pyr_, pyr_stride_, d_gray, frame_pitch, lvl0, nframes,
                             hipMemcpyDeviceToDevice, stream));
  // the whole batch in one launch sequence (splitting it into parts on stream pairs of their own
  // measured slower at 2 and 4 parts: the window is throughput-bound)
  run_part(0, nframes, stream, side_, nullptr, d_kps, d_desc, cap_per_frame, d_n);
  MMT_HIP(hipGetLastError());
}

// The launch sequence of frames [f0, f0 + nf) of the batch on a (main, side) stream pair: every
// per-frame buffer is frame-major, so the part's launches see its frames as frames 0..nf-1 of
// views offset by f0.  ev: the part's events (nullptr: the engine's own).
void OrbEngine::run_part(int f0, int nframes, hipStream_t stream, hipStream_t side,
                         hipEvent_t* ev, mmt_kp* d_kps_all, uint8_t* d_desc_all,
                         int cap_per_frame, int* d_n_all) {
  hipEvent_t e_gray = ev ? ev[0] : ev_gray_, e_pyr = ev ? ev[1] : ev_pyr_,
             e_blur = ev ? ev[2] : ev_blur_;
  uint8_t* pyr = d_pyr_ + (size_t)f0 * pyr_stride_;
  uint8_t* blurb = d_blur_ + (size_t)f0 * pyr_stride_;
  uint32_t* keys = d_keys_ + (size_t)f0 * total_slots_;
  uint32_t* lkeys = d_lkeys_ + (size_t)f0 * total_slots_;
  uint32_t* knode = d_knode_ + (size_t)f0 * total_slots_;
  uint8_t* kq = (uint8_t*)(d_knode_ + (size_t)max_batch_ * total_slots_) +
                (size_t)f0 * total_slots_;
  int* cellcnt = d_cellcnt_ + (size_t)f0 * ncells_;
  uint32_t* okeys = d_okeys_ + (size_t)f0 * out_slots_;
  int* ocount = d_ocount_ + (size_t)f0 * nlevels_;
  mmt_kp* d_kps = d_kps_all + (size_t)f0 * cap_per_frame;
  uint8_t* d_desc = d_desc_all + (size_t)f0 * cap_per_frame * 32;
  int* d_n = d_n_all + f0;
  // FAST on level 0 needs only the gray frames: it runs on the side stream while the main stream
  // walks the (latency-bound) resize chain; FAST on levels 1.. follows the chain
  const int fs = fast_cols_max_ <= kFSSmall ? kFSSmall : kFSMax;
  const int fast_lds = 4 * fast_wave_lds(fs, fast_rows_max_, fast_win_max_);
  auto fast = [&](int c0, int c1, hipStream_t st) {
    if (c1 <= c0) return;
    const int waves = (c1 - c0 + fast_cpw_ - 1) / fast_cpw_;  // fast_cpw_ cells per wave
    hipLaunchKernelGGL(fs == kFSSmall ? k_fast<kFSSmall> : k_fast<kFSMax>,
                       dim3((waves + 3) / 4, nframes), dim3(256), fast_lds, st, pyr,
                       pyr_stride_, d_lv_, d_cells_, ncells_, keys, total_slots_, cellcnt,
                       iniTh_, minTh_, fast_rows_max_, fast_win_max_, c0, c1);
  };
  auto octree = [&](int l0, int l1, hipStream_t st) {
    // level 0 alone: the full-LDS variant; levels 1..: two workgroups per CU when they fit
    const bool two = l0 > 0 && oct_two_per_cu_;
    hipLaunchKernelGGL(two ? k_octree<8> : k_octree<1>, dim3(nframes, l1 - l0), dim3(1024),
                       two ? octree_lds1_ : octree_lds_, st, d_lv_, d_cells_, ncells_, keys,
                       cellcnt, total_slots_, lkeys, knode, kq, okeys, out_slots_, ocount,
                       nlevels_, node_cap_, two ? key_cap1_ : key_cap_, l0, d_err_);
  };
  auto resize = [&](int l, hipStream_t st) {
    const LevelInfo& S = lv_[l - 1];
    const LevelInfo& L = lv_[l];
    dim3 grid((L.w + kResizeCols - 1) / kResizeCols, (L.h + kResizeRows - 1) / kResizeRows,
              nframes);
    hipLaunchKernelGGL(k_resize, grid, dim3(256), rs_lds_[l], st, pyr, pyr_stride_, S.off,
                       S.w, L.off, L.w, L.h, d_xtab_ + xtab_off_[l], d_ytab_ + ytab_off_[l],
                       rs_pitch_[l], xcd_order_ & 1);
  };
  auto pyramid = [&](hipStream_t st) {  // levels 1..: one k_pyramid launch, or the k_resize chain
    // k_pyramid for small batches, where the chain's seven launches are pure latency; from 64
    // frames on the chain is faster (at 128: 151 against 220 us standalone, the band workgroups'
    // per-level barriers and halo rows cost more than the launches; mmt_internal.h)
    if (pyr_bands_ > 0 && nframes <= pyr_max_frames_) {
      hipLaunchKernelGGL(k_pyramid, dim3(pyr_bands_, nframes), dim3(1024), pyr_lds_,
                         st, pyr, pyr_stride_, d_lv_, d_xtab_, d_ytab_, d_pyr_bands_, pyr_args_);
    } else {
      for (int l = 1; l < nlevels_; l++) resize(l, st);
    }
  };
  auto blur = [&](hipStream_t st) {
    hipLaunchKernelGGL(k_blur, dim3((ntiles_ + 3) / 4, nframes), dim3(256), 0, st, pyr,
                       blurb, pyr_stride_, d_lv_, d_tiles_, ntiles_, (xcd_order_ >> 1) & 1);
  };
  auto cells = [&](int l) { return std::make_pair(lv_[l].cell_begin, lv_[l].cell_end); };
  const int NL = nlevels_;
  if (sched_ & 2) {  // one stream: standalone kernel times (profiling)
    fast(cells(0).first, cells(0).second, stream);
    octree(0, 1, stream);
    pyramid(stream);
    blur(stream);
    fast(cells(0).second, ncells_, stream);
    if (NL > 1) octree(1, NL, stream);
  } else {
    // Two chains that meet before orientation:
    //   side:  FAST + octree of level 0 (they need only the gray frames), then the blur of
    //          every level once the pyramid is complete
    //   main:  the (latency-bound) chain of k_resize launches, FAST + octree of levels 1..
    // Tried and measured equal or slower (the window is throughput-bound once FAST overlaps
    // the chain): FAST per level as each level lands, FAST of levels 1-3 beside the chain, one
    // octree launch for every level, the chain on a high-priority stream.
    MMT_HIP(hipEventRecord(e_gray, stream));
    MMT_HIP(hipStreamWaitEvent(side, e_gray, 0));
    fast(cells(0).first, cells(0).second, side);
    octree(0, 1, side);
    pyramid(stream);
    MMT_HIP(hipEventRecord(e_pyr, stream));
    MMT_HIP(hipStreamWaitEvent(side, e_pyr, 0));
    blur(side);
    MMT_HIP(hipEventRecord(e_blur, side));
    fast(cells(0).second, ncells_, stream);
    if (NL > 1) octree(1, NL, stream);
    MMT_HIP(hipStreamWaitEvent(stream, e_blur, 0));
  }
  auto orient = [&](int s0, int s1, int write_total, hipStream_t st) {
    const int grid = 8 * ((nframes + 7) / 8) * ((s1 - s0 + 15) / 16);  // see k_orient_desc
    hipLaunchKernelGGL(k_orient_desc, dim3(grid), dim3(256), 0, st, pyr, blurb, pyr_stride_,
                       d_lv_, nlevels_, d_umax_, okeys, out_slots_, ocount, d_kps, d_desc,
                       cap_per_frame, d_n, nframes, s0, s1, write_total);
  };
  if (NL > 1 && !(sched_ & 2)) {
    // level 0's orientation on the side stream (its octree and the blur are done there) while
    // the main stream runs the octree of levels 1..; the main stream's own orientation of levels
    // 1.. writes the totals, then waits for the side stream
    orient(0, lv_[1].out_off, 0, side);
    MMT_HIP(hipEventRecord(e_pyr, side));
    orient(lv_[1].out_off, out_slots_, 1, stream);
    MMT_HIP(hipStreamWaitEvent(stream, e_pyr, 0));
  } else {
    orient(0, out_slots_, 1, stream);
  }
}

void OrbEngine::check_flags(hipStream_t stream) {
  int flags = 0;
  MMT_HIP(hipMemcpyAsync(&flags, d_err_, sizeof(int), hipMemcpyDeviceToHost, stream));
  MMT_HIP(hipStreamSynchronize(stream));
  check_flags_value(flags, stream);
}

void OrbEngine::check_flags_value(int flags, hipStream_t stream) {
  if (flags == 0) return;
  MMT_HIP(hipMemsetAsync(d_err_, 0, sizeof(int), stream));
  MMT_HIP(hipStreamSynchronize(stream));
  std::string what;
  if (flags & 1) what += " octree-pass-guard";
  if (flags & 2) what += " octree-node-capacity";
  if (flags & 4) what += " octree-output-truncated";
  char hex[16];
  snprintf(hex, sizeof(hex), "0x%x", flags);
  throw DeviceError(std::string("ORB device error flags ") + hex + ":" + what);
}

void OrbEngine::raise_flags(int flags, hipStream_t stream) {
  int cur = 0;
  MMT_HIP(hipMemcpyAsync(&cur, d_err_, sizeof(int), hipMemcpyDeviceToHost, stream));
  MMT_HIP(hipStreamSynchronize(stream));
  cur |= flags;
  MMT_HIP(hipMemcpyAsync(d_err_, &cur, sizeof(int), hipMemcpyHostToDevice, stream));
  MMT_HIP(hipStreamSynchronize(stream));
}

long OrbEngine::debug_fetch(int what, int frame, void* out, size_t cap, hipStream_t stream) {
  if (frame < 0 || frame >= max_batch_) throw ArgError("bad frame");
  const void* src = nullptr;
  size_t bytes = 0;
  size_t P = 0;
  for (auto& L : lv_) P += (size_t)L.w * L.h;
  switch (what) {
    case 0: src = d_pyr_ + frame * pyr_stride_; bytes = P; break;
    case 1: src = d_blur_ + frame * pyr_stride_; bytes = P; break;
    case 2: src = d_cellcnt_ + (size_t)frame * ncells_; bytes = sizeof(int) * ncells_; break;
    case 3: src = d_keys_ + (size_t)frame * total_slots_; bytes = 4 * (size_t)total_slots_; break;
    case 4: src = d_okeys_ + (size_t)frame * out_slots_; bytes = 4 * (size_t)out_slots_; break;
    case 5: src = d_ocount_ + (size_t)frame * nlevels_; bytes = sizeof(int) * nlevels_; break;
    case 6: src = d_err_; bytes = sizeof(int); break;
    default: throw ArgError("bad debug buffer id");
  }
  if (bytes > cap) throw ArgError("debug buffer too small");
  MMT_HIP(hipMemcpyAsync(out, src, bytes, hipMemcpyDeviceToHost, stream));
  MMT_HIP(hipStreamSynchronize(stream));
  return (long)bytes;
}

}  // namespace mmt
