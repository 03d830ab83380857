// multimot_track_amd/csrc/mmt_pnp.h -- device record of one object's D5 RANSAC problem.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mmt.h"

namespace mmt {

struct PnPObject {
  // inputs
  const int* n;             // member count (device)
  const int* members;       // ascending sample indices (ObjIdNew[i])
  const float2* last_keys;  // last frame's own object samples (mvObjKeys of mLastFrame)
  const float* last_depth;
  const float2* cur_keys;   // current mvObjKeys (= last mvObjCorres)
  float Tlast[16];
  float fx, fy, cx, cy;
  double reproj, confidence;
  const int* subsets;       // [max_iters][5] RNG((uint64)-1) draws for this count
  int use_mm;               // motion model available (PreObjID != -1)
  float MM[16];             // Tcw * last vObjMod[PreObjID]
  int use_mm_choice;        // set by the host after the counts are known
  // scratch / outputs
  float* pts3;              // [cap][3] pre_3d
  float2* pts2;             // [cap] cur_2d
  double* models;           // [max_iters][6] rvec, tvec
  double* hrec;             // [max_iters][kHypRec] per-hypothesis EPnP state (null space, L, ...)
  double* hout;             // [max_iters][3][kHypOut] err, R, t of the three beta estimates
  int* good;                // [max_iters]
  unsigned long long* masks;  // [max_iters][mask_words]
  int mask_words;
  int* inliers;             // RANSAC inliers (indices into the member list)
  int* mm_inliers;
  int* subset;              // D3 edge -> sample index
  int* n_subset;
  int* result;              // best, maxGood, iterations, n_ransac_inliers, n_mm_inliers,
                            // D6: refined inlier count (6)
  double* Rt;               // R (9), t (3)
  // D6 (PnPsolver) only
  int raw_pixels;           // EPnP inputs are the pixels as they are (add_correspondence)
  int rt_raw;               // refit R without the Rodrigues round trip
  const float* max_err;     // [n] mvMaxError = sigma2 * th2 (CheckInliers thresholds)
  double* hrt;              // [max_iters][12] R, t of each hypothesis' chosen estimate
};

constexpr int kHypRec = 160;  // doubles per hypothesis record
constexpr int kHypOut = 16;   // doubles per (hypothesis, beta variant) result

// RANSAC + refit (everything but the motion-model check)
void launch_pnp(PnPObject* d_objs, int nobj, int max_iters, hipStream_t st, bool gather = true);
// motion-model inliers (needs PnPObject::MM, i.e. the previous frame's object motions)
void launch_pnp_mm(PnPObject* d_objs, int nobj, hipStream_t st);
void launch_pnp_subset(PnPObject* d_objs, int nobj, hipStream_t st);
// D6: P4P hypotheses (subsets [K][4]), their chosen estimates (hrt) and CheckInliers (good,
// masks rows 0..K-1)
void launch_p4p_hypotheses(PnPObject* d_obj, int K, hipStream_t st);
// D6: PnPsolver::Refine on the inliers of masks row `row` (EPnP over them, CheckInliers of the
// refined pose: count in result[6], mask in row `row_out`, pose in Rt)
void launch_p4p_refine(PnPObject* d_obj, int row, int row_out, hipStream_t st);
// PnPsolver::SetRansacParameters + iterate(n_iterations) on the GPU (mmt_pnpsolver_iterate's
// semantics, include/mmt.h; throws ArgError on bad arguments)
void pnpsolver_iterate_gpu(hipStream_t s, const mmt_pnpsolver_problem* pr, const int32_t* randi,
                           int n_draw_iters, int n_iterations, mmt_pnpsolver_state* st,
                           float* Tcw_out, uint8_t* inliers_out, int* n_inliers, int* pose_found,
                           int* no_more);


#ifdef __HIPCC__
// motion-model inliers, ascending (GetInitModelObj, Tracking.cc:4380-4399); MM row-major float.
// Block-level (256 threads, every thread of the workgroup calls it).
__device__ inline void pnp_mm_inliers_block(PnPObject& o) {
  __shared__ int s_w[4];
  if (!o.use_mm) return;
  const int n = *o.n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    bool in = false;
    if (i < n) {
      float xc[3];
      for (int r = 0; r < 3; r++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += (double)o.MM[4 * r + k] * (double)o.pts3[3 * i + k];
        xc[r] = (float)s + o.MM[4 * r + 3];
      }
      const float invzc = (float)(1.0 / (double)xc[2]);
      const float u = o.fx * xc[0] * invzc + o.cx, v = o.fy * xc[1] * invzc + o.cy;
      const float2 q = o.pts2[i];
      const float u_ = q.x - u, v_ = q.y - v;
      const float Rpe = sqrtf(u_ * u_ + v_ * v_);
      in = (double)Rpe < o.reproj;
    }
    const unsigned long long bal = __ballot(in);
    if (lane == 0) s_w[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < wave) off += s_w[w];
      tot += s_w[w];
    }
    if (in) o.mm_inliers[base + off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) o.result[4] = base;
}

// D3 edge index list: ObjId_sub[i] = ObjId[inliers[i]] (sample indices) of the chosen model
__device__ inline void pnp_subset_block(PnPObject& o) {
  const int n = o.use_mm_choice ? o.result[4] : o.result[3];
  const int* src = o.use_mm_choice ? o.mm_inliers : o.inliers;
  for (int i = threadIdx.x; i < n; i += blockDim.x) o.subset[i] = o.members[src[i]];
  if (threadIdx.x == 0) *o.n_subset = n;
}
#endif

}  // namespace mmt
