// multimot_track_amd/csrc/mmt_track.h -- device-side records of the tracking kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mmt.h"

namespace mmt {

constexpr int kMaxLabel = 16;  // semantic labels 0..15 per frame (LoadMask keeps 1..3)

// Static samples of one frame: mvSiftKeysTmp / mvCorres / mvFlowNext / mvSiftDepthTmp.
struct SampleSet {
  float2* keys;
  float2* corres;
  float2* flow;
  float* depth;
  int* count;
  int cap;
};

// Object samples: mvObjKeys / mvObjCorres / mvObjFlowNext / mvObjDepth / vSemObjLabel.
struct ObjSampleSet {
  float2* keys;
  float2* corres;
  float2* flow;
  float* depth;
  int32_t* label;
  int* count;
  int cap;
  int* block_counts;  // per-workgroup counts of the two-pass compaction (64 ints)
};

// Current-frame arrays after the hand-off (mvSiftKeys/Depth, mvObjKeys/Depth, vSemObjLabel).
struct HandoffSet {
  float2* skeys;
  float* sdepth;
  int* ns;
  float2* okeys;
  float* odepth;
  int32_t* olabel;
  int* no;
};

struct LabelStats {
  int cnt, bcnt, sfcnt, members;
  float depth_sum;
  int pad[3];
};

struct GroupArgs {
  const int* n;
  const float2* cur_keys;
  const float* cur_depth;
  const int32_t* cur_label;
  const float2* last_keys;
  const float* last_depth;
  const int32_t* last_label;
  float Tcur[16], Tlast[16];
  float fx, fy, cx, cy;
  int W, H;
  int32_t* obj_label;  // vObjLabel (-1 / -2)
  int* members;        // [kMaxLabel][member_cap] ascending sample indices
  int member_cap;
  LabelStats* stats;   // [kMaxLabel]
  int* hist;           // [kMaxLabel][kMaxLabel]: current label x last label counts
  int* err;
};

// One flow-refined pose solve.
struct FlowSolveDesc {
  const int* d_n;  // device edge count (or null: n)
  int n;
  const int* idx;  // optional edge -> sample index map
  const float2* obs;
  const float2* flow;
  const float* depth;
  float Tcw_last[16];
  float init[16];
  float rp_thres;
  int use_noise;
  float g0;
  int max_iters;
  double prior_info;
  float fx, fy, cx, cy;
  double* scratch;
  int cap;
  float* pose_out;
  int* stats;  // iterations, inliers, status (1: fewer than 3 edges, pose not written)
  // optional: ObjCentre3D_pre (Tracking.cc:2032-2049), the mean world position of the solve's
  // last-frame points unprojected with the frame's depth noise (UnprojectStereoObject(i, 1),
  // Frame.cc:1118-1152: noise = gaussian(z^2 / 362.5 * 0.15) with the first draw g0)
  float* centre_out;
  // split solve (launch_flow_lm_split): the exchange granules of the solve's workgroups
  // (kFlowSplitGranules 8-byte words, zeroed once at allocation) and this launch's tag salt
  unsigned long long* gx;
  unsigned gx_seq;
  // spin bound of the exchange waits in 100 MHz wall-clock ticks (0: 0.1 s); a test hook shortens
  // it to force the not-resident status
  unsigned long long gx_spin;
};

// A large single solve split over up to kFlowSplitMax workgroups (one slice of the edges each),
// which meet at every reduction through tagged granules (flow_lm_body).
constexpr int kFlowSplitMax = 8;
constexpr int kFlowSplitGranules = 2 * kFlowSplitMax * 128;
// workgroups launch_flow_lm_split would use for an edge count (1: no split); MMT_LM_SPLIT=0
// disables the split, MMT_LM_SPLIT=<g> forces g workgroups
int flow_split_groups(int n_hint);
void launch_flow_lm_split(const FlowSolveDesc* d_desc, int groups, hipStream_t st);

void launch_gray_depth(const uint8_t* bgr, size_t bgr_pitch, const uint16_t* disp,
                       size_t disp_pitch, uint8_t* gray, size_t gray_pitch, float* depth,
                       size_t depth_pitch, int npix, int nframes, float bf, hipStream_t st);
void launch_static_samples(const mmt_kp* kps, const int* nkp, const float* depth,
                           const float2* flow, const int32_t* mask, int W, int H,
                           const SampleSet& out, hipStream_t st);
void launch_obj_samples(const float* depth, const float2* flow, const int32_t* mask, int W,
                        int H, const ObjSampleSet& out, hipStream_t st);
void launch_handoff(const float2* last_corres, const int* n_last, const float2* last_ocorres,
                    const int* n_olast, const float* depth, const int32_t* mask, int W, int H,
                    const HandoffSet& cur, hipStream_t st);
void launch_obj_group(const GroupArgs& a, hipStream_t st);
void launch_flow_lm(const FlowSolveDesc* d_descs, int nsolves, int n_hint, hipStream_t st);
size_t flow_scratch_doubles(int cap);

// D1: Optimizer::PoseOptimization on one frame's MapPoint observations (at most 2048 edges).
struct PoseOptDesc {
  int n;
  const float* Xw;          // n x 3
  const float* obs;         // n x (u, v, uR); uR < 0: mono edge
  const float* inv_sigma2;  // n
  float Tcw[16];
  double fx, fy, cx, cy, bf;
  float* pose_out;
  uint8_t* outlier;         // n: mvbOutlier
  int* n_inliers;
  // n > kPoseOptMaxEdges: per-edge errors (3 n doubles) and flags (n ints) in global memory
  double* e_scratch;
  int* f_scratch;
};
constexpr int kPoseOptMaxEdges = 2048;  // edges whose state fits the kernel's LDS
void launch_pose_opt(const PoseOptDesc* d_descs, int nsolves, int n_max, hipStream_t st);

}  // namespace mmt
