// multimot_track_amd/csrc/mmt_ba.h -- the solve of Optimizer::LocalBundleAdjustment
// (reference src/Optimizer.cc:3394-3665) on the GPU: a chain of short kernels per LM trial with
// the LM state on the device, or one persistent workgroup (MMT_BA_ONEWG=1) (mmt_ba.hip).  The host (mmt_localmap.hip) builds the graph exactly as the reference does
// (local keyframes, fixed keyframes, points, edges point by point in observation order) and
// applies the results (erase, SetPose, SetWorldPos).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

namespace mmt {

struct BADesc {
  int n_kf, n_pt, n_edge;
  int n_opt;                 // optimised (non-fixed) keyframes
  int n_blk;                 // keyframe-pair blocks of the reduced system (a <= b, optimised indices)
  const float* Tcw;          // n_kf x 16 row-major
  const int* opt_of;         // n_kf: optimised index or -1 (fixed)
  const int* opt_kf;         // n_opt: keyframe vertex of each optimised index
  const float* Xw;           // n_pt x 3
  const int* pt_start;       // n_pt + 1: point j's edges are [pt_start[j], pt_start[j + 1])
  const int* e_pt;           // n_edge
  const int* e_kf;           // n_edge: keyframe vertex
  const float* e_obs;        // n_edge x (u, v, uR); uR < 0: monocular
  const float* e_s;          // n_edge: mvInvLevelSigma2[octave]
  const int* kf_start;       // n_opt + 1 over kf_edges: each optimised keyframe's edges, edge order
  const int* kf_edges;
  const int* blk_ab;         // n_blk x 2
  const int* blk_start;      // n_blk + 1 over trip
  const int2* trip;          // (edge to a, edge to b) of one point, points in order
  float fx, fy, cx, cy, bf;
  double* ws;                // ba_workspace_bytes()
  float* T_out;              // n_kf x 16: Converter::toCvMat of every vertex's final estimate
  float* X_out;              // n_pt x 3
  uint8_t* erase;            // n_edge: the final inlier test failed
  int* stats;                // [iterations r1, r2, trials r1, r2, erased edges]
};

size_t ba_workspace_bytes(int n_kf, int n_pt, int n_edge, int n_opt);

// The graph as LocalBundleAdjustment builds it (Optimizer.cc:3408-3541): keyframe vertices (fixed
// or not), points, and the edges listed point by point (e_pt non-decreasing), each point's
// observations in keyframe order; e_obs uR < 0 marks a monocular edge.
struct BAHostProblem {
  int n_kf = 0, n_pt = 0, n_edge = 0;
  const float* Tcw = nullptr;
  const uint8_t* fixed = nullptr;
  const float* Xw = nullptr;
  const int* e_pt = nullptr;
  const int* e_kf = nullptr;
  const float* e_obs = nullptr;
  const float* e_s = nullptr;
  float fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
};

// Builds the device-side index structures (point CSR, keyframe-major edge lists, Schur triples per
// keyframe-pair block), uploads everything in one copy, runs k_local_ba and downloads the results
// in one copy.  Owns its (growing) device and pinned buffers; one call at a time.
class BARunner {
 public:
  ~BARunner();
  // T_out n_kf x 16, X_out n_pt x 3, erase n_edge, stats 5 (host pointers); synchronous on st
  void run(const BAHostProblem& P, hipStream_t st, float* T_out, float* X_out, uint8_t* erase,
           int* stats);

 private:
  void grow(uint8_t*& d, uint8_t*& h, size_t& cap, size_t need, hipStream_t st);
  uint8_t *d_up_ = nullptr, *h_up_ = nullptr, *d_dn_ = nullptr, *h_dn_ = nullptr;
  size_t up_cap_ = 0, dn_cap_ = 0;
  double* d_ws_ = nullptr;
  size_t ws_cap_ = 0;
  uint8_t* d_ws2_ = nullptr;  // the multi-kernel solve's workspace
  size_t ws2_cap_ = 0;
  int* h_flag_ = nullptr;     // pinned: the solve's done flag
};

size_t ba2_workspace_bytes(int n_kf, int n_pt, int n_edge, int n_opt, int n_blk, int gP);

}  // namespace mmt
