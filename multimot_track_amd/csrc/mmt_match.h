// multimot_track_amd/csrc/mmt_match.h -- device records of the frame grid (B3) and the projection
// matchers (C1-C3): Frame::ComputeStereoFromRGBD / AssignFeaturesToGrid / GetFeaturesInArea /
// isInFrustum, ORBmatcher::DescriptorDistance / SearchByProjection (reference Frame.cc,
// ORBmatcher.cc).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mmt.h"

namespace mmt {

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.h:37-38)
constexpr int kGridCells = kGridCols * kGridRows;
constexpr int kCandK = 8;              // candidates kept per point (sorted by distance, order)
constexpr int kMaxMatchKeys = 16384;   // current-frame keys a matcher accepts (LDS bitmap)
constexpr int kMaxLevels = 16;  // mmt_create accepts orb_nlevels <= 16

// One frame as the matchers read it (Frame's mvKeysUn, mDescriptors, mvuRight, mGrid).
struct GridFrame {
  const mmt_kp* keys;
  const uint8_t* desc;   // n x 32
  const float* uR;       // mvuRight (B3)
  const int* cell_start; // kGridCells + 1, cells ix * kGridRows + iy (CSR)
  const int* cell_idx;   // n, ascending key order inside a cell
  int n;
  float fx, fy, cx, cy, bf;
  float minX, maxX, minY, maxY, invW, invH;
  float scale[kMaxLevels];
  float logScale;
  int nlevels;
};

// A point's search window (GetFeaturesInArea arguments + the stereo check) for rescans.
struct PointWin {
  float x, y, r, ur, er;
  int minLevel, maxLevel, pad;
};

struct FrustumRec {  // isInFrustum outputs (MapPoint::mTrack* fields)
  int in_view, level;
  float u, v, uR, view_cos;
};

struct LocalPointDev {  // a local MapPoint: position, normal, distance invariance, state
  float Xw[3];
  float normal[3];
  float min_dist, max_dist;
  int skip;  // mnLastFrameSeen == frame (already matched) or isBad()
  int pad[3];
};

// Candidates of one matcher call: per point kCandK (dist << 20 | order) keys + key indices,
// the number of candidates that passed the filters (-1: point inactive) and its window.
struct CandSet {
  uint32_t* key;
  int* idx;
  int* n;
  PointWin* win;
  int* choice;  // per point: the binding the order-dependent pass settles on (scratch)
};

// B3 for nframes frames: keys/uR/kdepth/cell_idx at frame stride `cap`, cell_start at
// kGridCells + 1, depth map at depth_pitch floats.
// Optional host outputs of B3 (device-accessible pinned buffers at the same frame stride `cap`):
// keys, descriptors (read from ddesc), uR, depths of the valid entries, nkp[0..nframes) and, at
// nkp[nframes], the word at err_src (the ORB engine's error flags).
struct B3HostOut {
  mmt_kp* kps;
  uint8_t* desc;
  float* uR;
  float* kdepth;
  int* nkp;
  const uint8_t* ddesc;
  const int* err_src;
};
// the LDS budget of the grid build's cell lists (larger capacities sort in HBM)
constexpr size_t kStereoGridLds = 48 * 1024;
void launch_stereo_grid(const mmt_kp* keys, const int* nkp, int cap, const float* depth,
                        size_t depth_pitch, int W, int H, float bf, float invW, float invH,
                        float* uR, float* kdepth, int* cell_start, int* cell_idx, int nframes,
                        hipStream_t st, const B3HostOut* ho = nullptr);

// C2: SearchByProjection(Frame&, const Frame&, th, bMono) candidates + greedy replay.
struct LastFrameDev {
  const mmt_kp* keys;
  const float* Xw;          // n x 3
  const uint8_t* mp_desc;   // n x 32
  const uint8_t* active;    // MapPoint present and not an outlier
  // MapPoint::Observations() > 0 (null: all).  A key bound to a point without observations (a
  // temporal VO point of UpdateLastFrame) stays open to later points (ORBmatcher.cc:2033-2035).
  const uint8_t* obs;
  int n;
  float Tcw[16];
};
struct MapEdgeArgs;
// run_if (optional): the call runs only while *run_if < run_lt (C2's retry at a wider window when
// the first search found too few matches), decided on the device.  edges (optional): the matcher
// kernel also builds D1's edge list from its final bindings (k_map_edges' work, no launch of its
// own); a call that does not run leaves the previous call's list.
void launch_sbp_frame(const GridFrame& C, const float* Tcw, const LastFrameDev& L, float th,
                      int mono, int check_orientation, const CandSet& cs, int* match,
                      int* nmatches, hipStream_t st, const int* run_if = nullptr,
                      int run_lt = 0, const MapEdgeArgs* edges = nullptr);

// C3: SearchLocalPoints' isInFrustum pass + SearchByProjection(Frame&, vector<MapPoint*>, th).
// ids (null: point j is pts[j]) selects the local points from a resident pool, skip (null: the
// pool record's own flag) overrides their skip flag; fr (optional) receives the isInFrustum
// records, inview (optional) one byte per point.
struct LocalSel {
  const int* ids;
  const uint8_t* skip;
  uint8_t* inview;
};
void launch_search_local(const GridFrame& C, const float* Tcw, const LocalPointDev* pts,
                         const uint8_t* pdesc, int m, float th, const uint8_t* taken,
                         FrustumRec* fr, const CandSet& cs, int* match, int* nmatches,
                         hipStream_t st, const LocalSel* sel = nullptr,
                         const MapEdgeArgs* edges = nullptr);

// C4: ORBmatcher::SearchByBoW(KeyFrame*, Frame&) with caller-supplied DBoW2 FeatureVectors
// (node ids ascending, per-node feature lists in insertion order, every feature in one node).
struct BowFeatVec {
  int n_nodes;
  const uint32_t* node;
  const int* start;  // n_nodes + 1
  const int* feat;
};
constexpr int kBowMaxNodeFeatures = 64 * 32;  // frame features one node may hold (lane bitmasks)
// match (nF ints) receives the keyframe key index per frame key or -1, hist 30 ints and
// counters 2 ints of scratch; counters[1] = nmatches after the launch.
void launch_search_by_bow(const BowFeatVec& kf, const mmt_kp* kf_keys, const uint8_t* kf_desc,
                          const uint8_t* kf_ok, const BowFeatVec& f, const mmt_kp* f_keys,
                          const uint8_t* f_desc, int nF, float nnratio, int check_orientation,
                          int* match, int* hist, int* counters, hipStream_t st);

// The edge list of Optimizer::PoseOptimization (Optimizer.cc:3160-3230) built on the device from a
// matcher's output, in key order: key i is an edge when match[i] >= 0 (position src_X[match[i]],
// or pool[ids[match[i]]].Xw with a pool) or, without a new match, when has_base[i] (base_X[i]);
// obs = (x, y, uR) of the key, information 1/sigma^2 of its octave.  Nothing is built when
// *nm < min_matches.  X / obs / s2 hold cap edges; desc->n receives the edge count.
struct PoseOptDesc;
struct MapEdgeArgs {
  int n;
  const mmt_kp* keys;
  const float* uR;
  const int* match;
  const int* nm;
  int min_matches;
  const float* src_X;
  const LocalPointDev* pool;
  const int* ids;
  const uint8_t* has_base;
  const float* base_X;
  float inv_sigma2[kMaxLevels];
  float* X;
  float* obs;
  float* s2;
  PoseOptDesc* desc;
};
void launch_map_edges(const MapEdgeArgs& a, hipStream_t st);

// pool maintenance: scatter n packed (handle, record, descriptor) updates into the pool
struct alignas(16) PoolUpdate {
  int h;
  int pad[3];
  LocalPointDev p;   // offset 16
  uint8_t desc[32];  // offset 64 (16-byte aligned: copied as two uint4)
};
void launch_pool_scatter(const PoolUpdate* up, int n, LocalPointDev* pool, uint8_t* pool_desc,
                         hipStream_t st);

// ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>, th) candidates (ORBmatcher.cc:1200-1324): per
// (keyframe, point) query the best key of the keyframe (Hamming distance, first in
// GetFeaturesInArea order) among those the reference would compare; out[q] = (key, distance), or
// (-1, 256).  The map-changing part of Fuse is the host's.
struct FuseKF {  // one keyframe as Fuse reads it: its Frame grid, keys, mvuRight and pose
  const mmt_kp* keys;
  const uint8_t* desc;
  const float* uR;
  const int* cell_start;
  const int* cell_idx;
  float Tcw[16];
  float Ow[3];
  int n;
};
struct FuseQuery {
  int kft;  // index into the launch's keyframe table
  int h;    // map point (pool record)
};
struct FuseCam {
  float fx, fy, cx, cy, bf, W, H, invW, invH, logScale, th;
  int nlevels;
  float scale[kMaxLevels], invSigma2[kMaxLevels];
};
void launch_fuse_cand(const FuseKF* kfs, const FuseQuery* q, int nq, const LocalPointDev* pool,
                      const uint8_t* pool_desc, const FuseCam& cam, int2* out, hipStream_t st);

}  // namespace mmt
