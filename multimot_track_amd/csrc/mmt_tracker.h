// multimot_track_amd/csrc/mmt_tracker.h -- host tracker state (one sequence per context).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <deque>
#include <string>
#include <vector>

#include "mmt_internal.h"
#include "mmt_map.h"
#include "mmt_pnp.h"
#include "mmt_track.h"

namespace mmt {

// objects solved per frame: one per semantic label 1..15 (label 0 is the static background), so
// every object the grouping keeps is solved (the reference has no cap)
constexpr int kMaxObj = kMaxLabel - 1;
constexpr int kRansacIters = 500;  // solvePnPRansac iterationsCount (Tracking.cc:4361)

struct ObjOut {
  int label = 0, sem_label = 0, n_points = 0, n_ransac_inliers = 0, n_mm_inliers = -1;
  int ransac_iterations = 0, n_solve = 0, n_inliers = 0, iterations = 0;
  float init[16], X[16], motion[16];
  float centre_pre[3] = {0, 0, 0};  // ObjCentre3D_pre (Tracking.cc:2032-2049)
};

struct FrameOut {
  bool initialized = false;
  float Tcw[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  int n_keys = 0, n_obj_samples = 0, ego_iterations = 0, ego_inliers = 0;
  std::vector<ObjOut> objects;
  MapStatsH map;
  long seq = -1;        // the frame's index in the sequence (frames tracked since the reset)
  long obj_seq = -1;    // the frame whose object motions `objects` holds (deferred mode: an
                        // earlier one, or -1 for none); = seq otherwise
  bool obj_pending = false;  // deferred record: the frame's object path has not finished yet
};

float rng_first_gaussian(uint64_t seed);

// device side of object stage B (mmt_tracker.hip)
struct MMPrepArgs {
  PnPObject* objs;
  int nobj;
  int pre[kMaxObj];        // PreObjID per object (-1: no motion model)
  const float* prevX;      // previous frame's D3 poses (16 per object)
  const int* prevStats;    // previous frame's D3 stats (3 per object)
  float TcwPrev[16], TcwCur[16];
};
void launch_obj_mm_prep(const MMPrepArgs& a, hipStream_t st);
// the four kernels of stage B (motion-model matrix and inliers, model choice, D3 edge list) as
// one launch, one workgroup per object
void launch_obj_stage_b(const MMPrepArgs& a, FlowSolveDesc* descs, float* init, hipStream_t st);
void launch_obj_model_choice(PnPObject* objs, int nobj, FlowSolveDesc* descs, float* init,
                             hipStream_t st);
// RANSACPointSetRegistrator::getSubset draws (5-point subsets) for a point count.
void ransac_subsets(int count, int iters, std::vector<int>& idx);

class Tracker {
 public:
  ~Tracker();
  void setup(const mmt_config& cfg, OrbEngine* engine, int max_chunk);
  void reset();
  // Deferred object results: a call returns every frame's ego pose and map state, and the object
  // motions of the frames whose object path has finished, oldest first (FrameOut::obj_seq), so the
  // object pipeline keeps running across calls instead of draining at the end of each.
  // flush_deferred finishes the pipeline and returns the remaining records.
  void set_deferred(bool on);
  bool deferred() const { return defer_; }
  void flush_deferred(std::vector<FrameOut>& outs);
  // Frames of one sequence, device-resident, processed in order (ORB batched over the chunk).
  void track_chunk(const uint8_t* d_bgr, size_t bgr_pitch, const uint16_t* d_disp,
                   size_t disp_pitch, const float* d_flow, size_t flow_pitch,
                   const int32_t* d_mask, size_t mask_pitch, int nframes,
                   std::vector<FrameOut>& outs, hipStream_t st);
  int max_chunk() const { return max_chunk_; }
  // HIP events around the batched ORB launch sequence of every chunk (on the launch stream)
  void set_profiling(bool on);
  void read_profile(double* orb_ms, long long* orb_launches, long long* orb_frames, bool reset);
  // last chunk's ORB output (device) for probes
  const mmt_kp* kps() const { return d_kps_; }
  const int* nkp() const { return d_nkp_; }
  int kcap() const { return kcap_; }
  const MappingStats& mapping_stats() const { return map_.mapping_stats(); }
  const MapEngine& map() const { return map_; }
  void set_cull_ratio(double r) { map_.set_cull_ratio(r); }
  void set_vocabulary(Vocabulary* v) { map_.set_vocabulary(v); }
  const BowStatsH& bow_stats() const { return map_.bow_stats(); }
  long split_fallbacks() const { return split_fallbacks_; }
  // the last tracked frame's static samples (mvSiftKeys) and object samples (mvObjKeys,
  // vSemObjLabel), copied to the host (visualisation hook); counts clipped to the caps
  void frame_samples(float* sxy, int scap, int* ns, float* oxy, int32_t* olab, int ocap, int* no,
                     hipStream_t st);

 private:
  struct FrameSlot {
    SampleSet st;
    ObjSampleSet ob;
    HandoffSet ho;
    float Tcw[16];
    // the frame's pose as its successor sees it (mLastFrame.mTcw): UpdateLastFrame resets it to
    // Tlr * Tref (Tracking.cc:2900); the successor's flow solve, scene flow and object solves read
    // it, while this frame's own object path keeps Tcw
    float Tview[16];
    MapFrameH m;  // Frame's map fields (mnId, mvpMapPoints, mvbOutlier, mpReferenceKF, keys)
    bool bSecond = false;  // bSecondFrame as of this frame (label association, B8)
    int obj_slot = -1;     // object-pipeline slot of this frame's D3 output (-1: none)
    std::vector<int> nModLabel, nSemPosition;
    std::vector<std::vector<float>> vObjMod;
  };
  // Object work of one frame.  Stage A (grouping, B7/B8 on the host, PnP-RANSAC on oa_) needs
  // the frame's pose and the previous frame's labels; stage B (motion-model matrix from the
  // previous frame's D3 output, MM check, model choice, D3 on ob_) runs entirely on the device,
  // ordered behind the RANSAC by an event and behind the previous frame's D3 by the stream, so the
  // host enqueues both stages at once and only reads the results obj_lag_ frames later (finish).
  struct ObjFrame {
    bool active = false;
    bool a_launched = false;  // obj_stage_a_launch ran
    int cur = 0, last = 0, slot = 0, nobj = 0;
    FrameOut* out = nullptr;
    std::vector<int> labels, LabId, PreObjID, members;
    PnPObject* po = nullptr;  // oh_[slot]->po
  };
  struct FrameArgs {
    const float* depth;
    const float2* flow;
    const int32_t* mask;
    const mmt_kp* kps;
    const int* nkp;
    int n_keys;
    int f;    // index in the chunk
    int buf;  // host chunk buffer of the frame's map arrays
  };
  // One object's PnP buffers in one object slot: what stage B and D3 read after the RANSAC (the
  // gathered correspondences, the inlier lists, the D3 edge list and the results).
  struct PnPBuf {
    float* pts3;
    float2* pts2;
    int* inliers;
    int* mm_inliers;
    int* subset;
    int* n_subset;
    int* result;
    double* Rt;
  };
  template <typename T>
  T* alloc(size_t n);
  // ego part of a frame: samples, hand-off, D2 launched on `st` (no wait)
  void ego_launch(const FrameArgs& a, FrameOut& out, hipStream_t st);
  // waits for the ego solve, updates the motion model, queues the frame's object path
  void ego_map_finish(FrameOut& out);
  void ego_finish(FrameOut& out, hipStream_t st);
  void obj_stage_a(ObjFrame& F);    // grouping + B7/B8 + PnP-RANSAC launch (stream oa_)
  void obj_stage_a_launch(ObjFrame& F);  // its first half: the grouping kernel and its read-back
  void obj_stage_a_decide(ObjFrame& F);  // its second half: B7/B8 on the host, the RANSAC launch
  void obj_stage_b(ObjFrame& F);    // MM matrix, MM check, model choice, D3 (stream ob_, no wait)
  void obj_finish(ObjFrame& F);     // waits for the frame's D3, object motions, results
  void obj_advance();               // enqueue the queued frame's object path, finish old frames
  void obj_flush();

  mmt_config cfg_{};
  OrbEngine* engine_ = nullptr;
  // map tracking (ORB-SLAM2's TrackWithMotionModel / TrackLocalMap / keyframes), the frame grid
  // (B3) of every chunk frame on the device and its host copy (two chunk buffers: the first frame
  // of a chunk reads the last frame of the previous one)
  MapEngine map_;
  GridFrame grid0_{};  // camera, bounds and scales of every frame's GridFrame
  float* d_uR_ = nullptr;
  float* d_kdepth_ = nullptr;
  int* d_cell_start_ = nullptr;
  int* d_cell_idx_ = nullptr;
  struct HostChunk {
    mmt_kp* kps = nullptr;
    uint8_t* desc = nullptr;
    float* uR = nullptr;
    float* kdepth = nullptr;
    int* nkp = nullptr;  // [max_chunk] key counts, then the ORB error word
    B3HostOut dev;       // the same buffers as the device addresses them (k_stereo_grid writes)
  };
  HostChunk hc_[2];
  int chunk_buf_ = 0;
  bool reset_pending_ = false;  // System::Reset requested (LOST with <= 5 keyframes)
  int W_ = 0, H_ = 0, max_chunk_ = 0, kcap_ = 0, ocap_ = 0, lm_cap_ = 0, mask_words_ = 0;
  float g0_ = 0;
  int state_ = 0, cur_ = 0, last_ = 2;
  bool bFirstFrame_ = false, bSecondFrame_ = false, hasVelocity_ = false;
  float V_[16] = {0};
  // frame slots: the ego frame, the frames whose object path is in flight (up to obj_lag_ + 1) and
  // their last frames.  A frame's D3 reads its last frame's slot until the frame is finished,
  // obj_lag_ + 1 frames later, after that iteration's ego path has written its own slot: the
  // slot count must exceed obj_lag_ + 2.
  static constexpr int kSlots = 22;
  // object-pipeline buffers: at least the frames in flight (obj_lag_ + 1) plus one
  static constexpr int kObjSlots = 18;
  static constexpr int kObjLagMax = kObjSlots - 2;
  // frames between enqueueing a frame's D3 and reading it (1..kObjLagMax)
  int obj_lag_ = 16;
  int d3_iters_ = 200;  // PoseOptimizationFlow2's optimize(200) (Optimizer.cc:2292)
  FrameSlot slot_[kSlots];
  // ego in flight; its device->host results land in pinned memory so the copies stay
  // asynchronous while the host drives the previous frame's object path
  struct EgoHost {
    FlowSolveDesc d2;
    float Tcw[16];
    int st[3];
    int nlast_obj;
    int n_static[3];
  };
  bool ego_pending_ = false;
  float ego_Tinit_[16];
  EgoHost* eh_ = nullptr;
  ObjFrame qa_;                  // ego done, object path not yet enqueued
  bool defer_ = false;
  long frame_seq_ = 0;           // frames tracked since the reset
  std::deque<FrameOut> dq_;      // deferred object records, frame order (stable addresses)
  void deliver_deferred(std::vector<FrameOut>& outs, bool all);
  std::deque<ObjFrame> inflight_;  // object path enqueued, results not yet read
  int obj_slot_next_ = 0;
  // Pinned host side of the object path, one per object slot: every host<->device transfer of the
  // stages and the finish is a single asynchronous copy into or out of this block.
  // Everything the finish reads from the device: one block per object slot, written by the
  // RANSAC, stage B and D3 kernels and brought back with a single copy behind the D3 launch
  // (small copies cost a queue round trip each on the critical D3 stream).
  struct ObjResults {
    int res[8 * kMaxObj];      // PnP results of all objects
    float init[16 * kMaxObj];  // chosen D3 initial motion per object
    float X[16 * kMaxObj];     // D3 poses
    int lst[3 * kMaxObj];      // D3 stats
    int nsub[kMaxObj];
    float centre[3 * kMaxObj];  // ObjCentre3D_pre per object (D3 kernel output)
  };
  struct ObjHost {
    LabelStats stats[kMaxLabel];
    int hist[kMaxLabel * kMaxLabel];
    int err;
    PnPObject po[kMaxObj];
    int subsets[kMaxObj][5 * kRansacIters];
    FlowSolveDesc descs[kMaxObj];
    ObjResults r;
  };
  static constexpr size_t kObjStatsBytes = sizeof(LabelStats) * kMaxLabel + sizeof(int) * kMaxLabel * kMaxLabel;
  static constexpr size_t kObjPnpBytes = sizeof(PnPObject) * kMaxObj + sizeof(int) * kMaxObj * 5 * kRansacIters;
  ObjHost* oh_[kObjSlots] = {};
  ObjResults* d_r_[kObjSlots] = {};
  double* d_Rt_[kObjSlots] = {};
  FlowSolveDesc* d_descs3_[kObjSlots] = {};  // D3 solves of the slot's frame
  hipEvent_t ev_ransac_[kObjSlots] = {};
  hipEvent_t ev_grp_[kObjSlots] = {};  // the grouping statistics are on the host
  hipEvent_t ev_d3_[kObjSlots] = {};
  // subset draws depend only on the point count: cache the last few counts
  struct SubsetCache {
    int count = -1;
    std::vector<int> idx;
  };
  SubsetCache subset_cache_[16];
  int subset_cache_next_ = 0;
  const std::vector<int>& cached_subsets(int count);
  hipStream_t oa_ = nullptr, ob_ = nullptr;
  std::vector<void*> allocs_;
  float* d_depth_ = nullptr;
  mmt_kp* d_kps_ = nullptr;
  uint8_t* d_desc_ = nullptr;
  int* d_nkp_ = nullptr;
  int32_t* d_obj_label_[kObjSlots] = {};
  int* d_members_[kObjSlots] = {};
  LabelStats* d_stats_[kObjSlots] = {};
  int* d_hist_[kObjSlots] = {};
  int* d_err_ = nullptr;
  double* d_lm_scratch_ = nullptr;
  FlowSolveDesc* d_descs_ = nullptr;
  float* d_poses_ = nullptr;
  int* d_lmstats_ = nullptr;
  unsigned long long* d_gx_ = nullptr;  // the split ego solve's exchange granules
  unsigned gx_seq_ = 0;
  long split_fallbacks_ = 0;  // D2 split solves re-run on one workgroup (residency not met)
  unsigned long long split_spin_ = 0;  // MMT_DEBUG_SPLIT_SPIN (0: the kernel's 0.1 s)
  PnPObject* d_pnp_[kObjSlots] = {};
  PnPBuf pnp_[kObjSlots][kMaxObj];
  // The RANSAC-only scratch of an object index (subset draws, hypothesis records and models,
  // inlier counts and masks), shared by the object slots: only the RANSAC kernels touch it, and
  // they all run on oa_, so stream order keeps one frame's RANSAC off another's scratch.
  struct PnPScratch {
    double* models;
    double* hrec;
    double* hout;
    int* good;
    unsigned long long* masks;
  };
  PnPScratch pnp_scr_[kMaxObj];
  bool prof_ = false;
  bool map_finish_pending_ = false;
  // MMT_MAP_PROFILE: host wall time per frame in obj_advance / ego_launch / ego_finish
  bool hprof_ = false;
  double hprof_us_[7] = {0, 0, 0, 0, 0, 0, 0};  // + map finish, stage A, stage B, obj finish
  long hprof_n_ = 0;
  hipEvent_t ev_orb_[2] = {nullptr, nullptr};
  bool obj_ran_ = false;
  int device_ = 0;
  double orb_ms_ = 0;
  long long orb_launches_ = 0, orb_frames_ = 0;
};

}  // namespace mmt
