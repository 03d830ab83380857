// multimot_track_amd/csrc/mmt_tracker.hip -- host side of System::TrackRGBD for one sequence.
//
// Mirrors Tracking::GrabImageRGBD / Tracking::Track (reference src/Tracking.cc:438-661, 951-2499)
// and Tracking::StereoInitialization (:2512-2570): every per-pixel / per-sample / per-edge stage
// runs as HIP kernels (mmt_orb.hip, mmt_track.hip, mmt_pnp.hip); the host keeps the scalar
// state machine -- poses, motion model, label bookkeeping (B8), per-object decisions -- exactly
// where the reference keeps it.  The ego initial pose comes from ORB-SLAM2's map tracking
// (mmt_map.hip: TrackWithMotionModel / TrackLocalMap / keyframes on GPU matchers and solves).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mmt_internal.h"
#include "mmt_map.h"
#include "mmt_mat4.h"
#include "mmt_pnp.h"
#include "mmt_track.h"
#include "mmt_tracker.h"

namespace mmt {

// cv::RNG(seed).gaussian(1.0) first draw (randn_0_1_32f ziggurat; Frame.cc:1246-1251)
static inline uint64_t rng_next(uint64_t x) { return (uint64_t)(unsigned)x * 4164903690ULL + (x >> 32); }
float rng_first_gaussian(uint64_t seed) {
  static unsigned kn[128];
  static float wn[128], fn[128];
  static bool init = false;
  if (!init) {
    const double m1 = 2147483648.0;
    double dn = 3.442619855899, tn = dn, vn = 9.91256303526217e-3;
    const double q = vn / std::exp(-.5 * dn * dn);
    kn[0] = (unsigned)((dn / q) * m1);
    kn[1] = 0;
    wn[0] = (float)(q / m1);
    wn[127] = (float)(dn / m1);
    fn[0] = 1.f;
    fn[127] = (float)std::exp(-.5 * dn * dn);
    for (int i = 126; i >= 1; i--) {
      dn = std::sqrt(-2. * std::log(vn / dn + std::exp(-.5 * dn * dn)));
      kn[i + 1] = (unsigned)((dn / tn) * m1);
      tn = dn;
      fn[i] = (float)std::exp(-.5 * dn * dn);
      wn[i] = (float)(dn / m1);
    }
    init = true;
  }
  const float r = 3.442620f, rng_flt = 2.3283064365386962890625e-10f;
  uint64_t temp = seed ? seed : 0xffffffffULL;
  float x, y;
  for (;;) {
    const int hz = (int)temp;
    temp = rng_next(temp);
    const int iz = hz & 127;
    x = hz * wn[iz];
    if ((unsigned)std::abs(hz) < kn[iz]) break;
    if (iz == 0) {
      do {
        x = (unsigned)temp * rng_flt;
        temp = rng_next(temp);
        y = (unsigned)temp * rng_flt;
        temp = rng_next(temp);
        x = (float)(-std::log(x + FLT_MIN) * 0.2904764);
        y = (float)-std::log(y + FLT_MIN);
      } while (y + y < x * x);
      x = hz > 0 ? r + x : -r - x;
      break;
    }
    y = (unsigned)temp * rng_flt;
    temp = rng_next(temp);
    if (fn[iz] + y * (fn[iz - 1] - fn[iz]) < std::exp(-.5 * x * x)) break;
  }
  return x;
}

// RANSACPointSetRegistrator::getSubset draws with RNG((uint64)-1): depends on the count only.
void ransac_subsets(int count, int iters, std::vector<int>& idx) {
  uint64_t state = 0xFFFFFFFFFFFFFFFFULL;
  idx.assign((size_t)iters * 5, 0);
  for (int it = 0; it < iters; it++) {
    int* cur = &idx[(size_t)it * 5];
    for (int i = 0; i < 5; i++)
      for (;;) {
        state = (uint64_t)(unsigned)state * 4164903690ULL + (unsigned)(state >> 32);
        const int v = (int)((unsigned)state % (unsigned)count);
        cur[i] = v;
        int j = 0;
        for (; j < i; j++)
          if (v == cur[j]) break;
        if (j == i) break;
      }
  }
}

const std::vector<int>& Tracker::cached_subsets(int count) {
  for (SubsetCache& c : subset_cache_)
    if (c.count == count) return c.idx;
  SubsetCache& c = subset_cache_[subset_cache_next_];
  subset_cache_next_ = (subset_cache_next_ + 1) % 16;
  c.count = count;
  ransac_subsets(count, kRansacIters, c.idx);
  return c.idx;
}

template <typename T>
static T* dalloc(size_t n) {
  T* p = nullptr;
  MMT_HIP(hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T)));
  return p;
}

Tracker::~Tracker() {
  if (hprof_ && hprof_n_ > 0)
    fprintf(stderr, "[mmt tracker profile] %ld frames, host wall us per frame: map finish + obj_advance %.1f, "
            "ego_launch %.1f, ego_finish %.1f\n", hprof_n_, hprof_us_[0] / hprof_n_,
            hprof_us_[1] / hprof_n_, hprof_us_[2] / hprof_n_);
  if (hprof_ && hprof_n_ > 0)
    fprintf(stderr, "[mmt tracker profile] of which: map finish %.1f, object stage A %.1f, "
            "stage B %.1f, object results %.1f\n", hprof_us_[3] / hprof_n_,
            hprof_us_[4] / hprof_n_, hprof_us_[5] / hprof_n_, hprof_us_[6] / hprof_n_);
  for (hipStream_t* q : {&oa_, &ob_})
    if (*q) {
      (void)hipStreamSynchronize(*q);
      (void)hipStreamDestroy(*q);
    }
  for (void* p : allocs_) (void)hipFree(p);
  if (eh_) (void)hipHostFree(eh_);
  for (ObjHost* h : oh_)
    if (h) (void)hipHostFree(h);
  for (HostChunk& h : hc_)
    for (void* p : {(void*)h.kps, (void*)h.desc, (void*)h.uR, (void*)h.kdepth, (void*)h.nkp})
      if (p) (void)hipHostFree(p);
  for (int q = 0; q < kObjSlots; q++) {
    if (ev_ransac_[q]) (void)hipEventDestroy(ev_ransac_[q]);
    if (ev_grp_[q]) (void)hipEventDestroy(ev_grp_[q]);
    if (ev_d3_[q]) (void)hipEventDestroy(ev_d3_[q]);
  }
  for (hipEvent_t& e : ev_orb_)
    if (e) (void)hipEventDestroy(e);
}

void Tracker::set_profiling(bool on) {
  if (on && !ev_orb_[0]) {
    MMT_HIP(hipEventCreate(&ev_orb_[0]));
    MMT_HIP(hipEventCreate(&ev_orb_[1]));
  }
  prof_ = on;
}

void Tracker::read_profile(double* orb_ms, long long* orb_launches, long long* orb_frames,
                           bool reset) {
  *orb_ms = orb_ms_;
  *orb_launches = orb_launches_;
  *orb_frames = orb_frames_;
  if (reset) {
    orb_ms_ = 0;
    orb_launches_ = orb_frames_ = 0;
  }
}

template <typename T>
T* Tracker::alloc(size_t n) {
  T* p = dalloc<T>(n);
  allocs_.push_back(p);
  return p;
}

void Tracker::setup(const mmt_config& cfg, OrbEngine* engine, int max_chunk) {
  cfg_ = cfg;
  hprof_ = getenv("MMT_MAP_PROFILE") != nullptr;
  engine_ = engine;
  W_ = cfg.width;
  H_ = cfg.height;
  max_chunk_ = max_chunk;
  g0_ = rng_first_gaussian(cfg.noise_seed);
  kcap_ = engine->capacity();
  ocap_ = ((W_ + 3) / 4) * ((H_ + 3) / 4);
  const size_t npix = (size_t)W_ * H_;
  d_depth_ = alloc<float>(npix * max_chunk);
  d_kps_ = alloc<mmt_kp>((size_t)kcap_ * max_chunk);
  d_desc_ = alloc<uint8_t>((size_t)kcap_ * 32 * max_chunk);
  d_nkp_ = alloc<int>(max_chunk);
  for (int s = 0; s < kSlots; s++) {
    FrameSlot& F = slot_[s];
    F.st.keys = alloc<float2>(kcap_);
    F.st.corres = alloc<float2>(kcap_);
    F.st.flow = alloc<float2>(kcap_);
    F.st.depth = alloc<float>(kcap_);
    F.st.count = alloc<int>(1);
    F.st.cap = kcap_;
    F.ob.keys = alloc<float2>(ocap_);
    F.ob.corres = alloc<float2>(ocap_);
    F.ob.flow = alloc<float2>(ocap_);
    F.ob.depth = alloc<float>(ocap_);
    F.ob.label = alloc<int32_t>(ocap_);
    F.ob.count = alloc<int>(1);
    F.ob.cap = ocap_;
    F.ob.block_counts = alloc<int>(64);
    F.ho.skeys = alloc<float2>(kcap_);
    F.ho.sdepth = alloc<float>(kcap_);
    F.ho.ns = alloc<int>(1);
    F.ho.okeys = alloc<float2>(ocap_);
    F.ho.odepth = alloc<float>(ocap_);
    F.ho.olabel = alloc<int32_t>(ocap_);
    F.ho.no = alloc<int>(1);
    MMT_HIP(hipMemset(F.st.count, 0, sizeof(int)));
    MMT_HIP(hipMemset(F.ob.count, 0, sizeof(int)));
  }
  static_assert(offsetof(ObjHost, hist) == offsetof(ObjHost, stats) + sizeof(LabelStats) * kMaxLabel &&
                    offsetof(ObjHost, err) - offsetof(ObjHost, stats) == kObjStatsBytes,
                "ObjHost: stats, hist contiguous (one download)");
  static_assert(offsetof(ObjHost, subsets) == offsetof(ObjHost, po) + sizeof(PnPObject) * kMaxObj &&
                    sizeof(ObjHost::subsets) == sizeof(int) * kMaxObj * 5 * kRansacIters,
                "ObjHost: po, subsets contiguous (one upload)");
  for (int q = 0; q < kObjSlots; q++) {
    d_obj_label_[q] = alloc<int32_t>(ocap_);
    d_members_[q] = alloc<int>((size_t)kMaxLabel * ocap_);
    // the grouping statistics and the label histogram in one block laid out as ObjHost's, brought
    // back by one copy
    d_stats_[q] = (LabelStats*)alloc<uint8_t>(kObjStatsBytes);
    d_hist_[q] = (int*)((uint8_t*)d_stats_[q] + sizeof(LabelStats) * kMaxLabel);
  }
  d_err_ = alloc<int>(1);
  MMT_HIP(hipMemset(d_err_, 0, sizeof(int)));
  // solves: 1 ego + up to kMaxObj objects.  An object solve has at most ocap_ edges (its
  // samples), the ego solve at most kcap_, so no solve is ever truncated to the scratch capacity
  const int lmcap = std::max(kcap_, ocap_);
  lm_cap_ = lmcap;
  // scratch: the ego solve (caller stream) and the object solves (ob_, one D3 launch at a time)
  d_lm_scratch_ = alloc<double>(flow_scratch_doubles(lmcap) * (1 + kMaxObj));
  d_descs_ = alloc<FlowSolveDesc>(1);
  // D2's pose and stats in one block, brought back by one copy into EgoHost::Tcw / st
  static_assert(offsetof(EgoHost, st) == offsetof(EgoHost, Tcw) + 16 * sizeof(float),
                "EgoHost::st must follow Tcw");
  d_poses_ = alloc<float>(20);
  d_lmstats_ = (int*)(d_poses_ + 16);
  d_gx_ = alloc<unsigned long long>(kFlowSplitGranules);
  MMT_HIP(hipMemset(d_gx_, 0, sizeof(unsigned long long) * kFlowSplitGranules));
  // PnP
  mask_words_ = (ocap_ + 63) / 64;
  for (int q = 0; q < kObjSlots; q++) {
  // the PnP records and the RANSAC subset draws in one block laid out as ObjHost's po / subsets,
  // uploaded by one copy
  d_pnp_[q] = (PnPObject*)alloc<uint8_t>(kObjPnpBytes);
  d_r_[q] = alloc<ObjResults>(1);
  d_Rt_[q] = alloc<double>(12 * kMaxObj);
  d_descs3_[q] = alloc<FlowSolveDesc>(kMaxObj);
  if (!oh_[q]) MMT_HIP(hipHostMalloc((void**)&oh_[q], sizeof(ObjHost), hipHostMallocDefault));
  memset(oh_[q], 0, sizeof(ObjHost));
  if (!ev_ransac_[q]) MMT_HIP(hipEventCreateWithFlags(&ev_ransac_[q], hipEventDisableTiming));
  if (!ev_grp_[q]) MMT_HIP(hipEventCreateWithFlags(&ev_grp_[q], hipEventDisableTiming));
  if (!ev_d3_[q]) MMT_HIP(hipEventCreateWithFlags(&ev_d3_[q], hipEventDisableTiming));
  for (int o = 0; o < kMaxObj; o++) {
    PnPBuf& b = pnp_[q][o];
    b.pts3 = alloc<float>(3 * (size_t)ocap_);
    b.pts2 = alloc<float2>(ocap_);
    b.inliers = alloc<int>(ocap_);
    b.mm_inliers = alloc<int>(ocap_);
    b.subset = alloc<int>(ocap_);
    b.n_subset = d_r_[q]->nsub + o;
    b.result = d_r_[q]->res + 8 * o;
    b.Rt = d_Rt_[q] + 12 * o;
  }
  }
  for (int o = 0; o < kMaxObj; o++) {
    PnPScratch& r = pnp_scr_[o];
    r.models = alloc<double>(6 * kRansacIters);
    r.hrec = alloc<double>((size_t)kHypRec * kRansacIters);
    r.hout = alloc<double>((size_t)3 * kHypOut * kRansacIters);
    r.good = alloc<int>(kRansacIters);
    r.masks = alloc<unsigned long long>((size_t)kRansacIters * mask_words_);
  }
  // ---- map tracking: B3 grids of the chunk on the device, their host copies, the map engine
  d_uR_ = alloc<float>((size_t)kcap_ * max_chunk);
  d_kdepth_ = alloc<float>((size_t)kcap_ * max_chunk);
  d_cell_start_ = alloc<int>((size_t)(kGridCells + 1) * max_chunk);
  d_cell_idx_ = alloc<int>((size_t)kcap_ * max_chunk);
  for (HostChunk& h : hc_) {
    if (!h.kps) {
      MMT_HIP(hipHostMalloc((void**)&h.kps, sizeof(mmt_kp) * (size_t)kcap_ * max_chunk,
                            hipHostMallocDefault));
      MMT_HIP(hipHostMalloc((void**)&h.desc, 32 * (size_t)kcap_ * max_chunk,
                            hipHostMallocDefault));
      MMT_HIP(hipHostMalloc((void**)&h.uR, sizeof(float) * (size_t)kcap_ * max_chunk,
                            hipHostMallocDefault));
      MMT_HIP(hipHostMalloc((void**)&h.kdepth, sizeof(float) * (size_t)kcap_ * max_chunk,
                            hipHostMallocDefault));
      MMT_HIP(hipHostMalloc((void**)&h.nkp, sizeof(int) * ((size_t)max_chunk + 1),
                            hipHostMallocDefault));
      memset(&h.dev, 0, sizeof(h.dev));
      MMT_HIP(hipHostGetDevicePointer((void**)&h.dev.kps, h.kps, 0));
      MMT_HIP(hipHostGetDevicePointer((void**)&h.dev.desc, h.desc, 0));
      MMT_HIP(hipHostGetDevicePointer((void**)&h.dev.uR, h.uR, 0));
      MMT_HIP(hipHostGetDevicePointer((void**)&h.dev.kdepth, h.kdepth, 0));
      MMT_HIP(hipHostGetDevicePointer((void**)&h.dev.nkp, h.nkp, 0));
    }
  }
  {
    OrbTables t;
    t.init(cfg.orb_nfeatures, cfg.orb_scale_factor, cfg.orb_nlevels, cfg.orb_ini_th_fast,
           cfg.orb_min_th_fast);
    if (t.nlevels > kMaxLevels) throw ArgError("too many pyramid levels for the matchers");
    MapCamH mc;
    mc.W = W_;
    mc.H = H_;
    mc.fx = cfg.fx; mc.fy = cfg.fy; mc.cx = cfg.cx; mc.cy = cfg.cy; mc.bf = cfg.bf;
    mc.invfx = 1.0f / cfg.fx;
    mc.invfy = 1.0f / cfg.fy;
    mc.thDepth = cfg.bf * cfg.th_depth / cfg.fx;  // mbf * (float)ThDepth / fx (Tracking.cc:225)
    mc.maxFrames = (int)(cfg.fps == 0.f ? 30.f : cfg.fps);
    mc.nlevels = t.nlevels;
    mc.scale = t.scale;
    mc.invSigma2 = t.invSigma2;
    // mfLogScaleFactor = log(mfScaleFactor), as log in double rounded to float
    mc.logScale = (float)std::log((double)t.scale[t.nlevels > 1 ? 1 : 0]);
    map_.setup(mc, kcap_);
    GridFrame& G = grid0_;
    memset(&G, 0, sizeof(G));
    G.fx = cfg.fx; G.fy = cfg.fy; G.cx = cfg.cx; G.cy = cfg.cy; G.bf = cfg.bf;
    // Frame::ComputeImageBounds without distortion + grid element sizes (Frame.cc:581-584, 841)
    G.minX = 0.0f; G.maxX = (float)W_; G.minY = 0.0f; G.maxY = (float)H_;
    G.invW = static_cast<float>(kGridCols) / static_cast<float>(G.maxX - G.minX);
    G.invH = static_cast<float>(kGridRows) / static_cast<float>(G.maxY - G.minY);
    G.nlevels = t.nlevels;
    for (int l = 0; l < t.nlevels; l++) G.scale[l] = t.scale[l];
    G.logScale = mc.logScale;
  }
  // The two object stages run on streams of their own, both at low priority (a priority class
  // other than normal gets a hardware queue of its own; a normal-priority D3 stream shares the ego
  // chain's queue and halves C3).  Measured alternatives (round 3-4): the RANSAC
  // stream confined to every 4th CU and D3 at high priority, chunked C3 895 against 896 frames/s,
  // one frame per call 1.77 against 1.49 ms.
  int lo = 0, hi = 0;
  MMT_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  (void)hi;
  MMT_HIP(hipStreamCreateWithPriority(&oa_, hipStreamNonBlocking, lo));
  MMT_HIP(hipStreamCreateWithPriority(&ob_, hipStreamNonBlocking, lo));
  MMT_HIP(hipHostMalloc((void**)&eh_, sizeof(EgoHost), hipHostMallocDefault));
  memset(eh_, 0, sizeof(EgoHost));
  reset();
  device_ = cfg.device_id;
  // The previous frame's object path runs on this thread inside the first map chain of the frame,
  // while its kernels run (C3 895 -> 905 fps; a worker thread measured slower).
  // obj_lag_ = 16 frames between enqueueing a frame's object path and reading its results: the D3
  // chain's slow stretches no longer stall the host (interleaved A/B 905 / 915 / 920 fps at 2 / 3 /
  // 4, then 932 / 937 / 944 / 950 / 956 at 4 / 6 / 8 / 10 / 14; kObjSlots = 18 caps it at 16)
  static_assert(kSlots > kObjLagMax + 2, "frame slots too few for the object lag");
  // MMT_DEBUG_SPLIT_SPIN: the split ego solve's exchange spin bound in wall-clock ticks (test
  // hook: a tiny bound forces the not-resident status and so the one-workgroup re-run)
  if (const char* ss = getenv("MMT_DEBUG_SPLIT_SPIN")) split_spin_ = strtoull(ss, nullptr, 10);
}

void Tracker::reset() {
  if (oa_) MMT_HIP(hipStreamSynchronize(oa_));
  if (ob_) MMT_HIP(hipStreamSynchronize(ob_));
  if (d_err_) MMT_HIP(hipMemset(d_err_, 0, sizeof(int)));  // a bad label does not outlive a reset
  state_ = 0;
  bFirstFrame_ = false;  // uninitialised member in the reference (Tracking.h:180): pinned false
  bSecondFrame_ = false;
  hasVelocity_ = false;
  cur_ = 0;
  last_ = kSlots - 1;
  ego_pending_ = false;
  qa_ = ObjFrame();
  inflight_.clear();
  obj_slot_next_ = 0;
  dq_.clear();
  frame_seq_ = 0;
  for (FrameSlot& F : slot_) {
    F.nModLabel.clear();
    F.nSemPosition.clear();
    F.vObjMod.clear();
    F.bSecond = false;
    F.obj_slot = -1;
    mat4_eye(F.Tcw);
    mat4_eye(F.Tview);
    F.m = MapFrameH();
  }
  map_.reset();
  reset_pending_ = false;
}

void Tracker::track_chunk(const uint8_t* d_bgr, size_t bgr_pitch, const uint16_t* d_disp,
                          size_t disp_pitch, const float* d_flow, size_t flow_pitch,
                          const int32_t* d_mask, size_t mask_pitch, int nframes,
                          std::vector<FrameOut>& outs, hipStream_t st) {
  if (nframes < 1 || nframes > max_chunk_) throw ArgError("chunk size outside [1, max_batch]");
  const size_t npix = (size_t)W_ * H_;
  // ---- per-frame preparation and batched ORB extraction for the whole chunk
  // A1 + A2 (gray straight into level 0 of the ORB pyramid, depth) and A3-A9: the profiled ORB
  // window (mmt_profile_*) covers both
  if (prof_) MMT_HIP(hipEventRecord(ev_orb_[0], st));
  uint8_t* gray = engine_->level0();
  const size_t gpitch = engine_->pyramid_stride();
  launch_gray_depth(d_bgr, bgr_pitch, d_disp, disp_pitch / sizeof(uint16_t), gray, gpitch,
                    d_depth_, npix, (int)npix, nframes, cfg_.bf, st);
  engine_->run(gray, nframes, gpitch, d_kps_, d_desc_, kcap_, d_nkp_, st);
  if (prof_) MMT_HIP(hipEventRecord(ev_orb_[1], st));
  // B3 (ComputeStereoFromRGBD + AssignFeaturesToGrid) of every frame of the chunk; the same
  // kernel writes the host copies the map bookkeeping reads (keys, descriptors, mvuRight,
  // mvDepth, the key counts and the ORB error word) into pinned memory, valid entries only.  They
  // go to the buffer the last frame does not live in; it becomes the current one only once the
  // chunk's ORB passed its device checks (a failed chunk leaves no trace)
  const int nbuf = chunk_buf_ ^ 1;
  const HostChunk& hc = hc_[nbuf];
  std::vector<int> nkp(nframes);
  {
    B3HostOut ho = hc.dev;
    ho.ddesc = d_desc_;
    ho.err_src = engine_->err_word();
    launch_stereo_grid(d_kps_, d_nkp_, kcap_, d_depth_, npix, W_, H_, cfg_.bf, grid0_.invW,
                       grid0_.invH, d_uR_, d_kdepth_, d_cell_start_, d_cell_idx_, nframes, st,
                       &ho);
    MMT_HIP(hipStreamSynchronize(st));
    engine_->check_flags_value(hc.nkp[nframes], st);  // throws on a tripped octree guard
    std::copy(hc.nkp, hc.nkp + nframes, nkp.begin());
  }
  chunk_buf_ = nbuf;
  if (prof_) {
    float ms = 0;
    MMT_HIP(hipEventElapsedTime(&ms, ev_orb_[0], ev_orb_[1]));
    orb_ms_ += ms;
    orb_launches_ += 1;
    orb_frames_ += nframes;
  }
  outs.assign(nframes, FrameOut());
  // Two chains per sequence: ego (samples, hand-off, D2 of frame f needs frame f-1's pose) on
  // `st`, and objects (grouping, PnP, D3 of frame f need frame f's pose and frame f-1's objects)
  // on ost_.  Frame f's ego solve runs on the GPU while the host drives frame f-1's object path.
  try {
  for (int f = 0; f < nframes; f++) {
    obj_ran_ = false;
    FrameArgs a;
    a.depth = d_depth_ + npix * f;
    a.flow = (const float2*)((const uint8_t*)d_flow + flow_pitch * f);
    a.mask = (const int32_t*)((const uint8_t*)d_mask + mask_pitch * f);
    a.kps = d_kps_ + (size_t)kcap_ * f;
    a.nkp = d_nkp_ + f;
    a.n_keys = nkp[f];
    a.f = f;
    a.buf = chunk_buf_;
    if (hprof_) {
      auto now = [] {
        return std::chrono::duration<double, std::micro>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
      };
      const double t0 = now();
      ego_launch(a, outs[f], st);
      const double t1 = now();
      ego_map_finish(outs[f]);
      hprof_us_[3] += now() - t1;
      if (!obj_ran_) obj_advance();
      const double t2 = now();
      ego_finish(outs[f], st);
      hprof_us_[0] += t2 - t1;
      hprof_us_[1] += t1 - t0;
      hprof_us_[2] += now() - t2;
      hprof_n_++;
      continue;
    }
    // frame f's map branch up to its pose, then its flow solve (D2) on the GPU; while D2 runs the
    // host finishes the map branch (keyframes) and drives frame f-1's object path
    ego_launch(a, outs[f], st);
    ego_map_finish(outs[f]);
    if (!obj_ran_) obj_advance();  // when no map chain took it
    ego_finish(outs[f], st);
  }
  } catch (...) {
    // the inline path: frames still in flight (and the queued one) point into `outs`, which dies
    // with this call; let their device work finish and drop them (the object pipeline restarts)
    if (oa_) (void)hipStreamSynchronize(oa_);
    if (ob_) (void)hipStreamSynchronize(ob_);
    inflight_.clear();
    qa_ = ObjFrame();
    dq_.clear();  // deferred records of frames whose pipeline was dropped
    throw;
  }
  // the chunk's results are complete on return (deferred mode: the finished object records)
  if (!defer_) obj_flush();
  if (defer_) {
    deliver_deferred(outs, false);
  } else {
    for (FrameOut& o : outs) o.obj_seq = o.seq;
  }
}

void Tracker::frame_samples(float* sxy, int scap, int* ns, float* oxy, int32_t* olab, int ocap,
                            int* no, hipStream_t st) {
  *ns = *no = 0;
  if (state_ == 0 && frame_seq_ == 0) return;
  const FrameSlot& L = slot_[last_];
  int c[2] = {0, 0};
  MMT_HIP(hipMemcpyAsync(&c[0], L.st.count, sizeof(int), hipMemcpyDeviceToHost, st));
  MMT_HIP(hipMemcpyAsync(&c[1], L.ob.count, sizeof(int), hipMemcpyDeviceToHost, st));
  MMT_HIP(hipStreamSynchronize(st));
  const int n0 = std::max(0, std::min(c[0], std::min(scap, L.st.cap)));
  const int n1 = std::max(0, std::min(c[1], std::min(ocap, L.ob.cap)));
  if (n0 > 0 && sxy)
    MMT_HIP(hipMemcpyAsync(sxy, L.st.keys, sizeof(float2) * n0, hipMemcpyDeviceToHost, st));
  if (n1 > 0 && oxy)
    MMT_HIP(hipMemcpyAsync(oxy, L.ob.keys, sizeof(float2) * n1, hipMemcpyDeviceToHost, st));
  if (n1 > 0 && olab)
    MMT_HIP(hipMemcpyAsync(olab, L.ob.label, sizeof(int32_t) * n1, hipMemcpyDeviceToHost, st));
  MMT_HIP(hipStreamSynchronize(st));
  *ns = n0;
  *no = n1;
}

void Tracker::set_deferred(bool on) {
  if (on == defer_) return;
  if (!on) {  // results still owed are lost to a caller who turns the mode off: finish them first
    std::vector<FrameOut> drop;
    flush_deferred(drop);
  }
  defer_ = on;
}

// the finished records, oldest first, one per output slot (all: every record, the pipeline
// having been flushed)
void Tracker::deliver_deferred(std::vector<FrameOut>& outs, bool all) {
  size_t f = 0;
  while (!dq_.empty() && !dq_.front().obj_pending && (all || f < outs.size())) {
    if (f == outs.size()) outs.emplace_back();
    outs[f].objects = std::move(dq_.front().objects);
    outs[f].obj_seq = dq_.front().seq;
    dq_.pop_front();
    f++;
  }
  for (; f < outs.size(); f++) {
    outs[f].objects.clear();
    outs[f].obj_seq = -1;
  }
}

void Tracker::flush_deferred(std::vector<FrameOut>& outs) {
  outs.clear();
  if (!defer_) return;
  obj_flush();
  deliver_deferred(outs, true);
}

// Enqueue the queued frame's whole object path (stage A's host decisions need one wait for the
// grouping statistics; stage B is device-ordered), then read the results of frames older than
// obj_lag_.  Called while the next ego solve runs.
void Tracker::obj_advance() {
  obj_ran_ = true;
  auto now = [] {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  const double t0 = hprof_ ? now() : 0;
  double t1 = t0, t2 = t0;
  if (qa_.active) {
    obj_stage_a(qa_);
    if (hprof_) t1 = now();
    obj_stage_b(qa_);
    if (hprof_) t2 = now();
    inflight_.push_back(qa_);
    qa_ = ObjFrame();
  }
  while ((int)inflight_.size() > obj_lag_) {
    obj_finish(inflight_.front());
    inflight_.pop_front();
  }
  if (hprof_) {
    hprof_us_[4] += t1 - t0;
    hprof_us_[5] += t2 - t1;
    hprof_us_[6] += now() - t2;
  }
}

void Tracker::obj_flush() {
  if (qa_.active) {
    obj_stage_a(qa_);
    obj_stage_b(qa_);
    inflight_.push_back(qa_);
    qa_ = ObjFrame();
  }
  while (!inflight_.empty()) {
    obj_finish(inflight_.front());
    inflight_.pop_front();
  }
}

void Tracker::ego_launch(const FrameArgs& a, FrameOut& out, hipStream_t st) {
  if (reset_pending_) {  // System::TrackRGBD -> Tracking::Reset (System.cc:203-211)
    map_.reset();
    state_ = 0;
    reset_pending_ = false;
  }
  FrameSlot& C = slot_[cur_];
  FrameSlot& Ls = slot_[last_];
  out = FrameOut();
  out.seq = frame_seq_++;
  out.n_keys = a.n_keys;
  // ---- the Frame's map fields (Frame ctor: mnId, B3 arrays, empty mvpMapPoints)
  {
    const HostChunk& hc = hc_[a.buf];
    MapFrameH& m = C.m;
    m.id = map_.next_frame_id();
    m.n = a.n_keys;
    m.kps = hc.kps + (size_t)kcap_ * a.f;
    m.desc = hc.desc + 32 * (size_t)kcap_ * a.f;
    m.uR = hc.uR + (size_t)kcap_ * a.f;
    m.depth = hc.kdepth + (size_t)kcap_ * a.f;
    map_.prepare(m);
  }
  C.nModLabel.clear();
  C.nSemPosition.clear();
  C.vObjMod.clear();
  // ---- Frame(RGBD): B2 static samples, B1 object samples
  launch_static_samples(a.kps, a.nkp, a.depth, a.flow, a.mask, W_, H_, C.st, st);
  MMT_HIP(hipMemcpyAsync(&eh_->n_static[cur_], C.st.count, sizeof(int), hipMemcpyDeviceToHost, st));
  launch_obj_samples(a.depth, a.flow, a.mask, W_, H_, C.ob, st);
  // ---- GrabImageRGBD hand-off (B4)
  const bool handoff = bFirstFrame_ || bSecondFrame_;
  if (handoff)
    launch_handoff(Ls.st.corres, Ls.st.count, Ls.ob.corres, Ls.ob.count, a.depth, a.mask, W_, H_,
                   C.ho, st);
  // mCurrentFrame.mvObjKeys: the frame's own samples, or the hand-off once bFirstFrame is set
  MMT_HIP(hipMemcpyAsync(&eh_->nlast_obj, handoff ? Ls.ob.count : C.ob.count, sizeof(int),
                         hipMemcpyDeviceToHost, st));
  // the frame on the device as the matchers (and a keyframe made from it) read it
  GridFrame G = grid0_;
  G.keys = a.kps;
  G.desc = d_desc_ + 32 * (size_t)kcap_ * a.f;
  G.uR = d_uR_ + (size_t)kcap_ * a.f;
  G.cell_start = d_cell_start_ + (size_t)(kGridCells + 1) * a.f;
  G.cell_idx = d_cell_idx_ + (size_t)kcap_ * a.f;
  G.n = a.n_keys;
  map_.set_frame_grid(G);
  if (state_ == 0) {
    ego_pending_ = false;
    return;
  }
  // ---- ORB-SLAM2 map tracking (Tracking.cc:985-1176): the initial pose of the flow solve; it
  // may reset mLastFrame's pose (UpdateLastFrame), which the rest of this frame reads
  {
    MapStatsH& ms = out.map;
    // the previous frame's object path runs while a map chain is on the GPU: the C3 chain when the
    // C2 chain's wait holds the local map speculation (8-step bench 722 against 737 frames/s,
    // medians of 5, profiles/r06_ab_overlap_c3.txt), else the first chain (splitting it over the
    // two chains measured slower in round 4: 888 against 903 frames/s)
    map_.set_overlap([this] { obj_advance(); });
    const int rr = map_.track(C.m, G, ego_Tinit_, Ls.m, Ls.Tview, V_, hasVelocity_,
                              bSecondFrame_, ms, st);
    map_.set_overlap(nullptr);  // not taken (no chain ran): the loop runs it
    ms.state = map_.state();
    memcpy(ms.Tcw_map, ego_Tinit_, sizeof(ego_Tinit_));
    if (rr == 1) {  // LOST with <= 5 keyframes: mpSystem->Reset(); Track returns (:1165-1172)
      ms.n_keyframes = map_.n_keyframes();
      ms.n_mappoints = map_.n_mappoints();
      reset_pending_ = true;
      ego_pending_ = false;
      return;
    }
    map_finish_pending_ = true;
  }
  C.bSecond = bSecondFrame_;
  // ---- D2 (PoseOptimizationFlow2Cam)
  FlowSolveDesc& d2 = eh_->d2;  // pinned: the upload below stays asynchronous
  memset(&d2, 0, sizeof(d2));
  d2.d_n = Ls.st.count;
  d2.idx = nullptr;
  d2.obs = Ls.st.keys;  // mLastFrame.mvSiftKeys (= its own mvSiftKeysTmp)
  d2.flow = Ls.st.flow;
  d2.depth = Ls.st.depth;
  memcpy(d2.Tcw_last, Ls.Tview, sizeof(d2.Tcw_last));
  memcpy(d2.init, ego_Tinit_, sizeof(d2.init));
  d2.rp_thres = 0.04f;
  d2.use_noise = 1;
  d2.g0 = g0_;
  d2.max_iters = 100;
  d2.prior_info = 0.3;
  d2.fx = cfg_.fx; d2.fy = cfg_.fy; d2.cx = cfg_.cx; d2.cy = cfg_.cy;
  d2.scratch = d_lm_scratch_;
  d2.cap = lm_cap_;
  d2.pose_out = d_poses_;
  d2.stats = d_lmstats_;
  d2.gx = d_gx_;
  d2.gx_seq = ++gx_seq_;
  d2.gx_spin = split_spin_;
  // the granule tags carry 16 bits of gx_seq_: two launches with the same salt are always
  // separated by a wrap, where the granules are cleared (a slot no launch has rewritten since the
  // previous use of the salt could otherwise match)
  if ((gx_seq_ & 0xFFFFu) == 0)
    MMT_HIP(hipMemsetAsync(d_gx_, 0, sizeof(unsigned long long) * kFlowSplitGranules, st));
  MMT_HIP(hipMemcpyAsync(d_descs_, &d2, sizeof(d2), hipMemcpyHostToDevice, st));
  // the ego solve (1,500-1,700 edges on KITTI-like frames) split over workgroups
  const int groups = flow_split_groups(eh_->n_static[last_]);
  if (groups > 1)
    launch_flow_lm_split(d_descs_, groups, st);
  else
    launch_flow_lm(d_descs_, 1, eh_->n_static[last_], st);
  MMT_HIP(hipMemcpyAsync(eh_->Tcw, d_poses_, sizeof(eh_->Tcw) + sizeof(eh_->st),
                         hipMemcpyDeviceToHost, st));
  ego_pending_ = true;
}

// The map branch's host-only tail (keyframe decision and creation) while D2 runs on the GPU.
void Tracker::ego_map_finish(FrameOut& out) {
  if (!map_finish_pending_) return;
  map_finish_pending_ = false;
  FrameSlot& C = slot_[cur_];
  FrameSlot& Ls = slot_[last_];
  map_.track_finish(C.m, Ls.m, ego_Tinit_, out.map);
  out.map.n_keyframes = map_.n_keyframes();
  out.map.n_mappoints = map_.n_mappoints();
}

void Tracker::ego_finish(FrameOut& out, hipStream_t st) {
  FrameSlot& C = slot_[cur_];
  FrameSlot& Ls = slot_[last_];
  MMT_HIP(hipStreamSynchronize(st));
  if (defer_) {  // every frame's object record, in frame order (finished at once without a job)
    dq_.emplace_back();
    dq_.back().seq = out.seq;
  }
  out.n_obj_samples = eh_->nlast_obj;
  bool advance = true;
  if (reset_pending_) {
    // the reset frame: Track returned after the map branch (no flow solve, no objects, and
    // mLastFrame stays the previous frame)
    memcpy(out.Tcw, ego_Tinit_, sizeof(out.Tcw));
    out.initialized = false;
    return;
  }
  if (state_ == 0) {
    // ---- StereoInitialization (needs more than 500 keypoints)
    bFirstFrame_ = true;
    bSecondFrame_ = false;
    if (out.n_keys > 500) {
      mat4_eye(C.Tcw);
      memcpy(C.Tview, C.Tcw, sizeof(C.Tview));
      map_.initialize(C.m, C.Tcw);
      map_.frame_done(C.m, C.Tcw);
      memcpy(out.Tcw, C.Tcw, sizeof(out.Tcw));
      state_ = 1;
      out.initialized = true;
      out.map.state = map_.state();
      out.map.n_keyframes = map_.n_keyframes();
      out.map.n_mappoints = map_.n_mappoints();
      memcpy(out.map.Tcw_map, C.Tcw, sizeof(C.Tcw));
    } else {
      mat4_eye(out.Tcw);
      advance = false;  // the reference keeps its last frame until initialisation succeeds
    }
  } else {
    float Tcw[16];
    memcpy(Tcw, eh_->Tcw, sizeof(Tcw));
    if (eh_->st[2] == 2) {
      // the split solve's workgroups were not resident together within its spin bound (other
      // streams or processes held the CUs): the same solve on one workgroup, from the unchanged
      // descriptor
      launch_flow_lm(d_descs_, 1, eh_->n_static[last_], st);
      MMT_HIP(hipMemcpyAsync(eh_->Tcw, d_poses_, sizeof(eh_->Tcw) + sizeof(eh_->st),
                             hipMemcpyDeviceToHost, st));
      MMT_HIP(hipStreamSynchronize(st));
      split_fallbacks_++;
      memcpy(Tcw, eh_->Tcw, sizeof(Tcw));
    }
    if (eh_->st[2] != 0) memcpy(Tcw, ego_Tinit_, sizeof(Tcw));  // < 3 edges: pose unchanged
    memcpy(C.Tcw, Tcw, sizeof(Tcw));
    out.ego_iterations = eh_->st[0];
    out.ego_inliers = eh_->st[1];
    float LastTwc[16];
    inv_mat(Ls.Tview, LastTwc);  // mLastFrame's pose (Tracking.cc:1311-1317)
    mat4_mul(C.Tcw, LastTwc, V_);
    hasVelocity_ = true;
    memcpy(out.Tcw, C.Tcw, sizeof(out.Tcw));
    out.initialized = map_.state() == 1;
    map_.frame_done(C.m, C.Tcw);  // mlRelativeFramePoses (Tracking.cc:2481-2489)
    memcpy(C.Tview, C.Tcw, sizeof(C.Tview));
    // queue the frame's object work (also when there are no object samples: its labels and
    // motions must be reset for the next frame, in pipeline order)
    qa_ = ObjFrame();
    qa_.active = true;
    qa_.cur = cur_;
    qa_.last = last_;
    qa_.nobj = eh_->nlast_obj > 0 ? -1 : 0;  // -1: grouping decides
    qa_.out = defer_ ? &dq_.back() : &out;
    qa_.out->obj_pending = true;
  }
  ego_pending_ = false;
  if (advance) {
    // B9: the current slot becomes the last frame (Tracking.cc:2463-2477); its own samples
    // already live in the slot, so this is an index rotation over three slots (the object path
    // of this frame still reads this slot and the previous one)
    last_ = cur_;
    cur_ = (cur_ + 1) % kSlots;
  }
}

void Tracker::obj_stage_a(ObjFrame& F) {
  obj_stage_a_launch(F);
  obj_stage_a_decide(F);
}

void Tracker::obj_stage_a_launch(ObjFrame& F) {
  FrameSlot& C = slot_[F.cur];
  FrameSlot& Ls = slot_[F.last];
  hipStream_t st = oa_;
  if (F.a_launched) return;
  F.a_launched = true;
  F.slot = obj_slot_next_;
  obj_slot_next_ = (obj_slot_next_ + 1) % kObjSlots;
  const int q = F.slot;
  C.nModLabel.clear();
  C.nSemPosition.clear();
  C.vObjMod.clear();
  C.obj_slot = -1;
  if (F.nobj == 0) return;  // no object samples carried into this frame
  // ---- B6 + B7 statistics
  GroupArgs g;
  memset(&g, 0, sizeof(g));
  g.n = Ls.ob.count;
  g.cur_keys = C.ho.okeys;
  g.cur_depth = C.ho.odepth;
  g.cur_label = C.ho.olabel;
  g.last_keys = Ls.ob.keys;
  g.last_depth = Ls.ob.depth;
  g.last_label = Ls.ob.label;
  memcpy(g.Tcur, C.Tcw, sizeof(g.Tcur));
  memcpy(g.Tlast, Ls.Tview, sizeof(g.Tlast));
  g.fx = cfg_.fx; g.fy = cfg_.fy; g.cx = cfg_.cx; g.cy = cfg_.cy;
  g.W = W_;
  g.H = H_;
  g.obj_label = d_obj_label_[q];
  g.members = d_members_[q];
  g.member_cap = ocap_;
  g.stats = d_stats_[q];
  g.hist = d_hist_[q];
  g.err = d_err_;
  launch_obj_group(g, st);
  ObjHost& H = *oh_[q];
  MMT_HIP(hipMemcpyAsync(H.stats, d_stats_[q], kObjStatsBytes, hipMemcpyDeviceToHost, st));
  MMT_HIP(hipMemcpyAsync(&H.err, d_err_, sizeof(int), hipMemcpyDeviceToHost, st));
  MMT_HIP(hipEventRecord(ev_grp_[q], st));
}

void Tracker::obj_stage_a_decide(ObjFrame& F) {
  FrameSlot& C = slot_[F.cur];
  FrameSlot& Ls = slot_[F.last];
  hipStream_t st = oa_;
  if (!F.a_launched) obj_stage_a_launch(F);
  if (F.nobj == 0) return;  // no object samples carried into this frame
  const int q = F.slot;
  ObjHost& H = *oh_[q];
  MMT_HIP(hipEventSynchronize(ev_grp_[q]));
  if (H.err) {
    MMT_HIP(hipMemsetAsync(d_err_, 0, sizeof(int), st));  // the next frame starts clean
    MMT_HIP(hipStreamSynchronize(st));
    throw ArgError("semantic label outside [0, 15] on the object path");
  }
  const LabelStats* stats = H.stats;
  const int* hist = H.hist;
  // ---- B7 decisions (Tracking.cc:1424-1536); labels ascending = UniLab order
  std::vector<int> objLabelsNew;  // semantic label of each kept object
  for (int l = 1; l < kMaxLabel; l++) {
    const LabelStats& s = stats[l];
    if (s.cnt == 0) continue;
    const float count = (float)s.bcnt;
    if (count / s.cnt > 0.5f) continue;  // mostly on the image boundary
    if (!(s.cnt > 100)) continue;        // fewer than 100 points
    const float sf_count = (float)s.sfcnt;
    if (sf_count / s.cnt > 0.3f) continue;            // static object
    if (s.depth_sum / s.cnt > 25.0) continue;         // too far
    objLabelsNew.push_back(l);
  }
  // ---- B8 label association (Tracking.cc:1556-1630)
  int mx;
  if (C.bSecond)
    mx = 1;
  else if (!Ls.nModLabel.empty())
    mx = *std::max_element(Ls.nModLabel.begin(), Ls.nModLabel.end()) + 1;
  else
    mx = 1;  // uninitialised in the reference (Tracking.cc:1557): pinned 1
  const int nobj = (int)objLabelsNew.size();
  if (nobj > kMaxObj) throw ArgError("more dynamic objects than semantic labels 1..15");
  std::vector<int> LabId(nobj);
  for (int i = 0; i < nobj; i++) {
    const int l = objLabelsNew[i];
    int New_lab = 0, best = -1;
    for (int ll = 0; ll < kMaxLabel; ll++) {  // std::map order: ascending last label
      const int c = hist[l * kMaxLabel + ll];
      if (c > best && c > 0) {
        best = c;
        New_lab = ll;
      }
    }
    if (C.bSecond) {
      LabId[i] = mx++;
    } else {
      bool exist = false;
      for (size_t k = 0; k < Ls.nSemPosition.size(); k++)
        if (Ls.nSemPosition[k] == New_lab) {
          LabId[i] = Ls.nModLabel[k];
          exist = true;
          break;
        }
      if (!exist) LabId[i] = mx++;
    }
  }
  C.nModLabel = LabId;
  C.nSemPosition.assign(objLabelsNew.begin(), objLabelsNew.begin() + nobj);
  C.vObjMod.assign(nobj, std::vector<float>(16, 0.f));
  F.nobj = nobj;
  F.labels.assign(objLabelsNew.begin(), objLabelsNew.begin() + nobj);
  F.LabId = LabId;
  F.PreObjID.assign(nobj, -1);
  F.members.assign(nobj, 0);
  F.po = H.po;
  if (nobj == 0) return;
  C.obj_slot = q;
  // ---- D5: PnP-RANSAC per object (GetInitModelObj), motion-model check deferred to stage B
  for (int i = 0; i < nobj; i++) {
    const int l = objLabelsNew[i];
    PnPBuf& b = pnp_[q][i];
    const PnPScratch& r = pnp_scr_[i];
    PnPObject& o = F.po[i];
    int* d_sub = (int*)((uint8_t*)d_pnp_[q] + sizeof(PnPObject) * kMaxObj) + (size_t)i * 5 * kRansacIters;
    memset(&o, 0, sizeof(o));
    o.n = &d_stats_[q][l].members;
    o.members = d_members_[q] + (size_t)l * ocap_;
    o.last_keys = Ls.ob.keys;
    o.last_depth = Ls.ob.depth;
    o.cur_keys = C.ho.okeys;
    memcpy(o.Tlast, Ls.Tview, sizeof(o.Tlast));
    o.fx = cfg_.fx; o.fy = cfg_.fy; o.cx = cfg_.cx; o.cy = cfg_.cy;
    o.reproj = 0.3;
    o.confidence = 0.98;
    F.members[i] = stats[l].members;
    const std::vector<int>& sub = cached_subsets(std::max(stats[l].members, 1));
    memcpy(H.subsets[i], sub.data(), sizeof(H.subsets[i]));
    o.subsets = d_sub;
    for (size_t k = 0; k < Ls.nModLabel.size(); k++)
      if (Ls.nModLabel[k] == LabId[i]) {
        F.PreObjID[i] = (int)k;
        break;
      }
    o.use_mm = F.PreObjID[i] >= 0;
    o.pts3 = b.pts3;
    o.pts2 = b.pts2;
    o.models = r.models;
    o.hrec = r.hrec;
    o.hout = r.hout;
    o.good = r.good;
    o.masks = r.masks;
    o.mask_words = mask_words_;
    o.inliers = b.inliers;
    o.mm_inliers = b.mm_inliers;
    o.subset = b.subset;
    o.n_subset = b.n_subset;
    o.result = b.result;
    o.Rt = b.Rt;
  }
  // the records (all kMaxObj) and the first nobj subset draws behind them
  MMT_HIP(hipMemcpyAsync(d_pnp_[q], H.po, sizeof(PnPObject) * kMaxObj + sizeof(H.subsets[0]) * nobj,
                         hipMemcpyHostToDevice, st));
  launch_pnp(d_pnp_[q], nobj, kRansacIters, st);
  // ev_ransac_[q] is recorded by stage B, behind the D3 descriptors' copy on this stream
}

void Tracker::obj_stage_b(ObjFrame& F) {
  FrameSlot& C = slot_[F.cur];
  FrameSlot& Ls = slot_[F.last];
  const int nobj = F.nobj, q = F.slot;
  if (nobj <= 0) return;
  hipStream_t st = ob_;
  ObjHost& H = *oh_[q];
  // behind this frame's RANSAC (oa_) by an event, behind the previous frame's D3 (whose motions
  // the motion model needs) by the stream
  // D3 descriptors; the initial motion is the device's model choice (k_obj_model_choice)
  for (int i = 0; i < nobj; i++) {
    FlowSolveDesc& d = H.descs[i];
    memset(&d, 0, sizeof(d));
    d.d_n = pnp_[q][i].n_subset;
    d.idx = pnp_[q][i].subset;
    d.obs = Ls.ob.keys;
    d.flow = Ls.ob.flow;
    d.depth = Ls.ob.depth;
    memcpy(d.Tcw_last, Ls.Tview, sizeof(d.Tcw_last));
    d.rp_thres = 0.01f;
    d.use_noise = 0;
    d.max_iters = d3_iters_;
    d.prior_info = 0.5;
    d.fx = cfg_.fx; d.fy = cfg_.fy; d.cx = cfg_.cx; d.cy = cfg_.cy;
    d.scratch = d_lm_scratch_ + flow_scratch_doubles(lm_cap_) * (1 + i);
    d.cap = lm_cap_;
    d.pose_out = d_r_[q]->X + 16 * i;
    d.stats = d_r_[q]->lst + 3 * i;
    d.g0 = g0_;  // the centroid's depth noise (the solve itself runs without noise)
    d.centre_out = d_r_[q]->centre + 3 * i;
  }
  // the descriptors go up on the RANSAC stream, off the D3 chain
  MMT_HIP(hipMemcpyAsync(d_descs3_[q], H.descs, sizeof(FlowSolveDesc) * nobj,
                         hipMemcpyHostToDevice, oa_));
  MMT_HIP(hipEventRecord(ev_ransac_[q], oa_));
  MMT_HIP(hipStreamWaitEvent(st, ev_ransac_[q], 0));
  // motion model (Tracking.cc:4375-4405): MM = Tcw * vObjMod[PreObjID] of the previous frame,
  // whose D3 output is still in its slot's buffers
  bool any_mm = false;
  MMPrepArgs mp;
  memset(&mp, 0, sizeof(mp));
  mp.objs = d_pnp_[q];
  mp.nobj = nobj;
  for (int i = 0; i < nobj; i++) {
    mp.pre[i] = F.po[i].use_mm ? F.PreObjID[i] : -1;
    any_mm = any_mm || F.po[i].use_mm;
  }
  if (any_mm) {
    if (Ls.obj_slot < 0) throw ArgError("motion model without a previous object solve");
    mp.prevX = d_r_[Ls.obj_slot]->X;
    mp.prevStats = d_r_[Ls.obj_slot]->lst;
    memcpy(mp.TcwPrev, Ls.Tcw, sizeof(mp.TcwPrev));
    memcpy(mp.TcwCur, C.Tcw, sizeof(mp.TcwCur));
  }
  launch_obj_stage_b(mp, d_descs3_[q], d_r_[q]->init, st);
  launch_flow_lm(d_descs3_[q], nobj, 256, st);
  // everything the finish reads, in one pinned block
  MMT_HIP(hipMemcpyAsync(&H.r, d_r_[q], sizeof(ObjResults), hipMemcpyDeviceToHost, st));
  MMT_HIP(hipEventRecord(ev_d3_[q], st));
}

void Tracker::obj_finish(ObjFrame& F) {
  FrameSlot& C = slot_[F.cur];
  const int nobj = F.nobj, q = F.slot;
  FrameOut& out = *F.out;
  F.active = false;
  out.obj_pending = false;
  if (nobj <= 0) return;
  MMT_HIP(hipEventSynchronize(ev_d3_[q]));
  const ObjHost& H = *oh_[q];
  float TcwInv[16];
  inv_mat(C.Tcw, TcwInv);
  for (int i = 0; i < nobj; i++) {
    const int* res = H.r.res + 8 * i;
    ObjOut oo;
    oo.label = F.LabId[i];
    oo.sem_label = F.labels[i];
    oo.n_points = F.members[i];
    oo.n_ransac_inliers = res[0] >= 0 ? res[3] : 0;
    oo.n_mm_inliers = F.po[i].use_mm ? res[4] : -1;
    oo.ransac_iterations = res[2];
    memcpy(oo.init, H.r.init + 16 * i, 64);
    float Xi[16];
    if (H.r.lst[3 * i + 2] != 0)
      mat4_eye(Xi);  // fewer than 3 correspondences: PoseOptimizationFlow2 returns identity
    else
      memcpy(Xi, H.r.X + 16 * i, 64);
    mat4_mul(TcwInv, Xi, C.vObjMod[i].data());
    oo.n_solve = H.r.nsub[i];
    oo.n_inliers = H.r.lst[3 * i + 2] ? 0 : H.r.lst[3 * i + 1];
    oo.iterations = H.r.lst[3 * i];
    memcpy(oo.X, Xi, 64);
    memcpy(oo.motion, C.vObjMod[i].data(), 64);
    memcpy(oo.centre_pre, H.r.centre + 3 * i, 12);  // computed whatever the solve's size
    out.objects.push_back(oo);
  }
}

// ---------------------------------------------------------------- device side of stage B
__global__ void k_obj_mm_prep(MMPrepArgs a) {
  const int i = threadIdx.x;
  if (i >= a.nobj || a.pre[i] < 0) return;
  const int p = a.pre[i];
  float X[16], Ti[16], vobj[16], MM[16];
  if (a.prevStats[3 * p + 2] != 0)
    mat4_eye(X);
  else
    for (int k = 0; k < 16; k++) X[k] = a.prevX[16 * p + k];
  inv_mat(a.TcwPrev, Ti);
  mat4_mul(Ti, X, vobj);  // the previous frame's vObjMod[p] (its finish computes the same)
  mat4_mul(a.TcwCur, vobj, MM);
  for (int k = 0; k < 16; k++) a.objs[i].MM[k] = MM[k];
}

// GetInitModelObj's choice (Tracking.cc:4400-4420): the RANSAC model unless the motion model has
// at least as many inliers; the chosen motion seeds D3
__global__ void k_obj_model_choice(PnPObject* objs, int nobj, FlowSolveDesc* descs, float* init) {
  const int i = threadIdx.x;
  if (i >= nobj) return;
  PnPObject& o = objs[i];
  const int n_ransac = o.result[0] >= 0 ? o.result[3] : 0;
  const int n_mm = o.use_mm ? o.result[4] : -1;
  float Mod[16];
  mat4_eye(Mod);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) Mod[4 * r + c] = (float)o.Rt[3 * r + c];
    Mod[4 * r + 3] = (float)o.Rt[9 + r];
  }
  const bool choice = o.use_mm && !(n_ransac > n_mm);
  o.use_mm_choice = choice ? 1 : 0;
  for (int k = 0; k < 16; k++) {
    const float v = choice ? o.MM[k] : Mod[k];
    descs[i].init[k] = v;
    init[16 * i + k] = v;
  }
}

// Stage B of one frame's objects in one launch (one workgroup per object; the objects are
// independent): the motion-model matrix (k_obj_mm_prep), its inliers (pnp_mm_inliers_block), the
// model choice that seeds D3 (k_obj_model_choice) and D3's edge list (pnp_subset_block) -- the
// same results as the four separate kernels, without three dependent launches on the critical
// chain.
__global__ __launch_bounds__(256) void k_obj_stage_b(MMPrepArgs a, FlowSolveDesc* descs,
                                                     float* init) {
  __shared__ float s_MM[16];
  __shared__ int s_w[4];
  const int i = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  PnPObject& o = a.objs[i];
  // Everything this launch reads but does not write is loaded up front, so the dependent global
  // round trips on the critical D3 chain are the motion-model matrix and the inlier lists only.
  const int use_mm = o.use_mm;
  const int n = use_mm ? *o.n : 0;
  const float* pts3 = o.pts3;
  const float2* pts2 = o.pts2;
  const int* members = o.members;
  const int* rs_inliers = o.inliers;
  int* mm_inliers = o.mm_inliers;
  const float fx = o.fx, fy = o.fy, cx = o.cx, cy = o.cy;
  const double reproj = o.reproj;
  const int* res = o.result;
  const int res3 = res[3];
  const int n_ransac = res[0] >= 0 ? res3 : 0;
  if (tid == 0 && a.pre[i] >= 0) {  // MM = Tcw * vObjMod[PreObjID] (k_obj_mm_prep)
    const int p = a.pre[i];
    float X[16], Ti[16], vobj[16], MM[16];
    const int fail = a.prevStats[3 * p + 2];
    for (int k = 0; k < 16; k++) X[k] = a.prevX[16 * p + k];
    if (fail != 0) mat4_eye(X);
    inv_mat(a.TcwPrev, Ti);
    mat4_mul(Ti, X, vobj);
    mat4_mul(a.TcwCur, vobj, MM);
    for (int k = 0; k < 16; k++) {
      o.MM[k] = MM[k];
      s_MM[k] = MM[k];
    }
  }
  __syncthreads();
  // motion-model inliers, ascending (pnp_mm_inliers_block with the matrix from LDS)
  int n_mm = -1;
  if (use_mm) {
    float MM[16];
#pragma unroll
    for (int k = 0; k < 16; k++) MM[k] = s_MM[k];
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += blockDim.x) {
      const int j = i0 + tid;
      bool in = false;
      if (j < n) {
        float xc[3];
        for (int r = 0; r < 3; r++) {
          double sum = 0;
          for (int k = 0; k < 3; k++) sum += (double)MM[4 * r + k] * (double)pts3[3 * j + k];
          xc[r] = (float)sum + MM[4 * r + 3];
        }
        const float invzc = (float)(1.0 / (double)xc[2]);
        const float u = fx * xc[0] * invzc + cx, v = fy * xc[1] * invzc + cy;
        const float2 q = pts2[j];
        const float u_ = q.x - u, v_ = q.y - v;
        const float Rpe = sqrtf(u_ * u_ + v_ * v_);
        in = (double)Rpe < reproj;
      }
      const unsigned long long bal = __ballot(in);
      if (lane == 0) s_w[wave] = __popcll(bal);
      __syncthreads();
      int off = 0, tot = 0;
      for (int w = 0; w < 4; w++) {
        if (w < wave) off += s_w[w];
        tot += s_w[w];
      }
      if (in) mm_inliers[base + off + __popcll(bal & ((1ull << lane) - 1ull))] = j;
      base += tot;
      __syncthreads();
    }
    n_mm = base;
  }
  // model choice (k_obj_model_choice), the same in every thread
  const bool choice = use_mm && !(n_ransac > n_mm);
  if (tid == 0) {
    if (use_mm) o.result[4] = n_mm;
    o.use_mm_choice = choice ? 1 : 0;
    float Mod[16];
    if (choice) {
      for (int k = 0; k < 16; k++) Mod[k] = s_MM[k];
    } else {
      mat4_eye(Mod);
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Mod[4 * r + c] = (float)o.Rt[3 * r + c];
        Mod[4 * r + 3] = (float)o.Rt[9 + r];
      }
    }
    for (int k = 0; k < 16; k++) {
      descs[i].init[k] = Mod[k];
      init[16 * i + k] = Mod[k];
    }
  }
  // D3 edge list (pnp_subset_block): the chosen model's inliers as sample indices; the motion-model
  // list was completed before the inlier loop's last barrier
  const int n_sub = choice ? n_mm : res3;
  const int* src = choice ? mm_inliers : rs_inliers;
  int* sub = o.subset;
  for (int j = tid; j < n_sub; j += blockDim.x) sub[j] = members[src[j]];
  if (tid == 0) *o.n_subset = n_sub;
}

void launch_obj_stage_b(const MMPrepArgs& a, FlowSolveDesc* descs, float* init, hipStream_t st) {
  hipLaunchKernelGGL(k_obj_stage_b, dim3(a.nobj), dim3(256), 0, st, a, descs, init);
}

void launch_obj_mm_prep(const MMPrepArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_obj_mm_prep, dim3(1), dim3(64), 0, st, a);
}

void launch_obj_model_choice(PnPObject* objs, int nobj, FlowSolveDesc* descs, float* init,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_obj_model_choice, dim3(1), dim3(64), 0, st, objs, nobj, descs, init);
}

}  // namespace mmt
