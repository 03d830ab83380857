// multimot_track_amd/csrc/mmt_capi.hip -- the C-ABI of libmmt (include/mmt.h).
// Every entry point catches internal exceptions and returns an errno-style code; nothing exits.

#include <hip/hip_runtime.h>

#include <cstdint>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include <new>

#include "mmt_ctx.h"
#include "mmt_match.h"
#include "mmt_pnp.h"
#include "mmt_track.h"

using mmt::ArgError;
using mmt::DeviceError;

template <typename F>
static int guard(mmt_ctx* ctx, F&& body) {
  try {
    body();
  } catch (const ArgError& e) {
    if (ctx) ctx->err = e.msg;
    return MMT_EINVAL;
  } catch (const DeviceError& e) {
    if (ctx) ctx->err = e.msg;
    return MMT_EDEVICE;
  } catch (const std::bad_alloc&) {
    if (ctx) ctx->err = "host allocation failed";
    return MMT_ENOMEM;
  }
  return MMT_OK;
}

// Scoped device allocation for the probe entry points.
template <typename T>
struct DevBuf {
  T* p = nullptr;
  explicit DevBuf(size_t n) { MMT_HIP(hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T))); }
  ~DevBuf() { (void)hipFree(p); }
};

// The current frame of a matcher probe on the device: keys, descriptors, depth map, and the B3
// outputs (uR, depth, grid) built by k_stereo_grid.
struct DevMatchFrame {
  int n;
  DevBuf<mmt_kp> kps;
  DevBuf<uint8_t> desc;
  DevBuf<float> depth, uR, kdepth;
  DevBuf<int> nk, cell_start, cell_idx;
  mmt::GridFrame G;
  DevMatchFrame(mmt_ctx* ctx, const mmt_match_frame* cur, bool need_desc)
      : n(cur->n), kps(cur->n), desc(32 * (size_t)cur->n),
        depth((size_t)ctx->cfg.width * ctx->cfg.height), uR(cur->n), kdepth(cur->n), nk(1),
        cell_start(mmt::kGridCells + 1), cell_idx(cur->n) {
    const mmt_config& c = ctx->cfg;
    hipStream_t s = ctx->stream;
    if (n > 0) {
      MMT_HIP(hipMemcpyAsync(kps.p, cur->kps, sizeof(mmt_kp) * (size_t)n, hipMemcpyHostToDevice, s));
      if (need_desc)
        MMT_HIP(hipMemcpyAsync(desc.p, cur->desc, 32 * (size_t)n, hipMemcpyHostToDevice, s));
    }
    MMT_HIP(hipMemcpyAsync(depth.p, cur->depth, sizeof(float) * (size_t)c.width * c.height,
                           hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(nk.p, &n, sizeof(int), hipMemcpyHostToDevice, s));
    memset(&G, 0, sizeof(G));
    G.keys = kps.p;
    G.desc = desc.p;
    G.uR = uR.p;
    G.cell_start = cell_start.p;
    G.cell_idx = cell_idx.p;
    G.n = n;
    G.fx = c.fx; G.fy = c.fy; G.cx = c.cx; G.cy = c.cy; G.bf = c.bf;
    // Frame::ComputeImageBounds without distortion + grid element sizes (Frame.cc:581-584, 841-846)
    G.minX = 0.0f; G.maxX = (float)c.width; G.minY = 0.0f; G.maxY = (float)c.height;
    G.invW = static_cast<float>(mmt::kGridCols) / static_cast<float>(G.maxX - G.minX);
    G.invH = static_cast<float>(mmt::kGridRows) / static_cast<float>(G.maxY - G.minY);
    G.nlevels = ctx->orb.nlevels;
    for (int l = 0; l < G.nlevels && l < mmt::kMaxLevels; l++) G.scale[l] = ctx->orb.scale[l];
    // mfLogScaleFactor = log(mfScaleFactor), pinned as log in double rounded to float
    G.logScale = (float)std::log((double)ctx->orb.scale[G.nlevels > 1 ? 1 : 0]);
    mmt::launch_stereo_grid(kps.p, nk.p, std::max(n, 1), depth.p, (size_t)c.width * c.height,
                            c.width, c.height, c.bf, G.invW, G.invH, uR.p, kdepth.p,
                            cell_start.p, cell_idx.p, 1, s);
  }
};

static void check_match_frame(mmt_ctx* ctx, const mmt_match_frame* cur, bool need_desc) {
  if (!cur || cur->n < 0 || cur->n > mmt::kMaxMatchKeys) throw ArgError("bad current frame");
  if (cur->n > 0 && (!cur->kps || (need_desc && !cur->desc))) throw ArgError("null frame arrays");
  if (!cur->depth) throw ArgError("null depth map");
  if (ctx->orb.nlevels > mmt::kMaxLevels) throw ArgError("too many pyramid levels");
  const int W = ctx->cfg.width, H = ctx->cfg.height;
  for (int i = 0; i < cur->n; i++) {
    const mmt_kp& k = cur->kps[i];
    if (!(k.x >= 0 && k.y >= 0 && (int)k.x < W && (int)k.y < H))
      throw ArgError("keypoint outside the image");
    if (k.octave < 0 || k.octave >= ctx->orb.nlevels) throw ArgError("keypoint octave out of range");
  }
}

struct DevCands {
  DevBuf<uint32_t> key;
  DevBuf<int> idx, n, choice;
  DevBuf<mmt::PointWin> win;
  explicit DevCands(int m)
      : key((size_t)std::max(m, 1) * mmt::kCandK), idx((size_t)std::max(m, 1) * mmt::kCandK),
        n(std::max(m, 1)), choice(std::max(m, 1)), win(std::max(m, 1)) {}
  mmt::CandSet set() { return mmt::CandSet{key.p, idx.p, n.p, win.p, choice.p}; }
};

static thread_local std::string g_create_error;

extern "C" {

int mmt_version(void) { return 100; }

const char* mmt_last_error(const mmt_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

mmt_ctx* mmt_create(const mmt_config* cfg) {
  if (!cfg) {
    g_create_error = "null config";
    return nullptr;
  }
  mmt_ctx* ctx = new (std::nothrow) mmt_ctx();
  if (!ctx) return nullptr;
  ctx->cfg = *cfg;
  try {
    if (cfg->width <= 0 || cfg->height <= 0) throw ArgError("bad image size");
    if (cfg->k1 != 0.f) throw ArgError("distortion must be zero on this path (Frame.cc:789)");
    if (cfg->orb_nlevels < 1 || cfg->orb_nlevels > 16) throw ArgError("bad orb_nlevels");
    if (cfg->orb_nfeatures < 1) throw ArgError("bad orb_nfeatures");
    int ndev = 0;
    MMT_HIP(hipGetDeviceCount(&ndev));
    if (cfg->device_id < 0 || cfg->device_id >= ndev) throw ArgError("bad device_id");
    MMT_HIP(hipSetDevice(cfg->device_id));
    // the context stream (ORB window, ego chain) at normal priority (high measured within noise)
    MMT_HIP(hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, 0));
    ctx->orb.init(cfg->orb_nfeatures, cfg->orb_scale_factor, cfg->orb_nlevels,
                  cfg->orb_ini_th_fast, cfg->orb_min_th_fast);
    ctx->engine.setup(cfg->width, cfg->height, ctx->orb, cfg->max_batch > 0 ? cfg->max_batch : 1);
  } catch (const ArgError& e) {
    g_create_error = e.msg;
    delete ctx;
    return nullptr;
  } catch (const DeviceError& e) {
    g_create_error = e.msg;
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void mmt_destroy(mmt_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->cfg.device_id);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  (void)hipFree(ctx->d_in);
  (void)hipFree(ctx->d_kps);
  (void)hipFree(ctx->d_desc);
  (void)hipFree(ctx->d_n);
  (void)hipFree(ctx->t_bgr);
  (void)hipFree(ctx->t_disp);
  (void)hipFree(ctx->t_flow);
  (void)hipFree(ctx->t_mask);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int mmt_orb_levels(const mmt_ctx* ctx, float* scale, float* sigma2, int* n_per_level,
                   int* level_w, int* level_h) {
  if (!ctx) return MMT_EINVAL;
  const auto& lv = ctx->engine.levels();
  for (int l = 0; l < ctx->orb.nlevels; l++) {
    if (scale) scale[l] = ctx->orb.scale[l];
    if (sigma2) sigma2[l] = ctx->orb.sigma2[l];
    if (n_per_level) n_per_level[l] = ctx->orb.nPerLevel[l];
    if (level_w) level_w[l] = lv[l].w;
    if (level_h) level_h[l] = lv[l].h;
  }
  return MMT_OK;
}

int mmt_orb_capacity(const mmt_ctx* ctx) { return ctx ? ctx->engine.capacity() : MMT_EINVAL; }

static void ensure_staging(mmt_ctx* ctx, int nframes) {
  const size_t fb = (size_t)ctx->cfg.width * ctx->cfg.height;
  if (ctx->staged_frames >= nframes) return;
  (void)hipFree(ctx->d_in);
  (void)hipFree(ctx->d_kps);
  (void)hipFree(ctx->d_desc);
  (void)hipFree(ctx->d_n);
  ctx->d_in = nullptr;
  ctx->d_kps = nullptr;
  ctx->d_desc = nullptr;
  ctx->d_n = nullptr;
  const int cap = ctx->engine.capacity();
  MMT_HIP(hipMalloc((void**)&ctx->d_in, fb * nframes));
  MMT_HIP(hipMalloc((void**)&ctx->d_kps, sizeof(mmt_kp) * (size_t)cap * nframes));
  MMT_HIP(hipMalloc((void**)&ctx->d_desc, (size_t)32 * cap * nframes));
  MMT_HIP(hipMalloc((void**)&ctx->d_n, sizeof(int) * nframes));
  ctx->staged_frames = nframes;
}

int mmt_orb_extract_batch(mmt_ctx* ctx, const uint8_t* const* grays, int nframes, int stride,
                          mmt_kp* kps, uint8_t* desc, int cap_per_frame, int* n_per_frame) {
  if (!ctx || !grays || !kps || !desc || !n_per_frame || nframes < 1) return MMT_EINVAL;
  return guard(ctx, [&] {
    const int w = ctx->cfg.width, h = ctx->cfg.height;
    if (stride < w) throw ArgError("stride < width");
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    const int cap = ctx->engine.capacity();
    int done = 0;
    std::vector<int> counts(nframes, 0);
    while (done < nframes) {
      const int nb = std::min(nframes - done, ctx->cfg.max_batch > 0 ? ctx->cfg.max_batch : 1);
      ensure_staging(ctx, nb);
      const size_t fb = (size_t)w * h;
      for (int f = 0; f < nb; f++)
        MMT_HIP(hipMemcpy2DAsync(ctx->d_in + fb * f, w, grays[done + f], stride, w, h,
                                 hipMemcpyHostToDevice, ctx->stream));
      ctx->engine.run(ctx->d_in, nb, fb, ctx->d_kps, ctx->d_desc, cap, ctx->d_n, ctx->stream);
      MMT_HIP(hipMemcpyAsync(counts.data() + done, ctx->d_n, sizeof(int) * nb,
                             hipMemcpyDeviceToHost, ctx->stream));
      ctx->engine.check_flags(ctx->stream);  // synchronises the stream
      for (int f = 0; f < nb; f++) {
        const int n = counts[done + f];
        n_per_frame[done + f] = n;
        if (n > cap_per_frame) throw ArgError("cap_per_frame too small");
        MMT_HIP(hipMemcpyAsync(kps + (size_t)(done + f) * cap_per_frame,
                               ctx->d_kps + (size_t)f * cap, sizeof(mmt_kp) * n,
                               hipMemcpyDeviceToHost, ctx->stream));
        MMT_HIP(hipMemcpyAsync(desc + (size_t)(done + f) * cap_per_frame * 32,
                               ctx->d_desc + (size_t)f * cap * 32, (size_t)32 * n,
                               hipMemcpyDeviceToHost, ctx->stream));
      }
      MMT_HIP(hipStreamSynchronize(ctx->stream));
      done += nb;
    }
  });
}

int mmt_orb_extract(mmt_ctx* ctx, const uint8_t* gray, int w, int h, int stride, mmt_kp* kps,
                    uint8_t* desc, int cap, int* n) {
  if (!ctx || !gray || !kps || !desc || !n) return MMT_EINVAL;
  if (w != ctx->cfg.width || h != ctx->cfg.height) {
    ctx->err = "image size differs from the context configuration";
    return MMT_EINVAL;
  }
  const int fcap = ctx->engine.capacity();
  std::vector<mmt_kp> tk;
  std::vector<uint8_t> td;
  try {
    tk.resize(fcap);
    td.resize((size_t)fcap * 32);
  } catch (const std::bad_alloc&) {
    return MMT_ENOMEM;
  }
  const uint8_t* frames[1] = {gray};
  int cnt = 0;
  const int rc = mmt_orb_extract_batch(ctx, frames, 1, stride, tk.data(), td.data(), fcap, &cnt);
  if (rc) return rc;
  *n = cnt;
  if (cnt > cap) {
    ctx->err = "keypoint capacity too small";
    return MMT_ENOSPC;
  }
  memcpy(kps, tk.data(), sizeof(mmt_kp) * cnt);
  memcpy(desc, td.data(), (size_t)32 * cnt);
  return MMT_OK;
}

int mmt_orb_extract_device(mmt_ctx* ctx, const uint8_t* d_gray, int nframes, size_t frame_pitch,
                           mmt_kp* d_kps, uint8_t* d_desc, int cap_per_frame, int* d_n,
                           void* stream) {
  if (!ctx || !d_gray || !d_kps || !d_desc || !d_n) return MMT_EINVAL;
  return guard(ctx, [&] {
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    ctx->engine.run(d_gray, nframes, frame_pitch, d_kps, d_desc, cap_per_frame, d_n, s);
  });
}

int mmt_orb_device_status(mmt_ctx* ctx, void* stream) {
  if (!ctx) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ctx->engine.check_flags(stream ? (hipStream_t)stream : ctx->stream);
  });
}

int mmt_debug_orb_raise(mmt_ctx* ctx, int flags) {
  if (!ctx) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ctx->engine.raise_flags(flags, ctx->stream);
  });
}

static void ensure_tracker(mmt_ctx* ctx) {
  if (ctx->tracker_ready) return;
  const int B = ctx->cfg.max_batch > 0 ? ctx->cfg.max_batch : 1;
  ctx->tracker.setup(ctx->cfg, &ctx->engine, B);
  ctx->tracker_ready = true;
}

static void fill_results(const std::vector<mmt::FrameOut>& outs, mmt_frame_result* res,
                         mmt_motion* objs, int objs_cap) {
  for (size_t f = 0; f < outs.size(); f++) {
    const mmt::FrameOut& o = outs[f];
    mmt_frame_result& r = res[f];
    memcpy(r.Tcw, o.Tcw, sizeof(r.Tcw));
    r.initialized = o.initialized;
    r.n_keypoints = o.n_keys;
    r.n_obj_samples = o.n_obj_samples;
    r.ego_iterations = o.ego_iterations;
    r.ego_inliers = o.ego_inliers;
    r.n_objects = (int)o.objects.size();
    r.map_state = o.map.state;
    r.map_matches_mm = o.map.matches_mm;
    r.map_inliers_local = o.map.inliers_local;
    r.n_keyframes = o.map.n_keyframes;
    r.n_mappoints = o.map.n_mappoints;
    r.new_keyframe = o.map.new_keyframe;
    memcpy(r.Tcw_map, o.map.Tcw_map, sizeof(r.Tcw_map));
    r.frame_index = (int32_t)o.seq;
    r.objects_frame = (int32_t)o.obj_seq;
    if (!objs) continue;
    for (int i = 0; i < (int)o.objects.size() && i < objs_cap; i++) {
      const mmt::ObjOut& s = o.objects[i];
      mmt_motion& m = objs[f * objs_cap + i];
      m.label = s.label;
      m.sem_label = s.sem_label;
      m.n_points = s.n_points;
      m.n_inliers = s.n_inliers;
      m.n_ransac_inliers = s.n_ransac_inliers;
      m.n_mm_inliers = s.n_mm_inliers;
      m.n_solve = s.n_solve;
      m.iterations = s.iterations;
      memcpy(m.world_motion, s.motion, 64);
      memcpy(m.cam_pose, s.X, 64);
      memcpy(m.init_pose, s.init, 64);
      memcpy(m.centre_pre, s.centre_pre, 12);
    }
  }
}

int mmt_profile_enable(mmt_ctx* ctx, int on) {
  if (!ctx) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ensure_tracker(ctx);
    ctx->tracker.set_profiling(on != 0);
  });
}

int mmt_profile_read(mmt_ctx* ctx, mmt_profile* out, int reset) {
  if (!ctx || !out) return MMT_EINVAL;
  return guard(ctx, [&] {
    ensure_tracker(ctx);
    long long l = 0, f = 0;
    ctx->tracker.read_profile(&out->orb_ms, &l, &f, reset != 0);
    out->orb_launches = l;
    out->orb_frames = f;
  });
}

int mmt_reset(mmt_ctx* ctx) {
  if (!ctx) return MMT_EINVAL;
  return guard(ctx, [&] {
    ensure_tracker(ctx);
    ctx->tracker.reset();
    ctx->flushed.clear();
  });
}

int mmt_set_deferred_objects(mmt_ctx* ctx, int on) {
  if (!ctx) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ensure_tracker(ctx);
    ctx->tracker.set_deferred(on != 0);
    if (!on) ctx->flushed.clear();
  });
}

int mmt_flush_objects(mmt_ctx* ctx, mmt_frame_result* res, mmt_motion* objs, int objs_cap,
                      int res_cap, int* n) {
  if (!ctx || !res || !n || res_cap < 1 || objs_cap < 0) return MMT_EINVAL;
  *n = 0;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ensure_tracker(ctx);
    if (ctx->flushed.empty()) {
      std::vector<mmt::FrameOut> outs;
      ctx->tracker.flush_deferred(outs);
      for (auto& o : outs) ctx->flushed.push_back(std::move(o));
    }
    std::vector<mmt::FrameOut> part;
    while (!ctx->flushed.empty() && (int)part.size() < res_cap) {
      part.push_back(std::move(ctx->flushed.front()));
      ctx->flushed.pop_front();
    }
    for (auto& o : part) o.seq = -1;  // flush records carry objects only
    memset(res, 0, sizeof(mmt_frame_result) * (size_t)part.size());
    fill_results(part, res, objs, objs_cap);
    *n = (int)part.size();
  });
}

// Records a partial mmt_flush_objects left for a later call: tracking more frames before they
// are drained would deliver newer frames' motions ahead of them (the header promises order).
static int flush_owed(mmt_ctx* ctx) {
  if (ctx->flushed.empty()) return 0;
  ctx->err = "mmt_flush_objects has undelivered records: drain it before tracking more frames";
  return MMT_ESTATE;
}

int mmt_track_rgbd_chunk_device(mmt_ctx* ctx, int nframes, const uint8_t* d_bgr,
                                size_t bgr_pitch, const uint16_t* d_disp, size_t disp_pitch,
                                const float* d_flow, size_t flow_pitch, const int32_t* d_mask,
                                size_t mask_pitch, mmt_frame_result* res, mmt_motion* objs,
                                int objs_cap, void* stream) {
  if (!ctx || !d_bgr || !d_disp || !d_flow || !d_mask || !res || nframes < 1) return MMT_EINVAL;
  if (const int rc = flush_owed(ctx)) return rc;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ensure_tracker(ctx);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    std::vector<mmt::FrameOut> outs;
    ctx->tracker.track_chunk(d_bgr, bgr_pitch, d_disp, disp_pitch, d_flow, flow_pitch, d_mask,
                             mask_pitch, nframes, outs, s);
    fill_results(outs, res, objs, objs_cap);
  });
}

// device staging of the host-buffer entry points, nframes frames (frame-major, tight pitches)
static void ensure_track_staging(mmt_ctx* ctx, int nframes) {
  if (ctx->t_frames >= nframes) return;
  const size_t npix = (size_t)ctx->cfg.width * ctx->cfg.height;
  (void)hipFree(ctx->t_bgr);
  (void)hipFree(ctx->t_disp);
  (void)hipFree(ctx->t_flow);
  (void)hipFree(ctx->t_mask);
  ctx->t_bgr = nullptr;
  ctx->t_disp = nullptr;
  ctx->t_flow = nullptr;
  ctx->t_mask = nullptr;
  ctx->t_frames = 0;
  MMT_HIP(hipMalloc((void**)&ctx->t_bgr, npix * 3 * nframes));
  MMT_HIP(hipMalloc((void**)&ctx->t_disp, npix * 2 * nframes));
  MMT_HIP(hipMalloc((void**)&ctx->t_flow, npix * 8 * nframes));
  MMT_HIP(hipMalloc((void**)&ctx->t_mask, npix * 4 * nframes));
  ctx->t_frames = nframes;
}

static void track_host_frames(mmt_ctx* ctx, int nframes, const uint8_t* const* bgr,
                              const uint16_t* const* disp, const float* const* flow,
                              const int32_t* const* mask, mmt_frame_result* res, mmt_motion* objs,
                              int objs_cap) {
  MMT_HIP(hipSetDevice(ctx->cfg.device_id));
  ensure_tracker(ctx);
  ensure_track_staging(ctx, nframes);
  const size_t npix = (size_t)ctx->cfg.width * ctx->cfg.height;
  hipStream_t s = ctx->stream;
  for (int f = 0; f < nframes; f++) {
    MMT_HIP(hipMemcpyAsync(ctx->t_bgr + npix * 3 * f, bgr[f], npix * 3, hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(ctx->t_disp + npix * f, disp[f], npix * 2, hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(ctx->t_flow + npix * 2 * f, flow[f], npix * 8, hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(ctx->t_mask + npix * f, mask[f], npix * 4, hipMemcpyHostToDevice, s));
  }
  std::vector<mmt::FrameOut> outs;
  ctx->tracker.track_chunk(ctx->t_bgr, npix * 3, ctx->t_disp, npix * 2, ctx->t_flow, npix * 8,
                           ctx->t_mask, npix * 4, nframes, outs, s);
  fill_results(outs, res, objs, objs_cap);
}

int mmt_track_rgbd(mmt_ctx* ctx, const uint8_t* bgr, const uint16_t* disp256,
                   const float* flow_uv, const int32_t* mask, double timestamp,
                   mmt_frame_result* res, mmt_motion* objs, int objs_cap) {
  (void)timestamp;
  if (!ctx || !bgr || !disp256 || !flow_uv || !mask || !res) return MMT_EINVAL;
  if (const int rc = flush_owed(ctx)) return rc;
  return guard(ctx, [&] {
    track_host_frames(ctx, 1, &bgr, &disp256, &flow_uv, &mask, res, objs, objs_cap);
  });
}

int mmt_track_rgbd_chunk(mmt_ctx* ctx, int nframes, const uint8_t* const* bgr,
                         const uint16_t* const* disp256, const float* const* flow_uv,
                         const int32_t* const* mask, mmt_frame_result* res, mmt_motion* objs,
                         int objs_cap) {
  if (!ctx || !bgr || !disp256 || !flow_uv || !mask || !res || nframes < 1) return MMT_EINVAL;
  for (int f = 0; f < nframes; f++)
    if (!bgr[f] || !disp256[f] || !flow_uv[f] || !mask[f]) return MMT_EINVAL;
  if (const int rc = flush_owed(ctx)) return rc;
  return guard(ctx, [&] {
    if (nframes > std::max(1, ctx->cfg.max_batch))
      throw ArgError("chunk larger than config.max_batch");
    track_host_frames(ctx, nframes, bgr, disp256, flow_uv, mask, res, objs, objs_cap);
  });
}

void* mmt_host_alloc(mmt_ctx* ctx, size_t bytes) {
  if (!ctx || bytes == 0) return nullptr;
  void* p = nullptr;
  if (hipSetDevice(ctx->cfg.device_id) != hipSuccess) return nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void mmt_host_free(mmt_ctx* ctx, void* p) {
  (void)ctx;
  if (p) (void)hipHostFree(p);
}

int mmt_pose_flow_solve(mmt_ctx* ctx, const mmt_flow_problem* pr, float* pose_out,
                        int* stats_out) {
  if (!ctx || !pr || !pose_out || !stats_out || pr->n < 0) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    const int n = pr->n, cap = std::max(n, 1);
    DevBuf<float2> obs(cap), flow(cap);
    DevBuf<float> depth(cap), pose(16);
    DevBuf<double> scratch(mmt::flow_scratch_doubles(cap));
    DevBuf<int> st(3);
    DevBuf<mmt::FlowSolveDesc> dd(1);
    const int groups = mmt::flow_split_groups(n);
    DevBuf<unsigned long long> gx(groups > 1 ? mmt::kFlowSplitGranules : 1);
    if (groups > 1)
      MMT_HIP(hipMemsetAsync(gx.p, 0, sizeof(unsigned long long) * mmt::kFlowSplitGranules, s));
    if (n > 0) {
      MMT_HIP(hipMemcpyAsync(obs.p, pr->obs, 8 * (size_t)n, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(flow.p, pr->flow, 8 * (size_t)n, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(depth.p, pr->depth, 4 * (size_t)n, hipMemcpyHostToDevice, s));
    }
    mmt::FlowSolveDesc d;
    memset(&d, 0, sizeof(d));
    d.n = n;
    d.obs = obs.p;
    d.flow = flow.p;
    d.depth = depth.p;
    memcpy(d.Tcw_last, pr->Tcw_last, 64);
    memcpy(d.init, pr->init, 64);
    d.rp_thres = pr->rp_thres;
    d.use_noise = pr->use_noise;
    d.g0 = pr->g0;
    d.max_iters = pr->max_iters;
    d.prior_info = pr->prior_info;
    d.fx = pr->fx; d.fy = pr->fy; d.cx = pr->cx; d.cy = pr->cy;
    d.scratch = scratch.p;
    d.cap = cap;
    d.pose_out = pose.p;
    d.stats = st.p;
    d.gx = gx.p;
    d.gx_seq = 1;
    MMT_HIP(hipMemcpyAsync(dd.p, &d, sizeof(d), hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(pose.p, pr->init, 64, hipMemcpyHostToDevice, s));
    if (groups > 1)
      mmt::launch_flow_lm_split(dd.p, groups, s);
    else
      mmt::launch_flow_lm(dd.p, 1, n, s);
    MMT_HIP(hipMemcpyAsync(pose_out, pose.p, 64, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(stats_out, st.p, 12, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
    if (stats_out[2] == 2)
      throw mmt::DeviceError("pose flow solve: the split solve's workgroups were not resident together");
  });
}

int mmt_pose_optimization(mmt_ctx* ctx, const mmt_pose_opt_problem* pr, float* pose_out,
                          uint8_t* outlier_out, int* n_inliers) {
  if (!ctx || !pr || !pose_out || !n_inliers || pr->n < 0 ||
      (pr->n > 0 && (!pr->Xw || !pr->obs || !pr->inv_sigma2 || !outlier_out)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    const int n = pr->n, cap = std::max(n, 1);
    DevBuf<float> X(3 * (size_t)cap), ob(3 * (size_t)cap), s2(cap), pose(16);
    DevBuf<uint8_t> outl(cap);
    DevBuf<int> ninl(1), fsc(n > mmt::kPoseOptMaxEdges ? cap : 1);
    DevBuf<double> esc(n > mmt::kPoseOptMaxEdges ? 3 * (size_t)cap : 1);
    DevBuf<mmt::PoseOptDesc> dd(1);
    if (n > 0) {
      MMT_HIP(hipMemcpyAsync(X.p, pr->Xw, 12 * (size_t)n, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(ob.p, pr->obs, 12 * (size_t)n, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(s2.p, pr->inv_sigma2, 4 * (size_t)n, hipMemcpyHostToDevice, s));
    }
    mmt::PoseOptDesc d;
    memset(&d, 0, sizeof(d));
    d.n = n;
    d.Xw = X.p;
    d.obs = ob.p;
    d.inv_sigma2 = s2.p;
    memcpy(d.Tcw, pr->Tcw, 64);
    d.fx = pr->fx; d.fy = pr->fy; d.cx = pr->cx; d.cy = pr->cy; d.bf = pr->bf;
    d.pose_out = pose.p;
    d.outlier = outl.p;
    d.n_inliers = ninl.p;
    d.e_scratch = esc.p;
    d.f_scratch = fsc.p;
    MMT_HIP(hipMemcpyAsync(dd.p, &d, sizeof(d), hipMemcpyHostToDevice, s));
    mmt::launch_pose_opt(dd.p, 1, n, s);
    MMT_HIP(hipMemcpyAsync(pose_out, pose.p, 64, hipMemcpyDeviceToHost, s));
    if (n > 0) MMT_HIP(hipMemcpyAsync(outlier_out, outl.p, n, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(n_inliers, ninl.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
  });
}

int mmt_frame_grid(mmt_ctx* ctx, const mmt_match_frame* cur, float* uR_out, float* depth_out,
                   int* cell_start, int* cell_idx) {
  if (!ctx || !cur || !cell_start || (cur->n > 0 && (!uR_out || !depth_out || !cell_idx)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    check_match_frame(ctx, cur, false);
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    DevMatchFrame F(ctx, cur, false);
    const size_t n = (size_t)cur->n;
    if (n) {
      MMT_HIP(hipMemcpyAsync(uR_out, F.uR.p, 4 * n, hipMemcpyDeviceToHost, s));
      MMT_HIP(hipMemcpyAsync(depth_out, F.kdepth.p, 4 * n, hipMemcpyDeviceToHost, s));
    }
    MMT_HIP(hipMemcpyAsync(cell_start, F.cell_start.p, 4 * (mmt::kGridCells + 1),
                           hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
    const int total = cell_start[mmt::kGridCells];
    if (total > 0) {
      MMT_HIP(hipMemcpyAsync(cell_idx, F.cell_idx.p, 4 * (size_t)total, hipMemcpyDeviceToHost, s));
      MMT_HIP(hipStreamSynchronize(s));
    }
  });
}

int mmt_search_by_projection_frame(mmt_ctx* ctx, const mmt_match_frame* cur,
                                   const mmt_last_frame* last, float th, int mono,
                                   int check_orientation, int32_t* match_out, int* nmatches) {
  if (!ctx || !cur || !last || !nmatches || last->n < 0 || (cur->n > 0 && !match_out) ||
      (last->n > 0 && (!last->kps || !last->Xw || !last->mp_desc || !last->active)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    check_match_frame(ctx, cur, true);
    for (int i = 0; i < last->n; i++)
      if (last->active[i] && (last->kps[i].octave < 0 || last->kps[i].octave >= ctx->orb.nlevels))
        throw ArgError("last-frame octave out of range");
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    DevMatchFrame F(ctx, cur, true);
    const int n1 = last->n;
    DevBuf<mmt_kp> lk(n1);
    DevBuf<float> X(3 * (size_t)std::max(n1, 1));
    DevBuf<uint8_t> md(32 * (size_t)std::max(n1, 1)), act(n1), obs(n1);
    DevBuf<int> match(std::max(cur->n, 1)), nm(1);
    DevCands cands(n1);
    if (n1 > 0) {
      MMT_HIP(hipMemcpyAsync(lk.p, last->kps, sizeof(mmt_kp) * (size_t)n1, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(X.p, last->Xw, 12 * (size_t)n1, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(md.p, last->mp_desc, 32 * (size_t)n1, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(act.p, last->active, (size_t)n1, hipMemcpyHostToDevice, s));
      if (last->obs)
        MMT_HIP(hipMemcpyAsync(obs.p, last->obs, (size_t)n1, hipMemcpyHostToDevice, s));
    }
    mmt::LastFrameDev L;
    L.keys = lk.p;
    L.Xw = X.p;
    L.mp_desc = md.p;
    L.active = act.p;
    L.obs = last->obs ? obs.p : nullptr;
    L.n = n1;
    memcpy(L.Tcw, last->Tcw, 64);
    mmt::launch_sbp_frame(F.G, cur->Tcw, L, th, mono, check_orientation, cands.set(), match.p,
                          nm.p, s);
    if (cur->n > 0)
      MMT_HIP(hipMemcpyAsync(match_out, match.p, 4 * (size_t)cur->n, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(nmatches, nm.p, 4, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
  });
}

// host checks of a feature vector: ascending node ids, monotone starts from 0, features in
// [0, n); `once` (n bytes, optional) rejects a feature listed twice; nodes of at most max_node
static void check_feature_vector(const mmt_feature_vector* v, int n, std::vector<uint8_t>* once,
                                 int max_node) {
  if (v->n_nodes < 0) throw ArgError("negative node count");
  if (v->n_nodes == 0) return;
  if (!v->node_id || !v->node_start || !v->feat) throw ArgError("null feature vector arrays");
  if (v->node_start[0] != 0) throw ArgError("node_start[0] != 0");
  for (int k = 0; k < v->n_nodes; k++) {
    if (k > 0 && !(v->node_id[k - 1] < v->node_id[k])) throw ArgError("node ids not ascending");
    const int a = v->node_start[k], b = v->node_start[k + 1];
    if (b < a) throw ArgError("node_start not monotone");
    if (b - a > max_node) throw ArgError("a vocabulary node holds more than 2048 frame features");
    for (int q = a; q < b; q++) {
      const int f = v->feat[q];
      if (f < 0 || f >= n) throw ArgError("feature index out of range");
      if (once) {
        if ((*once)[f]) throw ArgError("a frame feature is listed in two nodes");
        (*once)[f] = 1;
      }
    }
  }
}

int mmt_fuse_candidates(mmt_ctx* ctx, const mmt_match_frame* kf, const mmt_local_points* pts,
                        float th, int32_t* best_idx, int32_t* best_dist) {
  if (!ctx || !kf || !pts || pts->m < 0 || (pts->m > 0 && (!best_idx || !best_dist || !pts->Xw ||
                                                           !pts->normal || !pts->min_dist ||
                                                           !pts->max_dist || !pts->desc)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    check_match_frame(ctx, kf, true);
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    DevMatchFrame F(ctx, kf, true);
    const int m = pts->m;
    std::vector<mmt::LocalPointDev> hp(std::max(m, 1));
    std::vector<mmt::FuseQuery> hq(std::max(m, 1));
    for (int j = 0; j < m; j++) {
      mmt::LocalPointDev& p = hp[j];
      memset(&p, 0, sizeof(p));
      memcpy(p.Xw, pts->Xw + 3 * (size_t)j, 12);
      memcpy(p.normal, pts->normal + 3 * (size_t)j, 12);
      p.min_dist = pts->min_dist[j];
      p.max_dist = pts->max_dist[j];
      hq[j] = mmt::FuseQuery{0, j};
    }
    mmt::FuseKF K;
    memset(&K, 0, sizeof(K));
    K.keys = F.G.keys;
    K.desc = F.G.desc;
    K.uR = F.G.uR;
    K.cell_start = F.G.cell_start;
    K.cell_idx = F.G.cell_idx;
    K.n = kf->n;
    memcpy(K.Tcw, kf->Tcw, 64);
    for (int r = 0; r < 3; r++) {  // KeyFrame::SetPose: Ow = -Rcw^T tcw
      double acc = 0;
      for (int k = 0; k < 3; k++) acc += (double)kf->Tcw[4 * k + r] * (double)kf->Tcw[4 * k + 3];
      K.Ow[r] = -(float)acc;
    }
    mmt::FuseCam c;
    memset(&c, 0, sizeof(c));
    const mmt_config& cf = ctx->cfg;
    c.fx = cf.fx; c.fy = cf.fy; c.cx = cf.cx; c.cy = cf.cy; c.bf = cf.bf;
    c.W = (float)cf.width;
    c.H = (float)cf.height;
    c.invW = F.G.invW;
    c.invH = F.G.invH;
    c.logScale = F.G.logScale;
    c.th = th;
    c.nlevels = ctx->orb.nlevels;
    for (int l = 0; l < c.nlevels && l < mmt::kMaxLevels; l++) {
      c.scale[l] = ctx->orb.scale[l];
      c.invSigma2[l] = ctx->orb.invSigma2[l];
    }
    DevBuf<mmt::LocalPointDev> dp(m);
    DevBuf<uint8_t> pd(32 * (size_t)std::max(m, 1));
    DevBuf<mmt::FuseKF> dk(1);
    DevBuf<mmt::FuseQuery> dq(m);
    DevBuf<int2> out(m);
    MMT_HIP(hipMemcpyAsync(dk.p, &K, sizeof(K), hipMemcpyHostToDevice, s));
    if (m > 0) {
      MMT_HIP(hipMemcpyAsync(dp.p, hp.data(), sizeof(mmt::LocalPointDev) * (size_t)m,
                             hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(pd.p, pts->desc, 32 * (size_t)m, hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(dq.p, hq.data(), sizeof(mmt::FuseQuery) * (size_t)m,
                             hipMemcpyHostToDevice, s));
    }
    mmt::launch_fuse_cand(dk.p, dq.p, m, dp.p, pd.p, c, out.p, s);
    std::vector<int2> ho(std::max(m, 1));
    if (m > 0)
      MMT_HIP(hipMemcpyAsync(ho.data(), out.p, sizeof(int2) * (size_t)m, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
    for (int j = 0; j < m; j++) {
      best_idx[j] = ho[j].x;
      best_dist[j] = ho[j].y;
    }
  });
}

int mmt_local_bundle_adjustment(mmt_ctx* ctx, const mmt_ba_problem* p, float* Tcw_out,
                                float* Xw_out, uint8_t* erase_out, int32_t* stats) {
  if (!ctx || !p || !stats || p->n_kf < 0 || p->n_pt < 0 || p->n_edge < 0 ||
      (p->n_kf > 0 && (!p->Tcw || !p->fixed || !Tcw_out)) ||
      (p->n_pt > 0 && (!p->Xw || !Xw_out)) ||
      (p->n_edge > 0 && (!p->e_pt || !p->e_kf || !p->e_obs || !p->e_inv_sigma2 || !erase_out)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    mmt::BAHostProblem P;
    P.n_kf = p->n_kf;
    P.n_pt = p->n_pt;
    P.n_edge = p->n_edge;
    P.Tcw = p->Tcw;
    P.fixed = p->fixed;
    P.Xw = p->Xw;
    P.e_pt = p->e_pt;
    P.e_kf = p->e_kf;
    P.e_obs = p->e_obs;
    P.e_s = p->e_inv_sigma2;
    const mmt_config& c = ctx->cfg;
    P.fx = c.fx; P.fy = c.fy; P.cx = c.cx; P.cy = c.cy; P.bf = c.bf;
    mmt::BARunner& runner = ctx->ba;
    std::vector<float> T(16 * (size_t)std::max(p->n_kf, 1)), X(3 * (size_t)std::max(p->n_pt, 1));
    std::vector<uint8_t> er(std::max(p->n_edge, 1));
    int st[5] = {0, 0, 0, 0, 0};
    runner.run(P, ctx->stream, T.data(), X.data(), er.data(), st);
    if (p->n_kf > 0) memcpy(Tcw_out, T.data(), 64 * (size_t)p->n_kf);
    if (p->n_pt > 0) memcpy(Xw_out, X.data(), 12 * (size_t)p->n_pt);
    if (p->n_edge > 0) memcpy(erase_out, er.data(), (size_t)p->n_edge);
    for (int i = 0; i < 5; i++) stats[i] = st[i];
  });
}

int mmt_frame_samples(mmt_ctx* ctx, float* static_xy, int static_cap, int* n_static,
                      float* obj_xy, int32_t* obj_label, int obj_cap, int* n_obj) {
  if (!ctx || !n_static || !n_obj || static_cap < 0 || obj_cap < 0) return MMT_EINVAL;
  return guard(ctx, [&] {
    *n_static = *n_obj = 0;
    if (!ctx->tracker_ready) return;
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ctx->tracker.frame_samples(static_xy, static_cap, n_static, obj_xy, obj_label, obj_cap, n_obj,
                               ctx->stream);
  });
}

int mmt_map_counters_read(mmt_ctx* ctx, mmt_map_counters* out) {
  if (!ctx || !out) return MMT_EINVAL;
  return guard(ctx, [&] {
    memset(out, 0, sizeof(*out));
    if (!ctx->tracker_ready) return;
    const mmt::MappingStats& m = ctx->tracker.mapping_stats();
    out->n_ba = m.n_ba;
    out->n_fused = m.n_fused;
    out->n_culled = m.n_culled;
    out->n_ba_erased = m.n_ba_erased;
    out->ba_trials = m.ba_trials;
    out->ba_edges = m.ba_edges;
    out->ba_kfs = m.ba_kfs;
    out->ba_pts = m.ba_pts;
    out->ba_max_opt = m.ba_max_opt;
    out->fuse_launches = m.fuse_launches;
    out->fuse_queries = m.fuse_queries;
    out->fuse_relaunches = m.fuse_relaunches;
    out->lm_us = m.lm_us;
    out->ba_us = m.ba_us;
    out->fuse_us = m.fuse_us;
    out->d2_split_fallbacks = ctx->tracker.split_fallbacks();
    out->n_reparent = m.n_reparent;
  });
}

int mmt_set_keyframe_culling_ratio(mmt_ctx* ctx, double ratio) {
  if (!ctx || !(ratio >= 0)) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ensure_tracker(ctx);
    ctx->tracker.set_cull_ratio(ratio);
  });
}

int mmt_load_vocabulary(mmt_ctx* ctx, const char* path) {
  if (!ctx || !path) return MMT_EINVAL;
  bool late = false;
  const int rc = guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    ensure_tracker(ctx);
    if (ctx->tracker.map().n_keyframes() > 0 || ctx->tracker.map().state() != 0) {
      late = true;
      return;
    }
    std::unique_ptr<mmt::Vocabulary> v(new mmt::Vocabulary());
    v->load_text(path);
    ctx->tracker.set_vocabulary(v.get());
    ctx->voc = std::move(v);
  });
  if (rc == MMT_OK && late) {
    ctx->err = "mmt_load_vocabulary: load the vocabulary before the first frame";
    return MMT_ESTATE;
  }
  return rc;
}

int mmt_bow_transform(mmt_ctx* ctx, const uint8_t* desc, int n, int levelsup, uint32_t* word,
                      double* weight, uint32_t* node) {
  if (!ctx || n < 0 || (n > 0 && (!desc || !word || !weight || !node))) return MMT_EINVAL;
  return guard(ctx, [&] {
    if (!ctx->voc) throw mmt::ArgError("mmt_bow_transform: no vocabulary loaded");
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    if (n == 0) return;
    ctx->voc->upload();
    hipStream_t s = ctx->stream;
    DevBuf<uint8_t> d(32 * (size_t)n);
    DevBuf<uint32_t> w(n), nd(n);
    DevBuf<double> x(n);
    MMT_HIP(hipMemcpyAsync(d.p, desc, 32 * (size_t)n, hipMemcpyHostToDevice, s));
    mmt::launch_bow_transform(ctx->voc->dev, d.p, n, levelsup, w.p, x.p, nd.p, s);
    MMT_HIP(hipMemcpyAsync(word, w.p, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(weight, x.p, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(node, nd.p, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
  });
}

int mmt_bow_counters_read(mmt_ctx* ctx, mmt_bow_counters* out) {
  if (!ctx || !out) return MMT_EINVAL;
  return guard(ctx, [&] {
    memset(out, 0, sizeof(*out));
    if (!ctx->tracker_ready) return;
    const mmt::BowStatsH& b = ctx->tracker.bow_stats();
    out->bow_frames = b.n_bow_frames;
    out->trk = b.n_trk;
    out->trk_ok = b.n_trk_ok;
    out->reloc = b.n_reloc;
    out->reloc_ok = b.n_reloc_ok;
    out->reloc_cands = b.n_reloc_cands;
    out->pnp_found = b.n_pnp_found;
    out->sbp_rounds = b.n_sbp_rounds;
    out->triangulated = b.n_triangulated;
    out->sft_matches = b.n_sft_matches;
    out->kfdb = b.n_kfdb;
  });
}

int mmt_map_dump(mmt_ctx* ctx, int32_t* sizes, const mmt_map_dump_arrays* out) {
  if (!ctx || !sizes) return MMT_EINVAL;
  return guard(ctx, [&] {
    if (!ctx->tracker_ready) {
      memset(sizes, 0, 7 * sizeof(int32_t));
      return;
    }
    ctx->tracker.map().dump(sizes, out);
  });
}

int mmt_search_by_bow(mmt_ctx* ctx, const mmt_bow_keyframe* kf, int n_cur, const mmt_kp* cur_kps,
                      const uint8_t* cur_desc, const mmt_feature_vector* cur_fv, float nn_ratio,
                      int check_orientation, int32_t* match_out, int* nmatches) {
  if (!ctx || !kf || !cur_fv || !nmatches || kf->n < 0 || n_cur < 0 ||
      (n_cur > 0 && (!match_out || !cur_kps || !cur_desc)) ||
      (kf->n > 0 && (!kf->kps || !kf->desc || !kf->mp_valid)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    check_feature_vector(&kf->fv, kf->n, nullptr, INT32_MAX);
    std::vector<uint8_t> once((size_t)std::max(n_cur, 1), 0);
    check_feature_vector(cur_fv, n_cur, &once, mmt::kBowMaxNodeFeatures);
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    const int nk = kf->n, nkn = kf->fv.n_nodes, nfn = cur_fv->n_nodes;
    const int nkfeat = nkn > 0 ? kf->fv.node_start[nkn] : 0;
    const int nffeat = nfn > 0 ? cur_fv->node_start[nfn] : 0;
    DevBuf<mmt_kp> kk(nk), fk(n_cur);
    DevBuf<uint8_t> kd(32 * (size_t)nk), ok(nk), fd(32 * (size_t)n_cur);
    DevBuf<uint32_t> kn(nkn), fnode(nfn);
    DevBuf<int> ks(nkn + 1), kfe(nkfeat), fs(nfn + 1), ffe(nffeat);
    DevBuf<int> match(n_cur), hist(32), cnt(2);
    auto up = [&](void* d, const void* h, size_t bytes) {
      if (bytes) MMT_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    };
    up(kk.p, kf->kps, sizeof(mmt_kp) * (size_t)nk);
    up(kd.p, kf->desc, 32 * (size_t)nk);
    up(ok.p, kf->mp_valid, (size_t)nk);
    up(fk.p, cur_kps, sizeof(mmt_kp) * (size_t)n_cur);
    up(fd.p, cur_desc, 32 * (size_t)n_cur);
    if (nkn > 0) {
      up(kn.p, kf->fv.node_id, 4 * (size_t)nkn);
      up(ks.p, kf->fv.node_start, 4 * (size_t)(nkn + 1));
      up(kfe.p, kf->fv.feat, 4 * (size_t)nkfeat);
    }
    if (nfn > 0) {
      up(fnode.p, cur_fv->node_id, 4 * (size_t)nfn);
      up(fs.p, cur_fv->node_start, 4 * (size_t)(nfn + 1));
      up(ffe.p, cur_fv->feat, 4 * (size_t)nffeat);
    }
    mmt::BowFeatVec a{nkn, kn.p, ks.p, kfe.p}, b{nfn, fnode.p, fs.p, ffe.p};
    mmt::launch_search_by_bow(a, kk.p, kd.p, ok.p, b, fk.p, fd.p, n_cur, nn_ratio,
                              check_orientation, match.p, hist.p, cnt.p, s);
    if (n_cur > 0)
      MMT_HIP(hipMemcpyAsync(match_out, match.p, 4 * (size_t)n_cur, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(nmatches, cnt.p + 1, 4, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
  });
}

int mmt_search_local_points(mmt_ctx* ctx, const mmt_match_frame* cur,
                            const mmt_local_points* pts, float th, const uint8_t* taken,
                            int32_t* match_out, float* frustum_out, int* nmatches) {
  if (!ctx || !cur || !pts || !nmatches || pts->m < 0 || (cur->n > 0 && !match_out) ||
      (pts->m > 0 && (!pts->Xw || !pts->normal || !pts->min_dist || !pts->max_dist ||
                      !pts->desc || !pts->skip)))
    return MMT_EINVAL;
  return guard(ctx, [&] {
    check_match_frame(ctx, cur, true);
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    DevMatchFrame F(ctx, cur, true);
    const int m = pts->m;
    std::vector<mmt::LocalPointDev> hp(std::max(m, 1));
    for (int j = 0; j < m; j++) {
      mmt::LocalPointDev& p = hp[j];
      memset(&p, 0, sizeof(p));
      memcpy(p.Xw, pts->Xw + 3 * (size_t)j, 12);
      memcpy(p.normal, pts->normal + 3 * (size_t)j, 12);
      p.min_dist = pts->min_dist[j];
      p.max_dist = pts->max_dist[j];
      p.skip = pts->skip[j] != 0;
    }
    DevBuf<mmt::LocalPointDev> dp(m);
    DevBuf<uint8_t> pd(32 * (size_t)std::max(m, 1)), tk(std::max(cur->n, 1));
    DevBuf<mmt::FrustumRec> fr(m);
    DevBuf<int> match(std::max(cur->n, 1)), nm(1);
    DevCands cands(m);
    if (m > 0) {
      MMT_HIP(hipMemcpyAsync(dp.p, hp.data(), sizeof(mmt::LocalPointDev) * (size_t)m,
                             hipMemcpyHostToDevice, s));
      MMT_HIP(hipMemcpyAsync(pd.p, pts->desc, 32 * (size_t)m, hipMemcpyHostToDevice, s));
    }
    if (taken && cur->n > 0)
      MMT_HIP(hipMemcpyAsync(tk.p, taken, (size_t)cur->n, hipMemcpyHostToDevice, s));
    mmt::launch_search_local(F.G, cur->Tcw, dp.p, pd.p, m, th, taken ? tk.p : nullptr, fr.p,
                             cands.set(), match.p, nm.p, s);
    std::vector<mmt::FrustumRec> hfr(std::max(m, 1));
    if (cur->n > 0)
      MMT_HIP(hipMemcpyAsync(match_out, match.p, 4 * (size_t)cur->n, hipMemcpyDeviceToHost, s));
    if (m > 0)
      MMT_HIP(hipMemcpyAsync(hfr.data(), fr.p, sizeof(mmt::FrustumRec) * (size_t)m,
                             hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(nmatches, nm.p, 4, hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
    if (frustum_out)
      for (int j = 0; j < m; j++) {
        float* o = frustum_out + 6 * (size_t)j;
        o[0] = (float)hfr[j].in_view;
        o[1] = (float)hfr[j].level;
        o[2] = hfr[j].u;
        o[3] = hfr[j].v;
        o[4] = hfr[j].uR;
        o[5] = hfr[j].view_cos;
      }
  });
}

int mmt_pnp_ransac(mmt_ctx* ctx, const float* pts3, const float* pts2, int n, float fx,
                   float fy, float cx, float cy, int max_iters, double reproj, double confidence,
                   double* R_out, double* t_out, int* inliers_out, int* n_inliers,
                   int* iters_out) {
  if (!ctx || !pts3 || !pts2 || !R_out || !t_out || !n_inliers || !iters_out || n < 5 ||
      max_iters < 1)
    return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    hipStream_t s = ctx->stream;
    const int words = (n + 63) / 64;
    DevBuf<float> p3(3 * (size_t)n);
    DevBuf<float2> p2(n);
    DevBuf<int> dn(1), sub(5 * (size_t)max_iters), good(max_iters), inl(n), mm(n), subset(n),
        nsub(1), res(8);
    DevBuf<double> models(6 * (size_t)max_iters), Rt(12);
    DevBuf<double> hrec((size_t)mmt::kHypRec * max_iters), hout((size_t)3 * mmt::kHypOut * max_iters);
    DevBuf<unsigned long long> masks((size_t)max_iters * words);
    DevBuf<mmt::PnPObject> po(1);
    std::vector<int> h_sub;
    mmt::ransac_subsets(n, max_iters, h_sub);
    MMT_HIP(hipMemcpyAsync(p3.p, pts3, 12 * (size_t)n, hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(p2.p, pts2, 8 * (size_t)n, hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(dn.p, &n, 4, hipMemcpyHostToDevice, s));
    MMT_HIP(hipMemcpyAsync(sub.p, h_sub.data(), 4 * h_sub.size(), hipMemcpyHostToDevice, s));
    mmt::PnPObject o;
    memset(&o, 0, sizeof(o));
    o.n = dn.p;
    o.fx = fx; o.fy = fy; o.cx = cx; o.cy = cy;
    o.reproj = reproj;
    o.confidence = confidence;
    o.subsets = sub.p;
    o.pts3 = p3.p;
    o.pts2 = p2.p;
    o.models = models.p;
    o.hrec = hrec.p;
    o.hout = hout.p;
    o.good = good.p;
    o.masks = masks.p;
    o.mask_words = words;
    o.inliers = inl.p;
    o.mm_inliers = mm.p;
    o.subset = subset.p;
    o.n_subset = nsub.p;
    o.result = res.p;
    o.Rt = Rt.p;
    MMT_HIP(hipMemcpyAsync(po.p, &o, sizeof(o), hipMemcpyHostToDevice, s));
    mmt::launch_pnp(po.p, 1, max_iters, s, false);
    int r[8];
    double rt[12];
    MMT_HIP(hipMemcpyAsync(r, res.p, sizeof(r), hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(rt, Rt.p, sizeof(rt), hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
    const int ni = r[0] >= 0 ? r[3] : 0;
    if (inliers_out && ni > 0)
      MMT_HIP(hipMemcpy(inliers_out, inl.p, 4 * (size_t)ni, hipMemcpyDeviceToHost));
    memcpy(R_out, rt, 72);
    memcpy(t_out, rt + 9, 24);
    *n_inliers = ni;
    iters_out[0] = r[2];
    iters_out[1] = r[0];
  });
}

// PnPsolver::SetRansacParameters + iterate (PnPsolver.cc:119-264): the hypotheses of every
// iteration this call can run are built and scored on the GPU in one batch (k_pnp_hyp<4>,
// k_pnp_beta<4>, k_p4p_check); the host replays iterate()'s loop over their inlier counts, and
// every Refine() it reaches runs on the GPU (EPnP over the best inliers + CheckInliers).
}  // extern "C"

// PnPsolver::iterate on the GPU (the C-ABI probe mmt_pnpsolver_iterate and the tracker's
// Relocalization): SetRansacParameters' arithmetic, every hypothesis the call can run scored in
// one launch, the host replaying iterate()'s loop and Refine() on the GPU
void mmt::pnpsolver_iterate_gpu(hipStream_t s, const mmt_pnpsolver_problem* pr,
                                const int32_t* randi, int n_draw_iters, int n_iterations,
                                mmt_pnpsolver_state* st, float* Tcw_out, uint8_t* inliers_out,
                                int* n_inliers, int* pose_found, int* no_more) {
  if (pr->min_set != 4) throw mmt::ArgError("PnPsolver: min_set must be 4 (P4P)");
  const int N = pr->n;
  // ---- SetRansacParameters (PnPsolver.cc:119-152), the reference's int/float arithmetic
  float eps = pr->epsilon;
  int minInl = pr->min_inliers;
  int nMinInliers = (int)(N * eps);
  if (nMinInliers < minInl) nMinInliers = minInl;
  if (nMinInliers < pr->min_set) nMinInliers = pr->min_set;
  minInl = nMinInliers;
  if (N > 0 && eps < (float)minInl / N) eps = (float)minInl / N;
  int nIt;
  if (minInl == N)
    nIt = 1;
  else
    nIt = (int)ceil(log(1 - pr->probability) / log(1 - pow(eps, 3)));
  const int maxIts = std::max(1, std::min(nIt, pr->max_iterations));
  // ---- iterate() (PnPsolver.cc:160-264)
  *no_more = 0;
  *pose_found = 0;
  *n_inliers = 0;
  memset(inliers_out, 0, (size_t)N);
  if (N < minInl) {
    *no_more = 1;
    return;
  }
  const int it0 = st->iterations;
  const int K = std::max(maxIts - it0, n_iterations);  // while (its < max || cur < nIt)
  if (K > n_draw_iters) throw mmt::ArgError("PnPsolver: randi covers fewer iterations than the call runs");
  const int words = (N + 63) / 64;
  // minimal sets: RandomInt draws through vAvailableIndices' swap-with-last removal
  std::vector<int> sub(4 * (size_t)std::max(K, 1));
  std::vector<int> avail(N);
  for (int k = 0; k < K; k++) {
    for (int i = 0; i < N; i++) avail[i] = i;
    int sz = N;
    for (int j = 0; j < 4; j++) {
      const int r = randi[4 * (size_t)k + j];
      if (r < 0 || r >= sz) throw mmt::ArgError("PnPsolver: randi value outside [0, n-1-j]");
      sub[4 * (size_t)k + j] = avail[r];
      avail[r] = avail[sz - 1];
      sz--;
    }
  }
  std::vector<float> maxErr(N);
  for (int i = 0; i < N; i++) maxErr[i] = pr->sigma2[i] * pr->th2;
  const int rows = K + 2;  // hypothesis masks, then the refine's input and output rows
  DevBuf<float> p3(3 * (size_t)N + 1), merr((size_t)N + 1);
  DevBuf<float2> p2((size_t)N + 1);
  DevBuf<int> dn(1), dsub(sub.size()), good((size_t)K + 1), inl((size_t)N + 1), res(8);
  DevBuf<double> hrec((size_t)mmt::kHypRec * std::max(K, 1)),
      hout((size_t)3 * mmt::kHypOut * std::max(K, 1)), hrt(12 * (size_t)std::max(K, 1)), Rt(12);
  DevBuf<unsigned long long> masks((size_t)rows * words + 1);
  DevBuf<mmt::PnPObject> po(1);
  MMT_HIP(hipMemcpyAsync(p3.p, pr->pts3, 12 * (size_t)N, hipMemcpyHostToDevice, s));
  MMT_HIP(hipMemcpyAsync(p2.p, pr->pts2, 8 * (size_t)N, hipMemcpyHostToDevice, s));
  MMT_HIP(hipMemcpyAsync(merr.p, maxErr.data(), 4 * (size_t)N, hipMemcpyHostToDevice, s));
  MMT_HIP(hipMemcpyAsync(dn.p, &N, 4, hipMemcpyHostToDevice, s));
  MMT_HIP(hipMemcpyAsync(dsub.p, sub.data(), 4 * sub.size(), hipMemcpyHostToDevice, s));
  mmt::PnPObject o;
  memset(&o, 0, sizeof(o));
  o.n = dn.p;
  o.fx = pr->fx; o.fy = pr->fy; o.cx = pr->cx; o.cy = pr->cy;
  o.subsets = dsub.p;
  o.pts3 = p3.p;
  o.pts2 = p2.p;
  o.hrec = hrec.p;
  o.hout = hout.p;
  o.good = good.p;
  o.masks = masks.p;
  o.mask_words = words;
  o.inliers = inl.p;
  o.result = res.p;
  o.Rt = Rt.p;
  o.raw_pixels = 1;
  o.rt_raw = 1;
  o.max_err = merr.p;
  o.hrt = hrt.p;
  MMT_HIP(hipMemcpyAsync(po.p, &o, sizeof(o), hipMemcpyHostToDevice, s));
  std::vector<int> h_good(std::max(K, 1));
  if (K > 0) {
    mmt::launch_p4p_hypotheses(po.p, K, s);
    MMT_HIP(hipMemcpyAsync(h_good.data(), good.p, 4 * (size_t)K, hipMemcpyDeviceToHost, s));
  }
  MMT_HIP(hipStreamSynchronize(s));
  auto fetch_mask = [&](int row, uint8_t* out) {
    std::vector<unsigned long long> w(words);
    MMT_HIP(hipMemcpy(w.data(), masks.p + (size_t)row * words, 8 * (size_t)words,
                      hipMemcpyDeviceToHost));
    for (int i = 0; i < N; i++) out[i] = (uint8_t)((w[i >> 6] >> (i & 63)) & 1ull);
  };
  auto pose_to_Tcw = [](const double* Rt12, float* T) {  // cv::Mat(R, t).convertTo(CV_32F)
    for (int r = 0; r < 4; r++)
      for (int c = 0; c < 4; c++) T[4 * r + c] = (r == c) ? 1.f : 0.f;
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) T[4 * r + c] = (float)Rt12[3 * r + c];
      T[4 * r + 3] = (float)Rt12[9 + r];
    }
  };
  // Refine() of the current best set (st->best_mask), cached while the best set is unchanged
  bool refined_valid = false;
  int refined_n = 0;
  float refined_T[16];
  std::vector<uint8_t> refined_mask(N);
  auto refine = [&]() {
    if (refined_valid) return;
    std::vector<unsigned long long> w(words, 0ull);
    for (int i = 0; i < N; i++)
      if (st->best_mask[i]) w[i >> 6] |= 1ull << (i & 63);
    MMT_HIP(hipMemcpyAsync(masks.p + (size_t)K * words, w.data(), 8 * (size_t)words,
                           hipMemcpyHostToDevice, s));
    mmt::launch_p4p_refine(po.p, K, K + 1, s);
    int r[8];
    double rt[12];
    MMT_HIP(hipMemcpyAsync(r, res.p, sizeof(r), hipMemcpyDeviceToHost, s));
    MMT_HIP(hipMemcpyAsync(rt, Rt.p, sizeof(rt), hipMemcpyDeviceToHost, s));
    MMT_HIP(hipStreamSynchronize(s));
    refined_n = r[6];
    pose_to_Tcw(rt, refined_T);
    fetch_mask(K + 1, refined_mask.data());
    refined_valid = true;
  };
  for (int k = 0; k < K; k++) {
    st->iterations = it0 + k + 1;
    const int g = h_good[k];
    if (g >= minInl) {
      if (g > st->best_inliers) {
        fetch_mask(k, st->best_mask);
        st->best_inliers = g;
        double rt[12];
        MMT_HIP(hipMemcpy(rt, hrt.p + 12 * (size_t)k, sizeof(rt), hipMemcpyDeviceToHost));
        pose_to_Tcw(rt, st->best_Tcw);
        refined_valid = false;
      }
      refine();
      if (refined_n > minInl) {  // Refine() succeeded: return the refined pose
        *pose_found = 1;
        *n_inliers = refined_n;
        memcpy(inliers_out, refined_mask.data(), (size_t)N);
        memcpy(Tcw_out, refined_T, sizeof(refined_T));
        return;
      }
    }
  }
  if (st->iterations >= maxIts) {
    *no_more = 1;
    if (st->best_inliers >= minInl) {
      *pose_found = 1;
      *n_inliers = st->best_inliers;
      memcpy(inliers_out, st->best_mask, (size_t)N);
      memcpy(Tcw_out, st->best_Tcw, sizeof(st->best_Tcw));
    }
  }
}

extern "C" {

int mmt_pnpsolver_iterate(mmt_ctx* ctx, const mmt_pnpsolver_problem* pr, const int32_t* randi,
                          int n_draw_iters, int n_iterations, mmt_pnpsolver_state* st,
                          float* Tcw_out, uint8_t* inliers_out, int* n_inliers, int* pose_found,
                          int* no_more) {
  if (!ctx || !pr || !st || !Tcw_out || !inliers_out || !n_inliers || !pose_found || !no_more ||
      pr->n < 0 || !st->best_mask || n_iterations < 0 || n_draw_iters < 0)
    return MMT_EINVAL;
  if (pr->n > 0 && (!pr->pts3 || !pr->pts2 || !pr->sigma2)) return MMT_EINVAL;
  return guard(ctx, [&] {
    MMT_HIP(hipSetDevice(ctx->cfg.device_id));
    mmt::pnpsolver_iterate_gpu(ctx->stream, pr, randi, n_draw_iters, n_iterations, st, Tcw_out,
                               inliers_out, n_inliers, pose_found, no_more);
  });
}

long mmt_debug_fetch(mmt_ctx* ctx, int what, int frame, void* out, size_t cap) {
  if (!ctx || !out) return MMT_EINVAL;
  long r = 0;
  const int rc = guard(ctx, [&] { r = ctx->engine.debug_fetch(what, frame, out, cap, ctx->stream); });
  return rc ? rc : r;
}

}  // extern "C"
