// multimot_track_amd/csrc/mmt_capi.hip -- the C-ABI of libmmt (include/mmt.h).
// Every entry point catches internal exceptions and returns an errno-style code; nothing exits.

#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

#include "mmt_internal.h"

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
    MMT_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
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
      MMT_HIP(hipStreamSynchronize(ctx->stream));
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

long mmt_debug_fetch(mmt_ctx* ctx, int what, int frame, void* out, size_t cap) {
  if (!ctx || !out) return MMT_EINVAL;
  long r = 0;
  const int rc = guard(ctx, [&] { r = ctx->engine.debug_fetch(what, frame, out, cap, ctx->stream); });
  return rc ? rc : r;
}

}  // extern "C"
