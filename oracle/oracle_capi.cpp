// oracle/oracle_capi.cpp -- TEST INFRASTRUCTURE ONLY.
// Flat C entry points so tests/ and bench.py (cpu_baseline leg) can drive the CPU restatement
// through ctypes.  Never linked into the product library.

#include <algorithm>
#include <cstring>

#include "oracle_common.h"

using namespace oracle;

extern "C" {

int oracle_orb_config(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th,
                      float* scale, float* sigma2, int* n_per_level, int* umax16) {
  OrbConfig c;
  orb_config_init(c, nfeatures, scale_factor, nlevels, ini_th, min_th);
  for (int l = 0; l < nlevels; l++) {
    scale[l] = c.scale[l];
    sigma2[l] = c.sigma2[l];
    n_per_level[l] = c.nPerLevel[l];
  }
  for (int v = 0; v < 16; v++) umax16[v] = c.umax[v];
  return 0;
}

int oracle_level_sizes(int nfeatures, float scale_factor, int nlevels, int w, int h, int* lw,
                       int* lh) {
  OrbConfig c;
  orb_config_init(c, nfeatures, scale_factor, nlevels, 20, 7);
  orb_level_sizes(c, w, h, lw, lh);
  return 0;
}

int oracle_gray_from_bgr(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray) {
  gray_from_bgr(bgr, w, h, stride, gray);
  return 0;
}

// Pyramid levels concatenated level-major, each unpadded w_l*h_l bytes.
int oracle_pyramid(const uint8_t* gray, int w, int h, int nlevels, float scale_factor,
                   uint8_t* out) {
  OrbConfig c;
  orb_config_init(c, 1000, scale_factor, nlevels, 20, 7);
  std::vector<Image> pyr;
  compute_pyramid(c, gray, w, h, pyr);
  size_t off = 0;
  for (auto& im : pyr) {
    memcpy(out + off, im.px.data(), im.px.size());
    off += im.px.size();
  }
  return 0;
}

int oracle_blur7(const uint8_t* src, int w, int h, uint8_t* dst) {
  Image s, d;
  s.w = w;
  s.h = h;
  s.px.assign(src, src + (size_t)w * h);
  gaussian_blur7(s, d);
  memcpy(dst, d.px.data(), d.px.size());
  return 0;
}

float oracle_fast_atan2(float y, float x) { return fast_atan2_deg(y, x); }

// FAST candidates of one level (coordinates relative to minBorder, before the octree), as
// (x, y, response) float triples.  Returns the count (or -count-needed if cap too small).
int oracle_level_candidates(const uint8_t* img, int w, int h, int ini_th, int min_th,
                            float* xyr, int cap) {
  OrbConfig c;
  orb_config_init(c, 1000, 1.2f, 1, ini_th, min_th);
  Image im;
  im.w = w;
  im.h = h;
  im.px.assign(img, img + (size_t)w * h);
  std::vector<Key> out, cand;
  level_keypoints(c, im, 0, out, &cand);
  if ((int)cand.size() > cap) return -(int)cand.size();
  for (size_t i = 0; i < cand.size(); i++) {
    xyr[3 * i] = cand[i].x;
    xyr[3 * i + 1] = cand[i].y;
    xyr[3 * i + 2] = cand[i].response;
  }
  return (int)cand.size();
}

// DistributeOctTree on an explicit candidate list (x, y, response triples).
int oracle_distribute(const float* xyr, int n, int min_x, int max_x, int min_y, int max_y,
                      int nfeat, float* out_xyr, int cap) {
  std::vector<Key> keys(n);
  for (int i = 0; i < n; i++) {
    keys[i].x = xyr[3 * i];
    keys[i].y = xyr[3 * i + 1];
    keys[i].response = xyr[3 * i + 2];
  }
  std::vector<Key> r = distribute_octree(keys, min_x, max_x, min_y, max_y, nfeat);
  if ((int)r.size() > cap) return -(int)r.size();
  for (size_t i = 0; i < r.size(); i++) {
    out_xyr[3 * i] = r[i].x;
    out_xyr[3 * i + 1] = r[i].y;
    out_xyr[3 * i + 2] = r[i].response;
  }
  return (int)r.size();
}

// Full ORBextractor::operator(): keypoints as 7-word records (x,y,size,angle,response as float
// bits, octave, class_id as int) + N x 32 descriptors.
int oracle_orb_extract(const uint8_t* gray, int w, int h, int nfeatures, float scale_factor,
                       int nlevels, int ini_th, int min_th, void* kps_out, uint8_t* desc_out,
                       int cap, int* n_out) {
  OrbConfig c;
  orb_config_init(c, nfeatures, scale_factor, nlevels, ini_th, min_th);
  std::vector<Key> kps;
  std::vector<uint8_t> desc;
  orb_extract(c, gray, w, h, kps, desc, nullptr, nullptr);
  *n_out = (int)kps.size();
  if ((int)kps.size() > cap) return -1;
  memcpy(kps_out, kps.data(), kps.size() * sizeof(Key));
  memcpy(desc_out, desc.data(), desc.size());
  return 0;
}

}  // extern "C"
