// oracle/oracle_common.h -- TEST INFRASTRUCTURE ONLY (see orb_ref.cpp header).
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#define DBL_EPSILON_D DBL_EPSILON

namespace oracle {

// cvRound / cvFloor / cvCeil (OpenCV core: round-half-even via the FPU default mode).
static inline int cv_round(float v) { return (int)lrintf(v); }
static inline int cv_round_d(double v) { return (int)lrint(v); }
static inline int cv_floor(float v) {
  int i = (int)v;
  return i - (i > v);
}
static inline int cv_ceil(float v) {
  int i = (int)v;
  return i + (i < v);
}

struct Image {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
};

// cv::KeyPoint restated (28 bytes in the same field order).
struct Key {
  float x = 0, y = 0, size = 7.f, angle = -1.f, response = 0;
  int octave = 0, class_id = -1;
};

struct OrbConfig {
  int nfeatures = 0, nlevels = 0, iniTh = 0, minTh = 0;
  std::vector<float> scale, invScale, sigma2, invSigma2;
  std::vector<int> nPerLevel, umax;
};

void orb_config_init(OrbConfig& c, int nfeatures, float scaleFactor, int nlevels, int iniTh,
                     int minTh);
void orb_level_sizes(const OrbConfig& c, int w, int h, int* lw, int* lh);
void gray_from_bgr(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray);
void resize_linear_u8(const Image& src, Image& dst);
void compute_pyramid(const OrbConfig& c, const uint8_t* gray, int w, int h,
                     std::vector<Image>& pyr);
void fast_cell(const Image& img, int r0, int r1, int c0, int c1, int threshold,
               std::vector<Key>& out);
std::vector<Key> distribute_octree(const std::vector<Key>& keys, int minX, int maxX, int minY,
                                   int maxY, int N);
void level_keypoints(const OrbConfig& c, const Image& img, int level, std::vector<Key>& out,
                     std::vector<Key>* cand);
float fast_atan2_deg(float y, float x);
float ic_angle(const OrbConfig& c, const Image& img, float px, float py);
extern const int kGaussTaps7[7];
void gaussian_blur7(const Image& src, Image& dst);
void orb_descriptor(const Image& blurred, const Key& kp, uint8_t* desc);
void orb_extract(const OrbConfig& c, const uint8_t* gray, int w, int h, std::vector<Key>& kps,
                 std::vector<uint8_t>& desc, std::vector<Image>* pyr_out,
                 std::vector<std::vector<Key>>* cand_out);

}  // namespace oracle
