// oracle/orb_ref.cpp -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference ORB extractor (ORB-SLAM2 ORBextractor.cc as vendored in
// cule/multimot_track) together with the OpenCV primitives it calls, with every
// build-dependent OpenCV choice pinned as SURVEY.md Appendix A/C prescribes.  This code is the
// *checker* for the HIP path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load it.  It is never linked into libmmt.
//
// Parity status: the reference cannot be built here (no OpenCV/Eigen), and the
// reference ships no golden vectors for this path, so this restatement is "parity unpinned"
// against a real OpenCV build; its in-tree constants (pattern, umax, level quotas, level sizes,
// Gaussian taps) are pinned by known-answer tests in tests/test_oracle_orb.py.
//
// Citations are reference-relative (src/ORBextractor.cc unless noted).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <vector>

#include "oracle_common.h"

namespace oracle {

static const int kPatchSize = 31;      // ORBextractor.cc:72
static const int kHalfPatch = 15;      // ORBextractor.cc:73
static const int kEdgeThreshold = 19;  // ORBextractor.cc:74

static const int kBitPattern31[256 * 4] = {
#include "../multimot_track_amd/csrc/orb_pattern.inc"
};

// ---------------------------------------------------------------- ctor (ORBextractor.cc:410-470)
void orb_config_init(OrbConfig& c, int nfeatures, float scaleFactorF, int nlevels, int iniTh,
                     int minTh) {
  c.nfeatures = nfeatures;
  c.nlevels = nlevels;
  c.iniTh = iniTh;
  c.minTh = minTh;
  const double scaleFactor = (double)scaleFactorF;  // member is double (ORBextractor.h:101)
  c.scale.assign(nlevels, 1.0f);
  c.sigma2.assign(nlevels, 1.0f);
  for (int i = 1; i < nlevels; i++) {
    c.scale[i] = (float)((double)c.scale[i - 1] * scaleFactor);  // :421 float*double
    c.sigma2[i] = c.scale[i] * c.scale[i];                       // :422
  }
  c.invScale.resize(nlevels);
  c.invSigma2.resize(nlevels);
  for (int i = 0; i < nlevels; i++) {
    c.invScale[i] = 1.0f / c.scale[i];
    c.invSigma2[i] = 1.0f / c.sigma2[i];
  }
  c.nPerLevel.assign(nlevels, 0);
  const float factor = (float)(1.0f / scaleFactor);  // :436
  float nDesired = nfeatures * (1 - factor) /
                   (1 - (float)pow((double)factor, (double)nlevels));  // :437
  int sum = 0;
  for (int level = 0; level < nlevels - 1; level++) {
    c.nPerLevel[level] = cv_round(nDesired);  // :442
    sum += c.nPerLevel[level];
    nDesired *= factor;
  }
  c.nPerLevel[nlevels - 1] = std::max(nfeatures - sum, 0);  // :446

  // umax (:454-469)
  c.umax.assign(kHalfPatch + 1, 0);
  const int vmax = cv_floor(kHalfPatch * sqrtf(2.f) / 2 + 1);
  const int vmin = cv_ceil(kHalfPatch * sqrtf(2.f) / 2);
  const double hp2 = kHalfPatch * kHalfPatch;
  int v, v0;
  for (v = 0; v <= vmax; ++v) c.umax[v] = cv_round_d(sqrt(hp2 - v * v));
  for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
    while (c.umax[v0] == c.umax[v0 + 1]) ++v0;
    c.umax[v] = v0;
    ++v0;
  }
}

// Level sizes (ComputePyramid :1116): cvRound((float)cols*invScale)
void orb_level_sizes(const OrbConfig& c, int w, int h, int* lw, int* lh) {
  for (int l = 0; l < c.nlevels; l++) {
    lw[l] = cv_round((float)w * c.invScale[l]);
    lh[l] = cv_round((float)h * c.invScale[l]);
  }
}

// ------------------------------------------------- cvtColor RGB2GRAY on BGR bytes (Appendix A.1)
void gray_from_bgr(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray) {
  for (int y = 0; y < h; y++) {
    const uint8_t* row = bgr + (size_t)y * stride;
    for (int x = 0; x < w; x++) {
      const int c0 = row[3 * x], c1 = row[3 * x + 1], c2 = row[3 * x + 2];
      gray[(size_t)y * w + x] = (uint8_t)((c0 * 4899 + c1 * 9617 + c2 * 1868 + (1 << 13)) >> 14);
    }
  }
}

// -------------------------------------------- resize INTER_LINEAR, 8U, scalar path (Appendix A.4)
static inline short sat_short(float v) {
  int i = cv_round(v);
  return (short)std::min(std::max(i, -32768), 32767);
}

void resize_linear_u8(const Image& src, Image& dst) {
  const int sw = src.w, sh = src.h, dw = dst.w, dh = dst.h;
  const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
  const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
  std::vector<int> xofs(dw);
  std::vector<short> ialpha(2 * dw);
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
    }
    xofs[dx] = sx;
    ialpha[2 * dx] = sat_short((1.f - fx) * 2048);
    ialpha[2 * dx + 1] = sat_short(fx * 2048);
  }
  std::vector<int> r0(dw), r1(dw);
  auto hresize = [&](int sy, std::vector<int>& out) {
    const uint8_t* S = &src.px[(size_t)sy * sw];
    for (int dx = 0; dx < dw; dx++) {
      const int sx = xofs[dx];
      if (dx < xmax)
        out[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
      else
        out[dx] = S[sx] * 2048;
    }
  };
  for (int dy = 0; dy < dh; dy++) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floor(fy);
    fy -= sy;
    const short b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
    auto clip = [&](int v) { return v >= 0 ? (v < sh ? v : sh - 1) : 0; };
    hresize(clip(sy), r0);
    hresize(clip(sy + 1), r1);
    uint8_t* D = &dst.px[(size_t)dy * dw];
    for (int x = 0; x < dw; x++) {
      int v = (b0 * r0[x] + b1 * r1[x] + (1 << 21)) >> 22;
      D[x] = (uint8_t)std::min(std::max(v, 0), 255);
    }
  }
}

// ComputePyramid (:1111-1136).  The 19-px REFLECT_101 padding is never read on this path
// (FAST windows and keypoint patches stay inside the level), so levels are stored unpadded.
void compute_pyramid(const OrbConfig& c, const uint8_t* gray, int w, int h,
                     std::vector<Image>& pyr) {
  pyr.assign(c.nlevels, Image());
  std::vector<int> lw(c.nlevels), lh(c.nlevels);
  orb_level_sizes(c, w, h, lw.data(), lh.data());
  for (int l = 0; l < c.nlevels; l++) {
    pyr[l].w = lw[l];
    pyr[l].h = lh[l];
    pyr[l].px.assign((size_t)lw[l] * lh[l], 0);
    if (l == 0)
      memcpy(pyr[0].px.data(), gray, (size_t)w * h);
    else
      resize_linear_u8(pyr[l - 1], pyr[l]);
  }
}

// ------------------------------------------------------------ FAST-9/16 (Appendix A.5)
// Offsets (x, y) of the Bresenham circle of radius 3 in OpenCV's makeOffsets order.
static const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                   {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                   {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

static int corner_score16(const uint8_t* ptr, const int* pixel, int threshold) {
  const int K = 8, N = K * 3 + 1;
  int v = ptr[0];
  short d[N];
  for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = std::min((int)d[k + 1], (int)d[k + 2]);
    a = std::min(a, (int)d[k + 3]);
    if (a <= a0) continue;
    a = std::min(a, (int)d[k + 4]);
    a = std::min(a, (int)d[k + 5]);
    a = std::min(a, (int)d[k + 6]);
    a = std::min(a, (int)d[k + 7]);
    a = std::min(a, (int)d[k + 8]);
    a0 = std::max(a0, std::min(a, (int)d[k]));
    a0 = std::max(a0, std::min(a, (int)d[k + 9]));
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = std::max((int)d[k + 1], (int)d[k + 2]);
    b = std::max(b, (int)d[k + 3]);
    b = std::max(b, (int)d[k + 4]);
    b = std::max(b, (int)d[k + 5]);
    if (b >= b0) continue;
    b = std::max(b, (int)d[k + 6]);
    b = std::max(b, (int)d[k + 7]);
    b = std::max(b, (int)d[k + 8]);
    b0 = std::min(b0, std::max(b, (int)d[k]));
    b0 = std::min(b0, std::max(b, (int)d[k + 9]));
  }
  return -b0 - 1;
}

// cv::FAST(img(rowRange(r0,r1), colRange(c0,c1)), kps, threshold, nonmax=true): scalar FAST_t<16>.
// Emits keypoints in the submatrix frame, row-major.
void fast_cell(const Image& img, int r0, int r1, int c0, int c1, int threshold,
               std::vector<Key>& out) {
  out.clear();
  const int rows = r1 - r0, cols = c1 - c0;
  const int step = img.w;
  int pixel[25];
  for (int k = 0; k < 16; k++) pixel[k] = kCircle[k][0] + kCircle[k][1] * step;
  for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
  threshold = std::min(std::max(threshold, 0), 255);
  uint8_t tab[512];
  for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
  if (cols < 7 || rows < 7) return;
  std::vector<uint8_t> bufs(3 * cols, 0);
  std::vector<int> cps(3 * (cols + 1), 0);
  uint8_t* buf[3] = {&bufs[0], &bufs[cols], &bufs[2 * cols]};
  int* cpbuf[3] = {&cps[1], &cps[cols + 2], &cps[2 * cols + 3]};
  const int K = 8, N = 25;
  for (int i = 3; i < rows - 2; i++) {
    const uint8_t* ptr = &img.px[(size_t)(r0 + i) * step + c0] + 3;
    uint8_t* curr = buf[(i - 3) % 3];
    int* cornerpos = cpbuf[(i - 3) % 3];
    memset(curr, 0, cols);
    int ncorners = 0;
    if (i < rows - 3) {
      for (int j = 3; j < cols - 3; j++, ptr++) {
        int v = ptr[0];
        const uint8_t* t = &tab[0] - v + 255;
        int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
        if (d == 0) continue;
        d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
        d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
        d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
        if (d == 0) continue;
        d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
        d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
        d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
        d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
        if (d & 1) {
          int vt = v - threshold, count = 0;
          for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x < vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else
              count = 0;
          }
        }
        if (d & 2) {
          int vt = v + threshold, count = 0;
          for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x > vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else
              count = 0;
          }
        }
      }
    }
    cornerpos[-1] = ncorners;
    if (i == 3) continue;
    const uint8_t* prev = buf[(i - 4 + 3) % 3];
    const uint8_t* pprev = buf[(i - 5 + 3) % 3];
    cornerpos = cpbuf[(i - 4 + 3) % 3];
    ncorners = cornerpos[-1];
    for (int k = 0; k < ncorners; k++) {
      int j = cornerpos[k];
      int score = prev[j];
      if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
          score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] &&
          score > curr[j + 1]) {
        Key kp;
        kp.x = (float)j;
        kp.y = (float)(i - 1);
        kp.response = (float)score;
        out.push_back(kp);
      }
    }
  }
}

// ----------------------------------------------------- DistributeOctTree (:481-763)
struct ExtractorNode {
  std::vector<Key> vKeys;
  int ULx, ULy, URx, URy, BLx, BLy, BRx, BRy;
  std::list<ExtractorNode>::iterator lit;
  bool bNoMore = false;
  long seq = 0;  // creation order: pinned tie-break for the pointer sort (Appendix C)
};

static void divide_node(const ExtractorNode& p, ExtractorNode& n1, ExtractorNode& n2,
                        ExtractorNode& n3, ExtractorNode& n4) {
  const int halfX = (int)ceil(static_cast<float>(p.URx - p.ULx) / 2);  // :483
  const int halfY = (int)ceil(static_cast<float>(p.BRy - p.ULy) / 2);
  n1.ULx = p.ULx; n1.ULy = p.ULy;
  n1.URx = p.ULx + halfX; n1.URy = p.ULy;
  n1.BLx = p.ULx; n1.BLy = p.ULy + halfY;
  n1.BRx = p.ULx + halfX; n1.BRy = p.ULy + halfY;
  n2.ULx = n1.URx; n2.ULy = n1.URy;
  n2.URx = p.URx; n2.URy = p.URy;
  n2.BLx = n1.BRx; n2.BLy = n1.BRy;
  n2.BRx = p.URx; n2.BRy = p.ULy + halfY;
  n3.ULx = n1.BLx; n3.ULy = n1.BLy;
  n3.URx = n1.BRx; n3.URy = n1.BRy;
  n3.BLx = p.BLx; n3.BLy = p.BLy;
  n3.BRx = n1.BRx; n3.BRy = p.BLy;
  n4.ULx = n3.URx; n4.ULy = n3.URy;
  n4.URx = n2.BRx; n4.URy = n2.BRy;
  n4.BLx = n3.BRx; n4.BLy = n3.BRy;
  n4.BRx = p.BRx; n4.BRy = p.BRy;
  for (const Key& kp : p.vKeys) {
    if (kp.x < n1.URx) {
      if (kp.y < n1.BRy) n1.vKeys.push_back(kp);
      else n3.vKeys.push_back(kp);
    } else if (kp.y < n1.BRy)
      n2.vKeys.push_back(kp);
    else
      n4.vKeys.push_back(kp);
  }
  if (n1.vKeys.size() == 1) n1.bNoMore = true;
  if (n2.vKeys.size() == 1) n2.bNoMore = true;
  if (n3.vKeys.size() == 1) n3.bNoMore = true;
  if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

typedef std::pair<std::pair<int, long>, ExtractorNode*> SizeSeqNode;

std::vector<Key> distribute_octree(const std::vector<Key>& keys, int minX, int maxX, int minY,
                                   int maxY, int N) {
  const int nIni = (int)round(static_cast<float>(maxX - minX) / (maxY - minY));  // :543
  const float hX = static_cast<float>(maxX - minX) / nIni;
  long seq = 0;
  std::list<ExtractorNode> lNodes;
  std::vector<ExtractorNode*> vpIniNodes(nIni);
  for (int i = 0; i < nIni; i++) {
    ExtractorNode ni;
    ni.ULx = (int)(hX * static_cast<float>(i)); ni.ULy = 0;
    ni.URx = (int)(hX * static_cast<float>(i + 1)); ni.URy = 0;
    ni.BLx = ni.ULx; ni.BLy = maxY - minY;
    ni.BRx = ni.URx; ni.BRy = maxY - minY;
    ni.seq = seq++;
    lNodes.push_back(ni);
    vpIniNodes[i] = &lNodes.back();
  }
  for (const Key& kp : keys) vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);  // :569

  auto lit = lNodes.begin();
  while (lit != lNodes.end()) {
    if (lit->vKeys.size() == 1) {
      lit->bNoMore = true;
      lit++;
    } else if (lit->vKeys.empty())
      lit = lNodes.erase(lit);
    else
      lit++;
  }

  bool bFinish = false;
  std::vector<SizeSeqNode> vSize;
  vSize.reserve(lNodes.size() * 4);
  auto push_child = [&](ExtractorNode& n, std::vector<SizeSeqNode>* track, int* nToExpand) {
    if (n.vKeys.size() > 0) {
      n.seq = seq++;
      lNodes.push_front(n);
      if (n.vKeys.size() > 1) {
        if (nToExpand) (*nToExpand)++;
        track->push_back(std::make_pair(std::make_pair((int)n.vKeys.size(), n.seq), &lNodes.front()));
        lNodes.front().lit = lNodes.begin();
      }
    }
  };

  while (!bFinish) {
    int prevSize = (int)lNodes.size();
    lit = lNodes.begin();
    int nToExpand = 0;
    vSize.clear();
    while (lit != lNodes.end()) {
      if (lit->bNoMore) {
        lit++;
        continue;
      }
      ExtractorNode n1, n2, n3, n4;
      divide_node(*lit, n1, n2, n3, n4);
      push_child(n1, &vSize, &nToExpand);
      push_child(n2, &vSize, &nToExpand);
      push_child(n3, &vSize, &nToExpand);
      push_child(n4, &vSize, &nToExpand);
      lit = lNodes.erase(lit);
    }
    if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
      bFinish = true;
    } else if (((int)lNodes.size() + nToExpand * 3) > N) {
      while (!bFinish) {
        prevSize = (int)lNodes.size();
        std::vector<SizeSeqNode> vPrev = vSize;
        vSize.clear();
        std::sort(vPrev.begin(), vPrev.end(),
                  [](const SizeSeqNode& a, const SizeSeqNode& b) { return a.first < b.first; });
        for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
          ExtractorNode n1, n2, n3, n4;
          divide_node(*vPrev[j].second, n1, n2, n3, n4);
          push_child(n1, &vSize, nullptr);
          push_child(n2, &vSize, nullptr);
          push_child(n3, &vSize, nullptr);
          push_child(n4, &vSize, nullptr);
          lNodes.erase(vPrev[j].second->lit);
          if ((int)lNodes.size() >= N) break;
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
      }
    }
  }

  std::vector<Key> result;
  result.reserve(lNodes.size());
  for (auto& node : lNodes) {
    const Key* best = &node.vKeys[0];
    float maxResponse = best->response;
    for (size_t k = 1; k < node.vKeys.size(); k++) {
      if (node.vKeys[k].response > maxResponse) {
        best = &node.vKeys[k];
        maxResponse = node.vKeys[k].response;
      }
    }
    result.push_back(*best);
  }
  return result;
}

// ------------------------------------------------ ComputeKeyPointsOctTree (:765-853), per level
// Returns the FAST candidates (relative to minBorder) before distribution when `cand` != null.
void level_keypoints(const OrbConfig& c, const Image& img, int level, std::vector<Key>& out,
                     std::vector<Key>* cand) {
  const float W = 30;
  const int minBorderX = kEdgeThreshold - 3, minBorderY = minBorderX;
  const int maxBorderX = img.w - kEdgeThreshold + 3, maxBorderY = img.h - kEdgeThreshold + 3;
  std::vector<Key> toDistribute;
  const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
  const int nCols = (int)(width / W), nRows = (int)(height / W);
  const int wCell = (int)ceil(width / nCols), hCell = (int)ceil(height / nRows);
  std::vector<Key> cell;
  for (int i = 0; i < nRows; i++) {
    const float iniY = (float)(minBorderY + i * hCell);
    float maxY = iniY + hCell + 6;
    if (iniY >= maxBorderY - 3) continue;
    if (maxY > maxBorderY) maxY = (float)maxBorderY;
    for (int j = 0; j < nCols; j++) {
      const float iniX = (float)(minBorderX + j * wCell);
      float maxX = iniX + wCell + 6;
      if (iniX >= maxBorderX - 6) continue;
      if (maxX > maxBorderX) maxX = (float)maxBorderX;
      fast_cell(img, (int)iniY, (int)maxY, (int)iniX, (int)maxX, c.iniTh, cell);
      if (cell.empty()) fast_cell(img, (int)iniY, (int)maxY, (int)iniX, (int)maxX, c.minTh, cell);
      for (Key k : cell) {
        k.x += j * wCell;
        k.y += i * hCell;
        toDistribute.push_back(k);
      }
    }
  }
  if (cand) *cand = toDistribute;
  out = distribute_octree(toDistribute, minBorderX, maxBorderX, minBorderY, maxBorderY,
                          c.nPerLevel[level]);
  const int scaledPatchSize = (int)(kPatchSize * c.scale[level]);  // :837
  for (Key& k : out) {
    k.x += minBorderX;
    k.y += minBorderY;
    k.octave = level;
    k.size = (float)scaledPatchSize;
  }
}

// ------------------------------------------------------ fastAtan2 (Appendix A.7)
float fast_atan2_deg(float y, float x) {
  static const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
  static const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
  static const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
  static const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
  const float ax = std::abs(x), ay = std::abs(y);
  float a, cc, c2;
  if (ax >= ay) {
    cc = ay / (ax + (float)DBL_EPSILON_D);
    c2 = cc * cc;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * cc;
  } else {
    cc = ax / (ay + (float)DBL_EPSILON_D);
    c2 = cc * cc;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * cc;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// IC_Angle (:77-104) on the unblurred level.
float ic_angle(const OrbConfig& c, const Image& img, float px, float py) {
  int m01 = 0, m10 = 0;
  const int cy = cv_round(py), cx = cv_round(px);
  const int step = img.w;
  const uint8_t* center = &img.px[(size_t)cy * step + cx];
  for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * center[u];
  for (int v = 1; v <= kHalfPatch; ++v) {
    int v_sum = 0;
    const int d = c.umax[v];
    for (int u = -d; u <= d; ++u) {
      const int vp = center[u + v * step], vm = center[u - v * step];
      v_sum += (vp - vm);
      m10 += u * (vp + vm);
    }
    m01 += v * v_sum;
  }
  return fast_atan2_deg((float)m01, (float)m10);
}

// ------------------------------------- GaussianBlur 7x7 sigma 2, 8U bit-exact (Appendix A.6)
// Q8 taps with error diffusion (sum 256); horizontal Q8, vertical Q16 with (v + 2^15) >> 16.
const int kGaussTaps7[7] = {18, 34, 48, 56, 48, 34, 18};

static inline int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

void gaussian_blur7(const Image& src, Image& dst) {
  const int w = src.w, h = src.h;
  dst.w = w;
  dst.h = h;
  dst.px.assign((size_t)w * h, 0);
  std::vector<uint32_t> hbuf((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      uint32_t s = 0;
      for (int k = 0; k < 7; k++) s += kGaussTaps7[k] * src.px[(size_t)y * w + reflect101(x + k - 3, w)];
      hbuf[(size_t)y * w + x] = s;
    }
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      uint32_t s = 0;
      for (int k = 0; k < 7; k++) s += kGaussTaps7[k] * hbuf[(size_t)reflect101(y + k - 3, h) * w + x];
      dst.px[(size_t)y * w + x] = (uint8_t)std::min<uint32_t>((s + (1u << 15)) >> 16, 255u);
    }
}

// ------------------------------------------------ computeOrbDescriptor (:108-147)
// cos/sin pinned to (float)cos((double)angle) (Appendix C: shared correctly-rounded routine).
void orb_descriptor(const Image& blurred, const Key& kp, uint8_t* desc) {
  const float factorPI = (float)(M_PI / 180.f);
  const float angle = kp.angle * factorPI;
  const float a = (float)cos((double)angle), b = (float)sin((double)angle);
  const int step = blurred.w;
  const uint8_t* center = &blurred.px[(size_t)cv_round(kp.y) * step + cv_round(kp.x)];
  const int* pattern = kBitPattern31;
  auto get = [&](int idx) {
    const float px = (float)pattern[2 * idx], py = (float)pattern[2 * idx + 1];
    const float ry = px * b + py * a;
    const float rx = px * a - py * b;
    return (int)center[cv_round(ry) * step + cv_round(rx)];
  };
  for (int i = 0; i < 32; ++i, pattern += 32) {
    int val = 0;
    for (int bit = 0; bit < 8; bit++) {
      const int t0 = get(2 * bit), t1 = get(2 * bit + 1);
      val |= (t0 < t1) << bit;
    }
    desc[i] = (uint8_t)val;
  }
}

// ------------------------------------------------ ORBextractor::operator() (:1046-1109)
void orb_extract(const OrbConfig& c, const uint8_t* gray, int w, int h, std::vector<Key>& kps,
                 std::vector<uint8_t>& desc, std::vector<Image>* pyr_out,
                 std::vector<std::vector<Key>>* cand_out) {
  std::vector<Image> pyr;
  compute_pyramid(c, gray, w, h, pyr);
  std::vector<std::vector<Key>> all(c.nlevels);
  if (cand_out) cand_out->assign(c.nlevels, std::vector<Key>());
  for (int l = 0; l < c.nlevels; l++)
    level_keypoints(c, pyr[l], l, all[l], cand_out ? &(*cand_out)[l] : nullptr);
  for (int l = 0; l < c.nlevels; l++)
    for (Key& k : all[l]) k.angle = ic_angle(c, pyr[l], k.x, k.y);
  kps.clear();
  desc.clear();
  for (int l = 0; l < c.nlevels; l++) {
    if (all[l].empty()) continue;
    Image blurred;
    gaussian_blur7(pyr[l], blurred);
    for (const Key& k : all[l]) {
      uint8_t d[32];
      orb_descriptor(blurred, k, d);
      desc.insert(desc.end(), d, d + 32);
    }
    if (l != 0) {
      const float scale = c.scale[l];
      for (Key& k : all[l]) {
        k.x *= scale;
        k.y *= scale;
      }
    }
    kps.insert(kps.end(), all[l].begin(), all[l].end());
  }
  if (pyr_out) *pyr_out = pyr;
}

}  // namespace oracle
