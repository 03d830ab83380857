// multimot_track_amd/cli/mmt_viz.h -- the reference's visual artifacts for rgbd_mmt --viz
// (Tracking.cc:684-878): feat.png (static samples and object samples over the
// image), speed.png (ground-truth boxes of the tracked objects) and traj.png (camera positions
// and object centroids seen from above).  A BGR canvas with the few primitives those use
// (cv::drawKeypoints' 3-pixel circle, cv::circle / cv::rectangle with a thickness, a filled
// rectangle).  Text (cv::putText) is not drawn: there is no font renderer here, and the values
// it would show (speeds, camera position) are printed by the evaluation lines.
#pragma once
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

namespace viz {

struct BGR {
  uint8_t b, g, r;
};

struct Canvas {
  int w = 0, h = 0;
  std::vector<uint8_t> px;  // BGR, row-major
  Canvas() = default;
  Canvas(int w_, int h_) : w(w_), h(h_), px((size_t)w_ * h_ * 3, 0) {}
  void set(int x, int y, BGR c) {
    if (x < 0 || y < 0 || x >= w || y >= h) return;
    uint8_t* p = &px[3 * ((size_t)y * w + x)];
    p[0] = c.b;
    p[1] = c.g;
    p[2] = c.r;
  }
  // cv::circle(center, radius, color, thickness): the ring |d - radius| <= thickness / 2
  void circle(int cx, int cy, int radius, BGR c, int thickness = 1) {
    const float half = thickness * 0.5f;
    const int R = radius + thickness;
    for (int y = cy - R; y <= cy + R; y++)
      for (int x = cx - R; x <= cx + R; x++) {
        const float d = std::sqrt((float)((x - cx) * (x - cx) + (y - cy) * (y - cy)));
        if (std::fabs(d - radius) <= half) set(x, y, c);
      }
  }
  // cv::rectangle(p1, p2, color, thickness); thickness < 0 fills (CV_FILLED)
  void rectangle(int x1, int y1, int x2, int y2, BGR c, int thickness) {
    if (x1 > x2) std::swap(x1, x2);
    if (y1 > y2) std::swap(y1, y2);
    if (thickness < 0) {
      for (int y = y1; y <= y2; y++)
        for (int x = x1; x <= x2; x++) set(x, y, c);
      return;
    }
    const int a = thickness / 2, b = (thickness - 1) / 2;
    for (int y = y1 - a; y <= y2 + a; y++)
      for (int x = x1 - a; x <= x2 + a; x++) {
        const bool edge = (x <= x1 + b) || (x >= x2 - b) || (y <= y1 + b) || (y >= y2 - b);
        if (edge) set(x, y, c);
      }
  }
};

// the label colours of Tracking.cc:704-778 (feat.png, cv::Scalar = BGR)
inline BGR feat_colour(int l, bool* known) {
  *known = true;
  switch (l) {
    case 0: return {0, 0, 255};
    case 1: return {255, 165, 0};
    case 2: return {0, 255, 0};
    case 3: return {255, 255, 0};
    case 4: return {255, 192, 203};
    case 5: return {0, 255, 255};
    case 6: return {128, 0, 128};
    case 7: return {255, 255, 255};
    case 8: return {255, 228, 196};
    case 9: return {180, 105, 255};
    case 10: return {165, 42, 42};
    case 11: return {35, 142, 107};
    case 12: return {45, 82, 160};
    case 41: return {60, 20, 220};
  }
  *known = false;
  return {0, 0, 0};
}

// the label colours of Tracking.cc:832-873 (traj.png, CV_RGB(r, g, b))
inline BGR traj_colour(int l, bool* known) {
  *known = true;
  switch (l) {
    case 1: return {255, 165, 0};
    case 2: return {0, 255, 0};
    case 3: return {255, 255, 0};
    case 4: return {255, 192, 203};
    case 5: return {0, 255, 255};
    case 6: return {128, 0, 128};
    case 7: return {255, 255, 255};
    case 8: return {255, 228, 196};
    case 9: return {255, 105, 180};
    case 10: return {165, 42, 42};
    case 11: return {107, 142, 35};
    case 12: return {160, 82, 45};
    case 41: return {220, 20, 60};
  }
  *known = false;
  return {0, 0, 0};
}

}  // namespace viz
