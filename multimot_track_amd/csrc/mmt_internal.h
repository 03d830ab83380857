// multimot_track_amd/csrc/mmt_internal.h -- shared host-side declarations of libmmt.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mmt.h"

namespace mmt {

#define MMT_HIP(call)                                                              \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess) throw mmt::DeviceError(std::string(#call) + ": " +        \
                                                 hipGetErrorString(e_));           \
  } while (0)

struct DeviceError {
  std::string msg;
  explicit DeviceError(std::string m) : msg(std::move(m)) {}
};
struct ArgError {
  std::string msg;
  explicit ArgError(std::string m) : msg(std::move(m)) {}
};

// ORB tables, computed on the host exactly like ORBextractor's ctor (ORBextractor.cc:410-470).
struct OrbTables {
  int nfeatures = 0, nlevels = 0, iniTh = 0, minTh = 0;
  std::vector<float> scale, invScale, sigma2, invSigma2;
  std::vector<int> nPerLevel, umax;
  void init(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh);
};

// Device-side geometry records (POD, uploaded once per context).
struct LevelInfo {
  int w, h;            // level size
  int off;             // byte offset of the level inside one frame's pyramid
  int nIni;            // DistributeOctTree initial node count (ORBextractor.cc:543)
  float hX;            // initial node width (ORBextractor.cc:545)
  int N;               // mnFeaturesPerLevel
  int cell_begin, cell_end;  // cell index range (row-major cells of this level)
  int key_off, key_cap;      // candidate-key slot range (per frame)
  int out_off, out_cap;      // octree output slot range (per frame)
  float scale;               // mvScaleFactor[level]
  float size;                // (float)(int)(31 * scale)  (ORBextractor.cc:837)
};

struct CellInfo {
  int level;
  int r0, c0;          // tile origin in level coordinates (= iniY, iniX)
  int rows, cols;      // tile size ((maxY-iniY) x (maxX-iniX))
  int slot_off, slot_cap;
  int pad;
};

struct ResizeX {  // horizontal INTER_LINEAR coefficients of one destination column
  int sx;
  short a0, a1;
};
struct ResizeY {
  int sy0, sy1;
  short b0, b1;
};

struct BlurTile {
  int level, x0, y0, pad;
};
// k_pyramid: the rows [lo, hi) of every level one band computes (its own rows and the halo rows
// the next level's rows read), and the per-level constants of the launch
constexpr int kPyrMaxLevels = 12;
struct PyrBand {
  int lo[kPyrMaxLevels], hi[kPyrMaxLevels];
};
struct PyrArgs {
  int nl, buf_bytes;
  int pitch[kPyrMaxLevels], xoff[kPyrMaxLevels], yoff[kPyrMaxLevels];
};

// Batched ORB extraction engine for one image size.
class OrbEngine {
 public:
  OrbEngine() = default;
  ~OrbEngine();
  void setup(int w, int h, const OrbTables& t, int max_batch);
  // d_gray: nframes x frame_pitch bytes, row pitch = width.  Outputs device pointers.
  void run(const uint8_t* d_gray, int nframes, size_t frame_pitch, mmt_kp* d_kps,
           uint8_t* d_desc, int cap_per_frame, int* d_n, hipStream_t stream);
  int capacity() const { return cap_frame_; }
  int width() const { return w_; }
  int height() const { return h_; }
  const std::vector<LevelInfo>& levels() const { return lv_; }
  // Device pyramid of the last run (frame-major, pyr_stride_ bytes per frame).
  const uint8_t* pyramid() const { return d_pyr_; }
  // Level 0 of frame f is written here by a producer that skips the staging copy: run() with
  // d_gray == level0() and frame_pitch == pyramid_stride() reads the pyramid in place.
  uint8_t* level0() { return d_pyr_; }
  size_t pyramid_stride() const { return pyr_stride_; }
  long debug_fetch(int what, int frame, void* out, size_t cap, hipStream_t stream);
  // Device-side error flags of the launches so far (k_octree: 1 pass guard, 2 node capacity,
  // 4 output truncated).  Reads them on `stream` (synchronising it); throws DeviceError and
  // clears them when any is set.
  void check_flags(hipStream_t stream);
  // the error word as read by the caller (after a sync): 0 returns, otherwise the word is cleared
  // on the device and the same DeviceError as check_flags is thrown
  void check_flags_value(int flags, hipStream_t stream);
  const int* err_word() const { return d_err_; }
  void raise_flags(int flags, hipStream_t stream);

 private:
  void release();
  int w_ = 0, h_ = 0, nlevels_ = 0, max_batch_ = 0, ncells_ = 0, ntiles_ = 0;
  int fast_rows_max_ = 0, fast_cols_max_ = 0, fast_win_max_ = 0;  // largest FAST tile / window
  int total_slots_ = 0, out_slots_ = 0, cap_frame_ = 0, node_cap_ = 0;
  int key_cap_ = 0;          // k_octree: keys per (level, frame) held in LDS
  size_t octree_lds_ = 0;    // k_octree dynamic LDS bytes
  int key_cap1_ = 0;         // the same for the launch of levels 1.. (two workgroups per CU)
  size_t octree_lds1_ = 0;
  bool oct_two_per_cu_ = false;
  // One side stream beside the caller's (run()): a process has 4 hardware queues
  // (GPU_MAX_HW_QUEUES), and streams beyond them end up sharing the caller's queue.
  hipStream_t side_ = nullptr;
  hipEvent_t ev_pyr_ = nullptr, ev_blur_ = nullptr, ev_gray_ = nullptr;
  void run_part(int f0, int nf, hipStream_t st_main, hipStream_t st_side, hipEvent_t* ev,
                mmt_kp* d_kps, uint8_t* d_desc, int cap_per_frame, int* d_n);
  int iniTh_ = 20, minTh_ = 7;
  size_t pyr_stride_ = 0;
  std::vector<LevelInfo> lv_;
  std::vector<CellInfo> cells_;
  std::vector<int> xtab_off_, ytab_off_;
  std::vector<int> rs_pitch_, rs_lds_;  // k_resize LDS row pitch and bytes per level
  // k_pyramid: bands per frame (0: the k_resize chain, e.g. when a band's rows do not fit the
  // LDS), the band table and the launch constants
  int pyr_bands_ = 0, pyr_lds_ = 0;
  // batches up to this many frames take k_pyramid; window against the chain
  // (round 5): batch 1 0.124 / 0.140 ms, 4 0.136 / 0.154, 16 0.202 / 0.218, 32 0.297 / 0.300,
  // 64 0.544 / 0.503, 128 1.029 / 0.919
  static constexpr int pyr_max_frames_ = 32;
  // XCD-contiguous workgroup order (bits: 1 k_resize, 2 k_blur).  Blur only: its FETCH 131 -> 105 MB per 128-frame window at the same time; the resize chain
  // fetches 101 -> 89 MB but runs 10 us slower (window 0.932 against 0.922 ms, round 5)
  static constexpr int xcd_order_ = 2;
  PyrBand* d_pyr_bands_ = nullptr;
  PyrArgs pyr_args_{};
  int sched_ = 0;  // MMT_ORB_SCHED=2: one stream (standalone kernel times for profiling)
  // FAST cells per wave: with more, each wave's next tile loads are in flight during its current
  // cell; measured 0.918 / 0.928 / 0.940 / 0.951 ms per 128-frame window at 1 / 2 / 4 / 8 (round 5)
  static constexpr int fast_cpw_ = 1;
  LevelInfo* d_lv_ = nullptr;
  CellInfo* d_cells_ = nullptr;
  ResizeX* d_xtab_ = nullptr;
  ResizeY* d_ytab_ = nullptr;
  BlurTile* d_tiles_ = nullptr;
  int* d_umax_ = nullptr;
  uint8_t* d_pyr_ = nullptr;
  uint8_t* d_blur_ = nullptr;
  uint32_t* d_keys_ = nullptr;   // candidate keys, per frame total_slots_
  uint32_t* d_lkeys_ = nullptr;  // per-level gathered keys
  uint32_t* d_knode_ = nullptr;  // key -> node
  int* d_cellcnt_ = nullptr;
  uint32_t* d_okeys_ = nullptr;  // octree output, per frame out_slots_
  int* d_ocount_ = nullptr;      // per frame nlevels
  int* d_err_ = nullptr;
};

}  // namespace mmt

