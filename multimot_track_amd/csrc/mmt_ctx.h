// multimot_track_amd/csrc/mmt_ctx.h -- the opaque mmt_ctx behind include/mmt.h.
#pragma once
#include <deque>
#include <memory>

#include "mmt_ba.h"
#include "mmt_bow.h"
#include "mmt_internal.h"
#include "mmt_tracker.h"

struct mmt_ctx {
  mmt_config cfg;
  mmt::OrbTables orb;
  mmt::OrbEngine engine;
  hipStream_t stream = nullptr;
  std::string err;
  // staging for the host-pointer entry points
  uint8_t* d_in = nullptr;
  size_t d_in_bytes = 0;
  mmt_kp* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  int* d_n = nullptr;
  int staged_frames = 0;
  // tracking (one sequence per context)
  mmt::Tracker tracker;
  bool tracker_ready = false;
  mmt::BARunner ba;  // mmt_local_bundle_adjustment's buffers (kept across calls)
  uint8_t* t_bgr = nullptr;
  uint16_t* t_disp = nullptr;
  float* t_flow = nullptr;
  int32_t* t_mask = nullptr;
  int t_frames = 0;  // frames the t_* staging buffers hold
  std::deque<mmt::FrameOut> flushed;  // mmt_flush_objects records not yet handed out
  std::unique_ptr<mmt::Vocabulary> voc;  // mmt_load_vocabulary (System's ORB vocabulary)
};
