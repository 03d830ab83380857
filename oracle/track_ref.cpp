// oracle/track_ref.cpp -- TEST INFRASTRUCTURE ONLY (checker; see orb_ref.cpp header).
//
// CPU restatement of the per-frame RGB-D multi-motion tracking path of the reference:
//   System::TrackRGBD                       src/System.cc:169-220
//   Tracking::GrabImageRGBD                 src/Tracking.cc:438-661   (depth, gray, hand-off B4)
//   Frame::Frame (RGB-D)                    src/Frame.cc:161-542      (ORB, B1 object sampling,
//                                                                      B2 static-key sampling)
//   Tracking::Track (initialised branch)    src/Tracking.cc:951-2499  (D2 ego solve, B6 scene
//                                           flow, B7 grouping, B8 labels, D5 + D3 per object,
//                                           B9 last-frame hand-off)
//   Tracking::StereoInitialization          src/Tracking.cc:2512-2570
// The ORB-SLAM2 map tracking that produces the ego initial pose (TrackWithMotionModel /
// TrackReferenceKeyFrame + TrackLocalMap, the keyframe policy and a synchronous LocalMapping) is
// oracle/map_ref.cpp; its pinned deviations (the BoW matcher of TrackReferenceKeyFrame and
// Relocalization, LocalMapping's BoW / BA steps) are listed in oracle_map.h.

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "oracle_solve.h"
#include "oracle_track.h"

namespace oracle {

// ------------------------------------------------------------ float cv::Mat helpers
// cv::Mat float products go through cv::gemm, which accumulates in double for CV_32F.
static void mat4_mul(const float* A, const float* B, float* C) {
  float R[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = 0;
      for (int k = 0; k < 4; k++) s += (double)A[4 * r + k] * (double)B[4 * k + c];
      R[4 * r + c] = (float)s;
    }
  memcpy(C, R, sizeof(R));
}

// Tracking::InvMatrix (Tracking.cc:5106-5121)
static void inv_mat(const float* T, float* Ti) {
  float R[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[4 * r + c] = T[4 * c + r];
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    R[4 * r + 3] = (float)(-s);
  }
  memcpy(Ti, R, sizeof(R));
}

static void mat4_eye(float* T) {
  for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.f : 0.f;
}

// Frame::UnprojectStereoObject(i, 0) (Frame.cc:1118-1152): world point of a pixel at depth z.
static void unproject_world(const TrackParams& P, const float* Tcw, float u, float v, float z,
                            float out[3]) {
  const float invfx = 1.0f / P.fx, invfy = 1.0f / P.fy;
  const float x = (u - P.cx) * z * invfx;
  const float y = (v - P.cy) * z * invfy;
  const float xc[3] = {x, y, z};
  float twl[3];
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)Tcw[4 * k + r] * (double)Tcw[4 * k + 3];
    twl[r] = (float)(-s);
  }
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)Tcw[4 * k + r] * (double)xc[k];
    out[r] = (float)s + twl[r];
  }
}

// ------------------------------------------------------------ Frame (RGB-D ctor)
void build_frame(const TrackParams& P, const OrbConfig& orb, const uint8_t* bgr,
                 const uint16_t* disp, const float* flow, const int32_t* mask, OFrame& F) {
  const int W = P.width, H = P.height;
  // depth from disparity*256 (Tracking.cc:447-456): bf / (float)(d / 256.0)
  F.depth.resize((size_t)W * H);
  for (size_t i = 0; i < (size_t)W * H; i++) {
    const float dp = (float)((float)disp[i] / 256.0);
    F.depth[i] = P.bf / dp;
  }
  std::vector<uint8_t> gray((size_t)W * H);
  gray_from_bgr(bgr, W, H, W * 3, gray.data());
  orb_extract(orb, gray.data(), W, H, F.keys, F.desc, nullptr, nullptr);
  const float* D = F.depth.data();
  // B1: semi-dense object samples, every 4th row/column (Frame.cc:188-217)
  for (int i = 0; i < H; i += 4)
    for (int j = 0; j < W; j += 4) {
      const size_t p = (size_t)i * W + j;
      if (mask[p] != 0 && D[p] < 25 && D[p] > 0) {
        const float fx = flow[2 * p], fy = flow[2 * p + 1];
        if (j + fx < W && j + fx > 0 && i + fy < H && i + fy > 0) {
          F.objFlow.push_back({fx, fy});
          F.objCorres.push_back({j + fx, i + fy});
          F.objKeys.push_back({(float)j, (float)i});
          F.objDepth.push_back(D[p]);
          F.semObjLabel.push_back(mask[p]);
        }
      }
    }
  // B2: static ORB keys associated through the flow (Frame.cc:228-324)
  for (const Key& k : F.keys) {
    const int x = (int)k.x, y = (int)k.y;
    const size_t p = (size_t)y * W + x;
    if (mask[p] != 0) continue;
    if (D[p] > 40 || D[p] <= 0) continue;
    const float fxe = flow[2 * p], fye = flow[2 * p + 1];
    if (fxe != 0 && fye != 0) {
      if (k.x + fxe < W && k.y + fye < H && k.x < W && k.y < H) {
        F.siftTmp.push_back({k.x, k.y});
        F.corres.push_back({k.x + fxe, k.y + fye});
        F.flowNext.push_back({fxe, fye});
      }
    }
  }
  F.siftDepthTmp.assign(F.siftTmp.size(), -1.f);
  for (size_t i = 0; i < F.siftTmp.size(); i++) {
    const float d = D[(size_t)(int)F.siftTmp[i].y * W + (int)F.siftTmp[i].x];
    if (d > 0) F.siftDepthTmp[i] = d;
  }
}

// ------------------------------------------------------------ Tracker
void OTracker::init(const TrackParams& p, const OrbConfig& orb) {
  P = p;
  orbc = orb;
  state = 0;
  bSecondFrame = false;
  bFirstFrame = false;  // uninitialised in the reference (Tracking.h:180): pinned false
  hasVelocity = false;
  reset_pending = false;
  g0 = cv_rng_first_gaussian(p.noise_seed);
  MapCam mc;
  mc.W = p.width;
  mc.H = p.height;
  mc.fx = p.fx; mc.fy = p.fy; mc.cx = p.cx; mc.cy = p.cy; mc.bf = p.bf;
  mc.invfx = 1.0f / p.fx;
  mc.invfy = 1.0f / p.fy;
  mc.thDepth = p.bf * p.th_depth / p.fx;  // mbf * (float)ThDepth / fx (Tracking.cc:225)
  mc.maxFrames = (int)(p.fps == 0 ? 30.f : p.fps);
  mc.nlevels = orb.nlevels;
  mc.scale = orb.scale;
  mc.invSigma2 = orb.invSigma2;
  mc.logScale = (float)std::log((double)orb.scale[orb.nlevels > 1 ? 1 : 0]);
  map.init(mc);
}

// GrabImageRGBD + Track for one frame.  Returns 0 and fills `out`.
int OTracker::track(const uint8_t* bgr, const uint16_t* disp, const float* flow,
                    const int32_t* mask, FrameResult& out) {
  const int W = P.width, H = P.height;
  const long frame_no = n_tracked++;
  if (reset_pending) {  // System::TrackRGBD -> Tracking::Reset (System.cc:203-211)
    map.reset();
    state = 0;
    reset_pending = false;
  }
  OFrame C;
  build_frame(P, orbc, bgr, disp, flow, mask, C);
  // ORACLE_ABLATE bit 8 (diagnostics only, tools/drift_ablation.py): a level-l keypoint at the
  // level-0 position of its pixel's centre, (x_l + 0.5) s - 0.5, instead of x_l s
  // (ORBextractor.cc:1100-1104 scales the corner, not the centre)
  static const bool centre = [] {
    const char* e = getenv("ORACLE_ABLATE");
    return e && (atoi(e) & 8);
  }();
  if (centre)
    for (Key& k : C.keys)
      if (k.octave > 0) {
        const float d = 0.5f * (orbc.scale[k.octave] - 1.f);
        k.x += d;
        k.y += d;
      }
  C.m.id = map.next_frame_id();
  map.prepare_frame(C.keys, C.depth.data(), C.m);
  std::vector<P2> mvTmpObjKeys;
  std::vector<float> mvTmpObjDepth;
  std::vector<int> mvTmpSemObjLabel;
  // ---- sample hand-off from the last frame (Tracking.cc:487-610)
  if (bFirstFrame || bSecondFrame) {
    C.siftKeys = L.corres;
    C.siftDepth.assign(C.siftKeys.size(), -1.f);
    for (size_t i = 0; i < C.siftKeys.size(); i++) {
      const float u = C.siftKeys[i].x, v = C.siftKeys[i].y;
      if (std::round(u) < W && std::round(u) > 0 && std::round(v) < H && std::round(v) > 0) {
        const float d = C.depth[(size_t)std::round(v) * W + (size_t)std::round(u)];
        if (d > 0) C.siftDepth[i] = d;
      }
    }
    mvTmpObjKeys = C.objKeys;
    mvTmpObjDepth = C.objDepth;
    mvTmpSemObjLabel = C.semObjLabel;
    C.objKeys = L.objCorres;
    C.objDepth.assign(C.objKeys.size(), -1.f);
    C.semObjLabel.assign(C.objKeys.size(), -1);
    for (size_t i = 0; i < C.objKeys.size(); i++) {
      const float u = C.objKeys[i].x, v = C.objKeys[i].y;
      if (std::round(u) < W && std::round(u) > 0 && std::round(v) < H && std::round(v) > 0) {
        const size_t p = (size_t)std::round(v) * W + (size_t)std::round(u);
        C.objDepth[i] = C.depth[p];
        C.semObjLabel[i] = mask[p];
      } else {
        C.objDepth[i] = 0.1f;
        C.semObjLabel[i] = 0;
      }
    }
  } else {
    C.siftKeys = C.siftTmp;
    C.siftDepth = C.siftDepthTmp;
  }
  C.objLabel.assign(C.objKeys.size(), -2);
  out = FrameResult();
  out.n_keys = (int)C.keys.size();
  out.n_static = (int)C.siftKeys.size();
  out.n_obj_samples = (int)C.objKeys.size();

  if (state == 0) {
    // ---- StereoInitialization (Tracking.cc:2512-2570)
    bFirstFrame = true;
    bSecondFrame = false;
    if ((int)C.keys.size() > 500) {
      mat4_eye(C.Tcw);
      C.hasPose = true;
      map.initialize(C.keys, C.desc, C.m, C.Tcw);
      map.frame_done(C.m, C.Tcw);
      L = C;  // Frame copy + the own-sample hand-off of :2545-2549
      L.siftKeys = C.siftTmp;
      L.siftDepth = C.siftDepthTmp;
      state = 1;
    }
    memcpy(out.Tcw, C.Tcw, sizeof(out.Tcw));
    out.initialized = state == 1;
    out.map.state = map.state();
    out.map.n_keyframes = map.n_keyframes();
    out.map.n_mappoints = map.n_mappoints();
    memcpy(out.map.Tcw_map, C.Tcw, sizeof(C.Tcw));
    return 0;
  }

  // ---- ORB-SLAM2 map tracking (Tracking.cc:985-1176): the initial pose of the flow solve.
  // It may reset mLastFrame's pose (UpdateLastFrame), which everything below then reads.
  float Tinit[16];
  {
    MapStats& ms = out.map;
    const int rr = map.track(C.keys, C.desc, C.m, Tinit, L.keys, L.desc, L.m, L.Tcw, V,
                             hasVelocity, bSecondFrame, ms);
    ms.state = map.state();
    ms.n_keyframes = map.n_keyframes();
    ms.n_mappoints = map.n_mappoints();
    memcpy(ms.Tcw_map, Tinit, sizeof(Tinit));
    memcpy(C.Tcw, Tinit, sizeof(Tinit));
    C.hasPose = true;
    if (rr == 1) {  // lost with <= 5 keyframes: mpSystem->Reset(); Track returns (Tracking.cc:1165-1172)
      reset_pending = true;
      memcpy(out.Tcw, C.Tcw, sizeof(out.Tcw));
      out.initialized = false;
      return 0;
    }
  }

  // ---- D2: PoseOptimizationFlow2Cam with identity temporal matches (Tracking.cc:1190-1307)
  {
    const int N = (int)C.siftKeys.size();
    std::vector<float> obs(2 * N), fl(2 * N), dep(N);
    for (int i = 0; i < N; i++) {
      obs[2 * i] = L.siftKeys[i].x;
      obs[2 * i + 1] = L.siftKeys[i].y;
      fl[2 * i] = L.flowNext[i].x;
      fl[2 * i + 1] = L.flowNext[i].y;
      dep[i] = noisy_depth(L.siftDepth[i], g0);  // ObtainFlowDepthCamera(i, addnoise=1)
    }
    FlowProblem fp;
    fp.n = N;
    fp.obs = obs.data();
    fp.flow = fl.data();
    fp.depth = dep.data();
    memcpy(fp.Tcw_last, L.Tcw, sizeof(fp.Tcw_last));
    memcpy(fp.init, Tinit, sizeof(fp.init));
    fp.rp_thres = 0.04f;
    fp.prior_info = 0.3;
    fp.max_iters = 100;
    fp.fx = P.fx; fp.fy = P.fy; fp.cx = P.cx; fp.cy = P.cy;
    float pose[16];
    FlowSolveStats st;
    if (flow_pose_solve(fp, pose, &st) == 0) memcpy(C.Tcw, pose, sizeof(pose));
    out.ego_iterations = st.iterations;
    out.ego_inliers = st.inliers;
  }
  // velocity (Tracking.cc:1311-1317)
  {
    float LastTwc[16];
    inv_mat(L.Tcw, LastTwc);
    mat4_mul(C.Tcw, LastTwc, V);
    hasVelocity = true;
  }

  // ---- B6: scene flow of object samples (GetSceneFlowObj, Tracking.cc:4007-4093)
  const int NO = (int)C.objKeys.size();
  C.flow3d.assign(NO, {0.f, 0.f, 0.f});
  for (int i = 0; i < NO; i++) {
    if (C.semObjLabel[i] <= 0 || L.semObjLabel[i] <= 0) {
      C.objLabel[i] = -1;
      continue;
    }
    float xp[3], xc[3];
    unproject_world(P, L.Tcw, L.objKeys[i].x, L.objKeys[i].y, L.objDepth[i], xp);
    unproject_world(P, C.Tcw, C.objKeys[i].x, C.objKeys[i].y, C.objDepth[i], xc);
    C.flow3d[i] = {xc[0] - xp[0], xc[1] - xp[1], xc[2] - xp[2]};
  }

  // ---- B7: semantic grouping + dynamic test (Tracking.cc:1396-1536)
  std::vector<int> UniLab = C.semObjLabel;
  std::sort(UniLab.begin(), UniLab.end());
  UniLab.erase(std::unique(UniLab.begin(), UniLab.end()), UniLab.end());
  std::vector<std::vector<int>> Posi(UniLab.size());
  for (int i = 0; i < NO; i++) {
    if (C.objLabel[i] == -1) continue;
    for (size_t j = 0; j < UniLab.size(); j++)
      if (C.semObjLabel[i] == UniLab[j]) {
        Posi[j].push_back(i);
        break;
      }
  }
  std::vector<std::vector<int>> ObjId;
  std::vector<int> sem_posi;
  for (size_t i = 0; i < Posi.size(); i++) {
    float count = 0, count_thres = 0.5;
    for (int idx : Posi[i]) {
      const float u = C.objKeys[idx].x, v = C.objKeys[idx].y;
      if (v < 25 || v > (H - 25) || u < 50 || u > (W - 50)) count = count + 1;
    }
    if (count / Posi[i].size() > count_thres) {
      for (int idx : Posi[i]) C.objLabel[idx] = -1;
      continue;
    }
    if (Posi[i].size() > 100) {
      ObjId.push_back(Posi[i]);
      sem_posi.push_back(UniLab[i]);
    } else {
      for (int idx : Posi[i]) C.objLabel[idx] = -1;
    }
  }
  const float sf_thres = 0.12f, sf_percent = 0.3f;
  std::vector<std::vector<int>> ObjIdNew;
  std::vector<int> SemPosNew;
  for (size_t i = 0; i < ObjId.size(); i++) {
    float center_depth = 0, sf_count = 0;
    for (int idx : ObjId[i]) {
      center_depth = center_depth + C.objDepth[idx];
      const float sf = std::sqrt(C.flow3d[idx][0] * C.flow3d[idx][0] + C.flow3d[idx][2] * C.flow3d[idx][2]);
      if (sf < sf_thres) sf_count = sf_count + 1;
    }
    if (sf_count / ObjId[i].size() > sf_percent) {
      for (int idx : ObjId[i]) C.objLabel[idx] = 0;
      continue;
    } else if (center_depth / ObjId[i].size() > 25.0) {
      for (int idx : ObjId[i]) C.objLabel[idx] = -1;
      continue;
    } else {
      ObjIdNew.push_back(ObjId[i]);
      SemPosNew.push_back(sem_posi[i]);
    }
  }

  // ---- B8: label association with the last frame (Tracking.cc:1556-1630)
  int mx;
  if (bSecondFrame)
    mx = 1;
  else if (!L.nModLabel.empty())
    mx = *std::max_element(L.nModLabel.begin(), L.nModLabel.end()) + 1;
  else
    mx = 1;  // uninitialised in the reference (Tracking.cc:1557): pinned 1
  std::vector<int> LabId(ObjIdNew.size());
  for (size_t i = 0; i < ObjIdNew.size(); i++) {
    std::map<int, int> dups;
    for (int idx : ObjIdNew[i]) ++dups[L.semObjLabel[idx]];
    // majority label; ties -> smallest label (std::sort of <= 16 pairs is an insertion sort)
    int New_lab = 0, best = -1;
    for (auto& kv : dups)
      if (kv.second > best) {
        best = kv.second;
        New_lab = kv.first;
      }
    if (bSecondFrame) {
      LabId[i] = mx;
      for (int idx : ObjIdNew[i]) C.objLabel[idx] = mx;
      mx = mx + 1;
    } else {
      bool exist = false;
      for (size_t k = 0; k < L.nSemPosition.size(); k++)
        if (L.nSemPosition[k] == New_lab) {
          LabId[i] = L.nModLabel[k];
          for (int idx : ObjIdNew[i]) C.objLabel[idx] = LabId[i];
          exist = true;
          break;
        }
      if (!exist) {
        LabId[i] = mx;
        for (int idx : ObjIdNew[i]) C.objLabel[idx] = mx;
        mx = mx + 1;
      }
    }
  }
  C.nModLabel = LabId;
  C.nSemPosition = SemPosNew;

  // ---- per object: D5 init (GetInitModelObj) + D3 (PoseOptimizationFlow2)
  C.vObjMod.assign(ObjIdNew.size(), std::vector<float>(16, 0.f));
  float TcwInv[16];
  inv_mat(C.Tcw, TcwInv);
  for (size_t oi = 0; oi < ObjIdNew.size(); oi++) {
    const std::vector<int>& ids = ObjIdNew[oi];
    const int N = (int)ids.size();
    std::vector<float> pre3(3 * N), cur2(2 * N);
    for (int i = 0; i < N; i++) {
      unproject_world(P, L.Tcw, L.objKeys[ids[i]].x, L.objKeys[ids[i]].y, L.objDepth[ids[i]], &pre3[3 * i]);
      cur2[2 * i] = C.objKeys[ids[i]].x;
      cur2[2 * i + 1] = C.objKeys[ids[i]].y;
    }
    PnPResult pr = pnp_ransac(pre3.data(), cur2.data(), N, P.fx, P.fy, P.cx, P.cy, 500, 0.3, 0.98);
    float Mod[16];
    mat4_eye(Mod);
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) Mod[4 * r + c] = (float)pr.R[3 * r + c];
      Mod[4 * r + 3] = (float)pr.t[r];
    }
    int PreObjID = -1;
    for (size_t k = 0; k < L.nModLabel.size(); k++)
      if (L.nModLabel[k] == C.nModLabel[oi]) {
        PreObjID = (int)k;
        break;
      }
    std::vector<int> sub;
    float Init[16];
    int mm_inliers = -1;
    if (PreObjID != -1) {
      float MM[16];
      mat4_mul(C.Tcw, L.vObjMod[PreObjID].data(), MM);
      std::vector<int> MM_inlier;
      for (int i = 0; i < N; i++) {
        float xc[3];
        for (int r = 0; r < 3; r++) {
          double s = 0;
          for (int k = 0; k < 3; k++) s += (double)MM[4 * r + k] * (double)pre3[3 * i + k];
          xc[r] = (float)s + MM[4 * r + 3];
        }
        const float invzc = (float)(1.0 / xc[2]);
        const float u = P.fx * xc[0] * invzc + P.cx, v = P.fy * xc[1] * invzc + P.cy;
        const float u_ = cur2[2 * i] - u, v_ = cur2[2 * i + 1] - v;
        const float Rpe = std::sqrt(u_ * u_ + v_ * v_);
        if (Rpe < 0.3) MM_inlier.push_back(i);
      }
      mm_inliers = (int)MM_inlier.size();
      if ((int)pr.inliers.size() > (int)MM_inlier.size()) {
        memcpy(Init, Mod, sizeof(Init));
        for (int k : pr.inliers) sub.push_back(ids[k]);
      } else {
        memcpy(Init, MM, sizeof(Init));
        for (int k : MM_inlier) sub.push_back(ids[k]);
      }
    } else {
      memcpy(Init, Mod, sizeof(Init));
      for (int k : pr.inliers) sub.push_back(ids[k]);
    }
    // D3
    const int NS = (int)sub.size();
    std::vector<float> obs(2 * NS), fl(2 * NS), dep(NS);
    for (int i = 0; i < NS; i++) {
      const int idx = sub[i];
      obs[2 * i] = L.objKeys[idx].x;
      obs[2 * i + 1] = L.objKeys[idx].y;
      fl[2 * i] = L.objFlow[idx].x;
      fl[2 * i + 1] = L.objFlow[idx].y;
      dep[i] = L.objDepth[idx];  // ObtainFlowDepthObject(i, addnoise=0)
    }
    FlowProblem fp;
    fp.n = NS;
    fp.obs = obs.data();
    fp.flow = fl.data();
    fp.depth = dep.data();
    memcpy(fp.Tcw_last, L.Tcw, sizeof(fp.Tcw_last));
    memcpy(fp.init, Init, sizeof(fp.init));
    fp.rp_thres = 0.01f;
    fp.prior_info = 0.5;
    fp.max_iters = 200;
    fp.fx = P.fx; fp.fy = P.fy; fp.cx = P.cx; fp.cy = P.cy;
    float X[16];
    FlowSolveStats st;
    if (d3_hook) d3_hook(fp, frame_no, (int)oi);
    const bool solved = flow_pose_solve(fp, X, &st) == 0;
    if (!solved) mat4_eye(X);
    // ObjCentre3D_pre (Tracking.cc:2032-2049): float sum, in order, of the last frame's
    // UnprojectStereoObject(j, 1) (Frame.cc:1118-1152: z + (float)gaussian(z^2 / 362.5 * 0.15),
    // the RNG's first draw g0), then cv::Mat / size: * (1.0 / n) in double, rounded to float.
    // Computed before the solve whatever its size: no points give 0 * (1 / 0) = NaN.
    float centre[3] = {0, 0, 0};
    {
      for (int i = 0; i < NS; i++) {
        float z = dep[i];
        const float noise = (float)((double)g0 * ((double)(z * z) / (725 * 0.5) * 0.15));
        z = z + noise;
        float xw[3];
        unproject_world(P, L.Tcw, obs[2 * i], obs[2 * i + 1], z, xw);
        for (int r = 0; r < 3; r++) centre[r] = centre[r] + xw[r];
      }
      for (int r = 0; r < 3; r++) centre[r] = (float)((double)centre[r] * (1.0 / NS));
    }
    mat4_mul(TcwInv, X, C.vObjMod[oi].data());
    ObjectResult r;
    r.label = C.nModLabel[oi];
    r.sem_label = C.nSemPosition[oi];
    r.n_points = N;
    r.n_ransac_inliers = (int)pr.inliers.size();
    r.n_mm_inliers = mm_inliers;
    r.n_solve = NS;
    r.n_inliers = st.inliers;
    r.iterations = st.iterations;
    memcpy(r.init, Init, sizeof(r.init));
    memcpy(r.X, X, sizeof(r.X));
    memcpy(r.motion, C.vObjMod[oi].data(), sizeof(r.motion));
    memcpy(r.centre_pre, centre, sizeof(r.centre_pre));
    r.ids = ids;
    r.sub = sub;
    out.objects.push_back(r);
  }
  memcpy(out.Tcw, C.Tcw, sizeof(out.Tcw));
  out.initialized = map.state() == 1;
  map.frame_done(C.m, C.Tcw);  // mlRelativeFramePoses (Tracking.cc:2481-2489)
  out.map.n_keyframes = map.n_keyframes();  // after the inserted keyframe's LocalMapping
  out.map.n_mappoints = map.n_mappoints();

  // ---- B9: last-frame hand-off (Tracking.cc:2463-2477)
  L = C;
  L.objKeys = mvTmpObjKeys;
  L.objDepth = mvTmpObjDepth;
  L.semObjLabel = mvTmpSemObjLabel;
  L.siftKeys = C.siftTmp;
  L.siftDepth = C.siftDepthTmp;
  return 0;
}

}  // namespace oracle
