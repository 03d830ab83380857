// multimot_track_amd/csrc/mmt_localmap.hip -- the rest of LocalMapping::Run's iteration after
// ProcessNewKeyFrame / MapPointCulling (reference src/LocalMapping.cc:68-87), run synchronously on
// every new keyframe:
//   SearchInNeighbors      LocalMapping.cc:458-538: the fusion targets (10 best covisibles and 5 of
//                          each of theirs), ORBmatcher::Fuse(target, current points) per target,
//                          Fuse(current, the targets' points), the points' descriptors / normals,
//                          UpdateConnections.  Fuse's per-point search (projection, scale, window,
//                          best Hamming key) runs on the GPU (k_fuse_cand) for all pairs of a sequence
//                          of Fuse calls at once; the host replays the calls in order with the
//                          reference's map edits (AddObservation, MapPoint::Replace, MapPoint.cc:
//                          177-215).  A point whose descriptor the replay has changed (a Replace
//                          survivor, ComputeDistinctiveDescriptors) is searched again, on the GPU,
//                          before its next use.
//   LocalBundleAdjustment  Optimizer.cc:3341-3666: the graph exactly as the reference builds it;
//                          the solve is one GPU workgroup (mmt_ba.hip); erase and recovery here.
//   KeyFrameCulling        LocalMapping.cc:636-700 with KeyFrame::SetBadFlag (KeyFrame.cc:453-545).
// CreateNewMapPoints (LocalMapping.cc:210-456) needs SearchForTriangulation, i.e. the BoW
// vocabulary, which the reference does not ship; it is skipped.
// Containers keyed by KeyFrame* iterate in keyframe creation order, as in the CPU checker
// (oracle/mapping_ref.cpp).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstring>
#include <map>
#include <set>

#include "mmt_map.h"
#include "mmt_mat4.h"

namespace mmt {

namespace {
size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
void cam_centre(const float* T, float* Ow) {  // -Rcw^T tcw
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    Ow[r] = -(float)s;
  }
}
}  // namespace

void MapEngine::grow_dev(uint8_t*& d, uint8_t*& h, size_t& cap, size_t need) {
  if (need <= cap && d) return;
  const size_t c = std::max(need + (need >> 1), (size_t)1 << 16);
  if (d) {
    MMT_HIP(hipStreamSynchronize(lm_s_));
    dallocs_.erase(std::find(dallocs_.begin(), dallocs_.end(), (void*)d));
    (void)hipFree(d);
    hallocs_.erase(std::find(hallocs_.begin(), hallocs_.end(), (void*)h));
    (void)hipHostFree(h);
  }
  d = dev<uint8_t>(c);
  h = pinned<uint8_t>(c);
  cap = c;
}

// ------------------------------------------------------------------ keyframe store
// KeyFrame(F): mvKeysUn, mDescriptors, mvuRight and mGrid copied from the frame (KeyFrame.cc:31-57),
// here from the frame's device buffers
void MapEngine::kf_store_add(int kf) {
  const int b = kf / kKFBlock, r = kf % kKFBlock;
  while ((int)kf_blocks_.size() <= b) kf_blocks_.push_back(dev<uint8_t>(kf_rec_bytes_ * kKFBlock));
  uint8_t* base = kf_blocks_[b] + kf_rec_bytes_ * r;
  const size_t o_desc = al16(sizeof(mmt_kp) * (size_t)kcap_);
  const size_t o_uR = o_desc + 32 * (size_t)kcap_;
  const size_t o_cs = o_uR + al16(4 * (size_t)kcap_);
  const size_t o_ci = o_cs + al16(4 * (size_t)(kGridCells + 1));
  KFrame& K = kfs_[kf];
  const int n = G_.n;
  MMT_HIP(hipMemcpyAsync(base, G_.keys, sizeof(mmt_kp) * (size_t)n, hipMemcpyDeviceToDevice, lm_s_));
  MMT_HIP(hipMemcpyAsync(base + o_desc, G_.desc, 32 * (size_t)n, hipMemcpyDeviceToDevice, lm_s_));
  MMT_HIP(hipMemcpyAsync(base + o_uR, G_.uR, 4 * (size_t)n, hipMemcpyDeviceToDevice, lm_s_));
  MMT_HIP(hipMemcpyAsync(base + o_cs, G_.cell_start, 4 * (size_t)(kGridCells + 1),
                         hipMemcpyDeviceToDevice, lm_s_));
  MMT_HIP(hipMemcpyAsync(base + o_ci, G_.cell_idx, 4 * (size_t)n, hipMemcpyDeviceToDevice, lm_s_));
  FuseKF& f = K.dev;
  f.keys = (const mmt_kp*)base;
  f.desc = base + o_desc;
  f.uR = (const float*)(base + o_uR);
  f.cell_start = (const int*)(base + o_cs);
  f.cell_idx = (const int*)(base + o_ci);
  f.n = n;
}

// ------------------------------------------------------------------ KeyFrame / MapPoint edits
void MapEngine::set_pose(int kf, const float* T) {  // KeyFrame::SetPose
  KFrame& K = kfs_[kf];
  memcpy(K.Tcw, T, 64);
  cam_centre(T, K.Ow);
  mat4_eye(K.Twc);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) K.Twc[4 * r + c] = T[4 * c + r];
    K.Twc[4 * r + 3] = K.Ow[r];
  }
}

void MapEngine::erase_observation(int h, int kf) {  // MapPoint::EraseObservation
  MPoint& p = mp(h);
  auto it = std::lower_bound(p.obs.begin(), p.obs.end(), std::make_pair(kf, INT_MIN));
  if (it == p.obs.end() || it->first != kf) return;
  if (kfs_[kf].uR[it->second] >= 0)
    p.nObs -= 2;
  else
    p.nObs--;
  p.obs.erase(it);
  // an emptied map's begin() is undefined in the reference; the point goes bad right below then
  if (p.refKF == kf) p.refKF = p.obs.empty() ? -1 : p.obs.front().first;
  if (p.nObs <= 2) set_bad(h);
}

void MapEngine::replace(int h, int by) {  // MapPoint::Replace (this = h, pMP = by)
  if (h == by) return;
  MPoint& p = mp(h);
  const std::vector<std::pair<int, int>> obs = p.obs;
  p.obs.clear();
  mark_bad(h);
  const int nvisible = p.visible, nfound = p.found;
  p.replaced = by;
  mark_dirty(h);
  for (const auto& kv : obs) {
    if (mp(by).obs_index(kv.first) < 0) {
      kfs_[kv.first].mps[kv.second] = by;  // ReplaceMapPointMatch
      add_observation(by, kv.first, kv.second);
    } else {
      kfs_[kv.first].mps[kv.second] = -1;  // EraseMapPointMatch(idx)
    }
  }
  MPoint& q = mp(by);
  q.found += nfound;
  q.visible += nvisible;
  compute_distinctive(by);
}

void MapEngine::erase_connection(int kf, int other) {  // KeyFrame::EraseConnection
  if (kfs_[kf].conn.erase(other)) update_best_covisibles(kf);
}

void MapEngine::kf_set_bad(int kf) {  // KeyFrame::SetBadFlag (mbNotErase is never set here)
  KFrame& K = kfs_[kf];
  if (K.id == 0) return;
  for (const auto& kv : std::map<int, int>(K.conn)) erase_connection(kv.first, kf);
  for (size_t i = 0; i < K.mps.size(); i++)
    if (K.mps[i] >= 0) erase_observation(K.mps[i], kf);
  K.conn.clear();
  K.ordered.clear();
  // the spanning tree: each round re-parents the child with the strongest link to a candidate
  std::set<int> cand;
  cand.insert(K.parent);
  while (!K.children.empty()) {
    bool bContinue = false;
    int mx = -1, pC = -1, pP = -1;
    for (int ch : K.children) {
      if (kfs_[ch].bad) continue;
      for (int c : kfs_[ch].ordered)
        for (int q : cand)
          if (c == q) {
            auto it = kfs_[ch].conn.find(c);  // GetWeight
            const int wgt = it == kfs_[ch].conn.end() ? 0 : it->second;
            if (wgt > mx) {
              pC = ch;
              pP = c;
              mx = wgt;
              bContinue = true;
            }
          }
    }
    if (!bContinue) break;
    kfs_[pC].parent = pP;  // ChangeParent
    kfs_[pP].children.insert(pC);
    mstats_.n_reparent++;
    cand.insert(pC);
    K.children.erase(pC);
  }
  if (K.parent >= 0) {
    for (int ch : K.children) {
      kfs_[ch].parent = K.parent;
      kfs_[K.parent].children.insert(ch);
      mstats_.n_reparent++;
    }
    kfs_[K.parent].children.erase(kf);
  }
  K.bad = true;
  kfdb_erase(kf);  // mpKeyFrameDB->erase(this) (KeyFrame.cc:544)
}

// ------------------------------------------------------------------ Fuse
// One launch: a table of the keyframes involved and the (keyframe, point) queries; the results
// land in res (host, pinned-backed copy).
void MapEngine::fuse_launch(const std::vector<int>& kft_kf, const std::vector<FuseQuery>& q,
                            int2* res) {
  const int nq = (int)q.size();
  if (nq == 0) return;
  const double t0 = prof_on_ ? now_us() : 0;
  double tq = t0;
  gpu_flush_pool(lm_s_);
  blk_time(10, tq);
  const size_t tb = al16(sizeof(FuseKF) * kft_kf.size());
  grow_dev(d_fup_, h_fup_, fup_cap_, tb + sizeof(FuseQuery) * (size_t)nq);
  {
    uint8_t* dres = (uint8_t*)d_fres_;
    uint8_t* hres = (uint8_t*)h_fres_;
    grow_dev(dres, hres, fres_cap_, sizeof(int2) * (size_t)nq);
    d_fres_ = (int2*)dres;
    h_fres_ = (int2*)hres;
  }
  FuseKF* tab = (FuseKF*)h_fup_;
  for (size_t t = 0; t < kft_kf.size(); t++) {
    const KFrame& K = kfs_[kft_kf[t]];
    tab[t] = K.dev;
    memcpy(tab[t].Tcw, K.Tcw, 64);
    memcpy(tab[t].Ow, K.Ow, 12);
  }
  memcpy(h_fup_ + tb, q.data(), sizeof(FuseQuery) * (size_t)nq);
  MMT_HIP(hipMemcpyAsync(d_fup_, h_fup_, tb + sizeof(FuseQuery) * (size_t)nq,
                         hipMemcpyHostToDevice, lm_s_));
  FuseCam c;
  memset(&c, 0, sizeof(c));
  c.fx = cam_.fx; c.fy = cam_.fy; c.cx = cam_.cx; c.cy = cam_.cy; c.bf = cam_.bf;
  c.W = (float)cam_.W;
  c.H = (float)cam_.H;
  c.invW = (float)kGridCols / (float)cam_.W;
  c.invH = (float)kGridRows / (float)cam_.H;
  c.logScale = cam_.logScale;
  c.th = 3.f;
  c.nlevels = cam_.nlevels;
  for (int l = 0; l < cam_.nlevels && l < kMaxLevels; l++) {
    c.scale[l] = cam_.scale[l];
    c.invSigma2[l] = cam_.invSigma2[l];
  }
  launch_fuse_cand((const FuseKF*)d_fup_, (const FuseQuery*)(d_fup_ + tb), nq, d_pool_,
                   d_pool_desc_, c, d_fres_, lm_s_);
  MMT_HIP(hipMemcpyAsync(h_fres_, d_fres_, sizeof(int2) * (size_t)nq, hipMemcpyDeviceToHost,
                         lm_s_));
  blk_time(11, tq);
  MMT_HIP(hipStreamSynchronize(lm_s_));
  blk_time(12, tq);
  memcpy(res, h_fres_, sizeof(int2) * (size_t)nq);
  mstats_.fuse_launches++;
  mstats_.fuse_queries += nq;
  if (prof_on_) mstats_.fuse_us += now_us() - t0;
}

// ORBmatcher::Fuse's decision for one point (ORBmatcher.cc:1326-1346)
void MapEngine::fuse_apply(int kf, int h, int bestIdx, int bestDist) {
  if (bestDist > 50) return;  // TH_LOW
  KFrame& K = kfs_[kf];
  const int pin = K.mps[bestIdx];
  if (pin >= 0) {
    if (!mp(pin).bad) {
      if (mp(pin).nObs > mp(h).nObs)
        replace(h, pin);
      else
        replace(pin, h);
    }
  } else {
    add_observation(h, kf, bestIdx);
    K.mps[bestIdx] = h;
  }
  mstats_.n_fused++;
}

// Fuse(kfl[0], pts), Fuse(kfl[1], pts), ... in order.  A (keyframe, point) pair the reference skips
// at the time of the launch (bad point, or already in the keyframe) stays skipped: a point never
// becomes good again, and within these calls an observation is never removed from a good point.
// Positions, normals and distance bounds do not change inside the calls; descriptors do (Replace
// survivors), which the per-point version number catches.
void MapEngine::fuse_sequence(const std::vector<int>& kfl, const std::vector<int>& pts) {
  const int nk = (int)kfl.size(), np = (int)pts.size();
  if (nk == 0 || np == 0) return;
  std::vector<int> qidx((size_t)nk * np, -1);
  std::vector<FuseQuery> q;
  std::vector<int> ver;
  for (int t = 0; t < nk; t++)
    for (int i = 0; i < np; i++) {
      if (t == 0 && i + 8 < np) prefetch_point(pts[i + 8]);
      const int h = pts[i];
      if (h < 0 || mp(h).bad || mp(h).obs_index(kfl[t]) >= 0) continue;
      qidx[(size_t)t * np + i] = (int)q.size();
      q.push_back(FuseQuery{t, h});
      ver.push_back(mp(h).desc_ver);
    }
  std::vector<int2> res(q.size());
  double tb = prof_on_ ? prof_now_us() : 0;
  fuse_launch(kfl, q, res.data());
  tb = prof_on_ ? prof_now_us() : 0;
  for (int t = 0; t < nk; t++) {
    const int kf = kfl[t];
    for (int i = 0; i < np; i++) {
      const int h = pts[i];
      if (h < 0) continue;
      const MPoint& p = mp(h);
      if (p.bad || p.obs_index(kf) >= 0) continue;
      const int qi = qidx[(size_t)t * np + i];
      if (qi < 0) continue;  // cannot happen (see above); defensive
      if (ver[qi] != p.desc_ver) {
        // stale: search again every remaining pair whose point has a newer descriptor
        std::vector<FuseQuery> rq;
        std::vector<int> rpos;
        for (int t2 = t; t2 < nk; t2++)
          for (int i2 = (t2 == t ? i : 0); i2 < np; i2++) {
            const int q2 = qidx[(size_t)t2 * np + i2];
            if (q2 < 0) continue;
            const int h2 = pts[i2];
            if (mp(h2).bad || ver[q2] == mp(h2).desc_ver) continue;
            rq.push_back(FuseQuery{t2, h2});
            rpos.push_back(q2);
          }
        std::vector<int2> rr(rq.size());
        fuse_launch(kfl, rq, rr.data());
        for (size_t k = 0; k < rq.size(); k++) {
          res[rpos[k]] = rr[k];
          ver[rpos[k]] = mp(rq[k].h).desc_ver;
        }
        mstats_.fuse_relaunches++;
      }
      fuse_apply(kf, h, res[qi].x, res[qi].y);
    }
  }
  blk_time(13, tb);
}

// ------------------------------------------------------------------ LocalMapping steps
void MapEngine::search_in_neighbors(int kf) {  // LocalMapping::SearchInNeighbors (RGB-D: nn 10)
  double tb = prof_on_ ? prof_now_us() : 0;
  const long cur = kfs_[kf].id;
  auto best = [&](int k, size_t n) {
    const std::vector<int>& o = kfs_[k].ordered;
    return std::vector<int>(o.begin(), o.begin() + std::min(o.size(), n));
  };
  std::vector<int> targets;
  for (int k : best(kf, 10)) {
    KFrame& Ki = kfs_[k];
    if (Ki.bad || Ki.fuseTarget == cur) continue;
    targets.push_back(k);
    Ki.fuseTarget = cur;
    for (int k2 : best(k, 5)) {
      const KFrame& K2 = kfs_[k2];
      if (K2.bad || K2.fuseTarget == cur || K2.id == cur) continue;
      targets.push_back(k2);
    }
  }
  const std::vector<int> matches = kfs_[kf].mps;
  blk_time(2, tb);
  fuse_sequence(targets, matches);
  blk_time(3, tb);
  std::vector<int> cands;
  for (int t : targets) {
    const std::vector<int> mps = kfs_[t].mps;
    for (int h : mps) {
      if (h < 0) continue;
      MPoint& p = mp(h);
      if (p.bad || p.fuseCand == cur) continue;
      p.fuseCand = cur;
      cands.push_back(h);
    }
  }
  blk_time(4, tb);
  fuse_sequence(std::vector<int>{kf}, cands);
  blk_time(5, tb);
  const std::vector<int> now = kfs_[kf].mps;
  for (size_t j = 0; j < now.size(); j++) {
    if (j + 8 < now.size()) prefetch_point(now[j + 8]);
    const int h = now[j];
    if (h < 0 || mp(h).bad) continue;
    compute_distinctive(h);
    update_normal_depth(h);
  }
  blk_time(6, tb);
  update_connections(kf);
  blk_time(7, tb);
}

void MapEngine::local_bundle_adjustment(int kf) {  // Optimizer::LocalBundleAdjustment
  const double t0 = prof_on_ ? now_us() : 0;
  const long cur = kfs_[kf].id;
  std::vector<int> local{kf};
  kfs_[kf].baLocal = cur;
  for (int k : kfs_[kf].ordered) {  // GetVectorCovisibleKeyFrames
    kfs_[k].baLocal = cur;
    if (!kfs_[k].bad) local.push_back(k);
  }
  std::vector<int> lpts;
  for (int k : local)
    for (int h : std::vector<int>(kfs_[k].mps)) {
      if (h < 0) continue;
      MPoint& p = mp(h);
      if (p.bad || p.baLocal == cur) continue;
      lpts.push_back(h);
      p.baLocal = cur;
    }
  std::vector<int> fixedKFs;
  for (int h : lpts)
    for (const auto& kv : mp(h).obs) {
      KFrame& Ki = kfs_[kv.first];
      if (Ki.baLocal != cur && Ki.baFixed != cur) {
        Ki.baFixed = cur;
        if (!Ki.bad) fixedKFs.push_back(kv.first);
      }
    }
  std::vector<int> verts = local;
  verts.insert(verts.end(), fixedKFs.begin(), fixedKFs.end());
  const int nK = (int)verts.size(), nP = (int)lpts.size();
  std::vector<int>& vIdx = ba_vidx_;  // keyframe -> vertex, -1 elsewhere (reset below)
  if (vIdx.size() < kfs_.size()) vIdx.resize(kfs_.size(), -1);
  std::vector<float> Tv(16 * (size_t)nK), Xv(3 * (size_t)nP);
  std::vector<uint8_t> fixed(nK);
  int nO = 0;
  for (int v = 0; v < nK; v++) {
    vIdx[verts[v]] = v;
    memcpy(&Tv[16 * (size_t)v], kfs_[verts[v]].Tcw, 64);
    fixed[v] = v >= (int)local.size() || kfs_[verts[v]].id == 0;
    nO += !fixed[v];
  }
  // edges point by point, each point's observations in keyframe order (Optimizer.cc:3460-3541)
  std::vector<int> e_pt, e_kf, e_kfid;
  std::vector<float> e_obs, e_s;
  for (int j = 0; j < nP; j++) {
    const MPoint& p = mp(lpts[j]);
    memcpy(&Xv[3 * (size_t)j], p.pos, 12);
    for (const auto& kv : p.obs) {
      const KFrame& Ki = kfs_[kv.first];
      if (Ki.bad) continue;
      const mmt_kp& kp = Ki.keys[kv.second];
      e_pt.push_back(j);
      e_kf.push_back(vIdx[kv.first]);
      e_kfid.push_back(kv.first);
      e_obs.push_back(kp.x);
      e_obs.push_back(kp.y);
      e_obs.push_back(Ki.uR[kv.second] < 0 ? -1.f : Ki.uR[kv.second]);
      e_s.push_back(cam_.invSigma2[kp.octave]);
    }
  }
  const int nE = (int)e_pt.size();
  for (int v = 0; v < nK; v++) vIdx[verts[v]] = -1;  // every edge's keyframe is a vertex
  BAHostProblem P;
  P.n_kf = nK;
  P.n_pt = nP;
  P.n_edge = nE;
  P.Tcw = Tv.data();
  P.fixed = fixed.data();
  P.Xw = Xv.data();
  P.e_pt = e_pt.data();
  P.e_kf = e_kf.data();
  P.e_obs = e_obs.data();
  P.e_s = e_s.data();
  P.fx = cam_.fx; P.fy = cam_.fy; P.cx = cam_.cx; P.cy = cam_.cy; P.bf = cam_.bf;
  std::vector<float> Tout(16 * (size_t)nK), Xout(3 * (size_t)nP);
  std::vector<uint8_t> er(std::max(nE, 1));
  int st[5];
  double tb = prof_on_ ? now_us() : 0;
  if (prof_on_) mstats_.blk_us[8] += tb - t0;
  ba_.run(P, lm_s_, Tout.data(), Xout.data(), er.data(), st);
  if (prof_on_) mstats_.basolve_us += now_us() - tb;
  tb = prof_on_ ? now_us() : 0;
  mstats_.n_ba++;
  mstats_.ba_trials += st[2] + st[3];
  mstats_.ba_edges += nE;
  mstats_.ba_kfs += nK;
  mstats_.ba_pts += nP;
  mstats_.ba_max_opt = std::max<long>(mstats_.ba_max_opt, nO);
  // vToErase: monocular edges, then stereo edges, each in creation order
  for (int pass = 0; pass < 2; pass++)
    for (int i = 0; i < nE; i++) {
      const bool stereo = !(e_obs[3 * (size_t)i + 2] < 0);
      if (stereo != (pass == 1) || !er[i]) continue;
      const int h = lpts[e_pt[i]], k = e_kfid[i];
      const int idx = mp(h).obs_index(k);  // KeyFrame::EraseMapPointMatch(pMP)
      if (idx >= 0) kfs_[k].mps[idx] = -1;
      erase_observation(h, k);
      mstats_.n_ba_erased++;
    }
  for (size_t v = 0; v < local.size(); v++) set_pose(local[v], &Tout[16 * v]);
  for (int j = 0; j < nP; j++) {
    MPoint& p = mp(lpts[j]);
    memcpy(p.pos, &Xout[3 * (size_t)j], 12);  // SetWorldPos
    mark_dirty(lpts[j]);
    update_normal_depth(lpts[j]);
  }
  blk_time(9, tb);
  if (prof_on_) mstats_.ba_us += now_us() - t0;
}

void MapEngine::keyframe_culling(int kf) {  // LocalMapping::KeyFrameCulling (RGB-D)
  const std::vector<int> local = kfs_[kf].ordered;
  for (int k : local) {
    KFrame& K = kfs_[k];
    if (K.id == 0) continue;
    const int thObs = 3;
    int nRedundant = 0, nMPs = 0;
    for (size_t i = 0; i < K.mps.size(); i++) {
      const int h = K.mps[i];
      if (h < 0) continue;
      const MPoint& p = mp(h);
      if (p.bad) continue;
      if (K.depth[i] > cam_.thDepth || K.depth[i] < 0) continue;
      nMPs++;
      if (p.nObs > thObs) {
        const int scaleLevel = K.keys[i].octave;
        int nObs = 0;
        for (const auto& kv : p.obs) {
          if (kv.first == k) continue;
          if (kfs_[kv.first].keys[kv.second].octave <= scaleLevel + 1) {
            nObs++;
            if (nObs >= thObs) break;
          }
        }
        if (nObs >= thObs) nRedundant++;
      }
    }
    if (nRedundant > cull_ratio_ * nMPs) {  // 0.9 (LocalMapping.cc:697) unless a test sets it
      kf_set_bad(k);
      mstats_.n_culled++;
    }
  }
}

void MapEngine::local_mapping(int kf) {
  const double t0 = prof_on_ ? now_us() : 0;
  // CreateNewMapPoints: SearchForTriangulation needs the vocabulary's FeatureVectors (without one
  // it is skipped, see mmt_map.h); mmt_bowmap.hip
  if (voc_) create_new_map_points(kf);
  if (prof_on_) mstats_.cnmp_us += now_us() - t0;
  search_in_neighbors(kf);
  const double t1 = prof_on_ ? now_us() : 0;
  if (n_keyframes() > 2) local_bundle_adjustment(kf);
  const double t2 = prof_on_ ? now_us() : 0;
  keyframe_culling(kf);
  const double t3 = prof_on_ ? now_us() : 0;
  // the keyframe-store copies read the chunk's frame buffers: done before the next chunk's ORB
  MMT_HIP(hipStreamSynchronize(lm_s_));
  if (prof_on_) {
    const double t4 = now_us();
    mstats_.lm_us += t4 - t0;
    mstats_.sin_us += t1 - t0;
    mstats_.cull_us += t3 - t2;
    mstats_.lmsync_us += t4 - t3;
    mstats_.n_lm++;
  }
}

}  // namespace mmt
