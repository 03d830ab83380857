// oracle/oracle_capi.cpp -- TEST INFRASTRUCTURE ONLY.
// Flat C entry points so tests/ and bench.py (cpu_baseline leg) can drive the CPU restatement
// through ctypes.  Never linked into the product library.

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>

#include "oracle_common.h"
#include "oracle_match.h"

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

// ------------------------------------------------------------------ tracker / solve probes
#include "oracle_map.h"
#include "oracle_solve.h"
#include "oracle_track.h"

extern "C" {

float oracle_rng_first_gaussian(unsigned long long seed) { return cv_rng_first_gaussian(seed); }

// Flow-refined pose solve probe (D2 when noise already applied to depth / D3).
int oracle_flow_solve(int n, const float* obs, const float* flow, const float* depth,
                      const float* tcw_last, const float* init, float rp_thres, double prior_info,
                      int max_iters, float fx, float fy, float cx, float cy, float* pose_out,
                      int* stats3) {
  FlowProblem p;
  p.n = n;
  p.obs = obs;
  p.flow = flow;
  p.depth = depth;
  memcpy(p.Tcw_last, tcw_last, sizeof(p.Tcw_last));
  memcpy(p.init, init, sizeof(p.init));
  p.rp_thres = rp_thres;
  p.prior_info = prior_info;
  p.max_iters = max_iters;
  p.fx = fx; p.fy = fy; p.cx = cx; p.cy = cy;
  FlowSolveStats st;
  const int rc = flow_pose_solve(p, pose_out, &st);
  stats3[0] = st.iterations;
  stats3[1] = st.inliers;
  stats3[2] = st.status;
  stats3[3] = st.rejections;
  stats3[4] = st.clean_rejections;
  stats3[5] = st.max_reject_run;
  return rc;
}

// Optimizer::PoseOptimization probe (D1).
int oracle_pose_optimization(int n, const float* Xw, const float* obs, const float* inv_sigma2,
                             const float* tcw, float fx, float fy, float cx, float cy, float bf,
                             float* pose_out, unsigned char* outlier) {
  PoseOptProblem p;
  p.n = n;
  p.Xw = Xw;
  p.obs = obs;
  p.inv_sigma2 = inv_sigma2;
  memcpy(p.Tcw, tcw, sizeof(p.Tcw));
  p.fx = fx; p.fy = fy; p.cx = cx; p.cy = cy; p.bf = bf;
  return pose_optimization(p, pose_out, outlier);
}

int oracle_pnp_ransac(const float* pts3, const float* pts2, int n, double fx, double fy,
                      double cx, double cy, int max_iters, double reproj, double conf,
                      double* R9, double* t3, int* inliers, int* n_inliers, int* iters) {
  PnPResult r = pnp_ransac(pts3, pts2, n, fx, fy, cx, cy, max_iters, reproj, conf);
  memcpy(R9, r.R, sizeof(r.R));
  memcpy(t3, r.t, sizeof(r.t));
  *n_inliers = (int)r.inliers.size();
  for (size_t i = 0; i < r.inliers.size(); i++) inliers[i] = r.inliers[i];
  iters[0] = r.iterations;
  iters[1] = r.best_iter;
  return r.ok ? 0 : 1;
}

// D6 probe: one iterate() call; state in/out (iterations, best_inliers, best_Tcw, best_mask)
int oracle_pnpsolver_iterate(const float* pts3, const float* pts2, const float* sigma2, int n,
                             double fx, double fy, double cx, double cy, double prob, int min_inl,
                             int max_it, int min_set, float eps, float th2, const int* randi,
                             int n_iterations, int* st_its, float* st_T, uint8_t* st_mask,
                             float* T_out, uint8_t* mask_out, int* out3) {
  P4PState st;
  st.iterations = st_its[0];
  st.best_inliers = st_its[1];
  memcpy(st.best_Tcw, st_T, sizeof(st.best_Tcw));
  st.best_mask.assign(st_mask, st_mask + n);
  P4PResult r = pnpsolver_iterate(pts3, pts2, sigma2, n, fx, fy, cx, cy, prob, min_inl, max_it,
                                  min_set, eps, th2, randi, n_iterations, &st);
  st_its[0] = st.iterations;
  st_its[1] = st.best_inliers;
  memcpy(st_T, st.best_Tcw, sizeof(st.best_Tcw));
  if (!st.best_mask.empty()) memcpy(st_mask, st.best_mask.data(), n);
  memcpy(T_out, r.Tcw, sizeof(r.Tcw));
  memset(mask_out, 0, n);
  if (!r.mask.empty()) memcpy(mask_out, r.mask.data(), n);
  out3[0] = r.found;
  out3[1] = r.no_more;
  out3[2] = r.n_inliers;
  return 0;
}

// DUtils::Random::RandomInt draws of a P4P RANSAC (4 per iteration: RandomInt(0, n-1-j)) from
// glibc's rand() stream seeded with `seed` (1 = an unseeded process)
int oracle_p4p_randi(int n, int iters, unsigned seed, int* out) {
  GlibcRand g(seed);
  for (int k = 0; k < iters; k++)
    for (int j = 0; j < 4; j++) out[4 * k + j] = g.random_int(0, n - 1 - j);
  return 0;
}

int oracle_glibc_rand(unsigned seed, int count, int* out) {
  GlibcRand g(seed);
  for (int i = 0; i < count; i++) out[i] = g.next();
  return 0;
}

int oracle_ransac_subsets(int count, int iters, int* out) {
  std::vector<int> idx;
  ransac_subsets(count, 5, iters, idx);
  memcpy(out, idx.data(), idx.size() * sizeof(int));
  return 0;
}

void* oracle_tracker_create(int w, int h, float fx, float fy, float cx, float cy, float bf,
                            unsigned long long seed, int nfeatures) {
  OTracker* t = new OTracker();
  TrackParams p;
  p.width = w;
  p.height = h;
  p.fx = fx; p.fy = fy; p.cx = cx; p.cy = cy; p.bf = bf;
  p.noise_seed = seed;
  OrbConfig c;
  orb_config_init(c, nfeatures, 1.2f, 8, 20, 7);
  t->init(p, c);
  return t;
}

void oracle_tracker_destroy(void* t) { delete (OTracker*)t; }

// System(voc, ...): the tracker runs the reference's BoW steps with this vocabulary (0 / -1)
int oracle_tracker_set_vocabulary(void* tp, const char* path) {
  OTracker* t = (OTracker*)tp;
  std::unique_ptr<Vocabulary> v(new Vocabulary());
  std::string err;
  if (v->load_text(path, &err) != 0) return -1;
  t->voc = std::move(v);
  t->map.set_vocabulary(t->voc.get());
  return 0;
}

// the BoW path's counters: [BoW frames, TrackReferenceKeyFrame calls, ok, Relocalization calls,
// ok, candidates, PnP poses, SearchByProjection(F, KF) rounds, triangulated points,
// SearchForTriangulation matches, database insertions]
void oracle_tracker_bow_stats(void* tp, long long* out) {
  const MapTracker::BowStats& b = ((OTracker*)tp)->map.bstats;
  const long v[11] = {b.n_bow_frames, b.n_trk, b.n_trk_ok, b.n_reloc, b.n_reloc_ok,
                      b.n_reloc_cands, b.n_pnp_found, b.n_sbp_rounds, b.n_triangulated,
                      b.n_sft_matches, b.n_kfdb};
  for (int i = 0; i < 11; i++) out[i] = v[i];
}

// ---- DBoW2 vocabulary probes (tests)
void* oracle_voc_load(const char* path) {
  Vocabulary* v = new Vocabulary();
  std::string err;
  if (v->load_text(path, &err) != 0) {
    delete v;
    return nullptr;
  }
  return v;
}
void oracle_voc_free(void* v) { delete (Vocabulary*)v; }
// sizes: [k, L, scoring, weighting, nodes, words]
void oracle_voc_info(void* vp, int* out) {
  const Vocabulary* v = (const Vocabulary*)vp;
  out[0] = v->k; out[1] = v->L; out[2] = v->scoring; out[3] = v->weighting;
  out[4] = (int)v->parent.size(); out[5] = (int)v->words.size();
}
// transform(features, BowVector, FeatureVector, levelsup): per feature its word, weight and node
// (feat_*: n each); the BowVector (words ascending, values) into bow_word / bow_value (cap n) and
// the FeatureVector flattened (fv_node, fv_start n + 1, fv_feat n); counts[0..1] = entries, nodes
int oracle_voc_transform(void* vp, const uint8_t* desc, int n, int levelsup, uint32_t* feat_word,
                         double* feat_weight, uint32_t* feat_node, uint32_t* bow_word,
                         double* bow_value, uint32_t* fv_node, int* fv_start, int* fv_feat,
                         int* counts) {
  const Vocabulary* v = (const Vocabulary*)vp;
  for (int i = 0; i < n; i++) {
    uint32_t w = 0, nd = 0;
    double x = 0;
    v->transform1(desc + 32 * (size_t)i, levelsup, w, x, nd);
    feat_word[i] = w;
    feat_weight[i] = x;
    feat_node[i] = nd;
  }
  BowVec b;
  FeatVecO f;
  v->transform(desc, n, levelsup, b, f);
  counts[0] = (int)b.word.size();
  counts[1] = (int)f.node.size();
  for (size_t i = 0; i < b.word.size(); i++) {
    bow_word[i] = b.word[i];
    bow_value[i] = b.value[i];
  }
  for (size_t i = 0; i < f.node.size(); i++) fv_node[i] = f.node[i];
  for (size_t i = 0; i < f.start.size(); i++) fv_start[i] = f.start[i];
  for (size_t i = 0; i < f.feat.size(); i++) fv_feat[i] = f.feat[i];
  return 0;
}
double oracle_voc_score(void* vp, const uint32_t* wa, const double* va, int na,
                        const uint32_t* wb, const double* vb, int nb) {
  BowVec a, b;
  a.word.assign(wa, wa + na);
  a.value.assign(va, va + na);
  b.word.assign(wb, wb + nb);
  b.value.assign(vb, vb + nb);
  return ((const Vocabulary*)vp)->score(a, b);
}

// LocalMapping counters: [BAs, fused, culled keyframes, BA-erased observations, BA trials, BA
// edges, BA keyframe vertices, BA points, largest count of optimised keyframes, re-parented
// spanning-tree children]
void oracle_tracker_map_stats(void* tp, long long* out) {
  const MapTracker::MappingStats& m = ((OTracker*)tp)->map.mstats;
  const long v[10] = {m.n_ba, m.n_fused, m.n_culled, m.n_ba_erased, m.ba_trials, m.ba_edges,
                      m.ba_kfs, m.ba_pts, m.ba_max_opt_kfs, m.n_reparent};
  for (int i = 0; i < 10; i++) out[i] = v[i];
}

void oracle_tracker_set_cull_ratio(void* tp, double r) { ((OTracker*)tp)->map.cullRatio = r; }

// Records the problem and result of the which-th LocalBundleAdjustment (0-based) of this tracker,
// as probe fixtures for the GPU solver.
struct BACapture {
  int want = -1, seen = 0, got = 0;
  std::vector<float> T, X, obs, s, rT, rX;
  std::vector<uint8_t> fixed, erase;
  std::vector<int> pt, kf;
  int n_kf = 0, n_pt = 0, n_edge = 0, it[2] = {0, 0}, tr[2] = {0, 0};
};
static std::map<void*, BACapture> g_cap;

void oracle_tracker_capture_ba(void* tp, int which) {
  BACapture& c = g_cap[tp];
  c = BACapture();
  c.want = which;
  ((OTracker*)tp)->map.ba_hook = [tp](const BAProblem& P, const BAResult& R) {
    BACapture& c = g_cap[tp];
    if (c.seen++ != c.want) return;
    c.got = 1;
    c.n_kf = P.n_kf; c.n_pt = P.n_pt; c.n_edge = P.n_edge;
    c.T.assign(P.Tcw, P.Tcw + 16 * (size_t)P.n_kf);
    c.fixed.assign(P.fixed, P.fixed + P.n_kf);
    c.X.assign(P.Xw, P.Xw + 3 * (size_t)P.n_pt);
    c.pt.assign(P.e_pt, P.e_pt + P.n_edge);
    c.kf.assign(P.e_kf, P.e_kf + P.n_edge);
    c.obs.assign(P.e_obs, P.e_obs + 3 * (size_t)P.n_edge);
    c.s.assign(P.e_inv_sigma2, P.e_inv_sigma2 + P.n_edge);
    c.rT = R.Tcw; c.rX = R.Xw; c.erase = R.erase;
    c.it[0] = R.iterations[0]; c.it[1] = R.iterations[1];
    c.tr[0] = R.trials[0]; c.tr[1] = R.trials[1];
  };
}

// D3 problem capture (test hook): the problem of object `obj` in the `frame`-th track() call
struct D3Capture {
  long frame = -1;
  int obj = -1, got = 0, n = 0;
  std::vector<float> obs, flow, depth;
  float Tl[16], init[16];
};
static std::map<void*, D3Capture> g_d3;

void oracle_tracker_capture_d3(void* tp, long frame, int obj) {
  D3Capture& c = g_d3[tp];
  c = D3Capture();
  c.frame = frame;
  c.obj = obj;
  ((OTracker*)tp)->d3_hook = [tp](const FlowProblem& p, long f, int o) {
    D3Capture& c = g_d3[tp];
    if (f != c.frame || o != c.obj) return;
    c.got = 1;
    c.n = p.n;
    c.obs.assign(p.obs, p.obs + 2 * (size_t)p.n);
    c.flow.assign(p.flow, p.flow + 2 * (size_t)p.n);
    c.depth.assign(p.depth, p.depth + p.n);
    memcpy(c.Tl, p.Tcw_last, sizeof(c.Tl));
    memcpy(c.init, p.init, sizeof(c.init));
  };
}

// *n = edges (-1 until captured); with non-null arrays, copies the problem out
int oracle_tracker_captured_d3(void* tp, int* n, float* obs, float* flow, float* depth, float* Tl,
                               float* init) {
  D3Capture& c = g_d3[tp];
  *n = c.got ? c.n : -1;
  if (!c.got || !obs) return c.got;
  memcpy(obs, c.obs.data(), 4 * c.obs.size());
  memcpy(flow, c.flow.data(), 4 * c.flow.size());
  memcpy(depth, c.depth.data(), 4 * c.depth.size());
  memcpy(Tl, c.Tl, sizeof(c.Tl));
  memcpy(init, c.init, sizeof(c.init));
  return 1;
}

// The tracker's map as flat arrays, laid out as the product's mmt_map_dump (include/mmt.h):
// sizes[7] = keyframes, map points, observations, connections, ordered covisibles, children,
// keyframe map-point slots; the arrays (a struct of pointers, field for field
// mmt_map_dump_arrays) are written when out is non-null.
struct OracleMapDump {
  long long* kf_i;
  float* kf_T;
  int* kf_mps_start;
  int* kf_mps;
  float* pt_f;
  int* pt_i;
  int* obs_start;
  int* obs_i;
  float* obs_f;
  int* conn;
  int* ord;
  int* child;
};

int oracle_tracker_map_dump(void* tp, int* sizes, const OracleMapDump* out) {
  const MapTracker& M = ((OTracker*)tp)->map;
  long nobs = 0, nconn = 0, nord = 0, nchild = 0, nslots = 0;
  for (const OMapPoint& p : M.pts) nobs += (long)p.obs.size();
  for (const OKeyFrame& K : M.kfs) {
    nconn += (long)K.conn.size();
    nord += (long)K.ordered.size();
    nchild += (long)K.children.size();
    nslots += (long)K.mps.size();
  }
  const long n[7] = {(long)M.kfs.size(), (long)M.pts.size(), nobs, nconn, nord, nchild, nslots};
  for (int i = 0; i < 7; i++) sizes[i] = (int)n[i];
  if (!out) return 0;
  long c = 0, o = 0, ch = 0, sl = 0;
  for (size_t k = 0; k < M.kfs.size(); k++) {
    const OKeyFrame& K = M.kfs[k];
    long long* ki = out->kf_i + 4 * k;
    ki[0] = K.id; ki[1] = K.frameId; ki[2] = K.bad; ki[3] = K.parent;
    memcpy(out->kf_T + 16 * k, K.Tcw, 64);
    out->kf_mps_start[k] = (int)sl;
    for (int h : K.mps) out->kf_mps[sl++] = h;
    for (const auto& kv : K.conn) {
      int* e = out->conn + 3 * c++;
      e[0] = (int)k; e[1] = kv.first; e[2] = kv.second;
    }
    for (size_t q = 0; q < K.ordered.size(); q++) {
      int* e = out->ord + 3 * o++;
      e[0] = (int)k; e[1] = K.ordered[q]; e[2] = K.orderedW[q];
    }
    for (int q : K.children) {
      int* e = out->child + 2 * ch++;
      e[0] = (int)k; e[1] = q;
    }
  }
  out->kf_mps_start[M.kfs.size()] = (int)sl;
  long b = 0;
  for (size_t j = 0; j < M.pts.size(); j++) {
    const OMapPoint& p = M.pts[j];
    memcpy(out->pt_f + 5 * j, p.pos, 12);
    out->pt_f[5 * j + 3] = p.minDist; out->pt_f[5 * j + 4] = p.maxDist;
    int* pi = out->pt_i + 5 * j;
    pi[0] = p.bad; pi[1] = p.nObs; pi[2] = p.refKF; pi[3] = p.firstKFid; pi[4] = p.replaced;
    out->obs_start[j] = (int)b;
    for (const auto& kv : p.obs) {
      const OKeyFrame& K = M.kfs[kv.first];
      int* oi = out->obs_i + 3 * b;
      float* of = out->obs_f + 4 * b;
      oi[0] = kv.first; oi[1] = kv.second; oi[2] = K.keys[kv.second].octave;
      of[0] = K.keys[kv.second].x; of[1] = K.keys[kv.second].y;
      of[2] = K.depth[kv.second]; of[3] = K.uR[kv.second];
      b++;
    }
  }
  out->obs_start[M.pts.size()] = (int)b;
  return 0;
}

// sizes[3] = n_kf, n_pt, n_edge (0s until captured); with non-null arrays, copies the problem out
int oracle_tracker_captured_ba(void* tp, int* sizes, float* T, uint8_t* fixed, float* X, int* pt,
                               int* kf, float* obs, float* s) {
  BACapture& c = g_cap[tp];
  sizes[0] = c.got ? c.n_kf : 0;
  sizes[1] = c.got ? c.n_pt : 0;
  sizes[2] = c.got ? c.n_edge : 0;
  if (!c.got || !T) return c.got;
  memcpy(T, c.T.data(), 4 * c.T.size());
  memcpy(fixed, c.fixed.data(), c.fixed.size());
  memcpy(X, c.X.data(), 4 * c.X.size());
  memcpy(pt, c.pt.data(), 4 * c.pt.size());
  memcpy(kf, c.kf.data(), 4 * c.kf.size());
  memcpy(obs, c.obs.data(), 4 * c.obs.size());
  memcpy(s, c.s.data(), 4 * c.s.size());
  return 1;
}

// ORBmatcher::Fuse's per-point search against one keyframe (mapping_ref.cpp).  kps n, desc n x 32,
// depth W x H (mvuRight / the grid as the frame's), Tcw; points m: pos, normal, min/max distance,
// descriptor.  cam: fx fy cx cy bf; scale / inv_sigma2 nlevels.
int oracle_fuse_candidates(int W, int H, const float* cam, int nlevels, const float* scale,
                           const float* inv_sigma2, int n, const Key* kps, const uint8_t* desc,
                           const float* depth, const float* Tcw, int m, const float* pos,
                           const float* normal, const float* min_dist, const float* max_dist,
                           const uint8_t* pdesc, float th, int* best_idx, int* best_dist) {
  MapCam mc;
  mc.W = W; mc.H = H;
  mc.fx = cam[0]; mc.fy = cam[1]; mc.cx = cam[2]; mc.cy = cam[3]; mc.bf = cam[4];
  mc.nlevels = nlevels;
  mc.scale.assign(scale, scale + nlevels);
  mc.invSigma2.assign(inv_sigma2, inv_sigma2 + nlevels);
  mc.logScale = (float)std::log((double)scale[nlevels > 1 ? 1 : 0]);
  MatchFrame G;
  G.n = n;
  G.keys = kps;
  G.bf = mc.bf;
  frame_stereo_grid(G, depth, W, H);
  OKeyFrame K;
  K.keys.assign(kps, kps + n);
  K.uR = G.uR;
  K.depth = G.depth;
  K.desc.assign(desc, desc + 32 * (size_t)n);
  K.grid = G.grid;
  memcpy(K.Tcw, Tcw, 64);
  cam_centre(Tcw, K.Ow);
  for (int j = 0; j < m; j++) {
    OMapPoint p;
    memcpy(p.pos, pos + 3 * (size_t)j, 12);
    memcpy(p.normal, normal + 3 * (size_t)j, 12);
    p.minDist = min_dist[j];
    p.maxDist = max_dist[j];
    memcpy(p.desc, pdesc + 32 * (size_t)j, 32);
    best_dist[j] = fuse_candidate(K, mc, p, th, &best_idx[j]);
  }
  return 0;
}

// LocalBundleAdjustment's solve on a caller-given problem (ba_ref.cpp).  stats: [iterations of
// round 1, of round 2, trials of round 1, of round 2, erased edges]
int oracle_local_ba(int n_kf, int n_pt, int n_edge, const float* T, const uint8_t* fixed,
                    const float* X, const int* pt, const int* kf, const float* obs, const float* s,
                    const float* cam, float* T_out, float* X_out, uint8_t* erase, int* stats) {
  BAProblem P;
  P.n_kf = n_kf; P.n_pt = n_pt; P.n_edge = n_edge;
  P.Tcw = T; P.fixed = fixed; P.Xw = X; P.e_pt = pt; P.e_kf = kf; P.e_obs = obs;
  P.e_inv_sigma2 = s;
  P.fx = cam[0]; P.fy = cam[1]; P.cx = cam[2]; P.cy = cam[3]; P.bf = cam[4];
  BAResult R;
  local_ba_solve(P, R);
  memcpy(T_out, R.Tcw.data(), 4 * R.Tcw.size());
  memcpy(X_out, R.Xw.data(), 4 * R.Xw.size());
  memcpy(erase, R.erase.data(), R.erase.size());
  stats[0] = R.iterations[0]; stats[1] = R.iterations[1];
  stats[2] = R.trials[0]; stats[3] = R.trials[1];
  stats[4] = R.n_erase;
  return 0;
}

// Tracks one frame.  info: [initialized, n_keys, n_static, n_obj_samples, ego_iters,
// ego_inliers, n_objects, map_state, map_matches_mm, map_inliers_local, n_keyframes,
// n_mappoints, new_keyframe].  tcw: 32 floats (the frame's pose, then the map branch's pose).
// objs: per object 8 ints (label, sem, n_points, ransac_inliers, mm_inliers, n_solve, n_inliers,
// iterations) + 51 floats (init, X, motion, centre_pre).
int oracle_tracker_track(void* tp, const uint8_t* bgr, const uint16_t* disp, const float* flow,
                         const int32_t* mask, float* tcw, int* info, int* obj_i, float* obj_f,
                         int obj_cap) {
  OTracker* t = (OTracker*)tp;
  FrameResult r;
  t->track(bgr, disp, flow, mask, r);
  memcpy(tcw, r.Tcw, sizeof(r.Tcw));
  memcpy(tcw + 16, r.map.Tcw_map, sizeof(r.map.Tcw_map));
  info[7] = r.map.state;
  info[8] = r.map.matches_mm;
  info[9] = r.map.inliers_local;
  info[10] = r.map.n_keyframes;
  info[11] = r.map.n_mappoints;
  info[12] = r.map.new_keyframe;
  info[0] = r.initialized;
  info[1] = r.n_keys;
  info[2] = r.n_static;
  info[3] = r.n_obj_samples;
  info[4] = r.ego_iterations;
  info[5] = r.ego_inliers;
  info[6] = (int)r.objects.size();
  for (int i = 0; i < (int)r.objects.size() && i < obj_cap; i++) {
    const ObjectResult& o = r.objects[i];
    int* oi = obj_i + 8 * i;
    oi[0] = o.label; oi[1] = o.sem_label; oi[2] = o.n_points; oi[3] = o.n_ransac_inliers;
    oi[4] = o.n_mm_inliers; oi[5] = o.n_solve; oi[6] = o.n_inliers; oi[7] = o.iterations;
    float* of = obj_f + 51 * i;
    memcpy(of, o.init, 64);
    memcpy(of + 16, o.X, 64);
    memcpy(of + 32, o.motion, 64);
    memcpy(of + 48, o.centre_pre, 12);
  }
  return 0;
}

// ---------------------------------------------------------------- B3 / C1-C3 (oracle_match.h)
// cam = fx, fy, cx, cy, bf; scale = mvScaleFactors (nlevels).
static void match_frame(MatchFrame& F, int n, const Key* keys, const uint8_t* desc,
                        const float* depth, int W, int H, const float* cam, const float* scale,
                        int nlevels) {
  F.n = n;
  F.keys = keys;
  F.desc = desc;
  F.fx = cam[0]; F.fy = cam[1]; F.cx = cam[2]; F.cy = cam[3]; F.bf = cam[4];
  F.scale.assign(scale, scale + nlevels);
  F.nlevels = nlevels;
  F.logScale = (float)std::log((double)scale[1]);  // mfLogScaleFactor = log(mfScaleFactor)
  frame_stereo_grid(F, depth, W, H);
}

// B3: uR, depth (n each); cell_start (64*48+1) and cell_idx (n) as CSR over cells ix*48+iy.
int oracle_frame_stereo_grid(int n, const Key* keys, const float* depth, int W, int H,
                             const float* cam, float* uR, float* dep, int* cell_start,
                             int* cell_idx) {
  MatchFrame F;
  const float scale[2] = {1.f, 1.2f};
  match_frame(F, n, keys, nullptr, depth, W, H, cam, scale, 2);
  int pos = 0;
  for (int c = 0; c < kGridCols * kGridRows; c++) {
    cell_start[c] = pos;
    for (int k : F.grid[c]) cell_idx[pos++] = k;
  }
  cell_start[kGridCols * kGridRows] = pos;
  for (int i = 0; i < n; i++) {
    uR[i] = F.uR[i];
    dep[i] = F.depth[i];
  }
  return pos;
}

int oracle_search_by_projection_frame(int n2, const Key* keys2, const uint8_t* desc2,
                                      const float* depth, int W, int H, const float* cam,
                                      const float* scale, int nlevels, const float* Tcw, int n1,
                                      const Key* keys1, const float* Xw, const uint8_t* mp_desc,
                                      const uint8_t* active, const float* Tlw, float th, int mono,
                                      int check_orientation, int* match, const uint8_t* obs) {
  MatchFrame C;
  match_frame(C, n2, keys2, desc2, depth, W, H, cam, scale, nlevels);
  LastFrameView L;
  L.n = n1;
  L.keys = keys1;
  L.Xw = Xw;
  L.mp_desc = mp_desc;
  L.active = active;
  L.obs = obs;
  memcpy(L.Tcw, Tlw, sizeof(L.Tcw));
  return search_by_projection_frame(C, Tcw, L, th, mono != 0, check_orientation != 0, match);
}

// frustum_out: m x 6 floats (in_view, level, u, v, uR, view_cos).
int oracle_search_local_points(int n, const Key* keys, const uint8_t* desc, const float* depth,
                               int W, int H, const float* cam, const float* scale, int nlevels,
                               const float* Tcw, int m, const float* Xw, const float* normal,
                               const float* min_dist, const float* max_dist,
                               const uint8_t* pdesc, const uint8_t* skip, float th,
                               const uint8_t* taken, int* match, float* frustum_out) {
  MatchFrame C;
  match_frame(C, n, keys, desc, depth, W, H, cam, scale, nlevels);
  std::vector<LocalPoint> pts(m);
  for (int j = 0; j < m; j++) {
    LocalPoint& p = pts[j];
    memcpy(p.Xw, Xw + 3 * j, 12);
    memcpy(p.normal, normal + 3 * j, 12);
    p.min_dist = min_dist[j];
    p.max_dist = max_dist[j];
    p.desc = pdesc + 32 * (size_t)j;
    p.skip = skip[j];
  }
  std::vector<FrustumOut> fr(m);
  const int nm = search_local_points(C, Tcw, pts.data(), m, th, taken, match, fr.data());
  for (int j = 0; j < m; j++) {
    float* o = frustum_out + 6 * j;
    o[0] = (float)fr[j].in_view;
    o[1] = (float)fr[j].level;
    o[2] = fr[j].u;
    o[3] = fr[j].v;
    o[4] = fr[j].uR;
    o[5] = fr[j].view_cos;
  }
  return nm;
}

// C4 probe: feature vectors as (n_nodes, node ids, starts, features) arrays.
int oracle_search_by_bow(int kf_nodes, const uint32_t* kf_node, const int* kf_start,
                         const int* kf_feat, const Key* kf_keys, const uint8_t* kf_desc,
                         const uint8_t* kf_mp_ok, int f_nodes, const uint32_t* f_node,
                         const int* f_start, const int* f_feat, int nF, const Key* f_keys,
                         const uint8_t* f_desc, float nnratio, int check_orientation, int* match) {
  FeatVec a, b;
  a.n_nodes = kf_nodes;
  a.node = kf_node;
  a.start = kf_start;
  a.feat = kf_feat;
  b.n_nodes = f_nodes;
  b.node = f_node;
  b.start = f_start;
  b.feat = f_feat;
  return search_by_bow(a, kf_keys, kf_desc, kf_mp_ok, b, f_keys, f_desc, nF, nnratio,
                       check_orientation != 0, match);
}

}  // extern "C"
