/* include/mmt.h -- C-ABI of libmmt, the MI355X-native per-frame front end of the
 * cule/multimot_track multi-motion tracker (ORB extraction -> flow/semantic association ->
 * per-motion pose solves).
 *
 * Plain pointers and sizes only; no OpenCV/Eigen/torch types.  Every entry point returns 0 on
 * success and a negative errno-style code on failure (never exit()); mmt_last_error() gives the
 * message.  One context per host thread, bound to one HIP device.  Inputs are caller-owned and
 * read-only (the reference mutates depthmap in place, Tracking.cc:447-456; we do not).
 *
 * Reference interfaces replaced (paths relative to the reference checkout):
 *   mmt_create          <- ORB_SLAM2::System::System(voc, settings, RGBD, viewer)  System.h:62,
 *                          Tracking::Tracking settings parse Tracking.cc:135-238,
 *                          ORBextractor::ORBextractor  ORBextractor.cc:410-470
 *   mmt_orb_extract     <- ORBextractor::operator()(image, mask, keypoints, descriptors)
 *                          ORBextractor.h:59-61 / ORBextractor.cc:1046-1109
 *   mmt_orb_extract_batch / _device
 *                       <- the same, over many frames (ORB extraction is stateless per frame)
 *   mmt_track_rgbd      <- System::TrackRGBD(im, depthmap, flowmap, masksem, ...) System.h:73-75,
 *                          System.cc:169-220 -> Tracking::GrabImageRGBD Tracking.cc:438-919
 *   mmt_track_rgbd_chunk / _chunk_device
 *                       <- the same over consecutive frames of the sequence (rgbd_tum.cc:158-176
 *                          calls it once per frame; frames of one sequence are a strict chain,
 *                          only ORB extraction is batched)
 *   mmt_pose_flow_solve <- Optimizer::PoseOptimizationFlow2Cam / PoseOptimizationFlow2
 *                          Optimizer.h:43-56, Optimizer.cc:396-601 / 2170-2377
 *   mmt_pose_optimization <- Optimizer::PoseOptimization(Frame*) Optimizer.cc:3121-3339
 *   mmt_frame_grid      <- Frame::ComputeStereoFromRGBD + AssignFeaturesToGrid Frame.cc:1041, 601
 *   mmt_search_by_projection_frame
 *                       <- ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
 *                          ORBmatcher.h / ORBmatcher.cc:1958-2102
 *   mmt_search_local_points
 *                       <- Tracking::SearchLocalPoints Tracking.cc:3416-3466 ->
 *                          ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) :418-502
 *   mmt_search_by_bow   <- ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&, ...)
 *                          ORBmatcher.cc:532-663 (TrackReferenceKeyFrame Tracking.cc:2841-2853,
 *                          Relocalization :3631-3651)
 *   mmt_fuse_candidates <- ORBmatcher::Fuse(KeyFrame*, const vector<MapPoint*>&, th)'s search,
 *                          ORBmatcher.cc:1200-1324 (LocalMapping::SearchInNeighbors
 *                          LocalMapping.cc:458-538)
 *   mmt_local_bundle_adjustment
 *                       <- Optimizer::LocalBundleAdjustment's two optimisation rounds and inlier
 *                          test, Optimizer.cc:3394-3631 (LocalMapping.cc:81-84)
 *   mmt_load_vocabulary <- System::System's mpVocabulary->loadFromTextFile(strVocFile)
 *                          System.cc:63-73 (TemplatedVocabulary::loadFromTextFile,
 *                          Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424)
 *   mmt_bow_transform   <- TemplatedVocabulary::transform(feature, word, weight, &node, levelsup)
 *                          TemplatedVocabulary.h:1218-1259 (Frame::ComputeBoW, Frame.cc:778-786)
 *   mmt_destroy         <- System::Shutdown / delete
 */
#ifndef MMT_H
#define MMT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMT_OK 0
#define MMT_EINVAL (-22)
#define MMT_ENOMEM (-12)
#define MMT_ENOSPC (-28)
#define MMT_EDEVICE (-5)
#define MMT_ESTATE (-77)

/* Most object motions a frame reports (semantic labels 1..15).  mmt_frame_result.n_objects is
 * the frame's full count; an objs_cap below it receives the first objs_cap motions only, so size
 * the motion arrays with MMT_MAX_OBJECTS per frame. */
#define MMT_MAX_OBJECTS 15

/* Settings of kitti03.yaml (Camera.*, ThDepth, ORBextractor.*) plus build-side knobs. */
typedef struct mmt_config {
  int width, height;              /* Camera.width / Camera.height                       */
  float fx, fy, cx, cy;           /* Camera.fx fy cx cy                                  */
  float k1, k2, p1, p2, k3;       /* distortion (must be 0 on this path)                 */
  float bf;                       /* Camera.bf                                           */
  float th_depth;                 /* ThDepth (baseline units, Tracking.cc:225)          */
  int rgb;                        /* Camera.RGB (1: cvtColor RGB2GRAY on the input)      */
  int orb_nfeatures;              /* ORBextractor.nFeatures                              */
  float orb_scale_factor;         /* ORBextractor.scaleFactor                            */
  int orb_nlevels;                /* ORBextractor.nLevels                                */
  int orb_ini_th_fast;            /* ORBextractor.iniThFAST                              */
  int orb_min_th_fast;            /* ORBextractor.minThFAST                              */
  uint32_t noise_seed;            /* replaces cv::RNG(time(NULL)), Frame.cc:1246         */
  int device_id;                  /* HIP device ordinal                                  */
  int max_batch;                  /* frames in flight for batched ORB extraction         */
  float fps;                      /* Camera.fps: mMaxFrames of the keyframe policy
                                     (Tracking.cc:170-176; 0 -> 30 as the reference)     */
} mmt_config;

/* cv::KeyPoint, same field order and size (28 bytes). */
typedef struct mmt_kp {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} mmt_kp;

/* One recovered object motion (Tracking.cc:2127-2129: vObjMod = Tcw^-1 * X). */
typedef struct mmt_motion {
  int32_t label;            /* nModLabel (track id)                                   */
  int32_t sem_label;        /* semantic label (nSemPosition)                          */
  int32_t n_points;         /* object samples (ObjIdNew[i].size())                    */
  int32_t n_inliers;        /* solve edges with chi2 <= 0.01 after PoseOptimizationFlow2 */
  int32_t n_ransac_inliers; /* solvePnPRansac inliers                                 */
  int32_t n_mm_inliers;     /* motion-model inliers (-1: no previous motion)          */
  int32_t n_solve;          /* flow vertices in the solve (ObjIdTest_in.size())        */
  int32_t iterations;       /* LM iterations                                          */
  float world_motion[16];   /* row-major 4x4 vObjMod = Tcw^-1 * X                      */
  float cam_pose[16];       /* row-major 4x4 X (PoseOptimizationFlow2 output)          */
  float init_pose[16];      /* row-major 4x4 mInitModel (PnP or motion model)          */
  float centre_pre[3];      /* ObjCentre3D_pre (Tracking.cc:2032-2049): mean world point of
                               the solve's last-frame samples, noisy depth (UnprojectStereoObject
                               (j, 1)); the object-speed estimate of Tracking.cc:2186 uses it.
                               The reference computes it before the solve whatever the count:
                               1-2 samples give their mean, none gives NaN (0 * (1 / 0))   */
} mmt_motion;

/* Per-frame tracking result (the Tcw cv::Mat returned by System::TrackRGBD + counters). */
typedef struct mmt_frame_result {
  float Tcw[16];            /* row-major camera pose (world -> camera)                 */
  int32_t initialized;      /* tracking state OK (StereoInitialization done)           */
  int32_t n_keypoints;      /* ORB keypoints of the frame                              */
  int32_t n_obj_samples;    /* mvObjKeys.size(): last frame's hand-off (own on frame 0) */
  int32_t ego_iterations;   /* LM iterations of PoseOptimizationFlow2Cam               */
  int32_t ego_inliers;      /* its inliers (chi2 <= 0.04)                              */
  int32_t n_objects;        /* dynamic objects solved this frame                       */
  /* ORB-SLAM2 map tracking (Tracking.cc:985-1176), which sets the flow solve's initial pose */
  int32_t map_state;        /* mState after the frame: 0 not initialised, 1 OK, 2 LOST     */
  int32_t map_matches_mm;   /* TrackWithMotionModel's SearchByProjection matches (-1: none) */
  int32_t map_inliers_local;/* mnMatchesInliers of TrackLocalMap (-1: not run)             */
  int32_t n_keyframes;      /* keyframes in the map                                      */
  int32_t n_mappoints;      /* map points in the map                                     */
  int32_t new_keyframe;     /* this frame became a keyframe                              */
  float Tcw_map[16];        /* row-major pose of the map branch (PoseOptimization's output,
                               the initial estimate of PoseOptimizationFlow2Cam)        */
  int32_t frame_index;      /* this frame's index in the sequence (frames since the reset) */
  int32_t objects_frame;    /* the frame whose object motions n_objects / objs describe: this
                               frame, or with deferred object results an earlier one (-1:
                               none in this slot)                                        */
} mmt_frame_result;

typedef struct mmt_ctx mmt_ctx;

int mmt_version(void);
const char* mmt_last_error(const mmt_ctx* ctx);

mmt_ctx* mmt_create(const mmt_config* cfg);
void mmt_destroy(mmt_ctx* ctx);

/* Per-level ORB tables derived exactly as ORBextractor's ctor (sizes nlevels). */
int mmt_orb_levels(const mmt_ctx* ctx, float* scale, float* sigma2, int* n_per_level,
                   int* level_w, int* level_h);

/* ORBextractor::operator() on one 8-bit gray image (host pointers). keypoints/descriptors are
 * level-major exactly as the reference.  *n receives the count; MMT_ENOSPC if cap is short. */
int mmt_orb_extract(mmt_ctx* ctx, const uint8_t* gray, int w, int h, int stride, mmt_kp* kps,
                    uint8_t* desc, int cap, int* n);

/* Same over `nframes` host frames (each w x h, row stride `stride`), processed as one batch
 * of device launches.  Outputs are frame-major with `cap_per_frame` slots per frame. */
int mmt_orb_extract_batch(mmt_ctx* ctx, const uint8_t* const* grays, int nframes, int stride,
                          mmt_kp* kps, uint8_t* desc, int cap_per_frame, int* n_per_frame);

/* Device-resident variant: d_gray holds nframes gray frames (pitch frame_pitch bytes, rows of
 * `width` bytes, tightly packed); all outputs are device pointers; runs on `stream`
 * (hipStream_t, may be NULL for the context stream).  No host synchronisation, so the device-side
 * error flags of these launches are reported by mmt_orb_device_status. */
int mmt_orb_extract_device(mmt_ctx* ctx, const uint8_t* d_gray, int nframes, size_t frame_pitch,
                           mmt_kp* d_kps, uint8_t* d_desc, int cap_per_frame, int* d_n,
                           void* stream);

/* Synchronises `stream` (NULL: the context stream) and reports the device-side error flags that
 * ORB launches set since the last check (octree pass guard, node capacity, output truncation):
 * MMT_OK, or MMT_EDEVICE with mmt_last_error naming the flags.  The flags are cleared.  The
 * synchronous entry points (mmt_orb_extract*, mmt_track_rgbd*) run this check themselves, so a
 * tripped guard is never returned as MMT_OK with truncated keypoints. */
int mmt_orb_device_status(mmt_ctx* ctx, void* stream);

/* System::TrackRGBD on one frame (host buffers): bgr 8UC3 (w*h*3), disparity*256 u16 (w*h),
 * flow t->t+1 (w*h*2 float), semantic labels (w*h int32, LoadMask-filtered).  Fills `res` and up
 * to objs_cap object motions.  The first call with > 500 keypoints initialises (Tcw = I). */
int mmt_track_rgbd(mmt_ctx* ctx, const uint8_t* bgr, const uint16_t* disp256,
                   const float* flow_uv, const int32_t* mask, double timestamp,
                   mmt_frame_result* res, mmt_motion* objs, int objs_cap);

/* System::TrackRGBD over nframes consecutive frames in host memory, one pointer per frame and
 * input (layouts as mmt_track_rgbd): the frames are staged on the device and tracked as one chunk
 * (batched ORB, then frame by frame), like mmt_track_rgbd_chunk_device.  nframes <=
 * config.max_batch; res[nframes], objs[nframes * objs_cap].  Frames in pinned memory from
 * mmt_host_alloc reach the GPU by DMA at full PCIe rate. */
int mmt_track_rgbd_chunk(mmt_ctx* ctx, int nframes, const uint8_t* const* bgr,
                         const uint16_t* const* disp256, const float* const* flow_uv,
                         const int32_t* const* mask, mmt_frame_result* res, mmt_motion* objs,
                         int objs_cap);

/* Page-locked host memory on the context's device (hipHostMalloc), for frames the caller decodes
 * and hands to the host-buffer entry points.  NULL on failure; release with mmt_host_free. */
void* mmt_host_alloc(mmt_ctx* ctx, size_t bytes);
void mmt_host_free(mmt_ctx* ctx, void* p);

/* Device-resident chunk of consecutive frames of the context's sequence (pitches in bytes):
 * ORB extraction is batched over the chunk, tracking then runs frame by frame.  res[nframes],
 * objs[nframes * objs_cap] are host arrays.
 * Errors (both track entry points): a chunk whose ORB run trips a device guard returns
 * MMT_EDEVICE before any of its frames is tracked, and the context keeps the state of the previous
 * call, so tracking may continue with the next frames (or restart after mmt_reset). */
int mmt_track_rgbd_chunk_device(mmt_ctx* ctx, int nframes, const uint8_t* d_bgr,
                                size_t bgr_pitch, const uint16_t* d_disp, size_t disp_pitch,
                                const float* d_flow, size_t flow_pitch, const int32_t* d_mask,
                                size_t mask_pitch, mmt_frame_result* res, mmt_motion* objs,
                                int objs_cap, void* stream);

/* One flow-refined pose solve (probe of PoseOptimizationFlow2Cam / PoseOptimizationFlow2).
 * obs/flow: n x 2 floats (last-frame sample pixel, its flow); depth: n floats. */
typedef struct mmt_flow_problem {
  int n;
  const float* obs;
  const float* flow;
  const float* depth;
  float Tcw_last[16];  /* row-major last camera pose; edges use its inverse (Twl)   */
  float init[16];      /* row-major initial estimate                                */
  float rp_thres;      /* 0.04 ego / 0.01 object (Huber delta^2)                    */
  double prior_info;   /* 0.3 ego / 0.5 object                                      */
  int max_iters;       /* 100 ego / 200 object                                      */
  int use_noise;       /* ego: depth += g0 * z^2/362.5*0.15 (ObtainFlowDepthCamera) */
  float g0;            /* the cv::RNG gaussian draw of the noise seed               */
  float fx, fy, cx, cy;
} mmt_flow_problem;
int mmt_pose_flow_solve(mmt_ctx* ctx, const mmt_flow_problem* problem, float* pose_out,
                        int* stats_out /* iterations, inliers, status */);

/* Optimizer::PoseOptimization(Frame*) (reference include/Optimizer.h:43, src/Optimizer.cc:3121-3339)
 * on the frame's MapPoint observations (the edges of the frame's non-null mvpMapPoints, in index
 * order): Xw n x 3 world positions, obs n x (u, v, uR) with uR = mvuRight (< 0: mono edge),
 * inv_sigma2 n = mvInvLevelSigma2[octave].  Tcw = pFrame->mTcw (row-major).  Writes the optimised
 * pose and mvbOutlier (outlier_out, n bytes); *n_inliers = the function's return value
 * (nInitialCorrespondences - nBad; 0 with the pose unchanged below 3 edges). */
typedef struct mmt_pose_opt_problem {
  int n;
  const float* Xw;
  const float* obs;
  const float* inv_sigma2;
  float Tcw[16];
  float fx, fy, cx, cy, bf;
} mmt_pose_opt_problem;
int mmt_pose_optimization(mmt_ctx* ctx, const mmt_pose_opt_problem* problem, float* pose_out,
                          uint8_t* outlier_out, int* n_inliers);

/* cv::solvePnPRansac(..., SOLVEPNP_AP3P) probe as called by GetInitModelObj: pts3 n x 3,
 * pts2 n x 2 floats.  R_out row-major 3x3 (after the Rodrigues round trip), t_out 3;
 * inliers_out (optional, n ints) receives the RANSAC inlier indices. */
int mmt_pnp_ransac(mmt_ctx* ctx, const float* pts3, const float* pts2, int n, float fx,
                   float fy, float cx, float cy, int max_iters, double reproj, double confidence,
                   double* R_out, double* t_out, int* inliers_out, int* n_inliers,
                   int* iters_out /* iterations run, best hypothesis */);

/* ---- PnPsolver (row D6): ORB-SLAM2's P4P EPnP-RANSAC of Tracking::Relocalization -------------
 * PnPsolver(F, vpMapPointMatches) + SetRansacParameters(probability, minInliers, maxIterations,
 * minSet, epsilon, th2) + iterate(nIterations, bNoMore, vbInliers, nInliers) (reference
 * src/PnPsolver.cc:67-339, driven by Tracking.cc:3659-3700 with (0.99, 10, 300, 4, 0.5, 5.991)
 * and nIterations 5).  The n correspondences in mvP2D / mvP3Dw order: pts3 n x 3 world points,
 * pts2 n x 2 pixels (mvKeysUn), sigma2 n = mvLevelSigma2[octave].  min_set must be 4.
 *
 * Random minimal sets: the reference draws them with DUtils::Random::RandomInt (rand()), so the
 * caller keeps that stream.  randi[4 k + j] = RandomInt(0, n - 1 - j) of draw j in iteration k of
 * this call; n_draw_iters must cover the call: max(maxIts - state->iterations, n_iterations),
 * maxIts being the iteration cap SetRansacParameters derives.  The solver's state across calls
 * (mnIterations, mnBestInliers, mBestTcw, mvbBestInliers) is *state, caller-owned (best_mask: n
 * bytes); zero it (iterations = best_inliers = 0) for a new solver.
 *
 * Outputs: *pose_found = 1 and Tcw_out / inliers_out (n bytes, mvKeyPointIndices order) /
 * *n_inliers when iterate() returns a pose (refined, or the best hypothesis once the iterations
 * are exhausted), 0 for the reference's empty cv::Mat; *no_more = bNoMore. */
typedef struct mmt_pnpsolver_problem {
  int n;
  const float* pts3;
  const float* pts2;
  const float* sigma2;
  float fx, fy, cx, cy;
  double probability;
  int min_inliers;
  int max_iterations;
  int min_set;
  float epsilon;
  float th2;
} mmt_pnpsolver_problem;

typedef struct mmt_pnpsolver_state {
  int iterations;          /* mnIterations                                                 */
  int best_inliers;        /* mnBestInliers                                                */
  float best_Tcw[16];      /* mBestTcw (row-major)                                         */
  uint8_t* best_mask;      /* mvbBestInliers, n bytes                                      */
} mmt_pnpsolver_state;

int mmt_pnpsolver_iterate(mmt_ctx* ctx, const mmt_pnpsolver_problem* problem,
                          const int32_t* randi, int n_draw_iters, int n_iterations,
                          mmt_pnpsolver_state* state, float* Tcw_out, uint8_t* inliers_out,
                          int* n_inliers, int* pose_found, int* no_more);

/* ---- Frame grid and projection matching (rows B3, C1-C3 of the hot path) ----------------------
 * The current Frame as the matchers read it: its ORB keys (mvKeysUn == mvKeys, no distortion),
 * descriptors (n x 32) and the metric depth map (w x h floats, the Tcw-independent part of
 * Frame::ComputeStereoFromRGBD).  Camera intrinsics, bf and the scale pyramid come from the
 * context's configuration; image bounds are [0, width] x [0, height] (Frame::ComputeImageBounds). */
typedef struct mmt_match_frame {
  int n;
  const mmt_kp* kps;
  const uint8_t* desc;
  const float* depth;
  float Tcw[16];        /* row-major mTcw used for the projections                         */
} mmt_match_frame;

/* Frame::ComputeStereoFromRGBD + AssignFeaturesToGrid (Frame.cc:1041-1062, 601-616, PosInGrid
 * 765-775): uR_out/depth_out (n) = mvuRight/mvDepth (-1 without depth); the 64 x 48 grid mGrid as
 * CSR: cell (ix, iy) holds cell_idx[cell_start[ix*48+iy] .. cell_start[ix*48+iy+1]) in ascending
 * key order; cell_start has 3073 entries, cell_idx n.  n <= 16384. */
int mmt_frame_grid(mmt_ctx* ctx, const mmt_match_frame* cur, float* uR_out, float* depth_out,
                   int* cell_start, int* cell_idx);

/* The last Frame as ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) reads it:
 * per last-frame key i, its keypoint (octave, angle), the world position and descriptor of
 * mvpMapPoints[i], and active[i] = (mvpMapPoints[i] != NULL && !mvbOutlier[i]). */
typedef struct mmt_last_frame {
  int n;
  const mmt_kp* kps;
  const float* Xw;          /* n x 3 */
  const uint8_t* mp_desc;   /* n x 32 */
  const uint8_t* active;    /* n */
  float Tcw[16];            /* row-major LastFrame.mTcw */
  const uint8_t* obs;       /* n, optional: mvpMapPoints[i]->Observations() > 0.  A current key
                               bound to a point without observations (a temporal visual-odometry
                               point of UpdateLastFrame) stays open to later points (NULL: every
                               point has observations) */
} mmt_last_frame;

/* ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) with mbCheckOrientation
 * (ORBmatcher.cc:1958-2102, called by Tracking::TrackWithMotionModel Tracking.cc:2962-3010; C1
 * DescriptorDistance ORBmatcher.cc:2279-2295).  The current frame starts with no MapPoints (as
 * after the fill(NULL) of Tracking.cc:2975); match_out[i2] (cur->n) = the last-frame index bound
 * to current key i2, or -1; *nmatches = the function's return value. */
int mmt_search_by_projection_frame(mmt_ctx* ctx, const mmt_match_frame* cur,
                                   const mmt_last_frame* last, float th, int mono,
                                   int check_orientation, int32_t* match_out, int* nmatches);

/* Local MapPoints as Tracking::SearchLocalPoints sees them (Tracking.cc:3416-3466): position,
 * mNormalVector, mfMinDistance / mfMaxDistance, mDescriptor, and skip = already matched in this
 * frame (mnLastFrameSeen == mCurrentFrame.mnId) or isBad(). */
typedef struct mmt_local_points {
  int m;
  const float* Xw;        /* m x 3  */
  const float* normal;    /* m x 3  */
  const float* min_dist;  /* m      */
  const float* max_dist;  /* m      */
  const uint8_t* desc;    /* m x 32 */
  const uint8_t* skip;    /* m      */
} mmt_local_points;

/* SearchLocalPoints' projection pass (Frame::isInFrustum(pMP, 0.5), Frame.cc:652-708, with
 * MapPoint::PredictScale MapPoint.cc:402-417) + ORBmatcher(0.8)::SearchByProjection(Frame&,
 * vector<MapPoint*>, th) (ORBmatcher.cc:418-502).  taken (cur->n bytes, optional) marks keys
 * that already hold a MapPoint; match_out[i] (cur->n) = the local point newly bound to key i, or
 * -1; frustum_out (m x 6 floats, optional) = in_view, predicted level, u, v, uR, view cos. */
int mmt_search_local_points(mmt_ctx* ctx, const mmt_match_frame* cur,
                            const mmt_local_points* pts, float th, const uint8_t* taken,
                            int32_t* match_out, float* frustum_out, int* nmatches);

/* DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>, FeatureVector.h) as flat
 * arrays: node_id ascending; the features of node k are feat[node_start[k] .. node_start[k+1])
 * in insertion order.  Every frame feature is listed in at most one node (DBoW2's transform puts
 * each feature in one node at the direct-index level), and a node holds at most 2048 of them. */
typedef struct mmt_feature_vector {
  int n_nodes;
  const uint32_t* node_id;    /* n_nodes              */
  const int32_t* node_start;  /* n_nodes + 1, from 0  */
  const int32_t* feat;        /* node_start[n_nodes]  */
} mmt_feature_vector;

/* A keyframe as SearchByBoW reads it: mvKeysUn (angle), mDescriptors, whether mvpMapPoints[i] holds
 * a MapPoint that is not bad, and mFeatVec. */
typedef struct mmt_bow_keyframe {
  int n;
  const mmt_kp* kps;
  const uint8_t* desc;      /* n x 32 */
  const uint8_t* mp_valid;  /* n      */
  mmt_feature_vector fv;
} mmt_bow_keyframe;

/* C4: ORBmatcher(nn_ratio, check_orientation)::SearchByBoW(pKF, F, vpMapPointMatches, ...)
 * (ORBmatcher.cc:532-663): per common vocabulary node, each keyframe feature with a good MapPoint
 * takes the closest unmatched frame feature of the node if its distance is <= TH_LOW (50) and below
 * nn_ratio times the second-best distance; then the rotation-consistency histogram.  match_out[i]
 * (n_cur) = the keyframe key whose MapPoint now matches frame key i (vpMapPointMatches[i] =
 * pKF->mvpMapPoints[match_out[i]]), or -1; *nmatches = the return value.  The reference uses
 * nn_ratio 0.7 in TrackReferenceKeyFrame and 0.75 in Relocalization. */
int mmt_search_by_bow(mmt_ctx* ctx, const mmt_bow_keyframe* kf, int n_cur, const mmt_kp* cur_kps,
                      const uint8_t* cur_desc, const mmt_feature_vector* cur_fv, float nn_ratio,
                      int check_orientation, int32_t* match_out, int* nmatches);

/* ORBmatcher::Fuse(pKF, vpMapPoints, th)'s per-point search (ORBmatcher.cc:1200-1324): the point
 * projected with the keyframe's pose (cur->Tcw), KeyFrame::IsInImage, the scale-invariance
 * distances (0.8 mfMinDistance, 1.2 mfMaxDistance), the 60-degree viewing angle, PredictScale, then
 * the keyframe keys in radius th * scale[level] at the predicted level or one below, gated by the
 * reprojection error (7.8 stereo, 5.99 monocular, times 1/sigma^2), and the closest descriptor
 * (first of equal distances).  best_idx / best_dist (m) = that key and its distance, or -1 / 256;
 * the reference fuses when best_dist <= 50.  The keyframe is a mmt_match_frame (its depth map
 * gives mvuRight); pts->skip is ignored (the caller skips bad points and points already in the
 * keyframe, ORBmatcher.cc:1224). */
int mmt_fuse_candidates(mmt_ctx* ctx, const mmt_match_frame* kf, const mmt_local_points* pts,
                        float th, int32_t* best_idx, int32_t* best_dist);

/* The graph of Optimizer::LocalBundleAdjustment (Optimizer.cc:3408-3541): keyframe vertices
 * (Tcw, fixed: the fixed cameras and keyframe 0), map points, and one edge per observation, listed
 * point by point (e_pt non-decreasing) with each point's observations in keyframe order. */
typedef struct mmt_ba_problem {
  int n_kf, n_pt, n_edge;
  const float* Tcw;            /* n_kf x 16 row-major                                  */
  const uint8_t* fixed;        /* n_kf                                                 */
  const float* Xw;             /* n_pt x 3                                             */
  const int32_t* e_pt;         /* n_edge                                               */
  const int32_t* e_kf;         /* n_edge                                               */
  const float* e_obs;          /* n_edge x (u, v, uR): keypoint and mvuRight (< 0: monocular,
                                  EdgeSE3ProjectXYZ; else EdgeStereoSE3ProjectXYZ)     */
  const float* e_inv_sigma2;   /* n_edge: mvInvLevelSigma2[octave] (the information)   */
} mmt_ba_problem;

/* LocalBundleAdjustment's solve (Optimizer.cc:3547-3631; g2o LM with BlockSolver_6_3, Huber
 * sqrt(5.991) / sqrt(7.815) in the first 5 iterations, the bad edges set aside, 10 more without the
 * kernel) on the GPU.  Tcw_out (n_kf x 16) and Xw_out (n_pt x 3) = Converter::toCvMat of the final
 * estimates; erase_out (n_edge) = the final inlier test failed (the observation the reference
 * erases); stats (5) = iterations of round 1, of round 2, LM trials of round 1, of round 2, erased
 * edges.  Camera from the context's configuration. */
int mmt_local_bundle_adjustment(mmt_ctx* ctx, const mmt_ba_problem* problem, float* Tcw_out,
                                float* Xw_out, uint8_t* erase_out, int32_t* stats);

/* LocalMapping counters of the context's tracker (no reference counterpart: test and profiling
 * hook).  Times are host wall microseconds, collected with MMT_MAP_PROFILE=1. */
typedef struct mmt_map_counters {
  int64_t n_ba, n_fused, n_culled, n_ba_erased, ba_trials, ba_edges, ba_kfs, ba_pts, ba_max_opt,
      fuse_launches, fuse_queries, fuse_relaunches;
  double lm_us, ba_us, fuse_us;
  int64_t d2_split_fallbacks;  /* ego flow solves re-run on one workgroup because the split
                                  solve's workgroups were not resident together             */
  int64_t n_reparent;          /* spanning-tree children re-parented by KeyFrame::SetBadFlag
                                  (KeyFrame.cc:480-537) when KeyFrameCulling culls a keyframe */
} mmt_map_counters;
int mmt_map_counters_read(mmt_ctx* ctx, mmt_map_counters* out);

/* Test knob (no reference counterpart): LocalMapping::KeyFrameCulling's redundancy ratio, a
 * keyframe is culled when more than ratio x its close map points are seen by 3 other keyframes
 * (0.9 in the reference, LocalMapping.cc:697; the default).  The synthetic sequences never reach
 * 0.9, so the culling tests lower it to exercise KeyFrame::SetBadFlag. */
int mmt_set_keyframe_culling_ratio(mmt_ctx* ctx, double ratio);

/* ---- ORB vocabulary ------------------------------------------------------------
 * System(voc, ...) loads DBoW2's text vocabulary (System.cc:63-73): the header "k L scoring
 * weighting", then one line per node "parent is_leaf d0 .. d31 weight".  With a vocabulary the
 * tracker runs the reference's TrackReferenceKeyFrame (SearchByBoW against the reference
 * keyframe, Tracking.cc:2836-2892), Relocalization (KeyFrameDatabase candidates, SearchByBoW,
 * PnPsolver, the SearchByProjection(F, KF, ...) rounds; Tracking.cc:3614-3776) and LocalMapping's
 * CreateNewMapPoints (SearchForTriangulation, LocalMapping.cc:210-456), and keeps the keyframe
 * database; without one it runs the documented substitutes.  Load it before
 * the first frame (MMT_ESTATE afterwards).  Scorings L1 / L2 (ORBvoc.txt: L1, TF-IDF); errors:
 * MMT_EINVAL with mmt_last_error (unreadable file, the reference's header check). */
int mmt_load_vocabulary(mmt_ctx* ctx, const char* path);

/* Probe of TemplatedVocabulary::transform(feature, id, w, &nid, levelsup) over n descriptors (host
 * n x 32) on the GPU: word id, word weight (0: stopped) and the node at level L - levelsup. */
int mmt_bow_transform(mmt_ctx* ctx, const uint8_t* desc, int n, int levelsup, uint32_t* word,
                      double* weight, uint32_t* node);

/* Counters of the vocabulary path (tests): BoW conversions of frames, TrackReferenceKeyFrame calls
 * and successes, Relocalization calls and successes, candidate keyframes, PnPsolver poses,
 * SearchByProjection(F, KF) rounds, triangulated points, SearchForTriangulation matches, database
 * insertions. */
typedef struct mmt_bow_counters {
  int64_t bow_frames, trk, trk_ok, reloc, reloc_ok, reloc_cands, pnp_found, sbp_rounds,
      triangulated, sft_matches, kfdb;
} mmt_bow_counters;
int mmt_bow_counters_read(mmt_ctx* ctx, mmt_bow_counters* out);

/* The tracker's map as flat arrays (no reference counterpart: the map invariant tests and the
 * map-graph parity against the CPU oracle read it).  Keyframes and map points are numbered in
 * creation order (the reference's mnId order).  sizes[7] (out): keyframes, map points,
 * observations, connections, ordered covisibles, children, keyframe map-point slots.  With
 * out == NULL only the sizes are written; otherwise every array must hold its size. */
typedef struct mmt_map_dump_arrays {
  int64_t* kf_i;          /* n_kf x 4: mnId, mnFrameId, isBad, parent (-1: none)             */
  float* kf_T;            /* n_kf x 16: Tcw                                                   */
  int32_t* kf_mps_start;  /* n_kf + 1: CSR offsets into kf_mps                                */
  int32_t* kf_mps;        /* slots: mvpMapPoints (map point number or -1)                     */
  float* pt_f;            /* n_pt x 5: world position, mfMinDistance, mfMaxDistance             */
  int32_t* pt_i;          /* n_pt x 5: isBad, nObs, mpRefKF, mnFirstKFid, mpReplaced (-1)     */
  int32_t* obs_start;     /* n_pt + 1: CSR offsets into obs_i / obs_f (mObservations)          */
  int32_t* obs_i;         /* n_obs x 3: keyframe, key index, key octave                        */
  float* obs_f;           /* n_obs x 4: key x, y, mvDepth, mvuRight                            */
  int32_t* conn;          /* n_conn x 3: keyframe, other, weight (mConnectedKeyFrameWeights)   */
  int32_t* ord;           /* n_ord x 3: keyframe, other, weight (mvpOrderedConnectedKeyFrames) */
  int32_t* child;         /* n_child x 2: keyframe, child (mspChildrens)                        */
} mmt_map_dump_arrays;
int mmt_map_dump(mmt_ctx* ctx, int32_t* sizes, const mmt_map_dump_arrays* out);

/* Visualisation hook (no reference counterpart; Tracking.cc:684-783 draws these into feat.png):
 * the static samples (mvSiftKeys, B2) and the object samples (mvObjKeys with vSemObjLabel, B1)
 * of the last frame the context tracked, xy as n x 2 floats.  Counts clipped to the caps. */
int mmt_frame_samples(mmt_ctx* ctx, float* static_xy, int static_cap, int* n_static,
                      float* obj_xy, int32_t* obj_label, int obj_cap, int* n_obj);

/* Stage timing with HIP events on the launch stream (no reference counterpart: measurement
 * hook for bench.py).  orb_ms sums the batched ORB launch sequences of the tracked chunks. */
typedef struct mmt_profile {
  double orb_ms;
  int64_t orb_launches;
  int64_t orb_frames;
} mmt_profile;
int mmt_profile_enable(mmt_ctx* ctx, int on);
int mmt_profile_read(mmt_ctx* ctx, mmt_profile* out, int reset);

/* Forget the sequence (Tracking::Reset). */
int mmt_reset(mmt_ctx* ctx);

/* Deferred object results (no reference counterpart; for callers that track one frame, or one
 * short chunk, per call).  By default every mmt_track_rgbd* call returns each frame with its own
 * object motions, which drains the object pipeline (PnP-RANSAC, PoseOptimizationFlow2 per object)
 * at the end of every call.  With on = 1 a call returns each frame's pose and map state at once,
 * and in the object fields of its results the motions of the frames whose object path has
 * finished, oldest first (res[i].objects_frame names the frame; -1: none yet): every frame's
 * motions arrive exactly once, in order, up to 17 frames later.  mmt_flush_objects finishes the
 * pipeline and returns the remaining records (res[k].objects_frame, n_objects and objs[k *
 * objs_cap ..] only), at most res_cap per call: *n = records written, 0 when none remain.
 * Turning the mode off flushes (and drops) the records still owed; mmt_reset drops them.  While
 * a flush has records left for a later mmt_flush_objects call, every mmt_track_rgbd* call returns
 * MMT_ESTATE (it would deliver newer frames' motions first).
 * MMT_EINVAL when the host object worker (MMT_OBJ_THREAD=1) is on. */
int mmt_set_deferred_objects(mmt_ctx* ctx, int on);
int mmt_flush_objects(mmt_ctx* ctx, mmt_frame_result* res, mmt_motion* objs, int objs_cap,
                      int res_cap, int* n);

/* Upper bound on keypoints per frame (sum over levels of quota + 3). */
int mmt_orb_capacity(const mmt_ctx* ctx);

/* ---- Debug and test hooks: not part of the stable interface, no reference counterpart ---- */

/* Test hook: OR `flags` into the ORB device error word (as a tripped kernel guard would). */
int mmt_debug_orb_raise(mmt_ctx* ctx, int flags);

/* Debug: copy an intermediate device buffer of the last ORB run (frame 0..max_batch-1) to the
 * host.  what: 0 pyramid, 1 blurred pyramid (both level-major, unpadded), 2 FAST per-cell
 * counts (int), 3 FAST candidate keys (packed u32), 4 octree output keys (packed u32),
 * 5 octree per-level counts (int), 6 device error flags (int).  Returns bytes written or <0. */
long mmt_debug_fetch(mmt_ctx* ctx, int what, int frame, void* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* MMT_H */
