/*
 * oracle/orb_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the HIP path in slam_framework_amd/. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product library
 * (libslamgpu.so) never links or calls anything in here.
 *
 * What it restates (every function cites the reference file:line it follows, paths relative
 * to the reference repository root):
 *   - Optimizer::PoseOptimization (src/optimizer/optimizer.cpp:209-411, on g2o): pose_oracle.c
 *   - Optimizer::LocalBundleAdjustment (optimizer.cpp:413-716, on g2o): ba_oracle.c
 *   - ORBextractor (src/orb_features/orb_extractor.cpp): ctor tables, ComputePyramid,
 *     ComputeKeyPointsOctTree (cell FAST + threshold fallback), DistributeOctTree,
 *     IC_Angle / computeOrientation, GaussianBlur + computeOrbDescriptor, Compute.
 *   - Frame::ComputeStereoMatches, AssignFeaturesToGrid, GetFeaturesInArea (src/data/frame.cpp).
 *   - OrbMatcher::DescriptorDistance and both per-frame SearchByProjection overloads
 *     (src/orb_features/orb_matcher.cpp).
 *   - The OpenCV 3.3.1 primitives those call (resize INTER_LINEAR 8U, GaussianBlur 7x7 8U,
 *     FAST_t<16> + cornerScore<16>, fastAtan2, cvRound) and glibc 2.35's x86-64 FMA sinf/cosf
 *     (the reference's `cos(float)`/`sin(float)` resolve to them, orb_extractor.cpp:54).
 *
 * PARITY STATUS: "parity unpinned" against the reference binary. The reference cannot be built
 * in this image (it needs OpenCV 3.x and Eigen3, neither present) and it ships no tests, golden
 * vectors or fixtures for this path. What IS pinned:
 *   - oc_sinf/oc_cosf are checked bit-exactly against this host's glibc 2.35 libm (FMA ifunc
 *     variant) -- tests/test_oracle_math.py and oracle/check_sincosf.c;
 *   - the ctor tables (level sizes, per-level budgets, umax) against SURVEY.md section 8;
 *   - FAST against a brute-force definition of the 9-of-16 segment test;
 *   - the Release-build (-O3 -march=native, GCC fp-contract=fast) FMA association of the
 *     reference's own float expressions, read from g++ 11 disassembly.
 * OpenCV-primitive semantics are the declared OpenCV 3.3.1 non-IPP paths.
 */
#ifndef SLAMGPU_ORB_ORACLE_H_
#define SLAMGPU_ORB_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OC_MAX_LEVELS 32

/* Byte-identical to cv::KeyPoint (28 bytes). */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} oc_keypoint;

/* ORBextractor constructor arguments (orb_extractor.h:35-39). */
typedef struct {
  int nfeatures;
  float scale_factor;
  int nlevels;
  int ini_th_fast;
  int min_th_fast;
} oc_orb_params;

/* Everything the ORBextractor ctor precomputes (orb_extractor.cpp:351-411). */
typedef struct {
  int nfeatures, nlevels, ini_th_fast, min_th_fast;
  double scale_factor; /* the member is a double (orb_extractor.h:80) */
  float scale[OC_MAX_LEVELS], inv_scale[OC_MAX_LEVELS];
  float sigma2[OC_MAX_LEVELS], inv_sigma2[OC_MAX_LEVELS];
  int features_per_level[OC_MAX_LEVELS];
  int umax[16];
} oc_orb_tables;

/* Image pyramid: level l is a w[l] x h[l] u8 image with row pitch step[l] (no border). */
typedef struct {
  int nlevels;
  int w[OC_MAX_LEVELS], h[OC_MAX_LEVELS];
  size_t step[OC_MAX_LEVELS];
  uint8_t* data[OC_MAX_LEVELS];
} oc_pyramid;

/* ---- OpenCV / glibc primitive semantics ------------------------------------------------- */
int oc_cv_round(float v);                              /* cvRound(float): half-to-even      */
float oc_fast_atan2(float y, float x);                 /* cv::fastAtan2, degrees [0,360)    */
float oc_sinf(float x);                                /* glibc 2.35 __sinf_fma             */
float oc_cosf(float x);                                /* glibc 2.35 __cosf_fma             */
float oc_logf(float x);                                /* glibc 2.35 __logf_fma             */
void oc_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t sstep, uint8_t* dst, int dw,
                         int dh, size_t dstep);
void oc_gaussian_blur7_u8(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst,
                          size_t dstep);
/* cv::FAST(img, kps, threshold, nonmax) on a w x h view; returns #kps (<= cap written). */
int oc_fast16(const uint8_t* img, int w, int h, size_t step, int threshold, int nonmax,
              oc_keypoint* out, int cap);

/* ---- ORBextractor ----------------------------------------------------------------------- */
void oc_orb_init(oc_orb_tables* t, const oc_orb_params* p);
void oc_level_size(const oc_orb_tables* t, int cols, int rows, int level, int* w, int* h);
int oc_pyramid_alloc(oc_pyramid* p, const oc_orb_tables* t, int cols, int rows);
void oc_pyramid_free(oc_pyramid* p);
void oc_compute_pyramid(const oc_orb_tables* t, const uint8_t* img, size_t step, oc_pyramid* p);
/* Cell FAST for one level: candidates in octree coordinates (level coords - minBorder). */
int oc_level_candidates(const oc_orb_tables* t, const oc_pyramid* p, int level,
                        oc_keypoint* out, int cap);
/* DistributeOctTree; returns #kept (<= cap written), list order. */
int oc_distribute_octree(const oc_keypoint* keys, int n, int minX, int maxX, int minY, int maxY,
                         int N, oc_keypoint* out, int cap);
float oc_ic_angle(const uint8_t* img, size_t step, float x, float y, const int* umax);
void oc_orb_descriptor(const oc_keypoint* kp, const uint8_t* blurred, size_t step,
                       uint8_t desc[32]);
/* Full ORBextractor::Compute. Returns #keypoints (or -needed if cap too small). If pyr is
 * non-NULL it must be allocated with oc_pyramid_alloc and receives the level images. */
int oc_orb_extract(const oc_orb_tables* t, const uint8_t* img, int rows, int cols, size_t step,
                   oc_keypoint* kps, uint8_t* desc, int cap, oc_pyramid* pyr);

/* ---- Matching ---------------------------------------------------------------------------- */
int oc_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Frame::ComputeStereoMatches. Outputs u_right[nl], depth[nl] (-1 = none) and, if non-NULL,
 * sad_best[nl] (the SAD score used by the median filter, -1 if no match). */
void oc_stereo_match(const oc_orb_tables* t, const oc_keypoint* kl, const uint8_t* dl, int nl,
                     const oc_keypoint* kr, const uint8_t* dr, int nr, const oc_pyramid* pl,
                     const oc_pyramid* pr, float fx, float bf, float* u_right, float* depth,
                     int* sad_best);

/* Frame image bounds and 64x48 grid (frame.cpp:211-248, 339-346, 678-703). */
typedef struct {
  float min_x, max_x, min_y, max_y;
  float cell_w, cell_h; /* grid_element_width_/height_ */
} oc_grid_geom;
void oc_grid_geom_init(oc_grid_geom* g, int cols, int rows);
/* Frame::ComputeImageBounds (frame.cpp:644-675) with DistCoef dist[ndist] (ndist 4 or 5): the
 * undistorted image corners when dist[0] != 0, else 0..cols x 0..rows; then the grid cell size. */
void oc_grid_geom_init_dist(oc_grid_geom* g, int cols, int rows, const float cam[4],
                            const float* dist, int ndist);
/* cv::undistortPoints(src, dst, K, D, noArray(), K) on n CV_32FC2 points (OpenCV 3.3.1
 * cvUndistortPoints); cam = fx, fy, cx, cy (f32 K), dist = k1 k2 p1 p2 [k3]. In place allowed. */
void oc_undistort_points(const float cam[4], const float* dist, int ndist, const float* xy_in,
                         float* xy_out, int n);
/* Frame::UndistortKeyPoints (frame.cpp:614-641): copies when dist[0] == 0, else undistorts pt. */
void oc_undistort_keypoints(const float cam[4], const float* dist, int ndist,
                            const oc_keypoint* in, oc_keypoint* out, int n);
/* Frame::GetFeaturesInArea; returns count (<= cap written), reference order. */
int oc_features_in_area(const oc_grid_geom* g, const oc_keypoint* kps, int n, float x, float y,
                        float r, int min_level, int max_level, int* out, int cap);

/* Map-point state shared by the two SearchByProjection restatements. mp ids index mp_nobs. */
typedef struct {
  const oc_keypoint* kps;  /* undistorted keypoints (== keypoints, k1 = 0) */
  const uint8_t* desc;     /* n x 32 */
  const float* u_right;    /* StereoCoordRight */
  int n;
  int* map_point;          /* in/out: mp id per keypoint or -1 (Frame::map_points_) */
} oc_frame_view;

/* OrbMatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (orb_matcher.cpp:1312-1453).
 * Last frame: its keypoints, map point ids and outlier flags. Map points: world xyz (3 floats
 * each), descriptors (32 B each), NumObservations. Pose: current Rcw (row-major 3x3), tcw,
 * tlc_z (z of the current camera centre in the last camera frame), baseline. */
int oc_search_by_projection_frame(const oc_grid_geom* g, const oc_orb_tables* t,
                                  oc_frame_view* cur, const oc_keypoint* last_kps,
                                  const int* last_mp, const uint8_t* last_outlier, int n_last,
                                  const float* mp_xyz, const uint8_t* mp_desc,
                                  const int* mp_nobs, const float* Rcw, const float* tcw,
                                  float tlc_z, float baseline, float fx, float fy, float cx,
                                  float cy, float bf, float th, int mono, int check_ori);

/* OrbMatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) (orb_matcher.cpp:13-103).
 * Query q is map point id q. in_view/is_bad/level/view_cos/proj_{x,y,xr} are its track_* data. */
int oc_search_by_projection_mps(const oc_grid_geom* g, const oc_orb_tables* t,
                                oc_frame_view* cur, int n_mp, const uint8_t* in_view,
                                const uint8_t* is_bad, const int* level, const float* view_cos,
                                const float* proj_x, const float* proj_y, const float* proj_xr,
                                const uint8_t* mp_desc, const int* mp_nobs, float nnratio,
                                int th);

/* ---- Optimizer::PoseOptimization (pose_oracle.c) --------------------------------------------- */
typedef struct {
  float xw[3];    /* map point world position (MapPoint::GetWorldPos, f32)            */
  float u, v;     /* undistorted keypoint                                             */
  float ur;       /* right coordinate (Frame::StereoCoordRight); < 0 -> monocular edge */
  int32_t octave; /* keypoint octave -> information = InvLevelSigma2[octave] * I      */
} oc_pose_edge;

/* Optimizer::PoseOptimization (optimizer.cpp:209-411). cam = fx, fy, cx, cy, bf (Frame's f32);
 * Tcw 4x4 row-major f32 in/out; outlier[n] out; returns #initial - #bad (0 if < 3 edges).
 * *lm_iterations (optional) counts g2o LM iterations over the 4 rounds. */
int oc_pose_optimization(const float cam[5], const float* inv_sigma2, const oc_pose_edge* edges,
                         int n, float Tcw[16], uint8_t* outlier, int* lm_iterations);
void oc_se3_exp(const double u[6], double R[9], double t[3]);
double oc_pose_edge_eval(const float cam[5], const double R[9], const double t[3],
                         const oc_pose_edge* e, float inv_sigma2, double err[3], double J[18]);

/* ---- Optimizer::LocalBundleAdjustment (ba_oracle.c) -------------------------------------- */
/* One observation of a local map point: keyframe index, undistorted keypoint, right coordinate
 * (< 0 monocular), octave. Observations are grouped by point (point_obs_start, CSR). */
typedef struct {
  int32_t keyframe;
  float u, v, ur;
  int32_t octave;
} oc_ba_obs;
/* kf_mode: 0 local (optimised, written back), 1 local but fixed (keyframe id 0; written back),
 * 2 fixed camera (neither). erase[e]: the reference's vToErase membership of observation e. */
int oc_local_bundle_adjustment(const float cam[5], const float* inv_sigma2, float* kf_Tcw,
                               const uint8_t* kf_mode, int n_kf, float* points, int n_points,
                               const int32_t* point_obs_start, const oc_ba_obs* obs,
                               uint8_t* erase, int* lm_iterations);
/* The same with the reference's stop_flag raised after `stop_after` polls of it (every
 * terminate() check of g2o and the reference counts one; < 0: never). */
int oc_local_bundle_adjustment_stop(const float cam[5], const float* inv_sigma2, float* kf_Tcw,
                                    const uint8_t* kf_mode, int n_kf, float* points, int n_points,
                                    const int32_t* point_obs_start, const oc_ba_obs* obs,
                                    int stop_after, uint8_t* erase, int* lm_iterations);
int oc_global_bundle_adjustment_stop(const float cam[5], const float* inv_sigma2, float* kf_Tcw,
                                     const uint8_t* kf_mode, int n_kf, float* points,
                                     int n_points, const int32_t* point_obs_start,
                                     const oc_ba_obs* obs, int n_iterations, int robust,
                                     int stop_after, int* lm_iterations);
double oc_ba_linearize(const float cam[5], const float* inv_sigma2, const float* kf_Tcw,
                       const uint8_t* kf_mode, int n_kf, const float* points, int n_points,
                       const int32_t* point_obs_start, const oc_ba_obs* obs, double* chi2,
                       double* hpl, double* hll, double* bl, double* hpp, double* bp);
double oc_ba_edge_eval(const float cam[5], const double R[9], const double t[3], const double X[3],
                       const oc_ba_obs* o, float inv_sigma2, double err[3], double Jl[9],
                       double Jp[18]);

/* ---- DBoW2 vocabulary, SearchByBoW, ComputeDistinctiveDescriptors, cvtColor (bow_oracle.c) - */
/* The arrays TemplatedVocabulary::loadFromTextFile builds (TemplatedVocabulary.h:1335-1421):
 * node 0 = root; node i >= 1 has parent[i] < i, the file's leaf flag, a descriptor and a weight.
 * scoring / weighting are DBoW2's ScoringType / WeightingType values. */
typedef struct {
  int k, L, scoring, weighting;
  int n_nodes;
  const int32_t* parent;
  const uint8_t* leaf_flag;
  const uint8_t* desc; /* [n_nodes][32] */
  const double* weight;
} oc_vocab_arrays;
typedef struct oc_vocab oc_vocab;
oc_vocab* oc_vocab_build(const oc_vocab_arrays* a);
void oc_vocab_free(oc_vocab* v);
void oc_vocab_transform_one(const oc_vocab* v, const uint8_t d[32], int levelsup, uint32_t* word,
                            double* weight, uint32_t* nid, uint32_t* leaf);
int oc_bow_transform(const oc_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* words,
                     double* values, int* n_words, uint32_t* nodes, int32_t* node_start,
                     uint32_t* node_feats, int* n_nodes);
int oc_search_by_bow(const uint8_t* a_desc, const oc_keypoint* a_kps, const uint8_t* a_valid,
                     int n_a, const uint32_t* a_nodes, const int32_t* a_start,
                     const uint32_t* a_feats, int a_nn, const uint8_t* b_desc,
                     const oc_keypoint* b_kps, const uint8_t* b_valid, int n_b,
                     const uint32_t* b_nodes, const int32_t* b_start, const uint32_t* b_feats,
                     int b_nn, int strict_lt, float nnratio, int check_ori, int32_t* match_a);
void oc_distinctive_descriptors(const uint8_t* desc, const int32_t* start, int n_points,
                                int32_t* best);
void oc_cvt_gray(const uint8_t* src, size_t sstep, int cn, int rgb, int cols, int rows,
                 uint8_t* dst, size_t dstep);

/* ---- keyframe-rate matchers (kfmatch_oracle.c) ---------------------------------------- */
typedef struct {
  float xyz[3];      /* GetWorldPos()                                              */
  float normal[3];   /* GetNormal()                                                */
  float min_dist;    /* min_dist_ (GetMinDistanceInvariance() = 0.8f * min_dist_)  */
  float max_dist;    /* max_dist_ (GetMaxDistanceInvariance() = 1.2f * max_dist_)  */
  int32_t skip;      /* !pMP || isBad() || IsInKeyFrame(pKF)                       */
  int32_t pad[3];
  uint8_t desc[32];  /* GetDescriptor()                                            */
} oc_fuse_point;     /* 80 B, == slamgpu_fuse_point */

int oc_check_dist_epipolar(const oc_keypoint* kp1, const oc_keypoint* kp2, const float* F,
                           const float* sigma2);
void oc_epipole(const float* C1w, const float* T2w, float fx, float fy, float cx, float cy,
                float* ex, float* ey);
int oc_search_for_triangulation(
    const oc_keypoint* k1, const uint8_t* d1, const float* ur1, const uint8_t* mp1, int n1,
    const uint32_t* nodes1, const int32_t* start1, const uint32_t* feats1, int nn1,
    const oc_keypoint* k2, const uint8_t* d2, const float* ur2, const uint8_t* mp2,
    const uint32_t* nodes2, const int32_t* start2, const uint32_t* feats2, int nn2,
    const float* C1w, const float* T2w, float fx, float fy, float cx, float cy,
    const float* scale, const float* sigma2, const float* F12, int only_stereo, int check_ori,
    int32_t* match12);
int oc_predict_scale(float max_dist, float dist, float log_scale_factor, int nlevels);
int oc_fuse(const oc_keypoint* kps, const uint8_t* desc, const float* ur, int n,
            const oc_grid_geom* g, const float* Rcw, const float* tcw, const float* Ow, float fx,
            float fy, float cx, float cy, float bf, const float* scale, const float* inv_sigma2,
            int nlevels, float log_scale_factor, const oc_fuse_point* pts, int n_pts, float th,
            int32_t* best_idx, int32_t* best_dist);

/* ---- OptimizeSim3 (sim3_oracle.c) ------------------------------------------------------ */
/* One correspondence of OptimizeSim3 (optimizer.cpp:1020-1096): the two map points in their
 * keyframes' camera frames (f32, as cv::Mat R*X + t gives them), the undistorted keypoints and
 * their octaves. 48 B, == slamgpu_sim3_match. */
typedef struct {
  float x1c[3], x2c[3];
  float u1, v1, u2, v2;
  int32_t octave1, octave2;
} oc_sim3_match;
/* S12: g2o::Sim3 as (qx, qy, qz, qw, tx, ty, tz, s); returns nIn (0 on the early return, S12
 * then untouched); inlier[i] = 0 where the reference nulls vpMatches1. */
int oc_optimize_sim3(const float K1[4], const float K2[4], const float* inv_sigma2_1,
                     const float* inv_sigma2_2, int nlevels, const oc_sim3_match* m, int n,
                     float th2, int fix_scale, double S12[8], uint8_t* inlier, int* lm_iterations);
void oc_sim3_exp(const double u[7], double out[8]);
void oc_sim3_log(const double in[8], double u[7]);
void oc_sim3_mul(const double a[8], const double b[8], double out[8]);
void oc_sim3_inverse(const double a[8], double out[8]);
void oc_sim3_map(const double a[8], const double x[3], double o[3]);
void oc_sim3_pair_eval(const float K1[4], const float K2[4], const oc_sim3_match* m,
                       const double S12[8], int fix_scale, double e[4], double J[28]);

/* ---- OptimizeEssentialGraph (eg_oracle.c) ---------------------------------------------- */
/* One EdgeSim3 of the essential graph (optimizer.cpp:784-909): _vertices[0] = i, [1] = j,
 * measurement Sji (qx, qy, qz, qw, t, s). 80 B, == slamgpu_sim3_edge. */
typedef struct {
  int32_t i, j;
  int32_t pad[2];
  double Sji[8];
} oc_sim3_edge;
int oc_optimize_essential_graph(int n, double* Scw, const uint8_t* fixed, const oc_sim3_edge* edges,
                                int n_edges, int fix_scale, int n_iterations, float* Tcw_out,
                                int* lm_iterations);
void oc_correct_points_sim3(const double* Scw_before, const double* Scw_after, const int32_t* ref,
                            float* points, int n_points);
double oc_sim3_edge_eval(const double Si[8], const double Sj[8], const double Sji[8], int fix_scale,
                         double e[7], double Ji[49], double Jj[49]);

#ifdef __cplusplus
}
#endif

#endif /* SLAMGPU_ORB_ORACLE_H_ */
