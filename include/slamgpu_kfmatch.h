/*
 * slamgpu_kfmatch.h -- C ABI of the keyframe-rate matchers the LocalMapper runs before
 * LocalBundleAdjustment (libslamgpu.so). SURVEY.md section 8(f) row 3, drop-in for (paths
 * relative to the reference repository root):
 *   OrbMatcher::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 *     src/orb_features/orb_matcher.cpp:634-802 (+ CheckDistEpipolarLine :114-131);
 *     caller LocalMapper::CreateNewMapPoints (src/core/local_mapper.cpp)
 *   OrbMatcher::Fuse(pKF, vpMapPoints, th)  orb_matcher.cpp:804-954 (+ MapPoint::PredictScale
 *     src/data/map_point.cpp:366-381, KeyFrame::GetFeaturesInArea keyframe.cpp:442-476);
 *     caller LocalMapper::SearchInNeighbors
 * Conventions as slamgpu.h: POD types, caller-owned buffers, 0 or a negative SLAMGPU_E* code
 * with the message in slamgpu_kfmatch_last_error() (per thread). The synchronous calls stage
 * through per-thread device buffers; the *_device calls take device pointers and a hipStream_t,
 * never allocate and return without synchronising.
 */
#ifndef SLAMGPU_KFMATCH_H_
#define SLAMGPU_KFMATCH_H_

#include <stddef.h>
#include <stdint.h>

#include "slamgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SLAMGPU_KF_MAX_FEATURES 4096

/* The per-level tables a KeyFrame copies from its extractor: log_scale_factor (float
 * log(scaleFactor)), scale_factors, level_sigma_sq, inv_level_sigma_sq (keyframe.h:167-170). */
typedef struct {
  int32_t nlevels;
  float log_scale_factor;
  float scale[32];
  float sigma2[32];
  float inv_sigma2[32];
} slamgpu_levels;

/* KeyFrame::min_x_ .. max_y_ (ints, keyframe.cpp:14-15) and grid_element_width_ / _height_ of
 * the 64 x 48 keypoint grid (Frame::AssignFeaturesToGrid frame.cpp:234-248). */
typedef struct {
  float min_x, max_x, min_y, max_y;
  float cell_w, cell_h;
} slamgpu_kf_grid;

/* One keyframe as the matchers read it: host pointers in the synchronous calls, device pointers
 * in the *_device calls. 128 bytes. */
typedef struct {
  const slamgpu_keypoint* kps; /* [n] undistorted_keypoints                                */
  const uint8_t* desc;         /* [n][32] descriptors                                       */
  const float* u_right;        /* [n] right_coords (< 0: monocular)                         */
  const uint8_t* has_mp;       /* [n] GetMapPoint(i) != NULL (SearchForTriangulation)       */
  const uint32_t* nodes;       /* FeatureVector: [n_nodes] ascending (SearchForTriangulation) */
  const int32_t* node_start;   /* [n_nodes + 1]                                             */
  const uint32_t* node_feats;  /* [node_start[n_nodes]]                                     */
  int32_t n, n_nodes;
  float Rcw[9];                /* GetRotation(), row-major                                  */
  float tcw[3];                /* GetTranslation()                                          */
  float Ow[3];                 /* GetCameraCenter()                                         */
  float pad;
} slamgpu_kf;

/* ---- SearchForTriangulation --------------------------------------------------------------- */
/* match12[i] = vMatches12[i] (the pKF2 keypoint matched to pKF1 keypoint i, or -1); the
 * reference's vMatchedPairs = the (i, match12[i]) with match12[i] >= 0, ascending i.
 * cam = pKF2's fx, fy, cx, cy (bf unused); lv = pKF2's level tables; F12 row-major. */
int slamgpu_search_for_triangulation(const slamgpu_kf* kf1, const slamgpu_kf* kf2,
                                     const float* F12, const slamgpu_camera* cam,
                                     const slamgpu_levels* lv, int only_stereo, int check_ori,
                                     int32_t* match12, int* nmatches);

/* A keyframe pair of a batched call: d_kfs[kf1] against d_kfs[kf2]. 48 bytes. */
typedef struct {
  int32_t kf1, kf2;
  float F12[9];
  int32_t only_stereo;
} slamgpu_tri_pair;

/* Pair p writes d_match12 + p * match_stride and d_nmatches[p] (-1 if a keyframe exceeds
 * SLAMGPU_KF_MAX_FEATURES, or its FeatureVector names a feature >= n, or a candidate keypoint's
 * octave is outside [0, nlevels): such a pair's match row is left partly written). */
int slamgpu_search_for_triangulation_device(const slamgpu_kf* d_kfs,
                                            const slamgpu_tri_pair* d_pairs, int n_pairs,
                                            const slamgpu_camera* cam, const slamgpu_levels* lv,
                                            int check_ori, int32_t* d_match12,
                                            int64_t match_stride, int32_t* d_nmatches,
                                            void* stream);

/* ---- Fuse ------------------------------------------------------------------------------------ */
/* A map point offered to Fuse(pKF, vpMapPoints, th). 80 bytes. */
typedef struct {
  float xyz[3];     /* GetWorldPos()                                                    */
  float normal[3];  /* GetNormal()                                                      */
  float min_dist;   /* min_dist_ (GetMinDistanceInvariance() = 0.8f * min_dist_)        */
  float max_dist;   /* max_dist_ (GetMaxDistanceInvariance() = 1.2f * max_dist_)        */
  int32_t skip;     /* !pMP || isBad() || IsInKeyFrame(pKF) when the call starts         */
  int32_t pad[3];
  uint8_t desc[32]; /* GetDescriptor()                                                  */
} slamgpu_fuse_point;

/* The candidate search of Fuse (:821-928) for every point: best_idx[i] = the keypoint point i
 * fuses into (bestDist <= TH_LOW), else -1; best_dist[i] = bestDist (256 if no candidate).
 * *nfused = #(best_idx >= 0). The adapter then walks the points in order and, re-checking
 * isBad() / IsInKeyFrame(pKF) (earlier Replace calls can change them), does the reference's
 * Replace / AddObservation (:931-949). cam = pKF's fx, fy, cx, cy, mbf. */
int slamgpu_fuse(const slamgpu_kf* kf, const slamgpu_fuse_point* pts, int n_pts, float th,
                 const slamgpu_camera* cam, const slamgpu_levels* lv, const slamgpu_kf_grid* grid,
                 int32_t* best_idx, int32_t* best_dist, int* nfused);

/* Batched: point i is fused into d_kfs[d_point_kf[i]]. */
int slamgpu_fuse_device(const slamgpu_kf* d_kfs, const slamgpu_fuse_point* d_pts,
                        const int32_t* d_point_kf, int n_pts, float th,
                        const slamgpu_camera* cam, const slamgpu_levels* lv,
                        const slamgpu_kf_grid* grid, int32_t* d_best_idx, int32_t* d_best_dist,
                        void* stream);

const char* slamgpu_kfmatch_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_KFMATCH_H_ */
