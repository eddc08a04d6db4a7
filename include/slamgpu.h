/*
 * slamgpu.h -- C ABI of the MI355X ORB front-end (libslamgpu.so).
 *
 * Drop-in boundary for the reference's hot path (ThorsteinnJonsson/SLAM_framework):
 *   ORBextractor            src/orb_features/orb_extractor.h:25-93
 *   Frame stereo matching   src/data/frame.cpp:406-577 (ComputeStereoMatches), grid :234-248
 *   OrbMatcher              src/orb_features/orb_matcher.h:14-119 (DescriptorDistance and the
 *                           two per-frame SearchByProjection overloads)
 * POD types and caller-owned buffers only; every function returns 0 on success or a negative
 * SLAMGPU_E* code, with a message in slamgpu_last_error(). One context owns one HIP device,
 * one stream and all device workspaces; functions on different contexts may run concurrently
 * from different threads, a single context is not re-entrant (like ORBextractor, whose
 * mvImagePyramid is mutable state).
 *
 * Two families of entry points:
 *   host-buffer calls  -- synchronous, exactly the reference call sites' data flow
 *                         (ORBextractor::Compute, GetImagePyramid, the Frame ctor's stereo
 *                         matching, SearchByProjection on one frame);
 *   *_device calls     -- asynchronous on the caller's HIP stream, inputs already in HBM,
 *                         batched over many frames (the throughput path bench.py measures).
 */
#ifndef SLAMGPU_H_
#define SLAMGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLAMGPU_OK 0
#define SLAMGPU_EINVAL -1   /* bad argument / unsupported configuration */
#define SLAMGPU_EHIP -2     /* HIP runtime error */
#define SLAMGPU_ECAP -3     /* caller buffer too small (see n_out) */
#define SLAMGPU_EDEVICE -4  /* a kernel reported a capacity overflow (see slamgpu_last_error) */

typedef struct slamgpu_ctx slamgpu_ctx;

/* Byte-identical to cv::KeyPoint (pt.x, pt.y, size, angle, response, octave, class_id). */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} slamgpu_keypoint;

/* ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)  orb_extractor.h:35-39 */
typedef struct {
  int nfeatures;
  float scale_factor;
  int nlevels;
  int ini_th_fast;
  int min_th_fast;
} slamgpu_orb_params;

/* Pinhole stereo camera as the Frame sees it (tracker.cpp:29-70): K entries and bf. Image
 * bounds are 0..cols x 0..rows, or the undistorted corners once slamgpu_set_distortion gave a
 * DistCoef with k1 != 0 (Frame::ComputeImageBounds frame.cpp:644-675). */
typedef struct {
  float fx, fy, cx, cy, bf;
} slamgpu_camera;

/* ---- lifecycle ---------------------------------------------------------------------------- */
/* Replaces: ORBextractor::ORBextractor (orb_extractor.cpp:351-411) for images of cols x rows,
 * batched up to max_frames stereo pairs (2 * max_frames images). Returns 0 and *out, or a
 * negative code with *out = NULL (nothing to destroy; the reason: slamgpu_last_error(NULL)).
 * Limits: at most 4096 keypoints per image (slamgpu_kp_capacity ~ nfeatures + 3 * nlevels: on
 * 1241 x 376 nfeatures up to ~4070, which covers the monocular initialiser's 2 * nFeatures
 * extractor of tracker.cpp:84-89) and <= 1024 octree nodes per level. */
int slamgpu_create(int device, const slamgpu_orb_params* params, int cols, int rows,
                   int max_frames, slamgpu_ctx** out);
void slamgpu_destroy(slamgpu_ctx* ctx);
/* The context's last error; with ctx == NULL, why the last slamgpu_create on this thread failed. */
const char* slamgpu_last_error(const slamgpu_ctx* ctx);
/* Max keypoints one image can produce (sum over levels of the octree list bound). */
int slamgpu_kp_capacity(const slamgpu_ctx* ctx);
/* ORBextractor getters GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares (orb_extractor.h:50-60) plus mnFeaturesPerLevel. Each array has
 * nlevels entries; any pointer may be NULL. */
int slamgpu_scale_tables(const slamgpu_ctx* ctx, float* scale, float* inv_scale, float* sigma2,
                         float* inv_sigma2, int* features_per_level);
/* The same tables from the ctor arguments alone (orb_extractor.cpp:351-387: they do not depend on
 * the image size), with no context and no device: what ORBextractor's getters return before the
 * first Compute. Returns SLAMGPU_EINVAL for nlevels outside [1, 12] or scale_factor <= 1. */
int slamgpu_orb_scale_tables(const slamgpu_orb_params* params, float* scale, float* inv_scale,
                             float* sigma2, float* inv_sigma2, int* features_per_level);

/* ---- ORBextractor ------------------------------------------------------------------------- */
/* Replaces: ORBextractor::Compute(image, mask, keypoints, descriptors)  orb_extractor.cpp:985.
 * img: rows x cols u8, `step` bytes per row. Writes n keypoints and n x 32 descriptor bytes
 * (row i = keypoint i) in the reference's order. cap too small -> SLAMGPU_ECAP, *n_out = n. */
int slamgpu_extract(slamgpu_ctx* ctx, const uint8_t* img, size_t step, slamgpu_keypoint* kps,
                    uint8_t* desc, int cap, int* n_out);
/* Replaces: ORBextractor::GetImagePyramid()[level] (orb_extractor.h:62) for image `img` of the
 * last extraction (slamgpu_extract: img 0; frame calls: 2f = left, 2f+1 = right). */
int slamgpu_get_pyramid_level(slamgpu_ctx* ctx, int img, int level, uint8_t* dst,
                              size_t dst_step, int* w_out, int* h_out);

/* Diagnostics for stage-level parity tests: packed keys (x_rel | y_rel << 12 | score << 23,
 * coordinates relative to minBorder = 16) of image `img`, level `level` of the last extraction.
 * stage 0: FAST survivors of ComputeKeyPointsOctTree's cell loop in vToDistributeKeys order
 * (orb_extractor.cpp:730-770); stage 1: DistributeOctTree output in list order (:480-704). */
int slamgpu_debug_level_keys(slamgpu_ctx* ctx, int img, int level, int stage, uint32_t* keys,
                             int cap, int* n_out);

/* ---- Frame: extraction of both views + ComputeStereoMatches ------------------------------- */
/* Replaces the stereo Frame ctor's hot part (frame.cpp:61-111): ExtractORB on left and right,
 * then ComputeStereoMatches (:406-577). Results stay in the context as frame 0 (download with
 * slamgpu_download_*). */
int slamgpu_frame_stereo(slamgpu_ctx* ctx, const uint8_t* left, const uint8_t* right,
                         size_t step, const slamgpu_camera* cam);

/* Batched device path: n_frames stereo pairs already in device memory. Left view of frame f at
 * d_left + f * frame_stride, right view at d_right + f * frame_stride, `pitch` bytes per row.
 * Enqueues extraction of all 2n images, stereo matching and the 64x48 grid of every left view
 * on `stream` (a hipStream_t; NULL = the context's stream). Returns without synchronising. */
int slamgpu_frontend_device(slamgpu_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right,
                            size_t frame_stride, size_t pitch, int n_frames,
                            const slamgpu_camera* cam, void* stream);
/* Waits for the context's work on `stream` and reports device-side capacity errors. */
int slamgpu_sync(slamgpu_ctx* ctx, void* stream);

/* Results of the last frontend/frame call. img = 2f (left) / 2f+1 (right). */
int slamgpu_download_keypoints(slamgpu_ctx* ctx, int img, slamgpu_keypoint* kps, uint8_t* desc,
                               int cap, int* n_out);
/* StereoCoordRight / StereoDepth of frame f's left keypoints (-1 = no match). */
int slamgpu_download_stereo(slamgpu_ctx* ctx, int frame, float* u_right, float* depth, int cap,
                            int* n_out);

/* Device views of the results, for chaining further device work without copies. */
typedef struct {
  const slamgpu_keypoint* kps; /* [2 * max_frames][kp_cap]     */
  const uint8_t* desc;         /* [2 * max_frames][kp_cap][32] */
  const int* nkps;             /* [2 * max_frames]             */
  const float* u_right;        /* [max_frames][kp_cap]          */
  const float* depth;          /* [max_frames][kp_cap]          */
  int kp_cap;
  const slamgpu_keypoint* kps_un; /* [2 * max_frames][kp_cap]: undistorted left views (= kps
                                     when k1 == 0; right-view slots unused)                   */
} slamgpu_device_view;
int slamgpu_device_results(const slamgpu_ctx* ctx, slamgpu_device_view* out);

/* ---- Frame: distortion (Frame::UndistortKeyPoints / ComputeImageBounds) ------------------ */
/* Sets the Frame's DistCoef (tracker.cpp:41-51: k1 k2 p1 p2 [k3]; n = 4 or 5, n = 0 clears).
 * With k1 != 0 every following frame call undistorts the left keypoints on the device after
 * ComputeStereoMatches (frame.cpp:96, :614-641), and the grid, the projection searches and
 * slamgpu_make_vo_queries_device read the undistorted keypoints (undistorted_keypoints_), the
 * image bounds are the undistorted corners. k1 == 0 is the reference's identity case. */
int slamgpu_set_distortion(slamgpu_ctx* ctx, const float* dist_coef, int n);
/* Replaces cv::undistortPoints(src, dst, K, DistCoef, noArray(), K) as the reference calls it
 * (frame.cpp:630, :659; OpenCV 3.3.1 semantics, undistort.h). Host, pure; n = 0: copy. */
int slamgpu_undistort_points(const slamgpu_camera* cam, const float* dist_coef, int n,
                             const float* xy_in, float* xy_out, int n_points);
/* Batched device Frame::UndistortKeyPoints: set f's d_counts[f * counts_stride] keypoints at
 * d_in + f * in_stride -> d_out + f * out_stride (pt undistorted, other fields copied; k1 == 0
 * copies). max_kps >= every count. Asynchronous on `stream`. */
int slamgpu_undistort_keypoints_device(const slamgpu_camera* cam, const float* dist_coef, int n,
                                       const slamgpu_keypoint* d_in, int64_t in_stride,
                                       const int* d_counts, int counts_stride,
                                       slamgpu_keypoint* d_out, int64_t out_stride, int n_sets,
                                       int max_kps, void* stream);
/* Frame f's undistorted left keypoints (GetUndistortedKeys) of the last frame/frontend call. */
int slamgpu_download_undistorted_keypoints(slamgpu_ctx* ctx, int frame, slamgpu_keypoint* kps,
                                           int cap, int* n_out);

/* Per-frame result record of the last frontend call, for gathering a frame-sharded job's
 * results to one rank (the stereo Frame ctor's outputs, frame.cpp:61-111 --
 * left/right keypoints and descriptors, Frame::ComputeStereoMatches' u_right/depth). Record
 * layout (kc = kp_cap; entries past nkps[v] are stale and must be ignored):
 *   [0, 56 kc)            slamgpu_keypoint kps[2][kc]   (left, right)
 *   [56 kc, 120 kc)       uint8_t desc[2][kc][32]
 *   [120 kc, 124 kc)      float u_right[kc]
 *   [124 kc, 128 kc)      float depth[kc]
 *   [128 kc, 128 kc + 8)  int32_t nkps[2]
 * padded to a multiple of 256 bytes (slamgpu_frame_record_bytes). */
size_t slamgpu_frame_record_bytes(const slamgpu_ctx* ctx);
/* Device-to-device copy of frames [first, first + n) of the last frontend call into n
 * consecutive records at d_dst, ordered on `stream` (NULL = the context's stream) after the
 * frontend's launches. Never allocates; graph-capturable. */
int slamgpu_pack_frame_records_device(slamgpu_ctx* ctx, int first, int n, void* d_dst,
                                      void* stream);

/* ---- OrbMatcher ---------------------------------------------------------------------------- */
/* Replaces: OrbMatcher::DescriptorDistance (orb_matcher.cpp:1630-1646). Host, pure. */
int slamgpu_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* A last-frame map point for SearchByProjection(CurrentFrame, LastFrame, th, bMono)
 * (orb_matcher.cpp:1312-1453). 64 bytes. */
typedef struct {
  float xyz[3];       /* MapPoint::GetWorldPos()                                    */
  float last_angle;   /* LastFrame.GetUndistortedKeys()[i].angle                    */
  int32_t last_octave;/* LastFrame.GetKeys()[i].octave                              */
  int32_t mp_id;      /* caller's identity of the map point, written into map_point */
  int32_t blocks;     /* MapPoint::NumObservations() > 0                            */
  int32_t pad;
  uint8_t desc[32];   /* MapPoint::GetDescriptor()                                  */
} slamgpu_f2f_query;

typedef struct {
  float Rcw[9];       /* CurrentFrame pose rotation, row major                     */
  float tcw[3];
  float tlc_z;        /* (Rlw * twc + tlw)(2): z of the current centre in the last frame */
  float baseline;     /* CurrentFrame.GetBaseline()                                */
  float th;           /* window factor (7 stereo, 14 on the retry, tracker.cpp:770-790) */
  int32_t mono;       /* bMono                                                     */
  int32_t check_ori;  /* OrbMatcher(nnratio, checkOri).mbCheckOrientation         */
  int32_t pad;
} slamgpu_f2f_pose;

/* Host call on frame `frame` of the last frontend/frame call (its left keypoints, descriptors,
 * stereo coordinates and grid). Only the non-outlier last-frame points that have a map point
 * are queries, in last-frame keypoint order. map_point[n] / blocked[n] are the current frame's
 * map point slots (in/out; blocked = the slot's map point has observations). */
int slamgpu_search_by_projection_frame(slamgpu_ctx* ctx, int frame,
                                       const slamgpu_f2f_query* queries, int n_queries,
                                       const slamgpu_f2f_pose* pose, int32_t* map_point,
                                       uint8_t* blocked, int n, int* nmatches);

/* A local map point for SearchByProjection(F, vpMapPoints, th) (orb_matcher.cpp:13-103) with
 * its Frame::IsInFrustum results (frame.cpp:277-337). 80 bytes. */
typedef struct {
  float proj_x, proj_y, proj_xr, view_cos; /* track_projected_x/_y/_x_right, track_view_cos */
  int32_t level;                           /* track_scale_level                             */
  int32_t in_view;                         /* track_is_in_view                              */
  int32_t is_bad;                          /* isBad()                                       */
  int32_t mp_id;
  int32_t blocks;                          /* NumObservations() > 0                         */
  int32_t pad[3];
  uint8_t desc[32];
} slamgpu_mps_query;

int slamgpu_search_by_projection_mps(slamgpu_ctx* ctx, int frame, const slamgpu_mps_query* queries,
                                     int n_queries, float nnratio, int th, int32_t* map_point,
                                     uint8_t* blocked, int n, int* nmatches);

/* Batched device versions over the frames of the last frontend call. Queries of frame f are
 * d_queries[d_q_start[f] .. d_q_start[f] + d_q_count[f]); max_queries >= every d_q_count[f];
 * total_queries >= every d_q_start[f] + d_q_count[f].
 * d_map_point / d_blocked: [n_frames][mp_stride] in/out; d_nmatches: [n_frames]. */
int slamgpu_search_by_projection_frame_device(slamgpu_ctx* ctx, const slamgpu_f2f_query* d_queries,
                                              int total_queries, const int* d_q_start, const int* d_q_count,
                                              int max_queries, const slamgpu_f2f_pose* d_poses,
                                              int32_t* d_map_point, uint8_t* d_blocked,
                                              int64_t mp_stride, int* d_nmatches, int n_frames,
                                              void* stream);
int slamgpu_search_by_projection_mps_device(slamgpu_ctx* ctx, const slamgpu_mps_query* d_queries,
                                            int total_queries, const int* d_q_start, const int* d_q_count,
                                            int max_queries, float nnratio, int th,
                                            int32_t* d_map_point, uint8_t* d_blocked,
                                            int64_t mp_stride, int* d_nmatches, int n_frames,
                                            void* stream);

/* Builds frame-to-frame queries on the device from the last frontend call: for frame f >= 1,
 * every left keypoint of frame f-1 with stereo depth becomes a map point at
 * Frame::UnprojectStereo(i) (frame.cpp:594-607) under d_poses[f-1] -- the visual-odometry points
 * of Tracker::UpdateLastFrame (tracker.cpp:695-753) with all stereo points kept. `blocks` sets
 * their NumObservations() > 0 flag. Frame f's queries go to d_queries[f * kp_cap ...]
 * (d_queries holds n_frames * kp_cap entries); frame 0 gets none. Feed the outputs to
 * slamgpu_search_by_projection_frame_device with total_queries = n_frames * kp_cap. */
int slamgpu_make_vo_queries_device(slamgpu_ctx* ctx, const slamgpu_f2f_pose* d_poses, int blocks,
                                   slamgpu_f2f_query* d_queries, int* d_q_start, int* d_q_count,
                                   int n_frames, void* stream);

/* ---- measurement ---------------------------------------------------------------------------- */
/* Brackets every launch of `kernel` ("*" = all kernels) with HIP events on its stream until
 * slamgpu_timing_stop; slamgpu_timing_read sums the recorded durations. Kernel names: pyr_down,
 * blur7, fast_cells, octree, orient_desc, stereo_rows, stereo_match, stereo_median, grid_build,
 * vo_queries, search_cand, search_resolve. */
int slamgpu_timing_start(slamgpu_ctx* ctx, const char* kernel, int max_launches);
/* Batches run level 0's FAST on a side stream beside the pyramid (the default, on = 1); on = 0
 * runs it after the pyramid on the call's stream, so that a timing pass sees each kernel alone.
 * (SLAMGPU_FORK=0 at context creation removes the side stream altogether.) */
int slamgpu_set_extract_fork(slamgpu_ctx* ctx, int on);
int slamgpu_timing_stop(slamgpu_ctx* ctx, void* stream);
int slamgpu_timing_read(slamgpu_ctx* ctx, const char* kernel, double* total_ms, int* launches);

/* Launches one empty kernel, `trace_marker_kernel`, with a 1 x `id` grid on `stream` (NULL =
 * the default stream): a mark a profiler's kernel trace shows in launch order. bench.py brackets
 * its timed region with ids 1 and 2 so that tools/stats_timed.py can average exactly the launches
 * the bench line's roofline times. */
int slamgpu_trace_marker(int id, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_H_ */
