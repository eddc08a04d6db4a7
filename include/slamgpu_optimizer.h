/*
 * slamgpu_optimizer.h -- C ABI of the MI355X motion-only / local bundle adjustment
 * (libslamgpu.so, same library as slamgpu.h).
 *
 * Drop-in boundary for the reference's Optimizer (src/optimizer/optimizer.h:13-50, a class of
 * static functions over g2o):
 *   slamgpu_pose_optimization         Optimizer::PoseOptimization(Frame&)  optimizer.cpp:209-411
 *   slamgpu_pose_optimization_device  the same, batched over frames, inputs resident in HBM
 *   slamgpu_local_bundle_adjustment   Optimizer::LocalBundleAdjustment     optimizer.cpp:413-716
 *   slamgpu_local_bundle_adjustment_device   the same, batched over independent problems
 *   slamgpu_global_bundle_adjustment  Optimizer::BundleAdjustment          optimizer.cpp:18-207
 *   slamgpu_optimize_sim3             Optimizer::OptimizeSim3              optimizer.cpp:962-1152
 *   slamgpu_optimize_sim3_device      the same, batched over loop candidates
 *   slamgpu_optimize_essential_graph  Optimizer::OptimizeEssentialGraph    optimizer.cpp:718-960
 * These calls hold no state, so they take no handle. Every function returns 0 or a negative
 * SLAMGPU_E* code (slamgpu.h) with a message in slamgpu_optimizer_last_error() (per thread).
 *
 * Arithmetic is FP64 on the device, with the reference's f32 inputs and f32 quirks (stereo
 * cam_project's float inverse depth, the f32 chi2 threshold tests, the f32 pose output); the
 * normal-equation sums are tree reductions, so results agree with the reference to rounding
 * (poses within 1e-5 relative), not bit for bit.
 */
#ifndef SLAMGPU_OPTIMIZER_H_
#define SLAMGPU_OPTIMIZER_H_

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "slamgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One correspondence of PoseOptimization (optimizer.cpp:239-309): the map point's world
 * position (MapPoint::GetWorldPos, f32), the undistorted keypoint (mvKeysUn[i].pt), its right
 * coordinate (mvuRight[i]; < 0 = monocular edge, otherwise stereo edge) and its octave, which
 * selects the information invSigma2 = mvInvLevelSigma2[octave]. 28 bytes. */
typedef struct {
  float xw[3];
  float u, v, ur;
  int32_t octave;
} slamgpu_pose_edge;

/* Largest edge count per frame the pose kernels take (frames carry <= nfeatures keypoints, so
 * nfeatures up to ~16k). Frames up to 4096 edges run with their edges in LDS; larger ones on an
 * 8-wave work-group reading them from L2. */
#define SLAMGPU_POSE_MAX_EDGES 16384
#define SLAMGPU_MAX_LEVELS 32

/* Replaces: int Optimizer::PoseOptimization(Frame* pFrame)  optimizer.cpp:209-411.
 * Tcw: the frame's pose (row-major 4x4 f32, Frame::mTcw), updated in place unless n < 3.
 * outlier[n]: Frame::mvbOutlier for the edges' keypoints, written for every edge.
 * inv_sigma2[nlevels]: Frame::mvInvLevelSigma2. *n_inliers: the reference's return value
 * (#initial correspondences - #bad in the last round; 0 when n < 3). Synchronous. */
int slamgpu_pose_optimization(const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
                              const slamgpu_pose_edge* edges, int n, float Tcw[16],
                              uint8_t* outlier, int* n_inliers);

/* Batched, asynchronous on `stream` (a hipStream_t; NULL = default stream), all pointers
 * device memory: frame f owns edges d_edges[d_edge_start[f] .. d_edge_start[f+1]), its pose
 * d_Tcw[16 f ...] (in/out), outlier flags at the edges' positions, d_n_inliers[f] (the
 * return value; -1 if the frame exceeds SLAMGPU_POSE_MAX_EDGES, pose then untouched) and, if
 * d_lm_iterations is not NULL, the Levenberg-Marquardt iterations it ran over its 4 rounds. */
int slamgpu_pose_optimization_device(const slamgpu_camera* cam, const float* inv_sigma2,
                                     int nlevels, const slamgpu_pose_edge* d_edges,
                                     const int32_t* d_edge_start, int n_frames, float* d_Tcw,
                                     uint8_t* d_outlier, int32_t* d_n_inliers,
                                     int32_t* d_lm_iterations, void* stream);

/* ---- LocalBundleAdjustment ----------------------------------------------------------------- */
/* One observation of a local map point (an EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ,
 * optimizer.cpp:548-606): the observing keyframe (index into the problem's keyframes), the
 * undistorted keypoint, its right coordinate (< 0 = monocular) and octave. 20 bytes.
 * Observations are grouped by map point in the order the reference inserts the edges
 * (point_obs_start is the CSR row pointer); a point has at most one observation per keyframe. */
typedef struct {
  int32_t keyframe;
  float u, v, ur;
  int32_t octave;
} slamgpu_ba_obs;

/* kf_mode: the role a keyframe vertex plays (optimizer.cpp:413-506). */
#define SLAMGPU_KF_LOCAL 0        /* local keyframe: optimised, pose written back */
#define SLAMGPU_KF_LOCAL_FIXED 1  /* local keyframe with id 0: fixed, pose written back */
#define SLAMGPU_KF_FIXED 2        /* fixed camera (sees a local point): neither */
/* Largest local (optimised) window and keyframe count per problem of the BATCHED device solver
 * (slamgpu_local_bundle_adjustment_device: one work-group per problem, S in LDS). */
#define SLAMGPU_BA_MAX_LOCAL_KF 24
#define SLAMGPU_BA_MAX_KF 256
/* Largest optimised window of the single-problem calls (slamgpu_local_bundle_adjustment,
 * slamgpu_global_bundle_adjustment: one problem over a cooperative grid, S in block-profile
 * storage in HBM -- its envelope follows the keyframes' co-observations, so a trajectory's map
 * stays near-banded; the bound is the factorisation's LDS row lists). */
#define SLAMGPU_BA_COOP_MAX_KF 4096

/* Replaces: void Optimizer::LocalBundleAdjustment(KeyFrame*, bool* stop_flag, const Map&)
 * (optimizer.cpp:413-716) after its graph gathering -- any local window (up to
 * SLAMGPU_BA_COOP_MAX_KF optimised keyframes), one problem spread over the GPU's CUs for
 * latency: kf_Tcw[16 n_kf] (row-major f32, updated for
 * modes 0 and 1), points[3 n_points] (MapPoint::GetWorldPos, all updated), the observations, and
 * erase[n_obs]: 1 where the reference puts (keyframe, point) in vToErase (the caller then runs
 * EraseMapPointMatch / EraseObservation and MapPoint::UpdateNormalAndDepth).
 * stop_flag (may be NULL) is the reference's bool* (LocalMapper::abort_BA_): it is live for the
 * whole call, as g2o's force-stop flag is (optimizer.cpp:474-476). It is read before optimising
 * (:616-618: raised -> return with nothing written and no erasures), and while the kernel runs
 * this thread mirrors it into host-mapped memory that the device polls at every point g2o calls
 * terminate(): each LM iteration (sparse_optimizer.cpp:376), each failed Levenberg trial
 * (optimization_algorithm_levenberg.cpp:149) and before the second optimize() (:625-627). So a
 * flag raised by another thread mid-run (LocalMapper::InsertKeyFrame, local_mapper.cpp:89-93;
 * RequestStop :95-100; InterruptBA :165-166) ends the optimisation within one LM iteration, and
 * the erase list and write-back use the state at that point, as in the reference.
 * *lm_iterations (may be NULL): LM iterations run. Synchronous. */
int slamgpu_local_bundle_adjustment(const slamgpu_camera* cam, const float* inv_sigma2,
                                    int nlevels, float* kf_Tcw, const uint8_t* kf_mode, int n_kf,
                                    float* points, int n_points, const int32_t* point_obs_start,
                                    const slamgpu_ba_obs* obs, const volatile bool* stop_flag,
                                    uint8_t* erase, int* lm_iterations);

/* Replaces: void Optimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF,
 * bRobust) (optimizer.cpp:33-207; GlobalBundleAdjustemnt :18-31 passes every keyframe and map
 * point) after its graph gathering: the keyframes (kf_mode SLAMGPU_KF_LOCAL, or
 * SLAMGPU_KF_LOCAL_FIXED for the keyframe with id 0, :53), the points and their observations in
 * the reference's edge order (bad keyframes / points left out by the caller, as :47-49, :82-84,
 * :95-97 skip them; a point with no observation is not optimised, :149-152). n_iterations
 * Levenberg-Marquardt iterations of one optimize() (:159-160), Huber kernels (deltas sqrt(5.99) /
 * sqrt(7.815)) when robust. kf_Tcw and points are updated in place: the caller stores them as
 * the pose / position or, for a loop-closure GBA (nLoopKF != 0), as Tcw_global_bundle_adj /
 * position_global_bundle_adj (:170-206). stop_flag: as slamgpu_local_bundle_adjustment's.
 * *lm_iterations (may be NULL): iterations run. Synchronous. */
int slamgpu_global_bundle_adjustment(const slamgpu_camera* cam, const float* inv_sigma2,
                                     int nlevels, float* kf_Tcw, const uint8_t* kf_mode, int n_kf,
                                     float* points, int n_points, const int32_t* point_obs_start,
                                     const slamgpu_ba_obs* obs, int n_iterations, int robust,
                                     const volatile bool* stop_flag, int* lm_iterations);

/* A problem of a batch: its keyframes d_kf_*[kf_begin, kf_begin + n_kf) and points
 * d_points[point_begin, point_begin + n_points); observations are
 * d_obs[d_point_obs_start[point_begin] .. d_point_obs_start[point_begin + n_points]) with
 * keyframe indices relative to kf_begin. */
typedef struct {
  int32_t kf_begin, n_kf, point_begin, n_points;
} slamgpu_ba_problem;

/* Device workspace the batched call needs for these totals over all problems. */
size_t slamgpu_local_ba_workspace_bytes(int total_kf, int total_points, int total_obs);

/* Batched, asynchronous on `stream`, every pointer device memory. d_point_obs_start has
 * total_points + 1 entries (global observation offsets). d_status[p]: LM iterations run (>= 0),
 * or -1 more than SLAMGPU_BA_MAX_LOCAL_KF local keyframes, -2 a point observed twice by one
 * keyframe, -3 a keyframe index outside the problem or more than SLAMGPU_BA_MAX_KF keyframes
 * (the problem's outputs are then untouched). d_stop_flag (may be NULL; may be host-mapped
 * memory): polled (one read per work-group, system scope) wherever g2o calls terminate() -- see
 * slamgpu_local_bundle_adjustment; a non-zero value ends the optimisation as g2o's force-stop
 * flag does. */
int slamgpu_local_bundle_adjustment_device(
    const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
    const slamgpu_ba_problem* d_problems, int n_problems, float* d_kf_Tcw,
    const uint8_t* d_kf_mode, float* d_points, const int32_t* d_point_obs_start,
    const slamgpu_ba_obs* d_obs, uint8_t* d_erase, int32_t* d_status, void* d_workspace,
    size_t workspace_bytes, int total_kf, int total_points, int total_obs,
    const int32_t* d_stop_flag, void* stream);

/* The reprojection residual / Jacobian / normal-equation build of LocalBundleAdjustment's first
 * optimize() (SparseOptimizer::computeActiveErrors + activeRobustChi2 + BlockSolver::buildSystem,
 * sparse_optimizer.cpp:61-114, block_solver.hpp:499-556, base_binary_edge.hpp:55-122) at the
 * input estimates, every edge at level 0 with its Huber kernel: the step every LM iteration of
 * the solver repeats, batched over problems. All arrays are device memory, doubles:
 *   chi2[obs], hpl[obs][18] (6x3 pose-point block, row-major; 0 for fixed keyframes),
 *   hll[points][6] and bl[points][3] (point block, packed 00 01 02 11 12 22, and b),
 *   hpp[keyframes][21] and bp[keyframes][6] (pose block, packed upper triangle row by row, and
 *   b; 0 unless kf_mode is SLAMGPU_KF_LOCAL), chi[problems] (the robust chi2).
 * g2o's sign convention: b = -J^T (rho' Omega) e. d_status[p]: 0 or the error codes of
 * slamgpu_local_bundle_adjustment_device. */
typedef struct {
  double* chi2;
  double* hpl;
  double* hll;
  double* bl;
  double* hpp;
  double* bp;
  double* chi;
} slamgpu_ba_linear;

int slamgpu_local_ba_linearize_device(
    const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
    const slamgpu_ba_problem* d_problems, int n_problems, const float* d_kf_Tcw,
    const uint8_t* d_kf_mode, const float* d_points, const int32_t* d_point_obs_start,
    const slamgpu_ba_obs* d_obs, const slamgpu_ba_linear* out, int32_t* d_status,
    void* d_workspace, size_t workspace_bytes, int total_kf, int total_points, int total_obs,
    void* stream);

/* ---- OptimizeSim3 ------------------------------------------------------------------------ */
/* One correspondence of Optimizer::OptimizeSim3 (optimizer.cpp:1020-1096), for a match i whose
 * map points are both good and seen by KF2 (:1033-1055; the caller skips the others): the
 * points in their keyframes' camera frames as the reference forms them (P3D1c = R1w * P3D1w +
 * t1w, P3D2c = R2w * P3D2w + t2w, f32 cv::Mat arithmetic), KF1's undistorted keypoint i, KF2's
 * undistorted keypoint GetIndexInKeyFrame(pKF2), and their octaves. 48 bytes. */
typedef struct {
  float x1c[3];
  float x2c[3];
  float u1, v1;
  float u2, v2;
  int32_t octave1, octave2;
} slamgpu_sim3_match;

/* Largest correspondence count per OptimizeSim3 problem. */
#define SLAMGPU_SIM3_MAX_MATCHES 4096

/* Replaces: int Optimizer::OptimizeSim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>&
 * vpMatches1, g2o::Sim3& g2oS12, float th2, bool bFixScale)  optimizer.cpp:962-1152.
 * K1 / K2: fx, fy, cx, cy of the keyframes' calib_mat; inv_sigma2_1 / _2[nlevels]: their
 * inv_level_sigma_sq. S12: the g2o::Sim3 as (qx, qy, qz, qw, tx, ty, tz, s) -- Sim3::operator[]
 * order -- updated in place unless the reference returns early. inlier[n]: 0 where the reference
 * sets vpMatches1[i] = NULL (pairs whose chi2 exceeds th2 after the first or the second
 * optimisation), 1 elsewhere. *n_inliers: the reference's return value (0 on its early return,
 * :1122-1125). Synchronous. */
int slamgpu_optimize_sim3(const float K1[4], const float K2[4], const float* inv_sigma2_1,
                          const float* inv_sigma2_2, int nlevels,
                          const slamgpu_sim3_match* matches, int n, float th2, int fix_scale,
                          double S12[8], uint8_t* inlier, int* n_inliers);

/* Batched (LoopCloser::ComputeSim3 tries its candidates in order and keeps the first with >= 20
 * inliers, loop_closer.cpp; every candidate can run at once and the caller takes the first),
 * asynchronous on `stream`, pointers device memory: problem p owns
 * d_matches[d_match_start[p] .. d_match_start[p+1]), d_S12[8 p ...] (in/out), inlier flags at
 * the matches' positions, d_n_inliers[p] (-1 when it exceeds SLAMGPU_SIM3_MAX_MATCHES, S12 then
 * untouched) and, if not NULL, d_lm_iterations[p]. The keyframe cameras / levels are shared. */
int slamgpu_optimize_sim3_device(const float K1[4], const float K2[4], const float* inv_sigma2_1,
                                 const float* inv_sigma2_2, int nlevels,
                                 const slamgpu_sim3_match* d_matches,
                                 const int32_t* d_match_start, int n_problems, float th2,
                                 int fix_scale, double* d_S12, uint8_t* d_inlier,
                                 int32_t* d_n_inliers, int32_t* d_lm_iterations, void* stream);

/* ---- OptimizeEssentialGraph --------------------------------------------------------------- */
/* One EdgeSim3 of the essential graph (optimizer.cpp:784-909): _vertices[0] = keyframe i,
 * _vertices[1] = keyframe j (indices into the call's keyframe arrays), measurement Sji (the
 * reference's Sjw * Swi, computed from vScw or the non-corrected poses as :789-898 do; same layout
 * as S12 above). Edges in the reference's insertion order. 80 bytes. */
typedef struct {
  int32_t i, j;
  int32_t pad[2];
  double Sji[8];
} slamgpu_sim3_edge;

/* Replaces: void Optimizer::OptimizeEssentialGraph(pMap, pLoopKF, pCurKF, NonCorrectedSim3,
 * CorrectedSim3, LoopConnections, bFixScale)  optimizer.cpp:718-960, after its graph gathering.
 * Scw[8 n_kf] (in/out): the vertices' vScw (the corrected Sim3 of the current keyframe's
 * neighbourhood, Sim3(R, t, 1) of the others), in keyframe id order; on return the optimised
 * CorrectedSiw. fixed[n_kf]: 1 for the loop keyframe. n_iterations: 20 in the reference.
 * Tcw[16 n_kf] (may be NULL): the recovered SE3 poses [R t/s; 0 1] for KeyFrame::SetPose.
 * points[3 n_points] (may be NULL), point_ref[n_points]: the map points (GetWorldPos) and the
 * keyframe index whose vScw / optimised Sim3 correct them (:941-947: corrected_reference when
 * the point was corrected by the current keyframe, else its reference keyframe); updated in place
 * (the caller then runs UpdateNormalAndDepth). *lm_iterations (may be NULL). Synchronous. */
int slamgpu_optimize_essential_graph(int n_kf, double* Scw, const uint8_t* fixed,
                                     const slamgpu_sim3_edge* edges, int n_edges, int fix_scale,
                                     int n_iterations, float* Tcw, float* points,
                                     const int32_t* point_ref, int n_points, int* lm_iterations);

const char* slamgpu_optimizer_last_error(void);

/* Diagnostic: the work-groups the cooperative BA solves running on `device` hold right now (the
 * residency budget shared by slamgpu_local_bundle_adjustment / slamgpu_global_bundle_adjustment
 * calls on concurrent threads, as the reference's LocalMapper and LoopCloser run them). */
int slamgpu_coop_slots_in_use(int device);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_OPTIMIZER_H_ */
