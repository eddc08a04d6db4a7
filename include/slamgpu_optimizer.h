/*
 * slamgpu_optimizer.h -- C ABI of the MI355X motion-only / local bundle adjustment
 * (libslamgpu.so, same library as slamgpu.h).
 *
 * Drop-in boundary for the reference's Optimizer (src/optimizer/optimizer.h:14-40, a class of
 * static functions over g2o):
 *   slamgpu_pose_optimization         Optimizer::PoseOptimization(Frame*)  optimizer.cpp:209-411
 *   slamgpu_pose_optimization_device  the same, batched over frames, inputs resident in HBM
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

/* Largest edge count per frame the pose kernel takes (frames carry <= nfeatures keypoints). */
#define SLAMGPU_POSE_MAX_EDGES 4096
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

const char* slamgpu_optimizer_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_OPTIMIZER_H_ */
