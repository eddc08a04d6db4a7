// pose_kernels.h -- launcher of the device PoseOptimization (pose_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slamgpu_optimizer.h"
#include "timing.h"

namespace slamgpu {

static_assert(sizeof(slamgpu_pose_edge) == 28, "pose edge layout");

// Kernel arguments shared by every frame of a batch: the stereo camera (Frame::fx..mbf) and
// Frame::mvInvLevelSigma2.
struct PoseParams {
  float fx, fy, cx, cy, bf;
  int nlevels;
  float inv_sigma2[SLAMGPU_MAX_LEVELS];
};

hipError_t launch_pose_optimization(const slamgpu_pose_edge* d_edges, const int32_t* d_edge_start,
                                    int n_frames, const PoseParams& P, float* d_Tcw,
                                    uint8_t* d_outlier, int32_t* d_n_inliers,
                                    int32_t* d_lm_iterations, hipStream_t st, int max_edges = -1);

}  // namespace slamgpu
