// sim3_kernels.h -- launcher of the device OptimizeSim3 (sim3_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slamgpu_optimizer.h"
#include "timing.h"

namespace slamgpu {

static_assert(sizeof(slamgpu_sim3_match) == 48, "sim3 match layout");

// Shared by every problem of a batch: the keyframes' calibration (f32 -> f64), their
// inv_level_sigma_sq, th2 and the Huber delta (float)sqrt(th2) (optimizer.cpp:1017).
struct Sim3Params {
  double K1[4], K2[4];
  float isig1[SLAMGPU_MAX_LEVELS], isig2[SLAMGPU_MAX_LEVELS];
  int nlevels;
  float th2;
  double delta;
  int fix_scale;
};

hipError_t launch_optimize_sim3(const slamgpu_sim3_match* d_matches, const int32_t* d_match_start,
                                int n_problems, const Sim3Params& P, double* d_S12,
                                uint8_t* d_inlier, int32_t* d_n_inliers,
                                int32_t* d_lm_iterations, hipStream_t st);

}  // namespace slamgpu
