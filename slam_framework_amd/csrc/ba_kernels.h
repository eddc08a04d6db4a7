// ba_kernels.h -- launcher and workspace of the device LocalBundleAdjustment (ba_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slamgpu_optimizer.h"
#include "pose_kernels.h"

namespace slamgpu {

static_assert(sizeof(slamgpu_ba_obs) == 20, "ba observation layout");

// Device scratch of a batch, indexed by global keyframe / point / observation index.
struct BaWorkspace {
  double* chi2;      // [obs] last computed chi2 (g2o keeps the last error per edge)
  double* hpl;       // [obs][6 x 3] Hpl block of a local-keyframe edge
  uint8_t* act;      // [obs] edge at level 0
  int32_t* psorted;  // [obs] a point's active local-keyframe edges sorted by keyframe
  int2* hits;        // [obs * ((MAX_LOCAL_KF + 2) / 2)] S-block point pairs
  double* pt;        // [27][points] (SoA) estimate, backup, Hll, bl, Dinv, db, xl
  double* ehb;       // [obs][9] an edge's Hll and bl terms / Hpl^T xp
  int32_t* opoint;   // [obs] the edge's point (index within its problem)
  int n_pt;          // total points (the SoA stride)
  uint32_t* pmask;   // [points] local keyframes with an active edge to the point
  double* kf;        // [keyframes][64] estimate (q, t, R), backup, Hpp, bp
};

// Outputs of the linearisation entry point (slamgpu_ba_linear in slamgpu_optimizer.h).
struct BaLinearOut {
  double* chi2;  // [obs]
  double* hpl;   // [obs][18]
  double* hll;   // [points][6]
  double* bl;    // [points][3]
  double* hpp;   // [keyframes][21]
  double* bp;    // [keyframes][6]
  double* chi;   // [problems]
};

// Lays the workspace out from `base` (nullptr: only computes *bytes).
BaWorkspace ba_workspace_layout(void* base, int total_kf, int total_points, int total_obs,
                                size_t* bytes);

hipError_t launch_local_ba_linearize(const PoseParams& P, const slamgpu_ba_problem* d_problems,
                                     int n_problems, const float* d_kf_Tcw,
                                     const uint8_t* d_kf_mode, const float* d_points,
                                     const int32_t* d_pstart, const slamgpu_ba_obs* d_obs,
                                     int32_t* d_status, const BaWorkspace& ws,
                                     const BaLinearOut& out, hipStream_t st);

hipError_t launch_local_ba(const PoseParams& P, const slamgpu_ba_problem* d_problems,
                           int n_problems, float* d_kf_Tcw, const uint8_t* d_kf_mode,
                           float* d_points, const int32_t* d_pstart, const slamgpu_ba_obs* d_obs,
                           uint8_t* d_erase, int32_t* d_status, const BaWorkspace& ws,
                           const int32_t* d_stop, hipStream_t st);

}  // namespace slamgpu
