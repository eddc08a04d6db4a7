// ba_coop.h -- one bundle-adjustment problem over a cooperative grid (ba_coop.hip): the
// single-problem LocalBundleAdjustment (any local window) and the global BundleAdjustment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slamgpu_optimizer.h"
#include "pose_kernels.h"

namespace slamgpu {

// The problem in device memory (keyframe poses / points are updated in place).
struct CoopProblem {
  const slamgpu_ba_obs* obs;   // [n_obs], grouped by point
  const int32_t* pstart;       // [n_pts + 1]
  const uint8_t* kf_mode;      // [n_kf] SLAMGPU_KF_*
  float* kf_Tcw;               // [n_kf][16]
  float* points;               // [n_pts][3]
  uint8_t* erase;              // [n_obs] or nullptr (global BA)
  int32_t* ctl_out;            // [8] copy of the control words at the end, or nullptr
  int n_obs, n_pts, n_kf;
  int K;                       // optimised keyframes (mode SLAMGPU_KF_LOCAL)
};

// Device workspace of one problem (coop_layout).
struct CoopWs {
  double* chi2;        // [obs] last computed chi2 per edge
  double* hpl;         // [obs][18] Hpl block of an edge to an optimised keyframe
  uint8_t* act;        // [obs] edge at level 0
  int32_t* opoint;     // [obs] the edge's point
  int32_t* psorted;    // [obs] a point's active optimised-keyframe edges by keyframe
  double* pt;          // [27][pts] SoA (ba_device.h PX.. fields)
  int n_pt;
  double* kf;          // [n_kf][64] keyframe records (ba_device.h KQ.. fields)
  const int32_t* free_of_kf;  // [n_kf] optimised index or -1
  const int32_t* kf_of_free;  // [K]
  int32_t* npairs;     // [pts + 1] S-block pairs per point
  int32_t* poff;       // [pts + 1] exclusive offsets
  uint32_t* keys[2];   // [pairs_cap] block key per pair (tri(kh) + kl), sort ping-pong
  int2* vals[2];       // [pairs_cap] (edge h, edge l) or (edge, point) on the diagonal
  uint32_t* run_key;   // [pairs_cap] distinct blocks (run-length encoding of the sorted keys)
  int32_t* run_cnt;    // [pairs_cap]
  int32_t* run_off;    // [pairs_cap]
  int32_t* n_runs;     // [1]
  int32_t* diag_run;   // [K] run of block (f, f) or -1
  double* hpp_part;    // [K][nch][27] Hpp (21) + bp (6) partial sums
  double* hpp_tot;     // [K][27] their totals (the keyframe's last chunk, chunk order)
  int32_t* kf_arrive;  // [K] chunk arrival counters
  int32_t* run_arrive; // [pairs_cap] chunk arrival counters per run
  double* S;           // reduced camera system, lower part in block-profile storage (below)
  // block profile of S (host-computed from the co-observations): block row I holds block columns
  // pfirst[I] .. I; scalar row i holds columns 6 pfirst[i / 6] .. i at S[prow[i] + k]. Every
  // fill-in of the LDLT stays inside this envelope.
  const int32_t* pfirst;  // [K]
  const int64_t* prow;    // [n]
  int64_t pnnz;           // doubles of the profile
  int na_max;             // most active block rows of any block column (host, from pfirst)
  int mwg;                // factor a profile S over the whole grid (factor_profile_grid)
  double* bs;          // [n] reduced right-hand side
  int nch;
  int32_t* run_nch;    // [pairs_cap] assembly chunks per run
  int32_t* run_ch0;    // [pairs_cap] first chunk of each run
  int32_t* chunk_run;  // [chunks] run of each chunk
  int32_t* n_chunks;   // [1]
  double* chunk_part;  // [chunks][42] partial S block (36) and reduced rhs (6) sums
  double* fac;         // factor storage when n > kCoopLdsN: profile L (pnnz), V (6n), dg, rhs, idg
  double* xp;          // [n] pose step of the last successful solve
  double* part;        // [G][8] work-group partials + [8] scalars of work-group 0
  uint32_t* bar;       // grid barrier: [0] arrivals, [1] generation
  int32_t* ctl;        // control words (CTL_*)
  double* prof;        // [8] per-phase wall time (us) of work-group 0, or nullptr
  void* cub_tmp;
  size_t cub_bytes;
  int pairs_cap;
  int end_bit;         // radix-sort key bits
};

// CTL_BEAT: work-group 0's heartbeat while the others wait at a barrier (bumped per block column
// of the factorisation); CTL_ARRIVED / CTL_GRID: on a barrier give-up, the arrivals the giving-up
// waiter last saw and the grid size (missing work-groups vs a slow one).
enum { CTL_ERR = 0, CTL_STOPPED = 1, CTL_LM = 2, CTL_POLL = 3, CTL_OK = 4, CTL_BEAT = 5,
       CTL_ARRIVED = 6, CTL_GRID = 7 };

// One optimize() call of the schedule.
struct CoopPhase {
  int iterations;
  int robust;
  double delta_mono, delta_stereo;  // Huber deltas (float sqrt of the thresholds, as g2o gets)
};

// The schedule: one or two optimize() calls (LocalBA: robust 5, outlier pass, plain 10).
struct CoopSchedule {
  CoopPhase ph[2];
  int n_phases;
  int outlier_pass;
};

constexpr int kCoopThreads = 512;
constexpr int kCoopLdsN = 144;  // reduced systems up to 6 x 24 keyframes factor in LDS

// Bytes of the workspace for a problem (base = nullptr) or lays it out.
CoopWs coop_layout(void* base, int n_kf, int n_pts, int n_obs, int K, int pairs_cap, int G,
                   int64_t pnnz, size_t* bytes);

// Enqueues the whole schedule on `st`: setup, then per phase the structure build and the
// cooperative LM kernel, the outlier pass between phases (LocalBA), the erase list and write-back.
// d_free / d_kf_of_free must already be in the workspace (uploaded by the caller).
// The cooperative kernel (for occupancy queries).
const void* coop_kernel_ptr();

hipError_t launch_coop_ba(const PoseParams& P, const CoopProblem& pb, const CoopWs& w,
                          const CoopPhase* phases, int n_phases, bool outlier_pass,
                          const int32_t* d_stop, int G, hipStream_t st);

}  // namespace slamgpu
