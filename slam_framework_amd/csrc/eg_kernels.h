// eg_kernels.h -- device pieces of OptimizeEssentialGraph (eg_kernels.hip); the LM loop runs on
// the host (optimizer_runtime.cpp), one synchronisation per Levenberg trial.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/slamgpu_optimizer.h"
#include "timing.h"

namespace slamgpu {

static_assert(sizeof(slamgpu_sim3_edge) == 80, "sim3 edge layout");

constexpr int kEgContrib = 3 * 49 + 2 * 7;  // per edge: Hii, Hjj, Hij (7x7), bi, bj

// The graph's fixed structure, built once on the host (device arrays).
struct EgGraph {
  int n, n_edges, F;           // vertices, edges, free vertices
  int fix_scale;
  const slamgpu_sim3_edge* edges;
  const int32_t* fidx;         // [n] free index or -1
  // profile of the 7F x 7F system: block row f stores blocks start[f] .. f at off[f]
  const int32_t* start;        // [F]
  const int64_t* off;          // [F + 1]
  // assembly targets: F diagonal blocks (+ b), then the structural off-diagonal blocks; target
  // t sums the contributions tgt_items[tgt_ptr[t] .. tgt_ptr[t + 1]) in edge order, item =
  // edge * 4 + kind (0: Hii as f's diagonal, 1: Hjj, 2: Hij, 3: Hij transposed)
  int n_targets;
  const int32_t* tgt_block;    // [n_targets] block index in the profile
  const int32_t* tgt_vertex;   // [n_targets] free vertex of a diagonal target, else -1
  const int32_t* tgt_ptr;      // [n_targets + 1]
  const int32_t* tgt_items;
  // column extents of the factorisation: rows i > k with start[i] <= k, increasing
  const int32_t* ext_ptr;      // [F + 1]
  const int32_t* ext_rows;
  const int64_t* ext_base;     // per extent entry: off[row] - start[row] (block (row, j) at + j)
  int n_ext;                   // extent entries (ext_ptr[F]; host copy, sizes the staged variant)
  int64_t n_blocks;            // blocks of the profile
};

// Mutable device state of one call.
struct EgState {
  double* S;        // [n][8] current estimates
  double* S_trial;  // [n][8]
  double* err;      // [n_edges][7]
  double* chi2;     // [n_edges]
  double* contrib;  // [n_edges][kEgContrib]
  double* J;        // [n_edges][98] numeric Jacobians Ji, Jj
  double* H;        // [blocks][49] assembled system
  double* b;        // [7F]
  double* L;        // [blocks][49] factor (copy of H)
  double* x;        // [7F]
  double* y;        // [7F]
  double* out;      // [4]: chi2 sum, scale term, solve ok
};

hipError_t launch_eg_linearize(const EgGraph& G, const EgState& W, hipStream_t st);
hipError_t launch_eg_errors(const EgGraph& G, const double* S, const EgState& W, hipStream_t st);
hipError_t launch_eg_chi2_sum(const EgGraph& G, const EgState& W, hipStream_t st);
hipError_t launch_eg_assemble(const EgGraph& G, const EgState& W, int64_t n_blocks, hipStream_t st);
hipError_t launch_eg_factor_solve(const EgGraph& G, const EgState& W, int64_t n_blocks,
                                  double lambda, hipStream_t st);
hipError_t launch_eg_update(const EgGraph& G, const EgState& W, hipStream_t st);
hipError_t launch_eg_finish(const EgGraph& G, const double* S_final, const double* S_init,
                            float* Tcw, float* points, const int32_t* point_ref, int n_points,
                            hipStream_t st);

}  // namespace slamgpu
