// ba_coop.hip -- one bundle-adjustment problem spread over a cooperative grid.
//
// Optimizer::LocalBundleAdjustment (optimizer.cpp:413-716) as the LocalMapper calls it -- one
// problem at a time, on the mapping thread's critical path -- and Optimizer::BundleAdjustment
// (the global BA, optimizer.cpp:33-207), with g2o's BlockSolver_6_3 + Levenberg-Marquardt
// arithmetic (the same statements as the one-work-group kernel in ba_kernels.hip) but:
//   * no cap on the optimised window: the reduced camera system S (6K x 6K) is dense in HBM and
//     only its structurally non-zero 6x6 blocks are listed, found per phase by a radix sort of the
//     (block, point-pair) keys every point contributes (hipcub, stable: each block's pairs stay in
//     point order, so every sum has a fixed order and the solver is deterministic);
//   * one problem over G work-groups (one per CU) of a cooperative launch, synchronised by a
//     grid barrier at each data dependency. Per LM iteration: the linearisation (a thread per
//     point over its edges: errors, Hll, bl, the 6x3 Hpl blocks; a wave per (keyframe, chunk):
//     partial Hpp, bp) -> barrier; per LM trial: the S blocks (a wave per block over its point
//     pairs, the point's (Hll + lambda I)^-1 formed on the fly) and the reduced rhs -> barrier ->
//     work-group 0 factors S (6x6-blocked LDLT, in LDS when 6K <= 144) and updates the keyframes
//     -> barrier -> a thread per point back-substitutes, updates and re-evaluates its edges ->
//     barrier. Three grid barriers per trial, one per iteration.
// Every LM decision (rho, lambda, the stop flag) is computed from the same per-work-group
// partials in the same order by every work-group, so the control flow is grid-uniform.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cmath>

#include "ba_coop.h"
#include "ba_device.h"
#include "timing.h"

namespace slamgpu {
namespace {

using namespace ba;

constexpr int kT = kCoopThreads, kW = kT / 64;
constexpr uint32_t kPadKey = 0xFFFFFFFFu;

struct CoopShared {
  double S[kCoopLdsN * (kCoopLdsN + 1) / 2];  // packed lower L of the factorisation
  double rhs[kCoopLdsN];
  double dg[kCoopLdsN];
  double V[kCoopLdsN * 6];
  double red[kW];
  float isig[SLAMGPU_MAX_LEVELS];
  int ok;
};

__device__ __forceinline__ double& ptf(const CoopWs& w, int p, int f) {
  return w.pt[(size_t)f * w.n_pt + p];
}
__device__ __forceinline__ double* kfr(const CoopWs& w, int k) { return w.kf + (size_t)k * 64; }

__device__ __forceinline__ void decode_key(uint32_t key, int& kh, int& kl) {
  int h = (int)((sqrt(8.0 * (double)key + 1.0) - 1.0) * 0.5);
  while (tri(h + 1) <= (int)key) h++;
  while (tri(h) > (int)key) h--;
  kh = h;
  kl = (int)key - tri(h);
}

// ---- grid barrier --------------------------------------------------------------------------
// Arrival counter + generation word in device memory; every thread releases its stores at
// device scope before and acquires after. Work-group 0 can carry a poll of the caller's stop flag
// (system scope: host-mapped memory) into CTL_POLL, which every work-group reads after the
// barrier -- so all of them take the same decision. A waiter gives up after ~2^22 sleeps and
// raises CTL_ERR (the host then reports a device error); later barriers do not wait once it is set.
__device__ void grid_sync(const CoopWs& w, const int32_t* stop_flag, bool poll) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (poll && blockIdx.x == 0) {
      const int32_t v =
          stop_flag ? __hip_atomic_load(stop_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
      __hip_atomic_store(&w.ctl[CTL_POLL], v != 0 ? 1 : 0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (__hip_atomic_load(&w.ctl[CTL_ERR], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      const uint32_t g = __hip_atomic_load(&w.bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t a =
          __hip_atomic_fetch_add(&w.bar[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (a == gridDim.x - 1) {
        __hip_atomic_store(&w.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&w.bar[1], g + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        uint32_t spins = 0;
        while (__hip_atomic_load(&w.bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 22)) {
            __hip_atomic_store(&w.ctl[CTL_ERR], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__device__ __forceinline__ int ctl_load(const CoopWs& w, int i) {
  return __hip_atomic_load(&w.ctl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Work-group sum (wave butterflies, then the waves in order by thread 0) -> part[wg][slot].
__device__ void wg_part(CoopShared& sh, const CoopWs& w, double v, int slot, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh.red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = sh.red[0];
    for (int k = 1; k < kW; k++) s = is_max ? fmax(s, sh.red[k]) : s + sh.red[k];
    w.part[(size_t)blockIdx.x * 8 + slot] = s;
  }
  __syncthreads();
}
// The grid total of a slot, in work-group order (identical in every work-group).
__device__ double grid_total(const CoopWs& w, int slot, bool is_max) {
  double s = w.part[slot];
  for (int g = 1; g < (int)gridDim.x; g++) {
    const double v = w.part[(size_t)g * 8 + slot];
    s = is_max ? fmax(s, v) : s + v;
  }
  return s;
}

// ---- setup and structure kernels -------------------------------------------------------------
__global__ __launch_bounds__(256) void coop_setup_kernel(CoopProblem pb, CoopWs w) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < pb.n_kf) {  // Converter::toSE3Quat
    const float* T = pb.kf_Tcw + (size_t)i * 16;
    double R[9];
    SE3 E;
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) R[3 * r + c] = T[4 * r + c];
      E.t[r] = T[4 * r + 3];
    }
    E.r = se3::quat_from_R(R);
    se3::normalize_rotation(E.r);
    store_T(kfr(w, i), E);
  }
  if (i < pb.n_pts) {
    for (int c = 0; c < 3; c++) {
      ptf(w, i, PX + c) = pb.points[(size_t)i * 3 + c];
      ptf(w, i, PXL + c) = 0.0;
    }
    for (int ge = pb.pstart[i]; ge < pb.pstart[i + 1]; ge++) w.opoint[ge] = i;
  }
  if (i < pb.n_obs) {
    w.act[i] = 1;
    w.chi2[i] = 0.0;
  }
  if (i < 6 * pb.K) w.xp[i] = 0.0;
  if (i < 8) w.ctl[i] = 0;
  if (i < 2) w.bar[i] = 0u;
}

// Per point: its active edges to optimised keyframes, sorted by keyframe, and its pair count.
__global__ __launch_bounds__(256) void coop_sort_kernel(CoopProblem pb, CoopWs w) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p > pb.n_pts) return;
  if (p == pb.n_pts) {
    w.npairs[p] = 0;
    return;
  }
  const int s = pb.pstart[p], e1 = pb.pstart[p + 1];
  int m = 0;
  for (int e = s; e < e1; e++) {
    if (!w.act[e]) continue;
    const int f = w.free_of_kf[pb.obs[e].keyframe];
    if (f < 0) continue;
    int i = m;
    while (i > 0) {
      const int prev = w.psorted[s + i - 1];
      if (w.free_of_kf[pb.obs[prev].keyframe] < f) break;
      w.psorted[s + i] = prev;
      i--;
    }
    w.psorted[s + i] = e;
    m++;
  }
  w.npairs[p] = m * (m + 1) / 2;
}

__global__ __launch_bounds__(256) void coop_emit_kernel(CoopProblem pb, CoopWs w) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= pb.n_pts) return;
  const int s = pb.pstart[p];
  const int np = w.npairs[p];
  int m = 0;
  while ((m + 1) * (m + 2) / 2 <= np) m++;
  const int base = w.poff[p];
  for (int i = 0; i < m; i++) {
    const int ei = w.psorted[s + i], fi = w.free_of_kf[pb.obs[ei].keyframe];
    for (int j = 0; j <= i; j++) {
      const int ej = w.psorted[s + j], fj = w.free_of_kf[pb.obs[ej].keyframe];
      const int o = base + i * (i + 1) / 2 + j;
      w.keys[0][o] = (uint32_t)(tri(fi) + fj);
      w.vals[0][o] = i == j ? make_int2(ei, p) : make_int2(ei, ej);
    }
  }
}

__global__ __launch_bounds__(256) void coop_runs_kernel(CoopWs w) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= *w.n_runs) return;
  const uint32_t key = w.run_key[r];
  if (key == kPadKey) return;
  int kh, kl;
  decode_key(key, kh, kl);
  if (kh == kl) w.diag_run[kh] = r;
}

// ---- the cooperative LM kernel ----------------------------------------------------------------
__device__ __forceinline__ double huber_rho(double c2, double d, double& wgt) {
  const double d2 = d * d;
  if (c2 > d2) {
    const double sq = sqrt(c2);
    wgt = d / sq;
    return 2 * sq * d - d2;
  }
  wgt = 1.0;
  return c2;
}

// Linearisation, part 1: a thread per point over its active edges (edge order): chi2 stored per
// edge, Hll and bl summed, the Hpl block of every edge to an optimised keyframe.
__device__ void lin_points(const CoopWs& w, const CoopProblem& pb, const PoseParams& P,
                           const float* isig, const CoopPhase& ph, double& chi, double& maxd) {
  const int GT = gridDim.x * kT;
  for (int p = blockIdx.x * kT + threadIdx.x; p < pb.n_pts; p += GT) {
    const double X[3] = {ptf(w, p, PX), ptf(w, p, PX + 1), ptf(w, p, PX + 2)};
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int nact = 0;
    for (int ge = pb.pstart[p]; ge < pb.pstart[p + 1]; ge++) {
      if (!w.act[ge]) continue;
      nact++;
      const slamgpu_ba_obs o = pb.obs[ge];
      const double* kr = kfr(w, o.keyframe);
      ObsEval v;
      const double c2 = eval_obs(o, P, isig, kr, X, v);
      w.chi2[ge] = c2;
      double wgt = 1.0;
      chi += ph.robust ? huber_rho(c2, v.stereo ? ph.delta_stereo : ph.delta_mono, wgt) : c2;
      double Jl[3][3], Jp[3][6];
      obs_jacobians(v, P, kr, Jl, Jp);
      const double W = wgt * v.info;
      const double or0 = -(v.info * v.e[0]) * wgt, or1 = -(v.info * v.e[1]) * wgt,
                   or2 = -(v.info * v.e[2]) * wgt;
      for (int i = 0; i < 3; i++) {
        H[6 + i] += Jl[0][i] * or0 + Jl[1][i] * or1 + Jl[2][i] * or2;
        for (int j = i; j < 3; j++)
          H[s3(i, j)] += (Jl[0][i] * W) * Jl[0][j] + (Jl[1][i] * W) * Jl[1][j] +
                         (Jl[2][i] * W) * Jl[2][j];
      }
      if (w.free_of_kf[o.keyframe] >= 0) {
        double* hp = w.hpl + (size_t)ge * 18;
        for (int i = 0; i < 6; i++)
          for (int j = 0; j < 3; j++)
            hp[3 * i + j] = (Jp[0][i] * W) * Jl[0][j] + (Jp[1][i] * W) * Jl[1][j] +
                            (Jp[2][i] * W) * Jl[2][j];
      }
    }
    for (int i = 0; i < 6; i++) ptf(w, p, PH + i) = H[i];
    for (int i = 0; i < 3; i++) ptf(w, p, PB + i) = H[6 + i];
    if (nact) maxd = fmax(maxd, fmax(fabs(H[0]), fmax(fabs(H[3]), fabs(H[5]))));
  }
}

// Linearisation, part 2: a wave per (optimised keyframe, chunk of its edge list) -> partial
// Hpp (packed upper) and bp.
__device__ void lin_keyframes(const CoopWs& w, const CoopProblem& pb, const PoseParams& P,
                              const float* isig, const CoopPhase& ph) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * kW, tasks = pb.K * w.nch;
  for (int t = blockIdx.x * kW + (threadIdx.x >> 6); t < tasks; t += nw) {
    const int f = t / w.nch, c = t - f * w.nch;
    const int r = w.diag_run[f];
    const int cnt = r >= 0 ? w.run_cnt[r] : 0, off = r >= 0 ? w.run_off[r] : 0;
    const int h0 = (int)((long long)cnt * c / w.nch), h1 = (int)((long long)cnt * (c + 1) / w.nch);
    const double* kr = kfr(w, w.kf_of_free[f]);
    double acc[32];
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = 0.0;
    for (int h = h0 + lane; h < h1; h += 64) {
      const int2 ep = w.vals[1][off + h];
      const double X[3] = {ptf(w, ep.y, PX), ptf(w, ep.y, PX + 1), ptf(w, ep.y, PX + 2)};
      ObsEval v;
      const double c2 = eval_obs(pb.obs[ep.x], P, isig, kr, X, v);
      double wgt = 1.0;
      if (ph.robust) (void)huber_rho(c2, v.stereo ? ph.delta_stereo : ph.delta_mono, wgt);
      double Jl[3][3], Jp[3][6];
      obs_jacobians(v, P, kr, Jl, Jp);
      const double W = wgt * v.info;
      const double or0 = -(v.info * v.e[0]) * wgt, or1 = -(v.info * v.e[1]) * wgt,
                   or2 = -(v.info * v.e[2]) * wgt;
      int hh = 0;
#pragma unroll
      for (int a = 0; a < 6; a++) {
        acc[21 + a] += Jp[0][a] * or0 + Jp[1][a] * or1 + Jp[2][a] * or2;
        const double wa0 = Jp[0][a] * W, wa1 = Jp[1][a] * W, wa2 = Jp[2][a] * W;
#pragma unroll
        for (int cc = a; cc < 6; cc++, hh++)
          acc[hh] += wa0 * Jp[0][cc] + wa1 * Jp[1][cc] + wa2 * Jp[2][cc];
      }
    }
    const double s = wave_reduce_scatter32(acc);
    if ((lane & 1) == 0 && (lane >> 1) < 27) w.hpp_part[((size_t)f * w.nch + c) * 27 + (lane >> 1)] = s;
  }
}

__device__ __forceinline__ double hpp_sum(const CoopWs& w, int f, int i) {
  double s = 0.0;
  for (int c = 0; c < w.nch; c++) s += w.hpp_part[((size_t)f * w.nch + c) * 27 + i];
  return s;
}

__device__ __forceinline__ void dinv_point(const CoopWs& w, int p, double lambda, double Di[6]) {
  double D[6];
  for (int i = 0; i < 6; i++) D[i] = ptf(w, p, PH + i);
  D[0] += lambda;
  D[3] += lambda;
  D[5] += lambda;
  inverse3_sym(D, Di);
}

// S blocks (a wave per distinct block, over its pairs in point order) and the reduced rhs of the
// diagonal blocks: S(kh, kl) = [kh == kl](Hpp + lambda I) - sum Hpl_eh Dinv_p Hpl_el^T,
// bs_k = bp_k - sum_e Hpl_e Dinv_p bl_p.
__device__ void assemble(const CoopWs& w, const CoopProblem& pb, double lambda, int n_runs) {
  const int lane = threadIdx.x & 63, n = 6 * pb.K;
  const int nw = gridDim.x * kW;
  for (int r = blockIdx.x * kW + (threadIdx.x >> 6); r < n_runs; r += nw) {
    const uint32_t key = w.run_key[r];
    if (key == kPadKey) continue;
    int kh, kl;
    decode_key(key, kh, kl);
    const bool diag = kh == kl;
    const int cnt = w.run_cnt[r], off = w.run_off[r];
    double acc[64];
#pragma unroll
    for (int i = 0; i < 64; i++) acc[i] = 0.0;
    for (int h = lane; h < cnt; h += 64) {
      const int2 ep = w.vals[1][off + h];
      const int eh = ep.x, el = diag ? ep.x : ep.y, p = diag ? ep.y : w.opoint[ep.x];
      double Di[6];
      dinv_point(w, p, lambda, Di);
      const double* hh = w.hpl + (size_t)eh * 18;
      const double* hp = w.hpl + (size_t)el * 18;
      double B[18];
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const double h0 = hh[3 * i], h1 = hh[3 * i + 1], h2 = hh[3 * i + 2];
        B[3 * i] = h0 * Di[0] + h1 * Di[1] + h2 * Di[2];
        B[3 * i + 1] = h0 * Di[1] + h1 * Di[3] + h2 * Di[4];
        B[3 * i + 2] = h0 * Di[2] + h1 * Di[4] + h2 * Di[5];
      }
#pragma unroll
      for (int rr = 0; rr < 6; rr++)
#pragma unroll
        for (int c = 0; c < 6; c++)
          acc[6 * rr + c] += B[3 * rr] * hp[3 * c] + B[3 * rr + 1] * hp[3 * c + 1] +
                             B[3 * rr + 2] * hp[3 * c + 2];
      if (diag) {
        const double b0 = ptf(w, p, PB), b1 = ptf(w, p, PB + 1), b2 = ptf(w, p, PB + 2);
        const double d0 = Di[0] * b0 + Di[1] * b1 + Di[2] * b2;
        const double d1 = Di[1] * b0 + Di[3] * b1 + Di[4] * b2;
        const double d2 = Di[2] * b0 + Di[4] * b1 + Di[5] * b2;
#pragma unroll
        for (int i = 0; i < 6; i++) acc[36 + i] += hh[3 * i] * d0 + hh[3 * i + 1] * d1 + hh[3 * i + 2] * d2;
      }
    }
    const double s0 = wave_reduce_scatter32(acc), s1 = wave_reduce_scatter32(acc + 32);
    const int idx = lane >> 1;
#pragma unroll
    for (int part = 0; part < 2; part++) {
      const int id = idx + 32 * part;
      if ((lane & 1) != 0) continue;
      const double sv = part ? s1 : s0;
      if (id < 36) {
        const int rr = id / 6, c = id % 6;
        const int i = 6 * kh + rr, j = 6 * kl + c;
        if (!diag || j <= i) {
          double base = 0.0;
          if (diag) base = hpp_sum(w, kh, hidx(c < rr ? c : rr, c < rr ? rr : c)) + (rr == c ? lambda : 0.0);
          w.S[(size_t)i * n + j] = base - sv;
        }
      } else if (diag && id < 42) {
        const int i = id - 36;
        w.bs[6 * kh + i] = hpp_sum(w, kh, 21 + i) - sv;
      }
    }
  }
}

// LDLT of S (6x6 block columns, right-looking, forward solve fused) by work-group 0, the same
// algorithm as ba_kernels.hip's factor_solve. L is packed lower at Lp (LDS or the global
// scratch). Sets sh.ok; on success writes the solution to w.xp (a failed solve keeps the previous
// step, which g2o applies anyway: optimization_algorithm_levenberg.cpp:107-109).
__device__ void factor_solve(CoopShared& sh, const CoopWs& w, int K, double* Lp, double* rhs,
                             double* dg, double* V) {
  const int tid = threadIdx.x, lane = tid & 63, n = 6 * K;
  for (int i = tid; i < n; i += kT) {
    rhs[i] = w.bs[i];
    for (int j = 0; j <= i; j++) Lp[sidx(i, j)] = w.S[(size_t)i * n + j];
  }
  if (tid == 0) sh.ok = 1;
  __syncthreads();
  for (int J = 0; J < K; J++) {
    const int j0 = 6 * J;
    if (tid == 0) {
      double A[6][6], d[6], y[6];
#pragma unroll
      for (int i = 0; i < 6; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) A[i][j] = Lp[sidx(j0 + i, j0 + j)];
        y[i] = rhs[j0 + i];
      }
      bool good = true;
#pragma unroll
      for (int j = 0; j < 6; j++) {
        double dj = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) dj -= A[j][k] * A[j][k] * d[k];
        good = good && dj != 0.0;
        d[j] = dj;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
          double s = A[i][j];
#pragma unroll
          for (int k = 0; k < j; k++) s -= A[i][k] * A[j][k] * d[k];
          A[i][j] = dj != 0.0 ? s / dj : 0.0;
        }
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
#pragma unroll
        for (int k = 0; k < i; k++) y[i] -= A[i][k] * y[k];
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
        dg[j0 + i] = d[i];
        rhs[j0 + i] = y[i];
#pragma unroll
        for (int j = 0; j < i; j++) Lp[sidx(j0 + i, j0 + j)] = A[i][j];
      }
      if (!good) sh.ok = 0;
    }
    __syncthreads();
    if (!sh.ok) return;
    for (int i = j0 + 6 + tid; i < n; i += kT) {
      double v[6];
      for (int c = 0; c < 6; c++) {
        double s = Lp[sidx(i, j0 + c)];
        for (int k = 0; k < c; k++) s -= v[k] * Lp[sidx(j0 + c, j0 + k)];
        v[c] = s;
      }
      double r = rhs[i];
      for (int c = 0; c < 6; c++) {
        V[(size_t)i * 6 + c] = v[c];
        const double l = v[c] / dg[j0 + c];
        Lp[sidx(i, j0 + c)] = l;
        r -= l * rhs[j0 + c];
      }
      rhs[i] = r;
    }
    __syncthreads();
    const int m = n - j0 - 6;
    for (int q = tid; q < m * m; q += kT) {
      const int ii = q / m, kk = q - ii * m;
      if (kk > ii) continue;
      const int i = j0 + 6 + ii, k = j0 + 6 + kk;
      double s = Lp[sidx(i, k)];
#pragma unroll
      for (int c = 0; c < 6; c++) s -= Lp[sidx(i, j0 + c)] * V[(size_t)k * 6 + c];
      Lp[sidx(i, k)] = s;
    }
    __syncthreads();
  }
  if ((tid >> 6) == 0) {
    for (int i = lane; i < n; i += 64) rhs[i] /= dg[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int k = n - 1; k > 0; k--) {
      const double xk = rhs[k];
      for (int i = lane; i < k; i += 64) rhs[i] -= Lp[sidx(k, i)] * xk;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    for (int i = lane; i < n; i += 64) w.xp[i] = rhs[i];
  }
  __syncthreads();
}

__device__ void restore_estimates(const CoopWs& w, const CoopProblem& pb) {
  const int GT = gridDim.x * kT;
  for (int p = blockIdx.x * kT + threadIdx.x; p < pb.n_pts; p += GT)
    for (int i = 0; i < 3; i++) ptf(w, p, PX + i) = ptf(w, p, PXB + i);
  for (int f = blockIdx.x * kT + threadIdx.x; f < pb.K; f += GT) {
    if (w.diag_run[f] < 0) continue;
    double* kr = kfr(w, w.kf_of_free[f]);
    SE3 T;
    T.r.x = kr[KBQ];
    T.r.y = kr[KBQ + 1];
    T.r.z = kr[KBQ + 2];
    T.r.w = kr[KBQ + 3];
    for (int i = 0; i < 3; i++) T.t[i] = kr[KBT + i];
    store_T(kr, T);
  }
}

__global__ __launch_bounds__(kT) void ba_coop_kernel(PoseParams P, CoopProblem pb, CoopWs w,
                                                     CoopPhase ph, const int32_t* stop_flag) {
#pragma clang fp contract(fast)  // tolerance-compared FP64 path
  __shared__ CoopShared sh;
  const int tid = threadIdx.x, wg = blockIdx.x, GT = gridDim.x * kT;
  if (ctl_load(w, CTL_STOPPED) || ctl_load(w, CTL_ERR)) return;  // written by earlier kernels
  if (tid < SLAMGPU_MAX_LEVELS) sh.isig[tid] = P.inv_sigma2[tid];
  const int K = pb.K, n = 6 * K;
  const int n_runs = *w.n_runs;
  double* Lp = n <= kCoopLdsN ? sh.S : w.fac;
  double* Vp = n <= kCoopLdsN ? sh.V : w.fac + (size_t)n * (n + 1) / 2;
  double* dgp = n <= kCoopLdsN ? sh.dg : Vp + (size_t)6 * n;
  double* rhsp = n <= kCoopLdsN ? sh.rhs : dgp + n;
  grid_sync(w, stop_flag, true);  // the first iteration's terminate() poll
  bool stop = ctl_load(w, CTL_POLL) != 0;
  double lambda = 0.0;
  int ni = 2, nbad = 0, lm_total = 0;
  bool stopped = false;
  for (int it = 0; it < ph.iterations; it++) {
    if (stop) {  // optimize(): i < iterations && !terminate()
      stopped = true;
      break;
    }
    // ---- linearise: computeActiveErrors + activeRobustChi2 + buildSystem ----
    double chi = 0.0, maxd = 0.0;
    lin_points(w, pb, P, sh.isig, ph, chi, maxd);
    lin_keyframes(w, pb, P, sh.isig, ph);
    wg_part(sh, w, chi, 0, false);
    wg_part(sh, w, maxd, 1, true);
    grid_sync(w, stop_flag, false);
    double currentChi = grid_total(w, 0, false);
    const double iniChi = currentChi;
    if (it == 0) {  // computeLambdaInit over the active vertices
      double m = grid_total(w, 1, true);
      for (int f = 0; f < K; f++) {
        if (w.diag_run[f] < 0) continue;
        const int dgi[6] = {0, 6, 11, 15, 18, 20};
        for (int i = 0; i < 6; i++) m = fmax(m, fabs(hpp_sum(w, f, dgi[i])));
      }
      lambda = 1e-5 * m;
      ni = 2;
      nbad = 0;
    }
    double rho = 0.0;
    int qmax = 0;
    bool rejected = false;
    do {
      // ---- S, reduced rhs (and the pop of a rejected trial's estimates) ----
      assemble(w, pb, lambda, n_runs);
      if (rejected) restore_estimates(w, pb);
      grid_sync(w, stop_flag, false);
      // ---- work-group 0: factor + solve, keyframe update (backup first) ----
      if (wg == 0) {
        factor_solve(sh, w, K, Lp, rhsp, dgp, Vp);
        double sc = 0.0;
        for (int f = tid; f < K; f += kT) {
          if (w.diag_run[f] < 0) continue;
          double* kr = kfr(w, w.kf_of_free[f]);
          double x[6];
          for (int i = 0; i < 6; i++) {
            x[i] = w.xp[6 * f + i];
            sc += x[i] * (lambda * x[i] + hpp_sum(w, f, 21 + i));
          }
          SE3 T;
          load_T(kr, T);
          for (int i = 0; i < 4; i++) kr[KBQ + i] = kr[KQ + i];
          for (int i = 0; i < 3; i++) kr[KBT + i] = kr[KT + i];
          store_T(kr, se3::se3_left_update(x, T));
        }
        wg_part(sh, w, sc, 4, false);  // work-group 0's slot 4: the keyframe share of `scale`
        if (tid == 0) w.ctl[CTL_OK] = sh.ok;
      }
      grid_sync(w, stop_flag, false);
      const bool ok = ctl_load(w, CTL_OK) != 0;
      // ---- points: back-substitution, update (backup first), errors of their edges ----
      double scale = 0.0, temp = 0.0;
      for (int p = wg * kT + tid; p < pb.n_pts; p += GT) {
        double c[3] = {ptf(w, p, PB), ptf(w, p, PB + 1), ptf(w, p, PB + 2)};
        int nact = 0;
        const int s = pb.pstart[p], e1 = pb.pstart[p + 1];
        for (int ge = s; ge < e1; ge++) {
          if (!w.act[ge]) continue;
          nact++;
          const int f = w.free_of_kf[pb.obs[ge].keyframe];
          if (!ok || f < 0) continue;
          const double* hp = w.hpl + (size_t)ge * 18;
          for (int i = 0; i < 6; i++) {
            const double x = w.xp[6 * f + i];
            c[0] -= hp[3 * i] * x;
            c[1] -= hp[3 * i + 1] * x;
            c[2] -= hp[3 * i + 2] * x;
          }
        }
        if (ok) {
          double Di[6];
          dinv_point(w, p, lambda, Di);
          ptf(w, p, PXL) = Di[0] * c[0] + Di[1] * c[1] + Di[2] * c[2];
          ptf(w, p, PXL + 1) = Di[1] * c[0] + Di[3] * c[1] + Di[4] * c[2];
          ptf(w, p, PXL + 2) = Di[2] * c[0] + Di[4] * c[1] + Di[5] * c[2];
        }
        double X[3];
        for (int i = 0; i < 3; i++) {
          X[i] = ptf(w, p, PX + i);
          ptf(w, p, PXB + i) = X[i];
        }
        if (nact) {  // oplus on the active vertices only
          for (int i = 0; i < 3; i++) {
            const double x = ptf(w, p, PXL + i);
            X[i] += x;
            ptf(w, p, PX + i) = X[i];
            scale += x * (lambda * x + ptf(w, p, PB + i));
          }
        }
        for (int ge = s; ge < e1; ge++) {
          if (!w.act[ge]) continue;
          const slamgpu_ba_obs o = pb.obs[ge];
          ObsEval v;
          const double c2 = eval_obs(o, P, sh.isig, kfr(w, o.keyframe), X, v);
          w.chi2[ge] = c2;
          double wgt;
          temp += ph.robust ? huber_rho(c2, v.stereo ? ph.delta_stereo : ph.delta_mono, wgt) : c2;
        }
      }
      wg_part(sh, w, temp, 2, false);
      wg_part(sh, w, scale, 3, false);
      grid_sync(w, stop_flag, true);  // carries the trial loop's terminate() poll
      stop = ctl_load(w, CTL_POLL) != 0;
      const double tempChi = ok ? grid_total(w, 2, false) : DBL_MAX;
      double sc = grid_total(w, 3, false) + w.part[4];
      sc += 1e-3;
      rho = (currentChi - tempChi) / sc;
      if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow(2 * rho - 1, 3.0);
        alpha = fmin(alpha, 2. / 3.);
        lambda *= fmax(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
        rejected = false;
      } else {
        lambda *= ni;
        ni *= 2;
        rejected = true;  // pop: restored with the next assembly, or below
      }
      qmax++;
    } while (rho < 0 && qmax < 10 && !stop);
    if (rejected) {
      restore_estimates(w, pb);
      grid_sync(w, stop_flag, false);
    }
    lm_total++;
    if (qmax == 10 || rho == 0) break;
    if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
    else nbad = 0;
    if (nbad >= 3) break;
  }
  if (wg == 0 && tid == 0) {
    w.ctl[CTL_LM] += lm_total;
    if (stopped) w.ctl[CTL_STOPPED] = 1;
  }
}

// ---- between the phases and after ------------------------------------------------------------
// optimizer.cpp:625-627: the stop flag is read once more before the second optimize().
__global__ void coop_poll_kernel(CoopWs w, const int32_t* stop_flag) {
  if (threadIdx.x == 0 && stop_flag &&
      __hip_atomic_load(stop_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)
    w.ctl[CTL_STOPPED] = 1;
}

// optimizer.cpp:632-665: chi2 > threshold or depth <= 0 -> level 1 (unless stopped).
__global__ __launch_bounds__(256) void coop_outlier_kernel(PoseParams P, CoopProblem pb, CoopWs w) {
  const int ge = blockIdx.x * 256 + threadIdx.x;
  if (ge >= pb.n_obs || w.ctl[CTL_STOPPED] || w.ctl[CTL_ERR]) return;
  float isig[SLAMGPU_MAX_LEVELS];
  for (int i = 0; i < P.nlevels; i++) isig[i] = P.inv_sigma2[i];
  const int p = w.opoint[ge];
  const double X[3] = {ptf(w, p, PX), ptf(w, p, PX + 1), ptf(w, p, PX + 2)};
  const slamgpu_ba_obs o = pb.obs[ge];
  ObsEval v;
  eval_obs(o, P, isig, kfr(w, o.keyframe), X, v);
  if (w.chi2[ge] > (o.ur >= 0 ? 7.815 : 5.991) || !(v.z > 0.0)) w.act[ge] = 0;
}

// optimizer.cpp:672-700 erase list (LocalBA), :702-716 / :170-206 write-back.
__global__ __launch_bounds__(256) void coop_finish_kernel(PoseParams P, CoopProblem pb, CoopWs w) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (w.ctl[CTL_ERR]) return;
  if (pb.erase && i < pb.n_obs) {
    float isig[SLAMGPU_MAX_LEVELS];
    for (int l = 0; l < P.nlevels; l++) isig[l] = P.inv_sigma2[l];
    const int p = w.opoint[i];
    const double X[3] = {ptf(w, p, PX), ptf(w, p, PX + 1), ptf(w, p, PX + 2)};
    const slamgpu_ba_obs o = pb.obs[i];
    ObsEval v;
    eval_obs(o, P, isig, kfr(w, o.keyframe), X, v);
    pb.erase[i] = (w.chi2[i] > (o.ur >= 0 ? 7.815 : 5.991) || !(v.z > 0.0)) ? 1 : 0;
  }
  if (i < pb.n_pts)
    for (int c = 0; c < 3; c++) pb.points[(size_t)i * 3 + c] = (float)ptf(w, i, PX + c);
  if (i < pb.n_kf && pb.kf_mode[i] != SLAMGPU_KF_FIXED) {
    const double* kr = kfr(w, i);
    float* T = pb.kf_Tcw + (size_t)i * 16;
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) T[4 * r + c] = (float)kr[KR + 3 * r + c];
      T[4 * r + 3] = (float)kr[KT + r];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
  }
}

size_t cub_bytes_needed(int pairs_cap, int end_bit) {
  size_t a = 0, b = 0, c = 0, d = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (int2*)nullptr, (int2*)nullptr, pairs_cap, 0, end_bit);
  (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                              (int32_t*)nullptr, (int32_t*)nullptr, pairs_cap);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int32_t*)nullptr, (int32_t*)nullptr,
                                         pairs_cap);
  return std::max(std::max(a, b), std::max(c, d));
}

int key_bits(int K) {
  const long long maxkey = (long long)K * (K + 1) / 2;  // pad key (2^bits - 1) > every real key
  int b = 1;
  while (((1ll << b) - 1) <= maxkey) b++;
  return b;
}

}  // namespace

CoopWs coop_layout(void* base, int n_kf, int n_pts, int n_obs, int K, int pairs_cap, int G,
                   size_t* bytes) {
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  size_t off = 0;
  char* b = static_cast<char*>(base);
  auto take = [&](size_t n) {
    char* p = b ? b + off : nullptr;
    off += al(n);
    return p;
  };
  const int n = 6 * K;
  const int pc = pairs_cap > 0 ? pairs_cap : 1;
  CoopWs w{};
  w.chi2 = reinterpret_cast<double*>(take(8 * (size_t)n_obs));
  w.hpl = reinterpret_cast<double*>(take(8 * 18 * (size_t)n_obs));
  w.act = reinterpret_cast<uint8_t*>(take((size_t)n_obs));
  w.opoint = reinterpret_cast<int32_t*>(take(4 * (size_t)n_obs));
  w.psorted = reinterpret_cast<int32_t*>(take(4 * (size_t)n_obs));
  w.pt = reinterpret_cast<double*>(take(8 * 27 * (size_t)n_pts));
  w.n_pt = n_pts;
  w.kf = reinterpret_cast<double*>(take(8 * 64 * (size_t)n_kf));
  w.free_of_kf = reinterpret_cast<int32_t*>(take(4 * (size_t)n_kf));
  w.kf_of_free = reinterpret_cast<int32_t*>(take(4 * (size_t)K + 4));
  w.npairs = reinterpret_cast<int32_t*>(take(4 * ((size_t)n_pts + 1)));
  w.poff = reinterpret_cast<int32_t*>(take(4 * ((size_t)n_pts + 1)));
  for (int i = 0; i < 2; i++) {
    w.keys[i] = reinterpret_cast<uint32_t*>(take(4 * (size_t)pc));
    w.vals[i] = reinterpret_cast<int2*>(take(8 * (size_t)pc));
  }
  w.run_key = reinterpret_cast<uint32_t*>(take(4 * (size_t)pc));
  w.run_cnt = reinterpret_cast<int32_t*>(take(4 * (size_t)pc));
  w.run_off = reinterpret_cast<int32_t*>(take(4 * (size_t)pc));
  w.n_runs = reinterpret_cast<int32_t*>(take(4));
  w.diag_run = reinterpret_cast<int32_t*>(take(4 * (size_t)K + 4));
  w.nch = std::max(1, std::min(32, (G * kW) / std::max(K, 1)));
  w.hpp_part = reinterpret_cast<double*>(take(8 * 27 * (size_t)K * w.nch + 8));
  w.S = reinterpret_cast<double*>(take(8 * (size_t)n * n + 8));
  w.bs = reinterpret_cast<double*>(take(8 * (size_t)n + 8));
  w.fac = reinterpret_cast<double*>(
      take(n > kCoopLdsN ? 8 * ((size_t)n * (n + 1) / 2 + 8 * (size_t)n) : 8));
  w.xp = reinterpret_cast<double*>(take(8 * (size_t)n + 8));
  w.part = reinterpret_cast<double*>(take(8 * 8 * (size_t)(G + 1)));
  w.bar = reinterpret_cast<uint32_t*>(take(64));
  w.ctl = reinterpret_cast<int32_t*>(take(64));
  w.pairs_cap = pc;
  w.end_bit = key_bits(K);
  w.cub_bytes = cub_bytes_needed(pc, w.end_bit);
  w.cub_tmp = take(w.cub_bytes + 256);
  if (bytes) *bytes = off + 256;
  return w;
}

const void* coop_kernel_ptr() { return reinterpret_cast<const void*>(&ba_coop_kernel); }

hipError_t launch_coop_ba(const PoseParams& P, const CoopProblem& pb, const CoopWs& w,
                          const CoopPhase* phases, int n_phases, bool outlier_pass,
                          const int32_t* d_stop, int G, hipStream_t st) {
  auto blocks = [](int n) { return dim3((unsigned)std::max(1, (n + 255) / 256)); };
  const int nmax = std::max(std::max(pb.n_kf, pb.n_pts), std::max(pb.n_obs, 6 * pb.K + 8));
  SLAMGPU_LAUNCH("ba_coop_setup", st, coop_setup_kernel, blocks(nmax), dim3(256), 0, st, pb, w);
  for (int ph = 0; ph < n_phases; ph++) {
    if (ph > 0) {
      if (outlier_pass) {
        SLAMGPU_LAUNCH("ba_coop_poll", st, coop_poll_kernel, dim3(1), dim3(64), 0, st, w, d_stop);
        SLAMGPU_LAUNCH("ba_coop_outlier", st, coop_outlier_kernel, blocks(pb.n_obs), dim3(256), 0,
                       st, P, pb, w);
      }
    }
    // structure of the active edge set: pairs per point -> offsets -> keys -> sorted runs
    SLAMGPU_LAUNCH("ba_coop_sort", st, coop_sort_kernel, blocks(pb.n_pts + 1), dim3(256), 0, st,
                   pb, w);
    size_t tb = w.cub_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, tb, w.npairs, w.poff,
                                                    pb.n_pts + 1, st);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.keys[0], 0xff, 4 * (size_t)w.pairs_cap, st)) != hipSuccess) return e;
    SLAMGPU_LAUNCH("ba_coop_emit", st, coop_emit_kernel, blocks(pb.n_pts), dim3(256), 0, st, pb, w);
    tb = w.cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, tb, w.keys[0], w.keys[1], w.vals[0],
                                           w.vals[1], w.pairs_cap, 0, w.end_bit, st);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.run_cnt, 0, 4 * (size_t)w.pairs_cap, st)) != hipSuccess) return e;
    tb = w.cub_bytes;
    e = hipcub::DeviceRunLengthEncode::Encode(w.cub_tmp, tb, w.keys[1], w.run_key, w.run_cnt,
                                              w.n_runs, w.pairs_cap, st);
    if (e != hipSuccess) return e;
    tb = w.cub_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, tb, w.run_cnt, w.run_off, w.pairs_cap, st);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.diag_run, 0xff, 4 * (size_t)pb.K + 4, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.S, 0, 8 * 36 * (size_t)pb.K * pb.K + 8, st)) != hipSuccess) return e;
    SLAMGPU_LAUNCH("ba_coop_runs", st, coop_runs_kernel, blocks(w.pairs_cap), dim3(256), 0, st, w);
    // the LM iterations: one cooperative launch (every work-group resident)
    CoopPhase cp = phases[ph];
    PoseParams Pc = P;
    CoopProblem pbc = pb;
    CoopWs wc = w;
    const int32_t* stop = d_stop;
    void* args[] = {&Pc, &pbc, &wc, &cp, &stop};
    if (g_timer) g_timer->begin("ba_coop", st);
    e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&ba_coop_kernel), dim3(G),
                                   dim3(kT), args, 0, st);
    if (g_timer) g_timer->end("ba_coop", st);
    if (e != hipSuccess) return e;
  }
  SLAMGPU_LAUNCH("ba_coop_finish", st, coop_finish_kernel, blocks(nmax), dim3(256), 0, st, P, pb, w);
  return hipGetLastError();
}

}  // namespace slamgpu
