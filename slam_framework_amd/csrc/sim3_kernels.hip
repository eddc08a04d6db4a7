// sim3_kernels.hip -- Optimizer::OptimizeSim3 (optimizer.cpp:962-1152) on the device.
//
// One work-group (2 waves) per problem runs the reference's whole schedule: optimize(5) with
// Huber kernels, the chi2 > th2 test that drops pairs from the graph, the early return when
// fewer than 10 pairs remain, optimize(5 or 10), the final inlier count. A problem is a loop
// candidate: LoopCloser::ComputeSim3 tries its candidates in order (loop_closer.cpp), so a batch
// of candidates is one launch, one work-group each.
//
// The graph: one Sim3 vertex (g2o::VertexSim3Expmap, oplus S <- Sim3(dx) * S, dx[6] = 0 when the
// scale is fixed) and, per correspondence, EdgeSim3ProjectXYZ (KF1's keypoint against S12 X2c)
// and EdgeInverseSim3ProjectXYZ (KF2's keypoint against S12^-1 X1c), both to fixed point
// vertices, so the system is the 7x7 Sim3 block. The edges have no analytic Jacobian: g2o
// differentiates them numerically, central differences with delta 1e-9 on each of the 7 update
// coordinates (base_binary_edge.hpp:131-203). Those 14 perturbed estimates are the same for
// every edge: per linearisation 15 threads build them (and their inverses) as affine maps into
// LDS, then a thread per correspondence evaluates its two edges at all of them.
//
// Per LM iteration: linearise pass (errors, chi2, Huber weights, Jacobians, the 28 + 7 + 1 sums
// of H, b and the robust chi2), then per trial one error pass. Sums are wave butterflies and a
// fixed-order sum over the 2 waves, so every thread holds the same totals and runs the LM control
// (7x7 LDLT, Sim3 exponential, lambda update) itself. g2o keeps each edge's last computed error,
// stale after a rejected step; the chi2 > th2 tests only read that, so a thread keeps one bit
// per pair (either edge's stored chi2 above th2).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "device_math.h"
#include "sim3_device.h"
#include "sim3_kernels.h"

namespace slamgpu {
namespace {

using sim3::Sim3;

constexpr int kSim3Waves = 2;
constexpr int kSim3Threads = 64 * kSim3Waves;
constexpr int kSim3Slots = SLAMGPU_SIM3_MAX_MATCHES / kSim3Threads;
static_assert(kSim3Slots <= 32, "slot masks are 32-bit");
constexpr int kNH7 = 28;         // upper triangle of the 7x7 H
constexpr int kNSum = kNH7 + 8;  // H, b (7), robust chi2
constexpr int kNAff = 15;        // the estimate and its 14 perturbations

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-91): rho(e), rho'(e).
__device__ __forceinline__ void huber(double e, double delta, double& r0, double& r1) {
  const double d2 = delta * delta;
  r0 = e;
  r1 = 1.0;
  if (e > d2) {
    const double s = sqrt(e);
    r0 = 2 * s * delta - d2;
    r1 = delta / s;
  }
}

// (e12, e21) of one correspondence at the estimate whose forward / inverse affine maps are F / I:
// e12 = obs1 - cam_map1(project(S X2c)), e21 = obs2 - cam_map2(project(S^-1 X1c)).
template <typename Ptr>
__device__ __forceinline__ void pair_errors(const slamgpu_sim3_match& m, const Sim3Params& P,
                                            Ptr F, Ptr I, double e[4]) {
  const double X2[3] = {m.x2c[0], m.x2c[1], m.x2c[2]};
  const double X1[3] = {m.x1c[0], m.x1c[1], m.x1c[2]};
  double p[3], q[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    p[i] = F[3 * i] * X2[0] + F[3 * i + 1] * X2[1] + F[3 * i + 2] * X2[2] + F[9 + i];
    q[i] = I[3 * i] * X1[0] + I[3 * i + 1] * X1[1] + I[3 * i + 2] * X1[2] + I[9 + i];
  }
  e[0] = (double)m.u1 - ((p[0] / p[2]) * P.K1[0] + P.K1[2]);
  e[1] = (double)m.v1 - ((p[1] / p[2]) * P.K1[1] + P.K1[3]);
  e[2] = (double)m.u2 - ((q[0] / q[2]) * P.K2[0] + P.K2[2]);
  e[3] = (double)m.v2 - ((q[1] / q[2]) * P.K2[1] + P.K2[3]);
}

__device__ __forceinline__ int clamp_level(int o, int n) { return o < 0 ? 0 : (o >= n ? n - 1 : o); }

// 7x7 (H + lambda I) x = b by LDLT without pivoting; zero pivots give zero components (Eigen's
// rule); a negative pivot fails the solve and x keeps its previous value (LinearSolverDense).
__device__ bool ldlt_solve7(const double* Hu, double lambda, const double* b, double x[7]) {
  double L[7][7], d[7];
  auto hij = [&](int i, int j) {  // packed upper triangle, i <= j
    return Hu[i * 7 - (i * (i - 1)) / 2 + (j - i)];
  };
#pragma unroll
  for (int j = 0; j < 7; j++) {
    double dj = hij(j, j) + lambda;
#pragma unroll
    for (int k = 0; k < j; k++) dj -= L[j][k] * L[j][k] * d[k];
    d[j] = dj;
    if (dj < 0) return false;
#pragma unroll
    for (int i = j + 1; i < 7; i++) {
      double s = hij(j, i);
#pragma unroll
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k] * d[k];
      L[i][j] = dj > DBL_MIN ? s / dj : 0.0;
    }
  }
  double y[7];
#pragma unroll
  for (int i = 0; i < 7; i++) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 7; i++) y[i] = fabs(d[i]) > DBL_MIN ? y[i] / d[i] : 0.0;
#pragma unroll
  for (int i = 6; i >= 0; i--) {
    double s = y[i];
#pragma unroll
    for (int k = i + 1; k < 7; k++) s -= L[k][i] * x[k];
    x[i] = s;
  }
  return true;
}

__global__ __launch_bounds__(kSim3Threads) void sim3_opt_kernel(
    const slamgpu_sim3_match* __restrict__ matches, const int32_t* __restrict__ match_start,
    Sim3Params P, double* __restrict__ S12, uint8_t* __restrict__ inlier_out,
    int32_t* __restrict__ n_inliers, int32_t* __restrict__ lm_iterations) {
  __shared__ double s_aff[kNAff][24];  // forward affine (12) | inverse affine (12)
  __shared__ double s_red[kSim3Waves][kNSum];
  __shared__ double s_tot[kNSum];
  __shared__ double s_J[kSim3Threads][29];  // a thread's Jacobian entries (odd row stride)
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int m0 = match_start[p];
  const int n = match_start[p + 1] - m0;
  if (n < 0 || n > SLAMGPU_SIM3_MAX_MATCHES) {
    if (tid == 0) {
      n_inliers[p] = -1;
      if (lm_iterations) lm_iterations[p] = 0;
    }
    return;
  }
  const slamgpu_sim3_match* M = matches + m0;
  uint8_t* inl = inlier_out + m0;
  const int nslots = tid < n ? (n - tid + kSim3Threads - 1) / kSim3Threads : 0;
  uint32_t active = nslots >= 32 ? ~0u : ((1u << nslots) - 1u);
  uint32_t bad = 0;
  double* Sp = S12 + 8 * p;
  Sim3 S = sim3::sim3_load(Sp);
  const double scalar = 1.0 / (2 * 1e-9);
  int lm_total = 0;

  // the sums of the work-group: every thread returns the same totals (in s_tot)
  auto reduce = [&](auto& v) {
    constexpr int nv = sizeof(v) / sizeof(double);
#pragma unroll
    for (int k = 0; k < nv; k++) {
      const double s = wave_sum(v[k]);
      if (lane == 0) s_red[w][k] = s;
    }
    __syncthreads();
    if (tid < nv) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < kSim3Waves; q++) t += s_red[q][tid];
      s_tot[tid] = t;
    }
    __syncthreads();
  };

  // SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg
  auto optimize = [&](int iterations) {
    double lambda = 0.0;
    int ni = 2, nbad = 0;
    double x[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int it = 0; it < iterations; it++) {
      // ---- the estimate and its 14 central-difference perturbations, as affine maps ----
      if (tid < kNAff) {
        Sim3 E = S;
        if (tid > 0) {
          const int dd = (tid - 1) >> 1;
          const double h = ((tid - 1) & 1) ? -1e-9 : 1e-9;
          double add[7];
#pragma unroll
          for (int i = 0; i < 7; i++) add[i] = i == dd ? h : 0.0;
          if (P.fix_scale) add[6] = 0;
          E = sim3::sim3_mul(sim3::sim3_exp(add), S);
        }
        sim3::sim3_affine(E, &s_aff[tid][0]);
        sim3::sim3_affine(sim3::sim3_inverse(E), &s_aff[tid][12]);
      }
      __syncthreads();
      // ---- linearise: computeActiveErrors + activeRobustChi2 + buildSystem ----
      double acc[kNSum];
#pragma unroll
      for (int k = 0; k < kNSum; k++) acc[k] = 0.0;
      for (int j = 0; j < nslots; j++) {
        if (!((active >> j) & 1u)) continue;
        const slamgpu_sim3_match m = M[tid + j * kSim3Threads];
        double e[4];
        pair_errors(m, P, (const double*)s_aff[0], (const double*)s_aff[0] + 12, e);
        const double i1 = (double)P.isig1[clamp_level(m.octave1, P.nlevels)];
        const double i2 = (double)P.isig2[clamp_level(m.octave2, P.nlevels)];
        const double c12 = e[0] * (i1 * e[0]) + e[1] * (i1 * e[1]);
        const double c21 = e[2] * (i2 * e[2]) + e[3] * (i2 * e[3]);
        bad = (c12 > (double)P.th2 || c21 > (double)P.th2) ? (bad | (1u << j)) : (bad & ~(1u << j));
        double r0a, r1a, r0b, r1b;
        huber(c12, P.delta, r0a, r1a);
        huber(c21, P.delta, r0b, r1b);
        acc[kNSum - 1] += r0a + r0b;
        // the 7 central differences of both edges, one column at a time into this thread's
        // LDS row (the 28 Jacobian entries are then read back together)
        double* Jrow = s_J[tid];
#pragma unroll 1
        for (int d = 0; d < 7; d++) {
          double ep[4], em[4];
          pair_errors(m, P, (const double*)s_aff[1 + 2 * d], (const double*)s_aff[1 + 2 * d] + 12, ep);
          pair_errors(m, P, (const double*)s_aff[2 + 2 * d], (const double*)s_aff[2 + 2 * d] + 12, em);
#pragma unroll
          for (int r = 0; r < 4; r++) Jrow[7 * r + d] = scalar * (ep[r] - em[r]);
        }
        double J[2][2][7];
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
          for (int r = 0; r < 2; r++)
#pragma unroll
            for (int d = 0; d < 7; d++) J[k][r][d] = Jrow[7 * (2 * k + r) + d];
        // b += J' omega_r, H += J' (rho' Omega) J (base_binary_edge.hpp:55-121, Sim3 block)
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const double info = k == 0 ? i1 : i2, r1 = k == 0 ? r1a : r1b;
          const double wt = r1 * info;
          const double o0 = -(info * e[2 * k]) * r1, o1 = -(info * e[2 * k + 1]) * r1;
          int h = 0;
#pragma unroll
          for (int a = 0; a < 7; a++) {
            acc[kNH7 + a] += J[k][0][a] * o0 + J[k][1][a] * o1;
            const double wa0 = J[k][0][a] * wt, wa1 = J[k][1][a] * wt;
#pragma unroll
            for (int c = a; c < 7; c++, h++) acc[h] += wa0 * J[k][0][c] + wa1 * J[k][1][c];
          }
        }
      }
      reduce(acc);
      double Hu[kNH7], b[7];
#pragma unroll
      for (int k = 0; k < kNH7; k++) Hu[k] = s_tot[k];
#pragma unroll
      for (int k = 0; k < 7; k++) b[k] = s_tot[kNH7 + k];
      double currentChi = s_tot[kNSum - 1];
      const double iniChi = currentChi;
      if (it == 0) {  // computeLambdaInit: tau * max |H_jj|, tau = 1e-5
        double maxd = 0.0;
#pragma unroll
        for (int j = 0; j < 7; j++) maxd = fmax(fabs(Hu[j * 7 - (j * (j - 1)) / 2]), maxd);
        lambda = 1e-5 * maxd;
        ni = 2;
        nbad = 0;
      }
      double rho = 0.0;
      int qmax = 0;
      do {
        const Sim3 backup = S;
        const bool ok = ldlt_solve7(Hu, lambda, b, x);
        if (P.fix_scale) x[6] = 0;  // VertexSim3Expmap::oplusImpl zeroes the solver's x[6]
        S = sim3::sim3_mul(sim3::sim3_exp(x), backup);
        // ---- trial: computeActiveErrors + activeRobustChi2 at the new estimate ----
        double F[12], I[12];
        sim3::sim3_affine(S, F);
        sim3::sim3_affine(sim3::sim3_inverse(S), I);
        double part = 0.0;
        for (int j = 0; j < nslots; j++) {
          if (!((active >> j) & 1u)) continue;
          const slamgpu_sim3_match m = M[tid + j * kSim3Threads];
          double e[4];
          pair_errors(m, P, (const double*)F, (const double*)I, e);
          const double i1 = (double)P.isig1[clamp_level(m.octave1, P.nlevels)];
          const double i2 = (double)P.isig2[clamp_level(m.octave2, P.nlevels)];
          const double c12 = e[0] * (i1 * e[0]) + e[1] * (i1 * e[1]);
          const double c21 = e[2] * (i2 * e[2]) + e[3] * (i2 * e[3]);
          bad = (c12 > (double)P.th2 || c21 > (double)P.th2) ? (bad | (1u << j)) : (bad & ~(1u << j));
          double r0a, r1a, r0b, r1b;
          huber(c12, P.delta, r0a, r1a);
          huber(c21, P.delta, r0b, r1b);
          part += r0a + r0b;
        }
        double part1[1] = {part};
        reduce(part1);
        double tempChi = s_tot[0];
        if (!ok) tempChi = DBL_MAX;
        double scale = 0.0;
#pragma unroll
        for (int j = 0; j < 7; j++) scale += x[j] * (lambda * x[j] + b[j]);
        scale += 1e-3;
        rho = (currentChi - tempChi) / scale;
        if (rho > 0 && isfinite(tempChi)) {
          double alpha = 1. - pow(2 * rho - 1, 3.0);
          alpha = fmin(alpha, 2. / 3.);
          lambda *= fmax(1. / 3., alpha);
          ni = 2;
          currentChi = tempChi;
        } else {
          lambda *= ni;
          ni *= 2;
          S = backup;  // pop: the edges keep the errors of the rejected estimate
        }
        qmax++;
      } while (rho < 0 && qmax < 10);
      lm_total++;
      if (qmax == 10 || rho == 0) break;
      if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
      else nbad = 0;
      if (nbad >= 3) break;
    }
  };

  auto count = [&](uint32_t mask) {
    double c[1] = {(double)__popc(mask)};
    reduce(c);
    return (int)s_tot[0];
  };

  optimize(5);
  // optimizer.cpp:1102-1120: pairs above th2 leave the graph (vpMatches1[i] = NULL)
  const uint32_t removed = active & bad;
  const int is_bad = count(removed);
  active &= ~removed;
  const bool early = n - is_bad < 10;  // :1122-1125: return 0, S12 untouched
  if (!early) optimize(is_bad > 0 ? 10 : 5);
  const uint32_t keep = early ? active : (active & ~bad);
  const int n_in = early ? 0 : count(keep);
  for (int j = 0; j < nslots; j++) inl[tid + j * kSim3Threads] = (keep >> j) & 1u;
  if (tid == 0) {
    if (!early) sim3::sim3_store(S, Sp);
    n_inliers[p] = n_in;
    if (lm_iterations) lm_iterations[p] = lm_total;
  }
}

}  // namespace

hipError_t launch_optimize_sim3(const slamgpu_sim3_match* d_matches, const int32_t* d_match_start,
                                int n_problems, const Sim3Params& P, double* d_S12,
                                uint8_t* d_inlier, int32_t* d_n_inliers,
                                int32_t* d_lm_iterations, hipStream_t st) {
  if (n_problems <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("sim3_opt", st, sim3_opt_kernel, dim3(n_problems), dim3(kSim3Threads), 0, st,
                 d_matches, d_match_start, P, d_S12, d_inlier, d_n_inliers, d_lm_iterations);
  return hipGetLastError();
}

}  // namespace slamgpu
