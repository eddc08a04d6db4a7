// pose_kernels.hip -- Optimizer::PoseOptimization (optimizer.cpp:209-411) on the device.
//
// One workgroup per frame runs the reference's whole schedule: 4 rounds of g2o's
// Levenberg-Marquardt (10 iterations each), outlier classification between rounds, robust kernel
// dropped after round 2. Nothing goes back to the host between iterations. Batches run one wave
// per frame (many frames resident per CU, no barriers); a handful of frames -- the per-frame
// tracking call -- runs 8 waves per frame to cut latency.
//
// Work split. Edge k of a frame is slot k / (64 W) of thread k % (64 W). Per slot the thread
// keeps two bits in registers: outlier (level 1, inactive), and whether the edge's last computed
// chi2 exceeds the f32 threshold. g2o keeps the last error per edge, stale after a rejected LM
// step (sparse_optimizer.cpp:61-88), and its classification only compares that chi2 with the
// threshold, so the bit is all the state it needs. Edge inputs (28 B) are re-read from L2 every
// pass; a 2000-edge frame is 56 KB.
//
// Per LM iteration there are 1 + #trials passes over the edges:
//   linearise pass : error, chi2, Huber weight, 2x6/3x6 Jacobian, and the 21 + 6 + 1 sums of
//                    H (upper triangle), b and the robust chi2 in one sweep (computeActiveErrors,
//                    activeRobustChi2 and buildSystem all evaluate at the same estimate);
//   trial pass     : error, chi2 and robust chi2 at exp(dx) * T.
// The sums are reductions (reduce-scatter across the wave through permlane / DPP exchanges, wave
// partials through LDS), after which every lane of every wave holds bitwise-identical totals.
// A one-wave frame runs the LM control (6x6 LDLT, exp, lambda update) in every lane with uniform
// branches; the latency variant lets wave 0 alone solve and broadcasts the step through LDS (all
// eight waves solving measured 0.527 ms per frame against 0.452, profiles/r4i_pose_*). The
// latency variant's solve is a dependent chain of ~800 FP64 instructions (~5 us per LM trial):
// one reciprocal per pivot, the exp map's Taylor coefficients for small steps, contraction.
//
// FP64 throughout, with the reference's f32 quirks: f32 inputs and outputs (Converter), float
// inverse depth in the stereo projection (types_six_dof_expmap.cpp:299-306), f32 Huber deltas and
// chi2 thresholds (optimizer.cpp:253-254, :352-401).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "device_math.h"
#include "pose_kernels.h"
#include "se3_device.h"

namespace slamgpu {
namespace {

using se3::Quat;
using se3::SE3;
using se3::normalize_rotation;
using se3::quat_from_R;
using se3::quat_to_R;

constexpr int kNH = 21;  // upper triangle of the 6x6 H
// Batches smaller than this run 8 waves per frame (latency); larger ones one wave per frame.
constexpr int kPoseLatencyFrames = 64;
constexpr int kPoseLdsEdges = 4096;  // edges of one frame the 1- and 8-wave variants take

// Tolerance-compared path: 1 / x and 1 / sqrt(x) from the hardware estimates (v_rcp_f64,
// v_rsq_f64) and two Newton steps -- within an ulp or two -- instead of the IEEE division and
// square-root expansions, for the solve's and the update's dependent chain (x > 0, finite).
__device__ __forceinline__ double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-x, y, 1.0);
  return __builtin_fma(y, e, y);
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double r = __builtin_fma(-h * y, y, 0.5);  // y <- y (1.5 - x y^2 / 2), twice
  y = __builtin_fma(y, r, y);
  r = __builtin_fma(-h * y, y, 0.5);
  return __builtin_fma(y, r, y);
}

// H x = b for the 6x6 H + lambda I, LDLT without pivoting; a zero pivot gives a zero component
// (Eigen's rule), a negative one fails the solve (LinearSolverDense::solve returns false and
// g2o applies the previous x). One reciprocal per pivot, and the unscaled column entries
// (L_ik d_k) kept for the later columns' sums: six divisions on the wave's dependent chain, not
// twenty-seven.
__device__ bool ldlt_solve6(const double H[kNH], double lambda, const double b[6], double x[6]) {
#pragma clang fp contract(fast)  // tolerance-compared: the column sums fuse
  double L[6][6], D[6][6], id[6];  // D[i][k] = L[i][k] d[k]
  bool neg = false;  // a negative pivot fails the solve; tested once, after the straight-line code
#pragma unroll
  for (int j = 0; j < 6; j++) {
    double dj = H[j * 6 - (j * (j - 1)) / 2] + lambda;  // H(j, j) in the packed upper triangle
#pragma unroll
    for (int k = 0; k < j; k++) dj -= L[j][k] * D[j][k];
    neg = neg || dj < 0;
    id[j] = dj > DBL_MIN ? rcp_nr(dj) : 0.0;
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      double s = H[j * 6 - (j * (j - 1)) / 2 + (i - j)];  // H(j, i) = H(i, j)
#pragma unroll
      for (int k = 0; k < j; k++) s -= L[i][k] * D[j][k];
      D[i][j] = s;
      L[i][j] = s * id[j];
    }
  }
  if (neg) return false;
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 6; i++) y[i] *= id[i];
#pragma unroll
  for (int i = 5; i >= 0; i--) {
    double s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; k++) s -= L[k][i] * x[k];
    x[i] = s;
  }
  return true;
}

// exp(dx) * T as se3::se3_left_update (SE3Quat::exp, se3quat.h:223-257), shortened for the
// wave's dependent chain: for 1e-5 <= theta < 1e-2 (LM steps of a tracked frame) the
// coefficients sin t / t, (1 - cos t) / t^2, (t - sin t) / t^3 come from their Taylor series
// (truncation below 1e-20 relative) instead of sincos and three divisions; the two
// normalisations take one reciprocal square root each. g2o's theta < 1e-5 branch (R = V = I + O
// + O^2) is kept as it is.
__device__ __forceinline__ void pose_normalize(Quat& q) {
  if (q.w < 0) {
    q.x = -q.x;
    q.y = -q.y;
    q.z = -q.z;
    q.w = -q.w;
  }
  const double in = rsq_nr(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x *= in;
  q.y *= in;
  q.z *= in;
  q.w *= in;
}
__device__ __forceinline__ SE3 pose_left_update(const double u[6], const SE3& T) {
#pragma clang fp contract(fast)
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double t2 = w0 * w0 + w1 * w1 + w2 * w2;  // theta^2: the branches test it, not theta
  const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
  double O2[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
  double a = 1.0, b = 1.0, c = 1.0;
  if (!(t2 < 1e-10)) {
    if (t2 < 1e-4) {
      // Horner in t^2 with constant reciprocals (multiplications, not divisions)
      constexpr double k6 = 1.0 / 6, k12 = 1.0 / 12, k20 = 1.0 / 20, k30 = 1.0 / 30;
      constexpr double k42 = 1.0 / 42, k56 = 1.0 / 56, k72 = 1.0 / 72, k90 = 1.0 / 90;
      constexpr double k110 = 1.0 / 110;
      a = 1.0 - t2 * k6 * (1.0 - t2 * k20 * (1.0 - t2 * k42 * (1.0 - t2 * k72)));
      b = 0.5 * (1.0 - t2 * k12 * (1.0 - t2 * k30 * (1.0 - t2 * k56 * (1.0 - t2 * k90))));
      c = k6 * (1.0 - t2 * k20 * (1.0 - t2 * k42 * (1.0 - t2 * k72 * (1.0 - t2 * k110))));
    } else {
      const double th = sqrt(t2);
      double s, co;
      sincos(th, &s, &co);
      const double it = rcp_nr(th);
      a = s * it;
      b = (1 - co) * it * it;
      c = (th - s) * it * it * it;
    }
  }
  double R[9], V[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const double I = (i % 4 == 0) ? 1.0 : 0.0;
    R[i] = I + a * O[i] + b * O2[i];
    V[i] = I + b * O[i] + c * O2[i];
  }
  SE3 E;
#pragma unroll
  for (int i = 0; i < 3; i++) E.t[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
  const double tr = R[0] + R[4] + R[8];
  if (tr > 0.0) {  // quat_from_R's first branch (a tracked frame's step), sqrt and 0.5 / t by rsq
    const double sq = tr + 1.0, rq = rsq_nr(sq), h = 0.5 * rq;
    E.r.w = 0.5 * (sq * rq);
    E.r.x = (R[7] - R[5]) * h;
    E.r.y = (R[2] - R[6]) * h;
    E.r.z = (R[3] - R[1]) * h;
  } else {
    E.r = quat_from_R(R);
  }
  pose_normalize(E.r);
  SE3 out;  // E * T
  double rt[3];
  se3::quat_rotate(E.r, T.t, rt);
#pragma unroll
  for (int i = 0; i < 3; i++) out.t[i] = E.t[i] + rt[i];
  const Quat& p = E.r;
  const Quat& q = T.r;
  out.r.w = p.w * q.w - p.x * q.x - p.y * q.y - p.z * q.z;
  out.r.x = p.w * q.x + p.x * q.w + p.y * q.z - p.z * q.y;
  out.r.y = p.w * q.y + p.y * q.w + p.z * q.x - p.x * q.z;
  out.r.z = p.w * q.z + p.z * q.w + p.x * q.y - p.y * q.x;
  pose_normalize(out.r);
  return out;
}

// RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-91): rho(e) and rho'(e). The sqrt and
// division run only for lanes past the kernel's corner (a skipped branch for inlier waves).
__device__ __forceinline__ double huber_rho0(double e, double delta) {
  double r = e;
  const double d2 = delta * delta;
  if (e > d2) r = 2 * sqrt(e) * delta - d2;
  return r;
}
// huber_rho0 without the branch (the latency variant's paired trial pass)
__device__ __forceinline__ double huber_rho0_sel(double e, double delta) {
  const double d2 = delta * delta;
  const double r = 2 * sqrt(e) * delta - d2;
  return e > d2 ? r : e;
}
__device__ __forceinline__ void huber_rho01(double e, double delta, double& r0, double& r1) {
  r0 = e;
  r1 = 1.0;
  const double d2 = delta * delta;
  if (e > d2) {
    const double s = sqrt(e);
    r0 = 2 * s * delta - d2;
    r1 = delta / s;
  }
}

// The estimate as the passes use it: Eigen maps points with the quaternion (q * v + t); the
// passes use the equal rotation matrix (one 3x3 product per edge instead of two cross products).
struct PassPose {
  double R[9], t[3];
};
// A double every lane holds the same bits of, moved to a scalar register pair (the passes read
// the pose through SGPR operands instead of 24 replicated VGPRs).
__device__ __forceinline__ double uniform_f64(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

__device__ __forceinline__ PassPose pass_pose(const SE3& T) {
  PassPose p;
  quat_to_R(T.r, p.R);
  for (int i = 0; i < 9; i++) p.R[i] = uniform_f64(p.R[i]);
  p.t[0] = uniform_f64(T.t[0]);
  p.t[1] = uniform_f64(T.t[1]);
  p.t[2] = uniform_f64(T.t[2]);
  return p;
}

struct EdgeEval {
  double e[3];
  double x, y, iz;  // camera coordinates, 1 / z
  bool stereo;
  double info;
};

// error = obs - cam_project(T.map(Xw)); returns chi2 = e' (info I) e. FMA contraction is allowed
// here: the pose path is compared with a tolerance, not bit for bit.
__device__ __forceinline__ double eval_edge(const slamgpu_pose_edge& E, const PoseParams& P,
                                            const float* isig, const PassPose& T, EdgeEval& v) {
#pragma clang fp contract(fast)
  const double X0 = E.xw[0], X1 = E.xw[1], X2 = E.xw[2];
  v.x = T.R[0] * X0 + T.R[1] * X1 + T.R[2] * X2 + T.t[0];
  v.y = T.R[3] * X0 + T.R[4] * X1 + T.R[5] * X2 + T.t[1];
  const double z = T.R[6] * X0 + T.R[7] * X1 + T.R[8] * X2 + T.t[2];
  v.iz = 1.0 / z;
  v.stereo = E.ur >= 0;
  int oct = E.octave;
  oct = oct < 0 ? 0 : (oct >= P.nlevels ? P.nlevels - 1 : oct);
  v.info = (double)isig[oct];
  // mono (EdgeSE3ProjectXYZOnlyPose, project2d): x / z, as x * (1/z) plus one residual step
  // (the correctly rounded quotient but for rare ties); stereo (EdgeStereoSE3ProjectXYZOnlyPose):
  // x * invz with `const float invz = 1.0f / z`
  const double izf = (double)(float)v.iz;
  double px = v.x * v.iz, py = v.y * v.iz;
  px = __builtin_fma(__builtin_fma(-px, z, v.x), v.iz, px);
  py = __builtin_fma(__builtin_fma(-py, z, v.y), v.iz, py);
  if (v.stereo) {
    px = v.x * izf;
    py = v.y * izf;
  }
  const double u = px * (double)P.fx + (double)P.cx;
  const double vv = py * (double)P.fy + (double)P.cy;
  v.e[0] = (double)E.u - u;
  v.e[1] = (double)E.v - vv;
  v.e[2] = v.stereo ? (double)E.ur - (u - (double)P.bf * izf) : 0.0;
  return v.info * (v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]);
}

// ---- reductions -------------------------------------------------------------------------------
// Sum 32 per-lane doubles over the wave: after 5 halving exchanges lane l holds the sum of value
// l >> 1 over 32 lanes; the last exchange completes it over all 64. The exchanges are
// lane_partner's permlane / DPP levels (pairs differ in bit log2(m)), not LDS permutes.
// Levels 32 and 16 exchange two registers' halves in one permlane swap per dword (no selects):
// after it the first holds (own, partner) of element i where the lane keeps i, the second the
// other order, and their sum is the same keep + partner (IEEE addition commutes).
template <int M>
__device__ __forceinline__ void swap_halves(double& a, double& b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = M == 32 ? __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false)
                          : __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = M == 32 ? __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false)
                          : __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = __builtin_bit_cast(double, (uint64_t)hi[0] << 32 | lo[0]);
  b = __builtin_bit_cast(double, (uint64_t)hi[1] << 32 | lo[1]);
}
__device__ __forceinline__ double wave_reduce_scatter32(double v[32]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    swap_halves<32>(v[i], v[i + 16]);
    v[i] = v[i] + v[i + 16];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    swap_halves<16>(v[i], v[i + 8]);
    v[i] = v[i] + v[i + 8];
  }
#pragma unroll
  for (int h = 4, m = 8; h >= 1; h >>= 1, m >>= 1) {
    // The upper lane of each pair keeps the upper half. Both candidates are read first and the
    // choice is made on the values (v_cndmask), never on their addresses (which would move v
    // to scratch).
    const uint64_t up = (lane & m) ? ~0ull : 0ull;
#pragma unroll
    for (int i = 0; i < h; i++) {
      const uint64_t lo = __builtin_bit_cast(uint64_t, v[i]);
      const uint64_t hi = __builtin_bit_cast(uint64_t, v[i + h]);
      const double send = __builtin_bit_cast(double, (lo & up) | (hi & ~up));
      const double keep = __builtin_bit_cast(double, (hi & up) | (lo & ~up));
      v[i] = keep + lane_partner(send, m);
    }
  }
  return v[0] + lane_partner(v[0], 1);
}

// butterfly: every lane ends with the same bits (each level adds a + b on one side and b + a on
// the other, and IEEE addition commutes).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += lane_partner(v, m);
  return v;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sums over the W waves of one frame's workgroup. Every wave ends with the same totals (its own
// copy, summed in the same order), so the LM control that reads them stays uniform.
template <int W>
struct FrameSum {
  double red[2][W][32];  // wave partials, double-buffered: a buffer is rewritten two sums later,
  double tot[W][32];     // after a barrier every reader has passed
  double bc[14];         // the trial step (x, T, ok) from wave 0 to the other waves
  int rb;

  // 32 sums (H, b, chi2) -> tot[wave][0..31]
  __device__ __forceinline__ const double* sum32(double v[32]) {
    const int lane = threadIdx.x & 63, w = wave_id();
    const double s = wave_reduce_scatter32(v);
    if (W == 1) {
      if ((lane & 1) == 0) tot[0][lane >> 1] = s;
    } else {
      if ((lane & 1) == 0) red[rb][w][lane >> 1] = s;
      __syncthreads();
      if (lane < 32) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < W; k++) t += red[rb][k][lane];
        tot[w][lane] = t;
      }
      rb ^= 1;
    }
    wave_lds_sync();
    return tot[w];
  }

  __device__ __forceinline__ double sum1(double v) {
    v = wave_sum(v);
    if (W == 1) return v;
    const int lane = threadIdx.x & 63, w = wave_id();
    if (lane == 0) red[rb][w][0] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < W; k++) t += red[rb][k][0];
    rb ^= 1;
    return t;
  }
};

// One edge's share of the linearisation (computeError + linearizeOplus + buildSystem): the
// robust chi2, b -= rho' J' Omega e and H += J' (rho' Omega) J into acc (H upper triangle, b,
// chi2).
__device__ __forceinline__ void lin_accumulate(const EdgeEval& ev, double wgt, double r0,
                                               const PoseParams& P, double (&acc)[32]) {
#pragma clang fp contract(fast)
  acc[27] += r0;
  // Jacobian of the error wrt [omega, upsilon] (types_six_dof_expmap.cpp:266-288, 311-364)
  const double iz = ev.iz, iz2 = iz * iz, x = ev.x, y = ev.y;
  const double fx = P.fx, fy = P.fy, bf = P.bf;
  double J[3][6];
  J[0][0] = x * y * iz2 * fx;
  J[0][1] = -(1 + (x * x * iz2)) * fx;
  J[0][2] = y * iz * fx;
  J[0][3] = -iz * fx;
  J[0][4] = 0;
  J[0][5] = x * iz2 * fx;
  J[1][0] = (1 + y * y * iz2) * fy;
  J[1][1] = -x * y * iz2 * fy;
  J[1][2] = -x * iz * fy;
  J[1][3] = 0;
  J[1][4] = -iz * fy;
  J[1][5] = y * iz2 * fy;
  const double sm = ev.stereo ? 1.0 : 0.0;  // the third row only for stereo edges
  J[2][0] = sm * (J[0][0] - bf * y * iz2);
  J[2][1] = sm * (J[0][1] + bf * x * iz2);
  J[2][2] = sm * J[0][2];
  J[2][3] = sm * J[0][3];
  J[2][4] = 0;
  J[2][5] = sm * (J[0][5] - bf * iz2);
  // b -= rho' J' Omega e ; H += J' (rho' Omega) J  (base_unary_edge.hpp:43-71)
  const double wi = wgt * ev.info;
  int h = 0;
#pragma unroll
  for (int a = 0; a < 6; a++) {
    const double ja0 = J[0][a] * ev.info, ja1 = J[1][a] * ev.info, ja2 = J[2][a] * ev.info;
    acc[kNH + a] -= wgt * (ja0 * ev.e[0] + ja1 * ev.e[1] + ja2 * ev.e[2]);
    const double wa0 = J[0][a] * wi, wa1 = J[1][a] * wi, wa2 = J[2][a] * wi;
#pragma unroll
    for (int c = a; c < 6; c++, h++) acc[h] += wa0 * J[0][c] + wa1 * J[1][c] + wa2 * J[2][c];
  }
}

// Optimizer::PoseOptimization for frame blockIdx.x with W waves. Edge k is slot k / (64 W) of
// thread k % (64 W); per slot a thread keeps two bits: the edge is an outlier (level 1,
// inactive), and the f32 test chi2 > threshold of the edge's last computed chi2 -- the only use
// g2o's classification makes of the stored (possibly stale) error.
#ifndef POSE_PROF
#define POSE_PROF 0
#endif
#ifndef POSE_LAT_W  // waves per frame of the latency variant
#define POSE_LAT_W 8
#endif
// kMaxE: the edges one frame may have in this variant (kMaxE / (64 W) slots per thread, <= 64).
// Frames with fewer than min_edges edges belong to another launch and are left untouched.
template <int W, int kMaxE>
__global__ __launch_bounds__(64 * W) void pose_opt_kernel(
    const slamgpu_pose_edge* __restrict__ edges, const int32_t* __restrict__ edge_start,
    PoseParams P, float* __restrict__ Tcw, uint8_t* __restrict__ outlier_out,
    int32_t* __restrict__ n_inliers, int32_t* __restrict__ lm_iterations, int min_edges) {
#pragma clang fp contract(fast)  // tolerance-compared FP64 path: let the edge sums fuse
  constexpr int kThreads = 64 * W;
  constexpr int kEpt = kMaxE / kThreads;
  static_assert(kEpt <= 64 && kEpt * kThreads == kMaxE, "slot masks are 64-bit");
  __shared__ FrameSum<W> fs;
  __shared__ float isig[SLAMGPU_MAX_LEVELS];  // Frame::mvInvLevelSigma2
  // the latency variant (one frame per work-group of W waves) keeps the frame's edges in LDS
  // (4096 x 28 B): the passes then wait on LDS, not on L2, for each edge slot
  constexpr bool kLdsEdges = W > 1 && kMaxE <= kPoseLdsEdges;
  constexpr bool kPairSlots = kLdsEdges;  // the latency variant pairs its trial slots
  __shared__ uint32_t s_edges[kLdsEdges ? kMaxE * 7 : 1];
  const int f = blockIdx.x, tid = threadIdx.x;
  const int e0 = edge_start[f];
  const int n = edge_start[f + 1] - e0;
  const slamgpu_pose_edge* E = edges + e0;
  uint8_t* outl_out = outlier_out + e0;
  if (n < min_edges) return;  // another launch's frame
  if (n > kMaxE || n < 0) {
    if (tid == 0) {
      n_inliers[f] = -1;
      if (lm_iterations) lm_iterations[f] = 0;
    }
    return;
  }
  if (n < 3) {  // optimizer.cpp:312-314 (edges exist, their outlier flags were cleared)
    for (int k = tid; k < n; k += kThreads) outl_out[k] = 0;
    if (tid == 0) {
      n_inliers[f] = 0;
      if (lm_iterations) lm_iterations[f] = 0;
    }
    return;
  }
  float* Tf = Tcw + 16 * f;
  if (tid < SLAMGPU_MAX_LEVELS) isig[tid] = P.inv_sigma2[tid];
  if constexpr (kLdsEdges) {
    static_assert(sizeof(slamgpu_pose_edge) == 28, "pose edge layout");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(E);
    for (int q = tid; q < 7 * n; q += kThreads) s_edges[q] = src[q];
  }
  auto edge = [&](int k) -> slamgpu_pose_edge {
    if constexpr (kLdsEdges) {
      slamgpu_pose_edge e;
      __builtin_memcpy(&e, &s_edges[7 * k], sizeof(e));
      return e;
    } else {
      return E[k];
    }
  };
  fs.rb = 0;
  __syncthreads();
  const double delta_mono = (double)(float)sqrt(5.991), delta_stereo = (double)(float)sqrt(7.815);
  const int nslots = tid < n ? (n - tid + kThreads - 1) / kThreads : 0;

  uint64_t outl = 0, lastbad = 0;
  int lm_total = 0, is_bad = 0;
#if POSE_PROF  // diagnostic build: thread 0's per-phase wall time (printf at the end)
  double pp[6] = {0, 0, 0, 0, 0, 0};
  uint64_t pt = __builtin_amdgcn_s_memrealtime();
  const uint64_t pc0 = clock64(), pw0 = pt;
  auto ptick = [&](int k) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    pp[k] += 0.01 * (double)(t - pt);
    pt = t;
  };
#else
  auto ptick = [](int) {};
#endif
  bool robust = true;
  SE3 T;

  for (int round = 0; round < 4; round++) {
    // optimizer.cpp:344 -- every round restarts from the frame's pose (Converter::toSE3Quat).
    // Re-derived from the f32 input each round rather than kept live.
    {
      double R[9];
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R[3 * i + j] = Tf[4 * i + j];
        T.t[i] = Tf[4 * i + 3];
      }
      T.r = quat_from_R(R);
      normalize_rotation(T.r);
    }
    double lambda = 0.0;
    int ni = 2, nbad = 0;
    for (int it = 0; it < 10; it++) {
      // ---- linearise: computeActiveErrors + activeRobustChi2 + buildSystem at T ----
      double acc[32];
#pragma unroll
      for (int i = 0; i < 32; i++) acc[i] = 0.0;
      const PassPose TP = pass_pose(T);
      // batched variant: a software pipeline, the next slot's edge loads (L2) under this one
      slamgpu_pose_edge en{};
      if (!kLdsEdges && nslots > 0) en = edge(tid);
      for (int j = 0; j < nslots; j++) {
        const slamgpu_pose_edge ec = kLdsEdges ? edge(tid + j * kThreads) : en;
        if (!kLdsEdges && j + 1 < nslots) en = edge(tid + (j + 1) * kThreads);
        if ((outl >> j) & 1) continue;
        EdgeEval ev;
        const double c2 = eval_edge(ec, P, isig, TP, ev);
        const uint64_t bit = 1ull << j;
        lastbad = ((float)c2 > (ev.stereo ? 7.815f : 5.991f)) ? (lastbad | bit) : (lastbad & ~bit);
        const double delta = ev.stereo ? delta_stereo : delta_mono;
        double wgt = 1.0, r0 = c2;
        if (robust) huber_rho01(c2, delta, r0, wgt);
        lin_accumulate(ev, wgt, r0, P, acc);
      }
      ptick(0);
      const double* S = fs.sum32(acc);
      ptick(1);
      const double* H = S;
      const double* b = S + kNH;
      double currentChi = S[27];
      const double iniChi = currentChi;
      if (it == 0) {  // computeLambdaInit: tau * max |H_jj|, tau = 1e-5
        double maxd = 0.0;
#pragma unroll
        for (int j = 0; j < 6; j++) maxd = fmax(fabs(H[j * 6 - (j * (j - 1)) / 2]), maxd);
        lambda = 1e-5 * maxd;
        ni = 2;
        nbad = 0;
      }
      double rho = 0.0, x[6] = {0, 0, 0, 0, 0, 0};
      int qmax = 0;
      do {
        const SE3 backup = T;
        bool ok;
        if constexpr (W == 1) {
          ok = ldlt_solve6(H, lambda, b, x);
          T = pose_left_update(x, backup);
        } else {  // wave 0 alone (its SIMD undisturbed), then a broadcast through LDS
          if (wave_id() == 0) {
            ok = ldlt_solve6(H, lambda, b, x);
            T = pose_left_update(x, backup);
            if ((tid & 63) == 0) {
#pragma unroll
              for (int j = 0; j < 6; j++) fs.bc[j] = x[j];
              fs.bc[6] = T.r.x;
              fs.bc[7] = T.r.y;
              fs.bc[8] = T.r.z;
              fs.bc[9] = T.r.w;
              fs.bc[10] = T.t[0];
              fs.bc[11] = T.t[1];
              fs.bc[12] = T.t[2];
              fs.bc[13] = ok ? 1.0 : 0.0;
            }
          }
          __syncthreads();  // the next write of bc follows sum1's barrier, after every read
#pragma unroll
          for (int j = 0; j < 6; j++) x[j] = fs.bc[j];
          T.r.x = fs.bc[6];
          T.r.y = fs.bc[7];
          T.r.z = fs.bc[8];
          T.r.w = fs.bc[9];
          T.t[0] = fs.bc[10];
          T.t[1] = fs.bc[11];
          T.t[2] = fs.bc[12];
          ok = fs.bc[13] != 0.0;
        }
        ptick(5);
        // ---- trial: computeActiveErrors + activeRobustChi2 at the new estimate ----
        double part = 0.0;
        const PassPose TP = pass_pose(T);
        if constexpr (kPairSlots) {
          // two slots per step, branch-free (an outlier's error is computed and discarded by
          // selects), so the two edges' dependent chains interleave; same order of additions
          for (int j = 0; j < nslots; j += 2) {
            const bool has1 = j + 1 < nslots;
            const slamgpu_pose_edge e0 = edge(tid + j * kThreads);
            const slamgpu_pose_edge e1 = edge(has1 ? tid + (j + 1) * kThreads : tid + j * kThreads);
            EdgeEval v0, v1;
            const double c0 = eval_edge(e0, P, isig, TP, v0);
            const double c1 = eval_edge(e1, P, isig, TP, v1);
            const bool a0 = !((outl >> j) & 1), a1 = has1 && !((outl >> (j + 1)) & 1);
            const uint64_t b0 = 1ull << j, b1 = has1 ? 1ull << (j + 1) : 0ull;
            if (a0)
              lastbad = ((float)c0 > (v0.stereo ? 7.815f : 5.991f)) ? (lastbad | b0) : (lastbad & ~b0);
            if (a1)
              lastbad = ((float)c1 > (v1.stereo ? 7.815f : 5.991f)) ? (lastbad | b1) : (lastbad & ~b1);
            const double r0 = robust ? huber_rho0_sel(c0, v0.stereo ? delta_stereo : delta_mono) : c0;
            const double r1 = robust ? huber_rho0_sel(c1, v1.stereo ? delta_stereo : delta_mono) : c1;
            part += a0 ? r0 : 0.0;
            part += a1 ? r1 : 0.0;
          }
        } else {
          slamgpu_pose_edge en{};
          if (!kLdsEdges && nslots > 0) en = edge(tid);
          for (int j = 0; j < nslots; j++) {
            const slamgpu_pose_edge ec = kLdsEdges ? edge(tid + j * kThreads) : en;
            if (!kLdsEdges && j + 1 < nslots) en = edge(tid + (j + 1) * kThreads);
            if ((outl >> j) & 1) continue;
            EdgeEval ev;
            const double c2 = eval_edge(ec, P, isig, TP, ev);
            const uint64_t bit = 1ull << j;
            lastbad = ((float)c2 > (ev.stereo ? 7.815f : 5.991f)) ? (lastbad | bit) : (lastbad & ~bit);
            part += robust ? huber_rho0(c2, ev.stereo ? delta_stereo : delta_mono) : c2;
          }
        }
        ptick(2);
        double tempChi = fs.sum1(part);
        ptick(3);
        if (!ok) tempChi = DBL_MAX;
        double scale = 0.0;
#pragma unroll
        for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
        scale += 1e-3;
        rho = (currentChi - tempChi) / scale;
        if (rho > 0 && isfinite(tempChi)) {
          const double rm = 2 * rho - 1;
          double alpha = 1. - rm * rm * rm;  // pow(2 rho - 1, 3)
          alpha = fmin(alpha, 2. / 3.);
          lambda *= fmax(1. / 3., alpha);
          ni = 2;
          currentChi = tempChi;
        } else {
          lambda *= ni;
          ni *= 2;
          T = backup;  // pop: the edges keep the errors of the rejected estimate
        }
        qmax++;
      } while (rho < 0 && qmax < 10);
      lm_total++;
      if (qmax == 10 || rho == 0) break;
      if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
      else nbad = 0;
      if (nbad >= 3) break;
    }
    // ---- classify (optimizer.cpp:352-401): inactive edges get their error at the final T ----
    double bad = 0.0;
    const PassPose TP = pass_pose(T);
    for (int j = 0; j < nslots; j++) {
      const uint64_t bit = 1ull << j;
      if (outl & bit) {
        EdgeEval ev;
        const double c2 = eval_edge(edge(tid + j * kThreads), P, isig, TP, ev);
        lastbad = ((float)c2 > (ev.stereo ? 7.815f : 5.991f)) ? (lastbad | bit) : (lastbad & ~bit);
      }
      bad += (lastbad & bit) ? 1.0 : 0.0;
    }
    outl = lastbad;
    is_bad = (int)fs.sum1(bad);
    ptick(4);
    if (round == 2) robust = false;
    if (n < 10) break;
  }
#if POSE_PROF
  const uint64_t pc1 = clock64(), pw1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0 && f == 0)
    printf("[pose W=%d] us: lin %.1f sum32 %.1f solve+update %.1f trial %.1f sum1 %.1f "
           "classify %.1f, %d LM iterations; shader clock %.0f MHz\n", W, pp[0], pp[1], pp[5],
           pp[2], pp[3], pp[4], lm_total, 100.0 * (double)(pc1 - pc0) / (double)(pw1 - pw0));
#endif
  // ---- write back: Frame::SetPose(Converter::toCvMat(SE3quat_recov)), mvbOutlier ----
  for (int j = 0; j < nslots; j++) outl_out[tid + j * kThreads] = (outl >> j) & 1;
  if (tid == 0) {
    double R[9];
    quat_to_R(T.r, R);
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) Tf[4 * i + j] = (float)R[3 * i + j];
      Tf[4 * i + 3] = (float)T.t[i];
    }
    Tf[12] = Tf[13] = Tf[14] = 0.f;
    Tf[15] = 1.f;
    n_inliers[f] = n - is_bad;
    if (lm_iterations) lm_iterations[f] = lm_total;
  }
}

}  // namespace

hipError_t launch_pose_optimization(const slamgpu_pose_edge* d_edges, const int32_t* d_edge_start,
                                    int n_frames, const PoseParams& P, float* d_Tcw,
                                    uint8_t* d_outlier, int32_t* d_n_inliers,
                                    int32_t* d_lm_iterations, hipStream_t st, int max_edges) {
  if (n_frames <= 0) return hipSuccess;
  if (n_frames < kPoseLatencyFrames) {
    // few frames: POSE_LAT_W waves per frame for latency (the per-frame tracking call)
    SLAMGPU_LAUNCH("pose_opt", st, (pose_opt_kernel<POSE_LAT_W, kPoseLdsEdges>), dim3(n_frames),
                   dim3(64 * POSE_LAT_W), 0, st, d_edges, d_edge_start, P, d_Tcw, d_outlier,
                   d_n_inliers, d_lm_iterations, 0);
  } else {
    // batches: one wave per frame, many frames resident per CU
    SLAMGPU_LAUNCH("pose_opt", st, (pose_opt_kernel<1, kPoseLdsEdges>), dim3(n_frames), dim3(64),
                   0, st, d_edges, d_edge_start, P, d_Tcw, d_outlier, d_n_inliers,
                   d_lm_iterations, 0);
  }
  // frames past the LDS variants' 4096 edges (the launch above marked them -1): 8 waves, 32
  // edge slots per thread read from L2, up to SLAMGPU_POSE_MAX_EDGES; max_edges < 0 = unknown
  // (device batches). 16 waves would cap the registers at 128 and spill.
  if (max_edges < 0 || max_edges > kPoseLdsEdges)
    SLAMGPU_LAUNCH("pose_opt", st, (pose_opt_kernel<8, SLAMGPU_POSE_MAX_EDGES>), dim3(n_frames),
                   dim3(64 * 8), 0, st, d_edges, d_edge_start, P, d_Tcw, d_outlier,
                   d_n_inliers, d_lm_iterations, kPoseLdsEdges + 1);
  return hipGetLastError();
}

}  // namespace slamgpu
