// ba_device.h -- device pieces shared by the LocalBundleAdjustment kernels (ba_kernels.hip:
// one work-group per problem; ba_coop.hip: one problem over a cooperative grid) and the global
// BundleAdjustment: the binary edges' error and Jacobians (types_six_dof_expmap.cpp:103-234),
// the keyframe record layout, wave reductions and the 3x3 symmetric inverse.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/slamgpu_optimizer.h"
#include "device_math.h"
#include "pose_kernels.h"
#include "se3_device.h"

namespace slamgpu {
namespace ba {

using se3::Quat;
using se3::SE3;

__device__ __forceinline__ int tri(int i) { return i * (i + 1) / 2; }
__device__ __forceinline__ int sidx(int i, int j) { return tri(i) + j; }  // lower, j <= i
__device__ __forceinline__ int hidx(int a, int c) {  // packed upper triangle of a 6x6, a <= c
  return a * 6 - (a * (a - 1)) / 2 + (c - a);
}

// ---- per-KF / per-point workspace records (ba_kernels.h: BaWorkspace) -----------------------
// kf record (64 doubles): q 0..3, t 4..6, R 8..16, backup q 17..20 t 21..23, Hpp 24..44,
// bp 45..50, xp 51..56, Hpp-diag max 57
constexpr int KQ = 0, KT = 4, KR = 8, KBQ = 17, KBT = 21, KH = 24, KB = 45;
// point fields (structure of arrays, ws.pt[field * ws.n_pt + point]): X 0..2, Xb 3..5,
// Hll 6..11 (00 01 02 11 12 22), bl 12..14, Dinv 15..20 (same packing), db 21..23, xl 24..26
constexpr int PX = 0, PXB = 3, PH = 6, PB = 12, PD = 15, PDB = 21, PXL = 24;
// per-edge scratch record (ws.ehb, 9 doubles): the edge's Hll (6) and bl (3) terms; in the update
// its first 3 hold Hpl^T xp
__device__ __forceinline__ int s3(int i, int j) {  // packed symmetric 3x3
  const int a = i < j ? i : j, b = i < j ? j : i;
  return a == 0 ? b : (a == 1 ? 2 + b : 5);
}

__device__ __forceinline__ void load_T(const double* kr, SE3& T) {
  T.r.x = kr[KQ];
  T.r.y = kr[KQ + 1];
  T.r.z = kr[KQ + 2];
  T.r.w = kr[KQ + 3];
  T.t[0] = kr[KT];
  T.t[1] = kr[KT + 1];
  T.t[2] = kr[KT + 2];
}
__device__ __forceinline__ void store_T(double* kr, const SE3& T) {
  kr[KQ] = T.r.x;
  kr[KQ + 1] = T.r.y;
  kr[KQ + 2] = T.r.z;
  kr[KQ + 3] = T.r.w;
  kr[KT] = T.t[0];
  kr[KT + 1] = T.t[1];
  kr[KT + 2] = T.t[2];
  double R[9];
  se3::quat_to_R(T.r, R);
  for (int i = 0; i < 9; i++) kr[KR + i] = R[i];
}

struct ObsEval {
  double x, y, z, iz;  // camera coordinates, 1 / z
  double e[3];
  double info;
  bool stereo;
};

// e = obs - cam_project(T.map(X)) for EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ; returns chi2.
__device__ __forceinline__ double eval_obs(const slamgpu_ba_obs& o, const PoseParams& P,
                                           const float* isig, const double* kr, const double X[3],
                                           ObsEval& v) {
  Quat q;
  q.x = kr[KQ];
  q.y = kr[KQ + 1];
  q.z = kr[KQ + 2];
  q.w = kr[KQ + 3];
  double p[3];
  se3::quat_rotate(q, X, p);
  v.x = p[0] + kr[KT];
  v.y = p[1] + kr[KT + 1];
  v.z = p[2] + kr[KT + 2];
  v.iz = 1.0 / v.z;
  v.stereo = o.ur >= 0;
  int oct = o.octave;
  oct = oct < 0 ? 0 : (oct >= P.nlevels ? P.nlevels - 1 : oct);
  v.info = (double)isig[oct];
  double px, py;
  if (!v.stereo) {  // project2d: x / z
    px = v.x / v.z;
    py = v.y / v.z;
  } else {          // const float invz = 1.0f / z
    const float izf = (float)v.iz;
    px = v.x * (double)izf;
    py = v.y * (double)izf;
  }
  const double u = px * (double)P.fx + (double)P.cx;
  const double vv = py * (double)P.fy + (double)P.cy;
  v.e[0] = (double)o.u - u;
  v.e[1] = (double)o.v - vv;
  v.e[2] = 0.0;
  if (v.stereo) {  // res[2] = res[0] - bf * invz with `const float& bf`: a float product
    const float bfz = P.bf * (float)v.iz;
    v.e[2] = (double)o.ur - (u - (double)bfz);
  }
  return v.info * (v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]);
}

// Jl (D x 3, wrt the point) and Jp (D x 6, wrt the pose); row 2 is zero for monocular edges
// (types_six_dof_expmap.cpp:103-137, 188-234).
__device__ __forceinline__ void obs_jacobians(const ObsEval& v, const PoseParams& P,
                                              const double* kr, double Jl[3][3], double Jp[3][6]) {
  const double fx = P.fx, fy = P.fy, bf = P.bf, x = v.x, y = v.y, iz = v.iz, iz2 = iz * iz;
  const double sm = v.stereo ? 1.0 : 0.0;
  for (int j = 0; j < 3; j++) {
    const double r0 = kr[KR + j], r1 = kr[KR + 3 + j], r2 = kr[KR + 6 + j];
    Jl[0][j] = -fx * r0 * iz + fx * x * r2 * iz2;
    Jl[1][j] = -fy * r1 * iz + fy * y * r2 * iz2;
    Jl[2][j] = sm * (Jl[0][j] - bf * r2 * iz2);
  }
  Jp[0][0] = x * y * iz2 * fx;
  Jp[0][1] = -(1 + x * x * iz2) * fx;
  Jp[0][2] = y * iz * fx;
  Jp[0][3] = -iz * fx;
  Jp[0][4] = 0;
  Jp[0][5] = x * iz2 * fx;
  Jp[1][0] = (1 + y * y * iz2) * fy;
  Jp[1][1] = -x * y * iz2 * fy;
  Jp[1][2] = -x * iz * fy;
  Jp[1][3] = 0;
  Jp[1][4] = -iz * fy;
  Jp[1][5] = y * iz2 * fy;
  Jp[2][0] = sm * (Jp[0][0] - bf * y * iz2);
  Jp[2][1] = sm * (Jp[0][1] + bf * x * iz2);
  Jp[2][2] = sm * Jp[0][2];
  Jp[2][3] = sm * Jp[0][3];
  Jp[2][4] = 0;
  Jp[2][5] = sm * (Jp[0][5] - bf * iz2);
}

__device__ __forceinline__ double huber_delta(bool stereo) {
  return stereo ? (double)(float)sqrt(7.815) : (double)(float)sqrt(5.991);
}

// ---- reductions -------------------------------------------------------------------------------
__device__ __forceinline__ double wave_reduce_scatter32(double v[32]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int h = 16, m = 32; h >= 1; h >>= 1, m >>= 1) {
    const uint64_t up = (lane & m) ? ~0ull : 0ull;
#pragma unroll
    for (int i = 0; i < h; i++) {
      const uint64_t lo = __builtin_bit_cast(uint64_t, v[i]);
      const uint64_t hi = __builtin_bit_cast(uint64_t, v[i + h]);
      const double send = __builtin_bit_cast(double, (lo & up) | (hi & ~up));
      const double keep = __builtin_bit_cast(double, (hi & up) | (lo & ~up));
      v[i] = keep + __shfl_xor(send, m);
    }
  }
  return v[0] + __shfl_xor(v[0], 1);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m));
  return v;
}


// Eigen's 3x3 inverse of a symmetric matrix in packed form (cofactors over the determinant).
__device__ __forceinline__ void inverse3_sym(const double m[6], double r[6]) {
  const double a00 = m[0], a01 = m[1], a02 = m[2], a11 = m[3], a12 = m[4], a22 = m[5];
  const double c00 = a11 * a22 - a12 * a12;
  const double c10 = a02 * a12 - a01 * a22;
  const double c20 = a01 * a12 - a02 * a11;
  const double det = c00 * a00 + c10 * a01 + c20 * a02;
  const double id = 1.0 / det;
  r[0] = c00 * id;
  r[1] = c10 * id;
  r[2] = c20 * id;
  r[3] = (a00 * a22 - a02 * a02) * id;
  r[4] = (a02 * a01 - a00 * a12) * id;
  r[5] = (a00 * a11 - a01 * a01) * id;
}

}  // namespace ba
}  // namespace slamgpu
