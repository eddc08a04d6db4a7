// se3_device.h -- g2o SE3Quat arithmetic on the device (FP64), shared by the pose and local BA
// kernels: Eigen's Quaternion(Matrix3), normalizeRotation, q * v, toRotationMatrix, and the
// left-multiplicative update exp(dx) * T of VertexSE3Expmap::oplusImpl.
#pragma once
#include <hip/hip_runtime.h>

namespace slamgpu {
namespace se3 {

struct Quat {
  double x, y, z, w;
};
struct SE3 {
  Quat r;
  double t[3];
};

// Eigen Quaternion(const Matrix3&): Shepperd's method on the largest diagonal term.
__device__ inline Quat quat_from_R(const double R[9]) {
  Quat q;
  const double tr = R[0] + R[4] + R[8];
  if (tr > 0.0) {
    double t = sqrt(tr + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (R[7] - R[5]) * t;
    q.y = (R[2] - R[6]) * t;
    q.z = (R[3] - R[1]) * t;
  } else if (R[4] <= R[0] && R[8] <= R[0]) {  // i = 0
    double t = sqrt(R[0] - R[4] - R[8] + 1.0);
    q.x = 0.5 * t;
    t = 0.5 / t;
    q.w = (R[7] - R[5]) * t;
    q.y = (R[3] + R[1]) * t;
    q.z = (R[6] + R[2]) * t;
  } else if (R[8] <= (R[4] > R[0] ? R[4] : R[0]) && R[4] > R[0]) {  // i = 1
    double t = sqrt(R[4] - R[8] - R[0] + 1.0);
    q.y = 0.5 * t;
    t = 0.5 / t;
    q.w = (R[2] - R[6]) * t;
    q.z = (R[7] + R[5]) * t;
    q.x = (R[1] + R[3]) * t;
  } else {  // i = 2
    double t = sqrt(R[8] - R[0] - R[4] + 1.0);
    q.z = 0.5 * t;
    t = 0.5 / t;
    q.w = (R[3] - R[1]) * t;
    q.x = (R[2] + R[6]) * t;
    q.y = (R[5] + R[7]) * t;
  }
  return q;
}

// SE3Quat::normalizeRotation (se3quat.h:280-285): w >= 0, unit norm.
__device__ inline void normalize_rotation(Quat& q) {
  if (q.w < 0) {
    q.x = -q.x;
    q.y = -q.y;
    q.z = -q.z;
    q.w = -q.w;
  }
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n;
  q.y /= n;
  q.z /= n;
  q.w /= n;
}

// q * v as Eigen evaluates it: v + 2w(q_v x v) + q_v x (2 q_v x v).
__device__ __forceinline__ void quat_rotate(const Quat& q, const double v[3], double o[3]) {
  double a = q.y * v[2] - q.z * v[1], b = q.z * v[0] - q.x * v[2], c = q.x * v[1] - q.y * v[0];
  a += a;
  b += b;
  c += c;
  o[0] = v[0] + q.w * a + (q.y * c - q.z * b);
  o[1] = v[1] + q.w * b + (q.z * a - q.x * c);
  o[2] = v[2] + q.w * c + (q.x * b - q.y * a);
}

__device__ inline void quat_to_R(const Quat& q, double R[9]) {  // Eigen toRotationMatrix
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz);
  R[1] = txy - twz;
  R[2] = txz + twy;
  R[3] = txy + twz;
  R[4] = 1 - (txx + tzz);
  R[5] = tyz - twx;
  R[6] = txz - twy;
  R[7] = tyz + twx;
  R[8] = 1 - (txx + tyy);
}

// exp(dx) * T, VertexSE3Expmap::oplusImpl (types_six_dof_expmap.h:73-76) with SE3Quat::exp
// (se3quat.h:223-257) and operator* (:92-99). dx = [omega, upsilon].
__device__ inline SE3 se3_left_update(const double u[6], const SE3& T) {
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double th = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
  double O2[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
  double a = 1.0, b = 1.0, c = 1.0;  // small-angle branch: R = V = I + O + O^2
  if (!(th < 0.00001)) {
    double s, co;
    sincos(th, &s, &co);
    a = s / th;
    b = (1 - co) / (th * th);
    c = (th - s) / (th * th * th);
  }
  double R[9], V[9];
  for (int i = 0; i < 9; i++) {
    const double I = (i % 4 == 0) ? 1.0 : 0.0;
    R[i] = I + a * O[i] + b * O2[i];
    V[i] = I + b * O[i] + c * O2[i];
  }
  SE3 E;
  for (int i = 0; i < 3; i++) E.t[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
  E.r = quat_from_R(R);
  normalize_rotation(E.r);
  SE3 out;  // E * T
  double rt[3];
  quat_rotate(E.r, T.t, rt);
  for (int i = 0; i < 3; i++) out.t[i] = E.t[i] + rt[i];
  const Quat& p = E.r;
  const Quat& q = T.r;
  out.r.w = p.w * q.w - p.x * q.x - p.y * q.y - p.z * q.z;
  out.r.x = p.w * q.x + p.x * q.w + p.y * q.z - p.z * q.y;
  out.r.y = p.w * q.y + p.y * q.w + p.z * q.x - p.x * q.z;
  out.r.z = p.w * q.z + p.z * q.w + p.x * q.y - p.y * q.x;
  normalize_rotation(out.r);
  return out;
}

}  // namespace se3
}  // namespace slamgpu
