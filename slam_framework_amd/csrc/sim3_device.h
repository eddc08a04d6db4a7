// sim3_device.h -- g2o::Sim3 arithmetic on the device (FP64), as g2o/types/sim3.h executes it:
// the exponential map of Sim3(const Vector7d&) (sim3.h:70-142), operator* (:266-272),
// inverse (:233-236), log (:148-230), map (:144-146). The quaternion is never normalised, as in
// sim3.h. Passes apply a Sim3 as the affine map x -> (s R(q)) x + t, R(q) = Eigen's
// toRotationMatrix, which is the same polynomial in q as Eigen's q * v (also for |q| != 1).
#pragma once
#include <hip/hip_runtime.h>

#include "se3_device.h"

namespace slamgpu {
namespace sim3 {

using se3::Quat;

struct Sim3 {
  Quat r;
  double t[3];
  double s;
};

__device__ __forceinline__ void skew(const double w[3], double O[9]) {
  O[0] = 0;
  O[1] = -w[2];
  O[2] = w[1];
  O[3] = w[2];
  O[4] = 0;
  O[5] = -w[0];
  O[6] = -w[1];
  O[7] = w[0];
  O[8] = 0;
}

__device__ __forceinline__ void mat3_mul(const double A[9], const double B[9], double C[9]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// Sim3(const Vector7d& update), update = (omega, upsilon, sigma).
__device__ inline Sim3 sim3_exp(const double u[7]) {
  const double omega[3] = {u[0], u[1], u[2]};
  const double sigma = u[6];
  const double theta = sqrt(omega[0] * omega[0] + omega[1] * omega[1] + omega[2] * omega[2]);
  double O[9], O2[9];
  skew(omega, O);
  mat3_mul(O, O, O2);
  Sim3 S;
  S.s = exp(sigma);
  const double eps = 0.00001;
  double A, B, C, ra = 1.0, rb = 1.0;  // R = I + ra O + rb O^2 (small angle: ra = rb = 1)
  if (!(theta < eps)) {
    double sn, cs;
    sincos(theta, &sn, &cs);
    ra = sn / theta;
    rb = (1 - cs) / (theta * theta);
  }
  if (fabs(sigma) < eps) {
    C = 1;
    if (theta < eps) {
      A = 1. / 2.;
      B = 1. / 6.;
    } else {
      double sn, cs;
      sincos(theta, &sn, &cs);
      const double theta2 = theta * theta;
      A = (1 - cs) / (theta2);
      B = (theta - sn) / (theta2 * theta);
    }
  } else {
    C = (S.s - 1) / sigma;
    if (theta < eps) {
      const double sigma2 = sigma * sigma;
      A = ((sigma - 1) * S.s + 1) / sigma2;
      B = ((0.5 * sigma2 - sigma + 1) * S.s) / (sigma2 * sigma);
    } else {
      double sn, cs;
      sincos(theta, &sn, &cs);
      const double a = S.s * sn, b = S.s * cs;
      const double theta2 = theta * theta, sigma2 = sigma * sigma;
      const double c = theta2 + sigma2;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  double R[9], W[9];
  for (int i = 0; i < 9; i++) {
    const double I = (i % 4 == 0) ? 1.0 : 0.0;
    R[i] = I + ra * O[i] + rb * O2[i];
    W[i] = A * O[i] + B * O2[i] + (i % 4 == 0 ? C : 0.0);
  }
  S.r = se3::quat_from_R(R);
  for (int i = 0; i < 3; i++) S.t[i] = W[3 * i] * u[3] + W[3 * i + 1] * u[4] + W[3 * i + 2] * u[5];
  return S;
}

__device__ __forceinline__ Quat quat_mul(const Quat& p, const Quat& q) {  // Eigen quat_product
  Quat o;
  o.w = p.w * q.w - p.x * q.x - p.y * q.y - p.z * q.z;
  o.x = p.w * q.x + p.x * q.w + p.y * q.z - p.z * q.y;
  o.y = p.w * q.y + p.y * q.w + p.z * q.x - p.x * q.z;
  o.z = p.w * q.z + p.z * q.w + p.x * q.y - p.y * q.x;
  return o;
}

__device__ inline Sim3 sim3_mul(const Sim3& a, const Sim3& b) {
  Sim3 o;
  o.r = quat_mul(a.r, b.r);
  double rt[3];
  se3::quat_rotate(a.r, b.t, rt);
  for (int i = 0; i < 3; i++) o.t[i] = a.s * rt[i] + a.t[i];
  o.s = a.s * b.s;
  return o;
}

__device__ inline Sim3 sim3_inverse(const Sim3& a) {
  Sim3 o;
  o.r.x = -a.r.x;
  o.r.y = -a.r.y;
  o.r.z = -a.r.z;
  o.r.w = a.r.w;
  const double k = -1. / a.s;
  const double v[3] = {k * a.t[0], k * a.t[1], k * a.t[2]};
  se3::quat_rotate(o.r, v, o.t);
  o.s = 1. / a.s;
  return o;
}

// x -> M[0..8] x + M[9..11]
__device__ __forceinline__ void sim3_affine(const Sim3& S, double M[12]) {
  double R[9];
  se3::quat_to_R(S.r, R);
  for (int i = 0; i < 9; i++) M[i] = S.s * R[i];
  M[9] = S.t[0];
  M[10] = S.t[1];
  M[11] = S.t[2];
}

// Eigen PartialPivLU<Matrix3d>(W).solve(b) (oracle/sim3_oracle.h lu3_solve).
__device__ inline void lu3_solve(const double Win[9], const double b[3], double x[3]) {
  double A[9];
  for (int i = 0; i < 9; i++) A[i] = Win[i];
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < 3; k++) {
    int p = k;
    double big = fabs(A[3 * k + k]);
    for (int i = k + 1; i < 3; i++)
      if (fabs(A[3 * i + k]) > big) {
        big = fabs(A[3 * i + k]);
        p = i;
      }
    if (big != 0.0) {
      if (p != k) {
        for (int j = 0; j < 3; j++) {
          const double tmp = A[3 * k + j];
          A[3 * k + j] = A[3 * p + j];
          A[3 * p + j] = tmp;
        }
        const int tp = perm[k];
        perm[k] = perm[p];
        perm[p] = tp;
      }
      for (int i = k + 1; i < 3; i++) A[3 * i + k] /= A[3 * k + k];
    }
    for (int i = k + 1; i < 3; i++)
      for (int j = k + 1; j < 3; j++) A[3 * i + j] -= A[3 * i + k] * A[3 * k + j];
  }
  double y[3] = {b[perm[0]], b[perm[1]], b[perm[2]]};
  for (int k = 0; k < 3; k++)
    for (int i = k + 1; i < 3; i++) y[i] -= y[k] * A[3 * i + k];
  for (int k = 2; k >= 0; k--) {
    y[k] /= A[3 * k + k];
    for (int i = 0; i < k; i++) y[i] -= y[k] * A[3 * i + k];
  }
  x[0] = y[0];
  x[1] = y[1];
  x[2] = y[2];
}

__device__ inline void sim3_log(const Sim3& S, double res[7]) {
  const double sigma = log(S.s);
  double R[9], O[9], O2[9], W[9], omega[3];
  se3::quat_to_R(S.r, R);
  const double d = 0.5 * (R[0] + R[4] + R[8] - 1);
  const double dR[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
  const double eps = 0.00001;
  double A, B, C;
  if (fabs(sigma) < eps) {
    C = 1;
    if (d > 1 - eps) {
      for (int i = 0; i < 3; i++) omega[i] = 0.5 * dR[i];
      A = 1. / 2.;
      B = 1. / 6.;
    } else {
      const double theta = acos(d), theta2 = theta * theta;
      const double f = theta / (2 * sqrt(1 - d * d));
      for (int i = 0; i < 3; i++) omega[i] = f * dR[i];
      double sn, cs;
      sincos(theta, &sn, &cs);
      A = (1 - cs) / (theta2);
      B = (theta - sn) / (theta2 * theta);
    }
  } else {
    C = (S.s - 1) / sigma;
    if (d > 1 - eps) {
      const double sigma2 = sigma * sigma;
      for (int i = 0; i < 3; i++) omega[i] = 0.5 * dR[i];
      A = ((sigma - 1) * S.s + 1) / (sigma2);
      B = ((0.5 * sigma2 - sigma + 1) * S.s) / (sigma2 * sigma);
    } else {
      const double theta = acos(d);
      const double f = theta / (2 * sqrt(1 - d * d));
      for (int i = 0; i < 3; i++) omega[i] = f * dR[i];
      double sn, cs;
      sincos(theta, &sn, &cs);
      const double theta2 = theta * theta;
      const double a = S.s * sn, b = S.s * cs;
      const double c = theta2 + sigma * sigma;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  skew(omega, O);
  mat3_mul(O, O, O2);
  for (int i = 0; i < 9; i++) W[i] = A * O[i] + B * O2[i] + (i % 4 == 0 ? C : 0.0);
  double ups[3];
  lu3_solve(W, S.t, ups);
  for (int i = 0; i < 3; i++) {
    res[i] = omega[i];
    res[i + 3] = ups[i];
  }
  res[6] = sigma;
}

__device__ __forceinline__ Sim3 sim3_load(const double v[8]) {
  Sim3 S;
  S.r.x = v[0];
  S.r.y = v[1];
  S.r.z = v[2];
  S.r.w = v[3];
  S.t[0] = v[4];
  S.t[1] = v[5];
  S.t[2] = v[6];
  S.s = v[7];
  return S;
}

__device__ __forceinline__ void sim3_store(const Sim3& S, double v[8]) {
  v[0] = S.r.x;
  v[1] = S.r.y;
  v[2] = S.r.z;
  v[3] = S.r.w;
  v[4] = S.t[0];
  v[5] = S.t[1];
  v[6] = S.t[2];
  v[7] = S.s;
}

}  // namespace sim3
}  // namespace slamgpu
