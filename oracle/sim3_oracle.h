/* oracle/sim3_oracle.h -- g2o::Sim3 arithmetic as the reference executes it (TEST INFRASTRUCTURE
 * ONLY: used by the OptimizeSim3 / OptimizeEssentialGraph restatements).
 *   g2o/types/sim3.h:70-142   Sim3(const Vector7d&)  (the exponential map, no normalisation)
 *   g2o/types/sim3.h:144-146  map: s * (r * x) + t
 *   g2o/types/sim3.h:148-230  log (acos branch, deltaR, W.lu().solve(t))
 *   g2o/types/sim3.h:233-236  inverse: (conj(r), conj(r) * ((-1/s) t), 1/s)
 *   g2o/types/sim3.h:266-272  operator*
 *   g2o/types/se3_ops.h       skew, deltaR
 * The quaternion is never normalised (Quaterniond(R) of the exponential, raw products), exactly
 * as sim3.h leaves it. Eigen's PartialPivLU (unblocked, column-major triangular solves) for the
 * 3x3 solve of log(). */
#ifndef SLAMGPU_SIM3_ORACLE_H_
#define SLAMGPU_SIM3_ORACLE_H_
#include <math.h>
#include <string.h>

#include "se3_oracle.h"

typedef struct {
  quat r;
  double t[3];
  double s;
} sim3;

static sim3 sim3_identity(void) {
  sim3 S;
  S.r.x = S.r.y = S.r.z = 0.0;
  S.r.w = 1.0;
  S.t[0] = S.t[1] = S.t[2] = 0.0;
  S.s = 1.0;
  return S;
}

static void skew3(const double w[3], double O[9]) {  // se3_ops.h skew
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

/* Sim3(const Vector7d& update): update = (omega, upsilon, sigma). */
static sim3 sim3_exp(const double u[7]) {
  const double omega[3] = {u[0], u[1], u[2]}, ups[3] = {u[3], u[4], u[5]};
  const double sigma = u[6];
  const double theta = sqrt(omega[0] * omega[0] + omega[1] * omega[1] + omega[2] * omega[2]);
  double O[9], O2[9], R[9], W[9];
  skew3(omega, O);
  sim3 S;
  S.s = exp(sigma);
  mat3_mul(O, O, O2);
  const double eps = 0.00001;
  double A, B, C;
  if (fabs(sigma) < eps) {
    C = 1;
    if (theta < eps) {
      A = 1. / 2.;
      B = 1. / 6.;
      for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
    } else {
      const double theta2 = theta * theta;
      A = (1 - cos(theta)) / (theta2);
      B = (theta - sin(theta)) / (theta2 * theta);
      const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
      for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * O[i] + b * O2[i];
    }
  } else {
    C = (S.s - 1) / sigma;
    if (theta < eps) {
      const double sigma2 = sigma * sigma;
      A = ((sigma - 1) * S.s + 1) / sigma2;
      B = ((0.5 * sigma2 - sigma + 1) * S.s) / (sigma2 * sigma);
      for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
    } else {
      const double a0 = sin(theta) / theta, b0 = (1 - cos(theta)) / (theta * theta);
      for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a0 * O[i] + b0 * O2[i];
      const double a = S.s * sin(theta);
      const double b = S.s * cos(theta);
      const double theta2 = theta * theta;
      const double sigma2 = sigma * sigma;
      const double c = theta2 + sigma2;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  S.r = quat_from_R(R);
  for (int i = 0; i < 9; i++) W[i] = A * O[i] + B * O2[i] + (i % 4 == 0 ? C : 0.0);
  for (int i = 0; i < 3; i++) S.t[i] = W[3 * i] * ups[0] + W[3 * i + 1] * ups[1] + W[3 * i + 2] * ups[2];
  return S;
}

static void sim3_map(const sim3* S, const double x[3], double o[3]) {
  double rx[3];
  quat_rotate(S->r, x, rx);
  for (int i = 0; i < 3; i++) o[i] = S->s * rx[i] + S->t[i];
}

static sim3 sim3_mul(const sim3* a, const sim3* b) {
  sim3 o;
  o.r = quat_mul(a->r, b->r);
  double rt[3];
  quat_rotate(a->r, b->t, rt);
  for (int i = 0; i < 3; i++) o.t[i] = a->s * rt[i] + a->t[i];
  o.s = a->s * b->s;
  return o;
}

static sim3 sim3_inverse(const sim3* a) {
  sim3 o;
  o.r.x = -a->r.x;
  o.r.y = -a->r.y;
  o.r.z = -a->r.z;
  o.r.w = a->r.w;
  const double k = -1. / a->s;
  const double v[3] = {k * a->t[0], k * a->t[1], k * a->t[2]};
  quat_rotate(o.r, v, o.t);
  o.s = 1. / a->s;
  return o;
}

/* Eigen PartialPivLU<Matrix3d>(W).solve(t): unblocked LU with row pivoting on the largest |a|
 * (first one on ties), column-major unit-lower then upper triangular solves. */
static void lu3_solve(const double Win[9], const double b[3], double x[3]) {
  double A[9];
  memcpy(A, Win, sizeof(A));
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
  for (int k = 0; k < 3; k++)  // unit lower, column by column
    for (int i = k + 1; i < 3; i++) y[i] -= y[k] * A[3 * i + k];
  for (int k = 2; k >= 0; k--) {  // upper, column by column from the last
    y[k] /= A[3 * k + k];
    for (int i = 0; i < k; i++) y[i] -= y[k] * A[3 * i + k];
  }
  memcpy(x, y, sizeof(y));
}

static void sim3_log(const sim3* S, double res[7]) {
  const double sigma = log(S->s);
  double omega[3], R[9], O[9], O2[9], W[9];
  quat_to_R(S->r, R);
  const double d = 0.5 * (R[0] + R[4] + R[8] - 1);
  const double dR[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};  // deltaR
  const double eps = 0.00001;
  double A, B, C;
  if (fabs(sigma) < eps) {
    C = 1;
    if (d > 1 - eps) {
      for (int i = 0; i < 3; i++) omega[i] = 0.5 * dR[i];
      A = 1. / 2.;
      B = 1. / 6.;
    } else {
      const double theta = acos(d);
      const double theta2 = theta * theta;
      const double f = theta / (2 * sqrt(1 - d * d));
      for (int i = 0; i < 3; i++) omega[i] = f * dR[i];
      A = (1 - cos(theta)) / (theta2);
      B = (theta - sin(theta)) / (theta2 * theta);
    }
  } else {
    C = (S->s - 1) / sigma;
    if (d > 1 - eps) {
      const double sigma2 = sigma * sigma;
      for (int i = 0; i < 3; i++) omega[i] = 0.5 * dR[i];
      A = ((sigma - 1) * S->s + 1) / (sigma2);
      B = ((0.5 * sigma2 - sigma + 1) * S->s) / (sigma2 * sigma);
    } else {
      const double theta = acos(d);
      const double f = theta / (2 * sqrt(1 - d * d));
      for (int i = 0; i < 3; i++) omega[i] = f * dR[i];
      const double theta2 = theta * theta;
      const double a = S->s * sin(theta);
      const double b = S->s * cos(theta);
      const double c = theta2 + sigma * sigma;
      A = (a * sigma + (1 - b) * theta) / (theta * c);
      B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
    }
  }
  skew3(omega, O);
  mat3_mul(O, O, O2);
  for (int i = 0; i < 9; i++) W[i] = A * O[i] + B * O2[i] + (i % 4 == 0 ? C : 0.0);
  double ups[3];
  lu3_solve(W, S->t, ups);
  for (int i = 0; i < 3; i++) {
    res[i] = omega[i];
    res[i + 3] = ups[i];
  }
  res[6] = sigma;
}

/* g2o's operator[] layout: r.coeffs() (x, y, z, w), t, s. */
static sim3 sim3_load(const double v[8]) {
  sim3 S;
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
static void sim3_store(const sim3* S, double v[8]) {
  v[0] = S->r.x;
  v[1] = S->r.y;
  v[2] = S->r.z;
  v[3] = S->r.w;
  v[4] = S->t[0];
  v[5] = S->t[1];
  v[6] = S->t[2];
  v[7] = S->s;
}

#endif
