/* oracle/se3_oracle.h -- g2o SE3Quat / Eigen quaternion arithmetic and the Huber kernel, shared by
 * the PoseOptimization and LocalBundleAdjustment restatements (TEST INFRASTRUCTURE ONLY).
 *   g2o/types/se3quat.h:40-285  SE3Quat (map, *, exp, normalizeRotation)
 *   g2o/core/robust_kernel_impl.cpp:78-91  RobustKernelHuber::robustify
 * plus Eigen's Quaternion(Matrix3), quaternion product, q*v (_transformVector) and
 * toRotationMatrix formulas. */
#ifndef SLAMGPU_SE3_ORACLE_H_
#define SLAMGPU_SE3_ORACLE_H_
#include <math.h>
#include <string.h>

typedef struct {
  double x, y, z, w;
} quat;
typedef struct {
  quat r;
  double t[3];
} se3;

static quat quat_from_R(const double R[9]) {  // Eigen quaternionbase_assign_impl<Matrix3>
  quat q;
  double t = R[0] + R[4] + R[8];
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (R[7] - R[5]) * t;
    q.y = (R[2] - R[6]) * t;
    q.z = (R[3] - R[1]) * t;
  } else {
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[3 * i + i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    t = sqrt(R[3 * i + i] - R[3 * j + j] - R[3 * k + k] + 1.0);
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (R[3 * k + j] - R[3 * j + k]) * t;
    c[j] = (R[3 * j + i] + R[3 * i + j]) * t;
    c[k] = (R[3 * k + i] + R[3 * i + k]) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
  }
  return q;
}

static void quat_normalize_rotation(quat* q) {  // SE3Quat::normalizeRotation
  if (q->w < 0) {
    q->x = -q->x;
    q->y = -q->y;
    q->z = -q->z;
    q->w = -q->w;
  }
  const double n = sqrt(q->x * q->x + q->y * q->y + q->z * q->z + q->w * q->w);
  q->x /= n;
  q->y /= n;
  q->z /= n;
  q->w /= n;
}

static quat quat_mul(quat a, quat b) {  // Eigen quat_product
  quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

static void quat_rotate(quat q, const double v[3], double o[3]) {  // Eigen _transformVector
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2],
                       q.x * uv[1] - q.y * uv[0]};
  for (int i = 0; i < 3; i++) o[i] = v[i] + q.w * uv[i] + c[i];
}

static void quat_to_R(quat q, double R[9]) {  // Eigen toRotationMatrix
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

static se3 se3_from_Rt(const double R[9], const double t[3]) {  // SE3Quat(R, t)
  se3 T;
  T.r = quat_from_R(R);
  quat_normalize_rotation(&T.r);
  memcpy(T.t, t, sizeof(T.t));
  return T;
}

static void se3_map(const se3* T, const double X[3], double o[3]) {  // _r*xyz + _t
  quat_rotate(T->r, X, o);
  for (int i = 0; i < 3; i++) o[i] += T->t[i];
}

static se3 se3_mul(const se3* a, const se3* b) {  // SE3Quat::operator*
  se3 r = *a;
  double rt[3];
  quat_rotate(a->r, b->t, rt);
  for (int i = 0; i < 3; i++) r.t[i] += rt[i];
  r.r = quat_mul(a->r, b->r);
  quat_normalize_rotation(&r.r);
  return r;
}

static void mat3_mul(const double A[9], const double B[9], double C[9]) {  // Eigen lazy product
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

static se3 se3_exp(const double u[6]) {  // SE3Quat::exp (se3quat.h:223-257)
  const double w[3] = {u[0], u[1], u[2]}, ups[3] = {u[3], u[4], u[5]};
  const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double O2[9], R[9], V[9];
  mat3_mul(O, O, O2);
  if (theta < 0.00001) {
    for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
    memcpy(V, R, sizeof(R));
  } else {
    const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
    const double c = (theta - sin(theta)) / pow(theta, 3);
    for (int i = 0; i < 9; i++) {
      R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * O[i] + b * O2[i];
      V[i] = (i % 4 == 0 ? 1.0 : 0.0) + b * O[i] + c * O2[i];
    }
  }
  double t[3];
  for (int i = 0; i < 3; i++) t[i] = V[3 * i] * ups[0] + V[3 * i + 1] * ups[1] + V[3 * i + 2] * ups[2];
  return se3_from_Rt(R, t);
}

static void huber(double e, double delta, double rho[3]) {  // RobustKernelHuber::robustify
  const double dsqr = delta * delta;
  if (e <= dsqr) {
    rho[0] = e;
    rho[1] = 1.;
    rho[2] = 0.;
  } else {
    const double sqrte = sqrt(e);
    rho[0] = 2 * sqrte * delta - dsqr;
    rho[1] = delta / sqrte;
    rho[2] = -0.5 * rho[1] / e;
  }
}

#endif /* SLAMGPU_SE3_ORACLE_H_ */
