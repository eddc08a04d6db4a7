// oracle/pose_oracle.c -- CPU restatement of Optimizer::PoseOptimization (TEST INFRASTRUCTURE).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this file; the product
// path is the HIP kernel in slam_framework_amd/csrc/pose_kernels.hip.
//
// Parity status: "parity unpinned" against the reference binary. g2o (third_party/g2o) needs
// Eigen3, which is absent from this image, so the reference cannot be built. This
// file restates, in FP64 and in the reference's operation order (sequential sums in edge id
// order), what the reference executes:
//   src/optimizer/optimizer.cpp:209-411              PoseOptimization schedule
//   g2o/types/types_six_dof_expmap.h:143-202, .cpp:266-364   unary mono / stereo edges
//   g2o/types/se3quat.h:40-285                       SE3Quat (map, *, exp, normalizeRotation)
//   g2o/core/base_unary_edge.hpp:43-71               constructQuadraticForm
//   g2o/core/robust_kernel_impl.cpp:78-91            RobustKernelHuber::robustify
//   g2o/core/optimization_algorithm_levenberg.cpp:61-189   LM step, lambda init, scale
//   g2o/core/sparse_optimizer.cpp:61-114, 354-435    active errors, robust chi2, optimize, update
//   g2o/solvers/linear_solver_dense.h:65-118         6x6 Eigen LDLT (zero pivots -> 0, Eigen's
//                                                    pseudo-inverse rule; no pivoting here)
//   src/util/converter.cpp:12-42                     f32 cv::Mat <-> f64 SE3Quat
// and Eigen's Quaternion(Matrix3), quaternion product, q*v (_transformVector) and
// toRotationMatrix formulas. It is pinned by finite-difference Jacobians, the exp/log round trip
// and noise-free known-answer scenes (tests/test_pose_oracle.py).
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "orb_oracle.h"
#include "se3_oracle.h"

// ---- edges ------------------------------------------------------------------------------------
typedef struct {
  double Xw[3], obs[3], info;  // information = invSigma2 * I
  int stereo;
} edge;

// error e = obs - cam_project(T.map(Xw)); returns chi2 = e' * Omega * e
static double edge_error(const edge* E, const se3* T, const double cam[5], double e[3]) {
  double p[3];
  se3_map(T, E->Xw, p);
  if (!E->stereo) {  // project2d, then * f + c
    const double u = p[0] / p[2] * cam[0] + cam[2], v = p[1] / p[2] * cam[1] + cam[3];
    e[0] = E->obs[0] - u;
    e[1] = E->obs[1] - v;
    e[2] = 0;
    return e[0] * (E->info * e[0]) + e[1] * (E->info * e[1]);
  }
  const float invz = (float)(1.0 / p[2]);  // types_six_dof_expmap.cpp:300 (const float invz)
  const double u = p[0] * invz * cam[0] + cam[2];
  const double v = p[1] * invz * cam[1] + cam[3];
  const double ur = u - cam[4] * invz;
  e[0] = E->obs[0] - u;
  e[1] = E->obs[1] - v;
  e[2] = E->obs[2] - ur;
  return e[0] * (E->info * e[0]) + e[1] * (E->info * e[1]) + e[2] * (E->info * e[2]);
}

static void edge_jacobian(const edge* E, const se3* T, const double cam[5], double J[18]) {
  double p[3];
  se3_map(T, E->Xw, p);
  const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
  const double fx = cam[0], fy = cam[1], bf = cam[4];
  J[0] = x * y * invz_2 * fx;
  J[1] = -(1 + (x * x * invz_2)) * fx;
  J[2] = y * invz * fx;
  J[3] = -invz * fx;
  J[4] = 0;
  J[5] = x * invz_2 * fx;
  J[6] = (1 + y * y * invz_2) * fy;
  J[7] = -x * y * invz_2 * fy;
  J[8] = -x * invz * fy;
  J[9] = 0;
  J[10] = -invz * fy;
  J[11] = y * invz_2 * fy;
  if (E->stereo) {
    J[12] = J[0] - bf * y * invz_2;
    J[13] = J[1] + bf * x * invz_2;
    J[14] = J[2];
    J[15] = J[3];
    J[16] = 0;
    J[17] = J[5] - bf * invz_2;
  }
}

// 6x6 LDLT solve of H x = b; zero pivots give zero components (Eigen's pseudo-inverse rule).
static int ldlt_solve6(const double Hin[36], const double b[6], double x[6]) {
  double A[36], d[6];
  memcpy(A, Hin, sizeof(A));
  for (int j = 0; j < 6; j++) {
    double dj = A[6 * j + j];
    for (int k = 0; k < j; k++) dj -= A[6 * j + k] * A[6 * j + k] * d[k];
    d[j] = dj;
    if (dj < 0) return 0;  // not positive (semi-)definite
    for (int i = j + 1; i < 6; i++) {
      double s = A[6 * i + j];
      for (int k = 0; k < j; k++) s -= A[6 * i + k] * A[6 * j + k] * d[k];
      A[6 * i + j] = dj > DBL_MIN ? s / dj : 0.0;
    }
  }
  double y[6];
  for (int i = 0; i < 6; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= A[6 * i + k] * y[k];
    y[i] = s;
  }
  for (int i = 0; i < 6; i++) y[i] = fabs(d[i]) > DBL_MIN ? y[i] / d[i] : 0.0;
  for (int i = 5; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < 6; k++) s -= A[6 * k + i] * x[k];
    x[i] = s;
  }
  return 1;
}

typedef struct {
  int n;
  const edge* E;
  const uint8_t* active;  // level 0
  const uint8_t* robust;
  double delta_mono, delta_stereo;
  double cam[5];
  double* err;   // [n][3] stored errors (g2o keeps the last computed error per edge)
  double* chi2;  // [n]
} problem;

static void compute_active_errors(problem* P, const se3* T) {
  for (int k = 0; k < P->n; k++)
    if (P->active[k]) P->chi2[k] = edge_error(&P->E[k], T, P->cam, &P->err[3 * k]);
}

// Diagnostic only (tools/pose_schedule.py): 1 sums the chi2 and the normal equations over the
// edges in reverse order -- a different rounding of the same sums -- to measure how often the LM
// schedule (iteration count) depends on the summation order alone. 0 (default): g2o's order.
static int g_sum_reverse = 0;
void oc_pose_set_sum_reverse(int on) { g_sum_reverse = on; }
#define EDGE_LOOP(k, n) for (int k##_ = 0, k = g_sum_reverse ? (n) - 1 : 0; k##_ < (n); \
                             k##_++, k = g_sum_reverse ? (n) - 1 - k##_ : k##_)

static double active_robust_chi2(const problem* P) {
  double chi = 0.0;
  EDGE_LOOP(k, P->n) {
    if (!P->active[k]) continue;
    if (P->robust[k]) {
      double rho[3];
      huber(P->chi2[k], P->E[k].stereo ? P->delta_stereo : P->delta_mono, rho);
      chi += rho[0];
    } else {
      chi += P->chi2[k];
    }
  }
  return chi;
}

static void build_system(const problem* P, const se3* T, double H[36], double b[6]) {
  memset(H, 0, 36 * sizeof(double));
  memset(b, 0, 6 * sizeof(double));
  EDGE_LOOP(k, P->n) {
    if (!P->active[k]) continue;
    const edge* E = &P->E[k];
    double J[18];
    edge_jacobian(E, T, P->cam, J);
    const int D = E->stereo ? 3 : 2;
    double w = 1.0;  // rho'(chi2) with a robust kernel
    if (P->robust[k]) {
      double rho[3];
      huber(P->chi2[k], E->stereo ? P->delta_stereo : P->delta_mono, rho);
      w = rho[1];
    }
    const double* e = &P->err[3 * k];
    // b -= w * J' * Omega * e ; H += J' * (w * Omega) * J   (Omega = info * I)
    for (int i = 0; i < 6; i++) {
      double s = 0;
      for (int r = 0; r < D; r++) s += (J[6 * r + i] * E->info) * e[r];
      b[i] -= w * s;
      for (int j = 0; j < 6; j++) {
        double h = 0;
        for (int r = 0; r < D; r++) h += (J[6 * r + i] * (w * E->info)) * J[6 * r + j];
        H[6 * i + j] += h;
      }
    }
  }
}

// SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg.
static int optimize(problem* P, se3* T, int iterations, int* lm_iters) {
  double lambda = 0;
  int ni = 2, nbad = 0, it;
  for (it = 0; it < iterations; it++) {
    compute_active_errors(P, T);
    double currentChi = active_robust_chi2(P);
    const double iniChi = currentChi;
    double H[36], b[6];
    build_system(P, T, H, b);
    if (it == 0) {
      double maxd = 0;
      for (int j = 0; j < 6; j++) maxd = fmax(fabs(H[7 * j]), maxd);
      lambda = 1e-5 * maxd;
      ni = 2;
      nbad = 0;
    }
    double rho = 0, x[6] = {0, 0, 0, 0, 0, 0};
    int qmax = 0;
    do {
      const se3 backup = *T;  // push
      double Hl[36];
      memcpy(Hl, H, sizeof(Hl));
      for (int j = 0; j < 6; j++) Hl[7 * j] += lambda;
      const int ok2 = ldlt_solve6(Hl, b, x);  // x keeps its last value if the solve fails
      *T = se3_exp(x);                         // update: exp(dx) * T
      *T = se3_mul(T, &backup);
      compute_active_errors(P, T);
      double tempChi = active_robust_chi2(P);
      if (!ok2) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      double scale = 0;
      for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        lambda *= fmax(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;  // discardTop
      } else {
        lambda *= ni;
        ni *= 2;
        *T = backup;  // pop; the edges keep the errors of the rejected estimate
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    if (lm_iters) (*lm_iters)++;
    if (qmax == 10 || rho == 0) break;
    if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
    else nbad = 0;
    if (nbad >= 3) break;
  }
  return it;
}

int oc_pose_optimization(const float cam[5], const float* inv_sigma2, const oc_pose_edge* edges,
                         int n, float Tcw[16], uint8_t* outlier, int* lm_iterations) {
  if (lm_iterations) *lm_iterations = 0;
  int ninit = 0;
  edge E[n > 0 ? n : 1];
  for (int i = 0; i < n; i++) {
    E[i].Xw[0] = edges[i].xw[0];
    E[i].Xw[1] = edges[i].xw[1];
    E[i].Xw[2] = edges[i].xw[2];
    E[i].obs[0] = edges[i].u;
    E[i].obs[1] = edges[i].v;
    E[i].obs[2] = edges[i].ur;
    E[i].stereo = edges[i].ur >= 0;  // frame.StereoCoordRight()[i] < 0 -> monocular
    E[i].info = (double)inv_sigma2[edges[i].octave];
    outlier[i] = 0;
    ninit++;
  }
  if (ninit < 3) return 0;
  double R[9], t[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) R[3 * i + j] = Tcw[4 * i + j];
    t[i] = Tcw[4 * i + 3];
  }
  const se3 T0 = se3_from_Rt(R, t);  // Converter::toSE3Quat(frame.GetPose())
  se3 T = T0;
  uint8_t active[n], robust[n];
  double err[3 * n], chi2[n];
  for (int i = 0; i < n; i++) {
    active[i] = 1;
    robust[i] = 1;
  }
  problem P = {n, E, active, robust, (double)sqrtf(5.991f), (double)sqrtf(7.815f),
               {cam[0], cam[1], cam[2], cam[3], cam[4]}, err, chi2};
  // const float delta = std::sqrt(5.991) is the double sqrt rounded to float
  P.delta_mono = (double)(float)sqrt(5.991);
  P.delta_stereo = (double)(float)sqrt(7.815);
  int is_bad = 0;
  for (int it = 0; it < 4; it++) {
    T = T0;  // each round restarts from the frame's pose (:344)
    optimize(&P, &T, 10, lm_iterations);
    is_bad = 0;
    for (int i = 0; i < n; i++) {
      if (outlier[i]) chi2[i] = edge_error(&E[i], &T, P.cam, &err[3 * i]);
      const float c = (float)chi2[i];
      if (c > (E[i].stereo ? 7.815f : 5.991f)) {
        outlier[i] = 1;
        active[i] = 0;
        is_bad++;
      } else {
        outlier[i] = 0;
        active[i] = 1;
      }
      if (it == 2) robust[i] = 0;
    }
    if (n < 10) break;
  }
  quat_to_R(T.r, R);
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) Tcw[4 * i + j] = (float)R[3 * i + j];
    Tcw[4 * i + 3] = (float)T.t[i];
  }
  Tcw[12] = Tcw[13] = Tcw[14] = 0.f;
  Tcw[15] = 1.f;
  return ninit - is_bad;
}

// ---- exported pieces for the finite-difference / known-answer tests ----------------------------
void oc_se3_exp(const double u[6], double R[9], double t[3]) {
  const se3 T = se3_exp(u);
  quat_to_R(T.r, R);
  memcpy(t, T.t, sizeof(T.t));
}

double oc_pose_edge_eval(const float cam[5], const double R[9], const double t[3],
                         const oc_pose_edge* ed, float inv_sigma2, double e[3], double J[18]) {
  edge E;
  for (int i = 0; i < 3; i++) E.Xw[i] = ed->xw[i];
  E.obs[0] = ed->u;
  E.obs[1] = ed->v;
  E.obs[2] = ed->ur;
  E.stereo = ed->ur >= 0;
  E.info = inv_sigma2;
  const se3 T = se3_from_Rt(R, t);
  const double c[5] = {cam[0], cam[1], cam[2], cam[3], cam[4]};
  if (J) edge_jacobian(&E, &T, c, J);
  return edge_error(&E, &T, c, e);
}
