// oracle/ba_oracle.c -- CPU restatement of Optimizer::LocalBundleAdjustment (TEST INFRASTRUCTURE).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this file; the product
// path is slam_framework_amd/csrc/ba_kernels.hip.
//
// Parity status: "parity unpinned" against the reference binary -- g2o needs Eigen3, absent from
// this image. This restates, in FP64 and in the reference's order of operations
// (edges in insertion order: map points in order, each point's observations in order):
//   src/optimizer/optimizer.cpp:413-716            graph, 5 robust + 10 plain LM iterations,
//                                                   level-1 outliers, erase list, write-back
//   g2o/types/types_six_dof_expmap.h:80-141, .cpp:103-234   EdgeSE3ProjectXYZ /
//                                                   EdgeStereoSE3ProjectXYZ (error, Jacobians,
//                                                   isDepthPositive; stereo bf passed as float)
//   g2o/types/types_sba.h:52-56                     VertexSBAPointXYZ::oplusImpl (X += dx)
//   g2o/core/base_binary_edge.hpp:55-122            constructQuadraticForm (Hll, Hpp, Hpl, b)
//   g2o/core/block_solver.hpp:351-600               Schur complement on the points, setLambda on
//                                                   every diagonal block, back-substitution
//   g2o/solvers/linear_solver_eigen.h:94-120        LDLT of the reduced pose system (fails only on
//                                                   an exact zero pivot); in keyframe order on the
//                                                   block profile (skyline) instead of Eigen's AMD
//                                                   permutation -- the same solution to rounding
//   g2o/core/optimization_algorithm_levenberg.cpp   as in pose_oracle.c
// Eigen's 3x3 inverse (cofactors over the determinant) inverts each point block.
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"
#include "se3_oracle.h"

typedef struct {
  int n_kf, n_pts, n_obs, n_free;
  const oc_ba_obs* obs;
  const int32_t* pstart;  // [n_pts + 1]
  int32_t* opoint;        // point of each edge
  int* free_idx;          // KF -> free index or -1
  double cam[5];
  float bf_f;
  const float* isig;
  se3* T;                 // every KF
  double* X;              // [n_pts][3]
  uint8_t* active;        // level 0
  int robust;
  double delta_mono, delta_stereo;  // Huber deltas of the robust kernels
  double* err;            // [n_obs][3] last computed error
  double* chi2;           // [n_obs]
  // linear system
  double* Hpp;  // [n_free][36]
  double* bp;   // [n_free][6]
  double* Hll;  // [n_pts][9]
  double* bl;   // [n_pts][3]
  double* Hpl;  // [n_obs][18] (6 x 3, pose rows x point columns)
  int* kf_nact;   // active edges per KF
  int* pt_nact;   // active edges per point
  // g2o's force-stop flag (optimizer.cpp:474-476): reads false for the first stop_after polls
  // and true from then on (stop_after < 0: never raised)
  int stop_after, polls;
} ba;

// SparseOptimizer::terminate() (sparse_optimizer.h:188), polled where g2o and the reference poll
// *stop_flag: the optimize() loop condition (sparse_optimizer.cpp:376), the Levenberg trial loop
// (optimization_algorithm_levenberg.cpp:149), before optimising and before the second
// optimize() (optimizer.cpp:616-627).
static int terminate_(ba* B) {
  if (B->stop_after < 0) return 0;
  return B->polls++ >= B->stop_after;
}

static int is_stereo(const oc_ba_obs* o) { return o->ur >= 0; }

// e = obs - cam_project(T.map(X)); returns chi2. Xc receives the camera coordinates.
static double ba_error(const ba* B, int e, double err[3], double Xc[3]) {
  const oc_ba_obs* o = &B->obs[e];
  se3_map(&B->T[o->keyframe], &B->X[3 * B->opoint[e]], Xc);
  const double* cam = B->cam;
  const double info = (double)B->isig[o->octave];
  if (!is_stereo(o)) {  // EdgeSE3ProjectXYZ::cam_project: project2d, * f + c
    const double u = Xc[0] / Xc[2] * cam[0] + cam[2], v = Xc[1] / Xc[2] * cam[1] + cam[3];
    err[0] = (double)o->u - u;
    err[1] = (double)o->v - v;
    err[2] = 0;
    return err[0] * (info * err[0]) + err[1] * (info * err[1]);
  }
  // EdgeStereoSE3ProjectXYZ::cam_project(trans_xyz, const float& bf): float invz, and bf * invz
  // is a float product (types_six_dof_expmap.cpp:150-157)
  const float invz = (float)(1.0 / Xc[2]);
  const double u = Xc[0] * invz * cam[0] + cam[2];
  const double v = Xc[1] * invz * cam[1] + cam[3];
  const float bfz = B->bf_f * invz;
  const double ur = u - (double)bfz;
  err[0] = (double)o->u - u;
  err[1] = (double)o->v - v;
  err[2] = (double)o->ur - ur;
  return err[0] * (info * err[0]) + err[1] * (info * err[1]) + err[2] * (info * err[2]);
}

// Jl (D x 3, wrt the point) and Jp (D x 6, wrt the pose), types_six_dof_expmap.cpp:103-137, 188-234
static void ba_jacobians(const ba* B, int e, double Jl[9], double Jp[18]) {
  const oc_ba_obs* o = &B->obs[e];
  const se3* T = &B->T[o->keyframe];
  double Xc[3], R[9];
  se3_map(T, &B->X[3 * B->opoint[e]], Xc);
  quat_to_R(T->r, R);
  const double x = Xc[0], y = Xc[1], z = Xc[2], z_2 = z * z;
  const double fx = B->cam[0], fy = B->cam[1], bf = B->cam[4];
  if (!is_stereo(o)) {
    const double tmp[6] = {fx, 0, -x / z * fx, 0, fy, -y / z * fy};
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += (-1. / z * tmp[3 * i + k]) * R[3 * k + j];
        Jl[3 * i + j] = s;
      }
  } else {
    for (int j = 0; j < 3; j++) {
      Jl[j] = -fx * R[j] / z + fx * x * R[6 + j] / z_2;
      Jl[3 + j] = -fy * R[3 + j] / z + fy * y * R[6 + j] / z_2;
      Jl[6 + j] = Jl[j] - bf * R[6 + j] / z_2;
    }
  }
  Jp[0] = x * y / z_2 * fx;
  Jp[1] = -(1 + (x * x / z_2)) * fx;
  Jp[2] = y / z * fx;
  Jp[3] = -1. / z * fx;
  Jp[4] = 0;
  Jp[5] = x / z_2 * fx;
  Jp[6] = (1 + y * y / z_2) * fy;
  Jp[7] = -x * y / z_2 * fy;
  Jp[8] = -x / z * fy;
  Jp[9] = 0;
  Jp[10] = -1. / z * fy;
  Jp[11] = y / z_2 * fy;
  if (is_stereo(o)) {
    Jp[12] = Jp[0] - bf * y / z_2;
    Jp[13] = Jp[1] + bf * x / z_2;
    Jp[14] = Jp[2];
    Jp[15] = Jp[3];
    Jp[16] = 0;
    Jp[17] = Jp[5] - bf / z_2;
  }
}

static void compute_active_errors(ba* B) {
  double Xc[3];
  for (int e = 0; e < B->n_obs; e++)
    if (B->active[e]) B->chi2[e] = ba_error(B, e, &B->err[3 * e], Xc);
}

static double delta_of(const ba* B, const oc_ba_obs* o) {
  return is_stereo(o) ? B->delta_stereo : B->delta_mono;
}

static double active_robust_chi2(const ba* B) {
  double chi = 0;
  for (int e = 0; e < B->n_obs; e++) {
    if (!B->active[e]) continue;
    if (B->robust) {
      double rho[3];
      huber(B->chi2[e], delta_of(B, &B->obs[e]), rho);
      chi += rho[0];
    } else {
      chi += B->chi2[e];
    }
  }
  return chi;
}

static void build_system(ba* B) {
  memset(B->Hpp, 0, sizeof(double) * 36 * B->n_free);
  memset(B->bp, 0, sizeof(double) * 6 * B->n_free);
  memset(B->Hll, 0, sizeof(double) * 9 * B->n_pts);
  memset(B->bl, 0, sizeof(double) * 3 * B->n_pts);
  for (int e = 0; e < B->n_obs; e++) {
    if (!B->active[e]) continue;
    const oc_ba_obs* o = &B->obs[e];
    const int D = is_stereo(o) ? 3 : 2, p = B->opoint[e], k = B->free_idx[o->keyframe];
    double Jl[9], Jp[18];
    ba_jacobians(B, e, Jl, Jp);
    const double info = (double)B->isig[o->octave];
    double w = 1.0;
    if (B->robust) {
      double rho[3];
      huber(B->chi2[e], delta_of(B, o), rho);
      w = rho[1];
    }
    const double* er = &B->err[3 * e];
    double omega_r[3];  // -Omega e (* rho')
    for (int r = 0; r < D; r++) omega_r[r] = -(info * er[r]) * w;
    const double W = w * info;
    double* Hll = &B->Hll[9 * p];
    double* bl = &B->bl[3 * p];
    for (int i = 0; i < 3; i++) {
      for (int r = 0; r < D; r++) bl[i] += Jl[3 * r + i] * omega_r[r];
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int r = 0; r < D; r++) s += (Jl[3 * r + i] * W) * Jl[3 * r + j];
        Hll[3 * i + j] += s;
      }
    }
    if (k < 0) continue;  // fixed keyframe: only the point block
    double* Hpp = &B->Hpp[36 * k];
    double* bp = &B->bp[6 * k];
    double* Hpl = &B->Hpl[18 * e];
    for (int i = 0; i < 6; i++) {
      for (int r = 0; r < D; r++) bp[i] += Jp[6 * r + i] * omega_r[r];
      for (int j = 0; j < 6; j++) {
        double s = 0;
        for (int r = 0; r < D; r++) s += (Jp[6 * r + i] * W) * Jp[6 * r + j];
        Hpp[6 * i + j] += s;
      }
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int r = 0; r < D; r++) s += (Jp[6 * r + i] * W) * Jl[3 * r + j];
        Hpl[3 * i + j] = s;
      }
    }
  }
}

// Eigen's 3x3 inverse: cofactor column 0, det = cofactors . col 0, result = adjugate / det.
static void inverse3(const double m[9], double r[9]) {
#define M(i, j) m[3 * (i) + (j)]
  const double c00 = M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1);
  const double c10 = M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2);  // cofactor_3x3<0,1>
  const double c20 = M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1);
  const double det = c00 * M(0, 0) + c10 * M(1, 0) + c20 * M(2, 0);
  const double id = 1.0 / det;
  r[0] = c00 * id;
  r[1] = c10 * id;
  r[2] = c20 * id;
  r[3] = (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * id;
  r[4] = (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * id;
  r[5] = (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * id;
  r[6] = (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * id;
  r[7] = (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * id;
  r[8] = (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * id;
#undef M
}

// The reduced system in block-profile (skyline) storage: scalar row i holds columns fc(i) ..
// i, fc(i) = 6 * first[i / 6] (first[k] = the smallest optimised keyframe sharing a point with
// k), at L[rb[i] + k]. The LDLT's fill-in stays inside this envelope, and the loops below are the
// dense LDLT's with the terms outside it -- exact zeros -- skipped, in the same order: the same
// numbers as the dense factorisation (no pivoting; fails on d == 0).
typedef struct {
  int n;
  int* fc;        // [n] first column of each row
  int64_t* rb;    // [n] row base: element (i, k) at L[rb[i] + k]
  double* L;
} profile_mat;

static int profile_init(profile_mat* P, const ba* B) {
  const int K = B->n_free, n = 6 * K;
  int* first = (int*)malloc(sizeof(int) * (K > 0 ? K : 1));
  for (int k = 0; k < K; k++) first[k] = k;
  for (int p = 0; p < B->n_pts; p++) {
    int mn = K;
    for (int e = B->pstart[p]; e < B->pstart[p + 1]; e++) {
      const int k = B->free_idx[B->obs[e].keyframe];
      if (k >= 0 && k < mn) mn = k;
    }
    for (int e = B->pstart[p]; e < B->pstart[p + 1]; e++) {
      const int k = B->free_idx[B->obs[e].keyframe];
      if (k >= 0 && mn < first[k]) first[k] = mn;
    }
  }
  P->n = n;
  P->fc = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
  P->rb = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
  int64_t nnz = 0;
  for (int i = 0; i < n; i++) {
    P->fc[i] = 6 * first[i / 6];
    P->rb[i] = nnz - P->fc[i];
    nnz += i - P->fc[i] + 1;
  }
  free(first);
  P->L = (double*)calloc((size_t)nnz + 1, sizeof(double));
  return P->L != NULL;
}

static void profile_free(profile_mat* P) {
  free(P->fc);
  free(P->rb);
  free(P->L);
}

#define PL(P, i, k) ((P)->L[(P)->rb[i] + (k)])

static int ldlt_solve_profile(profile_mat* P, const double* b, double* x) {
  const int n = P->n;
  double* d = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  for (int j = 0; j < n; j++) {
    double dj = PL(P, j, j);
    for (int k = P->fc[j]; k < j; k++) dj -= PL(P, j, k) * PL(P, j, k) * d[k];
    if (dj == 0.0) {
      free(d);
      return 0;
    }
    d[j] = dj;
    for (int i = j + 1; i < n; i++) {
      if (P->fc[i] > j) continue;  // L(i, j) = 0 outside the envelope
      double s = PL(P, i, j);
      const int k0 = P->fc[i] > P->fc[j] ? P->fc[i] : P->fc[j];
      for (int k = k0; k < j; k++) s -= PL(P, i, k) * PL(P, j, k) * d[k];
      PL(P, i, j) = s / dj;
    }
  }
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = P->fc[i]; k < i; k++) s -= PL(P, i, k) * x[k];
    x[i] = s;
  }
  for (int i = 0; i < n; i++) x[i] /= d[i];
  for (int i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int k = i + 1; k < n; k++)
      if (P->fc[k] <= i) s -= PL(P, k, i) * x[k];
    x[i] = s;
  }
  free(d);
  return 1;
}

// BlockSolver::solve with lambda on every diagonal block: xp (poses), xl (points).
static int schur_solve(ba* B, double lambda, double* xp, double* xl, double* Dinv) {
  const int n = 6 * B->n_free;
  profile_mat S;
  if (!profile_init(&S, B)) return 0;
  double* bs = (double*)malloc(sizeof(double) * (n + 1));
  for (int k = 0; k < B->n_free; k++)
    for (int i = 0; i < 6; i++) {
      for (int j = 0; j <= i; j++) PL(&S, 6 * k + i, 6 * k + j) = B->Hpp[36 * k + 6 * i + j];
      PL(&S, 6 * k + i, 6 * k + i) += lambda;
      bs[6 * k + i] = B->bp[6 * k + i];
    }
  for (int p = 0; p < B->n_pts; p++) {
    double D[9];
    memcpy(D, &B->Hll[9 * p], sizeof(D));
    for (int i = 0; i < 3; i++) D[4 * i] += lambda;
    double* Di = &Dinv[9 * p];
    inverse3(D, Di);
    double db[3];
    for (int i = 0; i < 3; i++)
      db[i] = Di[3 * i] * B->bl[3 * p] + Di[3 * i + 1] * B->bl[3 * p + 1] + Di[3 * i + 2] * B->bl[3 * p + 2];
    for (int e1 = B->pstart[p]; e1 < B->pstart[p + 1]; e1++) {
      const int k1 = B->free_idx[B->obs[e1].keyframe];
      if (!B->active[e1] || k1 < 0) continue;
      const double* B1 = &B->Hpl[18 * e1];
      double BD[18];
      for (int i = 0; i < 6; i++)
        for (int j = 0; j < 3; j++)
          BD[3 * i + j] = B1[3 * i] * Di[j] + B1[3 * i + 1] * Di[3 + j] + B1[3 * i + 2] * Di[6 + j];
      for (int i = 0; i < 6; i++)
        bs[6 * k1 + i] -= B1[3 * i] * db[0] + B1[3 * i + 1] * db[1] + B1[3 * i + 2] * db[2];
      for (int e2 = B->pstart[p]; e2 < B->pstart[p + 1]; e2++) {
        const int k2 = B->free_idx[B->obs[e2].keyframe];
        if (!B->active[e2] || k2 < 0 || k2 > k1) continue;  // the lower part
        const double* B2 = &B->Hpl[18 * e2];
        for (int i = 0; i < 6; i++)
          for (int j = 0; j < 6; j++) {
            if (k2 == k1 && j > i) continue;
            PL(&S, 6 * k1 + i, 6 * k2 + j) -=
                BD[3 * i] * B2[3 * j] + BD[3 * i + 1] * B2[3 * j + 1] + BD[3 * i + 2] * B2[3 * j + 2];
          }
      }
    }
  }
  const int ok = ldlt_solve_profile(&S, bs, xp);
  profile_free(&S);
  free(bs);
  if (!ok) return 0;
  for (int p = 0; p < B->n_pts; p++) {
    double c[3] = {B->bl[3 * p], B->bl[3 * p + 1], B->bl[3 * p + 2]};
    for (int e = B->pstart[p]; e < B->pstart[p + 1]; e++) {
      const int k = B->free_idx[B->obs[e].keyframe];
      if (!B->active[e] || k < 0) continue;
      const double* Bl = &B->Hpl[18 * e];
      for (int j = 0; j < 3; j++)
        for (int i = 0; i < 6; i++) c[j] -= Bl[3 * i + j] * xp[6 * k + i];
    }
    const double* Di = &Dinv[9 * p];
    for (int i = 0; i < 3; i++) xl[3 * p + i] = Di[3 * i] * c[0] + Di[3 * i + 1] * c[1] + Di[3 * i + 2] * c[2];
  }
  return 1;
}

static void count_active(ba* B) {
  memset(B->kf_nact, 0, sizeof(int) * B->n_kf);
  memset(B->pt_nact, 0, sizeof(int) * B->n_pts);
  for (int e = 0; e < B->n_obs; e++)
    if (B->active[e]) {
      B->kf_nact[B->obs[e].keyframe]++;
      B->pt_nact[B->opoint[e]]++;
    }
}

// SparseOptimizer::optimize(iterations) with Levenberg-Marquardt over the whole graph.
static void optimize(ba* B, int iterations, int* lm_iters) {
  const int nfree = B->n_free;
  double* xp = (double*)calloc(6 * nfree + 1, sizeof(double));
  double* xl = (double*)calloc(3 * B->n_pts + 1, sizeof(double));
  double* Dinv = (double*)malloc(sizeof(double) * (9 * B->n_pts + 1));
  se3* Tb = (se3*)malloc(sizeof(se3) * (B->n_kf + 1));
  double* Xb = (double*)malloc(sizeof(double) * (3 * B->n_pts + 1));
  int* kf_of_free = (int*)malloc(sizeof(int) * (nfree + 1));
  for (int k = 0; k < B->n_kf; k++)
    if (B->free_idx[k] >= 0) kf_of_free[B->free_idx[k]] = k;
  count_active(B);
  double lambda = 0;
  int ni = 2, nbad = 0;
  for (int it = 0; it < iterations && !terminate_(B); it++) {
    compute_active_errors(B);
    double currentChi = active_robust_chi2(B);
    const double iniChi = currentChi;
    build_system(B);
    if (it == 0) {  // computeLambdaInit over the active, non-fixed vertices
      double maxd = 0;
      for (int k = 0; k < nfree; k++)
        if (B->kf_nact[kf_of_free[k]])
          for (int j = 0; j < 6; j++) maxd = fmax(fabs(B->Hpp[36 * k + 7 * j]), maxd);
      for (int p = 0; p < B->n_pts; p++)
        if (B->pt_nact[p])
          for (int j = 0; j < 3; j++) maxd = fmax(fabs(B->Hll[9 * p + 4 * j]), maxd);
      lambda = 1e-5 * maxd;
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      memcpy(Tb, B->T, sizeof(se3) * B->n_kf);  // push
      memcpy(Xb, B->X, sizeof(double) * 3 * B->n_pts);
      const int ok2 = schur_solve(B, lambda, xp, xl, Dinv);
      for (int k = 0; k < nfree; k++) {  // oplus on the active vertices
        const int kf = kf_of_free[k];
        if (!B->kf_nact[kf]) continue;
        se3 E = se3_exp(&xp[6 * k]);
        B->T[kf] = se3_mul(&E, &Tb[kf]);
      }
      for (int p = 0; p < B->n_pts; p++)
        if (B->pt_nact[p])
          for (int i = 0; i < 3; i++) B->X[3 * p + i] += xl[3 * p + i];
      compute_active_errors(B);
      double tempChi = active_robust_chi2(B);
      if (!ok2) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      double scale = 0;  // computeScale over the active vertices' x and b
      for (int k = 0; k < nfree; k++)
        if (B->kf_nact[kf_of_free[k]])
          for (int j = 0; j < 6; j++) scale += xp[6 * k + j] * (lambda * xp[6 * k + j] + B->bp[6 * k + j]);
      for (int p = 0; p < B->n_pts; p++)
        if (B->pt_nact[p])
          for (int j = 0; j < 3; j++) scale += xl[3 * p + j] * (lambda * xl[3 * p + j] + B->bl[3 * p + j]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        lambda *= fmax(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        memcpy(B->T, Tb, sizeof(se3) * B->n_kf);  // pop; edges keep the rejected errors
        memcpy(B->X, Xb, sizeof(double) * 3 * B->n_pts);
      }
      qmax++;
    } while (rho < 0 && qmax < 10 && !terminate_(B));
    if (lm_iters) (*lm_iters)++;
    if (qmax == 10 || rho == 0) break;
    if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
    else nbad = 0;
    if (nbad >= 3) break;
  }
  free(xp);
  free(xl);
  free(Dinv);
  free(Tb);
  free(Xb);
  free(kf_of_free);
}

static int depth_positive(const ba* B, int e) {  // isDepthPositive at the current estimates
  double Xc[3];
  se3_map(&B->T[B->obs[e].keyframe], &B->X[3 * B->opoint[e]], Xc);
  return Xc[2] > 0.0;
}

static void ba_init(ba* B, const float cam[5], const float* inv_sigma2, const float* kf_Tcw,
                    const uint8_t* kf_mode, int n_kf, const float* points, int n_points,
                    const int32_t* point_obs_start, const oc_ba_obs* obs) {
  const int n_obs = point_obs_start[n_points];
  memset(B, 0, sizeof(*B));
  B->stop_after = -1;
  // LocalBundleAdjustment's const float thresholds sqrt(5.991) / sqrt(7.815) (optimizer.cpp:556,598)
  B->delta_mono = (double)(float)sqrt(5.991);
  B->delta_stereo = (double)(float)sqrt(7.815);
  B->n_kf = n_kf;
  B->n_pts = n_points;
  B->n_obs = n_obs;
  B->obs = obs;
  B->pstart = point_obs_start;
  for (int i = 0; i < 5; i++) B->cam[i] = cam[i];
  B->bf_f = cam[4];
  B->isig = inv_sigma2;
  B->opoint = (int32_t*)malloc(sizeof(int32_t) * (n_obs + 1));
  B->free_idx = (int*)malloc(sizeof(int) * (n_kf + 1));
  B->T = (se3*)malloc(sizeof(se3) * (n_kf + 1));
  B->X = (double*)malloc(sizeof(double) * (3 * n_points + 1));
  B->active = (uint8_t*)malloc(n_obs + 1);
  B->err = (double*)calloc(3 * n_obs + 1, sizeof(double));
  B->chi2 = (double*)calloc(n_obs + 1, sizeof(double));
  B->kf_nact = (int*)calloc(n_kf + 1, sizeof(int));
  B->pt_nact = (int*)calloc(n_points + 1, sizeof(int));
  for (int p = 0; p < n_points; p++)
    for (int e = point_obs_start[p]; e < point_obs_start[p + 1]; e++) B->opoint[e] = p;
  for (int k = 0; k < n_kf; k++) {
    B->free_idx[k] = kf_mode[k] == 0 ? B->n_free++ : -1;
    double R[9], t[3];
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) R[3 * i + j] = kf_Tcw[16 * k + 4 * i + j];
      t[i] = kf_Tcw[16 * k + 4 * i + 3];
    }
    B->T[k] = se3_from_Rt(R, t);  // Converter::toSE3Quat(GetPose())
  }
  for (int i = 0; i < 3 * n_points; i++) B->X[i] = points[i];
  B->Hpp = (double*)malloc(sizeof(double) * (36 * B->n_free + 1));
  B->bp = (double*)malloc(sizeof(double) * (6 * B->n_free + 1));
  B->Hll = (double*)malloc(sizeof(double) * (9 * n_points + 1));
  B->bl = (double*)malloc(sizeof(double) * (3 * n_points + 1));
  B->Hpl = (double*)calloc(18 * (size_t)n_obs + 1, sizeof(double));
  memset(B->active, 1, n_obs + 1);
}

static void ba_free(ba* B) {
  free(B->opoint);
  free(B->free_idx);
  free(B->T);
  free(B->X);
  free(B->active);
  free(B->err);
  free(B->chi2);
  free(B->kf_nact);
  free(B->pt_nact);
  free(B->Hpp);
  free(B->bp);
  free(B->Hll);
  free(B->bl);
  free(B->Hpl);
}

int oc_local_bundle_adjustment(const float cam[5], const float* inv_sigma2, float* kf_Tcw,
                               const uint8_t* kf_mode, int n_kf, float* points, int n_points,
                               const int32_t* point_obs_start, const oc_ba_obs* obs,
                               uint8_t* erase, int* lm_iterations) {
  return oc_local_bundle_adjustment_stop(cam, inv_sigma2, kf_Tcw, kf_mode, n_kf, points, n_points,
                                         point_obs_start, obs, -1, erase, lm_iterations);
}

int oc_local_bundle_adjustment_stop(const float cam[5], const float* inv_sigma2, float* kf_Tcw,
                                    const uint8_t* kf_mode, int n_kf, float* points, int n_points,
                                    const int32_t* point_obs_start, const oc_ba_obs* obs,
                                    int stop_after, uint8_t* erase, int* lm_iterations) {
  if (lm_iterations) *lm_iterations = 0;
  if (n_kf < 0 || n_points < 0 || point_obs_start[0] != 0) return -1;
  const int n_obs = point_obs_start[n_points];
  ba B;
  ba_init(&B, cam, inv_sigma2, kf_Tcw, kf_mode, n_kf, points, n_points, point_obs_start, obs);
  B.stop_after = stop_after;
  B.polls = 0;
  if (terminate_(&B)) {  // optimizer.cpp:616-618: return before optimising, nothing written
    for (int e = 0; e < n_obs; e++) erase[e] = 0;
    ba_free(&B);
    return 0;
  }

  B.robust = 1;
  optimize(&B, 5, lm_iterations);  // optimizer.cpp:622-623
  if (!terminate_(&B)) {           // :625-627 do_more
    // optimizer.cpp:632-665: outliers to level 1, robust kernels off
    for (int e = 0; e < n_obs; e++) {
      const double thr = is_stereo(&obs[e]) ? 7.815 : 5.991;
      if (B.chi2[e] > thr || !depth_positive(&B, e)) B.active[e] = 0;
    }
    B.robust = 0;
    optimize(&B, 10, lm_iterations);  // :668-669
  }
  // :672-700: erase list over every edge (level-1 edges keep their last computed chi2)
  for (int e = 0; e < n_obs; e++) {
    const double thr = is_stereo(&obs[e]) ? 7.815 : 5.991;
    erase[e] = (B.chi2[e] > thr || !depth_positive(&B, e)) ? 1 : 0;
  }
  // :712-724 write-back: local keyframes (mode 0 and 1) and every point
  for (int k = 0; k < n_kf; k++) {
    if (kf_mode[k] == 2) continue;
    double R[9];
    quat_to_R(B.T[k].r, R);
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) kf_Tcw[16 * k + 4 * i + j] = (float)R[3 * i + j];
      kf_Tcw[16 * k + 4 * i + 3] = (float)B.T[k].t[i];
    }
    kf_Tcw[16 * k + 12] = kf_Tcw[16 * k + 13] = kf_Tcw[16 * k + 14] = 0.f;
    kf_Tcw[16 * k + 15] = 1.f;
  }
  for (int i = 0; i < 3 * n_points; i++) points[i] = (float)B.X[i];
  ba_free(&B);
  return 0;
}

double oc_ba_edge_eval(const float cam[5], const double R[9], const double t[3], const double X[3],
                       const oc_ba_obs* o, float inv_sigma2, double err[3], double Jl[9],
                       double Jp[18]) {
  float isig[1] = {inv_sigma2};
  oc_ba_obs ob = *o;
  ob.keyframe = 0;
  ob.octave = 0;
  int32_t pstart[2] = {0, 1}, opoint[1] = {0};
  int fidx[1] = {0};
  se3 T = se3_from_Rt(R, t);
  double Xd[3] = {X[0], X[1], X[2]};
  ba B;
  memset(&B, 0, sizeof(B));
  B.n_kf = 1;
  B.n_pts = 1;
  B.n_obs = 1;
  B.obs = &ob;
  B.pstart = pstart;
  B.opoint = opoint;
  B.free_idx = fidx;
  for (int i = 0; i < 5; i++) B.cam[i] = cam[i];
  B.bf_f = cam[4];
  B.isig = isig;
  B.T = &T;
  B.X = Xd;
  double Xc[3];
  const double c = ba_error(&B, 0, err, Xc);
  if (Jl && Jp) ba_jacobians(&B, 0, Jl, Jp);
  return c;
}

// computeActiveErrors + activeRobustChi2 + buildSystem of the first optimize() (every edge at level
// 0, Huber kernels on) at the input estimates; the layout of slamgpu_ba_linear.
double oc_ba_linearize(const float cam[5], const float* inv_sigma2, const float* kf_Tcw,
                       const uint8_t* kf_mode, int n_kf, const float* points, int n_points,
                       const int32_t* point_obs_start, const oc_ba_obs* obs, double* chi2,
                       double* hpl, double* hll, double* bl, double* hpp, double* bp) {
  ba B;
  ba_init(&B, cam, inv_sigma2, kf_Tcw, kf_mode, n_kf, points, n_points, point_obs_start, obs);
  B.robust = 1;
  compute_active_errors(&B);
  const double chi = active_robust_chi2(&B);
  build_system(&B);
  for (int e = 0; e < B.n_obs; e++) {
    chi2[e] = B.chi2[e];
    for (int i = 0; i < 18; i++) hpl[18 * e + i] = B.free_idx[obs[e].keyframe] >= 0 ? B.Hpl[18 * e + i] : 0.0;
  }
  static const int s3[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
  for (int p = 0; p < n_points; p++) {
    for (int i = 0; i < 6; i++) hll[6 * p + i] = B.Hll[9 * p + 3 * s3[i][0] + s3[i][1]];
    for (int i = 0; i < 3; i++) bl[3 * p + i] = B.bl[3 * p + i];
  }
  for (int k = 0; k < n_kf; k++) {
    const int f = B.free_idx[k];
    int h = 0;
    for (int a = 0; a < 6; a++)
      for (int c = a; c < 6; c++, h++) hpp[21 * k + h] = f >= 0 ? B.Hpp[36 * f + 6 * a + c] : 0.0;
    for (int i = 0; i < 6; i++) bp[6 * k + i] = f >= 0 ? B.bp[6 * f + i] : 0.0;
  }
  ba_free(&B);
  return chi;
}

/* Optimizer::BundleAdjustment (optimizer.cpp:33-207) after its graph gathering: keyframe id 0
 * fixed (kf_mode 1), every other keyframe optimised (mode 0), every point; one
 * optimize(n_iterations) with Huber kernels (deltas sqrt(5.99) / sqrt(7.815) as float,
 * :69-70) when robust; poses and points written back (:163-206). stop_after as above (< 0:
 * never raised); g2o polls it at each iteration and failed trial only (no check before). */
int oc_global_bundle_adjustment_stop(const float cam[5], const float* inv_sigma2, float* kf_Tcw,
                                     const uint8_t* kf_mode, int n_kf, float* points,
                                     int n_points, const int32_t* point_obs_start,
                                     const oc_ba_obs* obs, int n_iterations, int robust,
                                     int stop_after, int* lm_iterations) {
  if (lm_iterations) *lm_iterations = 0;
  if (n_kf < 0 || n_points < 0 || point_obs_start[0] != 0) return -1;
  ba B;
  ba_init(&B, cam, inv_sigma2, kf_Tcw, kf_mode, n_kf, points, n_points, point_obs_start, obs);
  B.stop_after = stop_after;
  B.polls = 0;
  B.delta_mono = (double)(float)sqrt(5.99);
  B.delta_stereo = (double)(float)sqrt(7.815);
  B.robust = robust;
  optimize(&B, n_iterations, lm_iterations);
  for (int k = 0; k < n_kf; k++) {
    if (kf_mode[k] == 2) continue;
    double R[9];
    quat_to_R(B.T[k].r, R);
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) kf_Tcw[16 * k + 4 * i + j] = (float)R[3 * i + j];
      kf_Tcw[16 * k + 4 * i + 3] = (float)B.T[k].t[i];
    }
    kf_Tcw[16 * k + 12] = kf_Tcw[16 * k + 13] = kf_Tcw[16 * k + 14] = 0.f;
    kf_Tcw[16 * k + 15] = 1.f;
  }
  for (int i = 0; i < 3 * n_points; i++) points[i] = (float)B.X[i];
  ba_free(&B);
  return 0;
}
