// oracle/eg_oracle.c -- CPU restatement of Optimizer::OptimizeEssentialGraph (TEST
// INFRASTRUCTURE).
//
// Only tests/ may use this file; the product path is slam_framework_amd/csrc/eg_kernels.hip.
//
// Parity status: "parity unpinned" against the reference binary (g2o needs Eigen3, absent here;
// DESIGN.md §4). Restated in FP64:
//   src/optimizer/optimizer.cpp:718-960      OptimizeEssentialGraph: Sim3 vertices (the loop
//                                            keyframe fixed), EdgeSim3 with identity information,
//                                            LM with user lambda 1e-16, optimize(20), SE3 pose
//                                            recovery [R t/s], map point correction
//   g2o/types/types_seven_dof_expmap.h:99-126  EdgeSim3::computeError = log(Sji Si Sj^-1)
//   g2o/core/base_binary_edge.hpp:131-203    numeric Jacobians of both vertices (delta 1e-9)
//   g2o/core/base_binary_edge.hpp:55-121     constructQuadraticForm without a robust kernel
//   g2o/core/optimization_algorithm_levenberg.cpp:61-189   LM (user lambda init)
//   g2o/solvers/linear_solver_eigen.h:94-120 sparse LDLT of the 7x7-block system -- restated as
//                                            a profile (skyline) LDLT in vertex order without
//                                            pivoting; Eigen's AMD ordering changes rounding only
// The graph (which keyframe pairs get an edge and their measurements Sji = Sjw * Swi,
// optimizer.cpp:782-909) is gathered by the caller, as the device call takes it.
// Pinned by tests/test_eg_oracle.py: a noise-free loop closes exactly, the numeric Jacobians
// agree with an independent difference, and the optimum is a stationary point of the chi2.
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"
#include "sim3_oracle.h"

#pragma GCC diagnostic ignored "-Wunused-function"

typedef struct {
  int n, n_edges, F;        // vertices, edges, free vertices
  sim3* S;                  // [n] estimates
  const uint8_t* fixed;
  const oc_sim3_edge* E;
  sim3* meas;               // [n_edges]
  int fix_scale;
  int* fidx;                // [n] free index or -1
  int* start;               // [F] first free block column of block row f's envelope
  double* err;              // [n_edges][7]
} egraph;

static double edge_error(const egraph* G, int k, const sim3* S, double e[7]) {
  const oc_sim3_edge* ed = &G->E[k];
  const sim3 Sj_inv = sim3_inverse(&S[ed->j]);
  const sim3 a = sim3_mul(&G->meas[k], &S[ed->i]);
  const sim3 err = sim3_mul(&a, &Sj_inv);
  sim3_log(&err, e);
  double c = 0;
  for (int r = 0; r < 7; r++) c += e[r] * e[r];
  return c;
}

static double compute_errors(egraph* G, const sim3* S) {
  double chi = 0;
  for (int k = 0; k < G->n_edges; k++) chi += edge_error(G, k, S, &G->err[7 * k]);
  return chi;
}

static sim3 oplus(const sim3* S, double u[7], int fix_scale) {
  if (fix_scale) u[6] = 0;
  const sim3 D = sim3_exp(u);
  return sim3_mul(&D, S);
}

// column d of the Jacobian wrt vertex `which` (0: i, 1: j) by g2o's central difference
static void edge_jacobian(const egraph* G, int k, sim3* S, int which, double J[49]) {
  const int v = which ? G->E[k].j : G->E[k].i;
  const sim3 keep = S[v];
  const double delta = 1e-9, scalar = 1.0 / (2 * delta);
  for (int d = 0; d < 7; d++) {
    double add[7] = {0, 0, 0, 0, 0, 0, 0}, ep[7], em[7];
    add[d] = delta;
    S[v] = oplus(&keep, add, G->fix_scale);
    edge_error(G, k, S, ep);
    double add2[7] = {0, 0, 0, 0, 0, 0, 0};
    add2[d] = -delta;
    S[v] = oplus(&keep, add2, G->fix_scale);
    edge_error(G, k, S, em);
    S[v] = keep;
    for (int r = 0; r < 7; r++) J[7 * r + d] = scalar * (ep[r] - em[r]);
  }
}

// ---- profile storage of the 7F x 7F system: block row f holds blocks start[f] .. f ----------
typedef struct {
  int F;
  const int* start;
  size_t* off;     // [F + 1] block offset of row f
  double* A;       // blocks, row-major 7x7
  double* b;       // [7F]
} prof;

static double* blk(prof* P, int f, int g) { return P->A + 49 * (P->off[f] + (size_t)(g - P->start[f])); }

static void build_system(egraph* G, sim3* S, prof* P) {
  memset(P->A, 0, 49 * sizeof(double) * P->off[P->F]);
  memset(P->b, 0, 7 * sizeof(double) * P->F);
  for (int k = 0; k < G->n_edges; k++) {
    const int fi = G->fidx[G->E[k].i], fj = G->fidx[G->E[k].j];
    double A[49], B[49];
    if (fi >= 0) edge_jacobian(G, k, S, 0, A);
    if (fj >= 0) edge_jacobian(G, k, S, 1, B);
    const double* e = &G->err[7 * k];
    double r[7];
    for (int q = 0; q < 7; q++) r[q] = -e[q];  // omega_r = -Omega e, Omega = I
    if (fi >= 0) {
      double* Hii = blk(P, fi, fi);
      for (int a = 0; a < 7; a++) {
        double s = 0;
        for (int q = 0; q < 7; q++) s += A[7 * q + a] * r[q];
        P->b[7 * fi + a] += s;
        for (int c = 0; c < 7; c++) {
          double h = 0;
          for (int q = 0; q < 7; q++) h += A[7 * q + a] * A[7 * q + c];
          Hii[7 * a + c] += h;
        }
      }
      if (fj >= 0) {  // the off-diagonal block, stored in the later block row
        for (int a = 0; a < 7; a++)
          for (int c = 0; c < 7; c++) {
            double h = 0;
            for (int q = 0; q < 7; q++) h += A[7 * q + a] * B[7 * q + c];  // (A' B)(a, c)
            if (fi > fj) blk(P, fi, fj)[7 * a + c] += h;
            else blk(P, fj, fi)[7 * c + a] += h;
          }
      }
    }
    if (fj >= 0) {
      double* Hjj = blk(P, fj, fj);
      for (int a = 0; a < 7; a++) {
        double s = 0;
        for (int q = 0; q < 7; q++) s += B[7 * q + a] * r[q];
        P->b[7 * fj + a] += s;
        for (int c = 0; c < 7; c++) {
          double h = 0;
          for (int q = 0; q < 7; q++) h += B[7 * q + a] * B[7 * q + c];
          Hjj[7 * a + c] += h;
        }
      }
    }
  }
}

// Profile LDLT (Crout, scalar rows in vertex order) of H + lambda I, then the solve. Row i's
// envelope starts at scalar column s(i) = 7 start[i / 7]. Fails on a zero pivot.
static int profile_ldlt_solve(const prof* P, double lambda, double* x) {
  const int F = P->F, n = 7 * F;
  double* L = malloc(sizeof(double) * 49 * P->off[F]);
  double* D = malloc(sizeof(double) * (n > 0 ? n : 1));
  memcpy(L, P->A, sizeof(double) * 49 * P->off[F]);
  // scalar access: row i, column j (s(i) <= j <= i)
#define SROW(i) ((i) / 7)
#define SCOL0(i) (7 * P->start[SROW(i)])
#define AT(i, j) L[49 * (P->off[SROW(i)] + (size_t)((j) / 7 - P->start[SROW(i)])) + 7 * ((i) % 7) + (j) % 7]
  int ok = 1;
  for (int i = 0; i < n && ok; i++) {
    const int si = SCOL0(i);
    for (int j = si; j < i; j++) {
      const int sj = SCOL0(j);
      double s = AT(i, j);
      for (int k = (si > sj ? si : sj); k < j; k++) s -= AT(i, k) * D[k] * AT(j, k);
      AT(i, j) = s / D[j];
    }
    double d = AT(i, i) + lambda;
    for (int k = si; k < i; k++) d -= AT(i, k) * AT(i, k) * D[k];
    D[i] = d;
    if (d == 0.0) ok = 0;
  }
  if (ok) {
    for (int i = 0; i < n; i++) {  // L y = b
      double s = P->b[i];
      for (int k = SCOL0(i); k < i; k++) s -= AT(i, k) * x[k];
      x[i] = s;
    }
    for (int i = 0; i < n; i++) x[i] /= D[i];
    for (int i = n - 1; i >= 0; i--)  // L' x = y, column sweeps
      for (int k = SCOL0(i); k < i; k++) x[k] -= AT(i, k) * x[i];
  }
#undef AT
#undef SCOL0
#undef SROW
  free(L);
  free(D);
  return ok;
}

int oc_optimize_essential_graph(int n, double* Scw, const uint8_t* fixed, const oc_sim3_edge* edges,
                                int n_edges, int fix_scale, int n_iterations, float* Tcw_out,
                                int* lm_iterations) {
  if (lm_iterations) *lm_iterations = 0;
  egraph G;
  memset(&G, 0, sizeof(G));
  G.n = n;
  G.n_edges = n_edges;
  G.fixed = fixed;
  G.E = edges;
  G.fix_scale = fix_scale;
  G.S = malloc(sizeof(sim3) * (n > 0 ? n : 1));
  G.meas = malloc(sizeof(sim3) * (n_edges > 0 ? n_edges : 1));
  G.fidx = malloc(sizeof(int) * (n > 0 ? n : 1));
  G.err = malloc(sizeof(double) * 7 * (n_edges > 0 ? n_edges : 1));
  for (int v = 0; v < n; v++) G.S[v] = sim3_load(&Scw[8 * v]);
  for (int k = 0; k < n_edges; k++) G.meas[k] = sim3_load(edges[k].Sji);
  int F = 0;
  for (int v = 0; v < n; v++) G.fidx[v] = fixed[v] ? -1 : F++;
  G.F = F;
  int* start = malloc(sizeof(int) * (F > 0 ? F : 1));
  for (int f = 0; f < F; f++) start[f] = f;
  for (int k = 0; k < n_edges; k++) {
    const int a = G.fidx[edges[k].i], b = G.fidx[edges[k].j];
    if (a < 0 || b < 0) continue;
    const int hi = a > b ? a : b, lo = a > b ? b : a;
    if (lo < start[hi]) start[hi] = lo;
  }
  G.start = start;
  prof P;
  P.F = F;
  P.start = start;
  P.off = malloc(sizeof(size_t) * (F + 1));
  P.off[0] = 0;
  for (int f = 0; f < F; f++) P.off[f + 1] = P.off[f] + (size_t)(f - start[f] + 1);
  P.A = malloc(sizeof(double) * 49 * (P.off[F] > 0 ? P.off[F] : 1));
  P.b = malloc(sizeof(double) * 7 * (F > 0 ? F : 1));
  double* x = calloc(7 * (F > 0 ? F : 1), sizeof(double));
  sim3* backup = malloc(sizeof(sim3) * (n > 0 ? n : 1));

  // SparseOptimizer::optimize(n_iterations), OptimizationAlgorithmLevenberg
  double lambda = 1e-16;  // setUserLambdaInit(1e-16): computeLambdaInit returns it
  int ni = 2, nbad = 0;
  for (int it = 0; it < n_iterations && F > 0; it++) {
    double currentChi = compute_errors(&G, G.S);
    const double iniChi = currentChi;
    build_system(&G, G.S, &P);
    if (it == 0) {
      lambda = 1e-16;
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      memcpy(backup, G.S, sizeof(sim3) * n);
      const int ok2 = profile_ldlt_solve(&P, lambda, x);  // x keeps its last value on failure
      for (int v = 0; v < n; v++)
        if (G.fidx[v] >= 0) G.S[v] = oplus(&backup[v], &x[7 * G.fidx[v]], fix_scale);
      double tempChi = compute_errors(&G, G.S);
      if (!ok2) tempChi = DBL_MAX;
      rho = currentChi - tempChi;
      double scale = 0;
      for (int q = 0; q < 7 * F; q++) scale += x[q] * (lambda * x[q] + P.b[q]);
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
        memcpy(G.S, backup, sizeof(sim3) * n);
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    if (lm_iterations) (*lm_iterations)++;
    if (qmax == 10 || rho == 0) break;
    if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
    else nbad = 0;
    if (nbad >= 3) break;
  }
  for (int v = 0; v < n; v++) {
    sim3_store(&G.S[v], &Scw[8 * v]);
    if (Tcw_out) {  // SE3 pose recovery (:917-931): [R t/s; 0 1], f32
      double R[9];
      quat_to_R(G.S[v].r, R);
      const double is = 1. / G.S[v].s;
      float* T = &Tcw_out[16 * v];
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = (float)R[3 * i + j];
        T[4 * i + 3] = (float)(G.S[v].t[i] * is);
      }
      T[12] = T[13] = T[14] = 0.f;
      T[15] = 1.f;
    }
  }
  free(backup);
  free(x);
  free(P.b);
  free(P.A);
  free(P.off);
  free(start);
  free(G.err);
  free(G.fidx);
  free(G.meas);
  free(G.S);
  return 0;
}

// Map point correction (:933-959): P' = correctedSwr.map(Srw.map(P)), with Srw the keyframe's
// Sim3 before the optimisation (vScw) and correctedSwr the inverse of the optimised one; f32 in
// and out (Converter::toVector3d / toCvMat).
void oc_correct_points_sim3(const double* Scw_before, const double* Scw_after, const int32_t* ref,
                            float* points, int n_points) {
  for (int p = 0; p < n_points; p++) {
    const sim3 Srw = sim3_load(&Scw_before[8 * ref[p]]);
    const sim3 Sa = sim3_load(&Scw_after[8 * ref[p]]);
    const sim3 Swr = sim3_inverse(&Sa);
    const double X[3] = {points[3 * p], points[3 * p + 1], points[3 * p + 2]};
    double Y[3], Z[3];
    sim3_map(&Srw, X, Y);
    sim3_map(&Swr, Y, Z);
    for (int i = 0; i < 3; i++) points[3 * p + i] = (float)Z[i];
  }
}

// chi2 and the numeric Jacobians of one edge (for the oracle's own tests)
double oc_sim3_edge_eval(const double Si[8], const double Sj[8], const double Sji[8], int fix_scale,
                         double e[7], double Ji[49], double Jj[49]) {
  sim3 S[2] = {sim3_load(Si), sim3_load(Sj)};
  const sim3 M = sim3_load(Sji);
  oc_sim3_edge ed;
  memset(&ed, 0, sizeof(ed));
  ed.i = 0;
  ed.j = 1;
  egraph G;
  memset(&G, 0, sizeof(G));
  G.n = 2;
  G.n_edges = 1;
  G.E = &ed;
  G.meas = (sim3*)&M;
  G.fix_scale = fix_scale;
  const double c = edge_error(&G, 0, S, e);
  if (Ji) edge_jacobian(&G, 0, S, 0, Ji);
  if (Jj) edge_jacobian(&G, 0, S, 1, Jj);
  return c;
}
