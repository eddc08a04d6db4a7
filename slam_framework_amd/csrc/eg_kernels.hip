// eg_kernels.hip -- Optimizer::OptimizeEssentialGraph (optimizer.cpp:718-960) on the device.
//
// The graph: a g2o::VertexSim3Expmap per keyframe (the loop keyframe fixed) and an EdgeSim3 per
// spanning-tree / loop / covisibility link, error log(Sji Si Sj^-1), identity information, no
// robust kernel; Levenberg-Marquardt with user lambda 1e-16, 20 iterations; the linear system
// (7 x 7 blocks, BlockSolver_7_3 + LinearSolverEigen) solved by sparse LDLT.
//
// Device split (the host drives the LM loop: one synchronisation per trial for the chi2 and the
// solve status, optimizer_runtime.cpp):
//   eg_linearize   a thread per edge: error, chi2, g2o's numeric Jacobians of both vertices
//                  (central differences, delta 1e-9: 14 error evaluations per free vertex), and
//                  the edge's contributions Ji'Ji, Jj'Jj, Ji'Jj, -Ji'e, -Jj'e
//   eg_assemble    a wave per block of the system that an edge touches: the contributions summed
//                  in edge order (g2o's buildSystem order), so the sums are deterministic
//   eg_factor_solve one work-group: the LDLT of H + lambda I in the profile (skyline) storage of
//                  the vertex order -- keyframe ids order the graph along the trajectory, so the
//                  profile is a band plus the few long rows of loop edges -- right-looking by
//                  block column (diagonal block LDLT, panel, trailing update of the column's
//                  extent), then the forward / diagonal / backward solves and g2o's scale term
//   eg_update      a thread per vertex: Sim3(dx) * S (dx[6] = 0 with a fixed scale)
//   eg_errors, eg_chi2_sum  the trial's errors and their fixed-order sum
//   eg_finish      SE3 pose recovery [R t/s] (:917-931) and the map point correction (:933-959)
// The reference's Eigen sparse LDLT orders the unknowns by AMD; the profile LDLT in vertex order
// computes the same factorisation up to rounding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>

#include "device_math.h"
#include "eg_kernels.h"
#include "sim3_device.h"

namespace slamgpu {
namespace {

using sim3::Sim3;

__device__ __forceinline__ double edge_error(const Sim3& M, const Sim3& Si, const Sim3& Sj,
                                             double e[7]) {
  const Sim3 a = sim3::sim3_mul(M, Si);
  const Sim3 err = sim3::sim3_mul(a, sim3::sim3_inverse(Sj));
  sim3::sim3_log(err, e);
  double c = 0.0;
#pragma unroll
  for (int r = 0; r < 7; r++) c += e[r] * e[r];
  return c;
}

__device__ __forceinline__ Sim3 oplus_axis(const Sim3& S, int d, double h, int fix_scale) {
  double u[7];
#pragma unroll
  for (int i = 0; i < 7; i++) u[i] = i == d ? h : 0.0;
  if (fix_scale) u[6] = 0;
  return sim3::sim3_mul(sim3::sim3_exp(u), S);
}

// The linearisation in two launches, so an edge's 14 numeric-Jacobian columns (two error
// evaluations each: Sim3 exp, products, log) run on 14 threads instead of in turn on one --
// the one-thread-per-edge kernel kept a few hundred threads busy for ~20 serial evaluations.
// Same operations per value, so the same bits.
// eg_jac_kernel: thread (edge k, q): q < 14 the Jacobian column q (vertex q / 7, axis q % 7)
// by central differences (BaseBinaryEdge::linearizeOplus, delta 1e-9); q == 14 the error and
// chi2 at the estimate.
constexpr int kEgJacThreads = 15;
__global__ __launch_bounds__(256) void eg_jac_kernel(EgGraph G, EgState W) {
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gt >= (int64_t)G.n_edges * kEgJacThreads) return;
  const int k = (int)(gt / kEgJacThreads), q = (int)(gt % kEgJacThreads);
  const slamgpu_sim3_edge ed = G.edges[k];
  const Sim3 Si = sim3::sim3_load(W.S + 8 * ed.i), Sj = sim3::sim3_load(W.S + 8 * ed.j);
  const Sim3 M = sim3::sim3_load(ed.Sji);
  if (q == 14) {
    double e[7];
    W.chi2[k] = edge_error(M, Si, Sj, e);
#pragma unroll
    for (int r = 0; r < 7; r++) W.err[7 * k + r] = e[r];
    return;
  }
  const int which = q / 7, d = q % 7;
  if ((which ? G.fidx[ed.j] : G.fidx[ed.i]) < 0) return;  // a fixed vertex has no block
  const double delta = 1e-9, scalar = 1.0 / (2 * delta);
  double ep[7], em[7];
  if (which == 0) {
    edge_error(M, oplus_axis(Si, d, delta, G.fix_scale), Sj, ep);
    edge_error(M, oplus_axis(Si, d, -delta, G.fix_scale), Sj, em);
  } else {
    edge_error(M, Si, oplus_axis(Sj, d, delta, G.fix_scale), ep);
    edge_error(M, Si, oplus_axis(Sj, d, -delta, G.fix_scale), em);
  }
  double* J = W.J + (int64_t)k * 98 + 49 * which;
#pragma unroll
  for (int r = 0; r < 7; r++) J[7 * r + d] = scalar * (ep[r] - em[r]);
}

// eg_products_kernel: thread (edge k, row a): b += J' omega_r (omega_r = -e), H += J' J
// (base_binary_edge.hpp:55-121, Omega = I) -- row a of each product, sums over q in order.
__global__ __launch_bounds__(256) void eg_products_kernel(EgGraph G, EgState W) {
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gt >= (int64_t)G.n_edges * 7) return;
  const int k = (int)(gt / 7), a = (int)(gt % 7);
  const slamgpu_sim3_edge ed = G.edges[k];
  const int fi = G.fidx[ed.i], fj = G.fidx[ed.j];
  double e[7];
#pragma unroll
  for (int r = 0; r < 7; r++) e[r] = W.err[7 * k + r];
  double* c = W.contrib + (int64_t)k * kEgContrib;
  const double* Ja = W.J + (int64_t)k * 98;
  const double* Jb = Ja + 49;
  if (fi >= 0) {
    double s = 0.0;
    for (int q = 0; q < 7; q++) s += Ja[7 * q + a] * -e[q];
    c[147 + a] = s;
    for (int cc = 0; cc < 7; cc++) {
      double h = 0.0;
      for (int q = 0; q < 7; q++) h += Ja[7 * q + a] * Ja[7 * q + cc];
      c[7 * a + cc] = h;
    }
    if (fj >= 0)
      for (int cc = 0; cc < 7; cc++) {
        double h = 0.0;
        for (int q = 0; q < 7; q++) h += Ja[7 * q + a] * Jb[7 * q + cc];
        c[98 + 7 * a + cc] = h;
      }
  }
  if (fj >= 0) {
    double s = 0.0;
    for (int q = 0; q < 7; q++) s += Jb[7 * q + a] * -e[q];
    c[154 + a] = s;
    for (int cc = 0; cc < 7; cc++) {
      double h = 0.0;
      for (int q = 0; q < 7; q++) h += Jb[7 * q + a] * Jb[7 * q + cc];
      c[49 + 7 * a + cc] = h;
    }
  }
}

__global__ __launch_bounds__(256) void eg_errors_kernel(EgGraph G, const double* S, EgState W) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= G.n_edges) return;
  const slamgpu_sim3_edge ed = G.edges[k];
  double e[7];
  W.chi2[k] = edge_error(sim3::sim3_load(ed.Sji), sim3::sim3_load(S + 8 * ed.i),
                         sim3::sim3_load(S + 8 * ed.j), e);
}

// Deterministic sum of v[0..n): thread t sums v[t], v[t + 256], ... then a fixed tree.
__device__ double block_sum256(const double* v, int n, double* red) {
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  const double t = red[0];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(256) void eg_chi2_sum_kernel(EgGraph G, EgState W) {
  __shared__ double red[256];
  const double t = block_sum256(W.chi2, G.n_edges, red);
  if (threadIdx.x == 0) W.out[0] = t;
}

__global__ __launch_bounds__(64) void eg_assemble_kernel(EgGraph G, EgState W) {
  const int t = blockIdx.x, lane = threadIdx.x;
  const int blk = G.tgt_block[t], f = G.tgt_vertex[t];
  const int i0 = G.tgt_ptr[t], i1 = G.tgt_ptr[t + 1];
  const bool is_b = lane >= 49 && lane < 56 && f >= 0;
  if (lane >= 49 && !is_b) return;
  const int r = lane / 7, cc = lane % 7, rb = lane - 49;
  double s = 0.0;
  for (int q = i0; q < i1; q++) {
    const int item = G.tgt_items[q];
    const double* c = W.contrib + (int64_t)(item >> 2) * kEgContrib;
    const int kind = item & 3;
    if (is_b) s += c[(kind == 0 ? 147 : 154) + rb];
    else if (kind == 0) s += c[lane];
    else if (kind == 1) s += c[49 + lane];
    else if (kind == 2) s += c[98 + lane];
    else s += c[98 + 7 * cc + r];
  }
  if (is_b) W.b[7 * f + rb] = s;
  else W.H[(int64_t)blk * 49 + lane] = s;
}

#ifndef EG_EXACT_ROUNDING  // 1: the round-1 kernel's operation order, bit for bit
#define EG_EXACT_ROUNDING 1
#endif
constexpr int kFacThreads = 1024;
constexpr int kPanStage = 96;  // extent blocks whose panel is staged in LDS (37.6 KB)
constexpr int kXr = 64;        // columns of x the backward solve keeps in its LDS ring

// The LDLT of H + lambda I (profile storage, vertex order) and the solve, by one work-group of
// 16 waves. Right-looking by 7x7 block column k with a look-ahead: the panel (a thread per row of
// each extent block: L_ik = A_ik L_kk^-T D_k^-1, fused with the forward solve y_i -= L_ik y_k)
// -> barrier -> waves 1-15 apply the trailing update A_ij -= L_ik D_k L_jk' over the column's
// extent while wave 0 applies it to the next diagonal block and lane 0 factors that block in
// registers (pivot reciprocals, in-block forward solve) -> barrier: two barriers per column,
// the diagonal chain off the critical path. The panel's blocks also go to LDS (extents of up to
// kPanStage blocks), so the update and the next diagonal block read L_ik there instead of
// making another L2 round trip after the barrier; wave 0 loads the next diagonal block before
// the panel (it is final but for this column's update). Block (i, j) of an extent row lives at
// ext_base[e] + j (ext_base = off[i] - start[i], precomputed on the host: one dependent load).
// Then z = D^-1 y and the backward solve by wave 0 alone (lanes 0-6 sum a column's extent, lane 0
// solves the block; no work-group barriers), and g2o's scale term. EG_EXACT_ROUNDING (default)
// keeps the previous kernel's operation order (divisions, no contraction, the same sums), so the
// results are bit-identical to it; the LM stop test of this ill-conditioned system amplifies
// last-bit differences into different iteration counts.
// x of lane l, to every lane (l wave-uniform)
__device__ __forceinline__ double bcast(double x, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// x of lane l - 1 (DPP wave_shr:1; lane 0 gets 0)
__device__ __forceinline__ double bcast_dpp_shr1(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)u, 0x138, 0xf, 0xf, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(u >> 32), 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// kMeta: the factorisation's structure -- ext_ptr, ext_rows, ext_base and each column's
// diagonal block index -- is staged in LDS at the start (dynamic LDS, 4 B per entry), so the
// per-column chain of dependent structure loads (ext_ptr -> ext_base -> the block) reads LDS
// instead of L2. The host takes this variant whenever the structure fits (eg_meta_bytes).
template <bool kMeta>
__global__ __launch_bounds__(kFacThreads) void eg_factor_solve_kernel(EgGraph G, EgState W,
                                                                      int64_t n_blocks,
                                                                      double lambda) {
#if !EG_EXACT_ROUNDING
#pragma clang fp contract(fast)  // tolerance-compared FP64 path
#endif
  __shared__ int s_ok;
  __shared__ double red[256];
  __shared__ double s_kk[2][49];  // factored diagonal block of this / the next column
  __shared__ double s_rd[2][7];   // its pivot reciprocals
  __shared__ double s_y[2][7];    // its forward-solved rhs slice
  __shared__ double s_nx[49];     // the next diagonal block after its last update
  __shared__ double s_pan[kPanStage * 49];  // column k's panel blocks L_ik (extents <= kPanStage)
  __shared__ double s_xr[kXr * 7];          // the backward solve's x of the last kXr columns
  extern __shared__ int32_t s_meta[];  // kMeta: ext_ptr [F + 1], diag block [F], rows, bases
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, F = G.F;
  double* L = W.L;  // a copy of H (launch_eg_factor_solve)
  double* y = W.y;
  const int n_ext = kMeta ? G.ext_ptr[F] : 0;
  int32_t* const m_ep = s_meta;
  int32_t* const m_db = s_meta + F + 1;
  int32_t* const m_er = m_db + F;
  int32_t* const m_eb = m_er + n_ext;
  if constexpr (kMeta) {
    for (int q = tid; q <= F; q += kFacThreads) m_ep[q] = G.ext_ptr[q];
    for (int q = tid; q < F; q += kFacThreads) m_db[q] = (int32_t)(G.off[q] + (q - G.start[q]));
    for (int q = tid; q < n_ext; q += kFacThreads) {
      m_er[q] = G.ext_rows[q];
      m_eb[q] = (int32_t)G.ext_base[q];
    }
  }
  auto EP = [&](int k) -> int { return kMeta ? m_ep[k] : G.ext_ptr[k]; };
  auto ER = [&](int e) -> int { return kMeta ? m_er[e] : G.ext_rows[e]; };
  auto EB = [&](int e) -> int64_t { return kMeta ? (int64_t)m_eb[e] : G.ext_base[e]; };
  auto DB = [&](int k) -> int64_t {
    return kMeta ? (int64_t)m_db[k] : G.off[k] + (k - G.start[k]);
  };
  __syncthreads();
  for (int q = tid; q < 7 * F; q += kFacThreads) {
    const int v = q / 7, r = q % 7;
    L[DB(v) * 49 + 8 * r] += lambda;  // setLambda: H + lambda I
    y[q] = W.b[q];
  }
  if (tid == 0) s_ok = 1;
  __syncthreads();
  auto diag_of = [&](int k) { return L + DB(k) * 49; };
  // lanes 0-6 of a wave, lane r holding row r: LDLT of diagonal block k from src (lower
  // triangle + diagonal), the forward solve of y_k; L_kk / D_k to the profile and to s_kk[buf],
  // 1 / D_k to s_rd[buf], y_k to s_y[buf]. Column j: lane j forms the pivot, readlane broadcasts
  // it and row j, lanes i > j form L_ij. Every entry takes the operations, in the order, of the
  // serial version (one lane, rows in turn), so the bits are the same with a shorter chain.
  auto diag_factor = [&](int k, const double* src, int buf) {
    const int r = lane;
    double a[7], dm[7];
#pragma unroll
    for (int c = 0; c < 7; c++) a[c] = c <= r ? src[7 * r + c] : 0.0;
    bool ok = true;
    double my_rd = 0.0;
#pragma unroll
    for (int j = 0; j < 7; j++) {
      double d = a[j];  // lane j: the pivot
#pragma unroll
      for (int m = 0; m < j; m++) d -= a[m] * a[m] * dm[m];
      d = bcast(d, j);
      dm[j] = d;
      ok = ok && d != 0.0;
#if !EG_EXACT_ROUNDING  // the pivot reciprocals serve the tolerance-compared path only
      const double rdj = 1.0 / d;
      if (r == j) my_rd = rdj;
#endif
      double t = a[j];  // lanes i > j: L_ij
#pragma unroll
      for (int m = 0; m < j; m++) t -= a[m] * bcast(a[m], j) * dm[m];
#if EG_EXACT_ROUNDING
      t = t / d;
#else
      t = t * rdj;
#endif
      a[j] = r > j ? t : (r == j ? d : a[j]);
    }
    double v = y[7 * k + r];
#pragma unroll
    for (int m = 0; m < 6; m++) {
      const double vm = bcast(v, m);
      if (r > m) v -= a[m] * vm;
    }
    double* Akk = diag_of(k);
#pragma unroll
    for (int c = 0; c < 7; c++)
      if (c <= r) {
        Akk[7 * r + c] = a[c];
        s_kk[buf][7 * r + c] = a[c];
      }
    s_rd[buf][r] = my_rd;
    s_y[buf][r] = v;
    y[7 * k + r] = v;
    if (!ok && r == 0) s_ok = 0;
  };
  if (F > 0 && tid < 7) diag_factor(0, diag_of(0), 0);
  __syncthreads();
  // ---- factorisation + forward solve ----
  for (int k = 0; k < F; k++) {
    const int cur = k & 1;
    const int e0 = EP(k), ne = EP(k + 1) - e0;
    const bool staged = ne <= kPanStage;  // the panel also goes to LDS for the update below
    double an = 0.0;  // wave 0: the next diagonal block, final but for this column's update
    if (wid == 0 && lane < 49 && k + 1 < F) an = diag_of(k + 1)[lane];
    for (int q = tid; q < 7 * ne; q += kFacThreads) {  // panel rows
      const int t = q / 7, r = q % 7;
      double* Aik = L + (EB(e0 + t) + k) * 49 + 7 * r;
      double a[7];
#pragma unroll
      for (int c = 0; c < 7; c++) a[c] = Aik[c];
#pragma unroll
      for (int c = 0; c < 7; c++) {
        double t2 = a[c];
#pragma unroll
        for (int m = 0; m < c; m++) t2 -= a[m] * s_kk[cur][8 * m] * s_kk[cur][7 * c + m];
#if EG_EXACT_ROUNDING
        a[c] = t2 / s_kk[cur][8 * c];
#else
        a[c] = t2 * s_rd[cur][c];
#endif
      }
      double sy = 0.0;
#pragma unroll
      for (int c = 0; c < 7; c++) {
        Aik[c] = a[c];
        if (staged) s_pan[q * 7 + c] = a[c];
        sy += a[c] * s_y[cur][c];
      }
      y[7 * ER(e0 + t) + r] -= sy;
    }
    __syncthreads();
    const bool nxt_in = k + 1 < F && ne > 0 && ER(e0) == k + 1;
    if (wid == 0) {
      if (k + 1 < F) {  // the next diagonal block: its last update, then its factorisation
        if (lane < 49) {
          double v = an;
          if (nxt_in) {
            const int r = lane / 7, c = lane % 7;
            double t = 0.0;
            if (staged) {  // block (k + 1, k): panel block 0
#pragma unroll
              for (int m = 0; m < 7; m++) t += s_pan[7 * r + m] * s_kk[cur][8 * m] * s_pan[7 * c + m];
            } else {
              const double* Ln = L + (EB(e0) + k) * 49;
#pragma unroll
              for (int m = 0; m < 7; m++) t += Ln[7 * r + m] * s_kk[cur][8 * m] * Ln[7 * c + m];
            }
            v -= t;
          }
          s_nx[lane] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane < 7) diag_factor(k + 1, s_nx, cur ^ 1);
      }
    } else {  // trailing update of the rest of the extent (pair 0 is block (k+1, k+1) if nxt_in)
      const int npairs = ne * (ne + 1) / 2;
      for (int q = tid - 64 + (nxt_in ? 49 : 0); q < npairs * 49; q += kFacThreads - 64) {
        const int pair = q / 49, ent = q % 49;
        int ti = (int)((sqrtf(8.0f * (float)pair + 1.0f) - 1.0f) * 0.5f);
        while ((ti + 1) * (ti + 2) / 2 <= pair) ti++;
        while (ti * (ti + 1) / 2 > pair) ti--;
        const int tj = pair - ti * (ti + 1) / 2;
        const int j = ER(e0 + tj);
        const int64_t bi = EB(e0 + ti), bj = EB(e0 + tj);
        const int r = ent / 7, c = ent % 7;
        double t = 0.0;
        if (staged) {
          const double* Lik = s_pan + 49 * ti + 7 * r;
          const double* Ljk = s_pan + 49 * tj + 7 * c;
#pragma unroll
          for (int m = 0; m < 7; m++) t += Lik[m] * s_kk[cur][8 * m] * Ljk[m];
        } else {
          const double* Lik = L + (bi + k) * 49 + 7 * r;
          const double* Ljk = L + (bj + k) * 49 + 7 * c;
#pragma unroll
          for (int m = 0; m < 7; m++) t += Lik[m] * s_kk[cur][8 * m] * Ljk[m];
        }
        L[(bi + j) * 49 + ent] -= t;
      }
    }
    __syncthreads();
  }
  // ---- z = D^-1 y, then L' x = z by wave 0 (column k: x_k = L_kk^-T (z_k - sum L_ik' x_i)) ----
  for (int q = tid; q < 7 * F; q += kFacThreads) y[q] /= diag_of(q / 7)[8 * (q % 7)];
  __syncthreads();
  if (wid == 0) {
    // Lane l = 9 c + t (c < 7, t < 9): component c of extent block t (blocks in groups of 9).
    // Each lane forms its block's seven products L_ik(r, c) x_i(r) at once; the sum over the
    // extent keeps the serial order (block by block, r = 0..6 within a block) as a chain handed
    // from lane t - 1 to lane t (DPP wave shift), so the bits are those of the one-lane loop.
    // The column's L blocks are loaded one column ahead; x of the last kXr columns is read from
    // an LDS ring, older x (loop rows) from y in memory. Then lanes 0-6 solve the diagonal block
    // (lane r holds x_k(r); each subtraction in the serial order).
    const int c = lane / 9, t = lane - 9 * c;
    const bool lane_ok = c < 7;
    // block g0 + t of column k's extent: its L column c, and x of its row when that row is
    // older than the ring (written by this wave kXr+ columns ago; ordered by the wavefront-scope
    // release / acquire closing every column -- AMDGPU memory model, no wait needed)
    auto load_blk = [&](int k, int g0, double (&lv)[7], double (&xv)[7], int& iv) {
      const int e0 = EP(k), ne = EP(k + 1) - e0;
      if (lane_ok && g0 + t < ne) {
        const double* Lik = L + (EB(e0 + g0 + t) + k) * 49 + c;
#pragma unroll
        for (int r = 0; r < 7; r++) lv[r] = Lik[7 * r];
        const int i = ER(e0 + g0 + t);
        iv = i;
        if (i - k > kXr)
#pragma unroll
          for (int r = 0; r < 7; r++) xv[r] = y[7 * i + r];
      }
    };
    auto load_diag = [&](int k, double (&dv)[7]) {  // lane r < 7: Lkk(m, r) for m = 0..6
      if (lane < 7) {
        const double* Lkk = diag_of(k);
#pragma unroll
        for (int m = 0; m < 7; m++) dv[m] = Lkk[7 * m + lane];
      }
    };
    double lnext[7], dnext[7], xnext[7], znext = 0.0;
    int inext = 0;  // the lane's extent row (its block's row i)
#pragma unroll
    for (int r = 0; r < 7; r++) lnext[r] = dnext[r] = xnext[r] = 0.0;
    if (F > 0) {
      load_blk(F - 1, 0, lnext, xnext, inext);
      load_diag(F - 1, dnext);
      if (lane < 7) znext = y[7 * (F - 1) + lane];
    }
    for (int k = F - 1; k >= 0; k--) {
      const int e0 = EP(k), ne = EP(k + 1) - e0;
      double lcur[7], dcur[7], xcur[7];
      const double zcur = znext;  // z_k (lanes 0-6): y below column k is not yet overwritten
      int icur = inext;
#pragma unroll
      for (int r = 0; r < 7; r++) {
        lcur[r] = lnext[r];
        dcur[r] = dnext[r];
        xcur[r] = xnext[r];
      }
      if (k > 0) {  // the next column's blocks and z, in flight under this one
        load_blk(k - 1, 0, lnext, xnext, inext);
        load_diag(k - 1, dnext);
        if (lane < 7) znext = y[7 * (k - 1) + lane];
      }
      double acc = 0.0;
      for (int g0 = 0; g0 < ne; g0 += 9) {
        if (g0 > 0) load_blk(k, g0, lcur, xcur, icur);
        const int tt = g0 + t;
        const bool has = lane_ok && tt < ne;
        const int i = has ? icur : k;
        const bool far = has && i - k > kXr;
        double pr[7];
#pragma unroll
        for (int r = 0; r < 7; r++) {
          const double xi = !has ? 0.0 : far ? xcur[r] : s_xr[(i % kXr) * 7 + r];
          pr[r] = lcur[r] * xi;
        }
        const int steps = min(9, ne - g0);
        double carry = acc;  // lane 9 c + 8 of the previous group: its total, to lane 9 c
        if (g0 > 0) carry = __shfl(acc, lane + 8, 64);
#pragma unroll
        for (int st2 = 0; st2 < 9; st2++) {  // branch-free: lane t keeps step t's sum
          if (st2 < steps) {
            const double prev = bcast_dpp_shr1(acc);
            double v = st2 == 0 ? carry : prev;
#pragma unroll
            for (int r = 0; r < 7; r++) v += pr[r];
            acc = t == st2 ? v : acc;
          }
        }
      }
      // component c's sum sits in lane 9 c + (ne - 1) % 9; lanes 0-6 take it
      const double tot = __shfl(acc, 9 * min(lane, 6) + (ne > 0 ? (ne - 1) % 9 : 0), 64);
      double v = 0.0;
      if (lane < 7) {
        v = zcur;
        if (ne > 0) v -= tot;
      }
      // the diagonal block: x(r) -= Lkk(m, r) x(m) for m = r + 1 .. 6, r = 5 .. 0
      // (lane m - 1 finishes once x(m) is final: all of its subtractions m' = m .. 6 then, in
      // increasing m'; branch-free, the other lanes' copies discarded)
      double xm[7];
#pragma unroll
      for (int m = 6; m >= 1; m--) {
        xm[m] = bcast(v, m);
        double w = v;
#pragma unroll
        for (int mm = m; mm < 7; mm++) w -= dcur[mm] * xm[mm];
        v = lane == m - 1 ? w : v;
      }
      if (lane < 7) {
        s_xr[(k % kXr) * 7 + lane] = v;
        y[7 * k + lane] = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __syncthreads();
  // LinearSolverEigen: a failed factorisation leaves x as it was; the vertex oplus zeroes the
  // scale coordinate of the solver's x when the scale is fixed
  const bool ok = s_ok != 0;
  if (ok)
    for (int q = tid; q < 7 * F; q += kFacThreads) W.x[q] = (G.fix_scale && q % 7 == 6) ? 0.0 : y[q];
  __syncthreads();
  // computeScale: sum x (lambda x + b): 256 strided partials, then a fixed tree
  double sc = 0.0;
  if (tid < 256)
    for (int q = tid; q < 7 * F; q += 256) sc += W.x[q] * (lambda * W.x[q] + W.b[q]);
  if (tid < 256) red[tid] = sc;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) {
    const double t = red[0];
    W.out[1] = t;
    W.out[2] = ok ? 1.0 : 0.0;
  }
}

__global__ __launch_bounds__(256) void eg_update_kernel(EgGraph G, EgState W) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= G.n) return;
  const int f = G.fidx[v];
  double* o = W.S_trial + 8 * v;
  const double* s = W.S + 8 * v;
  if (f < 0) {
    for (int q = 0; q < 8; q++) o[q] = s[q];
    return;
  }
  double u[7];
  for (int q = 0; q < 7; q++) u[q] = W.x[7 * f + q];
  if (G.fix_scale) u[6] = 0;
  const Sim3 N = sim3::sim3_mul(sim3::sim3_exp(u), sim3::sim3_load(s));
  sim3::sim3_store(N, o);
}

__global__ __launch_bounds__(256) void eg_finish_kernel(EgGraph G, const double* S_final,
                                                        const double* S_init, float* Tcw,
                                                        float* points, const int32_t* ref,
                                                        int n_points) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < G.n) {
    if (!Tcw) return;
    const Sim3 S = sim3::sim3_load(S_final + 8 * q);
    double R[9];
    se3::quat_to_R(S.r, R);
    const double is = 1. / S.s;
    float* T = Tcw + 16 * q;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) T[4 * i + j] = (float)R[3 * i + j];
      T[4 * i + 3] = (float)(S.t[i] * is);
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
    return;
  }
  const int p = q - G.n;
  if (p >= n_points) return;
  const int v = ref[p];
  const Sim3 Srw = sim3::sim3_load(S_init + 8 * v);
  const Sim3 Swr = sim3::sim3_inverse(sim3::sim3_load(S_final + 8 * v));
  const double X[3] = {points[3 * p], points[3 * p + 1], points[3 * p + 2]};
  double Y[3], Z[3], r1[3], r2[3];
  se3::quat_rotate(Srw.r, X, r1);
  for (int i = 0; i < 3; i++) Y[i] = Srw.s * r1[i] + Srw.t[i];
  se3::quat_rotate(Swr.r, Y, r2);
  for (int i = 0; i < 3; i++) Z[i] = Swr.s * r2[i] + Swr.t[i];
  for (int i = 0; i < 3; i++) points[3 * p + i] = (float)Z[i];
}

int blocks_of(int n, int t) { return (n + t - 1) / t; }

}  // namespace

hipError_t launch_eg_linearize(const EgGraph& G, const EgState& W, hipStream_t st) {
  if (G.n_edges <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("eg_jac", st, eg_jac_kernel,
                 dim3(blocks_of(G.n_edges * kEgJacThreads, 256)), dim3(256), 0, st, G, W);
  SLAMGPU_LAUNCH("eg_products", st, eg_products_kernel, dim3(blocks_of(G.n_edges * 7, 256)),
                 dim3(256), 0, st, G, W);
  return hipGetLastError();
}

hipError_t launch_eg_errors(const EgGraph& G, const double* S, const EgState& W, hipStream_t st) {
  if (G.n_edges <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("eg_errors", st, eg_errors_kernel, dim3(blocks_of(G.n_edges, 256)), dim3(256), 0,
                 st, G, S, W);
  return hipGetLastError();
}

hipError_t launch_eg_chi2_sum(const EgGraph& G, const EgState& W, hipStream_t st) {
  SLAMGPU_LAUNCH("eg_chi2_sum", st, eg_chi2_sum_kernel, dim3(1), dim3(256), 0, st, G, W);
  return hipGetLastError();
}

hipError_t launch_eg_assemble(const EgGraph& G, const EgState& W, int64_t n_blocks,
                              hipStream_t st) {
  hipError_t e = hipMemsetAsync(W.H, 0, (size_t)n_blocks * 49 * sizeof(double), st);
  if (e != hipSuccess) return e;
  if (G.n_targets <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("eg_assemble", st, eg_assemble_kernel, dim3(G.n_targets), dim3(64), 0, st, G, W);
  return hipGetLastError();
}

// Dynamic LDS the staged variant may take on the current device: the per-work-group limit less
// the kernel's static arrays (s_pan and the rest, ~45 KB), at most 100 KB (the gfx950 choice);
// queried once per device.
static size_t eg_meta_limit() {
  static std::atomic<int64_t> cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  int64_t v = cache[dev].load(std::memory_order_relaxed);
  if (v == 0) {
    int max_lds = 0;
    hipFuncAttributes a{};
    if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) !=
            hipSuccess ||
        hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&eg_factor_solve_kernel<true>)) !=
            hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    v = std::min<int64_t>(100 * 1024, (int64_t)max_lds - (int64_t)a.sharedSizeBytes);
    v = std::max<int64_t>(v, -1);  // -1: nothing fits (cached as such)
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v > 0 ? (size_t)v : 0;
}

// Dynamic LDS of the staged-structure factorisation, 0 when it does not fit beside the static
// arrays on this device or a block index exceeds 31 bits (then the global-memory variant runs).
static size_t eg_meta_bytes(const EgGraph& G) {
  if (G.n_ext < 0 || G.n_blocks > INT32_MAX) return 0;
  const size_t b = 4 * (2 * (size_t)G.F + 1 + 2 * (size_t)G.n_ext);
  return b <= eg_meta_limit() ? b : 0;
}

hipError_t launch_eg_factor_solve(const EgGraph& G, const EgState& W, int64_t n_blocks,
                                  double lambda, hipStream_t st) {
  hipError_t e = hipMemcpyAsync(W.L, W.H, (size_t)n_blocks * 49 * sizeof(double),
                                hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return e;
  const size_t meta = eg_meta_bytes(G);
  if (meta > 0)
    SLAMGPU_LAUNCH("eg_factor_solve", st, eg_factor_solve_kernel<true>, dim3(1), dim3(kFacThreads),
                   meta, st, G, W, n_blocks, lambda);
  else
    SLAMGPU_LAUNCH("eg_factor_solve", st, eg_factor_solve_kernel<false>, dim3(1), dim3(kFacThreads),
                   0, st, G, W, n_blocks, lambda);
  return hipGetLastError();
}

hipError_t launch_eg_update(const EgGraph& G, const EgState& W, hipStream_t st) {
  if (G.n <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("eg_update", st, eg_update_kernel, dim3(blocks_of(G.n, 256)), dim3(256), 0, st,
                 G, W);
  return hipGetLastError();
}

hipError_t launch_eg_finish(const EgGraph& G, const double* S_final, const double* S_init,
                            float* Tcw, float* points, const int32_t* point_ref, int n_points,
                            hipStream_t st) {
  const int total = G.n + (points ? n_points : 0);
  if (total <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("eg_finish", st, eg_finish_kernel, dim3(blocks_of(total, 256)), dim3(256), 0, st,
                 G, S_final, S_init, Tcw, points, point_ref, points ? n_points : 0);
  return hipGetLastError();
}

}  // namespace slamgpu
