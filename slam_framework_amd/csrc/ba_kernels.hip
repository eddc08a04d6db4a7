// ba_kernels.hip -- Optimizer::LocalBundleAdjustment (optimizer.cpp:413-716) on the device.
//
// One 1024-thread workgroup per problem runs the reference's whole schedule: 5 robust LM
// iterations, the level-1 outlier test, 10 plain iterations, the erase test and the write-back.
// Every LM trial solves the full system by the Schur complement on the points, as g2o's
// BlockSolver does (block_solver.hpp:351-497):
//
//   point pass   (thread per point)   Dinv_p = (Hll_p + lambda I)^-1, db_p = Dinv_p bl_p
//   S assembly   (wave per 6x6 block) S(kh, kl) = [kh == kl](Hpp + lambda I)
//                                       - sum over the points seen by both Hpl_e(kh) Dinv_p Hpl_e(kl)^T
//                                     lanes over the block's point pairs, deterministic wave sums
//   reduced rhs  (wave per keyframe)  bs_k = bp_k - sum_e Hpl_e db_p
//   LDLT         (whole workgroup)    S in LDS (lower triangle, 6K <= 144), 6x6-blocked
//                                     right-looking factorisation with the forward solve fused
//   back-subst.  (thread per point)   xl_p = Dinv_p (bl_p - sum_e Hpl_e^T xp_k)
//
// The pairs of every S block are listed once per phase (the active edge set only changes between
// the phases) in point order with ballot prefix counts, so every sum runs in a fixed order: the
// kernel is deterministic, with no floating-point atomics. Linearisation is a point pass (error,
// chi2, Huber weight, point and pose Jacobians, Hll, bl, Hpl per edge) and a keyframe pass (a wave
// per local keyframe sums Hpp and bp over its edges). FP64 throughout, with the reference's f32
// quirks (types_six_dof_expmap.cpp:150-157: float inverse depth, bf * invz as a float product).
// MFMA is not used: the Schur blocks are 6x3 by 3x6 products scattered over ~10^4 point pairs,
// and FP64 MFMA has the FP64 vector rate on gfx950.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "ba_kernels.h"
#include "ba_device.h"
#include "device_math.h"
#include "se3_device.h"

namespace slamgpu {
namespace {

using namespace ba;

// SLAMGPU_BA_PROFILE: thread 0 accumulates shader-clock cycles per phase into status[] slots
// after the problem's own (tools/ba_profile.py, an instrumented build only). BA_TICK adds a
// barrier only in that build: the kernel's own barriers are explicit.
#ifdef SLAMGPU_BA_PROFILE
#define BA_TICK(slot)                                       \
  do {                                                      \
    __syncthreads();                                        \
    const long long t_ = clock64();                         \
    if (threadIdx.x == 0) prof[slot] += (double)(t_ - t_last); \
    t_last = t_;                                            \
  } while (0)
#else
#define BA_TICK(slot) \
  do {                \
  } while (0)
#endif

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxK = SLAMGPU_BA_MAX_LOCAL_KF;
constexpr int kMaxN = 6 * kMaxK;
constexpr int kMaxBlk = kMaxK * (kMaxK + 1) / 2;
constexpr int kPairsPerObs = (kMaxK + 2) / 2;  // >= (m + 1) / 2 pairs per free edge, m <= kMaxK


struct BaShared {
  double S[kMaxN * (kMaxN + 1) / 2];  // reduced camera system, packed lower triangle
  double rhs[kMaxN];                  // bs, then y = L^-1 bs, then the solution
  double xp[kMaxN];                   // the pose step of the last successful solve (g2o's _x)
  double dg[kMaxN];                   // D of the LDLT
  double V[kMaxN][6];                 // panel L_IJ D_J of the current block column
  double red[2][kWaves][2];           // block-sum partials (double-buffered)
  int blk_cnt[kMaxBlk];
  int blk_off[kMaxBlk + 1];
  int blk_run[kMaxBlk];
  int wcnt[kWaves][kMaxBlk];
  int blk_kk[kMaxBlk];  // kh << 8 | kl
  int8_t free_of_kf[SLAMGPU_BA_MAX_KF];
  int kf_of_free[kMaxK];
  int K, err, ok;
  int rb;
  int stop;  // the last stop-flag poll (one read per poll, by thread 0)
};

// g2o's SparseOptimizer::terminate() (*forceStopFlag, sparse_optimizer.h:188) for the whole
// work-group: thread 0 reads the flag once (system scope: the flag may be host-mapped memory a
// host thread raises while the kernel runs) and every thread takes that one value, so a flag
// raised mid-poll cannot split the work-group's control flow. Contains a barrier.
__device__ __forceinline__ bool poll_stop(BaShared& sh, const int32_t* stop_flag) {
  if (!stop_flag) return false;
  if (threadIdx.x == 0)
    sh.stop = __hip_atomic_load(stop_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  __syncthreads();
  const bool r = sh.stop != 0;
  __syncthreads();  // sh.stop is not rewritten before every thread has read it
  return r;
}

// Deterministic block sum of two values: wave butterflies (bitwise identical in every lane), wave
// partials summed in wave order by every thread.
__device__ __forceinline__ void block_sum2(BaShared& sh, double& a, double& b) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, w = wave_id();
  if (lane == 0) {
    sh.red[sh.rb][w][0] = a;
    sh.red[sh.rb][w][1] = b;
  }
  __syncthreads();
  double s0 = 0.0, s1 = 0.0;
  for (int k = 0; k < kWaves; k++) {
    s0 += sh.red[sh.rb][k][0];
    s1 += sh.red[sh.rb][k][1];
  }
  a = s0;
  b = s1;
  __syncthreads();  // every reader done before the buffer flips back
  if (threadIdx.x == 0) sh.rb ^= 1;
  __syncthreads();
}

__device__ __forceinline__ double block_max(BaShared& sh, double a) {
  a = wave_max(a);
  const int lane = threadIdx.x & 63, w = wave_id();
  if (lane == 0) sh.red[sh.rb][w][0] = a;
  __syncthreads();
  double m = 0.0;
  for (int k = 0; k < kWaves; k++) m = fmax(m, sh.red[sh.rb][k][0]);
  __syncthreads();
  if (threadIdx.x == 0) sh.rb ^= 1;
  __syncthreads();
  return m;
}


struct Problem {
  const slamgpu_ba_obs* obs;
  const int32_t* pstart;  // point's first observation (global)
  int o0, n_obs, p0, n_pts, k0, n_kf;
  BaWorkspace ws;
};

__device__ __forceinline__ double* kfrec(const Problem& pb, int kf) {
  return pb.ws.kf + (size_t)(pb.k0 + kf) * 64;
}
struct PtRef {  // the SoA fields of one point
  double* base;
  size_t stride;
  __device__ __forceinline__ double& operator[](int f) const { return base[(size_t)f * stride]; }
};
__device__ __forceinline__ PtRef ptrec(const Problem& pb, int p) {
  return PtRef{pb.ws.pt + pb.p0 + p, (size_t)pb.ws.n_pt};
}

// ---- structure of the active edge set ------------------------------------------------------------
// Per point: the mask of local keyframes it has active edges to and those edges sorted by local
// keyframe (psorted). Per S block (kh >= kl): the list of its point pairs in point order, built
// with wave ballots and prefix counts (no atomics on positions). A diagonal block (k, k) lists
// (edge, point): it doubles as keyframe k's edge list.
__device__ void build_structure(BaShared& sh, const Problem& pb, bool diag_only = false) {
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), K = sh.K;
  const int nblk = K * (K + 1) / 2;
  for (int b = tid; b < nblk; b += kThreads) {
    sh.blk_cnt[b] = 0;
    sh.blk_run[b] = 0;
  }
  // per point mask + sorted active free edges
  for (int p = tid; p < pb.n_pts; p += kThreads) {
    const int s = pb.pstart[pb.p0 + p] - pb.o0, e1 = pb.pstart[pb.p0 + p + 1] - pb.o0;
    uint32_t mask = 0;
    int m = 0;
    for (int e = s; e < e1; e++) {
      if (!pb.ws.act[pb.o0 + e]) continue;
      const int f = sh.free_of_kf[pb.obs[pb.o0 + e].keyframe];
      if (f < 0) continue;
      mask |= 1u << f;
      // insertion by local keyframe index into psorted[s .. s + m)
      int i = m;
      while (i > 0) {
        const int prev = pb.ws.psorted[pb.o0 + s + i - 1];
        if (sh.free_of_kf[pb.obs[pb.o0 + prev].keyframe] < f) break;
        pb.ws.psorted[pb.o0 + s + i] = prev;
        i--;
      }
      pb.ws.psorted[pb.o0 + s + i] = e;
      m++;
    }
    pb.ws.pmask[pb.p0 + p] = mask;
  }
  __syncthreads();
  // pass 1: pair counts per block
  for (int base = 0; base < pb.n_pts; base += kThreads) {
    const int p = base + tid;
    const uint32_t mask = p < pb.n_pts ? pb.ws.pmask[pb.p0 + p] : 0u;
    uint32_t om = 0;
    for (int k = 0; k < K; k++) om |= __ballot((mask >> k) & 1) ? (1u << k) : 0u;
    for (uint32_t a = om; a; a &= a - 1) {
      const int kh = __builtin_ctz(a);
      for (uint32_t c = diag_only ? (1u << kh) : om & ((2u << kh) - 1); c; c &= c - 1) {
        const int kl = __builtin_ctz(c);
        const uint64_t bal = __ballot(((mask >> kh) & 1) && ((mask >> kl) & 1));
        if (lane == 0 && bal) atomicAdd(&sh.blk_cnt[tri(kh) + kl], __popcll(bal));
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int off = 0;
    for (int b = 0; b < nblk; b++) {
      sh.blk_off[b] = off;
      off += sh.blk_cnt[b];
    }
    sh.blk_off[nblk] = off;
    for (int kh = 0; kh < K; kh++)
      for (int kl = 0; kl <= kh; kl++) sh.blk_kk[tri(kh) + kl] = kh << 8 | kl;
  }
  __syncthreads();
  // pass 2: positions (block offset + earlier rounds + earlier waves + earlier lanes)
  int2* hits = pb.ws.hits + (size_t)pb.o0 * kPairsPerObs;
  for (int base = 0; base < pb.n_pts; base += kThreads) {
    for (int i = tid; i < kWaves * nblk; i += kThreads) sh.wcnt[i / nblk][i % nblk] = 0;
    __syncthreads();
    const int p = base + tid;
    const uint32_t mask = p < pb.n_pts ? pb.ws.pmask[pb.p0 + p] : 0u;
    uint32_t om = 0;
    for (int k = 0; k < K; k++) om |= __ballot((mask >> k) & 1) ? (1u << k) : 0u;
    for (uint32_t a = om; a; a &= a - 1) {
      const int kh = __builtin_ctz(a);
      for (uint32_t c = diag_only ? (1u << kh) : om & ((2u << kh) - 1); c; c &= c - 1) {
        const int kl = __builtin_ctz(c);
        const uint64_t bal = __ballot(((mask >> kh) & 1) && ((mask >> kl) & 1));
        if (lane == 0) sh.wcnt[w][tri(kh) + kl] = __popcll(bal);
      }
    }
    __syncthreads();
    for (int b = tid; b < nblk; b += kThreads) {
      int run = sh.blk_run[b];
      for (int k = 0; k < kWaves; k++) {
        const int c = sh.wcnt[k][b];
        sh.wcnt[k][b] = run;
        run += c;
      }
      sh.blk_run[b] = run;
    }
    __syncthreads();
    const int s = p < pb.n_pts ? pb.pstart[pb.p0 + p] - pb.o0 : 0;
    for (uint32_t a = om; a; a &= a - 1) {
      const int kh = __builtin_ctz(a);
      for (uint32_t c = diag_only ? (1u << kh) : om & ((2u << kh) - 1); c; c &= c - 1) {
        const int kl = __builtin_ctz(c);
        const bool mine = ((mask >> kh) & 1) && ((mask >> kl) & 1);
        const uint64_t bal = __ballot(mine);
        if (mine) {
          const int b = tri(kh) + kl;
          const int pos = sh.blk_off[b] + sh.wcnt[w][b] + (int)lanes_below(bal);
          const int eh = pb.ws.psorted[pb.o0 + s + __popc(mask & ((1u << kh) - 1))];
          const int el = pb.ws.psorted[pb.o0 + s + __popc(mask & ((1u << kl) - 1))];
          hits[pos] = kh == kl ? make_int2(eh, p) : make_int2(eh, el);
        }
      }
    }
    __syncthreads();
  }
}

// ---- linearisation ------------------------------------------------------------------------------
// Edge pass: errors and chi2 of the active edges (stored: g2o keeps the last error per edge), the
// edge's Hll and bl terms and its Hpl block; adds this thread's robust chi2 to `chi`.
__device__ void linearise_edges(BaShared& sh, const Problem& pb, const PoseParams& P,
                                const float* isig, bool robust, double& chi) {
  for (int e = threadIdx.x; e < pb.n_obs; e += kThreads) {
    const int ge = pb.o0 + e;
    if (!pb.ws.act[ge]) continue;
    const PtRef pr = ptrec(pb, pb.ws.opoint[ge]);
    const double X[3] = {pr[PX], pr[PX + 1], pr[PX + 2]};
    const slamgpu_ba_obs o = pb.obs[ge];
    const double* kr = kfrec(pb, o.keyframe);
    ObsEval v;
    const double c2 = eval_obs(o, P, isig, kr, X, v);
    pb.ws.chi2[ge] = c2;
    double wgt = 1.0;
    if (robust) {
      const double d = huber_delta(v.stereo), d2 = d * d;
      if (c2 > d2) {
        const double sq = sqrt(c2);
        chi += 2 * sq * d - d2;
        wgt = d / sq;
      } else {
        chi += c2;
      }
    } else {
      chi += c2;
    }
    double Jl[3][3], Jp[3][6];
    obs_jacobians(v, P, kr, Jl, Jp);
    const double W = wgt * v.info;
    // omega_r = -Omega e * rho' (base_binary_edge.hpp:72-110)
    const double or0 = -(v.info * v.e[0]) * wgt, or1 = -(v.info * v.e[1]) * wgt,
                 or2 = -(v.info * v.e[2]) * wgt;
    double* hb = pb.ws.ehb + (size_t)ge * 9;
    for (int i = 0; i < 3; i++) {
      hb[6 + i] = Jl[0][i] * or0 + Jl[1][i] * or1 + Jl[2][i] * or2;
      for (int j = i; j < 3; j++)
        hb[s3(i, j)] = (Jl[0][i] * W) * Jl[0][j] + (Jl[1][i] * W) * Jl[1][j] +
                       (Jl[2][i] * W) * Jl[2][j];
    }
    if (sh.free_of_kf[o.keyframe] >= 0) {
      double* hp = pb.ws.hpl + (size_t)ge * 18;
      for (int i = 0; i < 6; i++)
        for (int j = 0; j < 3; j++)
          hp[3 * i + j] = (Jp[0][i] * W) * Jl[0][j] + (Jp[1][i] * W) * Jl[1][j] +
                          (Jp[2][i] * W) * Jl[2][j];
    }
  }
}

// Point pass: Hll and bl as the sums of the point's edge terms in edge order; max |Hll_jj|.
__device__ void sum_points(const Problem& pb, double& maxd) {
  for (int p = threadIdx.x; p < pb.n_pts; p += kThreads) {
    const PtRef pr = ptrec(pb, p);
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int nact = 0;
    const int s = pb.pstart[pb.p0 + p], e1 = pb.pstart[pb.p0 + p + 1];
    for (int ge = s; ge < e1; ge++) {
      if (!pb.ws.act[ge]) continue;
      nact++;
      const double* hb = pb.ws.ehb + (size_t)ge * 9;
#pragma unroll
      for (int i = 0; i < 9; i++) H[i] += hb[i];
    }
    for (int i = 0; i < 6; i++) pr[PH + i] = H[i];
    for (int i = 0; i < 3; i++) pr[PB + i] = H[6 + i];
    if (nact) maxd = fmax(maxd, fmax(fabs(H[0]), fmax(fabs(H[3]), fabs(H[5]))));
  }
}

// Keyframe pass: a wave per local keyframe sums Hpp (upper triangle) and bp over its active
// edges (the diagonal block's pair list, in point order); returns max |Hpp_jj| partials.
__device__ void linearise_keyframes(BaShared& sh, const Problem& pb, const PoseParams& P,
                                    const float* isig, bool robust, double& maxd) {
  const int lane = threadIdx.x & 63, w = wave_id(), K = sh.K;
  const int2* hits = pb.ws.hits + (size_t)pb.o0 * kPairsPerObs;
  for (int f = w; f < K; f += kWaves) {
    const int b = tri(f) + f, cnt = sh.blk_cnt[b], off = sh.blk_off[b];
    double* kr = kfrec(pb, sh.kf_of_free[f]);
    double acc[32];
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = 0.0;
    for (int h = lane; h < cnt; h += 64) {
      const int2 ep = hits[off + h];
      const int ge = pb.o0 + ep.x;
      const PtRef pr = ptrec(pb, ep.y);
      const double X[3] = {pr[PX], pr[PX + 1], pr[PX + 2]};
      ObsEval v;
      const double c2 = eval_obs(pb.obs[ge], P, isig, kr, X, v);
      double wgt = 1.0;
      if (robust) {
        const double d = huber_delta(v.stereo);
        if (c2 > d * d) wgt = d / sqrt(c2);
      }
      double Jl[3][3], Jp[3][6];
      obs_jacobians(v, P, kr, Jl, Jp);
      const double W = wgt * v.info;
      const double or0 = -(v.info * v.e[0]) * wgt, or1 = -(v.info * v.e[1]) * wgt,
                   or2 = -(v.info * v.e[2]) * wgt;
      int hh = 0;
#pragma unroll
      for (int a = 0; a < 6; a++) {
        acc[21 + a] += Jp[0][a] * or0 + Jp[1][a] * or1 + Jp[2][a] * or2;
        const double wa0 = Jp[0][a] * W, wa1 = Jp[1][a] * W, wa2 = Jp[2][a] * W;
#pragma unroll
        for (int c = a; c < 6; c++, hh++) acc[hh] += wa0 * Jp[0][c] + wa1 * Jp[1][c] + wa2 * Jp[2][c];
      }
    }
    const double s = wave_reduce_scatter32(acc);
    if ((lane & 1) == 0 && (lane >> 1) < 27) kr[KH + (lane >> 1)] = s;
    if (cnt > 0) {
      const bool dg = (lane & 1) == 0 && (lane >> 1) < 21 &&
                      ((lane >> 1) == 0 || (lane >> 1) == 6 || (lane >> 1) == 11 ||
                       (lane >> 1) == 15 || (lane >> 1) == 18 || (lane >> 1) == 20);
      maxd = fmax(maxd, dg ? fabs(s) : 0.0);
    }
  }
}

// ---- one LM trial: Schur solve ------------------------------------------------------------------
__device__ void schur_points(const Problem& pb, double lambda) {
  for (int p = threadIdx.x; p < pb.n_pts; p += kThreads) {
    const PtRef pr = ptrec(pb, p);
    double D[6], Di[6];
    for (int i = 0; i < 6; i++) D[i] = pr[PH + i];
    D[0] += lambda;
    D[3] += lambda;
    D[5] += lambda;
    inverse3_sym(D, Di);
    const double b0 = pr[PB], b1 = pr[PB + 1], b2 = pr[PB + 2];
    for (int i = 0; i < 6; i++) pr[PD + i] = Di[i];
    pr[PDB] = Di[0] * b0 + Di[1] * b1 + Di[2] * b2;
    pr[PDB + 1] = Di[1] * b0 + Di[3] * b1 + Di[4] * b2;
    pr[PDB + 2] = Di[2] * b0 + Di[4] * b1 + Di[5] * b2;
  }
}

__device__ void assemble_S(BaShared& sh, const Problem& pb, double lambda) {
  const int lane = threadIdx.x & 63, w = wave_id(), K = sh.K, nblk = K * (K + 1) / 2;
  const int2* hits = pb.ws.hits + (size_t)pb.o0 * kPairsPerObs;
  for (int b = w; b < nblk; b += kWaves) {
    const int kh = sh.blk_kk[b] >> 8, kl = sh.blk_kk[b] & 255;
    const int cnt = sh.blk_cnt[b], off = sh.blk_off[b];
    const bool diag = kh == kl;
    const double* kr = kfrec(pb, sh.kf_of_free[kh]);
    // one pass over the block's pairs: 36 accumulators (rows 0-5 x columns 0-5)
    double acc[64];
#pragma unroll
    for (int i = 0; i < 64; i++) acc[i] = 0.0;
    for (int h = lane; h < cnt; h += 64) {
      const int2 ep = hits[off + h];
      const int eh = pb.o0 + ep.x, el = pb.o0 + (diag ? ep.x : ep.y);
      // B = Hpl_eh Dinv_p, formed here rather than stored per edge (the kernel is bound by
      // the bytes it moves, not by these 54 FMAs)
      const double* hh = pb.ws.hpl + (size_t)eh * 18;
      const double* hp = pb.ws.hpl + (size_t)el * 18;
      const PtRef pr = ptrec(pb, pb.ws.opoint[eh]);
      double Di[6], B[18], Hl[18];
#pragma unroll
      for (int i = 0; i < 6; i++) Di[i] = pr[PD + i];
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const double h0 = hh[3 * i], h1 = hh[3 * i + 1], h2 = hh[3 * i + 2];
        B[3 * i] = h0 * Di[0] + h1 * Di[1] + h2 * Di[2];
        B[3 * i + 1] = h0 * Di[1] + h1 * Di[3] + h2 * Di[4];
        B[3 * i + 2] = h0 * Di[2] + h1 * Di[4] + h2 * Di[5];
      }
#pragma unroll
      for (int i = 0; i < 18; i++) Hl[i] = diag ? hh[i] : hp[i];
#pragma unroll
      for (int r = 0; r < 6; r++)
#pragma unroll
        for (int c = 0; c < 6; c++)
          acc[6 * r + c] += B[3 * r] * Hl[3 * c] + B[3 * r + 1] * Hl[3 * c + 1] +
                            B[3 * r + 2] * Hl[3 * c + 2];
    }
    const double s0 = wave_reduce_scatter32(acc), s1 = wave_reduce_scatter32(acc + 32);
    const int idx = lane >> 1;
#pragma unroll
    for (int part = 0; part < 2; part++) {
      const int id = idx + 32 * part;
      if ((lane & 1) == 0 && id < 36) {
        const int r = id / 6, c = id % 6;
        const int i = 6 * kh + r, j = 6 * kl + c;
        if (!diag || j <= i) {
          double base = 0.0;
          if (diag) base = kr[KH + hidx(c, r)] + (r == c ? lambda : 0.0);
          sh.S[sidx(i, j)] = base - (part ? s1 : s0);
        }
      }
    }
  }
  // reduced right-hand side: bs_k = bp_k - sum_e Hpl_e db_p
  for (int f = w; f < K; f += kWaves) {
    const int b = tri(f) + f, cnt = sh.blk_cnt[b], off = sh.blk_off[b];
    const double* kr = kfrec(pb, sh.kf_of_free[f]);
    double acc[32];
#pragma unroll
    for (int i = 0; i < 32; i++) acc[i] = 0.0;
    for (int h = lane; h < cnt; h += 64) {
      const int2 ep = hits[off + h];
      const double* hp = pb.ws.hpl + (size_t)(pb.o0 + ep.x) * 18;
      const PtRef pr = ptrec(pb, ep.y);
      const double d0 = pr[PDB], d1 = pr[PDB + 1], d2 = pr[PDB + 2];
#pragma unroll
      for (int i = 0; i < 6; i++) acc[i] += hp[3 * i] * d0 + hp[3 * i + 1] * d1 + hp[3 * i + 2] * d2;
    }
    const double s = wave_reduce_scatter32(acc);
    if ((lane & 1) == 0 && (lane >> 1) < 6) sh.rhs[6 * f + (lane >> 1)] = kr[KB + (lane >> 1)] - s;
  }
}

// LDLT of S (n = 6K, 6x6 block columns, right-looking) with the forward solve of the rhs fused;
// then D^-1 and the backward solve by wave 0. Fails (sh.ok = 0) on an exact zero pivot, as
// Eigen's SimplicialLDLT does. On success sh.xp receives the solution; on failure it keeps the
// previous one, which g2o applies anyway (optimization_algorithm_levenberg.cpp:107-109).
__device__ void factor_solve(BaShared& sh) {
  const int tid = threadIdx.x, lane = tid & 63, K = sh.K, n = 6 * K;
  if (tid == 0) sh.ok = 1;
  __syncthreads();
  for (int J = 0; J < K; J++) {
    const int j0 = 6 * J;
    // 1. diagonal block: unblocked LDLT of the 6x6 in one lane's registers, forward-solve its rhs
    if (tid == 0) {
      double A[6][6], d[6], y[6];
#pragma unroll
      for (int i = 0; i < 6; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) A[i][j] = sh.S[sidx(j0 + i, j0 + j)];
        y[i] = sh.rhs[j0 + i];
      }
      bool good = true;
#pragma unroll
      for (int j = 0; j < 6; j++) {
        double dj = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) dj -= A[j][k] * A[j][k] * d[k];
        good = good && dj != 0.0;
        d[j] = dj;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
          double s = A[i][j];
#pragma unroll
          for (int k = 0; k < j; k++) s -= A[i][k] * A[j][k] * d[k];
          A[i][j] = dj != 0.0 ? s / dj : 0.0;
        }
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
#pragma unroll
        for (int k = 0; k < i; k++) y[i] -= A[i][k] * y[k];
      }
#pragma unroll
      for (int i = 0; i < 6; i++) {
        sh.dg[j0 + i] = d[i];
        sh.rhs[j0 + i] = y[i];
#pragma unroll
        for (int j = 0; j < i; j++) sh.S[sidx(j0 + i, j0 + j)] = A[i][j];
      }
      if (!good) sh.ok = 0;
    }
    __syncthreads();
    if (!sh.ok) return;
    // 2. panel rows below: V_i = A_iJ L_JJ^-T (so that L_iJ = V_i D_J^-1); rhs_i -= L_iJ y_J
    for (int i = j0 + 6 + tid; i < n; i += kThreads) {
      double v[6];
      for (int c = 0; c < 6; c++) {
        double s = sh.S[sidx(i, j0 + c)];
        for (int k = 0; k < c; k++) s -= v[k] * sh.S[sidx(j0 + c, j0 + k)];
        v[c] = s;
      }
      double r = sh.rhs[i];
      for (int c = 0; c < 6; c++) {
        sh.V[i][c] = v[c];
        const double l = v[c] / sh.dg[j0 + c];
        sh.S[sidx(i, j0 + c)] = l;
        r -= l * sh.rhs[j0 + c];
      }
      sh.rhs[i] = r;
    }
    __syncthreads();
    // 3. trailing update A_ik -= sum_c L_ic D_c L_kc = sum_c L_ic V_kc, j0 + 6 <= k <= i
    const int m = n - j0 - 6;
    for (int q = tid; q < m * m; q += kThreads) {
      const int ii = q / m, kk = q - ii * m;
      if (kk > ii) continue;
      const int i = j0 + 6 + ii, k = j0 + 6 + kk;
      double s = sh.S[sidx(i, k)];
#pragma unroll
      for (int c = 0; c < 6; c++) s -= sh.S[sidx(i, j0 + c)] * sh.V[k][c];
      sh.S[sidx(i, k)] = s;
    }
    __syncthreads();
  }
  // D^-1, then L^T x = z (wave 0, column-oriented from the last row)
  if (wave_id() == 0) {
    for (int i = lane; i < n; i += 64) sh.rhs[i] /= sh.dg[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int k = n - 1; k > 0; k--) {
      const double xk = sh.rhs[k];
      for (int i = lane; i < k; i += 64) sh.rhs[i] -= sh.S[sidx(k, i)] * xk;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    for (int i = lane; i < n; i += 64) sh.xp[i] = sh.rhs[i];
  }
  __syncthreads();
}

// ---- kernel -----------------------------------------------------------------------------------
// Problem setup shared by the kernels: local-keyframe map, validation (status < 0 on error),
// initial estimates (Converter::toSE3Quat / toVector3d), every edge active.
__device__ bool ba_setup(BaShared& sh, Problem& pb, float* isig, const PoseParams& P,
                         const slamgpu_ba_problem* problems, const float* kf_Tcw,
                         const uint8_t* kf_mode, const float* points, const int32_t* pstart,
                         const slamgpu_ba_obs* obs, int32_t* status, const BaWorkspace& ws) {
  const int tid = threadIdx.x;
  const slamgpu_ba_problem pr = problems[blockIdx.x];
  pb.obs = obs;
  pb.pstart = pstart;
  pb.p0 = pr.point_begin;
  pb.n_pts = pr.n_points;
  pb.k0 = pr.kf_begin;
  pb.n_kf = pr.n_kf;
  pb.o0 = pstart[pb.p0];
  pb.n_obs = pstart[pb.p0 + pb.n_pts] - pb.o0;
  pb.ws = ws;
  if (tid < SLAMGPU_MAX_LEVELS) isig[tid] = P.inv_sigma2[tid];
  if (tid == 0) {
    sh.err = 0;
    sh.rb = 0;
    int K = 0;
    if (pb.n_kf > SLAMGPU_BA_MAX_KF || pb.n_kf < 0) {
      sh.err = -3;
    } else {
      for (int k = 0; k < pb.n_kf; k++) {
        const bool fr = kf_mode[pb.k0 + k] == SLAMGPU_KF_LOCAL;
        if (fr && K < kMaxK) sh.kf_of_free[K] = k;
        sh.free_of_kf[k] = fr ? (int8_t)(K < kMaxK ? K : -1) : (int8_t)-1;
        K += fr;
      }
      if (K > kMaxK) sh.err = -1;
    }
    sh.K = K;
  }
  __syncthreads();
  // validation: keyframe indices and one observation per keyframe per point
  if (sh.err == 0) {
    for (int p = tid; p < pb.n_pts; p += kThreads) {
      const int s = pstart[pb.p0 + p], e1 = pstart[pb.p0 + p + 1];
      for (int e = s; e < e1; e++) {
        const int k = obs[e].keyframe;
        if (k < 0 || k >= pb.n_kf) {
          atomicMin(&sh.err, -3);
          break;
        }
        for (int e2 = s; e2 < e; e2++)
          if (obs[e2].keyframe == k) atomicMin(&sh.err, -2);
      }
    }
  }
  __syncthreads();
  if (sh.err != 0) {
    if (tid == 0) status[blockIdx.x] = sh.err;
    return false;
  }
  for (int k = tid; k < pb.n_kf; k += kThreads) {
    const float* T = kf_Tcw + (size_t)(pb.k0 + k) * 16;
    double R[9];
    SE3 E;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) R[3 * i + j] = T[4 * i + j];
      E.t[i] = T[4 * i + 3];
    }
    E.r = se3::quat_from_R(R);
    se3::normalize_rotation(E.r);
    store_T(kfrec(pb, k), E);
  }
  for (int p = tid; p < pb.n_pts; p += kThreads) {
    const PtRef r = ptrec(pb, p);
    for (int i = 0; i < 3; i++) r[PX + i] = points[(size_t)(pb.p0 + p) * 3 + i];
    for (int i = 0; i < 3; i++) r[PXL + i] = 0.0;
    for (int ge = pstart[pb.p0 + p]; ge < pstart[pb.p0 + p + 1]; ge++) ws.opoint[ge] = p;
  }
  for (int e = tid; e < pb.n_obs; e += kThreads) {
    ws.act[pb.o0 + e] = 1;
    ws.chi2[pb.o0 + e] = 0.0;
  }
  if (tid < kMaxN) sh.xp[tid] = 0.0;
  __syncthreads();
  return true;
}

__global__ __launch_bounds__(kThreads) void local_ba_kernel(
    PoseParams P, const slamgpu_ba_problem* __restrict__ problems, float* __restrict__ kf_Tcw,
    const uint8_t* __restrict__ kf_mode, float* __restrict__ points,
    const int32_t* __restrict__ pstart, const slamgpu_ba_obs* __restrict__ obs,
    uint8_t* __restrict__ erase, int32_t* __restrict__ status, BaWorkspace ws,
    const int32_t* stop_flag) {
#pragma clang fp contract(fast)  // tolerance-compared FP64 path
  __shared__ BaShared sh;
  __shared__ float isig[SLAMGPU_MAX_LEVELS];
  const int tid = threadIdx.x;
  if (poll_stop(sh, stop_flag)) {  // optimizer.cpp:616-618: return before optimising
    const int32_t o0 = pstart[problems[blockIdx.x].point_begin];
    const int32_t o1 = pstart[problems[blockIdx.x].point_begin + problems[blockIdx.x].n_points];
    for (int e = o0 + tid; e < o1; e += kThreads) erase[e] = 0;
    if (tid == 0) status[blockIdx.x] = 0;
    return;
  }
  Problem pb;
  if (!ba_setup(sh, pb, isig, P, problems, kf_Tcw, kf_mode, points, pstart, obs, status, ws))
    return;

  const int K = sh.K, n = 6 * K;
  int lm_total = 0;
#ifdef SLAMGPU_BA_PROFILE
  double prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long t_last = clock64();
#endif
  bool stopped = false;
  for (int phase = 0; phase < 2 && !stopped; phase++) {
    const bool robust = phase == 0;
    const int iterations = phase == 0 ? 5 : 10;
    BA_TICK(7);
    build_structure(sh, pb);
    BA_TICK(0);
    double lambda = 0.0;
    int ni = 2, nbad = 0;
    for (int it = 0; it < iterations; it++) {
      if (poll_stop(sh, stop_flag)) {  // optimize(): i < iterations && !terminate() && ok
        stopped = true;
        break;
      }
      // ---- linearise: computeActiveErrors + activeRobustChi2 + buildSystem ----
      double chi = 0.0, maxd = 0.0;
      BA_TICK(7);
      linearise_edges(sh, pb, P, isig, robust, chi);
      linearise_keyframes(sh, pb, P, isig, robust, maxd);
      __syncthreads();
      sum_points(pb, maxd);
      BA_TICK(1);
      __syncthreads();
      double zero = 0.0;
      block_sum2(sh, chi, zero);
      double currentChi = chi;
      const double iniChi = currentChi;
      if (it == 0) {  // computeLambdaInit over the active vertices
        lambda = 1e-5 * block_max(sh, maxd);
        ni = 2;
        nbad = 0;
      }
      double rho = 0.0;
      int qmax = 0;
      do {
        // ---- solve ----
        BA_TICK(7);
        schur_points(pb, lambda);
        __syncthreads();
        BA_TICK(2);
        assemble_S(sh, pb, lambda);
        __syncthreads();
        BA_TICK(3);
        factor_solve(sh);  // ends with a barrier; sh.xp = the pose step when sh.ok
        BA_TICK(4);
        const bool ok = sh.ok;
        // ---- update (backup first): points X += xl, keyframes exp(xp) * T ----
        double scale = 0.0, temp = 0.0;
        if (ok) {  // Hpl_e^T xp per local-keyframe edge (a failed solve keeps g2o's old _x)
          for (int e = tid; e < pb.n_obs; e += kThreads) {
            const int ge = pb.o0 + e;
            const int f = sh.free_of_kf[obs[ge].keyframe];
            if (!ws.act[ge] || f < 0) continue;
            const double* hp = ws.hpl + (size_t)ge * 18;
            double c0 = 0, c1 = 0, c2 = 0;
            for (int i = 0; i < 6; i++) {
              const double x = sh.xp[6 * f + i];
              c0 += hp[3 * i] * x;
              c1 += hp[3 * i + 1] * x;
              c2 += hp[3 * i + 2] * x;
            }
            double* hb = ws.ehb + (size_t)ge * 9;
            hb[0] = c0;
            hb[1] = c1;
            hb[2] = c2;
          }
          __syncthreads();
        }
        for (int p = tid; p < pb.n_pts; p += kThreads) {
          const PtRef r = ptrec(pb, p);
          const int s = pstart[pb.p0 + p], e1 = pstart[pb.p0 + p + 1];
          int nact = 0;
          double c0 = r[PB], c1 = r[PB + 1], c2 = r[PB + 2];
          for (int ge = s; ge < e1; ge++) {
            if (!ws.act[ge]) continue;
            nact++;
            if (!ok || sh.free_of_kf[obs[ge].keyframe] < 0) continue;
            const double* hb = ws.ehb + (size_t)ge * 9;
            c0 -= hb[0];
            c1 -= hb[1];
            c2 -= hb[2];
          }
          if (ok) {
            r[PXL] = r[PD] * c0 + r[PD + 1] * c1 + r[PD + 2] * c2;
            r[PXL + 1] = r[PD + 1] * c0 + r[PD + 3] * c1 + r[PD + 4] * c2;
            r[PXL + 2] = r[PD + 2] * c0 + r[PD + 4] * c1 + r[PD + 5] * c2;
          }
          for (int i = 0; i < 3; i++) r[PXB + i] = r[PX + i];
          if (nact) {  // oplus on the active vertices only
            for (int i = 0; i < 3; i++) {
              const double x = r[PXL + i];
              r[PX + i] += x;
              scale += x * (lambda * x + r[PB + i]);
            }
          }
        }
        if (tid < K) {
          double* kr = kfrec(pb, sh.kf_of_free[tid]);
          if (sh.blk_cnt[tri(tid) + tid] > 0) {
            double x[6];
            for (int i = 0; i < 6; i++) {
              x[i] = sh.xp[6 * tid + i];
              scale += x[i] * (lambda * x[i] + kr[KB + i]);
            }
            SE3 T;
            load_T(kr, T);
            for (int i = 0; i < 4; i++) kr[KBQ + i] = kr[KQ + i];
            for (int i = 0; i < 3; i++) kr[KBT + i] = kr[KT + i];
            store_T(kr, se3::se3_left_update(x, T));
          }
        }
        __syncthreads();
        // ---- errors at the new estimate (edge-parallel) ----
        for (int e = tid; e < pb.n_obs; e += kThreads) {
          const int ge = pb.o0 + e;
          if (!ws.act[ge]) continue;
          const PtRef r = ptrec(pb, ws.opoint[ge]);
          const double X[3] = {r[PX], r[PX + 1], r[PX + 2]};
          const slamgpu_ba_obs o = obs[ge];
          ObsEval v;
          const double c2 = eval_obs(o, P, isig, kfrec(pb, o.keyframe), X, v);
          ws.chi2[ge] = c2;
          if (robust) {
            const double d = huber_delta(v.stereo), d2 = d * d;
            temp += c2 > d2 ? 2 * sqrt(c2) * d - d2 : c2;
          } else {
            temp += c2;
          }
        }
        BA_TICK(5);
        block_sum2(sh, temp, scale);
        BA_TICK(6);
        double tempChi = ok ? temp : DBL_MAX;
        scale += 1e-3;
        rho = (currentChi - tempChi) / scale;
        if (rho > 0 && isfinite(tempChi)) {
          double alpha = 1. - pow(2 * rho - 1, 3.0);
          alpha = fmin(alpha, 2. / 3.);
          lambda *= fmax(1. / 3., alpha);
          ni = 2;
          currentChi = tempChi;
        } else {
          lambda *= ni;
          ni *= 2;
          // pop: restore the estimates; the edges keep the rejected errors
          for (int p = tid; p < pb.n_pts; p += kThreads) {
            const PtRef r = ptrec(pb, p);
            for (int i = 0; i < 3; i++) r[PX + i] = r[PXB + i];
          }
          if (tid < K) {
            double* kr = kfrec(pb, sh.kf_of_free[tid]);
            if (sh.blk_cnt[tri(tid) + tid] > 0) {
              SE3 T;
              T.r.x = kr[KBQ];
              T.r.y = kr[KBQ + 1];
              T.r.z = kr[KBQ + 2];
              T.r.w = kr[KBQ + 3];
              for (int i = 0; i < 3; i++) T.t[i] = kr[KBT + i];
              store_T(kr, T);
            }
          }
          __syncthreads();
        }
        qmax++;
        // levenberg.cpp:149: while (rho < 0 && qmax < maxTrials && !terminate()); rho and qmax
        // are work-group uniform
      } while (rho < 0 && qmax < 10 && !poll_stop(sh, stop_flag));
      lm_total++;
      if (qmax == 10 || rho == 0) break;
      if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
      else nbad = 0;
      if (nbad >= 3) break;
    }
    if (phase == 0) {
      if (poll_stop(sh, stop_flag)) stopped = true;  // optimizer.cpp:625-627: do_more
      if (stopped) break;
      // optimizer.cpp:632-665: chi2 > threshold or depth <= 0 -> level 1
      for (int e = tid; e < pb.n_obs; e += kThreads) {
        const int ge = pb.o0 + e;
        const PtRef r = ptrec(pb, ws.opoint[ge]);
        const double X[3] = {r[PX], r[PX + 1], r[PX + 2]};
        const slamgpu_ba_obs o = obs[ge];
        ObsEval v;
        eval_obs(o, P, isig, kfrec(pb, o.keyframe), X, v);
        if (ws.chi2[ge] > (o.ur >= 0 ? 7.815 : 5.991) || !(v.z > 0.0)) ws.act[ge] = 0;
      }
      __syncthreads();
    }
  }
  // optimizer.cpp:672-700: erase list over every edge; :702-716 write-back
  for (int e = tid; e < pb.n_obs; e += kThreads) {
    const int ge = pb.o0 + e;
    const PtRef r = ptrec(pb, ws.opoint[ge]);
    const double X[3] = {r[PX], r[PX + 1], r[PX + 2]};
    const slamgpu_ba_obs o = obs[ge];
    ObsEval v;
    eval_obs(o, P, isig, kfrec(pb, o.keyframe), X, v);
    erase[ge] = (ws.chi2[ge] > (o.ur >= 0 ? 7.815 : 5.991) || !(v.z > 0.0)) ? 1 : 0;
  }
  for (int p = tid; p < pb.n_pts; p += kThreads) {
    const PtRef r = ptrec(pb, p);
    for (int i = 0; i < 3; i++) points[(size_t)(pb.p0 + p) * 3 + i] = (float)r[PX + i];
  }
  for (int k = tid; k < pb.n_kf; k += kThreads) {
    if (kf_mode[pb.k0 + k] == SLAMGPU_KF_FIXED) continue;
    const double* kr = kfrec(pb, k);
    float* T = kf_Tcw + (size_t)(pb.k0 + k) * 16;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) T[4 * i + j] = (float)kr[KR + 3 * i + j];
      T[4 * i + 3] = (float)kr[KT + i];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
  }
  if (tid == 0) status[blockIdx.x] = lm_total;
#ifdef SLAMGPU_BA_PROFILE
  if (tid == 0)
    for (int i = 0; i < 8; i++) reinterpret_cast<double*>(status + gridDim.x + 1)[blockIdx.x * 8 + i] = prof[i];
#endif
  (void)n;
}

// computeActiveErrors + activeRobustChi2 + buildSystem of LocalBundleAdjustment's first optimize()
// (every edge at level 0, Huber kernels on) at the input estimates, per problem: the reprojection
// residual / Jacobian / normal-equation build the LM iterations repeat, on its own.
__global__ __launch_bounds__(kThreads) void local_ba_linearize_kernel(
    PoseParams P, const slamgpu_ba_problem* __restrict__ problems,
    const float* __restrict__ kf_Tcw, const uint8_t* __restrict__ kf_mode,
    const float* __restrict__ points, const int32_t* __restrict__ pstart,
    const slamgpu_ba_obs* __restrict__ obs, int32_t* __restrict__ status, BaWorkspace ws,
    BaLinearOut out) {
#pragma clang fp contract(fast)
  __shared__ BaShared sh;
  __shared__ float isig[SLAMGPU_MAX_LEVELS];
  const int tid = threadIdx.x;
  Problem pb;
  // the edge pass writes chi2 and the Hpl blocks straight into the outputs (same global edge
  // indexing as the workspace; nothing else in this kernel reads them back)
  BaWorkspace wso = ws;
  wso.chi2 = out.chi2;
  wso.hpl = out.hpl;
  if (!ba_setup(sh, pb, isig, P, problems, kf_Tcw, kf_mode, points, pstart, obs, status, wso))
    return;
  build_structure(sh, pb, true);
  double chi = 0.0, maxd = 0.0, zero = 0.0;
  linearise_edges(sh, pb, P, isig, true, chi);
  linearise_keyframes(sh, pb, P, isig, true, maxd);
  __syncthreads();
  sum_points(pb, maxd);
  block_sum2(sh, chi, zero);
  for (int e = tid; e < pb.n_obs; e += kThreads) {  // edges to fixed cameras have no Hpl block
    const int ge = pb.o0 + e;
    if (sh.free_of_kf[obs[ge].keyframe] < 0)
      for (int i = 0; i < 18; i++) out.hpl[(size_t)ge * 18 + i] = 0.0;
  }
  for (int p = tid; p < pb.n_pts; p += kThreads) {
    const PtRef r = ptrec(pb, p);
    for (int i = 0; i < 6; i++) out.hll[(size_t)(pb.p0 + p) * 6 + i] = r[PH + i];
    for (int i = 0; i < 3; i++) out.bl[(size_t)(pb.p0 + p) * 3 + i] = r[PB + i];
  }
  for (int k = tid; k < pb.n_kf; k += kThreads) {
    const double* kr = kfrec(pb, k);
    const bool fr = sh.free_of_kf[k] >= 0;
    for (int i = 0; i < 21; i++) out.hpp[(size_t)(pb.k0 + k) * 21 + i] = fr ? kr[KH + i] : 0.0;
    for (int i = 0; i < 6; i++) out.bp[(size_t)(pb.k0 + k) * 6 + i] = fr ? kr[KB + i] : 0.0;
  }
  if (tid == 0) {
    out.chi[blockIdx.x] = chi;
    status[blockIdx.x] = 0;
  }
}

}  // namespace

BaWorkspace ba_workspace_layout(void* base, int total_kf, int total_points, int total_obs,
                                size_t* bytes) {
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  size_t off = 0;
  BaWorkspace w{};
  char* b = static_cast<char*>(base);
  auto take = [&](size_t n) {
    char* p = b ? b + off : nullptr;
    off += al(n);
    return p;
  };
  w.chi2 = reinterpret_cast<double*>(take(sizeof(double) * (size_t)total_obs));
  w.hpl = reinterpret_cast<double*>(take(sizeof(double) * 18 * (size_t)total_obs));
  w.act = reinterpret_cast<uint8_t*>(take((size_t)total_obs));
  w.psorted = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (size_t)total_obs));
  w.hits = reinterpret_cast<int2*>(take(sizeof(int2) * kPairsPerObs * (size_t)total_obs));
  w.pt = reinterpret_cast<double*>(take(sizeof(double) * 27 * (size_t)total_points));
  w.n_pt = total_points;
  w.ehb = reinterpret_cast<double*>(take(sizeof(double) * 9 * (size_t)total_obs));
  w.opoint = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (size_t)total_obs));
  w.pmask = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * (size_t)total_points));
  w.kf = reinterpret_cast<double*>(take(sizeof(double) * 64 * (size_t)total_kf));
  if (bytes) *bytes = off + 256;
  return w;
}

hipError_t launch_local_ba_linearize(const PoseParams& P, const slamgpu_ba_problem* d_problems,
                                     int n_problems, const float* d_kf_Tcw,
                                     const uint8_t* d_kf_mode, const float* d_points,
                                     const int32_t* d_pstart, const slamgpu_ba_obs* d_obs,
                                     int32_t* d_status, const BaWorkspace& ws,
                                     const BaLinearOut& out, hipStream_t st) {
  if (n_problems <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("local_ba_linearize", st, local_ba_linearize_kernel, dim3(n_problems),
                 dim3(kThreads), 0, st, P, d_problems, d_kf_Tcw, d_kf_mode, d_points, d_pstart,
                 d_obs, d_status, ws, out);
  return hipGetLastError();
}

hipError_t launch_local_ba(const PoseParams& P, const slamgpu_ba_problem* d_problems,
                           int n_problems, float* d_kf_Tcw, const uint8_t* d_kf_mode,
                           float* d_points, const int32_t* d_pstart, const slamgpu_ba_obs* d_obs,
                           uint8_t* d_erase, int32_t* d_status, const BaWorkspace& ws,
                           const int32_t* d_stop, hipStream_t st) {
  if (n_problems <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("local_ba", st, local_ba_kernel, dim3(n_problems), dim3(kThreads), 0, st, P,
                 d_problems, d_kf_Tcw, d_kf_mode, d_points, d_pstart, d_obs, d_erase, d_status, ws,
                 d_stop);
  return hipGetLastError();
}

}  // namespace slamgpu
