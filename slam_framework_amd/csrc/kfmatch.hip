// kfmatch.hip -- the keyframe-rate matchers of the LocalMapper on gfx950 (include/slamgpu_kfmatch.h).
//
//   search_tri   OrbMatcher::SearchForTriangulation (src/orb_features/orb_matcher.cpp:634-802):
//                one workgroup per keyframe pair, a wave per pKF1 FeatureVector entry (the
//                reference never marks vbMatched2, so the pKF1 features are independent), the
//                node's pKF2 candidates across lanes. The kept candidate is the last passing one
//                of minimal distance in node order (`dist > bestDist` skips, :717): the wave
//                minimum of (distance << 16 | ~position).
//   fuse         the candidate search of OrbMatcher::Fuse(pKF, vpMapPoints, th) (:804-928): a wave
//                per map point; projection, image / distance / viewing-angle gates and
//                PredictScale (glibc logf) on uniform values, then every keypoint of the keyframe
//                across lanes, in GetFeaturesInArea order (grid cell x-major, then index): the
//                first strict minimum is the minimum of (distance, cell, index).
// Float semantics follow oracle/kfmatch_oracle.c (the Release build's contractions as explicit
// fmaf, OpenCV's double sums).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/slamgpu_kfmatch.h"
#include "device_math.h"

namespace slamgpu {
namespace {

constexpr int kThLow = 50, kHisto = 30, kGridCols = 64, kGridRows = 48;
constexpr int kMaxFeat = SLAMGPU_KF_MAX_FEATURES;

static_assert(sizeof(slamgpu_kf) == 128, "slamgpu_kf layout");
static_assert(sizeof(slamgpu_fuse_point) == 80, "slamgpu_fuse_point layout");
static_assert(sizeof(slamgpu_tri_pair) == 48, "slamgpu_tri_pair layout");

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
  const uint4* p = reinterpret_cast<const uint4*>(a);
  const uint4* q = reinterpret_cast<const uint4*>(b);
  const uint4 a0 = p[0], a1 = p[1], b0 = q[0], b1 = q[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// OpenCV's small float gemm row (Rcw * X + tcw): float dot, then (double) add.
__device__ __forceinline__ float gemm_row(const float* R, const float* x, float c) {
  const float dot = R[0] * x[0] + R[1] * x[1] + R[2] * x[2];
  return (float)((double)dot + (double)c);
}

__device__ __forceinline__ int node_find(const uint32_t* nodes, int nn, uint32_t key) {
  int lo = 0, hi = nn;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (nodes[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return (lo < nn && nodes[lo] == key) ? lo : -1;
}

// ---------------------------------------------------------------------------------------
constexpr int kTriWaves = 8;

__global__ __launch_bounds__(64 * kTriWaves) void search_tri_kernel(
    const slamgpu_kf* __restrict__ kfs, const slamgpu_tri_pair* __restrict__ pairs,
    slamgpu_camera cam, slamgpu_levels lv, int check_ori, int32_t* __restrict__ match,
    int64_t match_stride, int32_t* __restrict__ nmatches) {
  __shared__ int8_t s_bin[kMaxFeat];
  __shared__ int s_hist[kHisto];
  __shared__ int s_acc[kTriWaves], s_rem[kTriWaves], s_ind[3], s_bad;
  const int pair = blockIdx.x, tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const slamgpu_tri_pair P = pairs[pair];
  const slamgpu_kf& A = kfs[P.kf1];
  const slamgpu_kf& B = kfs[P.kf2];
  const int na = A.n, nb = B.n;
  if (na < 0 || nb < 0 || na > kMaxFeat || nb > kMaxFeat) {
    if (tid == 0) nmatches[pair] = -1;
    return;
  }
  int32_t* out = match + (int64_t)pair * match_stride;
  for (int i = tid; i < na; i += 64 * kTriWaves) {
    out[i] = -1;
    s_bin[i] = -1;
  }
  if (tid < kHisto) s_hist[tid] = 0;
  if (tid == 0) s_bad = 0;
  // epipole of pKF1's centre in pKF2 (:643-649)
  const float c2x = gemm_row(B.Rcw, A.Ow, B.tcw[0]);
  const float c2y = gemm_row(B.Rcw + 3, A.Ow, B.tcw[1]);
  const float c2z = gemm_row(B.Rcw + 6, A.Ow, B.tcw[2]);
  const float invz = 1.0f / c2z;
  const float ex = fmaf(cam.fx * c2x, invz, cam.cx), ey = fmaf(cam.fy * c2y, invz, cam.cy);
  const float* F = P.F12;
  __syncthreads();
  const int n_entries = A.n_nodes > 0 ? A.node_start[A.n_nodes] : 0;
  int acc = 0;
  for (int p = wid; p < n_entries; p += kTriWaves) {
    int lo = 0, hi = A.n_nodes;  // node of entry p: last ia with node_start[ia] <= p
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (A.node_start[mid] <= p) lo = mid;
      else hi = mid;
    }
    const int ib = node_find(B.nodes, B.n_nodes, A.nodes[lo]);
    if (ib < 0) continue;
    const int idx1 = (int)A.node_feats[p];
    if ((unsigned)idx1 >= (unsigned)na) {  // malformed FeatureVector: flag the pair, touch nothing
      s_bad = 1;
      continue;
    }
    if (A.has_mp[idx1]) continue;
    const bool st1 = A.u_right[idx1] >= 0;
    if (P.only_stereo && !st1) continue;
    const slamgpu_keypoint kp1 = A.kps[idx1];
    // epipolar line of kp1 in pKF2 (CheckDistEpipolarLine :117-119)
    const float la = fmaf(kp1.x, F[0], kp1.y * F[3]) + F[6];
    const float lb = fmaf(kp1.x, F[1], kp1.y * F[4]) + F[7];
    const float lc = fmaf(kp1.x, F[2], kp1.y * F[5]) + F[8];
    const float den = fmaf(la, la, lb * lb);
    const uint8_t* d1 = A.desc + (int64_t)idx1 * 32;
    const int b0 = B.node_start[ib], nbn = B.node_start[ib + 1] - b0;
    uint32_t best = 0xffffffffu;
    for (int c = lane; c < nbn; c += 64) {
      const int idx2 = (int)B.node_feats[b0 + c];
      if ((unsigned)idx2 >= (unsigned)nb) {
        s_bad = 1;
        continue;
      }
      if (B.has_mp[idx2]) continue;
      const bool st2 = B.u_right[idx2] >= 0;
      if (P.only_stereo && !st2) continue;
      const int dist = hamming32(d1, B.desc + (int64_t)idx2 * 32);
      if (dist > kThLow) continue;
      const slamgpu_keypoint kp2 = B.kps[idx2];
      if ((unsigned)kp2.octave >= (unsigned)lv.nlevels) {
        s_bad = 1;
        continue;
      }
      if (!st1 && !st2) {
        const float dx = ex - kp2.x, dy = ey - kp2.y;
        if (fmaf(dx, dx, dy * dy) < 100.0f * lv.scale[kp2.octave]) continue;
      }
      if (den == 0) continue;
      const float num = fmaf(la, kp2.x, lb * kp2.y) + lc;
      const float dsqr = num * num / den;
      if (!((double)dsqr < 3.84 * (double)lv.sigma2[kp2.octave])) continue;
      best = min(best, (uint32_t)dist << 16 | (uint32_t)(0xffff - c));
    }
    best = wave_min(best);
    if (best == 0xffffffffu) continue;
    if (lane == 0) {
      const int idx2 = (int)B.node_feats[b0 + (0xffff - (int)(best & 0xffffu))];
      out[idx1] = idx2;
      if (check_ori) {
        float rot = kp1.angle - B.kps[idx2].angle;
        if (rot < 0.0f) rot += 360.0f;
        int bin = (int)roundf(rot * (1.0f / kHisto));
        if (bin == kHisto) bin = 0;
        s_bin[idx1] = (int8_t)bin;
        atomicAdd(&s_hist[bin], 1);
      }
    }
    acc++;
  }
  if (lane == 0) s_acc[wid] = acc;
  __syncthreads();
  if (tid == 0) {  // ComputeThreeMaxima (orb_matcher.cpp:1584-1625)
    int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
    for (int i = 0; i < kHisto; i++) {
      const int s = s_hist[i];
      if (s > m1) {
        m3 = m2; m2 = m1; m1 = s;
        i3 = i2; i2 = i1; i1 = i;
      } else if (s > m2) {
        m3 = m2; m2 = s;
        i3 = i2; i2 = i;
      } else if (s > m3) {
        m3 = s;
        i3 = i;
      }
    }
    if (m2 < 0.1f * (float)m1) {
      i2 = -1;
      i3 = -1;
    } else if (m3 < 0.1f * (float)m1) {
      i3 = -1;
    }
    s_ind[0] = i1;
    s_ind[1] = i2;
    s_ind[2] = i3;
  }
  __syncthreads();
  int removed = 0;
  if (check_ori) {
    const int i1 = s_ind[0], i2 = s_ind[1], i3 = s_ind[2];
    for (int i = tid; i < na; i += 64 * kTriWaves) {
      const int bin = s_bin[i];
      if (bin >= 0 && bin != i1 && bin != i2 && bin != i3) {
        out[i] = -1;
        removed++;
      }
    }
  }
  removed = wave_sum(removed);
  if (lane == 0) s_rem[wid] = removed;
  __syncthreads();
  if (tid == 0) {
    int nm = 0;
    for (int w = 0; w < kTriWaves; w++) nm += s_acc[w] - s_rem[w];
    nmatches[pair] = s_bad ? -1 : nm;
  }
}

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fuse_kernel(const slamgpu_kf* __restrict__ kfs,
                                                   const slamgpu_fuse_point* __restrict__ pts,
                                                   const int32_t* __restrict__ point_kf,
                                                   int n_pts, float th, slamgpu_camera cam,
                                                   slamgpu_levels lv, slamgpu_kf_grid g,
                                                   int32_t* __restrict__ best_idx,
                                                   int32_t* __restrict__ best_dist) {
  const int i = blockIdx.x * 4 + wave_id();
  if (i >= n_pts) return;
  const int lane = lane_id();
  const slamgpu_fuse_point& P = pts[i];
  int out_idx = -1, out_dist = 256;
  const int kfi = point_kf ? point_kf[i] : 0;
  const slamgpu_kf& K = kfs[kfi];
  const int n = min(K.n, kMaxFeat);
  do {
    if (P.skip) break;
    const float xc = gemm_row(K.Rcw, P.xyz, K.tcw[0]);
    const float yc = gemm_row(K.Rcw + 3, P.xyz, K.tcw[1]);
    const float zc = gemm_row(K.Rcw + 6, P.xyz, K.tcw[2]);
    if (zc < 0.0f) break;
    const float invz = 1.0f / zc;
    const float x = xc * invz, y = yc * invz;
    const float u = fmaf(cam.fx, x, cam.cx), v = fmaf(cam.fy, y, cam.cy);
    if (!(u >= g.min_x && u < g.max_x && v >= g.min_y && v < g.max_y)) break;
    const float urp = fmaf(-cam.bf, invz, u);
    const float maxD = 1.2f * P.max_dist, minD = 0.8f * P.min_dist;
    const float po0 = P.xyz[0] - K.Ow[0], po1 = P.xyz[1] - K.Ow[1], po2 = P.xyz[2] - K.Ow[2];
    double s = 0.0;
    s += (double)po0 * (double)po0;
    s += (double)po1 * (double)po1;
    s += (double)po2 * (double)po2;
    const float dist3D = (float)sqrt(s);
    if (dist3D < minD || dist3D > maxD) break;
    double dot = 0.0;
    dot += (double)po0 * (double)P.normal[0];
    dot += (double)po1 * (double)P.normal[1];
    dot += (double)po2 * (double)P.normal[2];
    if (dot < 0.5 * (double)dist3D) break;
    int lvl = (int)ceilf(glibc_logf(P.max_dist / dist3D) / lv.log_scale_factor);
    lvl = lvl < 0 ? 0 : (lvl >= lv.nlevels ? lv.nlevels - 1 : lvl);
    const float r = th * lv.scale[lvl];
    // KeyFrame::GetFeaturesInArea (keyframe.cpp:442-476) cell window
    const int cx0 = max(0, (int)floorf((u - g.min_x - r) / g.cell_w));
    const int cx1 = min(kGridCols - 1, (int)ceilf((u - g.min_x + r) / g.cell_w));
    const int cy0 = max(0, (int)floorf((v - g.min_y - r) / g.cell_h));
    const int cy1 = min(kGridRows - 1, (int)ceilf((v - g.min_y + r) / g.cell_h));
    if (cx1 < 0 || cx0 >= kGridCols || cy1 < 0 || cy0 >= kGridRows) break;
    uint64_t best = ~0ull;
    for (int j = lane; j < n; j += 64) {
      const slamgpu_keypoint kp = K.kps[j];
      // Frame::PosInGrid (frame.cpp:339-346): the cell AssignFeaturesToGrid put j in
      const int px = (int)roundf((kp.x - g.min_x) / g.cell_w);
      const int py = (int)roundf((kp.y - g.min_y) / g.cell_h);
      if (px < cx0 || px > cx1 || py < cy0 || py > cy1) continue;  // also drops off-grid kps
      const float dxk = kp.x - u, dyk = kp.y - v;
      if (!(fabsf(dxk) < r && fabsf(dyk) < r)) continue;
      const int kl = kp.octave;
      if (kl < lvl - 1 || kl > lvl) continue;
      const float ex = u - kp.x, ey = v - kp.y;
      const float kr = K.u_right[j];
      if (kr >= 0) {
        const float er = urp - kr;
        const float e2 = fmaf(er, er, fmaf(ex, ex, ey * ey));
        if ((double)(e2 * lv.inv_sigma2[kl]) > 7.8) continue;
      } else {
        const float e2 = fmaf(ex, ex, ey * ey);
        if ((double)(e2 * lv.inv_sigma2[kl]) > 5.99) continue;
      }
      const uint32_t dist = (uint32_t)hamming32(P.desc, K.desc + (int64_t)j * 32);
      const uint64_t key = (uint64_t)dist << 32 | (uint64_t)(px * kGridRows + py) << 12 | (uint32_t)j;
      best = best < key ? best : key;
    }
    best = wave_min(best);
    if (best == ~0ull) break;
    out_dist = (int)(best >> 32);
    if (out_dist <= kThLow) out_idx = (int)(best & 0xfffu);
  } while (false);
  if (lane == 0) {
    best_idx[i] = out_idx;
    best_dist[i] = out_dist;
  }
}

thread_local std::string t_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

#define KF_HIPCHECK(x)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(SLAMGPU_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

// Per-thread staging buffer + stream of the synchronous calls.
struct Stage {
  int device = -1;
  hipStream_t stream = nullptr;
  char* buf = nullptr;
  size_t bytes = 0;
  ~Stage() {
    if (buf) (void)hipFree(buf);
    if (stream) (void)hipStreamDestroy(stream);
  }
};
thread_local Stage t_stage;

int stage_reserve(size_t need) {
  Stage& S = t_stage;
  int dev = 0;
  KF_HIPCHECK(hipGetDevice(&dev));
  if (S.device != dev) {
    if (S.buf) (void)hipFree(S.buf);
    if (S.stream) (void)hipStreamDestroy(S.stream);
    S.buf = nullptr;
    S.stream = nullptr;
    S.bytes = 0;
    KF_HIPCHECK(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
    S.device = dev;
  }
  if (need > S.bytes) {
    if (S.buf) KF_HIPCHECK(hipFree(S.buf));
    S.buf = nullptr;
    S.bytes = 0;
    const size_t cap = need < (1u << 20) ? (1u << 20) : need;
    KF_HIPCHECK(hipMalloc(&S.buf, cap));
    S.bytes = cap;
  }
  return 0;
}

int check_levels(const slamgpu_levels* lv) {
  if (!lv || lv->nlevels < 1 || lv->nlevels > 32)
    return fail(SLAMGPU_EINVAL, "levels: nlevels outside [1, 32]");
  return 0;
}

int check_kf(const slamgpu_kf* k, bool fv, const char* name) {
  if (!k) return fail(SLAMGPU_EINVAL, "%s is NULL", name);
  if (k->n < 0 || k->n > kMaxFeat)
    return fail(SLAMGPU_EINVAL, "%s: n %d outside [0, %d]", name, k->n, kMaxFeat);
  if (k->n > 0 && (!k->kps || !k->desc || !k->u_right || (fv && !k->has_mp)))
    return fail(SLAMGPU_EINVAL, "%s: NULL keypoint arrays", name);
  if (fv) {
    if (k->n_nodes < 0 || k->n_nodes > k->n)
      return fail(SLAMGPU_EINVAL, "%s: n_nodes %d outside [0, n]", name, k->n_nodes);
    if (k->n_nodes > 0) {
      if (!k->nodes || !k->node_start || !k->node_feats)
        return fail(SLAMGPU_EINVAL, "%s: NULL FeatureVector", name);
      if (k->node_start[0] != 0) return fail(SLAMGPU_EINVAL, "%s: node_start[0] != 0", name);
      for (int i = 0; i < k->n_nodes; i++) {
        if (k->node_start[i + 1] < k->node_start[i] || k->node_start[i + 1] > k->n)
          return fail(SLAMGPU_EINVAL, "%s: node_start not ascending within [0, n]", name);
        if (i > 0 && k->nodes[i] <= k->nodes[i - 1])
          return fail(SLAMGPU_EINVAL, "%s: nodes not strictly ascending", name);
      }
      for (int j = 0; j < k->node_start[k->n_nodes]; j++)
        if (k->node_feats[j] >= (uint32_t)k->n)
          return fail(SLAMGPU_EINVAL, "%s: feature index >= n", name);
    }
  }
  for (int j = 0; j < k->n; j++)
    if (k->kps[j].octave < 0 || k->kps[j].octave >= 32)
      return fail(SLAMGPU_EINVAL, "%s: keypoint %d octave %d outside [0, 32)", name, j,
                  k->kps[j].octave);
  return 0;
}

// Copies a host keyframe's arrays into the staging buffer at *off; returns its device twin.
slamgpu_kf stage_kf(const slamgpu_kf& k, bool fv, size_t* off) {
  char* base = t_stage.buf;
  slamgpu_kf d = k;
  auto put = [&](const void* src, size_t bytes) -> void* {
    void* dst = base + *off;
    *off += al256(bytes ? bytes : 1);
    if (bytes) (void)hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, t_stage.stream);
    return dst;
  };
  d.kps = (const slamgpu_keypoint*)put(k.kps, (size_t)k.n * sizeof(slamgpu_keypoint));
  d.desc = (const uint8_t*)put(k.desc, (size_t)k.n * 32);
  d.u_right = (const float*)put(k.u_right, (size_t)k.n * 4);
  d.has_mp = fv ? (const uint8_t*)put(k.has_mp, (size_t)k.n) : nullptr;
  if (fv && k.n_nodes > 0) {
    d.nodes = (const uint32_t*)put(k.nodes, (size_t)k.n_nodes * 4);
    d.node_start = (const int32_t*)put(k.node_start, (size_t)(k.n_nodes + 1) * 4);
    d.node_feats = (const uint32_t*)put(k.node_feats, (size_t)k.node_start[k.n_nodes] * 4);
  } else {
    d.nodes = nullptr;
    d.node_start = nullptr;
    d.node_feats = nullptr;
    d.n_nodes = 0;
  }
  return d;
}

size_t kf_bytes(const slamgpu_kf& k, bool fv) {
  size_t b = al256((size_t)k.n * sizeof(slamgpu_keypoint) + 1) + al256((size_t)k.n * 32 + 1) +
             al256((size_t)k.n * 4 + 1) + al256((size_t)k.n + 1);
  if (fv && k.n_nodes > 0)
    b += al256((size_t)k.n_nodes * 4) + al256((size_t)(k.n_nodes + 1) * 4) +
         al256((size_t)k.node_start[k.n_nodes] * 4 + 1);
  return b;
}

}  // namespace
}  // namespace slamgpu

using namespace slamgpu;

extern "C" {

const char* slamgpu_kfmatch_last_error(void) { return t_err.c_str(); }

int slamgpu_search_for_triangulation_device(const slamgpu_kf* d_kfs,
                                            const slamgpu_tri_pair* d_pairs, int n_pairs,
                                            const slamgpu_camera* cam, const slamgpu_levels* lv,
                                            int check_ori, int32_t* d_match12,
                                            int64_t match_stride, int32_t* d_nmatches,
                                            void* stream) {
  if (n_pairs < 0) return fail(SLAMGPU_EINVAL, "n_pairs %d < 0", n_pairs);
  if (n_pairs == 0) return 0;
  if (!d_kfs || !d_pairs || !d_match12 || !d_nmatches || !cam)
    return fail(SLAMGPU_EINVAL, "NULL argument");
  if (int r = check_levels(lv)) return r;
  hipLaunchKernelGGL(search_tri_kernel, dim3(n_pairs), dim3(64 * kTriWaves), 0,
                     static_cast<hipStream_t>(stream), d_kfs, d_pairs, *cam, *lv,
                     check_ori ? 1 : 0, d_match12, match_stride, d_nmatches);
  KF_HIPCHECK(hipGetLastError());
  return 0;
}

int slamgpu_search_for_triangulation(const slamgpu_kf* kf1, const slamgpu_kf* kf2,
                                     const float* F12, const slamgpu_camera* cam,
                                     const slamgpu_levels* lv, int only_stereo, int check_ori,
                                     int32_t* match12, int* nmatches) {
  if (int r = check_kf(kf1, true, "kf1")) return r;
  if (int r = check_kf(kf2, true, "kf2")) return r;
  if (int r = check_levels(lv)) return r;
  if (!F12 || !cam || !nmatches || (kf1->n > 0 && !match12))
    return fail(SLAMGPU_EINVAL, "NULL argument");
  size_t need = kf_bytes(*kf1, true) + kf_bytes(*kf2, true) + al256(2 * sizeof(slamgpu_kf)) +
                al256(sizeof(slamgpu_tri_pair)) + al256((size_t)kf1->n * 4 + 4) + al256(4);
  if (int r = stage_reserve(need)) return r;
  size_t off = 0;
  slamgpu_kf dk[2] = {stage_kf(*kf1, true, &off), stage_kf(*kf2, true, &off)};
  char* base = t_stage.buf;
  hipStream_t st = t_stage.stream;
  slamgpu_kf* d_kfs = reinterpret_cast<slamgpu_kf*>(base + off);
  off += al256(sizeof(dk));
  slamgpu_tri_pair pr{};
  pr.kf1 = 0;
  pr.kf2 = 1;
  for (int i = 0; i < 9; i++) pr.F12[i] = F12[i];
  pr.only_stereo = only_stereo ? 1 : 0;
  slamgpu_tri_pair* d_pair = reinterpret_cast<slamgpu_tri_pair*>(base + off);
  off += al256(sizeof(pr));
  int32_t* d_match = reinterpret_cast<int32_t*>(base + off);
  off += al256((size_t)kf1->n * 4 + 4);
  int32_t* d_nm = reinterpret_cast<int32_t*>(base + off);
  KF_HIPCHECK(hipMemcpyAsync(d_kfs, dk, sizeof(dk), hipMemcpyHostToDevice, st));
  KF_HIPCHECK(hipMemcpyAsync(d_pair, &pr, sizeof(pr), hipMemcpyHostToDevice, st));
  if (int r = slamgpu_search_for_triangulation_device(d_kfs, d_pair, 1, cam, lv, check_ori,
                                                      d_match, 0, d_nm, st))
    return r;
  int32_t nm = 0;
  KF_HIPCHECK(hipMemcpyAsync(&nm, d_nm, 4, hipMemcpyDeviceToHost, st));
  if (kf1->n > 0)
    KF_HIPCHECK(hipMemcpyAsync(match12, d_match, (size_t)kf1->n * 4, hipMemcpyDeviceToHost, st));
  KF_HIPCHECK(hipStreamSynchronize(st));
  *nmatches = nm;
  return 0;
}

int slamgpu_fuse_device(const slamgpu_kf* d_kfs, const slamgpu_fuse_point* d_pts,
                        const int32_t* d_point_kf, int n_pts, float th,
                        const slamgpu_camera* cam, const slamgpu_levels* lv,
                        const slamgpu_kf_grid* grid, int32_t* d_best_idx, int32_t* d_best_dist,
                        void* stream) {
  if (n_pts < 0) return fail(SLAMGPU_EINVAL, "n_pts %d < 0", n_pts);
  if (n_pts == 0) return 0;
  if (!d_kfs || !d_pts || !d_best_idx || !d_best_dist || !cam || !grid)
    return fail(SLAMGPU_EINVAL, "NULL argument");
  if (int r = check_levels(lv)) return r;
  if (!(grid->cell_w > 0) || !(grid->cell_h > 0)) return fail(SLAMGPU_EINVAL, "grid cell size");
  hipLaunchKernelGGL(fuse_kernel, dim3((n_pts + 3) / 4), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_kfs, d_pts, d_point_kf, n_pts, th, *cam,
                     *lv, *grid, d_best_idx, d_best_dist);
  KF_HIPCHECK(hipGetLastError());
  return 0;
}

int slamgpu_fuse(const slamgpu_kf* kf, const slamgpu_fuse_point* pts, int n_pts, float th,
                 const slamgpu_camera* cam, const slamgpu_levels* lv, const slamgpu_kf_grid* grid,
                 int32_t* best_idx, int32_t* best_dist, int* nfused) {
  if (int r = check_kf(kf, false, "kf")) return r;
  if (int r = check_levels(lv)) return r;
  if (n_pts < 0 || !cam || !grid || !nfused || (n_pts > 0 && (!pts || !best_idx || !best_dist)))
    return fail(SLAMGPU_EINVAL, "bad arguments");
  for (int j = 0; j < kf->n; j++)
    if (kf->kps[j].octave >= lv->nlevels)
      return fail(SLAMGPU_EINVAL, "keypoint %d octave %d >= nlevels", j, kf->kps[j].octave);
  *nfused = 0;
  if (n_pts == 0) return 0;
  const size_t need = kf_bytes(*kf, false) + al256(sizeof(slamgpu_kf)) +
                      al256((size_t)n_pts * sizeof(slamgpu_fuse_point)) + 2 * al256((size_t)n_pts * 4);
  if (int r = stage_reserve(need)) return r;
  size_t off = 0;
  const slamgpu_kf dk = stage_kf(*kf, false, &off);
  char* base = t_stage.buf;
  hipStream_t st = t_stage.stream;
  slamgpu_kf* d_kf = reinterpret_cast<slamgpu_kf*>(base + off);
  off += al256(sizeof(dk));
  slamgpu_fuse_point* d_pts = reinterpret_cast<slamgpu_fuse_point*>(base + off);
  off += al256((size_t)n_pts * sizeof(slamgpu_fuse_point));
  int32_t* d_idx = reinterpret_cast<int32_t*>(base + off);
  off += al256((size_t)n_pts * 4);
  int32_t* d_dist = reinterpret_cast<int32_t*>(base + off);
  KF_HIPCHECK(hipMemcpyAsync(d_kf, &dk, sizeof(dk), hipMemcpyHostToDevice, st));
  KF_HIPCHECK(hipMemcpyAsync(d_pts, pts, (size_t)n_pts * sizeof(slamgpu_fuse_point),
                             hipMemcpyHostToDevice, st));
  if (int r = slamgpu_fuse_device(d_kf, d_pts, nullptr, n_pts, th, cam, lv, grid, d_idx, d_dist,
                                  st))
    return r;
  KF_HIPCHECK(hipMemcpyAsync(best_idx, d_idx, (size_t)n_pts * 4, hipMemcpyDeviceToHost, st));
  KF_HIPCHECK(hipMemcpyAsync(best_dist, d_dist, (size_t)n_pts * 4, hipMemcpyDeviceToHost, st));
  KF_HIPCHECK(hipStreamSynchronize(st));
  int nf = 0;
  for (int i = 0; i < n_pts; i++) nf += best_idx[i] >= 0;
  *nfused = nf;
  return 0;
}

}  // extern "C"
