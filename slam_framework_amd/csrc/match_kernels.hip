// match_kernels.hip -- stereo and projection matching on gfx950, batched over frames.
//
//   stereo_rows     right-keypoint row table          Frame::ComputeStereoMatches :412-433
//   stereo_match    row-band Hamming + 11x11 SAD      :446-562   (one wave per left keypoint)
//   stereo_median   2.1 x median SAD rejection        :564-576   (one workgroup per frame)
//   grid_build      64x48 keypoint grid (CSR)         Frame::AssignFeaturesToGrid :234-248
//   search_cand     projection + window + Hamming     OrbMatcher::SearchByProjection (both
//   search_resolve  greedy in-order claims            overloads, orb_matcher.cpp:13-103 and
//                                                     :1312-1453) + rotation histogram
// Every Hamming distance is popcount(a ^ b) over 4 x u64 (== DescriptorDistance, :1630-1646).
// The projection matchers are greedy in query order (a keypoint taken by an earlier query whose
// map point has observations is skipped, :59-63 / :1389-1393), so candidate search is parallel
// over queries and only a short claim-resolution pass per frame is sequential.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_math.h"
#include "timing.h"
#include "match_kernels.h"
#include "undistort.h"

namespace slamgpu {

#ifndef STEREO_LANES  // lanes per left keypoint in stereo_match (32: two per wave, 16: four)
#define STEREO_LANES 16
#endif

constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;
constexpr uint64_t kNoKey = ~0ull;

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
  const uint64_t* pa = reinterpret_cast<const uint64_t*>(a);
  const uint64_t* pb = reinterpret_cast<const uint64_t*>(b);
  return __popcll(pa[0] ^ pb[0]) + __popcll(pa[1] ^ pb[1]) + __popcll(pa[2] ^ pb[2]) +
         __popcll(pa[3] ^ pb[3]);
}

__device__ __forceinline__ const uint8_t* level_img(const ImageBatch& b, const OrbGeom* g,
                                                    int img, int level, int* pitch) {
  if (level == 0) {
    *pitch = b.in_pitch;
    return batch_image(b, img);
  }
  *pitch = g->lv[level].pitch;
  return b.pyr + (int64_t)img * g->pyr_bytes + g->lv[level].offset;
}

// NT-thread exclusive scan of arr[0..n) in place; returns the total. wsum: NT / 64 ints.
template <int CAP, int NT = 256>
__device__ int scan256(int* arr, int n, int* wsum) {
  constexpr int per = (CAP + NT - 1) / NT;
  const int lane = threadIdx.x & 63, wid = wave_id();
  const int base = threadIdx.x * per;
  int loc[per];
  int s = 0;
#pragma unroll
  for (int i = 0; i < per; i++) {
    loc[i] = (base + i < n) ? arr[base + i] : 0;
    s += loc[i];
  }
  int x = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    pre += (w < wid) ? wsum[w] : 0;
    tot += wsum[w];
  }
  pre += x - s;
#pragma unroll
  for (int i = 0; i < per; i++) {
    if (base + i < n) arr[base + i] = pre;
    pre += loc[i];
  }
  __syncthreads();
  return tot;
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v |= __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------------------------------
// Stereo (frame.cpp:406-577). Frame f: left = image 2f, right = image 2f+1.
constexpr int kMaxRows = 2048;

// NT threads per frame: 256 for batches, 1024 for the single-frame call (its one work-group is
// the whole launch: a quarter of the serial LDS-atomic loops per thread).
template <int NT>
__device__ __forceinline__ void stereo_rows_body(int f, const OrbGeom* __restrict__ g,
                                                 const FrameKps& ext, int nrows,
                                                 const StereoWorkspace& ws,
                                                 uint32_t* __restrict__ err) {
  __shared__ int cnt[kMaxRows + 1];
  __shared__ int wsum[NT / 64];
  const int tid = threadIdx.x;
  const int ir = 2 * f + 1;
  const KeyPoint* kr = ext.kps + ir * ext.stride;
  const int nr = ext.n[ir * ext.n_stride];
  int* rs = ws.row_start + (int64_t)f * (nrows + 1);
  uint2* items = ws.row_items + (int64_t)f * ws.row_cap;
  for (int i = tid; i <= nrows; i += NT) cnt[i] = 0;
  __syncthreads();
  // a thread's keypoints are loaded kChunk at a time before their row updates: one load latency
  // per chunk instead of one per keypoint (a single frame runs this as one work-group)
  constexpr int kChunk = 2048 / NT;
  // the row items carry the candidate's octave and x, the matcher's first filter (one load per
  // candidate instead of the item and then its keypoint)
  uint2 kit[kChunk];
  auto row_span = [&](int base, int (&lo)[kChunk], int (&hi)[kChunk]) {
    float ky[kChunk];
    int ko[kChunk];
#pragma unroll
    for (int u = 0; u < kChunk; u++) {
      const int i = base + NT * u + tid;
      ky[u] = 0.0f;
      ko[u] = -1;
      if (i < nr) {
        ky[u] = kr[i].y;
        ko[u] = kr[i].octave;
        kit[u] = make_uint2((uint32_t)i | (uint32_t)ko[u] << 16, __float_as_uint(kr[i].x));
      }
    }
#pragma unroll
    for (int u = 0; u < kChunk; u++) {
      lo[u] = 0;
      hi[u] = -1;
      if (ko[u] >= 0) {
        const float r = 2.0f * g->lv[ko[u]].scale;
        lo[u] = max((int)floorf(ky[u] - r), 0);
        hi[u] = min((int)ceilf(ky[u] + r), nrows - 1);
      }
    }
  };
  for (int base = 0; base < nr; base += NT * kChunk) {
    int lo[kChunk], hi[kChunk];
    row_span(base, lo, hi);
#pragma unroll
    for (int u = 0; u < kChunk; u++)
      for (int yi = lo[u]; yi <= hi[u]; ++yi) atomicAdd(&cnt[yi], 1);
  }
  __syncthreads();
  const int total = scan256<kMaxRows + 1, NT>(cnt, nrows, wsum);
  for (int i = tid; i < nrows; i += NT) rs[i] = cnt[i];
  if (tid == 0) {
    rs[nrows] = total;
    if (total > ws.row_cap) atomicOr(err, kErrRowOverflow);
  }
  __syncthreads();
  for (int base = 0; base < nr; base += NT * kChunk) {
    int lo[kChunk], hi[kChunk];
    row_span(base, lo, hi);
#pragma unroll
    for (int u = 0; u < kChunk; u++)
      for (int yi = lo[u]; yi <= hi[u]; ++yi) {
        const int pos = atomicAdd(&cnt[yi], 1);
        if (pos < ws.row_cap) items[pos] = kit[u];
      }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void stereo_rows_kernel(const OrbGeom* __restrict__ g,
                                                         FrameKps ext, int nrows,
                                                         StereoWorkspace ws,
                                                         uint32_t* __restrict__ err) {
  stereo_rows_body<NT>(blockIdx.x, g, ext, nrows, ws, err);
}

// One left keypoint per G lanes (G = 32: two per wave; G = 16: four): the kernel is a chain of
// dependent loads per keypoint (row table -> candidates -> descriptors -> SAD windows), so several
// independent chains per wave hide the latency at the same occupancy.
template <int G>
__device__ __forceinline__ uint32_t group_min(uint32_t v) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) {
    const uint32_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

template <int G>
__global__ __launch_bounds__(256) void stereo_match_kernel(ImageBatch b,
                                                           const OrbGeom* __restrict__ g,
                                                           FrameKps ext, Camera cam, int nrows,
                                                           StereoWorkspace ws, StereoOut out) {
  constexpr int NPW = 64 / G;  // keypoints per wave
  constexpr int kRounds = (121 + G - 1) / G;
  int f, bx;
  xcd_image_block(&f, &bx);  // a frame's work-groups share one XCD's L2 (its right keypoints)
  const int lane = threadIdx.x & 63, grp = lane / G, hl = lane % G;
  const int iL = (bx * 4 + wave_id()) * NPW + grp;
  const int il = 2 * f, ir = 2 * f + 1;
  const int nl = ext.n[il * ext.n_stride];
  const int64_t o = (int64_t)f * g->kp_cap + iL;
  bool ok = iL < nl;
  if (ok && hl == 0) {
    out.u_right[o] = -1.0f;
    out.depth[o] = -1.0f;
    ws.sad[o] = -1;
  }
  KeyPoint kpL{};
  if (ok) kpL = ext.kps[il * ext.stride + iL];
  const int levelL = kpL.octave;
  const float vL = kpL.y, uL = kpL.x;
  const int row = (int)vL;
  ok = ok && row >= 0 && row < nrows;
  const int* rs = ws.row_start + (int64_t)f * (nrows + 1);
  const uint2* items = ws.row_items + (int64_t)f * ws.row_cap;
  int c0 = 0, c1 = 0;
  if (ok) {
    c0 = rs[row];
    c1 = min(rs[row + 1], ws.row_cap);
  }
  ok = ok && c0 < c1;
  const float baseline = cam.bf / cam.fx;  // see DESIGN.md: maxD is UB in the reference (:436)
  const float minZ = baseline, minD = 0, maxD = cam.bf / minZ;
  const float minU = uL - maxD, maxU = uL - minD;
  ok = ok && !(maxU < 0);
  const uint8_t* dL = ext.desc + (il * ext.stride + (ok ? iL : 0)) * 32;
  const uint8_t* dRb = ext.desc + ir * ext.stride * 32;
  uint32_t best = ((uint32_t)TH_HIGH << 16) | 0xffffu;
  float bestU = 0.0f;  // x of this lane's best candidate
  if (ok) {
    // kCandU candidates per lane at a time, each stage's loads all in flight before the next
    // stage needs them: row items -> (octave, x) -> descriptors -> distances (the loop was a
    // chain of three dependent loads per candidate)
    // 2 and 4 measured equal (0.35 ms/step), 2 holds fewer VGPRs; with the packed row items
    // (two loads per candidate) 2 is still best, as are 16 lanes per keypoint (8 / 32 lanes and
    // 4 candidates: 0.29-0.36 ms against 0.28, profiles/r6d_stereo_lanes_ab.log)
    constexpr int kCandU = 2;
    const uint4* dLq = reinterpret_cast<const uint4*>(dL);
    const uint4 l0 = dLq[0], l1 = dLq[1];
    for (int cb = c0 + hl; cb < c1; cb += G * kCandU) {
      int iR[kCandU];
      float uR[kCandU];
      bool pass[kCandU];
#pragma unroll
      for (int u = 0; u < kCandU; u++) {
        const int c = cb + G * u;
        const uint2 it = c < c1 ? items[c] : make_uint2(0xffffffffu, 0u);
        iR[u] = (int)(it.x & 0xffffu);
        const int oct = (int)(it.x >> 16);
        uR[u] = __uint_as_float(it.y);
        pass[u] = c < c1 && oct >= levelL - 1 && oct <= levelL + 1 && uR[u] >= minU &&
                  uR[u] <= maxU;
      }
      uint4 r0[kCandU], r1[kCandU];
#pragma unroll
      for (int u = 0; u < kCandU; u++)
        if (pass[u]) {
          const uint4* dr = reinterpret_cast<const uint4*>(dRb + iR[u] * 32);
          r0[u] = dr[0];
          r1[u] = dr[1];
        }
#pragma unroll
      for (int u = 0; u < kCandU; u++)
        if (pass[u]) {
          const int dist = __popc(l0.x ^ r0[u].x) + __popc(l0.y ^ r0[u].y) + __popc(l0.z ^ r0[u].z) +
                           __popc(l0.w ^ r0[u].w) + __popc(l1.x ^ r1[u].x) + __popc(l1.y ^ r1[u].y) +
                           __popc(l1.z ^ r1[u].z) + __popc(l1.w ^ r1[u].w);
          const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)iR[u];
          if (dist < TH_HIGH && key < best) {
            best = key;
            bestU = uR[u];
          }
        }
    }
  }
  const uint32_t mine = best;
  best = group_min<G>(best);
  // the x of the group's best candidate from the lane that found it (keys are unique)
  const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (G * grp);
  const uint64_t hit = __ballot(mine == best) & gmask;
  const float uRbest = __shfl(bestU, hit ? __builtin_ctzll(hit) : lane, 64);
  const int bestDist = (int)(best >> 16);
  const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
  ok = ok && bestDist < thOrbDist;
  // sliding-window SAD at the left keypoint's level (:481-531)
  const float uR0 = ok ? uRbest : 0.f;
  const float scaleFactor = g->lv[levelL].inv_scale;
  const float scaleduL = roundf(kpL.x * scaleFactor);
  const float scaledvL = roundf(kpL.y * scaleFactor);
  const float scaleduR0 = roundf(uR0 * scaleFactor);
  const int w = 5, L = 5;
  const LevelGeom& LG = g->lv[levelL];
  const float iniu = scaleduR0 + L - w;
  const float endu = scaleduR0 + L + w + 1;
  ok = ok && !(iniu < 0 || endu >= (float)LG.w);
  const int yc = (int)scaledvL, xcl = (int)scaleduL, xcr = (int)scaleduR0;
  // windows the reference would reject with a cv::Mat ROI assertion are treated as no match
  ok = ok && !(yc - w < 0 || yc + w >= LG.h || xcl - w < 0 || xcl + w >= LG.w || xcr - L - w < 0);
  // SAD of the 11 window offsets: the 121 (offset, row) pairs over the group (kRounds rounds),
  // each lane summing one 11-pixel row; rows are then summed per offset through LDS. The window
  // bytes (left: columns xcl-5..xcl+5, right: xcr-10..xcr+10, rows yc-5..yc+5) are first staged
  // into LDS with dword loads (11 dwords per row: 4 left + 7 right); dwords past a row's last byte
  // are clamped to it (their bytes are never used). Caller images with an odd base or pitch take
  // byte loads instead.
  __shared__ int s_part[4][NPW][128];
  __shared__ uint32_t s_win[4][NPW][11][11];
  int* part = s_part[wave_id()][grp];
  uint32_t(*win)[11] = s_win[wave_id()][grp];
  int pl = 0, pr = 0;
  const uint8_t* IL = nullptr;
  const uint8_t* IR = nullptr;
  if (ok) {
    IL = level_img(b, g, il, levelL, &pl);
    IR = level_img(b, g, ir, levelL, &pr);
  }
  const int al = (xcl - w) & ~3, ar = (xcr - L - w) & ~3;
  const bool dw = ((((uintptr_t)IL | (uintptr_t)IR) | (uintptr_t)(pl | pr)) & 3) == 0;
  const int lastw = (LG.w - 1) >> 2;
  if (ok) {
#pragma unroll
    for (int rnd = 0; rnd < kRounds; rnd++) {
      const int p = hl + G * rnd;
      if (p < 121) {
        const int r = p / 11, d = p - 11 * r;  // window row, dword slot (0-3 left, 4-10 right)
        const bool left = d < 4;
        const uint8_t* img = left ? IL : IR;
        const int pitch = left ? pl : pr;
        const int x0 = left ? al + 4 * d : ar + 4 * (d - 4);
        const uint8_t* rowp = img + (int64_t)(yc - w + r) * pitch;
        uint32_t v;
        if (dw) {
          v = reinterpret_cast<const uint32_t*>(rowp)[min(x0 >> 2, lastw)];
        } else {
          v = 0;
          for (int j = 0; j < 4; j++)
            v |= (uint32_t)rowp[min(x0 + j, LG.w - 1)] << (8 * j);
        }
        win[r][d] = v;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint8_t* wb = reinterpret_cast<const uint8_t*>(&win[0][0]);  // row r at 44 r
  if (ok) {
    // A task (offset k, window row yr) sums |(IL - cl) - (IR - cr)| over 11 pixels as v_sad_u16
    // on u16 pairs: (IL + 512) - (IR + 512 + cl - cr); v_perm builds each pair with the +512 bias
    // bytes taken from a constant operand, and a 12th pair element is made equal on both sides.
    const uint32_t* ww = &win[0][0];
    const int oL = xcl - w - al, oR0 = xcr - L - w - ar;  // byte offsets of the rows (0..3)
    const int cl = wb[44 * w + (xcl - al)];
    constexpr uint32_t kBias = 0x02020202u;  // bias bytes: 0x0202 = 514 per u16 half
#pragma unroll
    for (int rnd = 0; rnd < kRounds; rnd++) {
      const int p = hl + G * rnd;
      if (p < 121) {
        const int k = p / 11, yr = p - 11 * k;  // offset k - L, window row yr - w
        const int cr = wb[44 * w + 16 + (xcr + k - L - ar)];
        const uint32_t* rowL = ww + 11 * yr;
        const int oR = oR0 + k;  // 0..13: the right row's bytes oR .. oR + 10 (of 28)
        const uint32_t* rowR = rowL + 4 + (oR >> 2);
        const uint32_t l0 = rowL[0], l1 = rowL[1], l2 = rowL[2], l3 = rowL[3];
        const uint32_t r0 = rowR[0], r1 = rowR[1], r2 = rowR[2], r3 = rowR[3];
        const uint32_t a[3] = {__builtin_amdgcn_alignbyte(l1, l0, oL),
                               __builtin_amdgcn_alignbyte(l2, l1, oL),
                               __builtin_amdgcn_alignbyte(l3, l2, oL)};
        const uint32_t bsh = (uint32_t)(oR & 3);
        const uint32_t bb[3] = {__builtin_amdgcn_alignbyte(r1, r0, bsh),
                                __builtin_amdgcn_alignbyte(r2, r1, bsh),
                                __builtin_amdgcn_alignbyte(r3, r2, bsh)};
        // cl - cr added to each u16 half (v_pk_add_u16 wraps per half; every sum lies in
        // [257, 1022]): the last pair's high half stays the bias on both sides
        typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
        const unsigned short d = (unsigned short)(cl - cr);
        const u16x2_t dd = {d, d}, dlast = {d, 0};
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) {
          const uint32_t sel = j == 5 ? 0x04040402u : (j & 1) ? 0x04030402u : 0x05010400u;
          const uint32_t A = __builtin_amdgcn_perm(kBias, a[j >> 1], sel);
          const u16x2_t B = __builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(kBias, bb[j >> 1], sel)) +
                            (j == 5 ? dlast : dd);
          acc = __builtin_amdgcn_sad_u16(A, __builtin_bit_cast(uint32_t, B), acc);
        }
        part[p] = (int)acc;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int sad = 0x7fffffff;
  if (ok && hl < 2 * L + 1) {
    int acc = 0;
#pragma unroll
    for (int yy = 0; yy < 2 * w + 1; yy++) acc += part[11 * hl + yy];
    sad = acc;
  }
  float vDists[11];
#pragma unroll
  for (int k = 0; k < 11; k++) vDists[k] = (float)__shfl(sad, G * grp + k, 64);
  if (!ok || hl != 0) return;
  int bestSad = 0x7fffffff, bestincR = 0;
#pragma unroll
  for (int k = 0; k < 11; k++) {
    if (vDists[k] < (float)bestSad) {
      bestSad = (int)vDists[k];
      bestincR = k - L;
    }
  }
  if (bestincR == -L || bestincR == L) return;
  const float dist1 = vDists[L + bestincR - 1];
  const float dist2 = vDists[L + bestincR];
  const float dist3 = vDists[L + bestincR + 1];
  const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
  if (deltaR < -1 || deltaR > 1) return;
  float bestuR = LG.scale * ((float)scaleduR0 + (float)bestincR + deltaR);
  float disparity = (uL - bestuR);
  if (disparity >= minD && disparity < maxD) {
    if (disparity <= 0) {
      disparity = 0.01f;
      bestuR = uL - 0.01f;
    }
    out.depth[o] = cam.bf / disparity;
    out.u_right[o] = bestuR;
    ws.sad[o] = bestSad;
  }
}

// Median SAD filter (:564-576): drop matches whose SAD >= 2.1 * median. The median (element
// n / 2 of the ascending sort, :564-566) is found by an MSB-first radix select over the SADs
// (four 8-bit digit histograms) instead of sorting them.
// pack (the single-frame call, frame 0 only): the frame's final u_right / depth also go to the
// packed host-mirror record (frame_pack_kernel's layout), and the device error word to its
// header slot 8 -- no frame_pack launch after this one on the call's critical path.
// NT threads per frame (1024 for the single-frame call). The digit rounds start at the highest
// non-zero byte of the OR of all SADs (SADs are below 121 * 510 < 2^16: two rounds, not four).
template <int NT>
__global__ __launch_bounds__(NT) void stereo_median_kernel(const OrbGeom* __restrict__ g,
                                                           FrameKps ext, StereoWorkspace ws,
                                                           StereoOut out,
                                                           uint8_t* __restrict__ pack,
                                                           const uint32_t* __restrict__ err) {
  constexpr int kCap = 4096;
  __shared__ uint32_t vals[kCap];
  __shared__ int hist[256];
  __shared__ int n_valid, s_digit, s_rank;
  __shared__ uint32_t s_or;
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int nl = min(ext.n[2 * f * ext.n_stride], kCap);
  const int64_t base = (int64_t)f * g->kp_cap;
  if (tid == 0) {
    n_valid = 0;
    s_or = 0;
  }
  __syncthreads();
  uint32_t vor = 0;
  for (int i0 = 0; i0 < nl; i0 += NT * 4) {  // 4 loads in flight per thread
    int sv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = i0 + NT * u + tid;
      sv[u] = i < nl ? ws.sad[base + i] : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (sv[u] >= 0) {
        vals[atomicAdd(&n_valid, 1)] = (uint32_t)sv[u];
        vor |= (uint32_t)sv[u];
      }
  }
  vor = wave_or(vor);
  if (lane == 0 && vor) atomicOr(&s_or, vor);
  __syncthreads();
  const int n = n_valid;
  const uint32_t all_or = s_or;
  // n == 0: the reference indexes an empty vector here (UB); we skip the filter
  uint32_t prefix = 0, mask = 0;
  int k = n / 2;  // rank of the median among the values matching prefix under mask
  const int top = all_or >> 24 ? 24 : all_or >> 16 ? 16 : all_or >> 8 ? 8 : 0;
  for (int shift = top; shift >= 0 && n > 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += NT) {
      const uint32_t v = vals[i];
      if ((v & mask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1);
    }
    __syncthreads();
    if (tid < 64) {  // the digit whose cumulative count passes k: lane owns bins 4 lane .. +3
      int h[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        h[j] = hist[4 * lane + j];
        sum += h[j];
      }
      int x = sum;  // inclusive scan over the wave
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      const int before = x - sum;
      if (before <= k && k < x) {  // exactly one lane
        int acc = before, d = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (d == 0 && acc + h[j] > k) d = j + 1;
          else if (d == 0) acc += h[j];
        s_digit = 4 * lane + d - 1;
        s_rank = k - acc;
      }
    }
    __syncthreads();
    prefix |= (uint32_t)s_digit << shift;
    mask |= 255u << shift;
    k = s_rank;
    __syncthreads();
  }
  const float median = (float)(int)prefix;
  const float thDist = (1.5f * 1.4f) * median;
  const size_t kc = (size_t)g->kp_cap;
  float* const pur = pack && f == 0
                         ? reinterpret_cast<float*>(pack + 16 + 2 * kc * sizeof(KeyPoint) + 2 * kc * 32)
                         : nullptr;
  const int nall = pur ? min(max(ext.n[0], 0), (int)kc) : nl;
  for (int i = tid; i < nall; i += NT) {
    const int s = i < nl ? ws.sad[base + i] : -1;
    if (n > 0 && s >= 0 && !((float)s < thDist)) {
      out.u_right[base + i] = -1.0f;
      out.depth[base + i] = -1.0f;
      ws.sad[base + i] = -1;
      if (pur) pur[i] = pur[kc + i] = -1.0f;
    } else if (pur) {
      pur[i] = out.u_right[base + i];
      pur[kc + i] = out.depth[base + i];
    }
  }
  __syncthreads();  // every error bit this stream's kernels raise is in err by now
  if (pur && tid == 0) reinterpret_cast<uint32_t*>(pack)[2] = *err;
}

// ---------------------------------------------------------------------------------------
// Frame results -> the host mirror's layout (see match_kernels.h), copied as dwords.
// parts: bit 0 -- the counts, both views' keypoints and descriptors, the error word to header
// slot 12; bit 1 -- u_right / depth, the error word to slot 8 (stereo_median_kernel does this part
// itself in the single-frame call). The host ORs the two error slots.
__device__ __forceinline__ void frame_pack_body(const FrameKps& ext,
                                                const float* __restrict__ u_right,
                                                const float* __restrict__ depth,
                                                const uint32_t* __restrict__ err, int kp_cap,
                                                uint8_t* __restrict__ dst, int parts, int gid,
                                                int gsz) {
  const int c0 = ext.n[0], c1 = ext.n[ext.n_stride];
  const int n0 = min(max(c0, 0), kp_cap), n1 = min(max(c1, 0), kp_cap);
  const size_t kc = (size_t)kp_cap;
  if (gid == 0) {
    int* h = reinterpret_cast<int*>(dst);
    if (parts & 1) {
      h[0] = c0;
      h[1] = c1;
      h[3] = (int)*err;
    }
    if (parts & 2) h[2] = (int)*err;
  }
  auto copy = [&](const void* src, size_t dst_off, int words) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + dst_off);
    for (int i = gid; i < words; i += gsz) d[i] = s[i];
  };
  const size_t kps_off = 16, desc_off = kps_off + 2 * kc * sizeof(KeyPoint);
  const size_t ur_off = desc_off + 2 * kc * 32, dp_off = ur_off + kc * sizeof(float);
  if (parts & 1) {
    copy(ext.kps, kps_off, 7 * n0);
    copy(ext.kps + ext.stride, kps_off + kc * sizeof(KeyPoint), 7 * n1);
    copy(ext.desc, desc_off, 8 * n0);
    copy(ext.desc + 32 * ext.stride, desc_off + 32 * kc, 8 * n1);
  }
  if (parts & 2) {
    copy(u_right, ur_off, n0);
    copy(depth, dp_off, n0);
  }
}
__global__ __launch_bounds__(256) void frame_pack_kernel(FrameKps ext,
                                                         const float* __restrict__ u_right,
                                                         const float* __restrict__ depth,
                                                         const uint32_t* __restrict__ err,
                                                         int kp_cap, uint8_t* __restrict__ dst,
                                                         int parts) {
  frame_pack_body(ext, u_right, depth, err, kp_cap, dst, parts,
                  blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

void launch_frame_pack(const FrameKps& ext, const float* u_right, const float* depth,
                       const uint32_t* err, int kp_cap, uint8_t* dst, hipStream_t st, int parts) {
  static_assert(sizeof(KeyPoint) == 28, "keypoint layout");
  SLAMGPU_LAUNCH("frame_pack", st, frame_pack_kernel, dim3(32), dim3(256), 0, st, ext, u_right,
                 depth, err, kp_cap, dst, parts);
}

__global__ void trace_marker_kernel() {}

void launch_trace_marker(int id, hipStream_t st) {
  hipLaunchKernelGGL(trace_marker_kernel, dim3(1, id), dim3(64), 0, st);
}

void launch_stereo(const ImageBatch& b, const OrbGeomDev& gd, const Camera& cam, int n_frames,
                   const StereoWorkspace& ws, const StereoOut& out, hipStream_t st,
                   uint8_t* pack, bool rows_done) {
  const OrbGeom& g = *gd.host;
  FrameKps ext{gd.out.kps, gd.out.desc, gd.out.nkps, g.kp_cap, 1};
  const int nrows = g.lv[0].h;
  if (rows_done) {  // frame_aux_kernel built them
  } else if (n_frames <= 8)
    SLAMGPU_LAUNCH("stereo_rows", st, stereo_rows_kernel<1024>, dim3(n_frames), dim3(1024), 0, st,
                   gd.dev, ext, nrows, ws, gd.ws.err);
  else
    SLAMGPU_LAUNCH("stereo_rows", st, stereo_rows_kernel<256>, dim3(n_frames), dim3(256), 0, st,
                   gd.dev, ext, nrows, ws, gd.ws.err);
  constexpr int kG = STEREO_LANES, kPerBlock = 4 * (64 / kG);
  SLAMGPU_LAUNCH("stereo_match", st, stereo_match_kernel<kG>,
                 dim3((g.kp_cap + kPerBlock - 1) / kPerBlock, n_frames), dim3(256), 0, st, b,
                 gd.dev, ext, cam, nrows, ws, out);
  if (n_frames <= 8)
    SLAMGPU_LAUNCH("stereo_median", st, stereo_median_kernel<1024>, dim3(n_frames), dim3(1024), 0,
                   st, gd.dev, ext, ws, out, pack, gd.ws.err);
  else
    SLAMGPU_LAUNCH("stereo_median", st, stereo_median_kernel<256>, dim3(n_frames), dim3(256), 0,
                   st, gd.dev, ext, ws, out, pack, gd.ws.err);
}

// ---------------------------------------------------------------------------------------
// Grid (AssignFeaturesToGrid + PosInGrid, frame.cpp:234-248, 339-346).
__device__ __forceinline__ int grid_cell(const Camera& cam, float x, float y) {
  const int px = (int)roundf((x - cam.min_x) / cam.cell_w);
  const int py = (int)roundf((y - cam.min_y) / cam.cell_h);
  if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) return -1;
  return px * kGridRows + py;
}

template <int NT>
__device__ __forceinline__ void grid_build_body(int f, const FrameKps& cur, const Camera& cam,
                                                int kp_cap, const GridWorkspace& gw) {
  __shared__ int cnt[kGridCells + 1];
  __shared__ int wsum[NT / 64];
  const int tid = threadIdx.x;
  const KeyPoint* k = cur.kps + f * cur.stride;
  const int n = cur.n[f * cur.n_stride];
  int* cs = gw.cell_start + (int64_t)f * (kGridCells + 1);
  uint4* items = gw.cell_items + (int64_t)f * kp_cap;
  for (int i = tid; i <= kGridCells; i += NT) cnt[i] = 0;
  // cells of a thread's keypoints, kChunk loads in flight at a time; the items carry the fields
  // the projection searches filter on first (one load per candidate instead of two)
  constexpr int kChunk = 2048 / NT;
  float kx[kChunk], ky[kChunk];
  int ko[kChunk];
  auto cells = [&](int base, int (&c)[kChunk]) {
#pragma unroll
    for (int u = 0; u < kChunk; u++) {
      const int i = base + NT * u + tid;
      kx[u] = ky[u] = 0.0f;
      ko[u] = 0;
      if (i < n) {
        kx[u] = k[i].x;
        ky[u] = k[i].y;
        ko[u] = k[i].octave;
      }
    }
#pragma unroll
    for (int u = 0; u < kChunk; u++)
      c[u] = base + NT * u + tid < n ? grid_cell(cam, kx[u], ky[u]) : -1;
  };
  __syncthreads();
  for (int base = 0; base < n; base += NT * kChunk) {
    int c[kChunk];
    cells(base, c);
#pragma unroll
    for (int u = 0; u < kChunk; u++)
      if (c[u] >= 0) atomicAdd(&cnt[c[u]], 1);
  }
  __syncthreads();
  const int total = scan256<kGridCells + 1, NT>(cnt, kGridCells, wsum);
  for (int i = tid; i < kGridCells; i += NT) cs[i] = cnt[i];
  if (tid == 0) cs[kGridCells] = total;
  __syncthreads();
  for (int base = 0; base < n; base += NT * kChunk) {
    int c[kChunk];
    cells(base, c);
#pragma unroll
    for (int u = 0; u < kChunk; u++)
      if (c[u] >= 0)
        items[atomicAdd(&cnt[c[u]], 1)] =
            make_uint4((uint32_t)(base + NT * u + tid) | (uint32_t)ko[u] << 16,
                       __float_as_uint(kx[u]), __float_as_uint(ky[u]), 0u);
  }
}
__global__ __launch_bounds__(256) void grid_build_kernel(FrameKps cur, Camera cam, int kp_cap,
                                                         GridWorkspace gw) {
  grid_build_body<256>(blockIdx.x, cur, cam, kp_cap, gw);
}

void launch_grid(const FrameKps& cur, const Camera& cam, int n_frames, int kp_cap,
                 const GridWorkspace& gw, hipStream_t st) {
  SLAMGPU_LAUNCH("grid_build", st, grid_build_kernel, dim3(n_frames), dim3(256), 0, st, cur, cam,
                 kp_cap, gw);
}

// The single-frame call's three independent steps after the descriptors, as three work-groups
// of one launch (side by side on three CUs): blockIdx.y 0 the stereo row tables, 1 the left
// view's grid, 2 the counts / keypoints / descriptors packed into the host mirror.
__global__ __launch_bounds__(1024) void frame_aux_kernel(const OrbGeom* __restrict__ g,
                                                         FrameKps ext, int nrows,
                                                         StereoWorkspace ws, uint32_t* err,
                                                         FrameKps left, Camera cam, int kp_cap,
                                                         GridWorkspace gw, uint8_t* pack) {
  switch (blockIdx.y) {
    case 0: stereo_rows_body<1024>(0, g, ext, nrows, ws, err); break;
    case 1: grid_build_body<1024>(0, left, cam, kp_cap, gw); break;
    default:
      frame_pack_body(ext, nullptr, nullptr, err, kp_cap, pack, 1, threadIdx.x, 1024);
      break;
  }
}

void launch_frame_aux(const OrbGeomDev& gd, const FrameKps& left, const Camera& cam,
                      const GridWorkspace& gw, const StereoWorkspace& ws, uint8_t* pack,
                      hipStream_t st) {
  const OrbGeom& g = *gd.host;
  FrameKps ext{gd.out.kps, gd.out.desc, gd.out.nkps, g.kp_cap, 1};
  SLAMGPU_LAUNCH("frame_aux", st, frame_aux_kernel, dim3(1, 3), dim3(1024), 0, st, gd.dev, ext,
                 g.lv[0].h, ws, gd.ws.err, left, cam, g.kp_cap, gw, pack);
}

// ---------------------------------------------------------------------------------------
// Frame::UndistortKeyPoints (frame.cpp:614-641): a thread per keypoint of every set, the
// keypoint copied with pt replaced by cv::undistortPoints (undistort.h; IEEE double, no
// contraction, bit-identical to the oracle). dist k1 == 0 copies (:616-619).
__global__ __launch_bounds__(256) void undistort_kernel(FrameKps src, KeyPoint* __restrict__ dst,
                                                        int64_t dst_stride, float fx, float fy,
                                                        float cx, float cy, Distortion dc) {
  const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  if (i >= src.n[f * src.n_stride]) return;
  KeyPoint kp = src.kps[f * src.stride + i];
  if (dc.k[0] != 0.0f) undistort_point(fx, fy, cx, cy, dc, kp.x, kp.y, &kp.x, &kp.y);
  dst[f * dst_stride + i] = kp;
}

void launch_undistort(const FrameKps& src, KeyPoint* dst, int64_t dst_stride, const Camera& cam,
                      const Distortion& dc, int n_sets, int kp_cap, hipStream_t st) {
  SLAMGPU_LAUNCH("undistort", st, undistort_kernel, dim3((kp_cap + 255) / 256, n_sets), dim3(256),
                 0, st, src, dst, dst_stride, cam.fx, cam.fy, cam.cx, cam.cy, dc);
}

// ---------------------------------------------------------------------------------------
// Candidate scan of one query by one wave: Frame::GetFeaturesInArea (frame.cpp:348-403) plus the
// matcher's per-candidate filters, keeping the kTopK best candidates by (distance, position in
// GetFeaturesInArea order). That order visits cells x-major then y, each cell by keypoint index,
// so the position key is (ix * 48 + iy, index) -- which makes the lexicographic minimum equal
// to the first strict-'<' winner of the reference's sequential loop.
struct ScanCtx {
  float x, y, r;         // GetFeaturesInArea(x, y, r, min_level, max_level)
  int min_level, max_level;
  float ur, gate;        // skip if u_right > 0 && fabsf(ur - u_right) > gate
  int max_dist;          // keep candidates with distance <= max_dist
  const uint8_t* desc;   // query descriptor
};

struct FrameView {
  const KeyPoint* kps;
  const uint8_t* desc;
  const float* u_right;
  const int* cell_start;
  const uint4* cell_items;
  const uint8_t* blocked;
};

// Wave reductions over the lanes by the permlane / DPP butterfly of lane_partner_u32 (no LDS
// round trips; every lane ends with the result). Keys are compared as unsigned integers.
__device__ __forceinline__ uint32_t wave_min_key(uint32_t v) {
#pragma unroll
  for (int M = 32; M >= 1; M >>= 1) v = min(v, lane_partner_u32(v, M));
  return v;
}
__device__ __forceinline__ uint64_t wave_min_key(uint64_t v) {
#pragma unroll
  for (int M = 32; M >= 1; M >>= 1) {
    const uint64_t o = (uint64_t)lane_partner_u32((uint32_t)(v >> 32), M) << 32 |
                       lane_partner_u32((uint32_t)v, M);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int wave_sum_bfly(int v) {
#pragma unroll
  for (int M = 32; M >= 1; M >>= 1) v += (int)lane_partner_u32((uint32_t)v, M);
  return v;
}
// Inclusive prefix sum over the 64 lanes: DPP row shifts within each row of 16 lanes, then the
// row totals carried by row_bcast:15 / row_bcast:31.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// The same over groups of G lanes (G = 16: a DPP row; 64: the wave); a butterfly level M < 16
// stays inside a row (lane_partner_u32)
template <int G>
__device__ __forceinline__ int group_incl_scan(int v) {
  static_assert(G == 16 || G == 64, "groups are DPP rows or the wave");
  if constexpr (G == 64) {
    return wave_incl_scan(v);
  } else {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    return v;
  }
}
template <int G>
__device__ __forceinline__ uint32_t group_min_key(uint32_t v) {
#pragma unroll
  for (int M = G / 2; M >= 1; M >>= 1) v = min(v, lane_partner_u32(v, M));
  return v;
}
template <int G>
__device__ __forceinline__ uint64_t group_min_key(uint64_t v) {
#pragma unroll
  for (int M = G / 2; M >= 1; M >>= 1) {
    const uint64_t o = (uint64_t)lane_partner_u32((uint32_t)(v >> 32), M) << 32 |
                       lane_partner_u32((uint32_t)v, M);
    v = o < v ? o : v;
  }
  return v;
}
template <int G>
__device__ __forceinline__ int group_sum(int v) {
#pragma unroll
  for (int M = G / 2; M >= 1; M >>= 1) v += (int)lane_partner_u32((uint32_t)v, M);
  return v;
}

// The scan's candidate key, ordered as (distance, cell, index): 32 bits -- dist (<= 256) << 23 |
// cell (< 4096) << 11 | index (< 2048) -- when the frame's keypoint capacity allows, else the 64-bit
// form the resolution pass reads (dist << 32 | cell << 12 | index).
template <typename K>
__device__ __forceinline__ K scan_key(int dist, int cell, int i) {
  if constexpr (sizeof(K) == 4)
    return (uint32_t)dist << 23 | (uint32_t)cell << 11 | (uint32_t)i;
  else
    return ((uint64_t)dist << 32) | ((uint64_t)cell << 12) | (uint64_t)i;
}
template <typename K>
__device__ __forceinline__ uint64_t key64(K k) {
  if constexpr (sizeof(K) == 4)
    return k == ~0u ? kNoKey
                    : ((uint64_t)(k >> 23) << 32) | ((uint64_t)((k >> 11) & 0xfffu) << 12) |
                          (uint64_t)(k & 0x7ffu);
  else
    return k;
}

// G lanes per query (the group of `lane`): 64 for the resolution pass's rescans, 16 for
// search_cand (a window holds a handful of keypoints: four queries per wave keep the lanes busy)
// float -> int of a cell coordinate with its argument held in range first: a float-to-int
// conversion out of int's range (or of NaN) is undefined, so no coordinate reaches one
__device__ __forceinline__ int cell_floor(float v) { return (int)floorf(fminf(fmaxf(v, -1e6f), 1e6f)); }
__device__ __forceinline__ int cell_ceil(float v) { return (int)ceilf(fminf(fmaxf(v, -1e6f), 1e6f)); }

// skip: the group has no query (or its context failed): it scans nothing -- no cell bound is
// derived from its coordinates -- but still takes part in the group's shuffles and the merge
template <typename K, int G = 64>
__device__ int scan_query_k(const ScanCtx& c, const Camera& cam, const FrameView& F,
                            const uint32_t* claimed, uint64_t* top, int lane, bool skip = false) {
  const int gl = lane & (G - 1), gb = lane & ~(G - 1);
  int nMinCellX = 0, nMaxCellX = -1, nMinCellY = 0, nMaxCellY = -1;  // empty window
  if (!skip) {
    nMinCellX = max(0, cell_floor((c.x - cam.min_x - c.r) / cam.cell_w));
    nMaxCellX = min(kGridCols - 1, cell_ceil((c.x - cam.min_x + c.r) / cam.cell_w));
    nMinCellY = max(0, cell_floor((c.y - cam.min_y - c.r) / cam.cell_h));
    nMaxCellY = min(kGridRows - 1, cell_ceil((c.y - cam.min_y + c.r) / cam.cell_h));
  }
  constexpr K kNone = (K)~(K)0;
  K t[kTopK];
#pragma unroll
  for (int k = 0; k < kTopK; k++) t[k] = kNone;
  int cnt = 0;
  if (!(nMaxCellX < 0 || nMinCellX >= kGridCols || nMaxCellY < 0 || nMinCellY >= kGridRows)) {
    const bool bCheckLevels = (c.min_level > 0) || (c.max_level >= 0);
    const int ny = nMaxCellY - nMinCellY + 1;
    const int total = (nMaxCellX - nMinCellX + 1) * ny;
    // The window's (cell, keypoint) pairs are spread over the lanes, one keypoint each: a lane
    // per cell would walk its cell's keypoints as one serial chain of dependent loads while the
    // lanes of empty or absent cells idle. Cells 64 at a time: per-lane keypoint counts, their
    // wave prefix sum, then lane k takes pair k (its cell found by a binary search over the
    // prefix sums). The kept candidates are an order-free minimum, so any order gives the same.
    for (int cb = 0; cb < total; cb += G) {
      const int ci = cb + gl;
      int cell = 0, q0 = 0, nq = 0;
      if (ci < total) {
        const int ix = nMinCellX + ci / ny, iy = nMinCellY + ci % ny;
        cell = ix * kGridRows + iy;
        q0 = F.cell_start[cell];
        nq = F.cell_start[cell + 1] - q0;
      }
      const int incl = group_incl_scan<G>(nq);
      const int excl = incl - nq;
      const int npairs = G == 64 ? __builtin_amdgcn_readlane(incl, 63) : __shfl(incl, gb + G - 1, 64);
      // every lane of the group takes part in the shuffles (a shuffle reads 0 from an inactive
      // lane); groups run their own trip counts, their shuffles stay inside the group
      for (int k0 = 0; k0 < npairs; k0 += G) {
        const int k = k0 + gl;
        int lo = 0;  // the group's last lane whose exclusive offset is <= k
#pragma unroll
        for (int step = G / 2; step >= 1; step >>= 1) {
          const int cand = lo + step;
          const int ec = __shfl(excl, gb + (cand & (G - 1)), 64);
          if (cand < G && ec <= k) lo = cand;
        }
        const int p = __shfl(q0, gb + lo, 64) + (k - __shfl(excl, gb + lo, 64));
        const int pcell = __shfl(cell, gb + lo, 64);
        if (k >= npairs) continue;
        const uint4 it = F.cell_items[p];
        const int i = (int)(it.x & 0xffffu), octave = (int)(it.x >> 16);
        if (bCheckLevels) {
          if (octave < c.min_level) continue;
          if (c.max_level >= 0 && octave > c.max_level) continue;
        }
        const float distx = __uint_as_float(it.y) - c.x, disty = __uint_as_float(it.z) - c.y;
        if (!(fabsf(distx) < c.r && fabsf(disty) < c.r)) continue;
        // the remaining filters' loads all in flight together (the filters commute)
        const bool blk = F.blocked[i] != 0;
        const float ur = F.u_right[i];
        const int dist = hamming32(c.desc, F.desc + i * 32);
        if (blk) continue;
        if (claimed && (claimed[i >> 5] >> (i & 31)) & 1u) continue;
        if (ur > 0 && fabsf(c.ur - ur) > c.gate) continue;
        if (dist > c.max_dist) continue;
        const K key = scan_key<K>(dist, pcell, i);
        cnt++;
        if (key < t[kTopK - 1]) {
          t[kTopK - 1] = key;
#pragma unroll
          for (int k2 = kTopK - 1; k2 > 0; k2--)
            if (t[k2] < t[k2 - 1]) {
              const K s2 = t[k2];
              t[k2] = t[k2 - 1];
              t[k2 - 1] = s2;
            }
        }
      }
    }
  }
  // merge the per-lane sorted lists: up to kTopK rounds of wave minimum, ending early once the
  // wave has no candidate left (most queries keep fewer than kTopK)
#pragma unroll
  for (int k = 0; k < kTopK; k++) top[k] = kNoKey;
#pragma unroll
  for (int k = 0; k < kTopK; k++) {
    const K m = G == 64 ? wave_min_key(t[0]) : group_min_key<G>(t[0]);
    if (G == 64) {
      if (m == kNone) break;  // wave-uniform
    } else if (__ballot(m != kNone) == 0) {
      break;  // no group has a candidate left
    }
    if (m != kNone) {
      if (t[0] == m) {
#pragma unroll
        for (int j = 0; j < kTopK - 1; j++) t[j] = t[j + 1];
        t[kTopK - 1] = kNone;
      }
      top[k] = key64<K>(m);
    }
  }
  return G == 64 ? wave_sum_bfly(cnt) : group_sum<G>(cnt);
}

// 32-bit keys whenever the frame's keypoint indices fit 11 bits (kp_cap <= 2048: nfeatures up to
// ~2000 with the per-level slack), the 64-bit form otherwise.
template <int G = 64>
__device__ __forceinline__ int scan_query(const ScanCtx& c, const Camera& cam, const FrameView& F,
                                          const uint32_t* claimed, uint64_t* top, int lane,
                                          int kp_cap, bool skip = false) {
  if (kp_cap <= 2048) return scan_query_k<uint32_t, G>(c, cam, F, claimed, top, lane, skip);
  return scan_query_k<uint64_t, G>(c, cam, F, claimed, top, lane, skip);
}

__device__ __forceinline__ int key_idx(uint64_t k) { return (int)(k & 0xfff); }
__device__ __forceinline__ int key_dist(uint64_t k) { return (int)(k >> 32); }

// OpenCV small float gemm d = A*b + c (matmul.cpp, len 3): float dot, then (float)((double)+).
__device__ __forceinline__ float mat3_row(const float* R, int r, const float* x, float c) {
  const float dot = R[3 * r] * x[0] + R[3 * r + 1] * x[1] + R[3 * r + 2] * x[2];
  return (float)((double)dot + (double)c);
}

// SearchByProjection(CurrentFrame, LastFrame) per-query setup (orb_matcher.cpp:1336-1376).
__device__ bool f2f_ctx(const F2FQuery& q, const F2FPose& P, const Camera& cam,
                        const OrbGeom* g, ScanCtx* c) {
  const float xc = mat3_row(P.Rcw, 0, q.xyz, P.tcw[0]);
  const float yc = mat3_row(P.Rcw, 1, q.xyz, P.tcw[1]);
  const float zc = mat3_row(P.Rcw, 2, q.xyz, P.tcw[2]);
  const float invzc = (float)(1.0 / (double)zc);
  if (invzc < 0) return false;
  const float u = fmaf(cam.fx * xc, invzc, cam.cx);
  const float v = fmaf(cam.fy * yc, invzc, cam.cy);
  if (u < cam.min_x || u > cam.max_x) return false;
  if (v < cam.min_y || v > cam.max_y) return false;
  const int nLastOctave = q.last_octave;
  const float radius = P.th * g->lv[nLastOctave].scale;
  const bool bForward = P.tlc_z > P.baseline && !P.mono;
  const bool bBackward = -P.tlc_z > P.baseline && !P.mono;
  c->x = u;
  c->y = v;
  c->r = radius;
  if (bForward) {
    c->min_level = nLastOctave;
    c->max_level = -1;
  } else if (bBackward) {
    c->min_level = 0;
    c->max_level = nLastOctave;
  } else {
    c->min_level = nLastOctave - 1;
    c->max_level = nLastOctave + 1;
  }
  c->ur = fmaf(-cam.bf, invzc, u);
  c->gate = radius;
  c->max_dist = TH_HIGH;  // a candidate above TH_HIGH can never become the accepted match
  c->desc = q.desc;
  return true;
}

// SearchByProjection(F, vpMapPoints, th) per-query setup (orb_matcher.cpp:21-41, 105-111).
__device__ bool mps_ctx(const MpsQuery& q, int th, const OrbGeom* g, ScanCtx* c) {
  if (!q.in_view || q.is_bad) return false;
  float r = ((double)q.view_cos > 0.998) ? 2.5f : 4.0f;
  if (th != 1) r *= (float)th;
  const float rs = r * g->lv[q.level].scale;
  c->x = q.proj_x;
  c->y = q.proj_y;
  c->r = rs;
  c->min_level = q.level - 1;
  c->max_level = q.level;
  c->ur = q.proj_xr;
  c->gate = rs;
  c->max_dist = 256;
  c->desc = q.desc;
  return true;
}

#ifndef SEARCH_LANES
#define SEARCH_LANES 16
#endif
constexpr int kSearchG = SEARCH_LANES;  // lanes per query in search_cand (16 or 64)
template <typename Q>
__global__ __launch_bounds__(256) void search_cand_kernel(
    FrameKps cur, const float* __restrict__ u_right, int64_t ur_stride, Camera cam,
    const OrbGeom* __restrict__ g, const Q* __restrict__ queries, const F2FPose* __restrict__ poses,
    int th, GridWorkspace gw, MatchWorkspace mw, MatchIO io) {
  int f, bx;
  xcd_image_block(&f, &bx);  // a frame's work-groups share one XCD's L2 (its grid and keypoints)
  // kSearchG lanes per query: 64 / kSearchG queries per wave
  const int lane = threadIdx.x & 63, gl = lane & (kSearchG - 1);
  const int qi = (bx * 4 + wave_id()) * (64 / kSearchG) + lane / kSearchG;
  const int qcount = io.q_count[f];
  if (__builtin_amdgcn_readfirstlane((bx * 4 + wave_id()) * (64 / kSearchG)) >= qcount) return;
  const bool live = qi < qcount;  // the wave's last groups may have no query
  const int q = io.q_start[f] + (live ? qi : 0);
  FrameView F;
  F.kps = cur.kps + f * cur.stride;
  F.desc = cur.desc + f * cur.stride * 32;
  F.u_right = u_right + f * ur_stride;
  F.cell_start = gw.cell_start + (int64_t)f * (kGridCells + 1);
  F.cell_items = gw.cell_items + (int64_t)f * g->kp_cap;
  F.blocked = io.blocked + f * io.mp_stride;
  ScanCtx c;
  bool ok;
  if constexpr (sizeof(Q) == sizeof(F2FQuery)) {
    ok = f2f_ctx(queries[q], poses[f], cam, g, &c);
  } else {
    ok = mps_ctx(queries[q], th, g, &c);
  }
  ok = ok && live;
  uint64_t top[kTopK];
  // a group without a query scans nothing but takes part in the merge
  const int n = scan_query<kSearchG>(c, cam, F, nullptr, top, lane, g->kp_cap, !ok);
  if (live && gl < kTopK) {
    uint64_t v = top[0];
#pragma unroll
    for (int k = 1; k < kTopK; k++)
      if (gl == k) v = top[k];
    mw.topk[(int64_t)q * kTopK + gl] = ok ? v : kNoKey;
  }
  if (live && gl == 0) mw.ncand[q] = ok ? n : 0;
}

// Sequential, in-query-order claim resolution: one wave per frame. The kernel is a chain of
// latency (a frame's queries in order), so everything it can take off that chain is: the
// keypoint fields it needs are staged with all loads in flight, the next 64 queries' candidates
// are loaded while the current ones resolve, a candidate's "claimed" state is read once per
// round (claims change only when a round commits), and the rotation-histogram bookkeeping of the
// first kResolveLdsQ queries stays in LDS (a frame's later queries, if any, use the workspace).
constexpr int kResolveLdsQ = 4096;
template <typename Q>
__global__ __launch_bounds__(64) void search_resolve_kernel(
    FrameKps cur, const float* __restrict__ u_right, int64_t ur_stride, Camera cam,
    const OrbGeom* __restrict__ g, const Q* __restrict__ queries, const F2FPose* __restrict__ poses,
    int th, float nnratio, GridWorkspace gw, MatchWorkspace mw, MatchIO io) {
  constexpr bool kF2F = sizeof(Q) == sizeof(F2FQuery);
  __shared__ uint32_t claimed[128];  // kp_cap <= 4096
  __shared__ int hist[HISTO_LENGTH];
  __shared__ float s_kang[kF2F ? 4096 : 1];
  __shared__ int8_t s_koct[kF2F ? 1 : 4096];
  __shared__ int owner[4096];
  __shared__ int8_t s_bin[kF2F ? kResolveLdsQ : 1];     // rotation bin of query qi (-1 none)
  __shared__ int16_t s_best[kF2F ? kResolveLdsQ : 1];   // its matched keypoint
  const int f = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = cur.n[f * cur.n_stride];
  for (int i = lane; i < 128; i += 64) claimed[i] = 0;
  if (lane < HISTO_LENGTH) hist[lane] = 0;
  FrameView F;
  F.kps = cur.kps + f * cur.stride;
  F.desc = cur.desc + f * cur.stride * 32;
  F.u_right = u_right + f * ur_stride;
  F.cell_start = gw.cell_start + (int64_t)f * (kGridCells + 1);
  F.cell_items = gw.cell_items + (int64_t)f * g->kp_cap;
  F.blocked = io.blocked + f * io.mp_stride;
  int* mp = io.map_point + f * io.mp_stride;
  uint8_t* blk = io.blocked + f * io.mp_stride;
  bool check_ori = false;
  if constexpr (kF2F) check_ori = poses[f].check_ori != 0;
  const int q0 = io.q_start[f], qn = io.q_count[f];
  int nm = 0;
  // The reference resolves queries strictly in order: a query takes its first candidate (in
  // (distance, GetFeaturesInArea) order) not claimed by an earlier *blocking* query
  // (orb_matcher.cpp:59-63, :1389-1393). Here 64 queries (one per lane) are resolved together
  // to the same result: each lane's choice is iterated to a fixed point against the claims
  // committed so far and the choices of the earlier lanes (owner[] holds the lowest blocking
  // lane per keypoint) -- lane i is final once lanes < i are, and conflicts are rare, so a few
  // rounds suffice. A lane whose kept top-K is exhausted while more candidates exist is rescanned
  // alone, at its place in the order. For non-blocking duplicates the last writer of mp[idx]
  // wins, as in the sequential loop.
  // keypoint fields (F2F: the angle, only with the rotation check; local map: the octave),
  // four loads in flight per lane
  for (int i0 = 0; i0 < n; i0 += 256) {
    float ang[4];
    int oct[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = i0 + 64 * u + lane;
      ang[u] = 0.f;
      oct[u] = 0;
      if (i < n) {
        if constexpr (kF2F) {
          if (check_ori) ang[u] = F.kps[i].angle;
        } else {
          oct[u] = F.kps[i].octave;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int i = i0 + 64 * u + lane;
      if (i < n) {
        if constexpr (kF2F) s_kang[i] = ang[u];
        else s_koct[i] = (int8_t)oct[u];
        owner[i] = INT_MAX;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int need = kF2F ? 1 : 2;
  auto is_claimed = [&](int idx) { return (claimed[idx >> 5] >> (idx & 31)) & 1u; };
  // one lane's query of a chunk: its kept candidates, candidate count, map point word, angle
  struct QIn {
    uint64_t key[kTopK];
    int nc, mpw;
    float qang;
  };
  auto load_chunk = [&](int c0, QIn& in) {
    const int qi = c0 + lane;
    if (qi < qn) {
      const int q = q0 + qi;
#pragma unroll
      for (int k = 0; k < kTopK; k++) in.key[k] = mw.topk[(int64_t)q * kTopK + k];
      in.nc = mw.ncand[q];
      const Q& qq = queries[q];
      in.mpw = (qq.mp_id & 0x7fffffff) | (qq.blocks ? (int)0x80000000u : 0);
      in.qang = 0.f;
      if constexpr (kF2F) in.qang = qq.last_angle;
    } else {
#pragma unroll
      for (int k = 0; k < kTopK; k++) in.key[k] = kNoKey;
      in.nc = 0;
      in.mpw = 0;
      in.qang = 0.f;
    }
  };
  auto set_bin = [&](int qi, int bin, int idx) {
    if (qi < kResolveLdsQ) {
      s_bin[qi] = (int8_t)bin;
      s_best[qi] = (int16_t)idx;
    } else {
      mw.rot_bin[q0 + qi] = bin;
      mw.best_idx[q0 + qi] = idx;
    }
  };
  QIn nx;
  load_chunk(0, nx);
  for (int c0 = 0; c0 < qn; c0 += 64) {
    const int qi = c0 + lane;
    const bool valid = qi < qn;
    const int q = q0 + qi;
    const QIn in = nx;
    if (c0 + 64 < qn) load_chunk(c0 + 64, nx);  // in flight while this chunk resolves
    const uint64_t* key = in.key;
    const int nc = in.nc, mpw = in.mpw;
    const float qang = in.qang;
    if constexpr (kF2F) {
      if (valid) set_bin(qi, -1, 0);
    }
    const bool qblocks = mpw < 0;
    int start = 0;
    while (start < 64 && c0 + start < qn) {
      const bool act = valid && lane >= start && nc > 0;
      // the kept candidates still unclaimed (claims change only at the commits below)
      uint32_t live = 0;
      if (act) {
#pragma unroll
        for (int k = 0; k < kTopK; k++)
          if (key[k] != kNoKey && !is_claimed(key_idx(key[k]))) live |= 1u << k;
      }
      // -- fixed point of the choices of lanes >= start
      uint64_t b1 = kNoKey, b2 = kNoKey;
      int navail = 0, mine = -1, prev = -2;
      for (int it = 0; it < 64; it++) {
        b1 = kNoKey;
        b2 = kNoKey;
        navail = 0;
#pragma unroll
        for (int k = 0; k < kTopK; k++) {
          if (!((live >> k) & 1u)) continue;
          if (owner[key_idx(key[k])] < lane) continue;
          if (navail == 0) b1 = key[k];
          else if (navail == 1) b2 = key[k];
          navail++;
        }
        // accepted blocking choice -> owner (the lowest such lane wins the keypoint)
        bool acc = b1 != kNoKey && key_dist(b1) <= TH_HIGH;
        if constexpr (!kF2F) {
          if (acc) {
            const int lv1 = s_koct[key_idx(b1)];
            const int d2 = b2 == kNoKey ? 256 : key_dist(b2);
            const int lv2 = b2 == kNoKey ? -1 : s_koct[key_idx(b2)];
            if (lv1 == lv2 && (float)key_dist(b1) > nnratio * (float)d2) acc = false;
          }
        }
        mine = (act && acc && qblocks) ? key_idx(b1) : -1;
        if (!__ballot(mine != prev)) break;
        if (prev >= 0) owner[prev] = INT_MAX;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (mine >= 0) atomicMin(&owner[mine], lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        prev = mine;
      }
      // -- the first lane that needs a rescan ends this round's committed range
      const uint64_t rs = __ballot(act && navail < need && nc > kTopK);
      const int r = rs ? __ffsll((long long)rs) - 1 : 64;
      if (prev >= 0) owner[prev] = INT_MAX;  // committed claims move to claimed[]
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      auto commit = [&](bool doit, uint64_t c1, uint64_t c2) {
        // acceptance (F2F: distance gate; local map: + ratio test, :76-99)
        const bool touched = doit && c1 != kNoKey;
        bool acc = touched && key_dist(c1) <= TH_HIGH;
        if constexpr (!kF2F) {
          if (acc) {
            const int lv1 = s_koct[key_idx(c1)];
            const int d2 = c2 == kNoKey ? 256 : key_dist(c2);
            const int lv2 = c2 == kNoKey ? -1 : s_koct[key_idx(c2)];
            if (lv1 == lv2 && (float)key_dist(c1) > nnratio * (float)d2) acc = false;
          }
        }
        const int idx = touched ? key_idx(c1) : 0;
        nm += __popcll(__ballot(acc));
        // last writer (highest lane) of each keypoint sets mp / blocked
        if (touched) owner[idx] = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (acc) atomicMax(&owner[idx], lane + 1);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (acc && owner[idx] == lane + 1) {
          mp[idx] = mpw & 0x7fffffff;
          blk[idx] = qblocks ? 1 : 0;
        }
        if (acc && qblocks) atomicOr(&claimed[idx >> 5], 1u << (idx & 31));
        if constexpr (kF2F) {
          if (acc && check_ori) {
            float rot = qang - s_kang[idx];
            if (rot < 0.0f) rot += 360.0f;
            const float factor = 1.0f / HISTO_LENGTH;
            int bin = (int)roundf(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            set_bin(qi, bin, idx);
            atomicAdd(&hist[bin], 1);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (touched) owner[idx] = INT_MAX;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      };
      commit(act && lane < r, b1, b2);
      if (r < 64 && c0 + r < qn) {
        // lane r: every kept candidate is taken -> rescan its window with the live claims
        ScanCtx c;
        bool okc;
        const int qr = q0 + c0 + r;
        if constexpr (kF2F) okc = f2f_ctx(queries[qr], poses[f], cam, g, &c);
        else okc = mps_ctx(queries[qr], th, g, &c);
        uint64_t top[kTopK];
        if (okc) scan_query(c, cam, F, claimed, top, lane, g->kp_cap);
        const uint64_t t1 = __shfl(okc ? top[0] : kNoKey, 0, 64);
        const uint64_t t2 = __shfl(okc ? top[1] : kNoKey, 0, 64);
        commit(lane == r, t1, t2);
      }
      start = r + 1;
    }
    (void)q;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if constexpr (kF2F) {
    if (check_ori) {
      // ComputeThreeMaxima (orb_matcher.cpp:1584-1625)
      int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
      for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = hist[i];
        if (s > max1) {
          max3 = max2; max2 = max1; max1 = s;
          ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
          max3 = max2; max2 = s;
          ind3 = ind2; ind2 = i;
        } else if (s > max3) {
          max3 = s;
          ind3 = i;
        }
      }
      if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
      } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
      }
      // SetMapPoint(rotHist[i][j], nullptr) for every entry of a rejected bin (:1441-1450)
      int removed = 0;
      for (int qi = lane; qi < qn; qi += 64) {
        const bool in_lds = qi < kResolveLdsQ;
        const int bin = in_lds ? (int)s_bin[qi] : mw.rot_bin[q0 + qi];
        if (bin >= 0 && bin != ind1 && bin != ind2 && bin != ind3) {
          const int idx = in_lds ? (int)s_best[qi] : mw.best_idx[q0 + qi];
          mp[idx] = -1;
          blk[idx] = 0;
          removed++;
        }
      }
      nm -= wave_sum(removed);
    }
  }
  (void)n;
  if (lane == 0) io.nmatches[f] = nm;
}

void launch_search_frame(const FrameKps& cur, const float* u_right, int64_t ur_stride,
                         const Camera& cam, const OrbGeomDev& g, const F2FQuery* queries,
                         const F2FPose* poses, int n_frames, int max_q, const GridWorkspace& gw,
                         const MatchWorkspace& mw, const MatchIO& io, hipStream_t st) {
  if (max_q > 0)
    SLAMGPU_LAUNCH("search_cand", st, search_cand_kernel<F2FQuery>,
                   dim3((max_q + 4 * (64 / kSearchG) - 1) / (4 * (64 / kSearchG)), n_frames), dim3(256),
                       0, st, cur, u_right, ur_stride, cam, g.dev, queries, poses, 0, gw, mw, io);
  SLAMGPU_LAUNCH("search_resolve", st, search_resolve_kernel<F2FQuery>, dim3(n_frames), dim3(64), 0, st, cur,
                     u_right, ur_stride, cam, g.dev, queries, poses, 0, 0.0f, gw, mw, io);
}

void launch_search_mps(const FrameKps& cur, const float* u_right, int64_t ur_stride,
                       const Camera& cam, const OrbGeomDev& g, const MpsQuery* queries,
                       float nnratio, int th, int n_frames, int max_q, const GridWorkspace& gw,
                       const MatchWorkspace& mw, const MatchIO& io, hipStream_t st) {
  if (max_q > 0)
    SLAMGPU_LAUNCH("search_cand", st, search_cand_kernel<MpsQuery>,
                   dim3((max_q + 4 * (64 / kSearchG) - 1) / (4 * (64 / kSearchG)), n_frames), dim3(256),
                       0, st, cur, u_right, ur_stride, cam, g.dev, queries,
                       (const F2FPose*)nullptr, th, gw, mw, io);
  SLAMGPU_LAUNCH("search_resolve", st, search_resolve_kernel<MpsQuery>, dim3(n_frames), dim3(64), 0, st, cur,
                     u_right, ur_stride, cam, g.dev, queries, (const F2FPose*)nullptr, th,
                     nnratio, gw, mw, io);
}

// ---------------------------------------------------------------------------------------
// VO map points of the previous frame as queries for frame f (Tracker::UpdateLastFrame's
// visual-odometry points, tracker.cpp:695-753, with every stereo keypoint kept): keypoint i of
// frame f-1 with depth > 0 becomes a point at Frame::UnprojectStereo(i) (frame.cpp:594-607).
// Queries keep last-frame keypoint order (block-wide ordered compaction).
__global__ __launch_bounds__(256) void vo_queries_kernel(FrameKps src, const float* __restrict__ depth,
                                                         int64_t depth_stride, Camera cam,
                                                         const F2FPose* __restrict__ poses,
                                                         int blocks, int kp_cap,
                                                         F2FQuery* __restrict__ queries,
                                                         int* __restrict__ q_start,
                                                         int* __restrict__ q_count) {
  __shared__ int wsum[4];
  __shared__ int base;
  const int f = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    q_start[f] = f * kp_cap;
    base = 0;
  }
  if (f == 0) {
    if (tid == 0) q_count[0] = 0;
    return;
  }
  const int s = f - 1;
  const KeyPoint* k = src.kps + s * src.stride;
  const uint8_t* d = src.desc + s * src.stride * 32;
  const int n = src.n[s * src.n_stride];
  const float* z = depth + s * depth_stride;
  const F2FPose& P = poses[s];
  // Twc: Rwc = Rcw^T, Ow = -Rcw^T tcw
  float Rwc[9], Ow[3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Rwc[3 * r + c] = P.Rcw[3 * c + r];
  for (int r = 0; r < 3; r++)
    Ow[r] = -(Rwc[3 * r] * P.tcw[0] + Rwc[3 * r + 1] * P.tcw[1] + Rwc[3 * r + 2] * P.tcw[2]);
  const float invfx = 1.0f / cam.fx, invfy = 1.0f / cam.fy;
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += 256) {
    const int i = c0 + tid;
    const bool ok = i < n && z[i] > 0;
    const int lane = tid & 63, wid = tid >> 6;
    const uint64_t m = __ballot(ok);
    if (lane == 0) wsum[wid] = __popcll(m);
    __syncthreads();
    int pre = base;
    for (int w = 0; w < wid; w++) pre += wsum[w];
    pre += lanes_below(m);
    if (ok) {
      const KeyPoint kp = k[i];
      const float zz = z[i];
      const float x = (kp.x - cam.cx) * zz * invfx;
      const float y = (kp.y - cam.cy) * zz * invfy;
      F2FQuery q;
      const float xc[3] = {x, y, zz};
      for (int r = 0; r < 3; r++) q.xyz[r] = mat3_row(Rwc, r, xc, Ow[r]);
      q.last_angle = kp.angle;
      q.last_octave = kp.octave;
      q.mp_id = i;
      q.blocks = blocks;
      q.pad = 0;
      for (int b = 0; b < 32; b++) q.desc[b] = d[i * 32 + b];
      queries[(int64_t)f * kp_cap + pre] = q;
    }
    __syncthreads();
    if (tid == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (tid == 0) q_count[f] = base;
}

void launch_vo_queries(const FrameKps& src, const float* depth, int64_t depth_stride,
                       const Camera& cam, const F2FPose* poses, int blocks, int kp_cap,
                       F2FQuery* queries, int* q_start, int* q_count, int n_frames,
                       hipStream_t st) {
  SLAMGPU_LAUNCH("vo_queries", st, vo_queries_kernel, dim3(n_frames), dim3(256), 0, st, src, depth,
                 depth_stride, cam, poses, blocks, kp_cap, queries, q_start, q_count);
}

}  // namespace slamgpu
