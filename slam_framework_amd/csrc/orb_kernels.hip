// orb_kernels.hip -- the ORBextractor::Compute hot path as gfx950 kernels, batched over images.
//
// Pipeline for a batch of n images (all levels of all images in flight together):
//   pyr_down      level l from level l-1 (resize INTER_LINEAR 8U)        one launch per level
//                 (batches: pyr_ring_kernel; opt-in pyr_cascade_kernel, one launch for all)
//   fast_cells    per-cell FAST-9 score, threshold fallback, cell NMS    8 cells per wave
//                 (batches: level 0 on a side stream beside the pyramid)
//   octree        DistributeOctTree, exact list / pointer-order semantics one work-group per
//                 image, a wave per level (small launches: a work-group per level)
//   orient_desc   IC_Angle + 7x7-blurred rBRIEF (the blur's row sums on the matrix cores, the
//                 vertical taps at the samples), in ORBextractor::Compute order
//                                                                        16 keypoints per wave
// Reference: src/orb_features/orb_extractor.cpp (citations per kernel). Built with
// -ffp-contract=off; fused multiply-adds are explicit where the reference's Release build fuses.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>
#include <cstdlib>

#include "device_math.h"
#include "timing.h"
#include "orb_geometry.h"
#include "orb_kernels.h"

namespace slamgpu {

__constant__ __attribute__((aligned(16))) int8_t c_pattern[1024] = {
#include "orb_pattern.inc"
};

// ---------------------------------------------------------------------------------------
// Level addressing. Level 0 is the caller's image; levels >= 1 live in the pyramid buffer.
__device__ __forceinline__ const uint8_t* level_ptr(const ImageBatch& b, const OrbGeom* g,
                                                    int img, int level, int* pitch) {
  if (level == 0) {
    *pitch = b.in_pitch;
    return batch_image(b, img);
  }
  *pitch = g->lv[level].pitch;
  return b.pyr + (int64_t)img * g->pyr_bytes + g->lv[level].offset;
}

// ---------------------------------------------------------------------------------------
// pyr_down: ComputePyramid (:1051-1075) -> cv::resize(level l-1, level l, INTER_LINEAR).
// HResizeLinear (int = S[sx]*a0 + S[sx+1]*a1, or S[sx]*2048 from xmax on) then VResizeLinear
// ((b0*(r0>>4))>>16) + ((b1*(r1>>4))>>16) + 2) >> 2.
// A lane owns 4 adjacent output columns and walks a 16-row strip. Each source row is fetched
// once (3 dwords, in prefetched chunks of 4 rows) and its horizontal pass is computed once: the
// 8-byte window starting at sx(x0) (host-checked to hold all 4 columns' pixel pairs) is cut with
// two alignbytes, v_perm turns each column's pixel pair into a u16 pair and v_dot2_u32_u16
// applies (a0, a1). An output row combines the current and previous source rows' results.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot2u(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c,
                                false);
}

#ifndef PYR_CHUNK
#define PYR_CHUNK 2
#endif
constexpr int kPyrStrip = PYR_STRIP;  // output rows per wave
constexpr int kPyrRingStrip = PYR_RING_STRIP;
constexpr int kPyrChunk = PYR_CHUNK;  // source rows fetched per batch
#ifndef PYR_SHORT_STRIP
#define PYR_SHORT_STRIP 4
#endif
constexpr int kPyrShortStrip = PYR_SHORT_STRIP, kPyrShortMaxImages = 16;

// kAligned: the source rows are dword-aligned (every level >= 1 source; level 0 when the caller's
// images and pitch are) -- the instantiation without the byte-gather path needs fewer VGPRs, so
// more waves per SIMD hide the strip's chain of row loads.
// kStrip: output rows per wave -- kPyrStrip for batches; small launches (a single frame) take
// short strips so that more waves share a level and each walks a shorter chain of row loads.
// One wave: output rows [dy0, dy0 + min(kStrip, nlim)) x columns [256 tx, 256 tx + 256) of
// `level`. A strip fetches every source row its rows need, so strips compose in any partition.
// kRing (pyr_ring_kernel): every source row of the strip is first staged in the wave's LDS
// slots (`ring`, D.pyr_slots KiB) by 16-byte buffer-to-LDS loads issued at once -- a strip's
// whole input in flight with no VGPRs held -- and the rows are then read from LDS.
template <bool kAligned, int kStrip, bool kRing = false>
__device__ __forceinline__ void pyr_strip(const ImageBatch& b, const OrbGeom* __restrict__ g,
                                          int level, int img, int tx, int dy0,
                                          const ResizeX* __restrict__ rxt,
                                          const ResizeY* __restrict__ ryt, int nlim = kStrip,
                                          const uint8_t* src_rows = nullptr, int src_row0 = 0,
                                          uint8_t* copy_rows = nullptr, int copy_row0 = 0,
                                          uint8_t* ring = nullptr) {
  const int lane = threadIdx.x & 63;
  const LevelGeom& D = g->lv[level];
  const LevelGeom& S = g->lv[level - 1];
  if (dy0 >= D.h || nlim <= 0) return;
  const int nrows = min(min(kStrip, D.h - dy0), nlim);
  // the strip's row table, one entry per lane (read back with readlane)
  int ry_y0 = 0, ry_y1 = 0, ry_b = 0;
  if (lane < nrows) {
    const ResizeY e = ryt[D.ry_base + dy0 + lane];
    ry_y0 = e.y0;
    ry_y1 = e.y1;
    ry_b = (int)(uint16_t)e.b0 | (int)e.b1 << 16;
  }
  const int sy_lo = __builtin_amdgcn_readlane(ry_y0, 0);
  const int sy_hi = __builtin_amdgcn_readlane(ry_y1, nrows - 1);
  // per-lane column constants
  const int x0 = (tx << 8) + 4 * lane;
  int s0 = 0;
  uint32_t sel[4], A[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int dx = min(x0 + k, D.w - 1);
    const ResizeX e = rxt[D.rx_base + dx];
    if (k == 0) s0 = e.sx;
    const uint32_t bk = (uint32_t)min(e.sx - s0, 6);
    sel[k] = bk | 0x0c00u | (bk + 1) << 16 | 0x0c000000u;  // bytes bk, bk+1 -> u16 lanes
    // coefficients x16 (<= 32768): the dot product yields 16 * r, see the vertical pass
    A[k] = dx < D.xmax ? ((uint32_t)(16 * e.a0) | (uint32_t)(16 * e.a1) << 16) : 32768u;
  }
  const int q0 = s0 >> 2, sh = s0 & 3, qmax = (S.w - 1) >> 2;
  int spitch;
  const uint8_t* src = level_ptr(b, g, img, level - 1, &spitch);
  int srow0 = 0;  // row of src's first row (rows staged elsewhere, e.g. LDS, start later)
  if (src_rows) {
    src = src_rows;
    srow0 = src_row0;
  }
  const bool aligned = kAligned;
  const int qa = min(q0, qmax), qb = min(q0 + 1, qmax), qc = min(q0 + 2, qmax);
  // Source rows in global memory (pyr_down) are read through a buffer descriptor of the source
  // level: the row offset is a scalar, the lane's dword offsets are constants, so a row costs
  // three buffer loads and no address arithmetic (a flat load needs a 64-bit add per lane each).
  spitch = __builtin_amdgcn_readfirstlane(spitch);
  const bool gsrc = src_rows == nullptr;
  const __amdgpu_buffer_rsrc_t srsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)uniform_ptr(src), 0, __builtin_amdgcn_readfirstlane(spitch * S.h), 0x00020000);
  const int oa = 4 * qa, ob = 4 * qb, oc = 4 * qc;
  // kRing: the strip's rows [sy_lo, sy_hi], row r in slot r / rpi at (r % rpi) * lpr * 16; each
  // row's bytes from seg0 (lane 0's first dword, rounded down to 16 bytes) on
  const int lpr = kRing ? D.pyr_lpr : 1, rpi = kRing ? D.pyr_rpi : 1;
  const int inv_rpi = kRing ? D.pyr_inv_rpi : 0;
  const int seg0 = kRing ? __builtin_amdgcn_readfirstlane(oa) & ~15 : 0;
  // the lane's first dword in a staged row; it reads that dword and the next two unclamped (a
  // byte past the row's end has zero weight, as behind the clamped reads' repeated dword)
  const int ra = (oa - seg0) >> 2;
  if constexpr (kRing) {
    const int rl = (lane * D.pyr_inv_lpr) >> 16, cl = lane - rl * lpr;  // row in a slot, chunk
    const int nsrc = sy_hi - sy_lo + 1;
    for (int k = 0; k * rpi < nsrc; k++) {
      // lanes past the slot's rows repeat its last row into the slot's unused tail
      const int r = min(k * rpi + min(rl, rpi - 1), nsrc - 1);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          srsrc, (__attribute__((address_space(3))) void*)(ring + 1024 * k), 16,
          (uint32_t)((sy_lo + r) * spitch + seg0 + 16 * cl), 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the rows have landed
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  auto fetch = [&](int sy, uint32_t (&wv)[3]) {
    const int roff = __builtin_amdgcn_readfirstlane((min(sy, sy_hi) - srow0) * spitch);
    const uint8_t* row = src + roff;  // wave-uniform
    if constexpr (kRing) {
      const int r = min(sy, sy_hi) - sy_lo, slot = (r * inv_rpi) >> 16;  // r < 64: exact
      const uint32_t* rw = reinterpret_cast<const uint32_t*>(
          ring + 1024 * slot + (r - slot * rpi) * lpr * 16);
      const uint32_t* rl_ = rw + (uint32_t)ra;
      wv[0] = rl_[0];
      wv[1] = rl_[1];
      wv[2] = rl_[2];
    } else if (aligned && gsrc) {  // clamped dwords stay inside the row; bytes past sx+1: zero weight
      wv[0] = __builtin_amdgcn_raw_buffer_load_b32(srsrc, oa, roff, 0);
      wv[1] = __builtin_amdgcn_raw_buffer_load_b32(srsrc, ob, roff, 0);
      wv[2] = __builtin_amdgcn_raw_buffer_load_b32(srsrc, oc, roff, 0);
    } else if (aligned) {  // rows staged in LDS by pyr_band_kernel
      const uint32_t* rw = reinterpret_cast<const uint32_t*>(row);
      wv[0] = rw[(uint32_t)qa];
      wv[1] = rw[(uint32_t)qb];
      wv[2] = rw[(uint32_t)qc];
    } else {
#pragma unroll
      for (int i = 0; i < 3; i++) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) v |= (uint32_t)row[min(4 * (q0 + i) + j, S.w - 1)] << (8 * j);
        wv[i] = v;
      }
    }
  };
  uint8_t* dst = b.pyr + (int64_t)img * g->pyr_bytes + D.offset;
  const int dpitch = __builtin_amdgcn_readfirstlane(D.pitch), dw = __builtin_amdgcn_readfirstlane(D.w);
  const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)uniform_ptr(dst), 0, __builtin_amdgcn_readfirstlane(dpitch * D.h), 0x00020000);
  uint32_t cur[kPyrChunk][3], nxt[kPyrChunk][3];
#pragma unroll
  for (int j = 0; j < kPyrChunk; j++) fetch(sy_lo + j, cur[j]);
  // hp / hc: the previous / current source row's horizontal results, already in the vertical
  // pass's operand form (r >> 4) << 8 = (16 r) & ~0xff (once per source row, not per output row)
  uint32_t hp[4] = {0, 0, 0, 0}, hc[4] = {0, 0, 0, 0};
  int nd = 0;  // next strip row to emit
  // one output row from source rows (r0, r1): v = ((b0*(r0>>4))>>16) + ((b1*(r1>>4))>>16) + 2)
  // >> 2 (<= 255 for any coefficient rounding), packed by two u16 pairs, one
  // v_pk_lshrrev_b16 each and one v_perm
  auto emit = [&](const uint32_t (&r0)[4], const uint32_t (&r1)[4], uint32_t b0, uint32_t b1) {
    uint32_t t[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      // v_mul_hi_u32_u24 as such: the operands are < 2^24 by construction (the C helper's masks
      // would be re-applied to the carried row, whose known bits the loop phi loses)
      uint32_t m0, m1;
      asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m0) : "s"(b0), "v"(r0[k]));
      asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m1) : "s"(b1), "v"(r1[k]));
      t[k] = m0 + m1 + 2u;
    }
    typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
    const u16x2_t two = {2, 2};
    const uint32_t p01 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, t[0] | t[1] << 16) >> two);
    const uint32_t p23 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, t[2] | t[3] << 16) >> two);
    const uint32_t packed = __builtin_amdgcn_perm(p23, p01, 0x06040200u);
    const int doff = __builtin_amdgcn_readfirstlane((dy0 + nd) * dpitch);
    uint8_t* drow = dst + doff;
    if (x0 + 4 <= dw) {  // pitch is a multiple of 64
      __builtin_amdgcn_raw_buffer_store_b32(packed, drsrc, x0, doff, 0);
      if (copy_rows)
        *reinterpret_cast<uint32_t*>(copy_rows + (dy0 + nd - copy_row0) * dpitch + x0) = packed;
    } else {
      for (int k = 0; x0 + k < dw; k++) drow[x0 + k] = (uint8_t)(packed >> (8 * k));
      if (copy_rows) {
        uint8_t* crow = copy_rows + (dy0 + nd - copy_row0) * dpitch;
        for (int k = 0; x0 + k < dw; k++) crow[x0 + k] = (uint8_t)(packed >> (8 * k));
      }
    }
  };
  for (int c0 = sy_lo; c0 <= sy_hi; c0 += kPyrChunk) {
    if (c0 + kPyrChunk <= sy_hi) {
#pragma unroll
      for (int j = 0; j < kPyrChunk; j++) fetch(c0 + kPyrChunk + j, nxt[j]);
    }
#pragma unroll
    for (int j = 0; j < kPyrChunk; j++) {
      const int sy = c0 + j;
      if (sy <= sy_hi) {
        const uint32_t W0 = __builtin_amdgcn_alignbyte(cur[j][1], cur[j][0], sh);
        const uint32_t W1 = __builtin_amdgcn_alignbyte(cur[j][2], cur[j][1], sh);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          hp[k] = hc[k];
          hc[k] = dot2u(__builtin_amdgcn_perm(W1, W0, sel[k]), A[k], 0u) & 0xffff00u;  // 16 r < 2^23
        }
        // emit the strip rows whose lower source row is sy (rows are in y1 order)
        while (nd < nrows && __builtin_amdgcn_readlane(ry_y1, nd) == sy) {
          const uint32_t bb = (uint32_t)__builtin_amdgcn_readlane(ry_b, nd);
          // (b * (r >> 4)) >> 16 == mulhi24(b << 8, (r >> 4) << 8) (all operands < 2^24)
          const uint32_t b0 = (bb & 0xffffu) << 8, b1 = (bb >> 16) << 8;
          if (__builtin_amdgcn_readlane(ry_y0, nd) == sy)  // both source rows are row sy
            emit(hc, hc, b0, b1);
          else
            emit(hp, hc, b0, b1);
          nd++;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kPyrChunk; j++)
#pragma unroll
      for (int e = 0; e < 3; e++) cur[j][e] = nxt[j][e];
  }
}


template <bool kAligned, int kStrip>
__global__ __launch_bounds__(256) void pyr_down_kernel(ImageBatch b, const OrbGeom* __restrict__ g,
                                                       int level,
                                                       const ResizeX* __restrict__ rxt,
                                                       const ResizeY* __restrict__ ryt) {
  int img, bx;
  xcd_image_block(&img, &bx);
  const int tiles_x = (g->lv[level].w + 255) >> 8;
  const int tx = bx % tiles_x, ty = bx / tiles_x;
  pyr_strip<kAligned, kStrip>(b, g, level, img, tx, (ty * 4 + wave_id()) * kStrip, rxt, ryt);
}

// pyr_down with each wave's source rows staged in LDS (pyr_strip kRing): g->pyr_ring_slots KiB
// of dynamic LDS per wave
__global__ __launch_bounds__(256) void pyr_ring_kernel(ImageBatch b, const OrbGeom* __restrict__ g,
                                                       int level,
                                                       const ResizeX* __restrict__ rxt,
                                                       const ResizeY* __restrict__ ryt) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_ring[];
  int img, bx;
  xcd_image_block(&img, &bx);
  const int tiles_x = (g->lv[level].w + 255) >> 8;
  const int tx = bx % tiles_x, ty = bx / tiles_x;
  uint8_t* ring = s_ring + 1024 * g->pyr_ring_slots * wave_id();
  pyr_strip<true, kPyrRingStrip, true>(b, g, level, img, tx, (ty * 4 + wave_id()) * kPyrRingStrip,
                                       rxt, ryt, kPyrRingStrip, nullptr, 0, nullptr, 0, ring);
}

// Small launches (the single-frame call): levels 2 .. nlevels - 1 in one launch of row bands
// (g->pyr_band, geometry): band s computes its rows of each level -- its share plus the source
// rows its next level needs, so it reads only rows it wrote itself (halo rows are computed by
// two bands with the same bytes) -- its 16 waves spread over the level's (tile, strip) tasks,
// a work-group barrier between levels. One launch instead of nlevels - 2 dependent ones (~5 us
// each on the call's critical path), with the levels' work still spread over many CUs.
// The band's rows of each level also go to LDS (two buffers of g->pyr_band_lds bytes, rows at
// the level's pitch), where the next level reads them: one global round trip (level 1) per band.
constexpr int kPyrBandWaves = 16;
__global__ __launch_bounds__(64 * kPyrBandWaves) void pyr_band_kernel(
    ImageBatch b, const OrbGeom* __restrict__ g, const ResizeX* __restrict__ rxt,
    const ResizeY* __restrict__ ryt) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_band[];
  const int band = blockIdx.x, img = blockIdx.y, wid = wave_id();
  const int half = g->pyr_band_lds;
  for (int l = 2; l < g->nlevels; l++) {
    const int r0 = g->pyr_band[band][l][0], r1 = g->pyr_band[band][l][1];
    const int tiles = (g->lv[l].w + 255) >> 8;
    const int chunks = (r1 - r0 + kPyrShortStrip - 1) / kPyrShortStrip;
    uint8_t* out = s_band + (l & 1) * half;
    const uint8_t* in = l > 2 ? s_band + ((l - 1) & 1) * half : nullptr;
    const int in_row0 = l > 2 ? g->pyr_band[band][l - 1][0] : 0;
    for (int t = wid; t < tiles * chunks; t += kPyrBandWaves) {
      const int tx = t % tiles, dy0 = r0 + (t / tiles) * kPyrShortStrip;
      pyr_strip<true, kPyrShortStrip>(b, g, l, img, tx, dy0, rxt, ryt, r1 - dy0, in, in_row0, out,
                                      r0);
    }
    __syncthreads();  // this level's rows (LDS) before the next level reads them
  }
}

// Batches: the whole pyramid of one image in one work-group, streamed top to bottom (a cascade
// of line buffers): every barrier step level 1 consumes the next level-0 row and each level
// l >= 2 the rows level l - 1 emitted in the step before, so all levels advance together and a
// level's rows go from LDS to the next level without a global round trip. One launch instead of
// nlevels - 1 dependent ones; level 0 is read once and every level written once (the section
// 8(d) bytes), and the small levels no longer pay a launch and a strip chain each.
// Lanes: task k of level l owns output columns x0 = 8 (k - casc_task_base[l]) .. x0 + 7 as two
// groups of 4 (the pyr_strip column math: an 8-byte window from the group's first source byte,
// v_perm + v_dot2 per column); it keeps the previous / current source row's horizontal results
// in registers (hp, hc) and emits output row y when its lower source row y1 arrives -- from
// (hp, hc), or (hc, hc) where the row table clamps y0 == y1. Every lane of a level takes the
// same steps; the level's first lane publishes the rows emitted so far (P[t & 1][l]).
// The loader wave streams level-0 rows into kCascR0 LDS slots kCascDepth rows ahead (16-byte
// buffer-to-LDS loads; only it issues vector-memory loads, so its vmcnt counts rows).
__global__ __launch_bounds__(1024) void pyr_cascade_kernel(ImageBatch b, const OrbGeom* __restrict__ g,
                                                           const ResizeX* __restrict__ rxt,
                                                           const ResizeY* __restrict__ ryt) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_c[];
  const int img = blockIdx.x, tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int nl = g->nlevels, nw = g->casc_waves, T = g->casc_steps;
  const int H0 = g->lv[0].h;
  const int ry0 = g->lv[1].ry_base, nry = g->lv[nl - 1].ry_base + g->lv[nl - 1].h - ry0;
  uint2* s_ry = reinterpret_cast<uint2*>(s_c + g->casc_ry_off);
  int* s_p = reinterpret_cast<int*>(s_c + g->casc_p_off);
  for (int i = tid; i < nry; i += blockDim.x) {
    const ResizeY e = ryt[ry0 + i];
    s_ry[i] = make_uint2((uint32_t)e.y1 | (uint32_t)(e.y0 == e.y1) << 16,
                         (uint32_t)(uint16_t)e.b0 | (uint32_t)(uint16_t)e.b1 << 16);
  }
  if (tid < 2 * kMaxLevels) s_p[tid] = 0;
  const bool loader = wid == nw;
  // ---- the loader: level-0 row r -> slot r % kCascR0, 16-byte chunks, ipr instructions per row
  const int chunks0 = (g->lv[0].w + 15) >> 4, ipr = (chunks0 + 63) >> 6;
  uint8_t* ring0 = s_c + g->casc_ring_off[0];
  const int stride0 = g->casc_ring_stride[0];
  const int pitch0 = __builtin_amdgcn_readfirstlane(b.in_pitch);
  const __amdgpu_buffer_rsrc_t rsrc0 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)uniform_ptr(batch_image(b, img)), 0, __builtin_amdgcn_readfirstlane(pitch0 * H0),
      0x00020000);
  auto issue = [&](int r) {
    uint8_t* dst = ring0 + (r % kCascR0) * stride0;
    for (int k = 0; k < ipr; k++)
      if (64 * k + lane < chunks0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsrc0, (__attribute__((address_space(3))) void*)(dst + 1024 * k), 16,
            (uint32_t)(r * pitch0 + 16 * (64 * k + lane)), 0, 0, 0);
  };
  // wait until row r has landed, rows up to min(r + kCascDepth - 1, H0 - 1) issued
  auto wait_row = [&](int r) {
    if (r + kCascDepth - 1 < H0) {
      if (ipr == 1) __builtin_amdgcn_s_waitcnt(0x0F70 | (kCascDepth - 1));
      else __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * (kCascDepth - 1)));
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
  };
  if (loader) {
    for (int r = 0; r < kCascDepth && r < H0; r++) issue(r);
    wait_row(0);
  }
  // ---- a compute lane's level, columns and constants
  const int task = wid * 64 + lane;
  int lvl = 0;
  if (!loader)
    for (int l = 1; l < nl; l++)
      if (task >= g->casc_task_base[l] && task < g->casc_task_base[l + 1]) lvl = l;
  const LevelGeom& D = g->lv[lvl > 0 ? lvl : 1];
  const int x0 = 8 * (task - g->casc_task_base[lvl > 0 ? lvl : 1]);
  const int Hl = D.h, Wl = D.w;
  uint32_t sel[8], A[8];
  int qo[2], sh[2];
#pragma unroll
  for (int gi = 0; gi < 2; gi++) {
    int s0 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int dx = min(x0 + 4 * gi + k, Wl - 1);
      const ResizeX e = rxt[D.rx_base + dx];
      if (k == 0) s0 = e.sx;
      const uint32_t bk = (uint32_t)min(e.sx - s0, 6);
      sel[4 * gi + k] = bk | 0x0c00u | (bk + 1) << 16 | 0x0c000000u;
      A[4 * gi + k] = dx < D.xmax ? ((uint32_t)(16 * e.a0) | (uint32_t)(16 * e.a1) << 16) : 32768u;
    }
    qo[gi] = 4 * (s0 >> 2);
    sh[gi] = s0 & 3;
  }
  // source ring (level lvl - 1) and destination ring (level lvl; none for the last level)
  const int sl = lvl > 0 ? lvl - 1 : 0;
  const uint8_t* sring = s_c + g->casc_ring_off[sl];
  const int sstride = g->casc_ring_stride[sl], smod = sl == 0 ? kCascR0 : kCascSlots;
  const bool to_lds = lvl > 0 && lvl + 1 < nl;
  uint8_t* dring = s_c + g->casc_ring_off[to_lds ? lvl : 0];
  const int dstride = g->casc_ring_stride[to_lds ? lvl : 0];
  uint8_t* dst = b.pyr + (int64_t)img * g->pyr_bytes + D.offset;
  const int dpitch = D.pitch;
  const uint2* rytab = s_ry + (D.ry_base - ry0);
  const bool leader = lvl > 0 && task == g->casc_task_base[lvl];
  const bool full = x0 + 8 <= Wl;
  __syncthreads();  // row tables, counters and level-0 row 0 in LDS
  int ns = 0, nd = 0;
  uint2 cur = rytab[0];
  uint32_t hp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t = 0; t < T; t++) {
    if (loader) {
      if (t + kCascDepth < H0) issue(t + kCascDepth);
    } else if (lvl > 0) {
      const int avail = lvl == 1 ? min(t + 1, H0) : s_p[((t + 1) & 1) * kMaxLevels + lvl - 1];
      while (ns < avail) {
        const uint8_t* row = sring + (ns & (smod - 1)) * sstride;
#pragma unroll
        for (int gi = 0; gi < 2; gi++) {
          const uint32_t* rw = reinterpret_cast<const uint32_t*>(row + qo[gi]);
          const uint32_t d0 = rw[0], d1 = rw[1], d2 = rw[2];
          const uint32_t W0 = __builtin_amdgcn_alignbyte(d1, d0, sh[gi]);
          const uint32_t W1 = __builtin_amdgcn_alignbyte(d2, d1, sh[gi]);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            hp[4 * gi + k] = hc[4 * gi + k];
            hc[4 * gi + k] =
                dot2u(__builtin_amdgcn_perm(W1, W0, sel[4 * gi + k]), A[4 * gi + k], 0u) & 0xffff00u;
          }
        }
        while (nd < Hl && (int)(cur.x & 0xffffu) == ns) {
          const uint32_t b0 = (cur.y & 0xffffu) << 8, b1 = (cur.y >> 16) << 8;
          if (cur.x >> 16) {  // y0 == y1 (the last rows): both source rows are this one
#pragma unroll
            for (int k = 0; k < 8; k++) hp[k] = hc[k];
          }
          uint32_t pk[2];
#pragma unroll
          for (int gi = 0; gi < 2; gi++) {
            uint32_t tt[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const uint32_t r0 = hp[4 * gi + k];
              uint32_t m0, m1;
              asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m0) : "v"(b0), "v"(r0));
              asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m1) : "v"(b1), "v"(hc[4 * gi + k]));
              tt[k] = m0 + m1 + 2u;
            }
            typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
            const u16x2_t two = {2, 2};
            const uint32_t p01 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, tt[0] | tt[1] << 16) >> two);
            const uint32_t p23 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, tt[2] | tt[3] << 16) >> two);
            pk[gi] = __builtin_amdgcn_perm(p23, p01, 0x06040200u);
          }
          if (to_lds)
            *reinterpret_cast<uint2*>(dring + ((uint32_t)nd % kCascSlots) * dstride + x0) =
                make_uint2(pk[0], pk[1]);
          uint8_t* drow = dst + (uint32_t)(nd * dpitch);
          if (full) {
            *reinterpret_cast<uint2*>(drow + x0) = make_uint2(pk[0], pk[1]);
          } else {
            for (int k = 0; x0 + k < Wl; k++) drow[x0 + k] = (uint8_t)(pk[k >> 2] >> (8 * (k & 3)));
          }
          nd++;
          cur = rytab[min(nd, Hl - 1)];
        }
        ns++;
      }
      if (leader) s_p[(t & 1) * kMaxLevels + lvl] = nd;
    }
    if (loader) wait_row(t + 1);
    // a work-group barrier that orders LDS only: __syncthreads() (or an LDS-scope fence, as the
    // loader's buffer-to-LDS loads are LDS writes counted by vmcnt) would make every wave wait
    // for its global stores of the step (vmcnt(0)) -- an HBM write latency per step
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int reflect101(int i, int n) {  // cv::BORDER_REFLECT_101, |overshoot| < n
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

// ---------------------------------------------------------------------------------------
// fast_cells: ComputeKeyPointsOctTree cell loop (:730-770) with cv::FAST(th, nonmax=true).
// For a FAST corner the cornerScore<16> value does not depend on the threshold it was found
// at: score = s - 1 with s = max over the 16 contiguous 9-arcs of min |I_ring - I_center|
// (same sign along the arc), and p is a corner at threshold t iff s > t. So one s-map per cell
// serves both passes: NMS at iniTh, and again at minTh if nothing survived (:753-757).
// NMS is strict '>' against the 8 neighbours' scores at that t, zero outside the detect area
// (cell-local, as cv::FAST sees only the cell view). Survivors are written in row-major order.
#ifndef FAST_CELL_WAVES
#define FAST_CELL_WAVES 1
#endif
constexpr int kCellWaves = FAST_CELL_WAVES;  // waves per work-group

// ---- byte-parallel comparisons (r5). v_lerp_u8 adds two bytes and a rounding bit per byte and
// halves, with no carry between bytes: lerp(x, ~y, r) = floor((x - y + 255 + r) / 2) encodes
// x - y in [-255, 255] as a byte, and a second lerp against a constant C sets bit 7 of a byte
// exactly when that byte is >= 256 - C. So "x - y >= t + 1" is bit 7 of two lerps for four
// pixels at once (t + r even makes the halving exact: r = t & 1, K = 128 + (t + r) / 2):
//   bright_a  (a - v >= t + 1) = bit 7 of lerp(lerp(a, ~v, r), 256 - K, 0)
//   !dark_a   (v - a <= t)     = bit 7 of lerp(lerp(~v, a, 1 - r), K, 0)
// (lerp(~v, a, 1 - r) = 255 - lerp(v, ~a, r), so the dark test needs no ~a.)
__device__ __forceinline__ uint32_t lerp_u8(uint32_t a, uint32_t b, uint32_t r) {
  return __builtin_amdgcn_lerp(a, b, r);
}

struct FastTh {        // one pass's threshold constants (wave-uniform)
  int th;              // clamped to [0, 255] as cv::FAST does
  uint32_t r, rn;      // rounding bytes r and 1 - r
  uint32_t cb, cd;     // second-level constants 256 - K and K
};
__device__ __forceinline__ FastTh fast_th(int th) {
  FastTh f;
  f.th = min(max(th, 0), 255);
  const int r = f.th & 1, K = 128 + ((f.th + r) >> 1);  // K = 256 at t = 255: no corner
  f.r = (uint32_t)r * 0x01010101u;
  f.rn = (uint32_t)(r ^ 1) * 0x01010101u;
  f.cb = (uint32_t)(256 - K) * 0x01010101u;
  f.cd = (uint32_t)min(K, 255) * 0x01010101u;
  return f;
}

// The FAST pre-test of 4 pixels (one tile dword c, its row neighbours cm / cp and the dwords 3
// rows below / above): a pixel can be a corner only if both opposite ring pairs (0, 8) and
// (4, 12) hold a pixel darker than v - t (or both a pixel brighter than v + t) -- every 9-arc of
// the ring contains one pixel of each pair. Bit 7 of each byte = that pixel survives.
__device__ __forceinline__ uint32_t fast_pretest4(uint32_t c, uint32_t cm, uint32_t cp,
                                                  uint32_t p0, uint32_t p8, const FastTh& f) {
  const uint32_t a4 = __builtin_amdgcn_alignbyte(cp, c, 3);   // (x + 3, y)
  const uint32_t a12 = __builtin_amdgcn_alignbyte(c, cm, 1);  // (x - 3, y)
  const uint32_t nv = ~c;
  auto B = [&](uint32_t a) { return lerp_u8(lerp_u8(a, nv, f.r), f.cb, 0u); };
  auto G = [&](uint32_t a) { return lerp_u8(lerp_u8(nv, a, f.rn), f.cd, 0u); };
  const uint32_t bright = (B(p0) | B(p8)) & (B(a4) | B(a12));
  const uint32_t ndark = (G(p0) & G(p8)) | (G(a4) & G(a12));
  return bright | ~ndark;  // bit 7 of each byte (other bits: don't care)
}

// Exact FAST-9 strength s of one pixel (see above) on the 16 ring differences as f16 pairs
// x = (v - p, p - v): as f16 bit patterns the bytes v and p are the denormals v 2^-24 and
// p 2^-24, so one v_pk_add_f16 (negation per half, the byte broadcast by op_sel_hi) forms both
// differences exactly, and v_pk_minimum3 / v_pk_maximum3 evaluate the min-over-9-arcs /
// max-over-arcs network three operands at a time (16 + 16 + 8 instructions for both signs).
// A non-negative result's bit pattern is the integer s; a negative one (sign bit) means s < 0.
__device__ __forceinline__ uint32_t pk_minimum3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint32_t pk_maximum3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
template <int ts>
__device__ __forceinline__ int fast_score(const uint8_t* w) {  // w: top-left of the 7x7 window
  constexpr int offs[16] = {3 + 6 * ts, 4 + 6 * ts, 5 + 5 * ts, 6 + 4 * ts, 6 + 3 * ts, 6 + 2 * ts,
                            5 + ts,     4,          3,          2,          1 + ts,     2 * ts,
                            3 * ts,     4 * ts,     1 + 5 * ts, 2 + 6 * ts};
  const uint32_t v = w[3 + 3 * ts];
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t p = w[offs[k]];
    asm("v_pk_add_f16 %0, %1, %2 op_sel_hi:[0,0] neg_lo:[1,0] neg_hi:[0,1]"
        : "=v"(x[k]) : "v"(p), "v"(v));
  }
  uint32_t m3[16], m9[16];
#pragma unroll
  for (int k = 0; k < 16; k++) m3[k] = pk_minimum3(x[k], x[(k + 1) & 15], x[(k + 2) & 15]);
#pragma unroll
  for (int k = 0; k < 16; k++) m9[k] = pk_minimum3(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]);
  const uint32_t u0 = pk_maximum3(pk_maximum3(m9[0], m9[1], m9[2]), pk_maximum3(m9[3], m9[4], m9[5]),
                                  pk_maximum3(m9[6], m9[7], m9[8]));
  const uint32_t u1 = pk_maximum3(pk_maximum3(m9[9], m9[10], m9[11]),
                                  pk_maximum3(m9[12], m9[13], m9[14]), m9[15]);
  const uint32_t best = pk_maximum3(u0, u1, u1);
  return max(max((int)(int16_t)(best & 0xffffu), (int)(int16_t)(best >> 16)), 0);
}

// A wave runs kCellsPerWave consecutive cells of one image.
constexpr int kCellsPerWave = FAST_CELLS_PER_WAVE;  // orb_geometry.h (4: 0.687 ms, 8: 0.670)
static_assert(kCellsPerWave == kCellGroup, "a wave's cells are one key group (orb_geometry.h)");

// ceil(4096 / n) for n = 1..32 (the pre-test's lane -> (row, dword) split by a multiply)
__constant__ int16_t c_inv4096[33] = {
    0,   4096, 2048, 1366, 1024, 820, 683, 586, 512, 456, 410, 373, 342, 316, 293, 274, 256,
    241, 228,  216,  205,  196,  187, 179, 171, 164, 158, 152, 147, 142, 137, 133, 128};

struct CellView {
  int level, ini_x, ini_y, vw, vh, pitch, ax, off, nd;
  const uint8_t* base;
  bool aligned;
};

template <int kAlign = 4>
__device__ __forceinline__ CellView cell_view(const ImageBatch& b, const OrbGeom* g, int img,
                                              int in_pitch, const uint4& d) {
  CellView v;
  v.level = (int)(int16_t)(d.x & 0xffff);
  v.ini_x = (int)(int16_t)(d.x >> 16);
  v.ini_y = (int)(int16_t)(d.y & 0xffff);
  v.vw = (int)(int16_t)(d.y >> 16);
  v.vh = (int)(int16_t)(d.z & 0xffff);
  const LevelGeom& L = g->lv[v.level];
  v.pitch = v.level == 0 ? in_pitch : L.pitch;
  v.base = v.level == 0 ? batch_image(b, img) : b.pyr + (int64_t)img * g->pyr_bytes + L.offset;
  v.ax = v.ini_x & -kAlign;
  v.off = v.ini_x - v.ax;
  v.nd = (v.vw + v.off + 3) >> 2;  // dwords per tile row (<= 18)
  v.aligned = (((uintptr_t)v.base | (uintptr_t)v.pitch) & 3) == 0;
  return v;
}

__device__ __forceinline__ uint4 readlane4(const uint4& x, int j) {
  return make_uint4(__builtin_amdgcn_readlane(x.x, j), __builtin_amdgcn_readlane(x.y, j),
                    __builtin_amdgcn_readlane(x.z, j), __builtin_amdgcn_readlane(x.w, j));
}

// GLDS: every cell view of the launch is 16-byte aligned (pyramid levels, and a caller image
// with 16-byte base/pitch/stride): tiles go HBM -> LDS by global_load_lds_dwordx4 (no VGPRs, one
// instruction per 1 KiB = 1024/TS tile rows). Otherwise dword loads staged through registers
// (4-byte aligned) or a byte copy.
template <int TS, bool GLDS>
__global__ __launch_bounds__(64 * kCellWaves, 1) void fast_cells_kernel(ImageBatch b,
                                                         const OrbGeom* __restrict__ g,
                                                         const CellDesc* __restrict__ cells,
                                                         uint32_t* __restrict__ cell_keys,
                                                         int* __restrict__ cell_count,
                                                         uint32_t* __restrict__ err,
                                                         int cell_lo, int cell_hi) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_fast[];
  const int wid = wave_id(), lane = threadIdx.x & 63;
  constexpr int kTileStride = TS, kScoreStride = TS;  // == g->fast_tile_stride
  constexpr int kLpr = TS / 4, kRps = 64 / kLpr;        // tile copy: lanes per row, rows per step
  constexpr int kTileSteps = (70 + kRps - 1) / kRps;    // cell views are <= 70 rows
  constexpr int kGLpr = TS / 16, kGRows = 64 / kGLpr;   // glds: lanes per row, rows per instr.
  constexpr int kGSteps = (70 + kGRows - 1) / kGRows;
  constexpr int kAlign = GLDS ? 16 : 4;
  int img, bx;
  xcd_image_block(&img, &bx);
  const int ncells = g->cells_per_image;  // per-image stride; this launch runs [cell_lo, cell_hi)
  const int c0 = cell_lo + (bx * kCellWaves + wid) * kCellsPerWave;
  if (c0 >= cell_hi) return;
  const int nc = min(kCellsPerWave, cell_hi - c0);
  const uint4 my_desc = lane < nc ? reinterpret_cast<const uint4*>(cells)[c0 + lane]
                                  : make_uint4(0, 0, 0, 0);
  const int in_pitch = __builtin_amdgcn_readfirstlane(b.in_pitch);
  // configuration scalars read once (the stores below would otherwise make the compiler reload
  // them inside the NMS loop, each behind a scalar-load wait)
  const int cell_cap = __builtin_amdgcn_readfirstlane(g->cell_cap);
  const FastTh th_ini = fast_th(__builtin_amdgcn_readfirstlane(g->ini_th));
  const FastTh th_min = fast_th(__builtin_amdgcn_readfirstlane(g->min_th));
  const int tile_bytes = (kTileStride * g->fast_tile_rows + 15) & ~15;
  uint8_t* tile0 = s_fast + wid * g->fast_lds_per_wave;
  uint8_t* sc = tile0 + tile_bytes;
  const int tile_rows = __builtin_amdgcn_readfirstlane(g->fast_tile_rows);
  uint16_t* cand =
      reinterpret_cast<uint16_t*>(sc + ((kScoreStride * g->fast_score_rows + 15) & ~15));
  {  // the score map starts zero; each FAST pass leaves it zero again
    const int zb = (kScoreStride * g->fast_score_rows + 15) & ~15;
    for (int o = 4 * lane; o < zb; o += 256) *reinterpret_cast<uint32_t*>(sc + o) = 0u;
  }

  // ---- tile prefetch: aligned dwords covering [ini_x & ~3, ini_x + vw) x [ini_y, ini_y + vh)
  // into registers, lane = (row within a step, dword): each element is a scalar row base plus a
  // per-lane offset. Tile column c = image column ax + c.
  const int plr = lane / kLpr, pld = lane % kLpr;
  uint32_t tv[GLDS ? 1 : kTileSteps];
  int tn = 0;
  auto prefetch = [&](const CellView& v) {
    tn = v.aligned ? (v.vh + kRps - 1) / kRps : 0;  // wave-uniform
    const uint8_t* src = v.base + (int64_t)v.ini_y * v.pitch + v.ax;
    const int goff = __umul24(plr, v.pitch) + 4 * pld;
    const bool dok = pld < v.nd;
#pragma unroll
    for (int k = 0; k < kTileSteps; k++)
      if (k < tn && dok && k * kRps + plr < v.vh)
        tv[k] = *reinterpret_cast<const uint32_t*>(src + (int64_t)(k * kRps) * v.pitch + goff);
  };
  // glds: tile row r of the view = image row ini_y + min(r, vh - 1) (rows past the view repeat
  // its last row; they are never read), 16-byte chunk lane % kGLpr of [ax, ax + TS). The view
  // ends >= 16 rows above the level's last row, so the TS-byte row reads stay in the image.
  // The row offsets are 32-bit lane offsets from one scalar base (saddr form).
  const int glr = lane / kGLpr, glc = 16 * (lane % kGLpr);
  auto issue = [&](const CellView& v, uint8_t* buf) {
    const uint8_t* src = v.base + (int64_t)v.ini_y * v.pitch + v.ax;  // wave-uniform
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(src);  // 32-bit lane offsets, no 64-bit adds
    const int n = (v.vh + kGRows - 1) / kGRows;
#pragma unroll
    for (int k = 0; k < kGSteps; k++)
      if (k < n && k * kGRows + glr < tile_rows)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(buf + 1024 * k), 16,
            (uint32_t)(min(k * kGRows + glr, v.vh - 1) * v.pitch + glc), 0, 0, 0);
  };
  CellView nxt = cell_view<kAlign>(b, g, img, in_pitch, readlane4(my_desc, 0));
  if constexpr (!GLDS) {
    if (nxt.vh > 0) prefetch(nxt);
  }

  // the group's keys, contiguous from its first cell's slot (kCellGroup == kCellsPerWave and
  // c0 is group-aligned: launch boundaries are level boundaries, padded to kCellGroup)
  uint32_t* const grp_keys = cell_keys + ((int64_t)img * ncells + c0) * cell_cap;
  int gfill = 0;
  for (int ci = 0; ci < nc; ci++) {
    const CellView v = nxt;
    const int64_t slot = (int64_t)img * ncells + c0 + ci;
    uint8_t* tile = tile0;
    if constexpr (GLDS) {
      // one tile buffer: this cell's rows are loaded now (the previous cell's tile reads have
      // all returned), other waves hide the latency
      if (ci + 1 < nc) nxt = cell_view<kAlign>(b, g, img, in_pitch, readlane4(my_desc, ci + 1));
      if (v.vh == 0) {  // empty cell (:737, :745)
        if (lane == 0) cell_count[slot] = 0;
        continue;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      issue(v, tile0);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    } else {
    if (v.vh == 0) {  // empty cell (:737, :745)
      if (lane == 0) cell_count[slot] = 0;
      if (ci + 1 < nc) {
        nxt = cell_view<kAlign>(b, g, img, in_pitch, readlane4(my_desc, ci + 1));
        if (nxt.vh > 0) prefetch(nxt);
      }
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();  // previous cell's LDS reads are done
    if (v.aligned) {
      const bool dok = pld < v.nd;
#pragma unroll
      for (int k = 0; k < kTileSteps; k++)
        if (k < tn && dok && k * kRps + plr < v.vh)
          *reinterpret_cast<uint32_t*>(tile + (k * kRps + plr) * TS + 4 * pld) = tv[k];
    } else {  // caller image with an odd pitch/base: byte copy
      for (int r = 0; r < v.vh; r++)
        for (int x = lane; x < v.vw + v.off; x += 64)
          tile[r * kTileStride + x] = v.base[(int64_t)(v.ini_y + r) * v.pitch + v.ax + x];
    }
    if (ci + 1 < nc) {  // next cell's loads fly while this one is processed
      nxt = cell_view<kAlign>(b, g, img, in_pitch, readlane4(my_desc, ci + 1));
      if (nxt.vh > 0) prefetch(nxt);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    }
    const int off = v.off;
    const int dh = v.vh - 6, dw = v.vw - 6;  // detect area [3, vh-3) x [3, vw-3)
    // ---- score map: rows -1 .. dh of the detect area, zeroed before each pass's scores (a zero
    // frame around the detect area lets the NMS read 3x3 neighbourhoods without bounds checks);
    // sc1 = row 0. Until then the pass keeps its prefilter records in the same bytes.
    uint8_t* sc1 = sc + kScoreStride;
    uint32_t* const recs = reinterpret_cast<uint32_t*>(sc);
    // ---- one FAST pass at threshold th: pre-test every detect pixel (4 pixels, one tile dword,
    // per lane), exact score of the survivors into the score map, NMS at th, survivors out in
    // row-major order.
    // Detect pixel (rr, col): tile row rr + 3, tile column col in [off + 3, off + 3 + dw).
    // Lane -> (row lr of a step, dword Q): rows_per rows of nq dwords per step.
    const int q_lo = (off + 3) >> 2, q_hi = (off + 2 + dw) >> 2;
    const int nq = q_hi - q_lo + 1;
    const int inv_nq = c_inv4096[nq];  // lane / nq = (lane * inv_nq) >> 12 (exact for lane < 64)
    const int rows_per = (64 * inv_nq) >> 12;
    const int lr = (lane * inv_nq) >> 12, Q = q_lo + (lane - lr * nq);
    const int blo = max(0, off + 3 - 4 * Q), bhi = min(4, off + 3 + dw - 4 * Q);
    const uint32_t vmask = lr < rows_per
        ? (uint32_t)(0x80808080ull >> (32 - 8 * bhi)) & (uint32_t)(0x80808080ull << (8 * blo))
        : 0u;
    const uint8_t* trow = tile + (lr + 3) * kTileStride + 4 * Q;  // this lane's dword, step 0
    uint32_t* out = grp_keys + gfill;  // this cell's survivors follow the group's earlier cells
    auto fast_pass = [&](const FastTh& f) -> int {
      if (f.th >= 255) return 0;  // FAST at 255: no pixel differs by more
      // pre-test: a lane with any surviving pixel appends one record -- its survivor flags (bit
      // 7 of each byte) | lane | step << 8 -- so records come out in row-major order
      int nrec = 0;
      auto step = [&](int it, int r0, auto tail_case) {
        constexpr bool kTail = decltype(tail_case)::value;
        const uint8_t* row = trow + r0 * kTileStride;
        auto rd = [&](int o) { return *reinterpret_cast<const uint32_t*>(row + o); };
        uint32_t m = fast_pretest4(rd(0), rd(-4), rd(4), rd(3 * kTileStride),
                                   rd(-3 * kTileStride), f) & vmask;
        if (kTail && r0 + lr >= dh) m = 0;
        const uint64_t act = __ballot(m != 0);
        if (m) recs[nrec + lanes_below(act)] = m | (uint32_t)lane | (uint32_t)it << 8;
        nrec += __popcll(act);
      };
      int it = 0, r0 = 0;
      for (; r0 + rows_per <= dh; r0 += rows_per, it++) step(it, r0, std::false_type{});
      if (r0 < dh) step(it, r0, std::true_type{});
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // records -> one candidate per surviving pixel, row-major (exclusive prefix of the
      // per-record counts via 3 ballots)
      int ncand = 0;
      for (int i0 = 0; i0 < nrec; i0 += 64) {
        const int i = i0 + lane;
        const uint32_t rec = i < nrec ? recs[i] : 0u;
        const uint32_t fl = rec & 0x80808080u;
        const int cnt = __popc(fl);
        const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2), b2 = __ballot(cnt & 4);
        int pos = ncand + lanes_below(b0) + 2 * lanes_below(b1) + 4 * lanes_below(b2);
        const int ln = (int)(rec & 63u), rit = (int)((rec >> 8) & 127u);
        const int lr2 = (ln * inv_nq) >> 12;
        const uint32_t pix0 =
            (uint32_t)((rit * rows_per + lr2) * kScoreStride + 4 * (q_lo + ln - lr2 * nq));
#pragma unroll
        for (int bb = 0; bb < 4; bb++)
          if (fl & (0x80u << (8 * bb))) cand[pos++] = (uint16_t)(pix0 + bb);
        ncand += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // the map is zero but for the records just read (it is zeroed once per wave and every
      // pass clears what it wrote): clear them
      for (int i = lane; i < nrec; i += 64) recs[i] = 0u;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // exact FAST score of the survivors (window top-left: tile (r, cc - 3) = tile + pix - 3)
      for (int i = lane; i < ncand; i += 64) {
        const int pix = cand[i];
        sc1[pix] = (uint8_t)fast_score<TS>(tile + pix - 3);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // NMS at th: cv::FAST keeps p iff s - 1 > ns for all 8 neighbours, ns = (q > th ? q - 1 :
      // 0), zero outside the detect area. With Q = max of the 8 neighbours' s that is
      //   s > th  &&  s >= 2  &&  Q < max(s, th + 1),
      // and a neighbour this pass did not score has s <= th < s_p (the pre-test is necessary),
      // so it cannot change the test.
      const int th = f.th;
      int count = 0;
      for (int i0 = 0; i0 < ncand; i0 += 64) {
        const int i = i0 + lane;
        bool keep = false;
        int sv = 0, r = 0, cc = 0;
        if (i < ncand) {
          const int pix = cand[i];
          r = pix / kScoreStride;
          cc = pix - r * kScoreStride;
          const uint8_t* nb = sc1 + pix - kScoreStride - 1;  // (r - 1, cc - 1)
          const int al = (int)((uintptr_t)nb & 3);
          const uint32_t* nw = reinterpret_cast<const uint32_t*>(nb - al);
          constexpr int kW = kScoreStride / 4;
          const uint32_t rA = __builtin_amdgcn_alignbyte(nw[1], nw[0], al);
          const uint32_t rB = __builtin_amdgcn_alignbyte(nw[kW + 1], nw[kW], al);
          const uint32_t rC = __builtin_amdgcn_alignbyte(nw[2 * kW + 1], nw[2 * kW], al);
          sv = (rB >> 8) & 255;
          const int q = max(max(max3((int)(rA & 255), (int)((rA >> 8) & 255), (int)((rA >> 16) & 255)),
                                max((int)(rB & 255), (int)((rB >> 16) & 255))),
                            max3((int)(rC & 255), (int)((rC >> 8) & 255), (int)((rC >> 16) & 255)));
          keep = sv > th && sv >= 2 && q < max(sv, th + 1);
        }
        const uint64_t mk = __ballot(keep);
        if (keep) {
          const int pos = count + lanes_below(mk);
          if (pos < cell_cap) out[pos] = pack_key(v.ax + cc - kMinBorder, v.ini_y + 3 + r - kMinBorder, sv - 1);
        }
        count += __popcll(mk);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int i = lane; i < ncand; i += 64) sc1[cand[i]] = 0;  // the map back to zero
      return count;
    };
    // FAST at iniTh; the reference re-runs the whole cell at minTh when the iniTh output (after
    // NMS) is empty (:753-757)
    int count = fast_pass(th_ini);
    if (count == 0) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      count = fast_pass(th_min);
    }
    if (count > cell_cap) {
      if (lane == 0) atomicOr(err, kErrCellOverflow);
      count = cell_cap;
    }
    if (lane == 0) cell_count[slot] = count;
    gfill += count;
  }
}
// ---------------------------------------------------------------------------------------
// octree: DistributeOctTree (:480-704), one 256-thread workgroup per (image, level).
// The std::list is kept as an array in list order and rebuilt every pass; node keys are
// contiguous index ranges that DivideNode splits by a stable 4-way partition (ballot ranks)
// into the other half of a ping-pong key buffer. Creation sequence numbers stand in for the
// heap addresses the reference sorts by (:625); see SURVEY.md Appendix B.1.
//   outer pass (:528-613): every node with > 1 key is divided, children are pushed to the front
//     in list order (n1..n4), so the new list is [children in reverse push order] + [nodes
//     with one key, in order];
//   inner loop (:615-676): the vPrev nodes are divided in descending (size, seq) order and the
//     loop stops once the list reaches N -- done speculatively in parallel, then cut with a
//     prefix sum; processed nodes leave the list and their children go to the front.
constexpr int kOctThreads = 256;
constexpr int kOctWaves = kOctThreads / 64;
constexpr int kOctCap = 2048;  // max list length / inner-loop set size held in LDS

struct OctShared {
  uint64_t sortk[kOctCap];
  int a[kOctCap];
  int b[kOctCap];
  int c[kOctCap];
  int wsum[16];  // per-wave totals (up to 16 waves)
  int bucket[64 + 1];
  int m, seq_next, mode, nexp, finish, ktotal, total;
};

// Block-wide exclusive scan of v (one value per thread of kThr); returns prefix, *total the sum.
template <int kThr>
__device__ __forceinline__ int block_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wid = wave_id();
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kThr / 64; w++) {
    const int s = wsum[w];
    pre += (w < wid) ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// Exclusive scan of arr[0..n) in place (n <= kOctCap) by kThr threads; returns the total.
template <int kThr>
__device__ int block_scan_array(int* arr, int n, int* wsum) {
  constexpr int per = kOctCap / kThr;
  const int base = threadIdx.x * per;
  int loc[per];
  int s = 0;
#pragma unroll
  for (int i = 0; i < per; i++) {
    loc[i] = (base + i < n) ? arr[base + i] : 0;
    s += loc[i];
  }
  int total;
  int pre = block_scan<kThr>(s, wsum, &total);
#pragma unroll
  for (int i = 0; i < per; i++) {
    if (base + i < n) arr[base + i] = pre;
    pre += loc[i];
  }
  __syncthreads();
  return total;
}

// DivideNode (:422-478) of `nd` by one wave: stable partition of its keys into n1..n4.
__device__ void divide_wave(const OctNode& nd, uint32_t* const keys[2], OctNode ch[4],
                            int lane) {
  const int hx = (nd.x1 - nd.x0 + 1) >> 1;  // ceil((float)(UR.x-UL.x)/2)
  const int hy = (nd.y1 - nd.y0 + 1) >> 1;  // ceil((float)(BR.y-UL.y)/2)
  const int xm = nd.x0 + hx, ym = nd.y0 + hy;
  const uint32_t* src = keys[nd.buf] + nd.kbeg;
  uint32_t* dst = keys[nd.buf ^ 1] + nd.kbeg;
  int cnt[4] = {0, 0, 0, 0};
  for (int s = 0; s < nd.n; s += 64) {
    const int i = s + lane;
    int q = -1;
    if (i < nd.n) {
      const uint32_t k = src[i];
      q = (key_x(k) >= xm ? 1 : 0) + (key_y(k) >= ym ? 2 : 0);
    }
#pragma unroll
    for (int qq = 0; qq < 4; qq++) cnt[qq] += __popcll(__ballot(q == qq));
  }
  int start[4];
  start[0] = 0;
  start[1] = cnt[0];
  start[2] = cnt[0] + cnt[1];
  start[3] = start[2] + cnt[2];
  int run[4] = {start[0], start[1], start[2], start[3]};
  for (int s = 0; s < nd.n; s += 64) {
    const int i = s + lane;
    int q = -1;
    uint32_t k = 0;
    if (i < nd.n) {
      k = src[i];
      q = (key_x(k) >= xm ? 1 : 0) + (key_y(k) >= ym ? 2 : 0);
    }
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
      const uint64_t m = __ballot(q == qq);
      if (q == qq) dst[run[qq] + lanes_below(m)] = k;
      run[qq] += __popcll(m);
    }
  }
  const int16_t xs[3] = {(int16_t)nd.x0, (int16_t)xm, (int16_t)nd.x1};
  const int16_t ys[3] = {(int16_t)nd.y0, (int16_t)ym, (int16_t)nd.y1};
#pragma unroll
  for (int qq = 0; qq < 4; qq++) {
    const int qx = qq & 1, qy = qq >> 1;
    ch[qq].x0 = xs[qx];
    ch[qq].x1 = xs[qx + 1];
    ch[qq].y0 = ys[qy];
    ch[qq].y1 = ys[qy + 1];
    ch[qq].kbeg = nd.kbeg + start[qq];
    ch[qq].n = cnt[qq];
    ch[qq].seq = 0;
    ch[qq].buf = nd.buf ^ 1;
  }
}

// The global-memory DistributeOctTree of one (level, image) by a 256-thread work-group, for the
// levels the LDS kernels cannot hold (their oct_count entry is -1). S: LDS scratch.
template <int kThr>
__device__ __forceinline__ void octree_global(
    OctShared& S, int level, int img, const OrbGeom* __restrict__ g,
    const uint32_t* __restrict__ cell_keys, const int* __restrict__ cell_count,
    uint32_t* __restrict__ key_scratch, OctNode* __restrict__ node_scratch,
    uint32_t* __restrict__ oct_keys, int* __restrict__ oct_count, uint32_t* __restrict__ err) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const LevelGeom& L = g->lv[level];
  const int N = L.budget;
  const int ncell = L.ncols * L.nrows;
  const int64_t cbase = (int64_t)img * g->cells_per_image + L.cell_base;
  uint32_t* const keys[2] = {key_scratch + img * g->keys_per_image + L.key_base,
                             key_scratch + img * g->keys_per_image + L.key_base + L.key_cap};
  OctNode* const lists[2] = {node_scratch + img * g->nodes_per_image + L.node_base,
                             node_scratch + img * g->nodes_per_image + L.node_base +
                                 2 * L.node_cap};
  OctNode* const child = node_scratch + img * g->nodes_per_image + L.node_base + 4 * L.node_cap;
  int* const outc = oct_count + img * g->nlevels + level;
  uint32_t* const outk = oct_keys + (int64_t)img * g->out_per_image + L.out_base;
  if (*outc != -1) return;  // done by octree_img_kernel

  // ---- 1. gather FAST candidates in cell row-major order into keys[0]
  for (int c0 = 0; c0 < ncell; c0 += kOctCap) {
    const int n = min(kOctCap, ncell - c0);
    for (int i = tid; i < n; i += kThr) S.a[i] = cell_count[cbase + c0 + i];
    __syncthreads();
    if (tid == 0) S.total = 0;
    const int tot = block_scan_array<kThr>(S.a, n, S.wsum);
    const int base = (c0 == 0) ? 0 : S.ktotal;
    for (int i = wid; i < n; i += (kThr / 64)) {
      const int cnt = cell_count[cbase + c0 + i];
      const int off = base + S.a[i];
      const int gi = i & ~(kCellGroup - 1);  // the cell's key group (c0 is group-aligned)
      const uint32_t* src = cell_keys + (cbase + c0 + gi) * g->cell_cap + (S.a[i] - S.a[gi]);
      for (int k = lane; k < cnt; k += 64)
        if (off + k < L.key_cap) keys[0][off + k] = src[k];
    }
    __syncthreads();
    if (tid == 0) S.ktotal = base + tot;
    __syncthreads();
  }
  int K = S.ktotal;
  if (K > L.key_cap) {
    if (tid == 0) atomicOr(err, kErrKeyOverflow);
    K = L.key_cap;
  }
  if (K == 0) {
    if (tid == 0) *outc = 0;
    return;
  }
  // ---- 2. initial nodes (:484-526): bucket (int)(x / hX), stable, by wave 0
  const int nIni = L.n_ini;
  const float hX = L.hx;
  if (wid == 0) {
    for (int q0 = 0; q0 < nIni; q0 += 64) {
      const int qn = min(64, nIni - q0);
      int cnt = 0;
      for (int s = 0; s < K; s += 64) {
        const int i = s + lane;
        int q = -1;
        if (i < K) q = (int)((float)key_x(keys[0][i]) / hX) - q0;
        for (int qq = 0; qq < qn; qq++) {
          const int pc = __popcll(__ballot(q == qq));
          if (lane == qq) cnt += pc;
        }
      }
      if (lane < qn) S.a[q0 + lane] = cnt;
    }
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int q = 0; q < nIni; q++) {
      const int c = S.a[q];
      S.b[q] = run;
      run += c;
    }
  }
  __syncthreads();
  if (wid == 0) {
    for (int q0 = 0; q0 < nIni; q0 += 64) {
      const int qn = min(64, nIni - q0);
      int run = (lane < qn) ? S.b[q0 + lane] : 0;
      for (int s = 0; s < K; s += 64) {
        const int i = s + lane;
        int q = -1;
        uint32_t k = 0;
        if (i < K) {
          k = keys[0][i];
          q = (int)((float)key_x(k) / hX) - q0;
        }
        for (int qq = 0; qq < qn; qq++) {
          const uint64_t m = __ballot(q == qq);
          const int r = __shfl(run, qq, 64);
          if (q == qq) keys[1][r + lanes_below(m)] = k;
          if (lane == qq) run += __popcll(m);
        }
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int m = 0;
    for (int i = 0; i < nIni; i++) {
      const int c = S.a[i];
      if (c == 0) continue;  // empty initial nodes are erased (:513-526)
      OctNode nd;
      nd.x0 = (int16_t)(int)(hX * (float)i);
      nd.x1 = (int16_t)(int)(hX * (float)(i + 1));
      nd.y0 = 0;
      nd.y1 = (int16_t)(L.max_by - kMinBorder);
      nd.kbeg = S.b[i];
      nd.n = c;
      nd.seq = i;
      nd.buf = 1;
      lists[0][m++] = nd;
    }
    S.m = m;
    S.seq_next = nIni;
    S.mode = 0;
    S.finish = 0;
    S.nexp = 0;
  }
  __syncthreads();
  int cur = 0;
  // ---- 3. passes
  while (true) {
    const int m = S.m;
    OctNode* const Lc = lists[cur];
    OctNode* const Ln = lists[cur ^ 1];
    if (S.mode == 0) {
      // outer pass: divide every node with > 1 key, in list order
      for (int j = wid; j < m; j += (kThr / 64)) {
        const OctNode nd = Lc[j];
        int t = 0, e = 0;
        if (nd.n > 1) {
          OctNode ch[4];
          divide_wave(nd, keys, ch, lane);
          if (lane == 0)
            for (int q = 0; q < 4; q++) {
              child[4 * j + q] = ch[q];
              t += ch[q].n > 0;
              e += ch[q].n > 1;
            }
        }
        if (lane == 0) {
          S.a[j] = t;               // children pushed
          S.b[j] = (nd.n == 1);     // survives in place
          S.c[j] = e;               // expandable children
        }
      }
      __syncthreads();
      const int T = block_scan_array<kThr>(S.a, m, S.wsum);
      const int U = block_scan_array<kThr>(S.b, m, S.wsum);
      const int E = block_scan_array<kThr>(S.c, m, S.wsum);
      const int newm = T + U;
      const int seq0 = S.seq_next;
      const bool ovf = newm > min(2 * L.node_cap, kOctCap) || E > kOctCap;
      if (!ovf) {
        for (int j = tid; j < m; j += kThr) {
          const OctNode nd = Lc[j];
          if (nd.n > 1) {
            int gpos = S.a[j], epos = S.c[j];
            for (int q = 0; q < 4; q++) {
              OctNode ch = child[4 * j + q];
              if (ch.n == 0) continue;
              ch.seq = seq0 + gpos;
              const int pos = T - 1 - gpos;
              Ln[pos] = ch;
              if (ch.n > 1) S.sortk[epos++] = (uint64_t)pos;  // vSize in push order
              gpos++;
            }
          } else {
            Ln[T + S.b[j]] = nd;
          }
        }
      }
      __syncthreads();
      if (tid == 0) {
        if (ovf) {
          atomicOr(err, kErrNodeOverflow);
          S.finish = 1;
        } else {
          S.m = newm;
          S.seq_next = seq0 + T;
          S.nexp = E;
          if (newm >= N || newm == m) S.finish = 1;
          else if (newm + E * 3 > N) S.mode = 1;
        }
      }
      if (!ovf) cur ^= 1;
      __syncthreads();
      if (S.finish) break;
    } else {
      // inner loop iteration: vPrev = S.sortk[0..V) (list positions, push order)
      const int V = S.nexp;
      int P2 = 1;
      while (P2 < V) P2 <<= 1;
      for (int i = tid; i < P2; i += kThr) {
        uint64_t key = 0;  // pads sort to the end (descending)
        if (i < V) {
          const int pos = (int)S.sortk[i];
          const OctNode& nd = Lc[pos];
          key = ((uint64_t)nd.n << 44) | ((uint64_t)(uint32_t)nd.seq << 12) | (uint64_t)pos;
        }
        S.sortk[i] = key;
      }
      __syncthreads();
      // bitonic sort, descending by (n, seq): reference processes sort() ascending from the end
      for (int k = 2; k <= P2; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          for (int i = tid; i < P2; i += kThr) {
            const int ixj = i ^ jj;
            if (ixj > i) {
              const uint64_t x = S.sortk[i], y = S.sortk[ixj];
              const bool desc = (i & k) == 0;
              if (desc ? (x < y) : (x > y)) {
                S.sortk[i] = y;
                S.sortk[ixj] = x;
              }
            }
          }
          __syncthreads();
        }
      }
      // speculative division of every vPrev node in processing order
      for (int j = wid; j < V; j += (kThr / 64)) {
        const int pos = (int)(S.sortk[j] & 0xfff);
        const OctNode nd = Lc[pos];
        OctNode ch[4];
        divide_wave(nd, keys, ch, lane);
        if (lane == 0) {
          int t = 0, e = 0;
          for (int q = 0; q < 4; q++) {
            child[4 * j + q] = ch[q];
            t += ch[q].n > 0;
            e += ch[q].n > 1;
          }
          S.a[j] = t;
          S.c[j] = e;
          S.b[j] = t - 1;
        }
      }
      __syncthreads();
      // cut: first j with m + sum_{i<=j}(t_i - 1) >= N
      for (int i = tid; i < V; i += kThr) S.b[i] = S.a[i] - 1;
      __syncthreads();
      block_scan_array<kThr>(S.b, V, S.wsum);  // exclusive prefix of (t - 1)
      if (tid == 0) S.total = V - 1;
      __syncthreads();
      for (int j = tid; j < V; j += kThr)
        if (m + S.b[j] + (S.a[j] - 1) >= N) atomicMin(&S.total, j);
      __syncthreads();
      const int J = S.total;  // last processed index
      const int nproc = J + 1;
      for (int i = tid; i < V; i += kThr)
        if (i >= nproc) {
          S.a[i] = 0;
          S.c[i] = 0;
        }
      __syncthreads();
      const int T = block_scan_array<kThr>(S.a, V, S.wsum);  // push-order child positions
      const int E = block_scan_array<kThr>(S.c, V, S.wsum);
      // survivors: old list minus processed nodes
      for (int i = tid; i < m; i += kThr) S.b[i] = 1;
      __syncthreads();
      for (int j = tid; j < nproc; j += kThr) S.b[(int)(S.sortk[j] & 0xfff)] = 0;
      __syncthreads();
      const int U = block_scan_array<kThr>(S.b, m, S.wsum);
      // block_scan_array overwrote the flags with prefixes; recover flags from processed set
      const int newm = T + U;
      const int seq0 = S.seq_next;
      const bool ovf = newm > min(2 * L.node_cap, kOctCap) || E > kOctCap;
      __shared__ uint8_t processed[kOctCap];
      for (int i = tid; i < m; i += kThr) processed[i] = 0;
      __syncthreads();
      for (int j = tid; j < nproc; j += kThr) processed[(int)(S.sortk[j] & 0xfff)] = 1;
      __syncthreads();
      // new vSize goes to a temporary (S.c keeps E prefixes): reuse child area tail? keep in LDS
      __shared__ int vnext[kOctCap];
      if (!ovf) {
        for (int j = tid; j < nproc; j += kThr) {
          int gpos = S.a[j], epos = S.c[j];
          for (int q = 0; q < 4; q++) {
            OctNode ch = child[4 * j + q];
            if (ch.n == 0) continue;
            ch.seq = seq0 + gpos;
            const int pos = T - 1 - gpos;
            Ln[pos] = ch;
            if (ch.n > 1) vnext[epos++] = pos;
            gpos++;
          }
        }
        for (int i = tid; i < m; i += kThr)
          if (!processed[i]) Ln[T + S.b[i]] = Lc[i];
      }
      __syncthreads();
      for (int i = tid; i < E; i += kThr) S.sortk[i] = (uint64_t)vnext[i];
      __syncthreads();
      if (tid == 0) {
        if (ovf) {
          atomicOr(err, kErrNodeOverflow);
          S.finish = 1;
        } else {
          S.m = newm;
          S.seq_next = seq0 + T;
          S.nexp = E;
          if (newm >= N || newm == m) S.finish = 1;
        }
      }
      if (!ovf) cur ^= 1;
      __syncthreads();
      if (S.finish) break;
    }
  }
  // ---- 4. retain the best key of each node (:682-701): strict '>' keeps the first maximum
  const int m = S.m;
  const OctNode* Lf = lists[cur];
  const int mout = min(m, L.out_cap);
  for (int j = tid; j < mout; j += kThr) {
    const OctNode nd = Lf[j];
    const uint32_t* ks = keys[nd.buf] + nd.kbeg;
    uint32_t best = ks[0];
    for (int k = 1; k < nd.n; k++) {
      const uint32_t kk = ks[k];
      if (key_score(kk) > key_score(best)) best = kk;
    }
    outk[j] = best;
  }
  if (tid == 0) {
    if (m > L.out_cap) atomicOr(err, kErrNodeOverflow);
    *outc = mout;
  }
}

// The fallback after octree_img_kernel: a grid of G <= kOctFbMaxGroups work-groups redoes the
// (image, level) entries octree_img left at -1; group b owns the entries e = b (mod G), reads
// their results at once (one load per thread) and redoes its -1 entries one after another.
// However many levels overflow -- all of them in a batch of busy textures -- they spread over
// the whole grid (at most total / G per group), and no group reads an entry another group
// writes. A batch whose levels all fit costs each group one load per thread.
constexpr int kOctFbMaxGroups = 256;
__global__ __launch_bounds__(kOctThreads) void octree_kernel(
    const OrbGeom* __restrict__ g, int n_images, const uint32_t* __restrict__ cell_keys,
    const int* __restrict__ cell_count, uint32_t* __restrict__ key_scratch,
    OctNode* __restrict__ node_scratch, uint32_t* __restrict__ oct_keys,
    int* __restrict__ oct_count, uint32_t* __restrict__ err) {
  __shared__ OctShared S;
  __shared__ int s_todo[kOctThreads];
  __shared__ int s_wcnt[kOctWaves];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, nlev = g->nlevels;
  const int total = n_images * nlev;  // entry e = img * nlevels + level (oct_count's layout)
  const int G = gridDim.x;
  for (int j0 = 0; (int)blockIdx.x + j0 * G < total; j0 += kOctThreads) {
    const int e = (int)blockIdx.x + (j0 + tid) * G;
    const bool redo = e < total && oct_count[e] == -1;
    const uint64_t m = __ballot(redo);
    if (lane == 0) s_wcnt[wid] = __popcll(m);
    __syncthreads();
    int off = 0, nt = 0;
    for (int w = 0; w < kOctWaves; w++) {
      if (w < wid) off += s_wcnt[w];
      nt += s_wcnt[w];
    }
    if (redo) s_todo[off + lanes_below(m)] = e;
    __syncthreads();
    for (int i = 0; i < nt; i++) {  // octree_global re-initialises everything it uses in S
      const int ei = s_todo[i];
      octree_global<kOctThreads>(S, ei % nlev, ei / nlev, g, cell_keys, cell_count, key_scratch,
                                 node_scratch, oct_keys, oct_count, err);
      __syncthreads();
    }
    __syncthreads();  // s_wcnt / s_todo read by every thread before the next sweep writes them
  }
}

// ---------------------------------------------------------------------------------------
// octree_img: the same DistributeOctTree for all levels of one image in one work-group, one wave
// per level, entirely in LDS and wave-synchronous (one work-group barrier, to allocate the key
// ranges). Per level: keys (one range, partitioned in place), two node lists and the
// count / prefix arrays of a pass (orb_geometry.cpp lays them out). A pass is
//   count children per node -> wave scans -> divide in place + put children at their final
//   list positions,
// so no child array exists. Dividing a node: a lane per node for n <= 32, the wave through
// registers for n <= 1024, the wave through global scratch above that.
// Creation order (the stand-in for the reference's pointer order, :625) only breaks ties inside
// vPrev, whose nodes were all created in the same pass -- in push order, i.e. ascending list
// position -- so nodes carry no sequence number. Levels whose keys do not fit set
// oct_count = -1 and octree_kernel (global memory) redoes them.
#ifndef OCT_PROF
#define OCT_PROF 0
#endif
#ifndef OCT_LANE_KEYS
#define OCT_LANE_KEYS 64
#endif
constexpr int kOctLaneKeys = OCT_LANE_KEYS;  // <= 255 (8-bit packed quadrant counts)
constexpr int kOctDivRegs = 16;

struct OctNodeS {
  int16_t x0, x1, y0, y1;
  uint32_t kn;  // kbeg | n << 16 (level-relative key range)
};
static_assert(sizeof(OctNodeS) == 12, "compact node");
__device__ __forceinline__ int node_kbeg(const OctNodeS& d) { return (int)(d.kn & 0xffffu); }
__device__ __forceinline__ int node_n(const OctNodeS& d) { return (int)(d.kn >> 16); }

// lane l's node (l wave-uniform): three readlanes instead of an LDS round trip
__device__ __forceinline__ OctNodeS readlane_node(const OctNodeS& nd, int l) {
  uint32_t w[3];
  __builtin_memcpy(w, &nd, sizeof(w));
#pragma unroll
  for (int i = 0; i < 3; i++) w[i] = (uint32_t)__builtin_amdgcn_readlane((int)w[i], l);
  OctNodeS o;
  __builtin_memcpy(&o, w, sizeof(w));
  return o;
}

__device__ __forceinline__ int quadrant(uint32_t k, int xm, int ym) {
  return (key_x(k) >= xm ? 1 : 0) + (key_y(k) >= ym ? 2 : 0);
}
__device__ __forceinline__ int node_xm(const OctNodeS& d) { return d.x0 + ((d.x1 - d.x0 + 1) >> 1); }
__device__ __forceinline__ int node_ym(const OctNodeS& d) { return d.y0 + ((d.y1 - d.y0 + 1) >> 1); }

// exclusive prefix sum over the wave (DPP: row shifts, then row broadcasts); *total = sum
__device__ __forceinline__ int wave_excl_scan(int v, int lane, int* total) {
  int x = v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  *total = __builtin_amdgcn_readlane(x, 63);
  (void)lane;
  return x - v;
}

// in-place exclusive scan of a[0..n) (int16) by one wave; returns the total
__device__ __forceinline__ int wave_scan_array(int16_t* a, int n, int lane) {
  int carry = 0;
  for (int c = 0; c < n; c += 64) {
    const int i = c + lane;
    const int v = i < n ? a[i] : 0;
    int tot;
    const int ex = wave_excl_scan(v, lane, &tot);
    if (i < n) a[i] = (int16_t)(carry + ex);
    carry += tot;
  }
  return carry;
}

// n <= kOctLaneKeys, one lane: 4 packed 8-bit quadrant counts; partitions in place if part
__device__ __forceinline__ uint32_t lane_divide(const OctNodeS& nd, uint32_t* keys, bool part) {
  const int xm = node_xm(nd), ym = node_ym(nd), kb = node_kbeg(nd), n = node_n(nd);
  uint32_t kr[kOctLaneKeys];
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < kOctLaneKeys; r++)
    if (r < n) {
      kr[r] = keys[kb + r];
      c += 1u << (8 * quadrant(kr[r], xm, ym));
    }
  if (part) {
    uint32_t run = (c << 8) + (c << 16) + (c << 24);  // byte q: keys in quadrants below q
#pragma unroll
    for (int r = 0; r < kOctLaneKeys; r++)
      if (r < n) {
        const int q = quadrant(kr[r], xm, ym);
        keys[kb + ((run >> (8 * q)) & 255)] = kr[r];
        run += 1u << (8 * q);
      }
  }
  return c;
}

// one wave: quadrant counts of a node (uniform)
__device__ __forceinline__ void wave_count(const OctNodeS& nd, const uint32_t* keys, int lane,
                                           int cnt[4]) {
  const int xm = node_xm(nd), ym = node_ym(nd), kb = node_kbeg(nd), n = node_n(nd);
#pragma unroll
  for (int q = 0; q < 4; q++) cnt[q] = 0;
  for (int s0 = 0; s0 < n; s0 += 64) {
    const int q = s0 + lane < n ? quadrant(keys[kb + s0 + lane], xm, ym) : -1;
#pragma unroll
    for (int qq = 0; qq < 4; qq++) cnt[qq] += __popcll(__ballot(q == qq));
  }
}

// one wave: stable in-place partition of a node's keys; returns the counts (uniform)
__device__ void wave_partition(const OctNodeS& nd, uint32_t* keys, uint32_t* gscratch, int lane,
                               int cnt[4]) {
  const int xm = node_xm(nd), ym = node_ym(nd), kb = node_kbeg(nd), n = node_n(nd);
  if (n <= 64 * kOctDivRegs) {  // through registers: one read of the keys, counted, then placed
    const int R = (n + 63) >> 6;
    uint32_t kr[kOctDivRegs];
    int qr[kOctDivRegs];
#pragma unroll
    for (int r = 0; r < kOctDivRegs; r++) {
      qr[r] = -1;
      if (r < R && 64 * r + lane < n) {
        kr[r] = keys[kb + 64 * r + lane];
        qr[r] = quadrant(kr[r], xm, ym);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) cnt[q] = 0;
#pragma unroll
    for (int r = 0; r < kOctDivRegs; r++)
      if (r < R) {
#pragma unroll
        for (int q = 0; q < 4; q++) cnt[q] += __popcll(__ballot(qr[r] == q));
      }
    int run[4] = {0, cnt[0], cnt[0] + cnt[1], cnt[0] + cnt[1] + cnt[2]};
#pragma unroll
    for (int r = 0; r < kOctDivRegs; r++)
      if (r < R) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint64_t m = __ballot(qr[r] == q);
          if (qr[r] == q) keys[kb + run[q] + lanes_below(m)] = kr[r];
          run[q] += __popcll(m);
        }
      }
  } else {  // through this level's global scratch (first passes of very dense levels only)
    wave_count(nd, keys, lane, cnt);
    int run[4] = {0, cnt[0], cnt[0] + cnt[1], cnt[0] + cnt[1] + cnt[2]};
    for (int i = lane; i < n; i += 64) gscratch[kb + i] = keys[kb + i];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    for (int s0 = 0; s0 < n; s0 += 64) {
      const int i = s0 + lane;
      uint32_t k = 0;
      int q = -1;
      if (i < n) {
        k = gscratch[kb + i];
        q = quadrant(k, xm, ym);
      }
#pragma unroll
      for (int qq = 0; qq < 4; qq++) {
        const uint64_t m = __ballot(q == qq);
        if (q == qq) keys[kb + run[qq] + lanes_below(m)] = k;
        run[qq] += __popcll(m);
      }
    }
  }
}

__global__ __launch_bounds__(64 * kMaxLevels) void octree_img_kernel(
    const OrbGeom* __restrict__ g, const uint32_t* __restrict__ cell_keys,
    const int* __restrict__ cell_count, uint32_t* __restrict__ key_scratch,
    uint32_t* __restrict__ oct_keys, int* __restrict__ oct_count, uint32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_oct[];
  __shared__ int s_K[kMaxLevels];
  const int img = blockIdx.x, lane = threadIdx.x & 63, level = wave_id();
  const int nlev = g->nlevels;
  const bool active = level < nlev;
  const LevelGeom& L = g->lv[active ? level : 0];
  const int ncell = L.ncols * L.nrows;
  const int64_t cbase = (int64_t)img * g->cells_per_image + L.cell_base;
#if OCT_PROF  // diagnostic build: per-phase shader cycles of images 0-1 (printf at the end)
  uint64_t op_t = clock64(), op_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int op_np = 0, op_V = 0;
  uint32_t op_pass[8][6] = {};  // per pass: V, big nodes, sort, count, scan, place cycles
  auto optick = [&](int i) {
    const uint64_t t = clock64();
    op_acc[i] += t - op_t;
    if (i >= 2 && i <= 5 && op_np >= 1 && op_np <= 8) op_pass[op_np - 1][i] += (uint32_t)(t - op_t);
    op_t = t;
  };
#else
  auto optick = [](int) {};
#endif
  // ---- 1. candidate counts -> this level's key range (levels that do not fit fall back)
  int K = 0;
  if (active) {
    for (int c = lane; c < ncell; c += 64) K += cell_count[cbase + c];
    K = wave_sum(K);
    if (lane == 0) s_K[level] = K;
  }
  __syncthreads();
  if (!active) return;
  optick(0);
  int* const outc = oct_count + img * nlev + level;
  uint32_t* const outk = oct_keys + (int64_t)img * g->out_per_image + L.out_base;
  const int nIni = L.n_ini;
  int koff = 0;
  bool fits = true;
  for (int l = 0; l <= level; l++) {
    const bool f = koff + s_K[l] <= g->oct_kcap;
    if (l == level) fits = f;
    else if (f) koff += s_K[l];
  }
  if (!fits || nIni > 16) {
    if (lane == 0) *outc = -1;  // octree_kernel redoes this level
    return;
  }
  if (K == 0) {
    if (lane == 0) *outc = 0;
    return;
  }
  uint32_t* const keys = reinterpret_cast<uint32_t*>(s_oct) + koff;
  uint32_t* const gscratch = key_scratch + img * g->keys_per_image + L.key_base;
  const int NC = L.oct_nc;
  OctNodeS* const lists = reinterpret_cast<OctNodeS*>(s_oct + L.oct_list_off);
  uint32_t* const sortk = reinterpret_cast<uint32_t*>(s_oct + L.oct_work_off);
  int16_t* const pt = reinterpret_cast<int16_t*>(sortk + NC);
  int16_t* const pe = pt + NC;
  int16_t* const pu = pe + NC;
  int16_t* const vnext = pu + NC;
  uint8_t* const processed = reinterpret_cast<uint8_t*>(vnext + NC);

  // ---- 2. gather in cell row-major order, stably bucketed into the initial nodes
  // (:484-526, bucket (int)(x / hX)). Fast path (<= 512 cells, K <= 3072): all cell counts
  // up front, keys stored in cell order with independent loads (a key slot finds its cell by a
  // binary search over the lanes' prefixes), then one in-place stable partition through
  // registers. Otherwise two sweeps over global memory (count, then place).
  const float hX = L.hx;
  constexpr int kGatherChunks = 8, kGatherRegs = 48;
  int bcnt = 0;  // lane b < nIni: keys in bucket b
  if (ncell <= 64 * kGatherChunks && K <= 64 * kGatherRegs && ncell + 1 <= NC) {
    // key-group prefixes in LDS (the level's sort scratch, free until the passes): a group's
    // keys are contiguous from its first slot, so a key slot needs only its group -- the
    // largest g with gp[g] <= s (empty groups repeat the next prefix and are skipped) -- found by
    // a branch-free binary search over the <= 64 groups whose probes for all the wave's slots
    // are issued together, step by step, then every key load at once
    int* const gp = reinterpret_cast<int*>(sortk);
    int ccnt[kGatherChunks];
#pragma unroll
    for (int ch = 0; ch < kGatherChunks; ch++) {
      const int c = 64 * ch + lane;
      ccnt[ch] = c < ncell ? cell_count[cbase + c] : 0;
    }
    int carry = 0;
#pragma unroll
    for (int ch = 0; ch < kGatherChunks; ch++) {
      if (64 * ch < ncell) {
        int ctot;
        const int cex = wave_excl_scan(ccnt[ch], lane, &ctot);
        const int c = 64 * ch + lane;
        if (c < ncell && (c & (kCellGroup - 1)) == 0) gp[c / kCellGroup] = carry + cex;
        carry += ctot;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int R = (K + 63) >> 6;
    const int ng = (ncell + kCellGroup - 1) / kCellGroup;  // <= 64
    uint32_t kr[kGatherRegs];
    int br[kGatherRegs];  // the slot's group during the search, its bucket after
#pragma unroll
    for (int r = 0; r < kGatherRegs; r++) br[r] = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
#pragma unroll
      for (int r = 0; r < kGatherRegs; r++) {
        if (r < R) {
          const int cand = br[r] + step;
          if (cand < ng && gp[cand] <= 64 * r + lane) br[r] = cand;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kGatherRegs; r++) {
      const int s = 64 * r + lane;
      if (r < R && s < K)
        kr[r] = cell_keys[(cbase + kCellGroup * br[r]) * g->cell_cap + (s - gp[br[r]])];
      br[r] = -1;
    }
#pragma unroll
    for (int r = 0; r < kGatherRegs; r++) {
      if (r < R && 64 * r + lane < K) {
        br[r] = (int)((float)key_x(kr[r]) / hX);
        if (br[r] >= nIni) br[r] = -1;
      }
    }
#pragma unroll
    for (int r = 0; r < kGatherRegs; r++)
      if (r < R)
        for (int bb = 0; bb < nIni; bb++) {
          const int pc = __popcll(__ballot(br[r] == bb));
          if (lane == bb) bcnt += pc;
        }
    int tot;
    int brun = wave_excl_scan(lane < nIni ? bcnt : 0, lane, &tot);
#pragma unroll
    for (int r = 0; r < kGatherRegs; r++)
      if (r < R)
        for (int bb = 0; bb < nIni; bb++) {
          const uint64_t mm = __ballot(br[r] == bb);
          const int at = __builtin_amdgcn_readlane(brun, bb);  // bb is wave-uniform
          if (br[r] == bb) keys[at + lanes_below(mm)] = kr[r];
          if (lane == bb) brun += __popcll(mm);
        }
  } else {
    for (int sweep = 0; sweep < 2; sweep++) {
      int brun = 0;  // lane b: next free slot of bucket b (sweep 2)
      if (sweep == 1) {
        int tot;
        brun = wave_excl_scan(lane < nIni ? bcnt : 0, lane, &tot);
      }
      for (int c0 = 0; c0 < ncell; c0 += 64) {
        const int cnt = c0 + lane < ncell ? cell_count[cbase + c0 + lane] : 0;
        int ctot;
        const int cex = wave_excl_scan(cnt, lane, &ctot);
        for (int r0 = 0; r0 < ctot; r0 += 64) {
          const int r = r0 + lane;
          // binary search on all lanes (shuffles read every lane's prefix)
          int lo = 0;
#pragma unroll
          for (int step = 32; step >= 1; step >>= 1) {
            const int cand = lo + step;
            const int pv = __shfl(cex, cand & 63, 64);
            if (cand < 64 && pv <= r) lo = cand;
          }
          const int gs = lo & ~(kCellGroup - 1);  // key group of cell lo (c0 is group-aligned)
          const int base = __shfl(cex, gs, 64);
          int b = -1;
          uint32_t k = 0;
          if (r < ctot) {
            k = cell_keys[(cbase + c0 + gs) * g->cell_cap + (r - base)];
            b = (int)((float)key_x(k) / hX);
            if (b >= nIni) b = -1;
          }
          for (int bb = 0; bb < nIni; bb++) {
            const uint64_t m = __ballot(b == bb);
            if (sweep == 1) {
              const int at = __builtin_amdgcn_readlane(brun, bb);  // bb is wave-uniform
              if (b == bb) keys[at + lanes_below(m)] = k;
              if (lane == bb) brun += __popcll(m);
            } else if (lane == bb) {
              bcnt += __popcll(m);
            }
          }
        }
      }
    }
  }
  // initial nodes: non-empty buckets in order (empty ones are erased, :513-526)
  int m = 0;
  {
    int tot;
    const int bbase = wave_excl_scan(lane < nIni ? bcnt : 0, lane, &tot);
    const bool has = lane < nIni && bcnt > 0;
    const uint64_t hm = __ballot(has);
    if (has) {
      OctNodeS nd;
      nd.x0 = (int16_t)(int)(hX * (float)lane);
      nd.x1 = (int16_t)(int)(hX * (float)(lane + 1));
      nd.y0 = 0;
      nd.y1 = (int16_t)(L.max_by - kMinBorder);
      nd.kn = (uint32_t)bbase | (uint32_t)bcnt << 16;
      lists[lanes_below(hm)] = nd;
    }
    m = __popcll(hm);
  }
  // ---- 3. passes
  optick(1);
  const int N = L.budget;
  int cur = 0, nexp = 0;
  bool outer = true;
  while (true) {
    const OctNodeS* Lc = lists + cur * NC;
    OctNodeS* Ln = lists + (cur ^ 1) * NC;
    const int V = outer ? m : nexp;
#if OCT_PROF
    op_np++;
    op_V += V;
    if (op_np <= 8) op_pass[op_np - 1][0] = V;
#endif
    if (!outer) {  // vPrev: positions in push order -> descending (n, creation order)
      int P2 = 64;
      while (P2 < V) P2 <<= 1;
      for (int i = lane; i < P2; i += 64) {
        uint32_t key = 0;  // pads sort to the end
        if (i < V) {
          const int pos = (int)sortk[i];
          key = (uint32_t)node_n(Lc[pos]) << 12 | (uint32_t)(4095 - pos);
        }
        sortk[i] = key;
      }
      for (int k = 2; k <= P2; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
          for (int i = lane; i < P2; i += 64) {
            const int ixj = i ^ jj;
            if (ixj > i) {
              const uint32_t x = sortk[i], y = sortk[ixj];
              const bool desc = (i & k) == 0;
              if (desc ? (x < y) : (x > y)) {
                sortk[i] = y;
                sortk[ixj] = x;
              }
            }
          }
        }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    optick(2);
    auto nidx = [&](int j) { return outer ? j : 4095 - (int)(sortk[j] & 0xfffu); };
    // -- count children: t (non-empty), e (> 1 key); pu = survivor flag (outer) or t - 1
    for (int j0 = 0; j0 < V; j0 += 64) {
      const int j = j0 + lane;
      const bool valid = j < V;
      OctNodeS nd{};
      if (valid) nd = Lc[nidx(j)];
      const int n = node_n(nd);
      int t = 0, e = 0;
      if (valid && n > 1 && n <= kOctLaneKeys) {
        const uint32_t c = lane_divide(nd, keys, false);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int cq = (c >> (8 * q)) & 255;
          t += cq > 0;
          e += cq > 1;
        }
      }
      uint64_t bigm = __ballot(valid && n > kOctLaneKeys);
#if OCT_PROF
      if (op_np <= 8) op_pass[op_np - 1][1] += __popcll(bigm);
#endif
      while (bigm) {
        const int bl = __builtin_ctzll(bigm);
        bigm &= bigm - 1;
        const OctNodeS nb = readlane_node(nd, bl);
        int cnt[4];
        wave_count(nb, keys, lane, cnt);
        if (lane == bl) {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            t += cnt[q] > 0;
            e += cnt[q] > 1;
          }
        }
      }
      if (valid) {
        pt[j] = (int16_t)t;
        pe[j] = (int16_t)e;
        pu[j] = (int16_t)(outer ? (n == 1) : t - 1);
      }
    }
    optick(3);
    int nproc = V;
    if (!outer) {
      // processing stops once the list reaches N: first j with m + sum_{i<=j}(t_i - 1) >= N
      int carry = 0;
      nproc = V;
      for (int j0 = 0; j0 < V; j0 += 64) {
        const int j = j0 + lane;
        const int v = j < V ? pu[j] : 0;
        int tot;
        const int incl = carry + wave_excl_scan(v, lane, &tot) + v;
        const uint64_t hit = __ballot(j < V && m + incl >= N);
        if (hit) {
          nproc = j0 + __builtin_ctzll(hit) + 1;
          break;
        }
        carry += tot;
      }
      for (int i = lane; i < m; i += 64) processed[i] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int j = lane; j < nproc; j += 64) processed[nidx(j)] = 1;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int i = lane; i < m; i += 64) pu[i] = (int16_t)(processed[i] ? 0 : 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int T = wave_scan_array(pt, nproc, lane);  // push-order child positions
    const int E = wave_scan_array(pe, nproc, lane);
    const int U = wave_scan_array(pu, m, lane);      // survivors keep their order
    const int newm = T + U;
    if (newm > NC || E > NC) {
      if (lane == 0) atomicOr(err, kErrNodeOverflow);
      break;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    optick(4);
    // -- divide in place and place children: push order gpos -> list position T-1-gpos
    auto place = [&](int j, const OctNodeS& nd, uint32_t c4) {
      int gpos = pt[j], epos = pe[j];
      const int xm = node_xm(nd), ym = node_ym(nd);
      const int16_t xs[3] = {nd.x0, (int16_t)xm, nd.x1};
      const int16_t ys[3] = {nd.y0, (int16_t)ym, nd.y1};
      int start = node_kbeg(nd);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int cq = (int)((c4 >> (8 * q)) & 255u);
        if (cq > 0) {
          OctNodeS ch;
          ch.x0 = xs[q & 1];
          ch.x1 = xs[(q & 1) + 1];
          ch.y0 = ys[q >> 1];
          ch.y1 = ys[(q >> 1) + 1];
          ch.kn = (uint32_t)start | (uint32_t)cq << 16;
          const int pos = T - 1 - gpos;
          Ln[pos] = ch;
          if (cq > 1) vnext[epos++] = (int16_t)pos;
          gpos++;
        }
        start += cq;
      }
    };
    for (int j0 = 0; j0 < nproc; j0 += 64) {
      const int j = j0 + lane;
      const bool valid = j < nproc;
      OctNodeS nd{};
      if (valid) nd = Lc[nidx(j)];
      const int n = node_n(nd);
      if (valid && n > 1 && n <= kOctLaneKeys) place(j, nd, lane_divide(nd, keys, true));
      uint64_t bigm = __ballot(valid && n > kOctLaneKeys);
      while (bigm) {
        const int bl = __builtin_ctzll(bigm);
        bigm &= bigm - 1;
        const OctNodeS nb = readlane_node(nd, bl);
        const int gpos0 = pt[j0 + bl], epos0 = pe[j0 + bl];  // read before the partition's stores
        int cnt[4];
        wave_partition(nb, keys, gscratch, lane, cnt);
        if (lane == 0) {
          // counts can exceed 255 here: place() takes 8-bit counts, so place big ones inline
          int gpos = gpos0, epos = epos0;
          const int xm = node_xm(nb), ym = node_ym(nb);
          const int16_t xs[3] = {nb.x0, (int16_t)xm, nb.x1};
          const int16_t ys[3] = {nb.y0, (int16_t)ym, nb.y1};
          int start = node_kbeg(nb);
          for (int q = 0; q < 4; q++) {
            if (cnt[q] > 0) {
              OctNodeS ch;
              ch.x0 = xs[q & 1];
              ch.x1 = xs[(q & 1) + 1];
              ch.y0 = ys[q >> 1];
              ch.y1 = ys[(q >> 1) + 1];
              ch.kn = (uint32_t)start | (uint32_t)cnt[q] << 16;
              const int pos = T - 1 - gpos;
              Ln[pos] = ch;
              if (cnt[q] > 1) vnext[epos++] = (int16_t)pos;
              gpos++;
            }
            start += cnt[q];
          }
        }
      }
    }
    for (int i = lane; i < m; i += 64) {
      const OctNodeS nd = Lc[i];
      if (outer ? node_n(nd) == 1 : !processed[i]) Ln[T + pu[i]] = nd;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < E; i += 64) sortk[i] = (uint32_t)vnext[i];
    optick(5);
    const int mprev = m;
    m = newm;
    nexp = E;
    cur ^= 1;
    if (newm >= N || newm == mprev) break;
    if (outer && newm + E * 3 > N) outer = false;
  }
  // ---- 4. retain the best key of each node (:682-701): strict '>' keeps the first maximum
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const OctNodeS* Lf = lists + cur * NC;
  const int mout = min(m, L.out_cap);
  for (int j = lane; j < mout; j += 64) {
    const OctNodeS nd = Lf[j];
    const int kb = node_kbeg(nd), n = node_n(nd);
    uint32_t best = keys[kb];
    for (int k = 1; k < n; k++) {
      const uint32_t kk = keys[kb + k];
      if (key_score(kk) > key_score(best)) best = kk;
    }
    outk[j] = best;
  }
  if (lane == 0) {
    if (m > L.out_cap) atomicOr(err, kErrNodeOverflow);
    *outc = mout;
  }
#if OCT_PROF
  optick(6);
  if (lane == 0 && img < 2)
    printf("[octprof] img %d level %d K %d passes %d V %d | cyc: count %llu gather %llu sort %llu "
           "count %llu scan %llu place %llu retain %llu\n", img, level, K, op_np, op_V,
           (unsigned long long)op_acc[0], (unsigned long long)op_acc[1],
           (unsigned long long)op_acc[2], (unsigned long long)op_acc[3],
           (unsigned long long)op_acc[4], (unsigned long long)op_acc[5],
           (unsigned long long)op_acc[6]);
  if (lane == 0 && img == 0 && level == 0)
    for (int i = 0; i < op_np && i < 8; i++)
      printf("[octpass] pass %d V %u big %u sort %u count %u scan %u place %u\n", i,
             op_pass[i][0], op_pass[i][1], op_pass[i][2], op_pass[i][3], op_pass[i][4], op_pass[i][5]);
#endif
}

// ---------------------------------------------------------------------------------------
// The same DistributeOctTree (:480-704) with one work-group of kOctLvlWaves waves per (level,
// image): the latency variant. One wave per level (octree_img_kernel) puts the level-0 wave on
// the critical path of a single frame (0.17 ms of a 0.46 ms frame call: gather 44 us, passes
// 120 us, profiles/r3f_lat_octprof.log); here the gather's loads, the vPrev sort, the per-node
// divides and the big nodes' partitions are spread over the waves. Same list semantics and
// output bytes; a level that does not fit its LDS falls back to octree_kernel as before.
constexpr int kOctLvlWaves = 8, kOctLvlThreads = 64 * kOctLvlWaves;
constexpr int kOctKpt = 16;  // key positions per thread of the passes: levels up to 8192 keys
#ifndef OCT_LVL_MAX_IMAGES
#define OCT_LVL_MAX_IMAGES 16
#endif
constexpr int kOctLvlMaxImages = OCT_LVL_MAX_IMAGES;

__device__ __forceinline__ int lvl_block_sum(int v, int* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[wave_id()] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int k = 0; k < kOctLvlWaves; k++) t += red[k];
  __syncthreads();
  return t;
}

// exclusive scan of a[0..n) in place by the whole work-group
__device__ void lvl_block_scan(int* a, int n, int* red) {
  const int lane = threadIdx.x & 63, w = wave_id();
  int carry = 0;
  for (int c = 0; c < n; c += kOctLvlThreads) {
    const int i = c + (int)threadIdx.x;
    const int v = i < n ? a[i] : 0;
    int wt;
    const int ex = wave_excl_scan(v, lane, &wt);
    if (lane == 0) red[w] = wt;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kOctLvlWaves; k++) {
      pre += k < w ? red[k] : 0;
      tot += red[k];
    }
    if (i < n) a[i] = carry + pre + ex;
    carry += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kOctLvlThreads) void octree_lvl_kernel(
    const OrbGeom* __restrict__ g, const uint32_t* __restrict__ cell_keys,
    const int* __restrict__ cell_count, uint32_t* __restrict__ key_scratch,
    OctNode* __restrict__ node_scratch, uint32_t* __restrict__ oct_keys,
    int* __restrict__ oct_count, uint32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_lvl[];
  __shared__ int s_red[kOctLvlWaves];
  __shared__ int s_bc[kOctLvlWaves][16];  // per-wave bucket counts of one placement round
  __shared__ int s_brun[16];              // next free slot of each initial bucket
  __shared__ int s_bcnt[16];              // keys per initial bucket
  __shared__ int s_u[4];                  // T, E, U of a pass; nproc
  __shared__ int s_scan[kOctLvlWaves][2];  // per-wave totals of the key scan
  const int level = blockIdx.x, img = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int nlev = g->nlevels;
  const LevelGeom& L = g->lv[level];
  const int ncell = L.ncols * L.nrows;
  const int64_t cbase = (int64_t)img * g->cells_per_image + L.cell_base;
  int* const outc = oct_count + img * nlev + level;
  auto otick = [](int) {};
  uint32_t* const outk = oct_keys + (int64_t)img * g->out_per_image + L.out_base;
  // ---- 1. candidate count; a level that does not fit is done here by the global-memory
  // algorithm (octree_global, its scratch on this work-group's LDS; the host checked it fits),
  // so the small launches need no octree_kernel launch after this one
  int K = 0;
  for (int c = tid; c < ncell; c += kOctLvlThreads) K += cell_count[cbase + c];
  K = lvl_block_sum(K, s_red);
  const int nIni = L.n_ini;
  const int NC = L.oct_nc;
  if (K > g->oct2_kcap || K > kOctKpt * kOctLvlThreads || nIni > 16 ||
      ncell + 1 > g->oct2_ccap || NC > g->oct2_nc) {
    if (tid == 0) *outc = -1;
    __syncthreads();
    octree_global<kOctLvlThreads>(*reinterpret_cast<OctShared*>(s_lvl), level, img, g, cell_keys,
                                  cell_count, key_scratch, node_scratch, oct_keys, oct_count, err);
    return;
  }
  if (K == 0) {
    if (tid == 0) *outc = 0;
    return;
  }
  uint32_t* const keys = reinterpret_cast<uint32_t*>(s_lvl);
  uint32_t* const tmp = reinterpret_cast<uint32_t*>(s_lvl + g->oct2_tmp_off);
  int* const cpre = reinterpret_cast<int*>(s_lvl + g->oct2_cpre_off);
  OctNodeS* const lists = reinterpret_cast<OctNodeS*>(s_lvl + g->oct2_list_off);
  uint32_t* const sortk = reinterpret_cast<uint32_t*>(s_lvl + g->oct2_work_off);
  int16_t* const pt = reinterpret_cast<int16_t*>(sortk + NC);
  int16_t* const pe = pt + NC;
  int16_t* const pu = pe + NC;
  int16_t* const vnext = pu + NC;
  uint8_t* const processed = reinterpret_cast<uint8_t*>(vnext + NC);
  uint8_t* const cand = processed + NC;  // the inner passes' candidates (vPrev), by list index
  uint2* const nst = reinterpret_cast<uint2*>(
      (reinterpret_cast<uintptr_t>(cand + NC) + 15) & ~static_cast<uintptr_t>(15));
  uint2* const nen = nst + NC;                         // prefix at / past a node's keys
  int16_t* const cb = reinterpret_cast<int16_t*>(nen + NC);  // first child's push index, or -1

  // ---- 2. gather in cell row-major order (a key slot finds its cell by binary search over the
  // cell prefix), then a stable placement into the initial nodes' buckets (:484-526)
  for (int c = tid; c < ncell; c += kOctLvlThreads) cpre[c] = cell_count[cbase + c];
  if (tid < 16) s_bcnt[tid] = 0;
  __syncthreads();
  lvl_block_scan(cpre, ncell, s_red);
  const float hX = L.hx;
  auto bucket = [&](uint32_t k) {
    const int b = (int)((float)key_x(k) / hX);
    return b >= nIni ? -1 : b;
  };
  constexpr int kGatherUnroll = 4;
  for (int s0 = 0; s0 < K; s0 += kGatherUnroll * kOctLvlThreads) {
    uint32_t kr[kGatherUnroll];
    int sr[kGatherUnroll];
#pragma unroll
    for (int r = 0; r < kGatherUnroll; r++) {
      const int s = s0 + r * kOctLvlThreads + tid;
      sr[r] = s;
      if (s < K) {
        int lo = 0, hi = ncell;  // largest c with cpre[c] <= s: the non-empty cell holding s
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (cpre[mid] <= s) lo = mid;
          else hi = mid;
        }
        const int gs = lo & ~(kCellGroup - 1);  // key group of cell lo: contiguous from gs
        kr[r] = cell_keys[(cbase + gs) * g->cell_cap + (s - cpre[gs])];
      }
    }
#pragma unroll
    for (int r = 0; r < kGatherUnroll; r++)
      if (sr[r] < K) {
        tmp[sr[r]] = kr[r];
        const int b = bucket(kr[r]);
        if (b >= 0) atomicAdd(&s_bcnt[b], 1);
      }
  }
  __syncthreads();
  if (w == 0) {
    int tot;
    const int bb = wave_excl_scan(lane < nIni ? s_bcnt[lane] : 0, lane, &tot);
    if (lane < 16) s_brun[lane] = bb;
  }
  __syncthreads();
  // stable placement, kOctLvlThreads slots per round in slot order
  for (int s0 = 0; s0 < K; s0 += kOctLvlThreads) {
    const int s = s0 + tid;
    uint32_t k = 0;
    int b = -1;
    if (s < K) {
      k = tmp[s];
      b = bucket(k);
    }
    int rank = 0;
    for (int bb = 0; bb < nIni; bb++) {
      const uint64_t m = __ballot(b == bb);
      if (b == bb) rank = lanes_below(m);
      if (lane == bb) s_bc[w][bb] = __popcll(m);
    }
    __syncthreads();
    if (b >= 0) {
      int pos = s_brun[b] + rank;
      for (int k2 = 0; k2 < w; k2++) pos += s_bc[k2][b];
      keys[pos] = k;
    }
    __syncthreads();
    if (tid < nIni) {
      int add = 0;
#pragma unroll
      for (int k2 = 0; k2 < kOctLvlWaves; k2++) add += s_bc[k2][tid];
      s_brun[tid] += add;
    }
    __syncthreads();
  }
  // initial nodes: non-empty buckets in order (empty ones are erased, :513-526)
  if (w == 0) {
    const int bcnt = lane < nIni ? s_bcnt[lane] : 0;
    int tot;
    const int bbase = wave_excl_scan(bcnt, lane, &tot);
    const bool has = lane < nIni && bcnt > 0;
    const uint64_t hm = __ballot(has);
    if (has) {
      OctNodeS nd;
      nd.x0 = (int16_t)(int)(hX * (float)lane);
      nd.x1 = (int16_t)(int)(hX * (float)(lane + 1));
      nd.y0 = 0;
      nd.y1 = (int16_t)(L.max_by - kMinBorder);
      nd.kn = (uint32_t)bbase | (uint32_t)bcnt << 16;
      lists[lanes_below(hm)] = nd;
    }
    if (lane == 0) s_u[0] = __popcll(hm);
  }
  __syncthreads();
  int m = s_u[0];
  __syncthreads();

  // ---- 3. passes: the list semantics of octree_img_kernel, divided key-parallel. Thread t owns
  // the key positions [t * kpt, (t + 1) * kpt) for the whole level: their keys, the node covering
  // each position and the position's exclusive prefix of quadrant one-hots (four 16-bit counters
  // in two words) stay in registers. A pass: one block scan of the one-hots over the candidate
  // nodes' keys -> every node's quadrant counts are the prefix difference across its segment
  // (recorded by the segment's first and last owners) -> the node list's counts, scans and
  // children as before -> each key moves to kbeg + (keys of lower quadrants) + (its rank in its
  // quadrant = its prefix minus the segment's), each position learns its new covering node.
  // No serial per-node loops over keys, and the same stable partition.
  otick(0);
  const int N = L.budget;
  int cur = 0, nexp = 0;
  bool outer = true;
  int Kn = 0;  // keys in the initial nodes (keys past the last bucket are dropped)
  for (int i = 0; i < m; i++) Kn += node_n(lists[i]);
  const int kpt = (Kn + kOctLvlThreads - 1) / kOctLvlThreads;  // <= kOctKpt (checked above)
  const int kb0 = tid * kpt;
  uint32_t kr[kOctKpt];
  int nd[kOctKpt];
  uint32_t plo[kOctKpt], phi[kOctKpt];
  uint64_t qbits = 0;  // 2 bits per position: its key's quadrant in this pass
#pragma unroll
  for (int i = 0; i < kOctKpt; i++) {
    nd[i] = 0;
    if (i < kpt && kb0 + i < Kn) {
      const int k = kb0 + i;
      kr[i] = keys[k];
      int c = 0;  // initial nodes are in key order: the last one starting at or before k
      for (int q = 1; q < m; q++) c += node_kbeg(lists[q]) <= k;
      nd[i] = c;
    }
  }
  while (true) {
    const OctNodeS* Lc = lists + cur * NC;
    OctNodeS* Ln = lists + (cur ^ 1) * NC;
    const int V = outer ? m : nexp;
    if (!outer) {  // vPrev: positions in push order -> descending (n, creation order)
      int P2 = 64;
      while (P2 < V) P2 <<= 1;
      for (int i = tid; i < P2; i += kOctLvlThreads) {
        uint32_t key = 0;  // pads sort to the end
        if (i < V) {
          const int pos = (int)sortk[i];
          key = (uint32_t)node_n(Lc[pos]) << 12 | (uint32_t)(4095 - pos);
        }
        sortk[i] = key;
      }
      for (int i = tid; i < m; i += kOctLvlThreads) cand[i] = 0;
      __syncthreads();
      for (int i = tid; i < V; i += kOctLvlThreads) cand[4095 - (int)(sortk[i] & 0xfffu)] = 1;
      __syncthreads();
      if (V <= 2 * kOctLvlThreads) {
        // rank sort (the keys are distinct): an element's place is the number of larger keys,
        // counted over the whole set with broadcast reads -- two barriers instead of the
        // bitonic network's log^2 steps
        uint32_t mine[2];
        int rk[2] = {0, 0};
#pragma unroll
        for (int r = 0; r < 2; r++) {
          const int i = tid + r * kOctLvlThreads;
          mine[r] = i < V ? sortk[i] : 0u;
        }
        const uint4* s4 = reinterpret_cast<const uint4*>(sortk);
        for (int j4 = 0; j4 < P2 / 4; j4++) {  // pads (0) count for nobody
          const uint4 o = s4[j4];
#pragma unroll
          for (int r = 0; r < 2; r++)
            rk[r] += (int)(o.x > mine[r]) + (int)(o.y > mine[r]) + (int)(o.z > mine[r]) +
                     (int)(o.w > mine[r]);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 2; r++)
          if (tid + r * kOctLvlThreads < V) sortk[rk[r]] = mine[r];
        __syncthreads();
      } else {
        for (int k = 2; k <= P2; k <<= 1)
          for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = tid; i < P2; i += kOctLvlThreads) {
              const int ixj = i ^ jj;
              if (ixj > i) {
                const uint32_t x = sortk[i], y = sortk[ixj];
                const bool desc = (i & k) == 0;
                if (desc ? (x < y) : (x > y)) {
                  sortk[i] = y;
                  sortk[ixj] = x;
                }
              }
            }
            __syncthreads();
          }
      }
    }
    otick(1);
    auto nidx = [&](int j) { return outer ? j : 4095 - (int)(sortk[j] & 0xfffu); };
    auto is_cand = [&](int i, const OctNodeS& nn) { return outer ? node_n(nn) > 1 : cand[i] != 0; };
    // -- the key scan: quadrant one-hots of the candidates' keys, exclusive prefix per position
    uint32_t slo = 0, shi = 0;
    qbits = 0;
#pragma unroll
    for (int i = 0; i < kOctKpt; i++) {
      if (i < kpt) {
        uint32_t olo = 0, ohi = 0;
        if (kb0 + i < Kn) {
          const OctNodeS nn = Lc[nd[i]];
          if (is_cand(nd[i], nn)) {
            const uint32_t q = (uint32_t)quadrant(kr[i], node_xm(nn), node_ym(nn));
            qbits |= (uint64_t)q << (2 * i);
            const uint32_t oh = 1u << (16 * (q & 1));
            olo = q < 2 ? oh : 0u;
            ohi = q < 2 ? 0u : oh;
          }
        }
        plo[i] = slo;
        phi[i] = shi;
        slo += olo;
        shi += ohi;
      }
    }
    {
      int tl, th;
      const int el = wave_excl_scan((int)slo, lane, &tl);
      const int eh = wave_excl_scan((int)shi, lane, &th);
      if (lane == 0) {
        s_scan[w][0] = tl;
        s_scan[w][1] = th;
      }
      __syncthreads();
      uint32_t blo = (uint32_t)el, bhi = (uint32_t)eh;
      for (int k = 0; k < w; k++) {
        blo += (uint32_t)s_scan[k][0];
        bhi += (uint32_t)s_scan[k][1];
      }
#pragma unroll
      for (int i = 0; i < kOctKpt; i++) {
        if (i < kpt) {
          plo[i] += blo;
          phi[i] += bhi;
        }
      }
    }
    // segment boundaries: the prefix at a candidate node's first key and past its last
#pragma unroll
    for (int i = 0; i < kOctKpt; i++) {
      if (i < kpt && kb0 + i < Kn) {
        const int k = kb0 + i;
        const OctNodeS nn = Lc[nd[i]];
        if (is_cand(nd[i], nn)) {
          if (k == node_kbeg(nn)) nst[nd[i]] = make_uint2(plo[i], phi[i]);
          if (k == node_kbeg(nn) + node_n(nn) - 1) {
            const uint32_t q = (uint32_t)(qbits >> (2 * i)) & 3u;
            const uint32_t oh = 1u << (16 * (q & 1));
            nen[nd[i]] = make_uint2(plo[i] + (q < 2 ? oh : 0u), phi[i] + (q < 2 ? 0u : oh));
          }
        }
      }
    }
    __syncthreads();
    auto counts = [&](int i, int c[4]) {
      const uint2 a0 = nst[i], a1 = nen[i];
      const uint32_t dl = a1.x - a0.x, dh = a1.y - a0.y;
      c[0] = (int)(dl & 0xffffu);
      c[1] = (int)(dl >> 16);
      c[2] = (int)(dh & 0xffffu);
      c[3] = (int)(dh >> 16);
    };
    // -- count children: t (non-empty), e (> 1 key); pu = survivor flag (outer) or t - 1
    for (int j = tid; j < V; j += kOctLvlThreads) {
      const int i = nidx(j);
      const OctNodeS nn = Lc[i];
      const int n = node_n(nn);
      int t = 0, e = 0;
      if (n > 1) {
        int c[4];
        counts(i, c);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          t += c[q] > 0;
          e += c[q] > 1;
        }
      }
      pt[j] = (int16_t)t;
      pe[j] = (int16_t)e;
      pu[j] = (int16_t)(outer ? (n == 1) : t - 1);
    }
    for (int i = tid; i < m; i += kOctLvlThreads) cb[i] = -1;
    __syncthreads();
    otick(2);
    int nproc = V;
    if (!outer) {
      // processing stops once the list reaches N: first j with m + sum_{i<=j}(t_i - 1) >= N
      if (w == 0) {
        int carry = 0, np = V;
        for (int j0 = 0; j0 < V; j0 += 64) {
          const int j = j0 + lane;
          const int v = j < V ? pu[j] : 0;
          int tot;
          const int incl = carry + wave_excl_scan(v, lane, &tot) + v;
          const uint64_t hit = __ballot(j < V && m + incl >= N);
          if (hit) {
            np = j0 + __builtin_ctzll(hit) + 1;
            break;
          }
          carry += tot;
        }
        if (lane == 0) s_u[3] = np;
      }
      for (int i = tid; i < m; i += kOctLvlThreads) processed[i] = 0;
      __syncthreads();
      nproc = s_u[3];
      for (int j = tid; j < nproc; j += kOctLvlThreads) processed[nidx(j)] = 1;
      __syncthreads();
      for (int i = tid; i < m; i += kOctLvlThreads) pu[i] = (int16_t)(processed[i] ? 0 : 1);
      __syncthreads();
    }
    // push-order child positions, survivors' order: one array per wave
    if (w == 0) {
      const int t = wave_scan_array(pt, nproc, lane);
      if (lane == 0) s_u[0] = t;
    } else if (w == 1) {
      const int t = wave_scan_array(pe, nproc, lane);
      if (lane == 0) s_u[1] = t;
    } else if (w == 2) {
      const int t = wave_scan_array(pu, m, lane);
      if (lane == 0) s_u[2] = t;
    }
    __syncthreads();
    otick(3);
    const int T = s_u[0], E = s_u[1], U = s_u[2];
    const int newm = T + U;
    if (newm > NC || E > NC) {
      if (tid == 0) atomicOr(err, kErrNodeOverflow);
      break;
    }
    // -- children at their final list positions: push order gpos -> list position T-1-gpos
    for (int j = tid; j < nproc; j += kOctLvlThreads) {
      const int i = nidx(j);
      const OctNodeS nn = Lc[i];
      if (node_n(nn) <= 1) continue;
      int c[4];
      counts(i, c);
      int gpos = pt[j], epos = pe[j];
      cb[i] = (int16_t)gpos;
      const int xm = node_xm(nn), ym = node_ym(nn);
      const int16_t xs[3] = {nn.x0, (int16_t)xm, nn.x1};
      const int16_t ys[3] = {nn.y0, (int16_t)ym, nn.y1};
      int start = node_kbeg(nn);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (c[q] > 0) {
          OctNodeS ch;
          ch.x0 = xs[q & 1];
          ch.x1 = xs[(q & 1) + 1];
          ch.y0 = ys[q >> 1];
          ch.y1 = ys[(q >> 1) + 1];
          ch.kn = (uint32_t)start | (uint32_t)c[q] << 16;
          const int pos = T - 1 - gpos;
          Ln[pos] = ch;
          if (c[q] > 1) vnext[epos++] = (int16_t)pos;
          gpos++;
        }
        start += c[q];
      }
    }
    otick(4);
    for (int i = tid; i < m; i += kOctLvlThreads) {
      const OctNodeS nn = Lc[i];
      if (outer ? node_n(nn) == 1 : !processed[i]) Ln[T + pu[i]] = nn;
    }
    __syncthreads();
    // -- keys to their quadrant's range; each position's covering node in the new list
#pragma unroll
    for (int i = 0; i < kOctKpt; i++) {
      if (i < kpt && kb0 + i < Kn) {
        const int k = kb0 + i;
        const int o = nd[i];
        const int base = cb[o];
        if (base >= 0) {
          const OctNodeS nn = Lc[o];
          int c[4];
          counts(o, c);
          const uint2 s0 = nst[o];
          const uint32_t q = (uint32_t)(qbits >> (2 * i)) & 3u;
          const uint32_t dl = plo[i] - s0.x, dh = phi[i] - s0.y;
          const int rank = (int)(((q < 2 ? dl : dh) >> (16 * (q & 1))) & 0xffffu);
          int off = 0;
#pragma unroll
          for (int qq = 0; qq < 4; qq++) off += (uint32_t)qq < q ? c[qq] : 0;
          const int kb = node_kbeg(nn);
          keys[kb + off + rank] = kr[i];
          // the child whose range holds position k: ranges in quadrant order from kb
          const int r = k - kb;
          int cum = 0, nz = 0, child = 0;
#pragma unroll
          for (int qq = 0; qq < 4; qq++) {
            if (c[qq] > 0 && r >= cum) child = nz;
            nz += c[qq] > 0;
            cum += c[qq];
          }
          nd[i] = T - 1 - (base + child);
        } else {
          nd[i] = T + pu[o];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kOctKpt; i++)
      if (i < kpt && kb0 + i < Kn) kr[i] = keys[kb0 + i];
    for (int i = tid; i < E; i += kOctLvlThreads) sortk[i] = (uint32_t)vnext[i];
    __syncthreads();
    otick(5);
    const int mprev = m;
    m = newm;
    nexp = E;
    cur ^= 1;
    if (newm >= N || newm == mprev) break;
    if (outer && newm + E * 3 > N) outer = false;
  }
  // ---- 4. retain the best key of each node (:682-701): strict '>' keeps the first maximum
  __syncthreads();
  const OctNodeS* Lf = lists + cur * NC;
  const int mout = min(m, L.out_cap);
  for (int j = tid; j < mout; j += kOctLvlThreads) {
    const OctNodeS nd = Lf[j];
    const int kb = node_kbeg(nd), n = node_n(nd);
    uint32_t best = keys[kb];
    for (int k = 1; k < n; k++) {
      const uint32_t kk = keys[kb + k];
      if (key_score(kk) > key_score(best)) best = kk;
    }
    outk[j] = best;
  }
  if (tid == 0) {
    if (m > L.out_cap) atomicOr(err, kErrNodeOverflow);
    *outc = mout;
  }
}

// ---------------------------------------------------------------------------------------
// compile-time loops (lane selects and writelane lanes as immediates)
template <class F, int... J>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int kKpPerWave = 16;        // batches: keypoints per wave (two halves of 8)
constexpr int kKpPerWaveSmall = 4;    // launches up to kOdSmallMaxImages images
constexpr int kOdSmallMaxImages = 16;
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Sum of the 16 per-lane values v[] over the wave; value i ends up in lanes 4i..4i+3.
__device__ __forceinline__ int reduce_scatter16(int (&v)[16], int lane) {
  int w[8], x[4], y[2];
#pragma unroll
  for (int k = 0; k < 8; k++) {  // lanes 32-63 keep index k+8
    auto p = __builtin_amdgcn_permlane32_swap(v[k], v[k + 8], false, false);
    w[k] = (int)p[0] + (int)p[1];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {  // odd rows keep index +4
    auto p = __builtin_amdgcn_permlane16_swap(w[k], w[k + 4], false, false);
    x[k] = (int)p[0] + (int)p[1];
  }
  const bool up8 = lane & 8, up4 = lane & 4;
#pragma unroll
  for (int k = 0; k < 2; k++) {  // row_mirror: partner lane ^ 15
    const int send = up8 ? x[k] : x[k + 2];
    y[k] = (up8 ? x[k + 2] : x[k]) + __builtin_amdgcn_mov_dpp(send, 0x140, 0xf, 0xf, false);
  }
  const int send = up4 ? y[0] : y[1];  // row_half_mirror: partner lane ^ 7
  int z = (up4 ? y[1] : y[0]) + __builtin_amdgcn_mov_dpp(send, 0x141, 0xf, 0xf, false);
  z += __builtin_amdgcn_mov_dpp(z, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  z += __builtin_amdgcn_mov_dpp(z, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  return z;
}

// ---------------------------------------------------------------------------------------
// orient_desc: computeOrientation/IC_Angle (:413-420, :18-45) on the unblurred level, then
// computeOrbDescriptor (:49-88) on the level blurred by cv::GaussianBlur(7x7, sigma 2) (:1029-1030),
// with the blur folded in: no blurred pyramid is written or read back. The blur is separable
// with exact integer sums: a pixel is round(sum_i k_i R_i / 2^16), R_i = the row
// sums sum_j k_j I(y+i-3, x+j-3) <= 255 * 257 (u16).
// Per keypoint the row sums of its window (rows y-21..y+21, the columns the rotated samples can
// reach) come from the matrix cores: a banded int8 GEMM per 16 x 16 tile of the window
// (v_mfma_i32_16x16x64_i8: A = the window's bytes - 128 as int8, B = the 7 taps, accumulator
// initialised to 128 * 257, so the i32 result IS the u16 row sum), 3 x 3 tiles per keypoint. The
// A rows are mapped so that a lane's 12 accumulator elements are 12 consecutive window rows of one
// column; it packs them as u16 pairs (one v_perm per pair) and stores them with three
// ds_write_b64 into the wave's transposed u16 table. A sample's 7 vertical taps are then 4
// dwords of its column (two ds_read2_b32, a v_alignbit each for an odd first row) and four
// v_dot2_u32_u16. It rounds with the column's rule (half to even inside the SSE span
// x < W - W%4, half up in the scalar tail); inside the span a test compares the two biased
// sums' high halves directly.
// Border keypoints (the window leaves the image: reflect-101 rows and columns) gather the A bytes
// into the same staging slots; the GEMM and the table are the same.
// Variants measured in round 6 (profiles/r7*): an overlapping-pair table
// (dwords R[e] | R[e+1] << 16, no v_alignbit but twice the bytes stored: 0.87 vs 0.82 ms), A
// operands loaded straight from global memory (16 rows per quarter-wave), 8 keypoints per wave.
// Round 3-5 variants are in git history and DESIGN.md sections 9-11.
// The table per wave: kWCols columns (window column c = image column x - 18 - s + c, s the window
// origin's misalignment) x kUs u16 (rows 0..47, 43 used; 52 u16 = 26 dwords per column, so the 16
// lanes of a ds_write_b64 group hit 16 distinct bank pairs).
constexpr int kWCols = 40, kUs = 52;
constexpr int kWN = kWCols * kUs / 2;  // dwords
// The window staging area per wave: 48 rows x 64 bytes from the dword-aligned origin, filled by
// buffer-to-LDS loads in row order (four lanes per row: each load instruction's quarter-waves
// fetch four rows as whole lines) and read back in the MFMA's A layout (16 rows per quarter-wave,
// which as direct loads made every quarter-wave touch 16 lines). Within a row the four 16-byte
// chunks sit in the order chunk ^ swz(row), a table found by search that makes the A reads
// (ds_read_b128, 16-lane groups) bank-conflict free for the three tile rows.
constexpr int kWinRows = 48, kWinBytes = kWinRows * 64;
__device__ __forceinline__ int win_swz(int r) {
  const uint32_t t = r < 16 ? 0x330dbacdu : r < 32 ? 0x3a652155u : 0x159bb6u;
  return (int)((t >> (2 * (r & 15))) & 3u);
}

// KPW (<= kKpPerWave) keypoints per wave: 8 for batches, 4 for small launches (more waves in
// flight for the single-frame call)
template <int KPW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void orient_desc_kernel(
    ImageBatch b, const OrbGeom* __restrict__ g, const uint32_t* __restrict__ oct_keys,
    const int* __restrict__ oct_count, KeyPoint* __restrict__ kps, uint8_t* __restrict__ desc,
    int* __restrict__ nkps) {
  __shared__ __attribute__((aligned(16))) uint32_t s_w[4][kWN + 4];  // + a 16-byte front pad
  __shared__ __attribute__((aligned(16))) uint8_t s_win[4][kWinBytes];
  int img, bx;
  xcd_image_block(&img, &bx);
  const int lane = threadIdx.x & 63, wid = wave_id();
  int lcount[kMaxLevels];
  int total = 0;
  for (int l = 0; l < g->nlevels; l++) {
    lcount[l] = oct_count[img * g->nlevels + l];
    total += lcount[l];
  }
  if (bx == 0 && threadIdx.x == 0) nkps[img] = total;
  const int k0 = (bx * 4 + wid) * KPW;
  if (k0 >= total) return;
  const int nk = min(KPW, total - k0);
  int my_level = 0, my_key = 0;
  if (lane < nk) {
    int t = k0 + lane, l = 0;
    while (t >= lcount[l]) {
      t -= lcount[l];
      l++;
    }
    my_level = l;
    my_key = (int)oct_keys[(int64_t)img * g->out_per_image + g->lv[l].out_base + t];
  }
  // IC_Angle lane roles: two slots of 16 patch rows, four lanes per row. Lane (row r, k) loads 12
  // bytes at 8 k from the row's dword-aligned start (x - 15) & ~3 -- one 16-row x 36-byte block
  // per load instruction, so the patch's rows are fetched as whole lines (a 2-lanes-per-row map
  // with 5 dword loads touched every row 5 times: the texture data path, not the VALU, bound the
  // kernel) -- and realigns them into its two patch dwords 2 k, 2 k + 1 (columns 8 k .. 8 k + 7 of
  // x - 15 .. x + 15) with v_alignbyte; wt / one: the circle's u + 20 weights and 0/1 masks.
  const int ick = lane & 3;
  const int icv[2] = {(lane >> 2) - 15, (lane >> 2) + 1};
  uint32_t wt[2][2], one[2][2];
  {
    const uint4* t = reinterpret_cast<const uint4*>(g->od_ic[lane]);
    const uint4 w = t[0], o = t[1];
    wt[0][0] = w.x; wt[0][1] = w.y; wt[1][0] = w.z; wt[1][1] = w.w;
    one[0][0] = o.x; one[0][1] = o.y; one[1][0] = o.z; one[1][1] = o.w;
  }
  const int in_pitch = __builtin_amdgcn_readfirstlane(b.in_pitch);
  // every keypoint's window geometry computed once, lane j for keypoint j (vector loads of its
  // level's geometry), then read back per keypoint by v_readlane: the per-keypoint scalar chain
  // (level table loads, 64-bit pointer arithmetic, the window tests) was ~60 SALU instructions
  // per keypoint on the wave's issue stream. gv_k: x | y << 12 | level << 24 | aligned << 28 |
  // fastp << 31 (aligned: level base and pitch dword-aligned; fastp: aligned and the whole
  // 43 x 46 window inside the level)
  uint32_t gv_org_lo, gv_org_hi, gv_pitch, gv_wh, gv_k;
  {
    const LevelGeom& L = g->lv[my_level];
    const int kx = key_x((uint32_t)my_key) + kMinBorder, ky = key_y((uint32_t)my_key) + kMinBorder;
    const int w = L.w, h = L.h;
    const int pitch = my_level == 0 ? in_pitch : L.pitch;
    const uint8_t* im = my_level == 0 ? batch_image(b, img)
                                      : b.pyr + (int64_t)img * g->pyr_bytes + L.offset;
    const bool al = ((((uintptr_t)im | (uintptr_t)pitch) & 3) == 0);
    const bool fastp = al && kx >= 21 && kx <= w - 31 && ky >= 21 && ky + 21 < h;
    const uintptr_t org = (uintptr_t)(im + (int64_t)(ky - 21) * pitch + ((kx - 21) & ~3));
    gv_org_lo = (uint32_t)org;
    gv_org_hi = (uint32_t)(org >> 32);
    gv_pitch = (uint32_t)pitch;
    gv_wh = (uint32_t)w | (uint32_t)h << 16;
    gv_k = (uint32_t)kx | (uint32_t)ky << 12 | (uint32_t)my_level << 24 | (al ? 1u << 28 : 0u) |
           (fastp ? 1u << 31 : 0u);
  }
  // Phases 1-2: the IC_Angle patches (raw level, registers), kPh12Split keypoints at a time,
  // then their moments. The patch base is the window origin + 6 rows + ((x - 15) & ~3) -
  // ((x - 21) & ~3) (4 or 8) bytes: no level lookup per keypoint.
  typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
  constexpr int kPh12Split = 4;
  constexpr int KIC = KPW > 8 ? 16 : 8;  // keypoints whose angles the wave computes
  int mom[2];
#pragma unroll
  for (int g8 = 0; g8 < KIC / 8; g8++) {  // eight keypoints' moments, then their reduction
  int mv[16];
#pragma unroll
  for (int j0 = 8 * g8; j0 < 8 * g8 + 8; j0 += kPh12Split) {
    u32x3 raw[kPh12Split][2];
    int ash[kPh12Split];
#pragma unroll
    for (int jj = 0; jj < kPh12Split; jj++) {
      const int j = min(j0 + jj, nk - 1);
      const uint32_t k = (uint32_t)__builtin_amdgcn_readlane(gv_k, j);
      const int x = (int)(k & 0xfffu);
      const int pitch = __builtin_amdgcn_readlane(gv_pitch, j);
      const uintptr_t org = (uintptr_t)(uint32_t)__builtin_amdgcn_readlane(gv_org_lo, j) |
                            (uintptr_t)(uint32_t)__builtin_amdgcn_readlane(gv_org_hi, j) << 32;
      const uint8_t* rbase = reinterpret_cast<const uint8_t*>(org) + 6 * pitch +
                             (((x - 15) & ~3) - ((x - 21) & ~3));
      ash[jj] = (x - 15) & 3;
      if ((k >> 28) & 1u) {
        // buffer loads off the patch's (wave-uniform) base: no 64-bit address per lane; row 31
        // (the second slot's last four lanes) lies past the 31-row range and reads zeros
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)uniform_ptr(rbase), 0, 30 * pitch + 36, 0x00020000);
#pragma unroll
        for (int q = 0; q < 2; q++)
          raw[jj][q] = __builtin_amdgcn_raw_buffer_load_b96(
              rs, __umul24((uint32_t)(16 * q + (lane >> 2)), (uint32_t)pitch) + 8u * ick, 0, 0);
      } else {
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const int r = 16 * q + (lane >> 2);
          uint32_t w3[3] = {0, 0, 0};
          if (r < 31) {
            const uint8_t* rp = rbase + (int64_t)r * pitch + 8 * ick;
#pragma unroll
            for (int kk = 0; kk < 12; kk++) w3[kk >> 2] |= (uint32_t)rp[kk] << (8 * (kk & 3));
          }
          raw[jj][q] = (u32x3){w3[0], w3[1], w3[2]};
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < kPh12Split; jj++) {
      const int j = j0 + jj;
      const int a = ash[jj];
      int m10 = 0, m01 = 0;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t e0 = __builtin_amdgcn_alignbyte(raw[jj][q].y, raw[jj][q].x, a);
        const uint32_t e1 = __builtin_amdgcn_alignbyte(raw[jj][q].z, raw[jj][q].y, a);
        const uint32_t s = __builtin_amdgcn_udot4(e1, one[q][1], __builtin_amdgcn_udot4(e0, one[q][0], 0u, false), false);
        const uint32_t t = __builtin_amdgcn_udot4(e1, wt[q][1], __builtin_amdgcn_udot4(e0, wt[q][0], 0u, false), false);
        m10 += (int)t - 20 * (int)s;
        m01 += icv[q] * (int)s;
      }
      mv[2 * (j & 7)] = m10;
      mv[2 * (j & 7) + 1] = m01;
    }
    __asm__ volatile("" ::: "memory");
  }
  mom[g8] = reduce_scatter16(mv, lane);  // keypoint j: m10 at lanes 8 j.., m01 at 8 j + 4..
  }
  // the moments reduced over the wave: keypoint j's at lane 8 (j & 7) + 4 (j >> 3) (a DPP row
  // shift merges the second group of 8 into the lanes the first leaves free)
  int m10v, m01v;
  {
    const int mom0 = mom[0];
    m10v = mom0;
    m01v = __builtin_amdgcn_mov_dpp(mom0, 0x104, 0xf, 0xf, false);  // row_shl:4
    if constexpr (KIC > 8) {
      const int mom1 = mom[1];
      const int m10h = __builtin_amdgcn_mov_dpp(mom1, 0x114, 0xf, 0xf, false);  // row_shr:4
      const bool up = lane & 4;
      m10v = up ? m10h : m10v;
      m01v = up ? mom1 : m01v;
    }
  }
  auto angle_lane = [](int j) { return 8 * (j & 7) + 4 * (j >> 3); };
  const float angle = cv_fast_atan2((float)m01v, (float)m10v);
  const float factorPI = (float)(3.14159265358979323846 / 180.0);
  float sa, ca;
  glibc_sincosf(angle * factorPI, &sa, &ca);
  // Phase 3: per keypoint, the pair table (LDS) then the 512 blurred samples
  // the lane's 4 tests (8 points) as int8 (x0, y0, x1, y1) words: 4 VGPRs instead of 32
  // as float pairs (x, y): 16 VGPRs; the packed products broadcast x or y by op_sel
  f32x2 pf[8];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t pw = reinterpret_cast<const uint32_t*>(c_pattern)[r * 64 + lane];
#pragma unroll
    for (int e = 0; e < 2; e++)
      pf[2 * r + e] = (f32x2){(float)(int)(int8_t)(pw >> (16 * e)),
                              (float)(int)(int8_t)(pw >> (16 * e + 8))};
  }
  const uint32_t q0 = g->gauss[0], q1 = g->gauss[1], q2 = g->gauss[2], q3 = g->gauss[3];
  const uint32_t K01 = q0 | q1 << 16, K23 = q2 | q3 << 16, K21 = q2 | q1 << 16, K0 = q0;
  // magic + 18: a rounded sample coordinate comes out as its window index (round(x) + 18; 18 is
  // even, so round-half-even is unchanged)
  const f32x2 magic = {12582930.0f, 12582930.0f};
  uint32_t dlo = 0, dhi = 0;
  // MFMA lane roles (v_mfma_i32_16x16x64_i8): lane l holds row / column l & 15 of A / B and 16
  // bytes of K (lane group g = l >> 4), C[4 g + i][l & 15] in element i (tools/mfma_i8_probe.hip
  // checks the 16x16x32 form's map; only "A and B bytes b of lane group g share one K index" is
  // relied on here, and the parity tests pin it). A lane's 16 K bytes are window bytes 16 g ..
  // 16 g + 15 of its row (from the dword-aligned origin xa = (x - 21) & ~3): one 16-byte load, the
  // row's four lanes one 64-byte block. Output column 16 tj + n is the row sum of bytes
  // 16 tj + n .. + 6, so B is the band shifted by 16 tj: one operand per tile column.
  typedef int v4i __attribute__((ext_vector_type(4)));
  const int mf_n = lane & 15, mf_g = lane >> 4;
  v4i bm[3];
#pragma unroll
  for (int tj = 0; tj < 3; tj++) {
    const uint4 t = reinterpret_cast<const uint4*>(g->od_band[tj])[lane];
    bm[tj] = (v4i){(int)t.x, (int)t.y, (int)t.z, (int)t.w};
  }
  // A rows: tile row ti's row m is window row 12 (m >> 2) + 4 ti + (m & 3), so lane (n, g) ends up
  // with window rows 12 g .. 12 g + 11 of column n. Rows past 42 repeat row 42 (they only feed the
  // table's zero-weight pad): the loads stay inside the window's 43 rows.
  uint32_t arow[3];
#pragma unroll
  for (int ti = 0; ti < 3; ti++)
    arow[ti] = (uint32_t)min(12 * (mf_n >> 2) + 4 * ti + (mf_n & 3), 42);
  struct RsGeo {
    const uint8_t* org;  // window origin (xa, y - 21)
    int pitch, w, h, kx, ky, level;
    bool fastp;          // the whole window is inside the level: buffer loads, no reflection
  };
  auto rs_geo = [&](int j) {
    RsGeo G;
    const int jj = min(j, nk - 1);
    const uintptr_t org = (uintptr_t)(uint32_t)__builtin_amdgcn_readlane(gv_org_lo, jj) |
                          (uintptr_t)(uint32_t)__builtin_amdgcn_readlane(gv_org_hi, jj) << 32;
    G.org = reinterpret_cast<const uint8_t*>(org);
    G.pitch = __builtin_amdgcn_readlane(gv_pitch, jj);
    const uint32_t wh = (uint32_t)__builtin_amdgcn_readlane(gv_wh, jj);
    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane(gv_k, jj);
    G.w = (int)(wh & 0xffffu);
    G.h = (int)(wh >> 16);
    G.kx = (int)(k & 0xfffu);
    G.ky = (int)((k >> 12) & 0xfffu);
    G.level = (int)((k >> 24) & 0xfu);
    G.fastp = (k >> 31) != 0;
    return G;
  };
  // The window of a keypoint into the wave's staging area: slot 64 i + lane (16 bytes) holds row
  // 16 i + (lane >> 2) (rows past 42 repeat row 42), chunk (lane & 3) ^ swz(row). Fast path: three
  // buffer-to-LDS loads off the (wave-uniform) window origin, bounded by the window's 43 rows
  // (pitch >= 64: every load is inside them; bytes past x + 24 only feed output columns past the
  // table's 40). Border windows (reflect-101 rows and columns) gather bytes into the same slots.
  uint8_t* win = &s_win[wid][0];
  uint32_t dma_row[3], dma_off[3], a_lds[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int r = 16 * i + (lane >> 2);
    dma_row[i] = (uint32_t)min(r, 42);
    dma_off[i] = 16u * (uint32_t)((lane & 3) ^ win_swz(r));
    // the A read of tile row i: row arow[i], chunk g
    a_lds[i] = 16u * (4u * arow[i] + (uint32_t)(mf_g ^ win_swz((int)arow[i])));
  }
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto win_fill = [&](const RsGeo& G) {
    if (G.fastp) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)uniform_ptr(G.org), 0, 43 * G.pitch, 0x00020000);
#pragma unroll
      for (int i = 0; i < 3; i++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(win + 1024 * i), 16,
            __umul24(dma_row[i], (uint32_t)G.pitch) + dma_off[i], 0, 0, 0);
    } else {
      // a dword whose 4 columns are inside the level is one aligned load; only the dwords that
      // straddle or leave an edge gather bytes (divergent, few lanes)
      const int xa = (G.kx - 21) & ~3;
      const uint8_t* im = G.level == 0 ? batch_image(b, img)
                                       : b.pyr + (int64_t)img * g->pyr_bytes + g->lv[G.level].offset;
      const bool al = (((uintptr_t)im | (uintptr_t)G.pitch) & 3) == 0;
#pragma unroll
      for (int i = 0; i < 3; i++) {
        const uint8_t* row =
            im + (int64_t)reflect101(G.ky - 21 + (int)dma_row[i], G.h) * G.pitch;
        uint32_t wv[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
          const int c = xa + (int)dma_off[i] + 4 * d;
          if (al && c >= 0 && c + 3 < G.w) {
            wv[d] = *reinterpret_cast<const uint32_t*>(row + c);
          } else {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) v |= (uint32_t)row[reflect101(c + k, G.w)] << (8 * k);
            wv[d] = v;
          }
        }
        reinterpret_cast<uint4*>(win + 1024 * i)[lane] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    }
  };
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  uint32_t* tw = &s_w[wid][4];
  // the lane's first table dword of tile column 0: column n, row 12 g
  uint32_t* tw_lane = tw + mf_n * (kUs / 2) + 6 * mf_g;  // u16 row 12 g of column n
  // Software pipeline over the wave's keypoints: iteration j issues keypoint j's MFMAs, stores
  // keypoint j's table, issues the next keypoint's window loads, finishes keypoint j - 1's tests
  // from the table reads it issued last iteration (their latency covered by this iteration's
  // MFMAs and stores), then issues keypoint j's sample reads. The table is single-buffered: a
  // wave's LDS operations execute in order, so j's stores cannot overtake j - 1's reads.
  // byte address of u16 (c, r) = tw + 2 kUs c + 2 r, c = cx + 18 + s, r = cy + 18:
  // umul24(X, 2 kUs) + 2 Y + 2 kUs s - 2 kUs 0x400000 - 2 M
  const uint32_t rt_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint32_t*)tw -
                          2u * (uint32_t)kUs * 0x400000u - 2u * 0x4B400000u;
  constexpr uint32_t kColBytes = 2u * kUs;
  uint32_t wr[8][4];         // the pending keypoint's sample reads
  uint32_t wsh[8];           // ... and their realignment shifts (u16 table)
  bool tail_p = false;       // ... whether its window reaches the row's scalar tail
  uint32_t xt_p = 0;         // ... and that tail's first column bits
  f32x2 ab_p = {0.f, 0.f}, nab_p = {0.f, 0.f};  // ... and its rotation (the tail case recomputes X)
  // the lane's 8 samples of keypoint j: addresses, then all 16 reads in flight
  auto issue_reads = [&](int alane, const RsGeo& G) {
    const uint32_t sft = (uint32_t)((G.kx - 21) & 3);
    const float cj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ca), alane));
    const float sj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sa), alane));
    const f32x2 ab = {sj, cj}, nab = {cj, -sj};
    // A sample (cx, cy) reads column c = cx + 18 + s, u16 rows cy + 18 .. cy + 24: four aligned
    // dwords from the one holding the first, realigned (v_alignbit by 16 for an odd first row)
    // into the pairs (R0, R1), (R2, R3), (R4, R5), (R6, R7) for v_dot2 -- R7 meets K0's zero high
    // half. The byte address comes straight from the rounded coordinates' float bits
    // X = M + 18 + cx, Y = M + 18 + cy (M = 0x4B400000, low 24 bits 0x400000): see rt_lds.
    const uint32_t rt_base = rt_lds + kColBytes * sft;
    // stage by stage over the 8 samples: a dependent packed-f32 / VALU pair needs a wait state,
    // a sample-at-a-time chain issued one s_nop per step
    // sp = fma({px, px}, ab, {py, py} * nab) + magic, x and y broadcast from the pair
    f32x2 sp[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
      asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(sp[k]) : "v"(pf[k]), "s"(nab));
#pragma unroll
    for (int k = 0; k < 8; k++)
      asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]"
          : "+v"(sp[k]) : "v"(pf[k]), "s"(ab));
#pragma unroll
    for (int k = 0; k < 8; k++) sp[k] = sp[k] + magic;
    uint32_t ta[8];
#pragma unroll
    for (int k = 0; k < 8; k++)  // X * 2 kUs + rt_base in one v_mad_u32_u24 (X's low 24 bits)
      asm("v_mad_u32_u24 %0, %1, %2, %3"
          : "=v"(ta[k]) : "v"(__float_as_uint(sp[k].y)), "v"(kColBytes), "s"(rt_base));
#pragma unroll
    for (int k = 0; k < 8; k++) {
      // 4 aligned dwords from the dword holding row cy: u16 rows cy .. cy + 7 (+ one before
      // when cy is odd); the realignment shift (16 for odd cy) rides along in wsh
      const uint32_t a = (__float_as_uint(sp[k].x) << 1) + ta[k];
      const lds_u32* rw = (const lds_u32*)(uintptr_t)(a & ~3u);
      wr[k][0] = rw[0];
      wr[k][1] = rw[1];
      wr[k][2] = rw[2];
      wr[k][3] = rw[3];
      wsh[k] = __float_as_uint(sp[k].x) << 4;
    }
    // kTail: the window reaches the scalar tail of the row (x >= W - W % 4, rounded half up
    // instead of half to even) -- a wave-uniform case
    const int xvec = G.w - (G.w & 3);
    tail_p = G.kx + 18 >= xvec;
    xt_p = (uint32_t)(xvec - G.kx + 18) + 0x4B400000u;  // X >= this: tail
    ab_p = ab;
    nab_p = nab;
  };
  // keypoint j's 256 tests from the pending reads: descriptor dwords of lanes 4 j .. 4 j + 3
  auto finish = [&](auto jc) {  // the keypoint's index within its half
    constexpr int j = decltype(jc)::value;
    auto run = [&](auto tail_case) {
      constexpr bool kTail = decltype(tail_case)::value;
      // the 8 samples' sums level by level: consecutive v_dot2 are independent (a dependent one
      // needs wait states)
#pragma unroll
      for (int k = 0; k < 8; k++) {  // (R0, R1), (R2, R3), (R4, R5), (R6, R7 | 0)
        wr[k][0] = __builtin_amdgcn_alignbit(wr[k][1], wr[k][0], wsh[k]);
        wr[k][1] = __builtin_amdgcn_alignbit(wr[k][2], wr[k][1], wsh[k]);
        wr[k][2] = __builtin_amdgcn_alignbit(wr[k][3], wr[k][2], wsh[k]);
        wr[k][3] = __builtin_amdgcn_alignbit(0u, wr[k][3], wsh[k]);
      }
      uint32_t smv[8];
#pragma unroll
      for (int k = 0; k < 8; k++) smv[k] = dot2u(wr[k][3], K0, 0u);
#pragma unroll
      for (int k = 0; k < 8; k++) smv[k] = dot2u(wr[k][2], K21, smv[k]);
#pragma unroll
      for (int k = 0; k < 8; k++) smv[k] = dot2u(wr[k][1], K23, smv[k]);
#pragma unroll
      for (int k = 0; k < 8; k++) smv[k] = dot2u(wr[k][0], K01, smv[k]);
      uint64_t words[4];
      static_for<4>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if constexpr (!kTail) {
          // rounded half to even: o = (s + 0x7fff + bit 16 of s) >> 16, saturated to 255; the
          // test min(o_a, 255) < min(o_b, 255) is (a >> 16) < (b >> 16) && a < 255 << 16 on the
          // biased sums -- compared on their high halves (SDWA) with no shift or clamp
          const uint32_t a = smv[2 * r] + 0x7fffu + ((smv[2 * r] >> 16) & 1u);
          const uint32_t b = smv[2 * r + 1] + 0x7fffu + ((smv[2 * r + 1] >> 16) & 1u);
          words[r] = __ballot((a >> 16) < (b >> 16)) & __ballot(a < 0xff0000u);
          return;
        }
        uint32_t v[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int k = 2 * r + e;
          const uint32_t sm = smv[k];
          uint32_t o;
          if (kTail) {
            f32x2 pq, sp;  // the sample's column bits again (rare case: no VGPRs held for it)
            asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]"
                : "=v"(pq) : "v"(pf[k]), "s"(nab_p));
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1]"
                : "=v"(sp) : "v"(pf[k]), "s"(ab_p), "v"(pq));
            sp = sp + magic;
            const bool tail = __float_as_uint(sp.y) >= xt_p;
            o = (sm + (tail ? 0x8000u : 0x7fffu + ((sm >> 16) & 1u))) >> 16;
          } else {
            o = (sm + 0x7fffu + ((sm >> 16) & 1u)) >> 16;
          }
          v[e] = o > 255u ? 255u : o;
        }
        words[r] = __ballot(v[0] < v[1]);
      });
      // descriptor dword pairs of lanes 4 j .. 4 j + 3 (v_writelane: no per-lane select; the
      // lane selects are inline constants, j and r being compile-time). A v_writelane that reads
      // an SGPR a VALU compare has just written needs wait states (measured: without them bit
      // 7 of ~12 % of the descriptor bytes came out wrong), so the four ballots come first and
      // one s_nop covers them all.
      uint32_t lo = dlo, hi = dhi;  // (local copies: the asm operands of a nested lambda)
      asm volatile("s_nop 4\n\t"
                   "v_writelane_b32 %0, %2, %10\n\tv_writelane_b32 %1, %3, %10\n\t"
                   "v_writelane_b32 %0, %4, %11\n\tv_writelane_b32 %1, %5, %11\n\t"
                   "v_writelane_b32 %0, %6, %12\n\tv_writelane_b32 %1, %7, %12\n\t"
                   "v_writelane_b32 %0, %8, %13\n\tv_writelane_b32 %1, %9, %13"
                   : "+v"(lo), "+v"(hi)
                   : "s"((uint32_t)words[0]), "s"((uint32_t)(words[0] >> 32)),
                     "s"((uint32_t)words[1]), "s"((uint32_t)(words[1] >> 32)),
                     "s"((uint32_t)words[2]), "s"((uint32_t)(words[2] >> 32)),
                     "s"((uint32_t)words[3]), "s"((uint32_t)(words[3] >> 32)),
                     "i"(4 * j), "i"(4 * j + 1), "i"(4 * j + 2), "i"(4 * j + 3));
      dlo = lo;
      dhi = hi;
    };
    if (tail_p) run(std::true_type{});
    else run(std::false_type{});
  };
  RsGeo gn = rs_geo(0);
  win_fill(gn);
  // halves of KH keypoints: the keypoint loop unrolled within a half (its writelane lanes are
  // constants), the halves rolled; each half stores its keypoints' descriptors
  constexpr int KH = KPW < 8 ? KPW : 8;
  const int64_t o = (int64_t)img * g->kp_cap + k0;
#pragma unroll 1
  for (int h = 0; h < KPW / KH; h++) {
    if (KH * h >= nk) break;
    static_for<KH>([&](auto jc) {
    constexpr int jj = decltype(jc)::value;
    const int j = KH * h + jj;
    const RsGeo G = gn;
    // the window has landed (buffer-to-LDS loads count in vmcnt; border windows were stored by
    // this wave's own ds_writes, which its LDS reads follow in order): the A operands
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    u32x4 axn[3];
#pragma unroll
    for (int ti = 0; ti < 3; ti++) axn[ti] = *reinterpret_cast<const u32x4*>(win + a_lds[ti]);
    // keypoint j - 1's tests (their table reads were issued last iteration; this VALU covers the
    // A reads' latency, and the sample reads' registers are free again before the MFMA results
    // need theirs)
    if constexpr (jj > 0) finish(std::integral_constant<int, jj - 1>{});
    // the row sums: 9 MFMAs (A bytes - 128 as int8: x ^ 0x80)
    v4i acc[3][3];
    {
      const v4i cinit = {128 * 257, 128 * 257, 128 * 257, 128 * 257};
#pragma unroll
      for (int ti = 0; ti < 3; ti++) {
        const u32x4 x = axn[ti] ^ 0x80808080u;
        const v4i av = {(int)x.x, (int)x.y, (int)x.z, (int)x.w};
#pragma unroll
        for (int tj = 0; tj < 3; tj++)
          acc[ti][tj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bm[tj], cinit, 0, 0, 0);
      }
    }
    if (j + 1 < nk) {
      // the next keypoint's window: its loads overwrite the staging area this keypoint's A reads
      // came from, so they wait for those (the MFMAs above consumed them); none is issued past
      // the wave's last keypoint (no buffer-to-LDS load outlives the wave)
      gn = rs_geo(j + 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      win_fill(gn);
    }
    // the u16 table: lane (n, g) writes rows 12 g .. 12 g + 11 of column 16 tj + n as three
    // 8-byte stores (rows past 43 land in the column's spare rows); columns past 39 are outside
    // the table (tile column 2, n >= 8)
    auto st64 = [&](int tj) {
#pragma unroll
      for (int q = 0; q < 3; q++) {
        const uint32_t lo = __builtin_amdgcn_perm((uint32_t)acc[q][tj][1], (uint32_t)acc[q][tj][0], 0x05040100u);
        const uint32_t hi = __builtin_amdgcn_perm((uint32_t)acc[q][tj][3], (uint32_t)acc[q][tj][2], 0x05040100u);
        reinterpret_cast<uint2*>(tw_lane + 16 * tj * (kUs / 2))[q] = make_uint2(lo, hi);
      }
    };
    st64(0);
    st64(1);
    if (mf_n < 8) st64(2);
    __asm__ volatile("" ::: "memory");
    issue_reads(angle_lane(j), G);
    __asm__ volatile("" ::: "memory");
    });
    finish(std::integral_constant<int, KH - 1>{});
    if (lane < 4 * min(KH, nk - KH * h))
      reinterpret_cast<uint64_t*>(desc + (o + KH * h) * 32)[lane] = ((uint64_t)dhi << 32) | dlo;
  }
  const float my_angle = __shfl(angle, angle_lane(lane), 64);
  if (lane < nk) {
    const LevelGeom& L = g->lv[my_level];
    KeyPoint kp;
    kp.x = (float)(key_x((uint32_t)my_key) + kMinBorder);
    kp.y = (float)(key_y((uint32_t)my_key) + kMinBorder);
    if (my_level != 0) {
      kp.x *= L.scale;
      kp.y *= L.scale;
    }
    kp.size = L.patch_size;
    kp.angle = my_angle;
    kp.response = (float)key_score((uint32_t)my_key);
    kp.octave = my_level;
    kp.class_id = -1;
    kps[o + lane] = kp;
  }
}

// ---------------------------------------------------------------------------------------
// Host-side launchers.

// Which octree kernel a launch of n_images uses: the per-level work-groups for small batches
// (the single-frame call's critical path), one work-group per image otherwise.
// SLAMGPU_OCT_LVL=0 / 1 forces one of them (A/B and tests).
static bool octree_per_level(int n_images) {
  static const int mode = [] {
    const char* e = std::getenv("SLAMGPU_OCT_LVL");
    return e ? std::atoi(e) : -1;
  }();
  if (mode >= 0) return mode != 0;
  return n_images <= kOctLvlMaxImages;
}
void launch_extract(const ImageBatch& b, const OrbGeomDev& gd, int n_images, hipStream_t st,
                    const ExtractStreams& fx) {
  const OrbGeom& g = *gd.host;
  // glds tiles need every cell view 16-byte aligned: the caller's level-0 images included
  const bool glds = ((reinterpret_cast<uintptr_t>(b.in_l) | reinterpret_cast<uintptr_t>(b.in_r) |
                      (uintptr_t)b.in_stride | (uintptr_t)b.in_pitch |
                      reinterpret_cast<uintptr_t>(b.pyr) | (uintptr_t)g.pyr_bytes) & 15) == 0;
  // FAST of level 0 reads only the caller's images: with a second side stream it runs beside
  // the pyramid (whose small levels leave the chip mostly idle)
  // (batches only: in the single-frame call the join's cross-queue dependency costs more than
  // the overlap saves -- 0.296 -> 0.276 ms per call without it, profiles/r4w_lat_ab.log)
  const bool split0 = fx.side0 && fx.fork0 && fx.join0 && g.nlevels > 1 &&
                      n_images > kPyrShortMaxImages;
  if (split0) {
    (void)hipEventRecord(fx.fork0, st);
    (void)hipStreamWaitEvent(fx.side0, fx.fork0, 0);
  }
  auto fast_level0 = [&]() {
    const dim3 block(64 * kCellWaves);
    const size_t lds = (size_t)kCellWaves * g.fast_lds_per_wave;
    const int lo = 0, hi = g.lv[1].cell_base;
    const dim3 grid((hi - lo + kCellWaves * kCellsPerWave - 1) / (kCellWaves * kCellsPerWave),
                    n_images);
    hipStream_t fs = fx.side0;
    if (g.fast_tile_stride == 64) {
      if (glds)
        SLAMGPU_LAUNCH("fast_cells", fs, (fast_cells_kernel<64, true>), grid, block, lds, fs, b,
                       gd.dev, gd.cells, gd.ws.cell_keys, gd.ws.cell_count, gd.ws.err, lo, hi);
      else
        SLAMGPU_LAUNCH("fast_cells", fs, (fast_cells_kernel<64, false>), grid, block, lds, fs, b,
                       gd.dev, gd.cells, gd.ws.cell_keys, gd.ws.cell_count, gd.ws.err, lo, hi);
    } else {
      if (glds)
        SLAMGPU_LAUNCH("fast_cells", fs, (fast_cells_kernel<128, true>), grid, block, lds, fs, b,
                       gd.dev, gd.cells, gd.ws.cell_keys, gd.ws.cell_count, gd.ws.err, lo, hi);
      else
        SLAMGPU_LAUNCH("fast_cells", fs, (fast_cells_kernel<128, false>), grid, block, lds, fs,
                       b, gd.dev, gd.cells, gd.ws.cell_keys, gd.ws.cell_count, gd.ws.err, lo, hi);
    }
    (void)hipEventRecord(fx.join0, fs);
  };
  if (split0) fast_level0();
  const bool in_aligned = (((uintptr_t)b.in_l | (uintptr_t)b.in_r | (uintptr_t)b.in_stride |
                           (uintptr_t)b.in_pitch) & 3) == 0;
  const bool short_strips = n_images <= kPyrShortMaxImages;
  // batches: the LDS-staged strips (16-byte buffer-to-LDS loads need 16-byte aligned rows)
  static const int ring_mode = [] {
    const char* e = std::getenv("SLAMGPU_PYR_RING");
    return e ? std::atoi(e) : 0x7ffffffe;  // every level >= 1
  }();
  // SLAMGPU_PYR_RING: bit l selects the LDS-staged kernel for level l (A/B)
  const bool ring_ok = glds && g.pyr_ring_slots > 0 && g.pyr_ring_slots <= 8;
  // small launches: level 1 over the chip, then levels 2+ in one launch of row bands
  // SLAMGPU_PYR_CASCADE=1: batches take the whole pyramid in one cascade launch where the
  // geometry allows it. Not the default: it is 0.57 ms standalone against the per-level
  // launches' 0.69, but its lanes idle in the steps their level emits nothing (186M VALU
  // wave-instructions against 134M) and it holds every CU for its whole run, so level 0's FAST
  // beside it stretches 0.68 -> 0.98 ms and the step gets slower, 2.45 -> 2.57 ms
  // (profiles/r8c_pyr_cascade_ab.log). Read per launch, so that tests can exercise both paths.
  const char* cenv = std::getenv("SLAMGPU_PYR_CASCADE");
  const bool cascade = cenv && std::atoi(cenv) != 0 && glds && !short_strips && g.casc_waves > 0;
  const int l_end = cascade ? 1 : (short_strips && g.pyr_bands > 0) ? 2 : g.nlevels;
  // SLAMGPU_PYR_SHORT_FROM=l: batches take short strips (more waves, shorter row chains) from
  // level l on (A/B)
  static const int short_from = [] {
    const char* e = std::getenv("SLAMGPU_PYR_SHORT_FROM");
    return e ? std::atoi(e) : kMaxLevels;
  }();
  for (int l = 1; l < l_end; l++) {
    const bool shortl = short_strips || l >= short_from;
    const bool ring = ring_ok && !shortl && ((ring_mode >> l) & 1);
    const int strip = shortl ? kPyrShortStrip : ring ? kPyrRingStrip : kPyrStrip;
    const int tiles = ((g.lv[l].w + 255) >> 8) * ((g.lv[l].h + 4 * strip - 1) / (4 * strip));
    const dim3 grid(tiles, n_images);
    if (shortl) {
      if (l > 1 || in_aligned)
        SLAMGPU_LAUNCH("pyr_down", st, (pyr_down_kernel<true, kPyrShortStrip>), grid, dim3(256), 0,
                       st, b, gd.dev, l, gd.rx, gd.ry);
      else
        SLAMGPU_LAUNCH("pyr_down", st, (pyr_down_kernel<false, kPyrShortStrip>), grid, dim3(256),
                       0, st, b, gd.dev, l, gd.rx, gd.ry);
    } else if (ring) {
      SLAMGPU_LAUNCH("pyr_down", st, pyr_ring_kernel, grid, dim3(256),
                     (size_t)4096 * g.pyr_ring_slots, st, b, gd.dev, l, gd.rx, gd.ry);
    } else if (l > 1 || in_aligned) {
      SLAMGPU_LAUNCH("pyr_down", st, (pyr_down_kernel<true, kPyrStrip>), grid, dim3(256), 0, st,
                     b, gd.dev, l, gd.rx, gd.ry);
    } else {
      SLAMGPU_LAUNCH("pyr_down", st, (pyr_down_kernel<false, kPyrStrip>), grid, dim3(256), 0, st,
                     b, gd.dev, l, gd.rx, gd.ry);
    }
  }
  if (cascade)
    SLAMGPU_LAUNCH("pyr_down", st, pyr_cascade_kernel, dim3(n_images), dim3(64 * (g.casc_waves + 1)),
                   (size_t)g.casc_lds, st, b, gd.dev, gd.rx, gd.ry);
  else if (l_end < g.nlevels)
    SLAMGPU_LAUNCH("pyr_down", st, pyr_band_kernel, dim3(g.pyr_bands, n_images),
                   dim3(64 * kPyrBandWaves), 2 * (size_t)g.pyr_band_lds, st, b, gd.dev, gd.rx,
                   gd.ry);
  {
    const dim3 block(64 * kCellWaves);
    const size_t lds = (size_t)kCellWaves * g.fast_lds_per_wave;
    auto fast = [&](int lo, int hi, hipStream_t fs) {
      const dim3 grid((hi - lo + kCellWaves * kCellsPerWave - 1) / (kCellWaves * kCellsPerWave),
                      n_images);
#define SLAMGPU_FAST(TS, GL)                                                                \
  do {                                                                                      \
    auto* kfn = &fast_cells_kernel<TS, GL>;                                                 \
    SLAMGPU_LAUNCH("fast_cells", fs, kfn, grid, block, lds, fs, b, gd.dev, gd.cells,        \
                   gd.ws.cell_keys, gd.ws.cell_count, gd.ws.err, lo, hi);                   \
  } while (0)
      if (g.fast_tile_stride == 64) {
        if (glds) SLAMGPU_FAST(64, true); else SLAMGPU_FAST(64, false);
      } else {
        if (glds) SLAMGPU_FAST(128, true); else SLAMGPU_FAST(128, false);
      }
#undef SLAMGPU_FAST
    };
    if (split0) {  // level 0 already ran beside the pyramid
      fast(g.lv[1].cell_base, g.cells_per_image, st);
      (void)hipStreamWaitEvent(st, fx.join0, 0);
    } else {
      fast(0, g.cells_per_image, st);
    }
  }
  // the per-level kernel redoes its oversized levels itself (its LDS sized for the global
  // algorithm's scratch too): no octree_kernel launch after it -- the single-frame call's chain
  // is one dependent launch shorter; after the per-image kernel octree_kernel does them
  const bool lvl = g.oct_kcap == 0 || octree_per_level(n_images);
  if (lvl)
    SLAMGPU_LAUNCH("octree", st, octree_lvl_kernel, dim3(g.nlevels, n_images),
                   dim3(kOctLvlThreads), std::max((size_t)g.oct2_lds_bytes, sizeof(OctShared)),
                   st, gd.dev, gd.ws.cell_keys, gd.ws.cell_count, gd.ws.key_scratch,
                   gd.ws.node_scratch, gd.ws.oct_keys, gd.ws.oct_count, gd.ws.err);
  else
    SLAMGPU_LAUNCH("octree", st, octree_img_kernel, dim3(n_images), dim3(64 * g.nlevels),
                   (size_t)g.oct_lds_bytes, st, gd.dev, gd.ws.cell_keys, gd.ws.cell_count,
                   gd.ws.key_scratch, gd.ws.oct_keys, gd.ws.oct_count, gd.ws.err);
  if (!lvl) {
    const int groups = std::min(g.nlevels * n_images, kOctFbMaxGroups);
    SLAMGPU_LAUNCH("octree_global", st, octree_kernel, dim3(groups), dim3(kOctThreads), 0, st,
                   gd.dev, n_images, gd.ws.cell_keys, gd.ws.cell_count, gd.ws.key_scratch,
                   gd.ws.node_scratch, gd.ws.oct_keys, gd.ws.oct_count, gd.ws.err);
  }
  if (n_images <= kOdSmallMaxImages) {
    constexpr int kpw = kKpPerWaveSmall;
    SLAMGPU_LAUNCH("orient_desc", st, orient_desc_kernel<kpw>,
                   dim3((g.kp_cap + 4 * kpw - 1) / (4 * kpw), n_images), dim3(256), 0, st, b,
                   gd.dev, gd.ws.oct_keys, gd.ws.oct_count, gd.out.kps, gd.out.desc, gd.out.nkps);
  } else {
    SLAMGPU_LAUNCH("orient_desc", st, orient_desc_kernel<kKpPerWave>,
                   dim3((g.kp_cap + 4 * kKpPerWave - 1) / (4 * kKpPerWave), n_images), dim3(256),
                   0, st, b, gd.dev, gd.ws.oct_keys, gd.ws.oct_count, gd.out.kps, gd.out.desc,
                   gd.out.nkps);
  }
}

bool extract_build_matches(const OrbGeom& g) {
  return g.pyr_ring_strip == kPyrRingStrip && g.cell_group == kCellsPerWave;
}

hipError_t octree_lds_limits(int device, int* img_bytes, int* lvl_bytes) {
  int max_lds = 0;
  hipError_t e = hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
  if (e != hipSuccess) return e;
  hipFuncAttributes a{};
  if ((e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&octree_img_kernel))) != hipSuccess)
    return e;
  *img_bytes = max_lds - (int)a.sharedSizeBytes;
  if ((e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&octree_lvl_kernel))) != hipSuccess)
    return e;
  // the per-level kernel's dynamic LDS is at least the global algorithm's OctShared
  *lvl_bytes = max_lds - (int)a.sharedSizeBytes;
  if (*lvl_bytes < (int)sizeof(OctShared)) *lvl_bytes = 0;
  return hipSuccess;
}

}  // namespace slamgpu
