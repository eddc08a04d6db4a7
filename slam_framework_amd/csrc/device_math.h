// device_math.h -- bit-exact device versions of the float semantics the hot path depends on.
//
// Built with -ffp-contract=off: every fused multiply-add below is an explicit fma()/fmaf(),
// placed where the reference's Release build (or the library it calls) fuses.
//   - glibc 2.35 sinf/cosf, x86-64 FMA variant (reference: std::cos(float)/std::sin(float) at
//     src/orb_features/orb_extractor.cpp:54). Double-precision polynomial on the VALU.
//   - OpenCV 3.3.1 fastAtan2 (reference: orb_extractor.cpp:44), no FMA.
//   - cvRound(float) = round half to even (v_rndne_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace slamgpu {

struct SinCosTable {
  double sign[4];
  double hpi_inv, hpi;
  double c0, c1, s1, c2, s2, c3, s3, c4;
};

__device__ __forceinline__ const SinCosTable& sincos_table(int k) {
  // Same constants as libm's __sincosf_table (second record negates the cosine terms).
  static __device__ __constant__ SinCosTable t[2] = {
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p+0,
       -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
       0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,
       0x1.99343027bf8c3p-16},
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p+0,
       0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
       0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13,
       -0x1.99343027bf8c3p-16}};
  return t[k];
}

__device__ __forceinline__ float sc_sin_poly(double x, double x2, const SinCosTable& p) {
  double s1 = fma(x2, p.s3, p.s2);
  double x3 = x2 * x;
  double x7 = x2 * x3;
  double s = fma(x3, p.s1, x);
  return (float)fma(s1, x7, s);
}

__device__ __forceinline__ float sc_cos_poly(double x2, const SinCosTable& p) {
  double x4 = x2 * x2;
  double c1 = fma(x2, p.c1, p.c0);
  double c2 = fma(x2, p.c4, p.c3);
  double x6 = x2 * x4;
  double c = fma(x4, p.c2, c1);
  return (float)fma(c2, x6, c);
}

// sin and cos of one float, as glibc's separate sinf() and cosf() calls return them.
// Valid for |y| < 120 (keypoint angles are in [0, 2pi)); larger inputs fall back to libm.
__device__ __forceinline__ void glibc_sincosf(float y, float* sout, float* cout) {
  const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ff;
  const double x = (double)y;
  if (top < 0x3f4) {
    if (top < 0x398) {
      *sout = y;
      *cout = 1.0f;
      return;
    }
    const double x2 = x * x;
    *sout = sc_sin_poly(x, x2, sincos_table(0));
    *cout = sc_cos_poly(x2, sincos_table(0));
    return;
  }
  if (top < 0x42f) {
    const SinCosTable& t0 = sincos_table(0);
    const double r = x * t0.hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double xr = fma(-(double)n, t0.hpi, x);
    const SinCosTable& p = sincos_table((n & 2) ? 1 : 0);
    const double x2 = xr * xr;
    const double xs = xr * t0.sign[n & 3];
    if ((n & 1) == 0) {
      *sout = sc_sin_poly(xs, x2, p);
      *cout = sc_cos_poly(x2, p);
    } else {
      *sout = sc_cos_poly(x2, p);
      *cout = sc_sin_poly(xs, x2, p);
    }
    return;
  }
  *sout = sinf(y);
  *cout = cosf(y);
}

// cv::fastAtan2 (OpenCV 3.3.1, degrees in [0, 360)).
__device__ __forceinline__ float cv_fast_atan2(float y, float x) {
  const float k180pi = (float)(180.0 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k180pi;
  const float p3 = -0.3258083974640975f * k180pi;
  const float p5 = 0.1555786518463281f * k180pi;
  const float p7 = -0.04432655554792128f * k180pi;
  const float eps = (float)2.2204460492503131e-16;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// A wave-uniform pointer as such (its value read from the first active lane into SGPRs).
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// A raw buffer descriptor over `bytes` bytes at the wave-uniform address p: loads through it take
// a 32-bit lane offset (+ a scalar one) instead of a 64-bit address computed per lane.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int bytes = 0x7ffffff0) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(p), 0, bytes, 0x00020000);
}

__device__ __forceinline__ int cv_round(float v) { return (int)rintf(v); }
__device__ __forceinline__ int max3(int a, int b, int c) { return max(max(a, b), c); }
// high 32 bits of a 24 x 24-bit product (v_mul_hi_u32_u24); a, b < 2^24
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)(a & 0xffffffu) * (uint64_t)(b & 0xffffffu)) >> 32);
}

// glibc 2.35 logf, x86-64 FMA variant (__logf_fma; reference: std::log(float) in
// MapPoint::PredictScale, src/data/map_point.cpp:372). Same table and polynomial as libm's
// __logf_data; oracle/oc_logf is pinned against host logf on every positive float. Inputs here
// are finite and positive (max_dist / dist); 0, inf and nan follow glibc too.
__device__ __forceinline__ float glibc_logf(float x) {
  static __device__ __constant__ double tab[16][2] = {
      {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
      {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
      {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
      {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
      {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
      {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
      {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
      {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
  uint32_t ix = __float_as_uint(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -__builtin_inff();
    if (ix == 0x7f800000u) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
    ix = __float_as_uint(x * 0x1p23f) - (23u << 23);
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) & 15);
  const int k = (int32_t)tmp >> 23;
  const double z = (double)__uint_as_float(ix - (tmp & 0xff800000u));
  const double r = fma(z, tab[i][0], -1.0);
  const double y0 = fma((double)k, 0x1.62e42fefa39efp-1, tab[i][1]);
  const double r2 = r * r;
  double y = fma(0x1.5575b0be00b6ap-2, r, -0x1.ffffef20a4123p-2);
  y = fma(-0x1.00ea348b88334p-2, r2, y);
  y = fma(y, r2, y0 + r);
  return (float)y;
}

// ---- wavefront (64-lane) helpers --------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }
// Wave index inside the workgroup, as a scalar (the compiler cannot prove threadIdx.x >> 6 is
// wave-uniform; without this every address derived from it is computed per lane).
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

// XCD-aware (image, block) of a (blocks per image, images) grid: workgroups are dealt
// round-robin over the 8 XCDs by linear id, so give every block of one image the same
// (linear id % 8) -- an image's rows then stay in one XCD's L2, where neighbouring blocks share
// their halo lines. Bijective when the image count is a multiple of 8; otherwise natural order.
__device__ __forceinline__ void xcd_image_block(int* img, int* bx) {
  const int bpi = gridDim.x;
  *img = blockIdx.y;
  *bx = blockIdx.x;
  if ((gridDim.y & 7) == 0) {
    const int lin = blockIdx.x + blockIdx.y * bpi;
    const int j = lin >> 3;
    *img = (lin & 7) + 8 * (j / bpi);
    *bx = j % bpi;
  }
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    T o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    T o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// The value of the partner lane in a butterfly whose level M (32, 16, ..., 1) pairs lanes that
// differ in bit log2(M) and agree above it: lane ^ 32 and lane ^ 16 through the gfx950 permlane
// swaps, lane ^ 15, ^ 7, ^ 3 (row mirror, half-row mirror, quad reverse) and ^ 1 through DPP --
// no LDS round trip (ds_bpermute). Each level is an xor with a constant, so levels 32 .. 1
// together reach all 64 lanes, and a butterfly that adds own + partner leaves every lane of a
// group with the same bits (IEEE addition commutes).
__device__ __forceinline__ uint32_t lane_partner_u32(uint32_t v, int M) {
  const int lane = __lane_id();
  switch (M) {
    case 32: {  // lanes 32-63 of the first operand <-> lanes 0-31 of the second
      const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      return (lane & 32) ? r[0] : r[1];
    }
    case 16: {  // odd rows of the first operand <-> even rows of the second
      const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
      return (lane & 16) ? r[0] : r[1];
    }
    case 8: return __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xf, 0xf, false);  // row_mirror
    case 4: return __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xf, 0xf, false);  // row_half_mirror
    case 2: return __builtin_amdgcn_update_dpp(0u, v, 0x1b, 0xf, 0xf, false);   // quad [3,2,1,0]
    default: return __builtin_amdgcn_update_dpp(0u, v, 0xb1, 0xf, 0xf, false);  // quad [1,0,3,2]
  }
}
__device__ __forceinline__ double lane_partner(double v, int M) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint64_t lo = lane_partner_u32((uint32_t)b, M), hi = lane_partner_u32((uint32_t)(b >> 32), M);
  return __builtin_bit_cast(double, hi << 32 | lo);
}

// Number of set bits of `mask` strictly below this lane.
__device__ __forceinline__ int lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

}  // namespace slamgpu
