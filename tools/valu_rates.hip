// Issue rate of the VALU instructions the front-end kernels are built from, chip-wide, at 1..8
// waves per SIMD: each wave runs N iterations of 8 independent dependency chains of one
// instruction; rate = wave-instructions per second against 256 CUs x 4 SIMD x 2.4 GHz / 2.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates && tools/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096, kChains = 8;

#define OPK(NAME, T, EXPR)                                                            \
  __global__ __launch_bounds__(256) void k_##NAME(T* out, T c1, T c2) {              \
    T x[kChains];                                                                     \
    for (int k = 0; k < kChains; k++) x[k] = (T)(threadIdx.x + k);                    \
    for (int i = 0; i < kIters; i++) {                                                \
      _Pragma("unroll") for (int k = 0; k < kChains; k++) { T v = x[k]; x[k] = EXPR; } \
    }                                                                                 \
    T s = x[0];                                                                       \
    for (int k = 1; k < kChains; k++) s = s ^ x[k];                                   \
    out[blockIdx.x * 256 + threadIdx.x] = s;                                          \
  }

OPK(add_u32, uint32_t, v + c1)
OPK(udot4, uint32_t, __builtin_amdgcn_udot4(v, c1, c2, false))
OPK(udot2, uint32_t, __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v), __builtin_bit_cast(u16x2, c1), c2, false))
OPK(alignbit, uint32_t, __builtin_amdgcn_alignbit(v, c1, c2))
OPK(alignbyte, uint32_t, __builtin_amdgcn_alignbyte(v, c1, c2))
OPK(perm, uint32_t, __builtin_amdgcn_perm(v, c1, c2))
OPK(mad_u24, uint32_t, __umul24(v, c1) + c2)
OPK(lshl_add, uint32_t, (v << 3) + c1)
OPK(bfe, uint32_t, __builtin_amdgcn_ubfe(v, c1 & 15, 8))
OPK(min_u32, uint32_t, (v < c1 ? v : c1) + c2)
OPK(mul_lo, uint32_t, v * c1)
OPK(add_xor, uint32_t, (v + c1) ^ c2)                       // 2 instructions
OPK(lshl_or, uint32_t, (v << 5) | c1)
OPK(add3, uint32_t, v + c1 + (v >> 3))                     // lshr + add3
OPK(xor_only, uint32_t, v ^ c1 ^ (v >> 2))                  // lshr + xor3?
OPK(bfe_add3, uint32_t, v + c1 + __builtin_amdgcn_ubfe(v, 16, 1))
OPK(cndmask, uint32_t, (v & 1) ? c1 : v + c2)
OPK(mad_u32_u24, uint32_t, __umul24(v, c1) + v)

__global__ __launch_bounds__(256) void k_pk_fma(float* out, float c1, float c2) {
  f32x2 x[kChains];
  const f32x2 a = {c1, c2}, b = {c2, c1};
  for (int k = 0; k < kChains; k++) x[k] = (f32x2){(float)threadIdx.x, (float)k};
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int k = 0; k < kChains; k++) x[k] = __builtin_elementwise_fma(x[k], a, b);
  }
  float s = 0;
  for (int k = 0; k < kChains; k++) s += x[k].x + x[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_cvt_f32_i32(float* out, float c1, float c2) {
  int x[kChains];
  for (int k = 0; k < kChains; k++) x[k] = threadIdx.x + k;
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int k = 0; k < kChains; k++) x[k] = __float_as_int((float)x[k]);
  }
  float s = 0;
  for (int k = 0; k < kChains; k++) s += (float)x[k];
  out[blockIdx.x * 256 + threadIdx.x] = s + c1 + c2;
}

template <typename K, typename T>
static void run(const char* name, K kern, T c1, T c2, T* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("%-12s", name);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * w;  // 256 threads = one wave per SIMD per block
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, c1, c2);
    hipEventRecord(e0);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, c1, c2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr = 3.0 * blocks * 4.0 * kIters * kChains;
    const double peak = cus * 4.0 * 2.4e9 / 2.0;
    printf("  w%d %.3f", w, instr / (ms * 1e-3) / peak);
  }
  printf("   (fraction of the 2-cycle wave64 issue peak)\n");
}

// LDS gather throughput: 8 waves per SIMD, each lane reads random u16 / dword pairs from a 3.5 KB
// per-wave table (the orient_desc row-sum window)
template <int MODE>
__global__ __launch_bounds__(256) void k_lds(uint32_t* out, uint32_t seed, uint32_t c2) {
  __shared__ uint16_t t[4][1760];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = lane; i < 1760; i += 64) t[w][i] = (uint16_t)(i * 7 + seed);
  __syncthreads();
  uint32_t x = lane * 2654435761u + seed, acc = 0;
  for (int i = 0; i < 512; i++) {
    x = x * 1664525u + 1013904223u;
    const uint32_t e = ((x >> 8) & 1023u) + (uint32_t)(lane & 7) * 89u;
    if (MODE == 0) {  // 7 u16 reads (immediate offsets)
      const uint16_t* p = &t[w][e];
      acc += p[0] + p[1] + p[2] + p[3] + p[4] + p[5] + p[6];
    } else {          // 4 dwords (2 x read2) at the containing dword
      const uint32_t* p = reinterpret_cast<const uint32_t*>(&t[w][0]) + (e >> 1);
      acc += p[0] + p[1] + p[2] + p[3];
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc + c2;
}

int main() {
  void* out = nullptr;
  hipMalloc(&out, 256 * 2048 * 8);
  uint32_t* u = (uint32_t*)out;
  float* f = (float*)out;
  run("add_u32", k_add_u32, 3u, 5u, u);
  run("udot4", k_udot4, 0x01020304u, 7u, u);
  run("udot2", k_udot2, 0x00030004u, 7u, u);
  run("alignbit", k_alignbit, 0x12345678u, 16u, u);
  run("alignbyte", k_alignbyte, 0x12345678u, 1u, u);
  run("perm", k_perm, 0x12345678u, 0x05040100u, u);
  run("mad_u24", k_mad_u24, 3u, 5u, u);
  run("lshl_add", k_lshl_add, 3u, 5u, u);
  run("bfe", k_bfe, 3u, 5u, u);
  run("min_u32", k_min_u32, 3000u, 5u, u);
  run("mul_lo", k_mul_lo, 3u, 5u, u);
  run("add_xor(2)", k_add_xor, 3u, 5u, u);
  run("lshl_or", k_lshl_or, 3u, 5u, u);
  run("add3(2)", k_add3, 3u, 5u, u);
  run("xor3(2)", k_xor_only, 3u, 5u, u);
  run("bfe_add3(2)", k_bfe_add3, 3u, 5u, u);
  run("cndmask(3)", k_cndmask, 3u, 5u, u);
  run("mad_u24_add", k_mad_u32_u24, 3u, 5u, u);
  run("lds_u16x7", k_lds<0>, 3u, 5u, u);
  run("lds_2xread2", k_lds<1>, 3u, 5u, u);
  run("pk_fma_f32", k_pk_fma, 0.5f, 0.25f, f);
  run("cvt_f32_i32", k_cvt_f32_i32, 0.5f, 0.25f, f);
  hipFree(out);
  return 0;
}
