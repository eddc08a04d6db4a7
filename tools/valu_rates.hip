// Issue rate of the VALU instructions the front-end kernels are built from, chip-wide, at 1..8
// waves per SIMD. Each wave runs kIters iterations of kChains independent dependency chains of
// ONE instruction, written as inline asm so that the compiler can neither fold a chain (the
// round-4 probe's `v + c1` chains were strength-reduced to one add, which is how add_u32 and
// mul_lo read 3x "the peak") nor change the instruction. rate = wave-instructions per second
// against the nominal issue rate 256 CUs x 4 SIMD x 2.4 GHz / 2 (one wave64 VALU instruction per
// 2 cycles per SIMD-32, MI355X_MICROARCH.md). Run it under
//   rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -- tools/valu_rates
// to check the per-dispatch instruction count against kIters x kChains x waves (+ the epilogue).
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates && tools/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kIters = 2048, kChains = 8;

// one instruction per chain step: "INS %0, %0, %1[, %2]" with x as the destination and first
// source, c1 / c2 wave-uniform VGPRs
#define OPK(NAME, ASM)                                                               \
  __global__ __launch_bounds__(256) void k_##NAME(uint32_t* out, uint32_t c1, uint32_t c2) { \
    uint32_t x[kChains];                                                             \
    const uint32_t a = c1 + threadIdx.x, b = c2 ^ threadIdx.x;                        \
    for (int k = 0; k < kChains; k++) x[k] = threadIdx.x * 0x01010101u + k;          \
    for (int i = 0; i < kIters; i++) {                                               \
      _Pragma("unroll") for (int k = 0; k < kChains; k++)                            \
        asm volatile(ASM : "+v"(x[k]) : "v"(a), "v"(b));                             \
    }                                                                                \
    uint32_t s = x[0];                                                               \
    for (int k = 1; k < kChains; k++) s ^= x[k];                                     \
    out[blockIdx.x * 256 + threadIdx.x] = s;                                         \
  }

OPK(add_u32, "v_add_u32 %0, %0, %1")
OPK(xor_b32, "v_xor_b32 %0, %0, %1")
OPK(mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
OPK(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
OPK(mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
OPK(lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
OPK(add3, "v_add3_u32 %0, %0, %1, %2")
OPK(bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xc8")
OPK(bfe_u32, "v_bfe_u32 %0, %0, 8, 8")
OPK(min_u32, "v_min_u32 %0, %0, %1")
OPK(cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
OPK(cndmask_s, "v_cndmask_b32_e64 %0, %0, %1, s[4:5]")
OPK(and_b32, "v_and_b32 %0, %0, %1")
OPK(lshrrev, "v_lshrrev_b32 %0, 3, %0")
OPK(sub_u32, "v_sub_u32 %0, %0, %1")
OPK(mul_f32, "v_mul_f32 %0, %0, %1")
OPK(udot4, "v_dot4_u32_u8 %0, %0, %1, %2")
OPK(udot2, "v_dot2_u32_u16 %0, %0, %1, %2")
OPK(alignbit, "v_alignbit_b32 %0, %0, %1, %2")
OPK(alignbyte, "v_alignbyte_b32 %0, %0, %1, 3")
OPK(perm, "v_perm_b32 %0, %0, %1, %2")
OPK(lerp_u8, "v_lerp_u8 %0, %0, %1, %2")
OPK(sad_u8, "v_sad_u8 %0, %0, %1, %2")
OPK(pk_add_u16, "v_pk_add_u16 %0, %0, %1")
OPK(pk_min_i16, "v_pk_min_i16 %0, %0, %1")
OPK(pk_mad_i16, "v_pk_mad_i16 %0, %0, %1, %2")
OPK(pk_add_f16, "v_pk_add_f16 %0, %0, %1")
OPK(pk_min_f16, "v_pk_min_f16 %0, %0, %1")
OPK(pk_minimum3_f16, "v_pk_minimum3_f16 %0, %0, %1, %2")
OPK(pk_maximum3_f16, "v_pk_maximum3_f16 %0, %0, %1, %2")
OPK(max3_u32, "v_max3_u32 %0, %0, %1, %2")
OPK(add_f32, "v_add_f32 %0, %0, %1")
OPK(fma_f32, "v_fma_f32 %0, %0, %1, %2")
OPK(cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
OPK(mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")

template <typename K>
static void run(const char* name, K kern, uint32_t* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("%-16s", name);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * w;  // 256 threads = one wave per SIMD per block
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0x12345u, 0x0c0c0201u);
    hipEventRecord(e0);
    for (int r = 0; r < 3; r++)
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0x12345u, 0x0c0c0201u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr = 3.0 * blocks * 4.0 * kIters * kChains;
    const double peak = cus * 4.0 * 2.4e9 / 2.0;
    printf("  w%d %.3f", w, instr / (ms * 1e-3) / peak);
  }
  printf("   (fraction of the 2-cycle wave64 issue rate; 0.5 = 4 cycles per instruction)\n");
}

int main() {
  void* out = nullptr;
  hipMalloc(&out, 256 * 2048 * 8 * 4);
  uint32_t* u = (uint32_t*)out;
#define R(NAME) run(#NAME, k_##NAME, u)
  R(add_u32); R(xor_b32); R(mul_lo_u32); R(mul_u32_u24); R(mad_u32_u24); R(lshl_add); R(add3);
  R(bitop3); R(bfe_u32); R(min_u32); R(cndmask); R(cndmask_s); R(and_b32); R(lshrrev); R(sub_u32);
  R(mul_f32); R(udot4); R(udot2); R(alignbit); R(alignbyte);
  R(perm); R(lerp_u8); R(sad_u8); R(pk_add_u16); R(pk_min_i16); R(pk_mad_i16); R(pk_add_f16);
  R(pk_min_f16); R(pk_minimum3_f16); R(pk_maximum3_f16); R(max3_u32); R(add_f32); R(fma_f32);
  R(cvt_f32_u32); R(mul_hi_u24);
  hipFree(out);
  return 0;
}
