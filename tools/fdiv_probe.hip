// Checks the pivot-reciprocal division of a measured-and-rejected EG factorisation variant
//  against the compiler's a / b, bit for bit, on 2^28 operand
// pairs inside the range where the division's expansion does not rescale (|b| in [2^-100, 2^100],
// |a| in [2^-600, 2^600] or +0; random signs, mantissas and exponents, plus exponent-skewed and
// near-1 mantissa cases), and counts the pairs outside it that differ (expected: some).
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/fdiv_probe.hip -o tools/fdiv_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double recip_as_div(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-b, y, 1.0);
  return __builtin_fma(y, e, y);
}
__device__ __forceinline__ double div_by_recip(double a, double b, double y) {
  const double q0 = a * y;
  return __builtin_fma(__builtin_fma(-b, q0, a), y, q0);
}
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
__device__ double make(uint64_t r, int emin, int emax, int mode) {
  uint64_t mant = r & ((1ull << 52) - 1);
  if (mode == 1) mant &= 0xfull;                       // near a power of two
  if (mode == 2) mant |= ((1ull << 52) - 1) ^ 0xfull;  // near the next one
  const int e = emin + (int)((r >> 52) % (uint64_t)(emax - emin + 1));
  const uint64_t sign = (r >> 63) << 63;
  return __builtin_bit_cast(double, sign | ((uint64_t)(e + 1023) << 52) | mant);
}
__global__ void probe(uint64_t seed, unsigned long long* bad_in, unsigned long long* bad_out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long nin = 0, nout = 0;
  for (int k = 0; k < 16; k++) {
    const uint64_t r1 = mix(seed ^ (i * 16 + k) * 0x9e3779b97f4a7c15ull);
    const uint64_t r2 = mix(r1 + 0x632be59bd9b4e019ull);
    const int mode = (int)(r1 % 3), mb = (int)(r2 % 3);
    const double b = make(r2, -100, 100, mb);
    const double a = (r1 & 0xff) == 0 ? 0.0 : make(r1, -600, 600, mode);  // +0 numerators too
    const double q = a / b, f = div_by_recip(a, b, recip_as_div(b));
    nin += __builtin_bit_cast(uint64_t, q) != __builtin_bit_cast(uint64_t, f);
    const double ao = make(r1 ^ 0x5555, -1022, 1023, mode), bo = make(r2 ^ 0xaaaa, -1022, 1023, mb);
    const double qo = ao / bo, fo = div_by_recip(ao, bo, recip_as_div(bo));
    nout += __builtin_bit_cast(uint64_t, qo) != __builtin_bit_cast(uint64_t, fo);
  }
  if (nin) atomicAdd(bad_in, nin);
  if (nout) atomicAdd(bad_out, nout);
}
int main() {
  unsigned long long *d, h[2];
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  unsigned long long tin = 0, tout = 0, n = 0;
  for (int rep = 0; rep < 16; rep++) {
    if (hipMemset(d, 0, 16) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(4096), dim3(256), 0, 0, 1234567ull + rep * 7919ull, d, d + 1);
    if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    tin += h[0];
    tout += h[1];
    n += 4096ull * 256 * 16;
  }
  std::printf("pairs %llu: in range differing %llu, full range differing %llu\n", n, tin, tout);
  return tin == 0 ? 0 : 2;
}
