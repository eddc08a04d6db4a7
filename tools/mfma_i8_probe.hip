// tools/mfma_i8_probe.hip -- checks the lane layout of v_mfma_i32_16x16x32_i8 on this GPU with
// exact, asymmetric integer data (not part of the product): A (16x32) and B (32x16) are loaded
// with the assumed maps -- lane l holds A[l & 15][8 (l >> 4) + j] and B[8 (l >> 4) + j][l & 15]
// in byte j of its 64-bit operand, and C[4 (l >> 4) + i][l & 15] in element i -- and the product
// is compared with a host GEMM. Prints "layout ok" or the first mismatches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x;
  uint64_t a = 0, b = 0;
  for (int j = 0; j < 8; j++) {
    a |= (uint64_t)(uint8_t)A[(l & 15) * 32 + 8 * (l >> 4) + j] << (8 * j);
    b |= (uint64_t)(uint8_t)B[(8 * (l >> 4) + j) * 16 + (l & 15)] << (8 * j);
  }
  v4i acc = {1000, 2000, 3000, 4000};
  acc = __builtin_amdgcn_mfma_i32_16x16x32_i8((long)a, (long)b, acc, 0, 0, 0);
  for (int i = 0; i < 4; i++) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

int main() {
  int8_t hA[16 * 32], hB[32 * 16];
  for (int i = 0; i < 16 * 32; i++) hA[i] = (int8_t)((i * 37 + 11) % 251 - 125);
  for (int i = 0; i < 32 * 16; i++) hB[i] = (int8_t)((i * 53 + 7) % 241 - 120);
  int8_t *dA, *dB;
  int* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, 16 * 16 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  int hC[256];
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int r = 0; r < 16; r++)
    for (int c = 0; c < 16; c++) {
      int ref = 1000 * (1 + (r & 3));
      for (int k = 0; k < 32; k++) ref += hA[r * 32 + k] * hB[k * 16 + c];
      if (ref != hC[r * 16 + c] && bad++ < 8) printf("C[%d][%d] = %d, expected %d\n", r, c, hC[r * 16 + c], ref);
    }
  printf(bad ? "layout MISMATCH (%d)\n" : "layout ok\n", bad);
  return bad != 0;
}
