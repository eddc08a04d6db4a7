// tools/membench.hip -- calibration of this box's memory system for the access shapes the ORB
// kernels use (not part of the product). Prints GB/s for each pattern.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("%s: %s\n", #x, hipGetErrorString(e));                               \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void copy16(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

__global__ void copy4(const uint32_t* __restrict__ a, uint32_t* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

// copy16 through LDS: each wave moves 1 KiB per step HBM -> LDS by one 16-byte-per-lane
// buffer-to-LDS load (the orient_desc / fast_cells / pyr_ring load form), then LDS -> HBM
__global__ void copylds(const uint8_t* __restrict__ a, uint8_t* __restrict__ b, size_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t s[4][1024];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, 0x7fffffff, 0x00020000);
  for (size_t base = ((size_t)blockIdx.x * 4 + w) * 1024; base < n; base += (size_t)gridDim.x * 4096) {
    const uint8_t* src = a + base;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)src, 0, 1024, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)s[w], 16,
                                             16 * lane, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    reinterpret_cast<uint4*>(b + base)[lane] = reinterpret_cast<const uint4*>(s[w])[lane];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  (void)rs;
}

// blur7-like: each thread owns 4 columns of a 32-row strip, 3 dword loads per input row,
// one dword store per output row; trivial arithmetic (sum of the 12 bytes' dwords).
__global__ void strip3(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int w, int h,
                       int pitch, int nimg) {
  const int tiles_x = (w + 255) / 256;
  const int img = blockIdx.y;
  const int tile = blockIdx.x;
  const int x = (tile % tiles_x) * 256 + 4 * (threadIdx.x & 63);
  const int y0 = (tile / tiles_x) * 128 + (threadIdx.x >> 6) * 32;
  if (x < 4 || x + 8 > w || y0 >= h) return;
  const uint8_t* s = src + (size_t)img * pitch * h;
  uint8_t* d = dst + (size_t)img * pitch * h;
  uint32_t acc = 0;
  for (int r = y0 - 3; r < min(y0 + 32, h) + 3; r++) {
    const int rr = r < 0 ? -r : (r >= h ? 2 * h - 2 - r : r);
    const uint8_t* row = s + (size_t)rr * pitch;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + x - 4);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(row + x);
    const uint32_t w2 = *reinterpret_cast<const uint32_t*>(row + x + 4);
    acc = acc * 3 + (w0 ^ w1) + w2;
    if (r - 3 >= y0) *reinterpret_cast<uint32_t*>(d + (size_t)(r - 3) * pitch + x) = acc;
  }
}

int main() {
  const size_t bytes = (size_t)512 << 20;
  void *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double moved, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; i++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    printf("%-28s %8.3f ms  %8.1f GB/s\n", name, ms, moved / (ms * 1e-3) / 1e9);
  };
  timeit("copy16 512MB", 2.0 * bytes, [&] {
    hipLaunchKernelGGL(copy16, dim3(4096), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
  });
  timeit("copy4 512MB", 2.0 * bytes, [&] {
    hipLaunchKernelGGL(copy4, dim3(4096), dim3(256), 0, 0, (const uint32_t*)a, (uint32_t*)b, bytes / 4);
  });
  timeit("copylds 512MB", 2.0 * bytes, [&] {
    hipLaunchKernelGGL(copylds, dim3(4096), dim3(256), 0, 0, (const uint8_t*)a, (uint8_t*)b, bytes);
  });
  const int w = 1241, h = 376, pitch = 1280, nimg = 256;
  timeit("strip3 256 x 1241x376", 2.0 * nimg * w * h, [&] {
    hipLaunchKernelGGL(strip3, dim3(((w + 255) / 256) * ((h + 127) / 128), nimg), dim3(256), 0, 0,
                       (const uint8_t*)a, (uint8_t*)b, w, h, pitch, nimg);
  });
  return 0;
}
