// Effective shader clock of small launches: a one-wave kernel runs a dependent FMA chain and
// reads clock64() (shader cycles) and wall_clock64() (the 100 MHz constant clock) around it; the
// ratio is the clock the launch ran at. Cases: launches separated by host sleeps (a per-frame
// caller), launches back to back, and launches right after a chip-wide load.
//   hipcc -O3 --offload-arch=gfx950 tools/clock_probe.hip -o tools/clock_probe && tools/clock_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                         \
    }                                                                   \
  } while (0)

__global__ void chain_kernel(int iters, float seed, unsigned long long* out, float* sink) {
  const unsigned long long c0 = clock64(), w0 = wall_clock64();
  float x = seed + threadIdx.x;
  for (int i = 0; i < iters; i++) x = __builtin_fmaf(x, 0.999999f, 1e-7f);
  const unsigned long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
  if (x == 12345.f) sink[threadIdx.x] = x;
}

__global__ void load_kernel(float* buf, int n, int reps) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float x = buf[i];
    for (int r = 0; r < reps; r++) x = __builtin_fmaf(x, 0.999f, 0.5f);
    buf[i] = x;
  }
}

static int probe(const char* what, int iters, unsigned long long* d_out, float* d_sink) {
  unsigned long long h[2];
  hipLaunchKernelGGL(chain_kernel, dim3(1), dim3(64), 0, 0, iters, 1.0f, d_out, d_sink);
  CK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
  const double us = h[1] / 100.0;
  std::printf("%-34s iters %8d  %9.1f us  %10llu cycles  %7.0f MHz\n", what, iters, us, h[0],
              h[0] / us);
  return 0;
}

int main() {
  unsigned long long* d_out;
  float *d_sink, *d_buf;
  const int n = 64 << 20;
  CK(hipMalloc(&d_out, 16));
  CK(hipMalloc(&d_sink, 256));
  CK(hipMalloc(&d_buf, n * sizeof(float)));
  CK(hipMemset(d_buf, 0, n * sizeof(float)));
  CK(hipDeviceSynchronize());
  for (int k = 0; k < 4; k++) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (probe("after 50 ms idle", 2000, d_out, d_sink)) return 1;
  }
  for (int k = 0; k < 4; k++) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (probe("after 50 ms idle (long chain)", 200000, d_out, d_sink)) return 1;
  }
  for (int k = 0; k < 4; k++)
    if (probe("back to back", 2000, d_out, d_sink)) return 1;
  for (int k = 0; k < 4; k++) {
    std::this_thread::sleep_for(std::chrono::microseconds(300));
    if (probe("after 0.3 ms idle", 2000, d_out, d_sink)) return 1;
  }
  for (int k = 0; k < 3; k++) {
    hipLaunchKernelGGL(load_kernel, dim3(4096), dim3(256), 0, 0, d_buf, n, 64);
    for (int r = 0; r < 20; r++) hipLaunchKernelGGL(load_kernel, dim3(4096), dim3(256), 0, 0, d_buf, n, 64);
    if (probe("right after a chip-wide load", 2000, d_out, d_sink)) return 1;
  }
  // a loaded chip: the probe launched while the load kernels run on another stream
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (int r = 0; r < 40; r++) hipLaunchKernelGGL(load_kernel, dim3(4096), dim3(256), 0, s2, d_buf, n, 64);
  unsigned long long h[2];
  hipLaunchKernelGGL(chain_kernel, dim3(1), dim3(64), 0, 0, 2000, 1.0f, d_out, d_sink);
  CK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
  std::printf("%-34s iters %8d  %9.1f us  %10llu cycles  %7.0f MHz\n", "beside a chip-wide load", 2000,
              h[1] / 100.0, h[0], h[0] / (h[1] / 100.0));
  CK(hipStreamSynchronize(s2));
  CK(hipDeviceSynchronize());
  std::printf("ok\n");
  return 0;
}
