// Cost of one exchange round between G work-groups: each stores 32 doubles (write-through,
// agent-scope relaxed atomics), drains, arrives on a monotonic counter, spins until all G have
// arrived, then reads all G x 32 partials (L1-bypassing) and sums them in work-group order -- the
// hand-off a multi-work-group PoseOptimization would make twice per LM iteration. Cases: G
// work-groups spread over the XCDs, or all on one XCD (8 G blocks launched, only every 8th works).
//   hipcc -O3 --offload-arch=gfx950 tools/gridbar_probe.hip -o tools/gridbar_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                         \
    }                                                                   \
  } while (0)

__global__ __launch_bounds__(256) void exch_kernel(int rounds, int stride, double* part,
                                                   int* counter, double* out, int* err) {
  if (blockIdx.x % stride != 0) return;
  const int g = blockIdx.x / stride, G = gridDim.x / stride;
  __shared__ double tot[32];
  double acc = 1.0 + g;
  for (int r = 0; r < rounds; r++) {
    if (threadIdx.x < 32)
      __hip_atomic_store(&part[((r & 1) * G + g) * 32 + threadIdx.x], acc + threadIdx.x,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int target = (r + 1) * G;
      long spins = 0;
      while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (++spins > (1l << 26)) {
          *err = 1;
          break;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      double s = 0.0;
      for (int k = 0; k < G; k++)
        s += __hip_atomic_load(&part[((r & 1) * G + k) * 32 + threadIdx.x], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      tot[threadIdx.x] = s;
    }
    __syncthreads();
    acc = tot[threadIdx.x & 31] * 1e-3;
  }
  if (g == 0 && threadIdx.x < 32) out[threadIdx.x] = acc;
}

int main() {
  double *part, *out;
  int *counter, *err;
  CK(hipMalloc(&part, 2 * 256 * 32 * sizeof(double)));
  CK(hipMalloc(&out, 32 * sizeof(double)));
  CK(hipMalloc(&counter, 4));
  CK(hipMalloc(&err, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int rounds = 2000;
  for (int G : {1, 2, 4, 8, 16, 32}) {
    for (int stride : {1, 8}) {
      for (int rep = 0; rep < 2; rep++) {
        CK(hipMemset(counter, 0, 4));
        CK(hipMemset(err, 0, 4));
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(exch_kernel, dim3(G * stride), dim3(256), 0, 0, rounds, stride, part,
                           counter, out, err);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int h_err;
        CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
        if (rep == 1)
          std::printf("G %2d %-9s %7.3f us per exchange round%s\n", G,
                      stride == 1 ? "spread" : "one XCD", 1e3 * ms / rounds,
                      h_err ? " (GAVE UP)" : "");
      }
    }
  }
  std::printf("ok\n");
  return 0;
}
