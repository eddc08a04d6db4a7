// optimizer_runtime.cpp -- host side of include/slamgpu_optimizer.h.
//
// The device call validates its scalar arguments and launches one kernel on the caller's
// stream. The host call (the per-frame drop-in for Optimizer::PoseOptimization) stages the
// frame's edges through a per-thread device buffer that grows on demand, runs the same kernel
// on a per-thread stream and synchronises.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/slamgpu_optimizer.h"
#include "pose_kernels.h"

using namespace slamgpu;

namespace {

thread_local std::string t_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

#define OPT_HIPCHECK(x)                                                                 \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(SLAMGPU_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

int make_params(const slamgpu_camera* cam, const float* inv_sigma2, int nlevels, PoseParams* P) {
  if (!cam || !inv_sigma2) return fail(SLAMGPU_EINVAL, "camera and inv_sigma2 are required");
  if (nlevels < 1 || nlevels > SLAMGPU_MAX_LEVELS)
    return fail(SLAMGPU_EINVAL, "nlevels %d outside [1, %d]", nlevels, SLAMGPU_MAX_LEVELS);
  std::memset(P, 0, sizeof(*P));
  P->fx = cam->fx;
  P->fy = cam->fy;
  P->cx = cam->cx;
  P->cy = cam->cy;
  P->bf = cam->bf;
  P->nlevels = nlevels;
  for (int i = 0; i < nlevels; i++) P->inv_sigma2[i] = inv_sigma2[i];
  return 0;
}

// Per-thread staging for the synchronous call: [start offsets | edges | Tcw | outlier | result].
struct HostStage {
  int device = -1;
  hipStream_t stream = nullptr;
  void* buf = nullptr;
  size_t bytes = 0;
  ~HostStage() {
    if (buf) (void)hipFree(buf);
    if (stream) (void)hipStreamDestroy(stream);
  }
};
thread_local HostStage t_stage;

}  // namespace

extern "C" {

const char* slamgpu_optimizer_last_error(void) { return t_err.c_str(); }

int slamgpu_pose_optimization_device(const slamgpu_camera* cam, const float* inv_sigma2,
                                     int nlevels, const slamgpu_pose_edge* d_edges,
                                     const int32_t* d_edge_start, int n_frames, float* d_Tcw,
                                     uint8_t* d_outlier, int32_t* d_n_inliers,
                                     int32_t* d_lm_iterations, void* stream) {
  PoseParams P;
  if (int r = make_params(cam, inv_sigma2, nlevels, &P)) return r;
  if (n_frames < 0) return fail(SLAMGPU_EINVAL, "n_frames %d < 0", n_frames);
  if (n_frames > 0 && (!d_edge_start || !d_Tcw || !d_n_inliers || !d_edges || !d_outlier))
    return fail(SLAMGPU_EINVAL, "null device buffer");
  OPT_HIPCHECK(launch_pose_optimization(d_edges, d_edge_start, n_frames, P, d_Tcw, d_outlier,
                                        d_n_inliers, d_lm_iterations,
                                        static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_pose_optimization(const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
                              const slamgpu_pose_edge* edges, int n, float Tcw[16],
                              uint8_t* outlier, int* n_inliers) {
  PoseParams P;
  if (int r = make_params(cam, inv_sigma2, nlevels, &P)) return r;
  if (!Tcw || !n_inliers || n < 0 || (n > 0 && (!edges || !outlier)))
    return fail(SLAMGPU_EINVAL, "bad arguments");
  if (n > SLAMGPU_POSE_MAX_EDGES)
    return fail(SLAMGPU_ECAP, "%d edges > SLAMGPU_POSE_MAX_EDGES (%d)", n, SLAMGPU_POSE_MAX_EDGES);
  for (int i = 0; i < n; i++)
    if (edges[i].octave < 0 || edges[i].octave >= nlevels)
      return fail(SLAMGPU_EINVAL, "edge %d: octave %d outside [0, %d)", i, edges[i].octave, nlevels);
  int dev = 0;
  OPT_HIPCHECK(hipGetDevice(&dev));
  HostStage& S = t_stage;
  if (S.device != dev) {
    if (S.buf) (void)hipFree(S.buf);
    if (S.stream) (void)hipStreamDestroy(S.stream);
    S.buf = nullptr;
    S.stream = nullptr;
    S.bytes = 0;
    OPT_HIPCHECK(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
    S.device = dev;
  }
  const size_t off_e = 256, off_T = off_e + ((size_t)n * sizeof(slamgpu_pose_edge) + 255) / 256 * 256;
  const size_t off_o = off_T + 256, off_r = off_o + ((size_t)n + 255) / 256 * 256;
  const size_t need = off_r + 256;
  if (need > S.bytes) {
    if (S.buf) OPT_HIPCHECK(hipFree(S.buf));
    S.buf = nullptr;
    S.bytes = 0;
    const size_t cap = need < (1u << 20) ? (1u << 20) : need;
    OPT_HIPCHECK(hipMalloc(&S.buf, cap));
    S.bytes = cap;
  }
  char* b = static_cast<char*>(S.buf);
  const int32_t start[2] = {0, n};
  OPT_HIPCHECK(hipMemcpyAsync(b, start, sizeof(start), hipMemcpyHostToDevice, S.stream));
  if (n > 0)
    OPT_HIPCHECK(hipMemcpyAsync(b + off_e, edges, (size_t)n * sizeof(slamgpu_pose_edge),
                                hipMemcpyHostToDevice, S.stream));
  OPT_HIPCHECK(hipMemcpyAsync(b + off_T, Tcw, 16 * sizeof(float), hipMemcpyHostToDevice, S.stream));
  OPT_HIPCHECK(launch_pose_optimization(
      reinterpret_cast<const slamgpu_pose_edge*>(b + off_e), reinterpret_cast<int32_t*>(b), 1, P,
      reinterpret_cast<float*>(b + off_T), reinterpret_cast<uint8_t*>(b + off_o),
      reinterpret_cast<int32_t*>(b + off_r), nullptr, S.stream));
  int32_t res = 0;
  OPT_HIPCHECK(hipMemcpyAsync(&res, b + off_r, sizeof(res), hipMemcpyDeviceToHost, S.stream));
  OPT_HIPCHECK(hipMemcpyAsync(Tcw, b + off_T, 16 * sizeof(float), hipMemcpyDeviceToHost, S.stream));
  if (n > 0)
    OPT_HIPCHECK(hipMemcpyAsync(outlier, b + off_o, n, hipMemcpyDeviceToHost, S.stream));
  OPT_HIPCHECK(hipStreamSynchronize(S.stream));
  *n_inliers = res;
  return 0;
}

}  // extern "C"
