// optimizer_runtime.cpp -- host side of include/slamgpu_optimizer.h.
//
// The device call validates its scalar arguments and launches one kernel on the caller's
// stream. The host call (the per-frame drop-in for Optimizer::PoseOptimization) stages the
// frame's edges through a per-thread device buffer that grows on demand, runs the same kernel
// on a per-thread stream and synchronises.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

#include <cfloat>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/slamgpu_optimizer.h"
#include "ba_coop.h"
#include "ba_kernels.h"
#include "eg_kernels.h"
#include "pose_kernels.h"
#include "sim3_kernels.h"

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

// Per-thread staging buffer of the synchronous calls (grown on demand).
struct HostStage {
  int device = -1;
  hipStream_t stream = nullptr;
  void* buf = nullptr;
  size_t bytes = 0;
  // host-mapped mirror of a caller's stop flag, polled by the local BA kernel
  int32_t* stop_host = nullptr;
  int32_t* stop_dev = nullptr;
  // pinned host twin of the inputs / outputs region of the single-problem BA calls
  char* pin = nullptr;
  size_t pin_bytes = 0;
};
// One per calling thread, never destroyed: its device / pinned buffers and stream live until the
// process ends (the runtime reclaims them); freeing them from a thread-exit destructor at process
// exit would run after the HIP runtime's own teardown has begun.
HostStage& thread_stage() {
  thread_local HostStage* s = new HostStage();
  return *s;
}

int stage_reserve(HostStage& S, size_t need) {
  int dev = 0;
  OPT_HIPCHECK(hipGetDevice(&dev));
  if (S.device != dev) {
    if (S.buf) (void)hipFree(S.buf);
    if (S.stop_host) (void)hipHostFree(S.stop_host);
    if (S.stream) (void)hipStreamDestroy(S.stream);
    S.buf = nullptr;
    S.stop_host = S.stop_dev = nullptr;
    S.stream = nullptr;
    S.bytes = 0;
    OPT_HIPCHECK(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
    S.device = dev;
  }
  if (need > S.bytes) {
    if (S.buf) OPT_HIPCHECK(hipFree(S.buf));
    S.buf = nullptr;
    S.bytes = 0;
    const size_t cap = need < (1u << 20) ? (1u << 20) : need;
    OPT_HIPCHECK(hipMalloc(&S.buf, cap));
    S.bytes = cap;
  }
  return 0;
}

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

int make_sim3_params(const float K1[4], const float K2[4], const float* isig1, const float* isig2,
                     int nlevels, float th2, int fix_scale, Sim3Params* P) {
  if (!K1 || !K2 || !isig1 || !isig2)
    return fail(SLAMGPU_EINVAL, "calibrations and inv_sigma2 arrays are required");
  if (nlevels < 1 || nlevels > SLAMGPU_MAX_LEVELS)
    return fail(SLAMGPU_EINVAL, "nlevels %d outside [1, %d]", nlevels, SLAMGPU_MAX_LEVELS);
  if (!(th2 >= 0.f)) return fail(SLAMGPU_EINVAL, "th2 %g is not a threshold", (double)th2);
  std::memset(P, 0, sizeof(*P));
  for (int i = 0; i < 4; i++) {
    P->K1[i] = (double)K1[i];
    P->K2[i] = (double)K2[i];
  }
  for (int i = 0; i < nlevels; i++) {
    P->isig1[i] = isig1[i];
    P->isig2[i] = isig2[i];
  }
  P->nlevels = nlevels;
  P->th2 = th2;
  P->delta = (double)std::sqrt(th2);  // const float deltaHuber = sqrt(th2) (optimizer.cpp:1017)
  P->fix_scale = fix_scale ? 1 : 0;
  return 0;
}

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
  HostStage& S = thread_stage();
  const size_t off_e = 256, off_T = off_e + al256((size_t)n * sizeof(slamgpu_pose_edge));
  const size_t off_o = off_T + 256, off_r = off_o + al256((size_t)n);
  if (int r = stage_reserve(S, off_r + 256)) return r;
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
      reinterpret_cast<int32_t*>(b + off_r), nullptr, S.stream, n));
  int32_t res = 0;
  OPT_HIPCHECK(hipMemcpyAsync(&res, b + off_r, sizeof(res), hipMemcpyDeviceToHost, S.stream));
  OPT_HIPCHECK(hipMemcpyAsync(Tcw, b + off_T, 16 * sizeof(float), hipMemcpyDeviceToHost, S.stream));
  if (n > 0)
    OPT_HIPCHECK(hipMemcpyAsync(outlier, b + off_o, n, hipMemcpyDeviceToHost, S.stream));
  OPT_HIPCHECK(hipStreamSynchronize(S.stream));
  *n_inliers = res;
  return 0;
}

size_t slamgpu_local_ba_workspace_bytes(int total_kf, int total_points, int total_obs) {
  size_t bytes = 0;
  ba_workspace_layout(nullptr, total_kf < 0 ? 0 : total_kf, total_points < 0 ? 0 : total_points,
                      total_obs < 0 ? 0 : total_obs, &bytes);
  return bytes;
}

int slamgpu_local_bundle_adjustment_device(
    const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
    const slamgpu_ba_problem* d_problems, int n_problems, float* d_kf_Tcw,
    const uint8_t* d_kf_mode, float* d_points, const int32_t* d_point_obs_start,
    const slamgpu_ba_obs* d_obs, uint8_t* d_erase, int32_t* d_status, void* d_workspace,
    size_t workspace_bytes, int total_kf, int total_points, int total_obs,
    const int32_t* d_stop_flag, void* stream) {
  PoseParams P;
  if (int r = make_params(cam, inv_sigma2, nlevels, &P)) return r;
  if (n_problems < 0 || total_kf < 0 || total_points < 0 || total_obs < 0)
    return fail(SLAMGPU_EINVAL, "negative sizes");
  if (n_problems == 0) return 0;
  if (!d_problems || !d_kf_Tcw || !d_kf_mode || !d_point_obs_start || !d_status ||
      (total_points > 0 && !d_points) || (total_obs > 0 && (!d_obs || !d_erase)))
    return fail(SLAMGPU_EINVAL, "null device buffer");
  size_t need = 0;
  ba_workspace_layout(nullptr, total_kf, total_points, total_obs, &need);
  if (!d_workspace || workspace_bytes < need)
    return fail(SLAMGPU_ECAP, "workspace of %zu bytes < %zu needed", workspace_bytes, need);
  const BaWorkspace ws = ba_workspace_layout(d_workspace, total_kf, total_points, total_obs, nullptr);
  OPT_HIPCHECK(launch_local_ba(P, d_problems, n_problems, d_kf_Tcw, d_kf_mode, d_points,
                               d_point_obs_start, d_obs, d_erase, d_status, ws, d_stop_flag,
                               static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_local_ba_linearize_device(
    const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
    const slamgpu_ba_problem* d_problems, int n_problems, const float* d_kf_Tcw,
    const uint8_t* d_kf_mode, const float* d_points, const int32_t* d_point_obs_start,
    const slamgpu_ba_obs* d_obs, const slamgpu_ba_linear* out, int32_t* d_status,
    void* d_workspace, size_t workspace_bytes, int total_kf, int total_points, int total_obs,
    void* stream) {
  PoseParams P;
  if (int r = make_params(cam, inv_sigma2, nlevels, &P)) return r;
  if (n_problems < 0 || total_kf < 0 || total_points < 0 || total_obs < 0 || !out)
    return fail(SLAMGPU_EINVAL, "bad arguments");
  if (n_problems == 0) return 0;
  if (!d_problems || !d_kf_Tcw || !d_kf_mode || !d_point_obs_start || !d_status || !out->chi ||
      (total_points > 0 && (!d_points || !out->hll || !out->bl)) ||
      (total_obs > 0 && (!d_obs || !out->chi2 || !out->hpl)) || !out->hpp || !out->bp)
    return fail(SLAMGPU_EINVAL, "null device buffer");
  size_t need = 0;
  ba_workspace_layout(nullptr, total_kf, total_points, total_obs, &need);
  if (!d_workspace || workspace_bytes < need)
    return fail(SLAMGPU_ECAP, "workspace of %zu bytes < %zu needed", workspace_bytes, need);
  const BaWorkspace ws = ba_workspace_layout(d_workspace, total_kf, total_points, total_obs, nullptr);
  const BaLinearOut o{out->chi2, out->hpl, out->hll, out->bl, out->hpp, out->bp, out->chi};
  OPT_HIPCHECK(launch_local_ba_linearize(P, d_problems, n_problems, d_kf_Tcw, d_kf_mode, d_points,
                                         d_point_obs_start, d_obs, d_status, ws, o,
                                         static_cast<hipStream_t>(stream)));
  return 0;
}

}  // extern "C"

namespace {

constexpr int kMaxDevices = 64;

// Work-groups of a coop BA launch over K optimised keyframes, never more than can be resident at
// once (the device's limits computed once per device: the mapping and loop-closing threads may
// make their first calls at the same time): 64 (sweep at the round-3 end,
// profiles/r3zv_ba_grid_sweep.log: C5 2.9 / 3.0 / 3.1 ms at 32 / 64 / 128 work-groups is flat to
// 64, while a 54-keyframe window 8.7 -> 8.3 ms and GBA-100 15.5 -> 13.5 ms gain; 192 CUs stay free
// for the tracking front end), and 128 for map-scale systems (K >= 512: GBA-1500 116 -> 110 ms),
// bounded by the CUs and the kernel's occupancy; SLAMGPU_BA_WGS fixes it.
static int coop_cap[kMaxDevices];  // work-groups of the coop kernel the device keeps resident

int coop_grid(int device, int K) {
  static std::once_flag once[kMaxDevices];
  static int grid[kMaxDevices];
  static bool fixed[kMaxDevices];
  int* const cap = coop_cap;
  if (device < 0 || device >= kMaxDevices) return 1;
  std::call_once(once[device], [device, cap]() {
    hipDeviceProp_t prop{};
    int c = 256;
    const bool have = hipGetDeviceProperties(&prop, device) == hipSuccess &&
                      prop.multiProcessorCount > 0;
    if (have) c = std::min(c, prop.multiProcessorCount);
    int per_cu = 0;
    if (have && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, coop_kernel_ptr(),
                                                             kCoopThreads, 0) == hipSuccess &&
        per_cu > 0)
      c = std::min(c, per_cu * prop.multiProcessorCount);
    cap[device] = std::max(1, c);
    const char* e = getenv("SLAMGPU_BA_WGS");
    fixed[device] = e != nullptr;
    grid[device] = std::min(cap[device], e ? std::min(256, std::max(1, atoi(e))) : 64);
  });
  if (!fixed[device] && K >= 512) return std::min(cap[device], 2 * grid[device]);
  return grid[device];
}

// The coop solves running on one device hold at most coop_cap work-groups together: each one's G
// work-groups must all be resident for its grid barriers to complete, so two solves that could
// not be resident at once would each hold part of the slots and wait forever. Within the budget
// they run concurrently, as the reference's LocalMapper LocalBA and LoopCloser global BA do
// (local_mapper.cpp:53, loop_closer.cpp:77): a C5-size LocalBA (64 work-groups) beside a
// map-scale GBA (128) takes 192 of MI355X's 256 -- it does not wait behind the GBA. A solve that
// does not fit waits for the running ones to release theirs. The front end and PoseOptimization
// on other streams only delay residency (their work-groups finish and free their CUs); the
// barrier waits for as long as arrivals keep coming.
class CoopSlots {
 public:
  // stop: the LocalMapper's abort flag (LocalBundleAdjustment only): while the solve waits for
  // slots it is polled every millisecond, and a raised flag ends the wait without slots -- the
  // caller then returns as the reference does when the flag is set before optimising
  // (optimizer.cpp:616-618).
  CoopSlots(int device, int G, const volatile bool* stop = nullptr)
      : d_(device < 0 || device >= kMaxDevices ? 0 : device), g_(G) {
    std::unique_lock<std::mutex> lk(m_[d_]);
    const int cap = std::max(coop_cap[d_], 1);
    g_ = std::min(g_, cap);  // (G never exceeds the cap: coop_grid)
    while (used_[d_] + g_ > cap) {
      if (stop && *stop) {
        g_ = 0;
        stopped_ = true;
        return;
      }
      cv_[d_].wait_for(lk, std::chrono::milliseconds(1));
    }
    used_[d_] += g_;
  }
  ~CoopSlots() {
    if (stopped_) return;
    {
      std::lock_guard<std::mutex> lk(m_[d_]);
      used_[d_] -= g_;
    }
    cv_[d_].notify_all();
  }
  bool stopped() const { return stopped_; }
  static int in_use(int device) {
    if (device < 0 || device >= kMaxDevices) return 0;
    std::lock_guard<std::mutex> lk(m_[device]);
    return used_[device];
  }
  CoopSlots(const CoopSlots&) = delete;
  CoopSlots& operator=(const CoopSlots&) = delete;

 private:
  static std::mutex m_[kMaxDevices];
  static std::condition_variable cv_[kMaxDevices];
  static int used_[kMaxDevices];
  int d_, g_;
  bool stopped_ = false;
};
std::mutex CoopSlots::m_[kMaxDevices];
std::condition_variable CoopSlots::cv_[kMaxDevices];
int CoopSlots::used_[kMaxDevices];

// One problem (LocalBundleAdjustment after its graph gathering, or the global BundleAdjustment)
// on the cooperative solver: validate, stage, run the schedule asynchronously while mirroring the
// caller's stop flag into host-mapped memory, read back.
int coop_host(const char* what, const slamgpu_camera* cam, const float* inv_sigma2, int nlevels,
              float* kf_Tcw, const uint8_t* kf_mode, int n_kf, float* points, int n_points,
              const int32_t* point_obs_start, const slamgpu_ba_obs* obs,
              const volatile bool* stop_flag, uint8_t* erase, const CoopPhase* phases,
              int n_phases, bool local, int* lm_iterations) {
  PoseParams P;
  if (int r = make_params(cam, inv_sigma2, nlevels, &P)) return r;
  if (lm_iterations) *lm_iterations = 0;
  if (n_kf < 0 || n_points < 0 || !kf_Tcw || !kf_mode || !point_obs_start || (n_points && !points))
    return fail(SLAMGPU_EINVAL, "%s: bad arguments", what);
  if (point_obs_start[0] != 0) return fail(SLAMGPU_EINVAL, "point_obs_start[0] must be 0");
  const int n_obs = point_obs_start[n_points];
  if (n_obs < 0 || (n_obs > 0 && !obs) || (local && n_obs > 0 && !erase))
    return fail(SLAMGPU_EINVAL, "%s: bad observations", what);
  std::vector<int32_t> free_of(n_kf, -1), kf_of;
  for (int k = 0; k < n_kf; k++) {
    if (kf_mode[k] > SLAMGPU_KF_FIXED) return fail(SLAMGPU_EINVAL, "kf_mode[%d] = %d", k, kf_mode[k]);
    if (kf_mode[k] == SLAMGPU_KF_LOCAL) {
      free_of[k] = (int32_t)kf_of.size();
      kf_of.push_back(k);
    }
  }
  const int K = (int)kf_of.size();
  if (K > SLAMGPU_BA_COOP_MAX_KF)
    return fail(SLAMGPU_ECAP, "%s: %d optimised keyframes > SLAMGPU_BA_COOP_MAX_KF (%d)", what, K,
                SLAMGPU_BA_COOP_MAX_KF);
  long long pairs = 0;
  std::vector<int> seen(n_kf, -1);
  for (int p = 0; p < n_points; p++) {
    const int s = point_obs_start[p], e1 = point_obs_start[p + 1];
    if (e1 < s) return fail(SLAMGPU_EINVAL, "point_obs_start not monotone at %d", p);
    long long m = 0;
    for (int e = s; e < e1; e++) {
      const int k = obs[e].keyframe;
      if (k < 0 || k >= n_kf)
        return fail(SLAMGPU_EINVAL, "observation %d: keyframe %d outside [0, %d)", e, k, n_kf);
      if (obs[e].octave < 0 || obs[e].octave >= nlevels)
        return fail(SLAMGPU_EINVAL, "observation %d: octave %d outside [0, %d)", e, obs[e].octave, nlevels);
      if (seen[k] == p) return fail(SLAMGPU_EINVAL, "a map point is observed twice by one keyframe");
      seen[k] = p;
      m += free_of[k] >= 0;
    }
    pairs += m * (m + 1) / 2;
  }
  if (pairs > (1ll << 30)) return fail(SLAMGPU_ECAP, "%s: %lld Schur pairs", what, pairs);
  // block profile of the reduced camera system: block row f spans block columns pfirst[f] .. f,
  // pfirst[f] = the smallest optimised keyframe sharing a map point with f (any observation: a
  // superset of every phase's active structure). Row i of S at S[prow[i] + k], k <= i.
  std::vector<int32_t> pfirst(K);
  for (int f = 0; f < K; f++) pfirst[f] = f;
  for (int p = 0; p < n_points; p++) {
    int mn = K;
    for (int e = point_obs_start[p]; e < point_obs_start[p + 1]; e++) {
      const int f = free_of[obs[e].keyframe];
      if (f >= 0 && f < mn) mn = f;
    }
    for (int e = point_obs_start[p]; e < point_obs_start[p + 1]; e++) {
      const int f = free_of[obs[e].keyframe];
      if (f >= 0 && mn < pfirst[f]) pfirst[f] = mn;
    }
  }
  // active block rows of block column J: A_J = {I > J : pfirst[I] <= J} (I contributes to J in
  // [pfirst[I], I - 1]); the grid factorisation stages their V rows in LDS and keeps a replica of
  // each one's diagonal block, plus those of the blocks entering A_{J+1} and one being recycled:
  // na_max = max_J |A_J| + |{I > J + 1 : pfirst[I] = J + 1}| + 1 slots
  int na_max = 0;
  {
    std::vector<int32_t> d((size_t)K + 1, 0), enter((size_t)K + 1, 0);
    for (int f = 0; f < K; f++)
      if (pfirst[f] < f) {
        d[pfirst[f]]++;
        d[f]--;
        if (pfirst[f] >= 1 && f > pfirst[f]) enter[pfirst[f]]++;
      }
    int run = 0;
    for (int j = 0; j < K; j++) {
      run += d[j];
      na_max = std::max(na_max, run + (j + 1 < K ? enter[j + 1] : 0) + 1);
    }
  }
  std::vector<int64_t> prow(6 * (size_t)K);
  int64_t pnnz = 0;
  for (int i = 0; i < 6 * K; i++) {
    const int64_t fc = 6 * (int64_t)pfirst[i / 6];
    prow[i] = pnnz - fc;
    pnnz += i - fc + 1;
  }
  if (local && stop_flag && *stop_flag) {  // optimizer.cpp:616-618: return before optimising
    for (int e = 0; e < n_obs; e++) erase[e] = 0;
    return 0;
  }
  using clk = std::chrono::steady_clock;
  const auto t_host0 = clk::now();
  int dev = 0;
  OPT_HIPCHECK(hipGetDevice(&dev));
  const int G = coop_grid(dev, K);
  size_t wsb = 0;
  coop_layout(nullptr, n_kf, n_points, n_obs, K, (int)pairs, G, pnnz, &wsb);
  // inputs and outputs in one region (one DMA each way through a pinned twin), then workspace
  const size_t o_T = 0, o_mode = o_T + al256(64 * (size_t)n_kf);
  const size_t o_pts = o_mode + al256(n_kf + 1), o_ps = o_pts + al256(12 * (size_t)n_points + 4);
  const size_t o_obs = o_ps + al256(4 * ((size_t)n_points + 1));
  const size_t o_free = o_obs + al256(sizeof(slamgpu_ba_obs) * (size_t)n_obs + 4);
  const size_t o_kof = o_free + al256(4 * (size_t)n_kf + 4);
  const size_t o_pf = o_kof + al256(4 * (size_t)K + 4);
  const size_t o_prow = o_pf + al256(4 * (size_t)K + 4);
  const size_t o_er = o_prow + al256(8 * 6 * (size_t)K + 8);
  const size_t o_ctl = o_er + al256((size_t)n_obs + 4);
  const size_t o_io = o_ctl + 256, o_ws = o_io;
  HostStage& S = thread_stage();
  if (int r = stage_reserve(S, o_ws + wsb)) return r;
  if (S.pin_bytes < o_io) {
    if (S.pin) OPT_HIPCHECK(hipHostFree(S.pin));
    S.pin = nullptr;
    S.pin_bytes = 0;
    OPT_HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&S.pin), o_io, hipHostMallocDefault));
    S.pin_bytes = o_io;
  }
  char* b = static_cast<char*>(S.buf);
  char* h = S.pin;
  CoopSlots slots(dev, G, local ? stop_flag : nullptr);  // the device's coop residency budget
  if (slots.stopped()) {  // the LocalMapper aborted while the solve waited for slots
    for (int e = 0; e < n_obs; e++) erase[e] = 0;
    return 0;
  }
  static const bool prof = getenv("SLAMGPU_BA_PROFILE") != nullptr;
  CoopWs w = coop_layout(b + o_ws, n_kf, n_points, n_obs, K, (int)pairs, G, pnnz, nullptr);
  w.free_of_kf = reinterpret_cast<const int32_t*>(b + o_free);
  w.kf_of_free = reinterpret_cast<const int32_t*>(b + o_kof);
  w.pfirst = reinterpret_cast<const int32_t*>(b + o_pf);
  w.prow = reinterpret_cast<const int64_t*>(b + o_prow);
  if (!prof) w.prof = nullptr;
  w.na_max = na_max;
  {  // the grid factorisation wherever S takes the profile path (6K > 144): the one-hand-off
     // version beats work-group 0 alone from there on (30 keyframes 4.5 -> 3.7 ms, 54: 13.1 ->
     // 8.8 ms); SLAMGPU_GBA_MWG=0 / SLAMGPU_GBA_MWG_MIN_KF select work-group 0 for A/B
    const char* e0 = getenv("SLAMGPU_GBA_MWG");  // read per call: tests switch both paths
    const char* e1 = getenv("SLAMGPU_GBA_MWG_MIN_KF");
    const int mwg_env = e0 ? atoi(e0) : 1, mwg_min = e1 ? atoi(e1) : 0;
    w.mwg = mwg_env && K >= mwg_min;
  }
  const CoopProblem pb{reinterpret_cast<const slamgpu_ba_obs*>(b + o_obs),
                       reinterpret_cast<const int32_t*>(b + o_ps),
                       reinterpret_cast<const uint8_t*>(b + o_mode),
                       reinterpret_cast<float*>(b + o_T),
                       reinterpret_cast<float*>(b + o_pts),
                       local ? reinterpret_cast<uint8_t*>(b + o_er) : nullptr,
                       reinterpret_cast<int32_t*>(b + o_ctl),
                       n_obs, n_points, n_kf, K};
  volatile int32_t* mirror = nullptr;
  if (stop_flag) {
    if (!S.stop_host) {
      void* hm = nullptr;
      OPT_HIPCHECK(hipHostMalloc(&hm, 64, hipHostMallocMapped | hipHostMallocCoherent));
      S.stop_host = static_cast<int32_t*>(hm);
      void* d = nullptr;
      OPT_HIPCHECK(hipHostGetDevicePointer(&d, hm, 0));
      S.stop_dev = static_cast<int32_t*>(d);
    }
    mirror = S.stop_host;
  }
  // A barrier that gives up (CTL_ERR) leaves the caller's arrays untouched; when work-groups were
  // missing (never resident), the solve is staged and run once more before reporting.
  int32_t ctl[8];
  clk::time_point t_launch0, t_launch1, t_done;
  for (int attempt = 0;; attempt++) {
    std::memcpy(h + o_T, kf_Tcw, 64 * (size_t)n_kf);
    std::memcpy(h + o_mode, kf_mode, n_kf);
    if (n_points) std::memcpy(h + o_pts, points, 12 * (size_t)n_points);
    std::memcpy(h + o_ps, point_obs_start, 4 * ((size_t)n_points + 1));
    if (n_obs) std::memcpy(h + o_obs, obs, sizeof(slamgpu_ba_obs) * (size_t)n_obs);
    if (n_kf) std::memcpy(h + o_free, free_of.data(), 4 * (size_t)n_kf);
    if (K) std::memcpy(h + o_kof, kf_of.data(), 4 * (size_t)K);
    if (K) std::memcpy(h + o_pf, pfirst.data(), 4 * (size_t)K);
    if (K) std::memcpy(h + o_prow, prow.data(), 8 * 6 * (size_t)K);
    OPT_HIPCHECK(hipMemcpyAsync(b, h, o_er, hipMemcpyHostToDevice, S.stream));
    if (mirror) *mirror = *stop_flag ? 1 : 0;
    t_launch0 = clk::now();
    OPT_HIPCHECK(launch_coop_ba(P, pb, w, phases, n_phases, local,
                                stop_flag ? S.stop_dev : nullptr, G, S.stream));
    // the outputs and the control words come back in the same region (pinned: asynchronous)
    OPT_HIPCHECK(hipMemcpyAsync(h, b, o_io, hipMemcpyDeviceToHost, S.stream));
    t_launch1 = clk::now();
    // keep the device's view of the caller's flag live until the work is done
    if (mirror) {
      hipError_t q;
      while ((q = hipStreamQuery(S.stream)) == hipErrorNotReady) {
        *mirror = *stop_flag ? 1 : 0;
        std::this_thread::sleep_for(std::chrono::microseconds(5));
      }
      if (q != hipSuccess) return fail(SLAMGPU_EHIP, "%s: %s", what, hipGetErrorString(q));
    }
    OPT_HIPCHECK(hipStreamSynchronize(S.stream));
    t_done = clk::now();
    std::memcpy(ctl, h + o_ctl, sizeof(ctl));
    if (!ctl[CTL_ERR]) break;
    const bool missing = ctl[CTL_ARRIVED] < ctl[CTL_GRID] - 1;
    if (!missing || attempt > 0)
      return fail(SLAMGPU_EDEVICE, "%s: grid barrier gave up after ~2 s without progress: %d of "
                  "%d work-groups had arrived (%s)", what, ctl[CTL_ARRIVED], ctl[CTL_GRID],
                  missing ? "work-groups never became resident, twice" : "a work-group stalled");
    fprintf(stderr, "slamgpu %s: %d of %d work-groups resident at a grid barrier; retrying once\n",
            what, ctl[CTL_ARRIVED], ctl[CTL_GRID]);
  }
  std::memcpy(kf_Tcw, h + o_T, 64 * (size_t)n_kf);
  if (n_points) std::memcpy(points, h + o_pts, 12 * (size_t)n_points);
  if (local && n_obs) std::memcpy(erase, h + o_er, n_obs);
  if (prof) {
    auto us = [](clk::time_point a, clk::time_point b2) {
      return std::chrono::duration<double, std::micro>(b2 - a).count();
    };
    fprintf(stderr, "[%s] host us: stage %.0f enqueue %.0f device-wait %.0f\n", what,
            us(t_host0, t_launch0), us(t_launch0, t_launch1), us(t_launch1, t_done));
  }
  if (lm_iterations) *lm_iterations = ctl[CTL_LM];
  if (w.prof) {  // SLAMGPU_BA_PROFILE: work-group 0's per-phase wall time
    double pr[16];
    OPT_HIPCHECK(hipMemcpy(pr, w.prof, sizeof(pr), hipMemcpyDeviceToHost));
    fprintf(stderr, "[%s] us: lin %.0f barrier %.0f assemble %.0f build_S %.0f factor %.0f "
            "kf_update %.0f points %.0f first-sync %.0f (G %d, K %d)\n", what, pr[0], pr[1],
            pr[2], pr[5], pr[6], pr[3], pr[4], pr[7], G, K);
    if (pr[13] < 0)  // FS_PROF build, grid factorisation: work-group 0's split per column
      fprintf(stderr, "[%s] grid factor split us: diag-wait %.0f panel %.0f pcnt-wait %.0f "
              "trailing %.0f lists %.0f (%.0f factorisations)\n", what, pr[8], pr[9], pr[10],
              pr[11], pr[12], -pr[13]);
    if (pr[13] > 0)  // FS_PROF diagnostic build of ba_coop.hip
      fprintf(stderr, "[%s] factor split us: panel %.0f bar1 %.0f wave0-diag %.0f bar2 %.0f "
              "solve %.0f (%.0f factorisations; active block rows per column: mean %.1f, "
              "max %.0f)\n", what, pr[8], pr[9], pr[10], pr[11], pr[12], pr[13],
              pr[14] / std::max(1.0, pr[13] * (K > 0 ? K : 1)), pr[15]);
  }
  return 0;
}

}  // namespace

extern "C" {

int slamgpu_local_bundle_adjustment(const slamgpu_camera* cam, const float* inv_sigma2,
                                    int nlevels, float* kf_Tcw, const uint8_t* kf_mode, int n_kf,
                                    float* points, int n_points, const int32_t* point_obs_start,
                                    const slamgpu_ba_obs* obs, const volatile bool* stop_flag,
                                    uint8_t* erase, int* lm_iterations) {
  // optimizer.cpp:611-613 optimize(5) with Huber kernels (deltas sqrt(5.991) / sqrt(7.815) as
  // float, :556 / :598), the outlier pass, then optimize(10) without them (:667-670)
  const CoopPhase ph[2] = {{5, 1, (double)(float)sqrt(5.991), (double)(float)sqrt(7.815)},
                           {10, 0, 0.0, 0.0}};
  return coop_host("local BA", cam, inv_sigma2, nlevels, kf_Tcw, kf_mode, n_kf, points, n_points,
                   point_obs_start, obs, stop_flag, erase, ph, 2, true, lm_iterations);
}

int slamgpu_coop_slots_in_use(int device) { return CoopSlots::in_use(device); }

int slamgpu_global_bundle_adjustment(const slamgpu_camera* cam, const float* inv_sigma2,
                                     int nlevels, float* kf_Tcw, const uint8_t* kf_mode, int n_kf,
                                     float* points, int n_points, const int32_t* point_obs_start,
                                     const slamgpu_ba_obs* obs, int n_iterations, int robust,
                                     const volatile bool* stop_flag, int* lm_iterations) {
  if (n_iterations < 0) return fail(SLAMGPU_EINVAL, "n_iterations %d < 0", n_iterations);
  // optimizer.cpp:69-70 huber_thresh_2d = sqrt(5.99), huber_thresh_3d = sqrt(7.815) (float);
  // one optimize(num_iter) (:159-160)
  const CoopPhase ph[1] = {{n_iterations, robust ? 1 : 0, (double)(float)sqrt(5.99),
                            (double)(float)sqrt(7.815)}};
  return coop_host("global BA", cam, inv_sigma2, nlevels, kf_Tcw, kf_mode, n_kf, points, n_points,
                   point_obs_start, obs, stop_flag, nullptr, ph, 1, false, lm_iterations);
}

int slamgpu_optimize_sim3_device(const float K1[4], const float K2[4], const float* inv_sigma2_1,
                                 const float* inv_sigma2_2, int nlevels,
                                 const slamgpu_sim3_match* d_matches,
                                 const int32_t* d_match_start, int n_problems, float th2,
                                 int fix_scale, double* d_S12, uint8_t* d_inlier,
                                 int32_t* d_n_inliers, int32_t* d_lm_iterations, void* stream) {
  Sim3Params P;
  if (int r = make_sim3_params(K1, K2, inv_sigma2_1, inv_sigma2_2, nlevels, th2, fix_scale, &P))
    return r;
  if (n_problems < 0) return fail(SLAMGPU_EINVAL, "n_problems %d < 0", n_problems);
  if (n_problems > 0 && (!d_match_start || !d_S12 || !d_n_inliers || !d_matches || !d_inlier))
    return fail(SLAMGPU_EINVAL, "null device buffer");
  OPT_HIPCHECK(launch_optimize_sim3(d_matches, d_match_start, n_problems, P, d_S12, d_inlier,
                                    d_n_inliers, d_lm_iterations,
                                    static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_optimize_sim3(const float K1[4], const float K2[4], const float* inv_sigma2_1,
                          const float* inv_sigma2_2, int nlevels,
                          const slamgpu_sim3_match* matches, int n, float th2, int fix_scale,
                          double S12[8], uint8_t* inlier, int* n_inliers) {
  Sim3Params P;
  if (int r = make_sim3_params(K1, K2, inv_sigma2_1, inv_sigma2_2, nlevels, th2, fix_scale, &P))
    return r;
  if (!S12 || !n_inliers || n < 0 || (n > 0 && (!matches || !inlier)))
    return fail(SLAMGPU_EINVAL, "bad arguments");
  if (n > SLAMGPU_SIM3_MAX_MATCHES)
    return fail(SLAMGPU_ECAP, "%d matches > SLAMGPU_SIM3_MAX_MATCHES (%d)", n,
                SLAMGPU_SIM3_MAX_MATCHES);
  for (int i = 0; i < n; i++)
    if (matches[i].octave1 < 0 || matches[i].octave1 >= nlevels || matches[i].octave2 < 0 ||
        matches[i].octave2 >= nlevels)
      return fail(SLAMGPU_EINVAL, "match %d: octave outside [0, %d)", i, nlevels);
  HostStage& S = thread_stage();
  const size_t off_m = 256, off_S = off_m + al256((size_t)n * sizeof(slamgpu_sim3_match));
  const size_t off_i = off_S + 256, off_r = off_i + al256((size_t)n);
  if (int r = stage_reserve(S, off_r + 256)) return r;
  char* b = static_cast<char*>(S.buf);
  const int32_t start[2] = {0, n};
  OPT_HIPCHECK(hipMemcpyAsync(b, start, sizeof(start), hipMemcpyHostToDevice, S.stream));
  if (n > 0)
    OPT_HIPCHECK(hipMemcpyAsync(b + off_m, matches, (size_t)n * sizeof(slamgpu_sim3_match),
                                hipMemcpyHostToDevice, S.stream));
  OPT_HIPCHECK(hipMemcpyAsync(b + off_S, S12, 8 * sizeof(double), hipMemcpyHostToDevice, S.stream));
  OPT_HIPCHECK(launch_optimize_sim3(
      reinterpret_cast<const slamgpu_sim3_match*>(b + off_m), reinterpret_cast<int32_t*>(b), 1, P,
      reinterpret_cast<double*>(b + off_S), reinterpret_cast<uint8_t*>(b + off_i),
      reinterpret_cast<int32_t*>(b + off_r), nullptr, S.stream));
  int32_t res = 0;
  OPT_HIPCHECK(hipMemcpyAsync(&res, b + off_r, sizeof(res), hipMemcpyDeviceToHost, S.stream));
  OPT_HIPCHECK(hipMemcpyAsync(S12, b + off_S, 8 * sizeof(double), hipMemcpyDeviceToHost, S.stream));
  if (n > 0) OPT_HIPCHECK(hipMemcpyAsync(inlier, b + off_i, n, hipMemcpyDeviceToHost, S.stream));
  OPT_HIPCHECK(hipStreamSynchronize(S.stream));
  *n_inliers = res;
  return 0;
}

int slamgpu_optimize_essential_graph(int n_kf, double* Scw, const uint8_t* fixed,
                                     const slamgpu_sim3_edge* edges, int n_edges, int fix_scale,
                                     int n_iterations, float* Tcw, float* points,
                                     const int32_t* point_ref, int n_points, int* lm_iterations) {
  if (lm_iterations) *lm_iterations = 0;
  if (n_kf < 0 || n_edges < 0 || n_points < 0 || n_iterations < 0)
    return fail(SLAMGPU_EINVAL, "negative sizes");
  if ((n_kf > 0 && (!Scw || !fixed)) || (n_edges > 0 && !edges) ||
      (n_points > 0 && points && !point_ref))
    return fail(SLAMGPU_EINVAL, "null buffer");
  for (int k = 0; k < n_edges; k++)
    if (edges[k].i < 0 || edges[k].i >= n_kf || edges[k].j < 0 || edges[k].j >= n_kf ||
        edges[k].i == edges[k].j)
      return fail(SLAMGPU_EINVAL, "edge %d: keyframes (%d, %d) invalid for %d keyframes", k,
                  edges[k].i, edges[k].j, n_kf);
  if (points)
    for (int q = 0; q < n_points; q++)
      if (point_ref[q] < 0 || point_ref[q] >= n_kf)
        return fail(SLAMGPU_EINVAL, "point %d: reference keyframe %d outside [0, %d)", q,
                    point_ref[q], n_kf);
  if (n_kf == 0) return 0;
  // ---- the graph's structure (host): free vertices, profile, assembly targets, extents ----
  std::vector<int32_t> fidx(n_kf);
  int F = 0;
  for (int v = 0; v < n_kf; v++) fidx[v] = fixed[v] ? -1 : F++;
  std::vector<int32_t> start(F);
  for (int f = 0; f < F; f++) start[f] = f;
  for (int k = 0; k < n_edges; k++) {
    const int a = fidx[edges[k].i], b = fidx[edges[k].j];
    if (a < 0 || b < 0) continue;
    const int hi = std::max(a, b), lo = std::min(a, b);
    start[hi] = std::min(start[hi], lo);
  }
  std::vector<int64_t> off(F + 1, 0);
  for (int f = 0; f < F; f++) off[f + 1] = off[f] + (f - start[f] + 1);
  const int64_t n_blocks = off[F];
  std::vector<std::vector<int32_t>> items(F);
  std::vector<int32_t> tgt_block, tgt_vertex;
  std::vector<std::vector<int32_t>> off_items;
  std::vector<std::pair<int64_t, int32_t>> off_key;  // (block, target) of off-diagonal targets
  std::vector<int32_t> block_target;
  {
    std::vector<int32_t> blk2t((size_t)n_blocks, -1);
    for (int k = 0; k < n_edges; k++) {
      const int a = fidx[edges[k].i], b = fidx[edges[k].j];
      if (a >= 0) items[a].push_back(4 * k + 0);
      if (b >= 0) items[b].push_back(4 * k + 1);
      if (a >= 0 && b >= 0) {
        const int hi = std::max(a, b), lo = std::min(a, b);
        const int64_t blk = off[hi] + (lo - start[hi]);
        if (blk2t[blk] < 0) {
          blk2t[blk] = (int32_t)off_items.size();
          off_items.emplace_back();
          off_key.emplace_back(blk, 0);
        }
        off_items[blk2t[blk]].push_back(4 * k + (a > b ? 2 : 3));
      }
    }
  }
  std::vector<int32_t> tgt_ptr(1, 0), tgt_items;
  for (int f = 0; f < F; f++) {
    tgt_block.push_back((int32_t)(off[f] + (f - start[f])));
    tgt_vertex.push_back(f);
    tgt_items.insert(tgt_items.end(), items[f].begin(), items[f].end());
    tgt_ptr.push_back((int32_t)tgt_items.size());
  }
  for (size_t t = 0; t < off_items.size(); t++) {
    tgt_block.push_back((int32_t)off_key[t].first);
    tgt_vertex.push_back(-1);
    tgt_items.insert(tgt_items.end(), off_items[t].begin(), off_items[t].end());
    tgt_ptr.push_back((int32_t)tgt_items.size());
  }
  const int n_targets = (int)tgt_block.size();
  std::vector<std::vector<int32_t>> ext(F);
  for (int i = 0; i < F; i++)
    for (int k = start[i]; k < i; k++) ext[k].push_back(i);
  std::vector<int32_t> ext_ptr(1, 0), ext_rows;
  std::vector<int64_t> ext_base;
  for (int k = 0; k < F; k++) {
    ext_rows.insert(ext_rows.end(), ext[k].begin(), ext[k].end());
    for (int i : ext[k]) ext_base.push_back(off[i] - start[i]);
    ext_ptr.push_back((int32_t)ext_rows.size());
  }
  // ---- one device region: inputs, structure, state ----
  const size_t E = (size_t)n_edges, N = (size_t)n_kf, P7 = 7 * (size_t)F;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += al256(bytes + 1);
    return at;
  };
  const size_t o_edges = take(E * sizeof(slamgpu_sim3_edge)), o_fidx = take(4 * N);
  const size_t o_start = take(4 * (size_t)F), o_off = take(8 * ((size_t)F + 1));
  const size_t o_tb = take(4 * (size_t)n_targets), o_tv = take(4 * (size_t)n_targets);
  const size_t o_tp = take(4 * ((size_t)n_targets + 1)), o_ti = take(4 * tgt_items.size());
  const size_t o_ep = take(4 * ((size_t)F + 1)), o_er = take(4 * ext_rows.size());
  const size_t o_eb = take(8 * ext_base.size());
  const size_t o_S = take(8 * 8 * N), o_S2 = take(8 * 8 * N), o_S0 = take(8 * 8 * N);
  const size_t o_err = take(8 * 7 * E), o_chi = take(8 * E), o_con = take(8 * kEgContrib * E);
  const size_t o_J = take(8 * 98 * E);
  const size_t o_H = take(8 * 49 * (size_t)n_blocks), o_b = take(8 * P7);
  const size_t o_L = take(8 * 49 * (size_t)n_blocks), o_x = take(8 * P7), o_y = take(8 * P7);
  const size_t o_out = take(64), o_T = take(Tcw ? 64 * N : 0);
  const size_t o_pts = take(points ? 12 * (size_t)n_points : 0);
  const size_t o_ref = take(points ? 4 * (size_t)n_points : 0);
  HostStage& HS = thread_stage();
  if (int r = stage_reserve(HS, o)) return r;
  char* d = static_cast<char*>(HS.buf);
  hipStream_t st = HS.stream;
  auto up = [&](size_t at, const void* src, size_t bytes) -> hipError_t {
    return bytes ? hipMemcpyAsync(d + at, src, bytes, hipMemcpyHostToDevice, st) : hipSuccess;
  };
  OPT_HIPCHECK(up(o_edges, edges, E * sizeof(slamgpu_sim3_edge)));
  OPT_HIPCHECK(up(o_fidx, fidx.data(), 4 * N));
  OPT_HIPCHECK(up(o_start, start.data(), 4 * (size_t)F));
  OPT_HIPCHECK(up(o_off, off.data(), 8 * ((size_t)F + 1)));
  OPT_HIPCHECK(up(o_tb, tgt_block.data(), 4 * (size_t)n_targets));
  OPT_HIPCHECK(up(o_tv, tgt_vertex.data(), 4 * (size_t)n_targets));
  OPT_HIPCHECK(up(o_tp, tgt_ptr.data(), 4 * ((size_t)n_targets + 1)));
  OPT_HIPCHECK(up(o_ti, tgt_items.data(), 4 * tgt_items.size()));
  OPT_HIPCHECK(up(o_ep, ext_ptr.data(), 4 * ((size_t)F + 1)));
  OPT_HIPCHECK(up(o_er, ext_rows.data(), 4 * ext_rows.size()));
  OPT_HIPCHECK(up(o_eb, ext_base.data(), 8 * ext_base.size()));
  OPT_HIPCHECK(up(o_S, Scw, 64 * N));
  OPT_HIPCHECK(up(o_S0, Scw, 64 * N));
  OPT_HIPCHECK(hipMemsetAsync(d + o_x, 0, 8 * P7 + 1, st));
  if (points) {
    OPT_HIPCHECK(up(o_pts, points, 12 * (size_t)n_points));
    OPT_HIPCHECK(up(o_ref, point_ref, 4 * (size_t)n_points));
  }
  EgGraph G;
  G.n = n_kf;
  G.n_edges = n_edges;
  G.F = F;
  G.fix_scale = fix_scale ? 1 : 0;
  G.edges = reinterpret_cast<const slamgpu_sim3_edge*>(d + o_edges);
  G.fidx = reinterpret_cast<const int32_t*>(d + o_fidx);
  G.start = reinterpret_cast<const int32_t*>(d + o_start);
  G.off = reinterpret_cast<const int64_t*>(d + o_off);
  G.n_targets = n_targets;
  G.tgt_block = reinterpret_cast<const int32_t*>(d + o_tb);
  G.tgt_vertex = reinterpret_cast<const int32_t*>(d + o_tv);
  G.tgt_ptr = reinterpret_cast<const int32_t*>(d + o_tp);
  G.tgt_items = reinterpret_cast<const int32_t*>(d + o_ti);
  G.ext_ptr = reinterpret_cast<const int32_t*>(d + o_ep);
  G.ext_rows = reinterpret_cast<const int32_t*>(d + o_er);
  G.ext_base = reinterpret_cast<const int64_t*>(d + o_eb);
  G.n_ext = (int)ext_rows.size();
  G.n_blocks = n_blocks;
  EgState W;
  W.S = reinterpret_cast<double*>(d + o_S);
  W.S_trial = reinterpret_cast<double*>(d + o_S2);
  W.err = reinterpret_cast<double*>(d + o_err);
  W.chi2 = reinterpret_cast<double*>(d + o_chi);
  W.contrib = reinterpret_cast<double*>(d + o_con);
  W.J = reinterpret_cast<double*>(d + o_J);
  W.H = reinterpret_cast<double*>(d + o_H);
  W.b = reinterpret_cast<double*>(d + o_b);
  W.L = reinterpret_cast<double*>(d + o_L);
  W.x = reinterpret_cast<double*>(d + o_x);
  W.y = reinterpret_cast<double*>(d + o_y);
  W.out = reinterpret_cast<double*>(d + o_out);
  auto read_out = [&](double* h) -> hipError_t {
    hipError_t e = hipMemcpyAsync(h, W.out, 3 * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(st);
  };
  // ---- SparseOptimizer::optimize(n_iterations), OptimizationAlgorithmLevenberg ----
  double lambda = 1e-16;  // setUserLambdaInit(1e-16) (:732)
  int ni = 2, nbad = 0, its = 0;
  for (int it = 0; it < n_iterations && F > 0; it++) {
    OPT_HIPCHECK(launch_eg_linearize(G, W, st));
    OPT_HIPCHECK(launch_eg_chi2_sum(G, W, st));
    OPT_HIPCHECK(launch_eg_assemble(G, W, n_blocks, st));
    double h[3];
    OPT_HIPCHECK(read_out(h));
    double currentChi = h[0];
    const double iniChi = currentChi;
    if (it == 0) {
      lambda = 1e-16;
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      OPT_HIPCHECK(launch_eg_factor_solve(G, W, n_blocks, lambda, st));
      OPT_HIPCHECK(launch_eg_update(G, W, st));
      OPT_HIPCHECK(launch_eg_errors(G, W.S_trial, W, st));
      OPT_HIPCHECK(launch_eg_chi2_sum(G, W, st));
      OPT_HIPCHECK(read_out(h));
      double tempChi = h[0];
      if (h[2] == 0.0) tempChi = DBL_MAX;
      rho = (currentChi - tempChi) / (h[1] + 1e-3);
      if (rho > 0 && std::isfinite(tempChi)) {
        double alpha = 1. - std::pow(2 * rho - 1, 3.0);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
        std::swap(W.S, W.S_trial);  // accept
      } else {
        lambda *= ni;
        ni *= 2;
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    its++;
    if (qmax == 10 || rho == 0) break;
    if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
    else nbad = 0;
    if (nbad >= 3) break;
  }
  OPT_HIPCHECK(launch_eg_finish(G, W.S, reinterpret_cast<double*>(d + o_S0),
                                Tcw ? reinterpret_cast<float*>(d + o_T) : nullptr,
                                points ? reinterpret_cast<float*>(d + o_pts) : nullptr,
                                reinterpret_cast<const int32_t*>(d + o_ref), n_points, st));
  OPT_HIPCHECK(hipMemcpyAsync(Scw, W.S, 64 * N, hipMemcpyDeviceToHost, st));
  if (Tcw) OPT_HIPCHECK(hipMemcpyAsync(Tcw, d + o_T, 64 * N, hipMemcpyDeviceToHost, st));
  if (points && n_points)
    OPT_HIPCHECK(hipMemcpyAsync(points, d + o_pts, 12 * (size_t)n_points, hipMemcpyDeviceToHost, st));
  OPT_HIPCHECK(hipStreamSynchronize(st));
  if (lm_iterations) *lm_iterations = its;
  return 0;
}

}  // extern "C"
