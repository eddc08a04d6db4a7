// runtime.cpp -- host runtime behind the C ABI (include/slamgpu.h).
//
// One slamgpu_ctx = one device + stream + every workspace the batched kernels need, sized at
// creation for max_frames stereo pairs so that the *_device calls never allocate (they can be
// captured into a HIP graph). The host-buffer calls are thin wrappers that stage through the
// context's own device buffers and synchronise, mirroring the reference call sites:
// ORBextractor::Compute (orb_extractor.cpp:985), the stereo Frame ctor (frame.cpp:61-111) and
// OrbMatcher::SearchByProjection (orb_matcher.cpp:13, :1312).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/slamgpu.h"
#include "match_kernels.h"
#include "undistort.h"
#include "orb_kernels.h"
#include "orb_tables.h"
#include "timing.h"

using namespace slamgpu;

namespace slamgpu {
thread_local KernelTimer* g_timer = nullptr;
}

struct slamgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  ExtractStreams fx;  // side streams of the extraction (launch_extract)
  bool fork_level0 = true;  // level 0's FAST on fx.side0 beside the pyramid (slamgpu_set_extract_fork)
  OrbParams params{};
  OrbTables tables{};
  OrbGeom geom{};
  int max_frames = 0, max_images = 0;
  std::string err;
  // device geometry
  OrbGeom* d_geom = nullptr;
  ResizeX* d_rx = nullptr;
  ResizeY* d_ry = nullptr;
  CellDesc* d_cells = nullptr;
  // images staged by the host-buffer calls (left at d_in, right at d_in + in_stride)
  uint8_t* d_in = nullptr;
  uint8_t* h_in = nullptr;  // pinned twin of d_in: one DMA per call instead of per-row copies
  // pinned mirror of one stereo frame's results (counts, both views' keypoints + descriptors,
  // u_right / depth), filled by slamgpu_frame_stereo before its synchronisation: the downloads
  // that follow it copy host memory instead of issuing synchronous device reads
  uint8_t* h_res = nullptr;
  uint8_t* d_res = nullptr;  // its device twin: the frame's results packed, then one DMA
  bool res_valid = false;
  // slamgpu_frame_stereo's device work (H2D of the staged pair, the frontend, the mirror copies)
  // as one HIP graph, re-captured when the camera or the distortion changes
  hipGraph_t fgraph = nullptr;
  hipGraphExec_t fexec = nullptr;
  Camera fcam{};
  Distortion fdist{};
  bool fdist_on = false;
  int in_pitch = 0;
  int64_t in_stride = 0;
  // batch state
  ImageBatch batch{};
  int n_frames_last = 0, n_images_last = 0;
  Camera cam{};
  bool have_cam = false;
  // Frame::dist_coeff_ (k1 k2 p1 p2 k3); with k1 != 0 the left keypoints are undistorted into
  // kps_un ([2 * max_frames][kp_cap], left views only) and the grid / matchers read those
  Distortion dist{};
  int ndist = 0;
  bool dist_on = false;
  KeyPoint* kps_un = nullptr;
  // extractor buffers
  uint8_t* d_pyr = nullptr;
  ExtractWorkspace ws{};
  ExtractOutput out{};
  // stereo
  StereoWorkspace sws{};
  StereoOut sout{};
  // grid + matchers
  GridWorkspace gws{};
  MatchWorkspace mws{};
  int mw_cap = 0;
  int* d_qmeta = nullptr;  // [2][max_frames] q_start / q_count for host calls
  int* d_nm = nullptr;
  void* d_qbuf = nullptr;
  size_t qbuf_bytes = 0;
  int32_t* d_mp = nullptr;
  uint8_t* d_blk = nullptr;
  std::vector<void*> allocs;
  KernelTimer timer;
  OrbGeomDev gd() const {
    OrbGeomDev g;
    g.host = &geom;
    g.dev = d_geom;
    g.rx = d_rx;
    g.ry = d_ry;
    g.cells = d_cells;
    g.ws = ws;
    g.out = out;
    return g;
  }
};

// Makes the context's timer visible to the SLAMGPU_LAUNCH sites for the duration of a call.
struct TimerScope {
  KernelTimer* prev;
  explicit TimerScope(slamgpu_ctx* c) : prev(g_timer) { g_timer = c && c->timer.on ? &c->timer : nullptr; }
  ~TimerScope() { g_timer = prev; }
};

static int fail(slamgpu_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

// Why the last slamgpu_create on this thread failed (no context exists to hold the message).
thread_local std::string t_create_err;
static int create_fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_create_err = buf;
  return code;
}

#define HIPCHECK(c, x)                                                                 \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail(c, SLAMGPU_EHIP, "%s failed: %s", #x, hipGetErrorString(e_));        \
  } while (0)

template <typename T>
static int dalloc(slamgpu_ctx* c, T** p, size_t count) {
  void* q = nullptr;
  const size_t bytes = count * sizeof(T) + 256;
  hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess)
    return fail(c, SLAMGPU_EHIP, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  c->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return 0;
}

static int hcheck(slamgpu_ctx* c, hipError_t e) {
  return e == hipSuccess ? 0 : fail(c, SLAMGPU_EHIP, "HIP error: %s", hipGetErrorString(e));
}

static hipStream_t pick_stream(slamgpu_ctx* c, void* s) {
  return s ? static_cast<hipStream_t>(s) : c->stream;
}

static void set_camera(slamgpu_ctx* c, const slamgpu_camera* cam) {
  Camera k;
  k.fx = cam->fx;
  k.fy = cam->fy;
  k.cx = cam->cx;
  k.cy = cam->cy;
  k.bf = cam->bf;
  // Frame::ComputeImageBounds (k1 == 0) and MakeInitialComputations (frame.cpp:197-209)
  k.min_x = 0.0f;
  k.max_x = (float)c->geom.cols;
  k.min_y = 0.0f;
  k.max_y = (float)c->geom.rows;
  if (c->dist_on) {  // the undistorted corners (frame.cpp:646-667)
    const float cols = (float)c->geom.cols, rows = (float)c->geom.rows;
    const float cx[4] = {0.0f, cols, 0.0f, cols}, cy[4] = {0.0f, 0.0f, rows, rows};
    float ux[4], uy[4];
    for (int i = 0; i < 4; i++)
      undistort_point(cam->fx, cam->fy, cam->cx, cam->cy, c->dist, cx[i], cy[i], &ux[i], &uy[i]);
    k.min_x = std::min(ux[0], ux[2]);
    k.max_x = std::max(ux[1], ux[3]);
    k.min_y = std::min(uy[0], uy[1]);
    k.max_y = std::max(uy[2], uy[3]);
  }
  k.cell_w = (float)(k.max_x - k.min_x) / (kGridCols);
  k.cell_h = (float)(k.max_y - k.min_y) / (kGridRows);
  c->cam = k;
  c->have_cam = true;
}

// The left views as the matchers see them: Frame::undistorted_keypoints_ (== the keypoints when
// k1 == 0), the descriptors and counts of the extraction.
static FrameKps left_views(const slamgpu_ctx* c) {
  return FrameKps{c->dist_on ? c->kps_un : c->out.kps, c->out.desc, c->out.nkps,
                  2 * (int64_t)c->geom.kp_cap, 2};
}

// Layout of the pinned result mirror (slamgpu_frame_stereo): two counts (16 B), both views'
// keypoints and descriptors at kp_cap each, then frame 0's u_right and depth.
struct ResMirror {
  int* nkps;
  uint32_t* err;  // [2]: the device error word, copied by the two packing kernels
  KeyPoint* kps;
  uint8_t* desc;
  float* u_right;
  float* depth;
};
static size_t res_mirror_bytes(int kp_cap) {
  const size_t kc = (size_t)kp_cap;
  return 16 + 2 * kc * sizeof(KeyPoint) + 2 * kc * 32 + 2 * kc * sizeof(float);
}
static ResMirror res_mirror(const slamgpu_ctx* c) {
  const size_t kc = (size_t)c->geom.kp_cap;
  uint8_t* h = c->h_res;
  ResMirror m;
  m.nkps = reinterpret_cast<int*>(h);
  m.err = reinterpret_cast<uint32_t*>(h + 8);
  m.kps = reinterpret_cast<KeyPoint*>(h + 16);
  m.desc = h + 16 + 2 * kc * sizeof(KeyPoint);
  m.u_right = reinterpret_cast<float*>(m.desc + 2 * kc * 32);
  m.depth = m.u_right + kc;
  return m;
}

static int round_up_cells(int n) { return (n + kCellGroup - 1) / kCellGroup * kCellGroup; }

static int check_device_err(slamgpu_ctx* c) {
  uint32_t e = 0;
  HIPCHECK(c, hipMemcpy(&e, c->ws.err, sizeof(e), hipMemcpyDeviceToHost));
  if (e) {
    (void)hipMemset(c->ws.err, 0, sizeof(uint32_t));
    return fail(c, SLAMGPU_EDEVICE, "device capacity overflow (bits 0x%x)", e);
  }
  return 0;
}

extern "C" {

int slamgpu_create(int device, const slamgpu_orb_params* p, int cols, int rows, int max_frames,
                   slamgpu_ctx** out) {
  if (!p || !out || max_frames < 1) return SLAMGPU_EINVAL;
  *out = nullptr;
  slamgpu_ctx* c = new slamgpu_ctx();
  c->params = OrbParams{p->nfeatures, p->scale_factor, p->nlevels,
                        std::min(std::max(p->ini_th_fast, 0), 255),
                        std::min(std::max(p->min_th_fast, 0), 255)};
  std::vector<ResizeX> rx;
  std::vector<ResizeY> ry;
  // the octree kernels' LDS limits on this device (without a usable device: the gfx950 budgets;
  // hipSetDevice below then reports the failure)
  int oct_img_lds = 1 << 30, oct_lvl_lds = 1 << 30;
  if (hipSetDevice(device) != hipSuccess ||
      octree_lds_limits(device, &oct_img_lds, &oct_lvl_lds) != hipSuccess) {
    oct_img_lds = oct_lvl_lds = 1 << 30;
    (void)hipGetLastError();
  }
  if (int gr = compute_geometry(c->params, cols, rows, &c->geom, &rx, &ry, oct_img_lds,
                                oct_lvl_lds)) {
    static const char* why[] = {
        "", "bad parameters",
        "image too small: a pyramid level is under 2*19+8 pixels (the reference's FAST cell grid "
        "would be empty, orb_extractor.cpp:712-733)",
        "a pyramid level yields no initial octree node (orb_extractor.cpp:484-486)",
        "FAST cell wider than 64 pixels", "resize span exceeds the pyr_down window",
        "unsupported Gaussian kernel",
        "a level's octree nodes overflow octree_lvl_kernel's LDS budget"};
    delete c;
    return create_fail(SLAMGPU_EINVAL, "slamgpu_create(%dx%d, nlevels %d, scale %g): %s", cols,
                       rows, p->nlevels, (double)p->scale_factor,
                       why[std::min(std::max(-gr, 0), 7)]);
  }
  if (!extract_build_matches(c->geom)) {
    delete c;
    return create_fail(SLAMGPU_EINVAL,
                       "slamgpu_create: orb_geometry.cpp and orb_kernels.hip were built with "
                       "different PYR_RING_STRIP / FAST_CELLS_PER_WAVE");
  }
  compute_tables(c->params, &c->tables);
  if (c->geom.kp_cap > 4096) {  // matcher keys carry a 12-bit keypoint index
    const int kpc = c->geom.kp_cap;
    delete c;
    return create_fail(SLAMGPU_EINVAL, "slamgpu_create: nfeatures %d gives %d keypoints per image "
                       "> 4096", p->nfeatures, kpc);
  }
  for (int l = 0; l < c->geom.nlevels; l++)
    if (c->geom.lv[l].node_cap > 1024) {
      const int need = c->geom.lv[l].node_cap;
      delete c;
      return create_fail(SLAMGPU_EINVAL, "slamgpu_create: level %d needs %d octree nodes > 1024",
                         l, need);  // octree LDS arrays hold <= 2048 list nodes
    }
  c->device = device;
  c->max_frames = max_frames;
  c->max_images = 2 * max_frames;
  int rc = 0;
  // on failure the partial context is destroyed here and its message kept for
  // slamgpu_last_error(NULL); *out stays NULL
#define TRY(x)                           \
  do {                                   \
    if ((rc = (x)) != 0) {               \
      t_create_err = c->err;             \
      slamgpu_destroy(c);                \
      return rc;                         \
    }                                    \
  } while (0)
  TRY(hipSetDevice(device) == hipSuccess ? 0 : fail(c, SLAMGPU_EHIP, "hipSetDevice"));
  TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess
          ? 0
          : fail(c, SLAMGPU_EHIP, "hipStreamCreate"));
  {  // the side stream of launch_extract's level-0 FAST (SLAMGPU_FORK=0 disables it)
    const char* e = getenv("SLAMGPU_FORK");
    const int mode = e ? atoi(e) : 1;
    ExtractStreams& fx = c->fx;
    if (mode >= 1)
      TRY(hipStreamCreateWithFlags(&fx.side0, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreateWithFlags(&fx.fork0, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&fx.join0, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&fx.fork1, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&fx.join1, hipEventDisableTiming) == hipSuccess
              ? 0
              : fail(c, SLAMGPU_EHIP, "side stream / events"));
  }
  const OrbGeom& g = c->geom;
  const int n = c->max_images;
  TRY(dalloc(c, &c->d_geom, 1));
  TRY(dalloc(c, &c->d_rx, rx.size() + 1));
  TRY(dalloc(c, &c->d_ry, ry.size() + 1));
  std::vector<CellDesc> cells;
  build_cells(g, &cells);
  TRY(dalloc(c, &c->d_cells, cells.size()));
  TRY(hcheck(c, hipMemcpy(c->d_geom, &g, sizeof(OrbGeom), hipMemcpyHostToDevice)));
  TRY(hcheck(c, hipMemcpy(c->d_rx, rx.data(), rx.size() * sizeof(ResizeX), hipMemcpyHostToDevice)));
  TRY(hcheck(c, hipMemcpy(c->d_ry, ry.data(), ry.size() * sizeof(ResizeY), hipMemcpyHostToDevice)));
  TRY(hcheck(c, hipMemcpy(c->d_cells, cells.data(), cells.size() * sizeof(CellDesc),
                          hipMemcpyHostToDevice)));
  c->in_pitch = (cols + 63) / 64 * 64;
  c->in_stride = (int64_t)c->in_pitch * rows;
  TRY(dalloc(c, &c->d_in, 2 * (size_t)c->in_stride));
  TRY(hcheck(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_in), 2 * (size_t)c->in_stride,
                              hipHostMallocDefault)));
  TRY(dalloc(c, &c->d_pyr, (size_t)n * g.pyr_bytes));
  TRY(dalloc(c, &c->ws.cell_keys, (size_t)n * g.cells_per_image * g.cell_cap));
  TRY(dalloc(c, &c->ws.cell_count, (size_t)n * g.cells_per_image));
  TRY(dalloc(c, &c->ws.key_scratch, (size_t)n * g.keys_per_image));
  TRY(dalloc(c, &c->ws.node_scratch, (size_t)n * g.nodes_per_image));
  TRY(dalloc(c, &c->ws.oct_keys, (size_t)n * g.out_per_image));
  TRY(dalloc(c, &c->ws.oct_count, (size_t)n * g.nlevels));
  TRY(dalloc(c, &c->ws.err, 4));
  TRY(hcheck(c, hipMemset(c->ws.err, 0, sizeof(uint32_t))));
  TRY(dalloc(c, &c->out.kps, (size_t)n * g.kp_cap));
  TRY(dalloc(c, &c->out.desc, (size_t)n * g.kp_cap * 32));
  TRY(dalloc(c, &c->out.nkps, (size_t)n));
  TRY(hcheck(c, hipMemset(c->out.nkps, 0, sizeof(int) * n)));
  const int rows0 = g.lv[0].h;
  c->sws.row_cap = g.kp_cap * 24;
  TRY(dalloc(c, &c->sws.row_start, (size_t)max_frames * (rows0 + 1)));
  TRY(dalloc(c, &c->sws.row_items, (size_t)max_frames * c->sws.row_cap));
  TRY(dalloc(c, &c->sws.sad, (size_t)max_frames * g.kp_cap));
  TRY(dalloc(c, &c->sout.u_right, (size_t)max_frames * g.kp_cap));
  TRY(dalloc(c, &c->sout.depth, (size_t)max_frames * g.kp_cap));
  TRY(dalloc(c, &c->gws.cell_start, (size_t)max_frames * (kGridCells + 1)));
  TRY(dalloc(c, &c->gws.cell_items, (size_t)max_frames * g.kp_cap));
  TRY(dalloc(c, &c->gws.cell_fill, (size_t)max_frames * kGridCells));
  TRY(dalloc(c, &c->d_qmeta, 2 * (size_t)max_frames));
  TRY(dalloc(c, &c->d_nm, (size_t)max_frames));
  TRY(dalloc(c, &c->d_mp, (size_t)g.kp_cap));
  TRY(dalloc(c, &c->d_blk, (size_t)g.kp_cap));
  TRY(hcheck(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_res), res_mirror_bytes(g.kp_cap),
                              hipHostMallocDefault)));
  TRY(dalloc(c, &c->d_res, res_mirror_bytes(g.kp_cap)));
#undef TRY
  *out = c;
  return 0;
}

void slamgpu_destroy(slamgpu_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->fexec) (void)hipGraphExecDestroy(c->fexec);
  if (c->fgraph) (void)hipGraphDestroy(c->fgraph);
  for (hipEvent_t e : c->timer.pool) (void)hipEventDestroy(e);
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->h_in) (void)hipHostFree(c->h_in);
  if (c->h_res) (void)hipHostFree(c->h_res);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->fx.side0) (void)hipStreamDestroy(c->fx.side0);
  for (hipEvent_t e : {c->fx.fork0, c->fx.join0, c->fx.fork1, c->fx.join1})
    if (e) (void)hipEventDestroy(e);
  delete c;
}

const char* slamgpu_last_error(const slamgpu_ctx* c) {
  return c ? c->err.c_str() : t_create_err.c_str();
}

int slamgpu_kp_capacity(const slamgpu_ctx* c) { return c ? c->geom.kp_cap : 0; }

int slamgpu_scale_tables(const slamgpu_ctx* c, float* scale, float* inv_scale, float* sigma2,
                         float* inv_sigma2, int* fpl) {
  if (!c) return SLAMGPU_EINVAL;
  for (int l = 0; l < c->tables.nlevels; l++) {
    if (scale) scale[l] = c->tables.scale[l];
    if (inv_scale) inv_scale[l] = c->tables.inv_scale[l];
    if (sigma2) sigma2[l] = c->tables.sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = c->tables.inv_sigma2[l];
    if (fpl) fpl[l] = c->tables.features_per_level[l];
  }
  return 0;
}

int slamgpu_orb_scale_tables(const slamgpu_orb_params* p, float* scale, float* inv_scale,
                             float* sigma2, float* inv_sigma2, int* fpl) {
  if (!p || p->nlevels < 1 || p->nlevels > kMaxLevels || !(p->scale_factor > 1.0f) ||
      p->nfeatures < 0)
    return SLAMGPU_EINVAL;
  OrbTables t;
  compute_tables(OrbParams{p->nfeatures, p->scale_factor, p->nlevels, p->ini_th_fast,
                           p->min_th_fast},
                 &t);
  for (int l = 0; l < t.nlevels; l++) {
    if (scale) scale[l] = t.scale[l];
    if (inv_scale) inv_scale[l] = t.inv_scale[l];
    if (sigma2) sigma2[l] = t.sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = t.inv_sigma2[l];
    if (fpl) fpl[l] = t.features_per_level[l];
  }
  return 0;
}

// pack (the single-frame call): the frame's results are also packed into this record for one
// D2H copy -- keypoints and descriptors on the side stream beside stereo matching, u_right /
// depth by stereo_median_kernel.
static int run_frontend(slamgpu_ctx* c, const ImageBatch& b, int n_frames, int n_images,
                        bool stereo, hipStream_t st, uint8_t* pack = nullptr) {
  TimerScope ts(c);
  c->res_valid = false;
  c->batch = b;
  c->n_frames_last = n_frames;
  c->n_images_last = n_images;
  OrbGeomDev g = c->gd();
  ExtractStreams fx = c->fx;
  if (!c->fork_level0) fx.side0 = nullptr;  // level 0's FAST after the pyramid, on `st`
  launch_extract(b, g, n_images, st, fx);
  if (stereo) {
    // UndistortKeyPoints + AssignFeaturesToGrid read only the left views' keypoints (frame.cpp:
    // 96, 110; stereo matching reads the distorted ones): on the side stream beside
    // ComputeStereoMatches, joined after it -- two fewer launches on the call's critical path
    const ExtractStreams& fx = c->fx;
    // (batches only, as launch_extract's level-0 FAST fork: a small launch's join costs more)
    const bool fork = fx.side0 && fx.fork1 && fx.join1 && n_frames > 8;
    hipStream_t gs = fork ? fx.side0 : st;
    if (fork) {
      HIPCHECK(c, hipEventRecord(fx.fork1, st));
      HIPCHECK(c, hipStreamWaitEvent(gs, fx.fork1, 0));
    }
    if (c->dist_on)
      launch_undistort(FrameKps{c->out.kps, c->out.desc, c->out.nkps, 2 * (int64_t)c->geom.kp_cap, 2},
                       c->kps_un, 2 * (int64_t)c->geom.kp_cap, c->cam, c->dist, n_frames,
                       c->geom.kp_cap, gs);
    // one frame with a host mirror (the single-frame call): row tables, grid and packing as
    // three work-groups of one launch, side by side
    const bool aux = pack && n_frames == 1 && !fork;
    if (aux) {
      launch_frame_aux(g, left_views(c), c->cam, c->gws, c->sws, pack, st);
    } else {
      launch_grid(left_views(c), c->cam, n_frames, c->geom.kp_cap, c->gws, gs);
      if (pack)
        launch_frame_pack(FrameKps{c->out.kps, c->out.desc, c->out.nkps, c->geom.kp_cap, 1},
                          c->sout.u_right, c->sout.depth, c->ws.err, c->geom.kp_cap, pack, gs, 1);
    }
    launch_stereo(b, g, c->cam, n_frames, c->sws, c->sout, st, pack, aux);
    if (fork) {
      HIPCHECK(c, hipEventRecord(fx.join1, gs));
      HIPCHECK(c, hipStreamWaitEvent(st, fx.join1, 0));
    }
  }
  HIPCHECK(c, hipGetLastError());
  return 0;
}

// Host images -> d_in: rows packed into the pinned staging buffer at the device pitch, then one
// DMA of the whole buffer (pageable 2-D copies go row by row: ~5 ms for a stereo pair). The
// previous call on this context has synchronised, so the staging buffer is free.
static void stage_host(slamgpu_ctx* c, const uint8_t* const* imgs, int n, size_t step) {
  const int cols = c->geom.cols, rows = c->geom.rows;
  for (int i = 0; i < n; i++) {
    uint8_t* dst = c->h_in + i * c->in_stride;
    if (step == (size_t)c->in_pitch) {  // already at the device pitch: one copy per image
      std::memcpy(dst, imgs[i], (size_t)(rows - 1) * c->in_pitch + cols);
      continue;
    }
    for (int y = 0; y < rows; y++)
      std::memcpy(dst + (int64_t)y * c->in_pitch, imgs[i] + y * step, cols);
  }
}
static int stage_images(slamgpu_ctx* c, const uint8_t* const* imgs, int n, size_t step) {
  stage_host(c, imgs, n, step);
  HIPCHECK(c, hipMemcpyAsync(c->d_in, c->h_in, (size_t)n * c->in_stride, hipMemcpyHostToDevice,
                             c->stream));
  return 0;
}
// The same, pipelined for the single-frame call: each image in two row halves, a half's DMA
// issued as soon as its rows are packed, so the host's packing of the next half runs under it
// (the packing is the larger part: ~933 KB of row copies against ~23 us of DMA).
static int stage_images_pipelined(slamgpu_ctx* c, const uint8_t* const* imgs, int n,
                                  size_t step) {
  const int cols = c->geom.cols, rows = c->geom.rows, pitch = c->in_pitch;
  for (int i = 0; i < n; i++) {
    uint8_t* dst = c->h_in + i * c->in_stride;
    for (int part = 0; part < 2; part++) {
      const int y0 = part ? rows / 2 : 0, y1 = part ? rows : rows / 2;
      if (step == (size_t)pitch) {
        std::memcpy(dst + (int64_t)y0 * pitch, imgs[i] + (int64_t)y0 * pitch,
                    (size_t)(y1 - y0 - 1) * pitch + cols);
      } else {
        for (int y = y0; y < y1; y++)
          std::memcpy(dst + (int64_t)y * pitch, imgs[i] + y * step, cols);
      }
      const size_t off = (size_t)i * c->in_stride + (size_t)y0 * pitch;
      HIPCHECK(c, hipMemcpyAsync(c->d_in + off, c->h_in + off, (size_t)(y1 - y0) * pitch,
                                 hipMemcpyHostToDevice, c->stream));
    }
  }
  return 0;
}

int slamgpu_extract(slamgpu_ctx* c, const uint8_t* img, size_t step, slamgpu_keypoint* kps,
                    uint8_t* desc, int cap, int* n_out) {
  if (!c || !img) return SLAMGPU_EINVAL;
  HIPCHECK(c, hipSetDevice(c->device));
  if (int r = stage_images(c, &img, 1, step)) return r;
  ImageBatch b{c->d_in, c->d_in + c->in_stride, 2 * c->in_stride, c->in_pitch, c->d_pyr};
  int rc = run_frontend(c, b, 1, 1, false, c->stream);
  if (rc) return rc;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  if ((rc = check_device_err(c))) return rc;
  return slamgpu_download_keypoints(c, 0, kps, desc, cap, n_out);
}

int slamgpu_get_pyramid_level(slamgpu_ctx* c, int img, int level, uint8_t* dst, size_t dst_step,
                              int* w_out, int* h_out) {
  if (!c || img < 0 || img >= c->n_images_last || level < 0 || level >= c->geom.nlevels)
    return SLAMGPU_EINVAL;
  const LevelGeom& L = c->geom.lv[level];
  if (w_out) *w_out = L.w;
  if (h_out) *h_out = L.h;
  if (!dst) return 0;
  const uint8_t* src;
  size_t pitch;
  if (level == 0) {
    src = ((img & 1) ? c->batch.in_r : c->batch.in_l) + (int64_t)(img >> 1) * c->batch.in_stride;
    pitch = c->batch.in_pitch;
  } else {
    src = c->d_pyr + (int64_t)img * c->geom.pyr_bytes + L.offset;
    pitch = L.pitch;
  }
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  HIPCHECK(c, hipMemcpy2D(dst, dst_step, src, pitch, L.w, L.h, hipMemcpyDeviceToHost));
  return 0;
}

int slamgpu_debug_level_keys(slamgpu_ctx* c, int img, int level, int stage, uint32_t* keys,
                             int cap, int* n_out) {
  if (!c || img < 0 || img >= c->n_images_last || level < 0 || level >= c->geom.nlevels)
    return SLAMGPU_EINVAL;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  const OrbGeom& g = c->geom;
  const LevelGeom& L = g.lv[level];
  std::vector<uint32_t> out;
  if (stage == 0) {
    const int ncell = L.ncols * L.nrows;
    std::vector<int> cnt(ncell);
    const int64_t cb = (int64_t)img * g.cells_per_image + L.cell_base;
    HIPCHECK(c, hipMemcpy(cnt.data(), c->ws.cell_count + cb, sizeof(int) * ncell,
                          hipMemcpyDeviceToHost));
    // the level's key slots at once; a cell's keys follow its group's earlier cells
    // (kCellGroup, fast_cells_kernel)
    std::vector<uint32_t> keys((size_t)round_up_cells(ncell) * g.cell_cap);
    HIPCHECK(c, hipMemcpy(keys.data(), c->ws.cell_keys + cb * g.cell_cap,
                          sizeof(uint32_t) * keys.size(), hipMemcpyDeviceToHost));
    int gfill = 0;
    for (int i = 0; i < ncell; i++) {
      if (i % kCellGroup == 0) gfill = 0;
      const uint32_t* src = keys.data() + (size_t)(i - i % kCellGroup) * g.cell_cap + gfill;
      out.insert(out.end(), src, src + cnt[i]);
      gfill += cnt[i];
    }
  } else {
    int n = 0;
    HIPCHECK(c, hipMemcpy(&n, c->ws.oct_count + img * g.nlevels + level, sizeof(int),
                          hipMemcpyDeviceToHost));
    out.resize(n);
    if (n)
      HIPCHECK(c, hipMemcpy(out.data(), c->ws.oct_keys + (int64_t)img * g.out_per_image + L.out_base,
                            sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
  }
  if (n_out) *n_out = (int)out.size();
  if ((int)out.size() > cap) return fail(c, SLAMGPU_ECAP, "need %zu keys", out.size());
  if (keys && !out.empty()) std::memcpy(keys, out.data(), out.size() * sizeof(uint32_t));
  return 0;
}

// The device half of slamgpu_frame_stereo on c->stream: the staged pair's DMA, the frontend,
// then the frame's results and the device error word into the pinned mirror.
// (the images are already on their way: stage_images_pipelined, before this)
static int enqueue_frame_stereo(slamgpu_ctx* c) {
  ImageBatch b{c->d_in, c->d_in + c->in_stride, 2 * c->in_stride, c->in_pitch, c->d_pyr};
  if (int rc = run_frontend(c, b, 1, 2, true, c->stream, c->d_res)) return rc;
  HIPCHECK(c, hipMemcpyAsync(c->h_res, c->d_res, res_mirror_bytes(c->geom.kp_cap),
                             hipMemcpyDeviceToHost, c->stream));
  return 0;
}

// SLAMGPU_FRAME_GRAPH=0 issues the frame call's launches one by one (A/B). With the results
// packed for one D2H copy the graph is the faster of the two on MI355X: 0.353 vs 0.383 ms per
// call (profiles/r3g_lat*.log; with six D2H copies as graph nodes it had been the slower one,
// 0.488 vs 0.463 ms, profiles/r3f_lat*.log).
static bool frame_graph_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("SLAMGPU_FRAME_GRAPH");
    return !(e && e[0] == '0');
  }();
  return on;
}

static void drop_frame_graph(slamgpu_ctx* c) {
  if (c->fexec) (void)hipGraphExecDestroy(c->fexec);
  if (c->fgraph) (void)hipGraphDestroy(c->fgraph);
  c->fexec = nullptr;
  c->fgraph = nullptr;
}

// One graph launch per frame: the launch chain costs the host one call instead of ~25, and the
// device sees the whole dependency graph at once. Captured on first use and whenever the kernels'
// by-value arguments (camera, distortion) change; the buffers it names are the context's own.
static int launch_frame_graph(slamgpu_ctx* c) {
  const bool same = c->fexec && std::memcmp(&c->fcam, &c->cam, sizeof(Camera)) == 0 &&
                    c->fdist_on == c->dist_on &&
                    std::memcmp(&c->fdist, &c->dist, sizeof(Distortion)) == 0;
  if (!same) {
    drop_frame_graph(c);
    HIPCHECK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    const int rc = enqueue_frame_stereo(c);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (rc || e != hipSuccess) {
      if (g) (void)hipGraphDestroy(g);
      return rc ? rc : fail(c, SLAMGPU_EHIP, "frame graph capture: %s", hipGetErrorString(e));
    }
    const hipError_t ei = hipGraphInstantiate(&c->fexec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      (void)hipGraphDestroy(g);
      c->fexec = nullptr;
      return fail(c, SLAMGPU_EHIP, "frame graph instantiate: %s", hipGetErrorString(ei));
    }
    c->fgraph = g;
    c->fcam = c->cam;
    c->fdist = c->dist;
    c->fdist_on = c->dist_on;
  } else {  // the host-side state run_frontend records
    c->res_valid = false;
    c->batch = ImageBatch{c->d_in, c->d_in + c->in_stride, 2 * c->in_stride, c->in_pitch, c->d_pyr};
    c->n_frames_last = 1;
    c->n_images_last = 2;
  }
  HIPCHECK(c, hipGraphLaunch(c->fexec, c->stream));
  return 0;
}

int slamgpu_frame_stereo(slamgpu_ctx* c, const uint8_t* left, const uint8_t* right, size_t step,
                         const slamgpu_camera* cam) {
  if (!c || !left || !right || !cam) return SLAMGPU_EINVAL;
  HIPCHECK(c, hipSetDevice(c->device));
  set_camera(c, cam);
  const uint8_t* imgs[2] = {left, right};
  if (int r = stage_images_pipelined(c, imgs, 2, step)) return r;
  // kernel timing records events around each launch: those calls stay eager
  const int rc = frame_graph_enabled() && !c->timer.on ? launch_frame_graph(c)
                                                       : enqueue_frame_stereo(c);
  if (rc) return rc;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  const ResMirror m = res_mirror(c);
  if (m.err[0] | m.err[1]) {  // the error word as the two packing kernels saw it
    const uint32_t e = m.err[0] | m.err[1];
    (void)hipMemset(c->ws.err, 0, sizeof(uint32_t));
    return fail(c, SLAMGPU_EDEVICE, "device capacity overflow (bits 0x%x)", e);
  }
  c->res_valid = true;
  return 0;
}

int slamgpu_frontend_device(slamgpu_ctx* c, const uint8_t* d_left, const uint8_t* d_right,
                            size_t frame_stride, size_t pitch, int n_frames,
                            const slamgpu_camera* cam, void* stream) {
  if (!c || !d_left || !d_right || !cam || n_frames < 1 || n_frames > c->max_frames ||
      pitch < (size_t)c->geom.cols)
    return fail(c, SLAMGPU_EINVAL, "slamgpu_frontend_device: bad arguments");
  set_camera(c, cam);
  ImageBatch b{d_left, d_right, (int64_t)frame_stride, (int)pitch, c->d_pyr};
  return run_frontend(c, b, n_frames, 2 * n_frames, true, pick_stream(c, stream));
}

int slamgpu_sync(slamgpu_ctx* c, void* stream) {
  if (!c) return SLAMGPU_EINVAL;
  HIPCHECK(c, hipStreamSynchronize(pick_stream(c, stream)));
  return check_device_err(c);
}

int slamgpu_download_keypoints(slamgpu_ctx* c, int img, slamgpu_keypoint* kps, uint8_t* desc,
                               int cap, int* n_out) {
  if (!c || img < 0 || img >= c->n_images_last) return SLAMGPU_EINVAL;
  if (c->res_valid && img < 2) {  // slamgpu_frame_stereo's mirror
    const ResMirror m = res_mirror(c);
    const int n = m.nkps[img];
    if (n_out) *n_out = n;
    if (n > cap) return fail(c, SLAMGPU_ECAP, "need %d keypoints, cap %d", n, cap);
    const size_t o = (size_t)img * c->geom.kp_cap;
    if (kps && n) std::memcpy(kps, m.kps + o, sizeof(KeyPoint) * n);
    if (desc && n) std::memcpy(desc, m.desc + o * 32, 32 * (size_t)n);
    return 0;
  }
  int n = 0;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  HIPCHECK(c, hipMemcpy(&n, c->out.nkps + img, sizeof(int), hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  if (n > cap) return fail(c, SLAMGPU_ECAP, "need %d keypoints, cap %d", n, cap);
  const int64_t o = (int64_t)img * c->geom.kp_cap;
  if (kps && n)
    HIPCHECK(c, hipMemcpy(kps, c->out.kps + o, sizeof(KeyPoint) * n, hipMemcpyDeviceToHost));
  if (desc && n)
    HIPCHECK(c, hipMemcpy(desc, c->out.desc + o * 32, 32 * (size_t)n, hipMemcpyDeviceToHost));
  return 0;
}

int slamgpu_download_stereo(slamgpu_ctx* c, int frame, float* u_right, float* depth, int cap,
                            int* n_out) {
  if (!c || frame < 0 || frame >= c->n_frames_last) return SLAMGPU_EINVAL;
  if (c->res_valid && frame == 0) {
    const ResMirror m = res_mirror(c);
    const int n = m.nkps[0];
    if (n_out) *n_out = n;
    if (n > cap) return fail(c, SLAMGPU_ECAP, "need %d entries, cap %d", n, cap);
    if (u_right && n) std::memcpy(u_right, m.u_right, 4 * (size_t)n);
    if (depth && n) std::memcpy(depth, m.depth, 4 * (size_t)n);
    return 0;
  }
  int n = 0;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  HIPCHECK(c, hipMemcpy(&n, c->out.nkps + 2 * frame, sizeof(int), hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  if (n > cap) return fail(c, SLAMGPU_ECAP, "need %d entries, cap %d", n, cap);
  const int64_t o = (int64_t)frame * c->geom.kp_cap;
  if (u_right && n)
    HIPCHECK(c, hipMemcpy(u_right, c->sout.u_right + o, 4 * (size_t)n, hipMemcpyDeviceToHost));
  if (depth && n)
    HIPCHECK(c, hipMemcpy(depth, c->sout.depth + o, 4 * (size_t)n, hipMemcpyDeviceToHost));
  return 0;
}

int slamgpu_device_results(const slamgpu_ctx* c, slamgpu_device_view* v) {
  if (!c || !v) return SLAMGPU_EINVAL;
  v->kps = reinterpret_cast<const slamgpu_keypoint*>(c->out.kps);
  v->desc = c->out.desc;
  v->nkps = c->out.nkps;
  v->u_right = c->sout.u_right;
  v->depth = c->sout.depth;
  v->kp_cap = c->geom.kp_cap;
  v->kps_un = reinterpret_cast<const slamgpu_keypoint*>(c->dist_on ? c->kps_un : c->out.kps);
  return 0;
}

static int parse_dist(const float* dist, int n, Distortion* d) {
  if (n != 0 && n != 4 && n != 5) return -1;
  if (n && !dist) return -1;
  *d = Distortion{};
  for (int i = 0; i < n; i++) d->k[i] = dist[i];
  return 0;
}

int slamgpu_set_distortion(slamgpu_ctx* c, const float* dist, int n) {
  if (!c) return SLAMGPU_EINVAL;
  Distortion d;
  if (parse_dist(dist, n, &d)) return fail(c, SLAMGPU_EINVAL, "DistCoef needs 4 or 5 values");
  if (d.k[0] != 0.0f && !c->kps_un) {
    HIPCHECK(c, hipSetDevice(c->device));
    if (int rc = dalloc(c, &c->kps_un, (size_t)c->max_images * c->geom.kp_cap)) return rc;
  }
  c->dist = d;
  c->ndist = n;
  c->dist_on = d.k[0] != 0.0f;  // Frame::UndistortKeyPoints tests k1 only (frame.cpp:616)
  c->have_cam = false;          // image bounds follow the distortion: set again by the next call
  return 0;
}

int slamgpu_undistort_points(const slamgpu_camera* cam, const float* dist, int n,
                             const float* xy_in, float* xy_out, int n_points) {
  Distortion d;
  if (!cam || parse_dist(dist, n, &d) || n_points < 0 || (n_points && (!xy_in || !xy_out)))
    return SLAMGPU_EINVAL;
  for (int i = 0; i < n_points; i++) {
    float u = xy_in[2 * i], v = xy_in[2 * i + 1];
    if (n) undistort_point(cam->fx, cam->fy, cam->cx, cam->cy, d, u, v, &u, &v);
    xy_out[2 * i] = u;
    xy_out[2 * i + 1] = v;
  }
  return 0;
}

int slamgpu_undistort_keypoints_device(const slamgpu_camera* cam, const float* dist, int n,
                                       const slamgpu_keypoint* d_in, int64_t in_stride,
                                       const int* d_counts, int counts_stride,
                                       slamgpu_keypoint* d_out, int64_t out_stride, int n_sets,
                                       int max_kps, void* stream) {
  Distortion d;
  if (!cam || parse_dist(dist, n, &d) || !d_in || !d_out || !d_counts || n_sets < 0 ||
      max_kps < 0 || counts_stride < 1)
    return SLAMGPU_EINVAL;
  if (n_sets == 0 || max_kps == 0) return 0;
  Camera k{};
  k.fx = cam->fx;
  k.fy = cam->fy;
  k.cx = cam->cx;
  k.cy = cam->cy;
  launch_undistort(FrameKps{reinterpret_cast<const KeyPoint*>(d_in), nullptr, d_counts, in_stride,
                            counts_stride},
                   reinterpret_cast<KeyPoint*>(d_out), out_stride, k, d, n_sets, max_kps,
                   static_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : SLAMGPU_EHIP;
}

int slamgpu_download_undistorted_keypoints(slamgpu_ctx* c, int frame, slamgpu_keypoint* kps,
                                           int cap, int* n_out) {
  if (!c || frame < 0 || frame >= c->n_frames_last) return SLAMGPU_EINVAL;
  if (!c->dist_on) return slamgpu_download_keypoints(c, 2 * frame, kps, nullptr, cap, n_out);
  int n = 0;
  HIPCHECK(c, hipStreamSynchronize(c->stream));
  HIPCHECK(c, hipMemcpy(&n, c->out.nkps + 2 * frame, sizeof(int), hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  if (n > cap) return fail(c, SLAMGPU_ECAP, "need %d keypoints, cap %d", n, cap);
  if (kps && n)
    HIPCHECK(c, hipMemcpy(kps, c->kps_un + (int64_t)2 * frame * c->geom.kp_cap,
                          sizeof(KeyPoint) * n, hipMemcpyDeviceToHost));
  return 0;
}

size_t slamgpu_frame_record_bytes(const slamgpu_ctx* c) {
  if (!c) return 0;
  return ((size_t)128 * c->geom.kp_cap + 8 + 255) / 256 * 256;
}

int slamgpu_pack_frame_records_device(slamgpu_ctx* c, int first, int n, void* d_dst,
                                      void* stream) {
  if (!c || !d_dst || n < 0 || first < 0 || first + n > c->n_frames_last)
    return fail(c, SLAMGPU_EINVAL, "pack_frame_records_device: frames [%d, %d) of %d", first,
                first + n, c->n_frames_last);
  if (n == 0) return 0;
  const size_t kc = c->geom.kp_cap, rec = slamgpu_frame_record_bytes(c);
  uint8_t* d = static_cast<uint8_t*>(d_dst);
  hipStream_t s = pick_stream(c, stream);
  // one strided copy per field: source rows are frames (pitch = the field's bytes per frame),
  // destination rows are records
  struct { size_t dst_off; const void* src; size_t width; } f[5] = {
      {0, c->out.kps + 2 * kc * first, 56 * kc},
      {56 * kc, c->out.desc + 64 * kc * first, 64 * kc},
      {120 * kc, c->sout.u_right + kc * first, 4 * kc},
      {124 * kc, c->sout.depth + kc * first, 4 * kc},
      {128 * kc, c->out.nkps + 2 * first, 8}};
  for (auto& x : f)
    HIPCHECK(c, hipMemcpy2DAsync(d + x.dst_off, rec, x.src, x.width, x.width, (size_t)n,
                                 hipMemcpyDeviceToDevice, s));
  return 0;
}

int slamgpu_make_vo_queries_device(slamgpu_ctx* c, const slamgpu_f2f_pose* d_poses, int blocks,
                                   slamgpu_f2f_query* d_queries, int* d_q_start, int* d_q_count,
                                   int n_frames, void* stream) {
  if (!c || !c->have_cam || n_frames < 1 || n_frames > c->n_frames_last)
    return fail(c, SLAMGPU_EINVAL, "make_vo_queries_device: bad arguments");
  TimerScope ts(c);
  launch_vo_queries(left_views(c), c->sout.depth, c->geom.kp_cap, c->cam,
                    reinterpret_cast<const F2FPose*>(d_poses), blocks, c->geom.kp_cap,
                    reinterpret_cast<F2FQuery*>(d_queries), d_q_start, d_q_count, n_frames,
                    pick_stream(c, stream));
  HIPCHECK(c, hipGetLastError());
  return 0;
}

int slamgpu_set_extract_fork(slamgpu_ctx* c, int on) {
  if (!c) return SLAMGPU_EINVAL;
  c->fork_level0 = on != 0;
  return 0;
}

int slamgpu_timing_start(slamgpu_ctx* c, const char* kernel, int max_launches) {
  if (!c || !kernel || max_launches < 1) return SLAMGPU_EINVAL;
  HIPCHECK(c, hipSetDevice(c->device));
  KernelTimer& t = c->timer;
  while ((int)t.pool.size() < 2 * max_launches) {
    hipEvent_t e;
    HIPCHECK(c, hipEventCreate(&e));
    t.pool.push_back(e);
  }
  t.target = kernel;
  t.used = 0;
  t.names.clear();
  t.overflow = false;
  t.on = true;
  return 0;
}

int slamgpu_timing_stop(slamgpu_ctx* c, void* stream) {
  if (!c) return SLAMGPU_EINVAL;
  c->timer.on = false;
  HIPCHECK(c, hipStreamSynchronize(pick_stream(c, stream)));
  HIPCHECK(c, hipDeviceSynchronize());
  if (c->timer.overflow) return fail(c, SLAMGPU_ECAP, "timing event pool exhausted");
  return 0;
}

int slamgpu_timing_read(slamgpu_ctx* c, const char* kernel, double* total_ms, int* launches) {
  if (!c || !kernel) return SLAMGPU_EINVAL;
  double tot = 0;
  int n = 0;
  for (size_t i = 0; i < c->timer.used; i++) {
    if (std::strcmp(kernel, "*") != 0 && std::strcmp(kernel, c->timer.names[i]) != 0) continue;
    float ms = 0;
    HIPCHECK(c, hipEventElapsedTime(&ms, c->timer.pool[2 * i], c->timer.pool[2 * i + 1]));
    tot += ms;
    n++;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  return 0;
}

int slamgpu_trace_marker(int id, void* stream) {
  if (id < 1) return SLAMGPU_EINVAL;
  launch_trace_marker(id, static_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? 0 : SLAMGPU_EHIP;
}

int slamgpu_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 32; i++) dist += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return dist;
}

// ---- matchers ------------------------------------------------------------------------------
static int ensure_match_ws(slamgpu_ctx* c, int total_queries) {
  if (total_queries <= c->mw_cap) return 0;
  int cap = std::max(total_queries, 4096);
  int rc;
  if ((rc = dalloc(c, &c->mws.topk, (size_t)cap * kTopK))) return rc;
  if ((rc = dalloc(c, &c->mws.ncand, (size_t)cap))) return rc;
  if ((rc = dalloc(c, &c->mws.rot_bin, (size_t)cap))) return rc;
  if ((rc = dalloc(c, &c->mws.best_idx, (size_t)cap))) return rc;
  c->mw_cap = cap;
  return 0;
}


int slamgpu_search_by_projection_frame_device(slamgpu_ctx* c, const slamgpu_f2f_query* d_q,
                                              int total_queries, const int* d_q_start,
                                              const int* d_q_count, int max_queries,
                                              const slamgpu_f2f_pose* d_poses,
                                              int32_t* d_map_point, uint8_t* d_blocked,
                                              int64_t mp_stride, int* d_nmatches, int n_frames,
                                              void* stream) {
  if (!c || !c->have_cam || n_frames < 1 || n_frames > c->n_frames_last ||
      mp_stride < c->geom.kp_cap)
    return fail(c, SLAMGPU_EINVAL, "search_by_projection_frame_device: bad arguments");
  int rc = ensure_match_ws(c, total_queries);
  if (rc) return rc;
  MatchIO io{d_q_start, d_q_count, d_map_point, d_blocked, d_nmatches, mp_stride};
  TimerScope ts(c);
  launch_search_frame(left_views(c), c->sout.u_right, c->geom.kp_cap, c->cam, c->gd(),
                      reinterpret_cast<const F2FQuery*>(d_q),
                      reinterpret_cast<const F2FPose*>(d_poses), n_frames, max_queries, c->gws,
                      c->mws, io, pick_stream(c, stream));
  HIPCHECK(c, hipGetLastError());
  return 0;
}

int slamgpu_search_by_projection_mps_device(slamgpu_ctx* c, const slamgpu_mps_query* d_q,
                                            int total_queries, const int* d_q_start,
                                            const int* d_q_count, int max_queries, float nnratio,
                                            int th, int32_t* d_map_point, uint8_t* d_blocked,
                                            int64_t mp_stride, int* d_nmatches, int n_frames,
                                            void* stream) {
  if (!c || !c->have_cam || n_frames < 1 || n_frames > c->n_frames_last ||
      mp_stride < c->geom.kp_cap)
    return fail(c, SLAMGPU_EINVAL, "search_by_projection_mps_device: bad arguments");
  int rc = ensure_match_ws(c, total_queries);
  if (rc) return rc;
  MatchIO io{d_q_start, d_q_count, d_map_point, d_blocked, d_nmatches, mp_stride};
  TimerScope ts(c);
  launch_search_mps(left_views(c), c->sout.u_right, c->geom.kp_cap, c->cam, c->gd(),
                    reinterpret_cast<const MpsQuery*>(d_q), nnratio, th, n_frames, max_queries,
                    c->gws, c->mws, io, pick_stream(c, stream));
  HIPCHECK(c, hipGetLastError());
  return 0;
}

}  // extern "C"

// Host-buffer matcher calls on one frame of the last frontend/frame call.
template <typename QT>
static int host_search(slamgpu_ctx* c, int frame, const QT* queries, int nq, int32_t* map_point,
                       uint8_t* blocked, int n, int* nmatches, size_t extra_bytes,
                       const void* extra, bool f2f, float nnratio, int th) {
  if (!c || frame < 0 || frame >= c->n_frames_last || nq < 0 || !map_point || !blocked)
    return SLAMGPU_EINVAL;
  if (n > c->geom.kp_cap) return fail(c, SLAMGPU_EINVAL, "n > kp capacity");
  const size_t need = sizeof(QT) * (size_t)std::max(nq, 1) + extra_bytes + 256;
  if (need > c->qbuf_bytes) {
    int rc = dalloc(c, reinterpret_cast<uint8_t**>(&c->d_qbuf), need);
    if (rc) return rc;
    c->qbuf_bytes = need;
  }
  int rc = ensure_match_ws(c, nq);
  if (rc) return rc;
  hipStream_t st = c->stream;
  uint8_t* qb = static_cast<uint8_t*>(c->d_qbuf);
  if (nq) HIPCHECK(c, hipMemcpyAsync(qb, queries, sizeof(QT) * nq, hipMemcpyHostToDevice, st));
  uint8_t* eb = qb + (sizeof(QT) * (size_t)std::max(nq, 1) + 255) / 256 * 256;
  if (extra_bytes)
    HIPCHECK(c, hipMemcpyAsync(eb, extra, extra_bytes, hipMemcpyHostToDevice, st));
  // frame `frame` only: use a one-frame view shifted to that frame
  int meta[2] = {0, nq};
  HIPCHECK(c, hipMemcpyAsync(c->d_qmeta, meta, sizeof(meta), hipMemcpyHostToDevice, st));
  HIPCHECK(c, hipMemsetAsync(c->d_mp, 0xff, sizeof(int32_t) * c->geom.kp_cap, st));
  HIPCHECK(c, hipMemsetAsync(c->d_blk, 0, c->geom.kp_cap, st));
  if (n) {
    HIPCHECK(c, hipMemcpyAsync(c->d_mp, map_point, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
    HIPCHECK(c, hipMemcpyAsync(c->d_blk, blocked, n, hipMemcpyHostToDevice, st));
  }
  const int64_t kc = c->geom.kp_cap;
  FrameKps cur{(c->dist_on ? c->kps_un : c->out.kps) + 2 * frame * kc,
               c->out.desc + 2 * frame * kc * 32, c->out.nkps + 2 * frame, 2 * kc, 2};
  GridWorkspace gw = c->gws;
  gw.cell_start += (int64_t)frame * (kGridCells + 1);
  gw.cell_items += (int64_t)frame * kc;
  MatchIO io{c->d_qmeta, c->d_qmeta + 1, c->d_mp, c->d_blk, c->d_nm, kc};
  TimerScope ts(c);
  if (f2f)
    launch_search_frame(cur, c->sout.u_right + frame * kc, kc, c->cam, c->gd(),
                        reinterpret_cast<const F2FQuery*>(qb),
                        reinterpret_cast<const F2FPose*>(eb), 1, nq, gw, c->mws, io, st);
  else
    launch_search_mps(cur, c->sout.u_right + frame * kc, kc, c->cam, c->gd(),
                      reinterpret_cast<const MpsQuery*>(qb), nnratio, th, 1, nq, gw, c->mws, io,
                      st);
  HIPCHECK(c, hipGetLastError());
  if (n) {
    HIPCHECK(c, hipMemcpyAsync(map_point, c->d_mp, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
    HIPCHECK(c, hipMemcpyAsync(blocked, c->d_blk, n, hipMemcpyDeviceToHost, st));
  }
  int nm = 0;
  HIPCHECK(c, hipMemcpyAsync(&nm, c->d_nm, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHECK(c, hipStreamSynchronize(st));
  if (nmatches) *nmatches = nm;
  return check_device_err(c);
}

extern "C" {

int slamgpu_search_by_projection_frame(slamgpu_ctx* c, int frame, const slamgpu_f2f_query* q,
                                       int nq, const slamgpu_f2f_pose* pose, int32_t* map_point,
                                       uint8_t* blocked, int n, int* nmatches) {
  if (!pose) return SLAMGPU_EINVAL;
  return host_search(c, frame, q, nq, map_point, blocked, n, nmatches, sizeof(slamgpu_f2f_pose),
                     pose, true, 0.f, 0);
}

int slamgpu_search_by_projection_mps(slamgpu_ctx* c, int frame, const slamgpu_mps_query* q,
                                     int nq, float nnratio, int th, int32_t* map_point,
                                     uint8_t* blocked, int n, int* nmatches) {
  return host_search(c, frame, q, nq, map_point, blocked, n, nmatches, 0, nullptr, false,
                     nnratio, th);
}

}  // extern "C"
