// capi_check.cpp -- the drop-in boundary exercised from C++ with no Python in between: a program
// built by g++ against include/*.h and linked to libslamgpu.so, as the reference's C++ callers
// would be (ORBextractor::Compute orb_extractor.h:25-93, Optimizer::PoseOptimization /
// LocalBundleAdjustment optimizer.h:13-52). Test infrastructure (tests/test_capi_cpp.py writes
// the inputs, runs this binary on the GPU box and compares its outputs with the committed golden
// fixture and the oracle).
//
//   capi_check <dir>
// reads   <dir>/image.u8            rows x cols u8 + <dir>/image.hdr "cols rows nfeatures"
//         <dir>/pose.bin            camera[5] f32, nlevels i32, inv_sigma2[nlevels] f32,
//                                   n i32, edges[n] (slamgpu_pose_edge), Tcw[16] f32
//         <dir>/lba.bin             camera[5], nlevels, inv_sigma2[], n_kf i32, kf_Tcw[16 n_kf],
//                                   kf_mode[n_kf] u8 (zero-padded to a multiple of 4),
//                                   n_points i32, points[3 n_points] f32,
//                                   point_obs_start[n_points + 1] i32, obs[n_obs]
//         <dir>/stereo.bin          cols, rows, nfeatures i32, camera[5] f32, left, right u8
//         <dir>/mps.bin             n_mp i32, per map point: bad, n_obs i32, desc[32], in_view
//                                   i32, proj_x, proj_y, proj_xr, view_cos f32, level i32;
//                                   n_local i32, local[n_local] i32, nnratio f32, th i32,
//                                   n i32, the current frame's map points[n] i32
// writes  <dir>/extract.kps, extract.desc      (n x 28, n x 32 bytes)
//         <dir>/pose.out            n_inliers i32, Tcw[16] f32, outlier[n] u8
//         <dir>/lba.out             lm_iterations i32, kf_Tcw[16 n_kf], points[3 n_points],
//                                   erase[n_obs] u8
//         <dir>/stereo.out          N, N_right i32, keys[N], desc[N], keys_right, desc_right,
//                                   right_coords[N], depth[N] f32, undist_keys[N]
//         <dir>/mps.out             nmatches i32, map points after the call[n] i32
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "slamgpu.h"
#include "slamgpu_adapters.hpp"
#include "slamgpu_optimizer.h"

namespace {

std::vector<char> slurp(const std::string& path) {
  std::vector<char> v;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", path.c_str());
    std::exit(2);
  }
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}

void spit(const std::string& path, const void* p, size_t n) {
  FILE* f = std::fopen(path.c_str(), "ab");
  if (!f || std::fwrite(p, 1, n, f) != n) {
    std::fprintf(stderr, "cannot write %s\n", path.c_str());
    std::exit(2);
  }
  std::fclose(f);
}

struct Reader {  // sequential reads out of a loaded file
  const std::vector<char>& b;
  size_t off = 0;
  template <typename T>
  const T* take(size_t count) {
    const size_t bytes = sizeof(T) * count;
    if (off + bytes > b.size()) {
      std::fprintf(stderr, "truncated input\n");
      std::exit(2);
    }
    const T* p = reinterpret_cast<const T*>(b.data() + off);
    off += bytes;
    return p;
  }
};

int check(int rc, const char* what, const char* err) {
  if (rc != 0) {
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, err ? err : "");
    std::exit(1);
  }
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: capi_check <dir>\n");
    return 2;
  }
  const std::string dir = argv[1];
  for (const char* f : {"/extract.kps", "/extract.desc", "/core.kps", "/core.desc", "/core.pyr1",
                        "/pose.out", "/lba.out", "/stereo.out", "/mps.out"})
    std::remove((dir + f).c_str());

  // ---- ORBextractor::Compute ----
  int cols = 0, rows = 0, nfeat = 0;
  {
    FILE* h = std::fopen((dir + "/image.hdr").c_str(), "r");
    if (!h || std::fscanf(h, "%d %d %d", &cols, &rows, &nfeat) != 3) return 2;
    std::fclose(h);
  }
  const std::vector<char> img = slurp(dir + "/image.u8");
  if ((int)img.size() != cols * rows) return 2;
  const slamgpu_orb_params prm = {nfeat, 1.2f, 8, 20, 7};
  slamgpu_ctx* ctx = nullptr;
  check(slamgpu_create(0, &prm, cols, rows, 1, &ctx), "slamgpu_create", slamgpu_last_error(nullptr));
  const int cap = slamgpu_kp_capacity(ctx);
  std::vector<slamgpu_keypoint> kps(cap);
  std::vector<uint8_t> desc((size_t)cap * 32);
  int n = 0;
  check(slamgpu_extract(ctx, reinterpret_cast<const uint8_t*>(img.data()), cols, kps.data(),
                        desc.data(), cap, &n),
        "slamgpu_extract", slamgpu_last_error(ctx));
  spit(dir + "/extract.kps", kps.data(), sizeof(slamgpu_keypoint) * n);
  spit(dir + "/extract.desc", desc.data(), 32 * (size_t)n);
  slamgpu_destroy(ctx);

  // ---- the same through the adapters' OpenCV-free ORBextractor (slamgpu_adapters.hpp) ----
  {
    slamgpu_adapter::OrbExtractorCore ex(nfeat, 1.2f, 8, 20, 7);
    std::vector<slamgpu_keypoint> k2;
    std::vector<uint8_t> d2;
    const int n2 = ex.Compute(reinterpret_cast<const uint8_t*>(img.data()), rows, cols,
                              (size_t)cols, k2, d2);
    if (n2 != n || (int)k2.size() != n || d2.size() != 32 * (size_t)n) return 3;
    spit(dir + "/core.kps", k2.data(), sizeof(slamgpu_keypoint) * n2);
    spit(dir + "/core.desc", d2.data(), d2.size());
    const std::vector<std::vector<uint8_t>>& pyr = ex.GetImagePyramid();
    if ((int)pyr.size() != 8 || ex.pyramid_size(0).first != cols) return 3;
    spit(dir + "/core.pyr1", pyr[1].data(), pyr[1].size());
    if (ex.GetScaleFactors().size() != 8 || ex.GetInverseScaleSigmaSquares()[7] <= 0.f) return 3;
  }

  // ---- Optimizer::PoseOptimization ----
  {
    const std::vector<char> b = slurp(dir + "/pose.bin");
    Reader r{b};
    const slamgpu_camera cam = *r.take<slamgpu_camera>(1);
    const int nl = *r.take<int32_t>(1);
    const float* isig = r.take<float>(nl);
    const int ne = *r.take<int32_t>(1);
    const slamgpu_pose_edge* edges = r.take<slamgpu_pose_edge>(ne);
    float T[16];
    for (int i = 0; i < 16; i++) T[i] = r.take<float>(1)[0];
    std::vector<uint8_t> outl(ne > 0 ? ne : 1);
    int inl = 0;
    check(slamgpu_pose_optimization(&cam, isig, nl, edges, ne, T, outl.data(), &inl),
          "slamgpu_pose_optimization", slamgpu_optimizer_last_error());
    spit(dir + "/pose.out", &inl, 4);
    spit(dir + "/pose.out", T, sizeof(T));
    spit(dir + "/pose.out", outl.data(), ne);
  }

  // ---- Optimizer::LocalBundleAdjustment (the reference's bool* stop flag, never raised) ----
  {
    const std::vector<char> b = slurp(dir + "/lba.bin");
    Reader r{b};
    const slamgpu_camera cam = *r.take<slamgpu_camera>(1);
    const int nl = *r.take<int32_t>(1);
    const float* isig = r.take<float>(nl);
    const int nk = *r.take<int32_t>(1);
    const float* kf0 = r.take<float>(16 * (size_t)nk);
    std::vector<float> kf(kf0, kf0 + 16 * (size_t)nk);
    const uint8_t* mode = r.take<uint8_t>((nk + 3) & ~3);  // padded to 4 bytes
    const int np = *r.take<int32_t>(1);
    const float* p0 = r.take<float>(3 * (size_t)np);
    std::vector<float> pts(p0, p0 + 3 * (size_t)np);
    const int32_t* start = r.take<int32_t>(np + 1);
    const int no = start[np];
    const slamgpu_ba_obs* obs = r.take<slamgpu_ba_obs>(no);
    std::vector<uint8_t> erase(no > 0 ? no : 1);
    bool stop = false;
    int its = 0;
    check(slamgpu_local_bundle_adjustment(&cam, isig, nl, kf.data(), mode, nk, pts.data(), np,
                                          start, obs, &stop, erase.data(), &its),
          "slamgpu_local_bundle_adjustment", slamgpu_optimizer_last_error());
    spit(dir + "/lba.out", &its, 4);
    spit(dir + "/lba.out", kf.data(), kf.size() * 4);
    spit(dir + "/lba.out", pts.data(), pts.size() * 4);
    spit(dir + "/lba.out", erase.data(), no);
  }
  // ---- the stereo Frame ctor (slamgpu_adapters.hpp StereoFrameCore over slamgpu_frame_stereo),
  // then SearchByProjection(F, vpMapPoints, th) on that frame through the adapter's one call ----
  {
    const std::vector<char> b = slurp(dir + "/stereo.bin");
    Reader r{b};
    const int sc = *r.take<int32_t>(1), sr = *r.take<int32_t>(1), sn = *r.take<int32_t>(1);
    const slamgpu_camera cam = *r.take<slamgpu_camera>(1);
    const uint8_t* left = r.take<uint8_t>((size_t)sc * sr);
    const uint8_t* right = r.take<uint8_t>((size_t)sc * sr);
    const slamgpu_orb_params sp = {sn, 1.2f, 8, 20, 7};
    slamgpu_adapter::StereoFrameCore core(sp, cam);
    slamgpu_adapter::StereoFrame f;
    core.Make(left, right, sr, sc, (size_t)sc, f);
    const std::string so = dir + "/stereo.out";
    const int32_t nn[2] = {f.N, (int32_t)f.keys_right.size()};
    spit(so, nn, sizeof nn);
    spit(so, f.keys.data(), sizeof(slamgpu_keypoint) * f.keys.size());
    spit(so, f.desc.data(), f.desc.size());
    spit(so, f.keys_right.data(), sizeof(slamgpu_keypoint) * f.keys_right.size());
    spit(so, f.desc_right.data(), f.desc_right.size());
    spit(so, f.right_coords.data(), 4 * f.right_coords.size());
    spit(so, f.depth.data(), 4 * f.depth.size());
    spit(so, f.undist_keys.data(), sizeof(slamgpu_keypoint) * f.undist_keys.size());

    const std::vector<char> m = slurp(dir + "/mps.bin");
    Reader q{m};
    const int n_mp = *q.take<int32_t>(1);
    std::vector<slamgpu_adapter::MapPointView> mps(n_mp);
    std::vector<slamgpu_adapter::TrackView> track(n_mp);
    for (int i = 0; i < n_mp; ++i) {
      mps[i] = slamgpu_adapter::MapPointView{};
      mps[i].id = i;
      mps[i].bad = *q.take<int32_t>(1) != 0;
      mps[i].n_obs = *q.take<int32_t>(1);
      mps[i].desc = q.take<uint8_t>(32);
      track[i].in_view = *q.take<int32_t>(1) != 0;
      const float* t = q.take<float>(4);
      track[i].proj_x = t[0];
      track[i].proj_y = t[1];
      track[i].proj_xr = t[2];
      track[i].view_cos = t[3];
      track[i].level = *q.take<int32_t>(1);
    }
    const int n_local = *q.take<int32_t>(1);
    const int32_t* local = q.take<int32_t>(n_local);
    const float nnratio = *q.take<float>(1);
    const int th = *q.take<int32_t>(1);
    const int nk = *q.take<int32_t>(1);
    if (nk != f.N) return 4;
    const int32_t* mp0 = q.take<int32_t>(nk);
    f.map_points.assign(mp0, mp0 + nk);
    const float Tcw[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const slamgpu_adapter::FrameView cv = slamgpu_adapter::StereoFrameCore::view(f, Tcw);
    std::vector<int32_t> after(f.map_points);
    const int nm = slamgpu_adapter::search_by_projection_mps(core.context(), 0, cv, mps.data(),
                                                             local, n_local, track.data(),
                                                             nnratio, th, after.data());
    spit(dir + "/mps.out", &nm, 4);
    spit(dir + "/mps.out", after.data(), 4 * after.size());
  }
  std::printf("capi_check ok: %d keypoints\n", n);
  return 0;
}
