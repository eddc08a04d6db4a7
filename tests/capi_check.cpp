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
// writes  <dir>/extract.kps, extract.desc      (n x 28, n x 32 bytes)
//         <dir>/pose.out            n_inliers i32, Tcw[16] f32, outlier[n] u8
//         <dir>/lba.out             lm_iterations i32, kf_Tcw[16 n_kf], points[3 n_points],
//                                   erase[n_obs] u8
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
                        "/pose.out", "/lba.out"})
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
  std::printf("capi_check ok: %d keypoints\n", n);
  return 0;
}
