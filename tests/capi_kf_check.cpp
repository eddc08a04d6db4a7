// capi_kf_check.cpp -- the keyframe-rate surfaces of the drop-in boundary driven from
// C++ through include/slamgpu_adapters.hpp, as a reference-side adapter would call them: views of
// a map (KeyFrames, MapPoints) in, the adapters' gathering, the device calls through the C ABI,
// the write-back out. Test infrastructure: tests/test_capi_kf_cpp.py writes the map and the
// calls, runs this binary on the GPU box and compares its outputs with the oracle.
//
//   capi_kf_check <dir>
// reads   <dir>/map.bin    n_kf, n_mp i32; per keyframe: id i64, bad i32, Tcw[16], Ow[3] f32,
//                          n i32, undist_kps[n] (28 B), right_coords[n] f32, map_points[n] i32,
//                          desc[32 n], n_nodes i32, nodes[n_nodes] u32, node_start[n_nodes+1]
//                          i32, node_feats[node_start[n_nodes]] u32;
//                          per map point: id i64, bad i32, xyz[3] f32, desc[32], n_obs i32,
//                          obs[n_obs] (keyframe, keypoint) i32, normal[3], min_dist, max_dist
//                          f32, num_observations i32
//         <dir>/calls.bin  camera[5] f32, slamgpu_levels, slamgpu_kf_grid, nlevels i32,
//                          inv_sigma2[nlevels] f32;
//                          SearchByBoW(KF, Frame): kf, frame-keyframe i32, nnratio f32, ori i32;
//                          SearchByBoW(KF, KF): kf1, kf2 i32, nnratio f32, ori i32;
//                          SearchForTriangulation: kf1, kf2 i32, F12[9] f32, only_stereo, ori;
//                          Fuse: kf i32, th f32, n i32, points[n] i32;
//                          OptimizeSim3: kf1, kf2 i32, n i32, matches1[n] i32, K1[4], K2[4] f32,
//                          th2 f32, fix_scale i32, S12[8] f64;
//                          GBA: n_iterations, robust i32
// writes  <dir>/kf.out     (appended in the order above) bow1: nmatches, matches[n_frame];
//                          bow2: nmatches, matches12[n_kf1]; tri: n_pairs, pairs[2 n_pairs];
//                          fuse: nfused, n_actions, actions[4 n_actions]; sim3: n_in i32,
//                          S12[8] f64, matches1[n] i32; gba: lm_iterations, n_kfv, keyframe[],
//                          kf_Tcw[16 n_kfv] f32, n_pts, map_point[], points[3 n_pts] f32,
//                          n_obs, obs[n_obs] (slamgpu_ba_obs)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "slamgpu_adapters.hpp"

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

struct Writer {
  FILE* f;
  template <typename T>
  void put(const T* p, size_t count) {
    if (count && std::fwrite(p, sizeof(T), count, f) != count) {
      std::fprintf(stderr, "write failed\n");
      std::exit(2);
    }
  }
  template <typename T>
  void put1(T v) { put(&v, 1); }
};

struct Reader {
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
  template <typename T>
  T get() { return *take<T>(1); }
};

}  // namespace

int main(int argc, char** argv) {
  using namespace slamgpu_adapter;
  if (argc != 2) {
    std::fprintf(stderr, "usage: capi_kf_check <dir>\n");
    return 2;
  }
  const std::string dir = argv[1];
  const std::vector<char> mb = slurp(dir + "/map.bin"), cb = slurp(dir + "/calls.bin");
  Reader m{mb};
  const int n_kf = m.get<int32_t>(), n_mp = m.get<int32_t>();
  std::vector<KeyFrameView> kfs(n_kf);
  std::vector<KeyFrameFeatures> kff(n_kf);
  for (int k = 0; k < n_kf; ++k) {
    KeyFrameView& v = kfs[k];
    v.id = m.get<int64_t>();
    v.bad = m.get<int32_t>() != 0;
    v.Tcw = m.take<float>(16);
    kff[k].Ow = m.take<float>(3);
    v.n_kps = m.get<int32_t>();
    v.undist_kps = m.take<slamgpu_keypoint>(v.n_kps);
    v.right_coords = m.take<float>(v.n_kps);
    v.map_points = m.take<int32_t>(v.n_kps);
    v.covisible = nullptr;
    v.n_covisible = 0;
    kff[k].desc = m.take<uint8_t>(32 * (size_t)v.n_kps);
    FeatureVecView& fv = kff[k].fv;
    fv.n_nodes = m.get<int32_t>();
    fv.nodes = m.take<uint32_t>(fv.n_nodes);
    fv.node_start = m.take<int32_t>(fv.n_nodes + 1);
    fv.node_feats = m.take<uint32_t>(fv.node_start[fv.n_nodes]);
  }
  std::vector<MapPointView> mps(n_mp);
  std::vector<MapPointGeometry> geom(n_mp);
  for (int p = 0; p < n_mp; ++p) {
    MapPointView& v = mps[p];
    v.id = m.get<int64_t>();
    v.bad = m.get<int32_t>() != 0;
    const float* x = m.take<float>(3);
    for (int i = 0; i < 3; ++i) v.xyz[i] = x[i];
    v.desc = m.take<uint8_t>(32);
    v.n_obs = m.get<int32_t>();
    v.obs = m.take<ObsRef>(v.n_obs);
    const float* nm = m.take<float>(3);
    for (int i = 0; i < 3; ++i) geom[p].normal[i] = nm[i];
    geom[p].min_dist = m.get<float>();
    geom[p].max_dist = m.get<float>();
    geom[p].num_observations = m.get<int32_t>();
  }

  Reader c{cb};
  const float* camf = c.take<float>(5);
  const slamgpu_camera cam = {camf[0], camf[1], camf[2], camf[3], camf[4]};
  const slamgpu_levels lv = c.get<slamgpu_levels>();
  const slamgpu_kf_grid grid = c.get<slamgpu_kf_grid>();
  const int nlevels = c.get<int32_t>();
  const float* inv_sigma2 = c.take<float>(nlevels);

  const std::string out_path = dir + "/kf.out";
  std::remove(out_path.c_str());
  Writer w{std::fopen(out_path.c_str(), "wb")};
  if (!w.f) return 2;
  try {
    {  // SearchByBoW(KeyFrame*, Frame&): the Frame is another keyframe's features here
      const int k = c.get<int32_t>(), f = c.get<int32_t>();
      const float nnratio = c.get<float>();
      const bool ori = c.get<int32_t>() != 0;
      std::vector<int32_t> mpm;
      const int nm = search_by_bow(kfs[k], kff[k], mps.data(), kfs[f].undist_kps, kff[f].desc,
                                   kfs[f].n_kps, kff[f].fv, nnratio, ori, mpm);
      w.put1<int32_t>(nm);
      w.put(mpm.data(), mpm.size());
    }
    {  // SearchByBoW(KeyFrame*, KeyFrame*)
      const int k1 = c.get<int32_t>(), k2 = c.get<int32_t>();
      const float nnratio = c.get<float>();
      const bool ori = c.get<int32_t>() != 0;
      std::vector<int32_t> m12;
      const int nm = search_by_bow(kfs[k1], kff[k1], kfs[k2], kff[k2], mps.data(), nnratio, ori, m12);
      w.put1<int32_t>(nm);
      w.put(m12.data(), m12.size());
    }
    {  // SearchForTriangulation
      const int k1 = c.get<int32_t>(), k2 = c.get<int32_t>();
      const float* F12 = c.take<float>(9);
      const bool only_stereo = c.get<int32_t>() != 0, ori = c.get<int32_t>() != 0;
      const auto pairs =
          search_for_triangulation(kfs[k1], kff[k1], kfs[k2], kff[k2], F12, cam, lv, only_stereo, ori);
      w.put1<int32_t>((int32_t)pairs.size());
      for (const auto& p : pairs) {
        w.put1<int32_t>(p.first);
        w.put1<int32_t>(p.second);
      }
    }
    {  // Fuse(pKF, vpMapPoints, th)
      const int k = c.get<int32_t>();
      const float th = c.get<float>();
      const int n = c.get<int32_t>();
      const int32_t* pts = c.take<int32_t>(n);
      const FuseResult r = fuse(k, kfs.data(), kff[k], mps.data(), geom.data(), n_mp, pts, n, th,
                                cam, lv, grid);
      w.put1<int32_t>(r.nfused);
      w.put1<int32_t>((int32_t)r.actions.size());
      for (const FuseAction& a : r.actions) {
        w.put1<int32_t>(a.kind);
        w.put1<int32_t>(a.point);
        w.put1<int32_t>(a.other);
        w.put1<int32_t>(a.keypoint);
      }
    }
    {  // OptimizeSim3
      const int k1 = c.get<int32_t>(), k2 = c.get<int32_t>(), n = c.get<int32_t>();
      const int32_t* m1 = c.take<int32_t>(n);
      std::vector<int32_t> matches1(m1, m1 + n);
      const float* K1 = c.take<float>(4);
      const float* K2 = c.take<float>(4);
      const float th2 = c.get<float>();
      const bool fix = c.get<int32_t>() != 0;
      double S12[8];
      const double* s0 = c.take<double>(8);
      for (int i = 0; i < 8; ++i) S12[i] = s0[i];
      const int n_in = optimize_sim3(k1, k2, kfs.data(), mps.data(), matches1.data(), n, K1, K2,
                                     lv.inv_sigma2, lv.inv_sigma2, lv.nlevels, S12, th2, fix);
      w.put1<int32_t>(n_in);
      w.put(S12, 8);
      w.put(matches1.data(), matches1.size());
    }
    {  // the global BundleAdjustment
      const int n_it = c.get<int32_t>();
      const bool robust = c.get<int32_t>() != 0;
      LocalBaGraph g = gather_global_bundle_adjustment(kfs.data(), n_kf, mps.data(), n_mp);
      const int its = global_bundle_adjustment(g, cam, inv_sigma2, nlevels, n_it, robust, nullptr);
      w.put1<int32_t>(its);
      w.put1<int32_t>((int32_t)g.keyframe.size());
      w.put(g.keyframe.data(), g.keyframe.size());
      w.put(g.kf_Tcw.data(), g.kf_Tcw.size());
      w.put1<int32_t>((int32_t)g.map_point.size());
      w.put(g.map_point.data(), g.map_point.size());
      w.put(g.points.data(), g.points.size());
      w.put1<int32_t>((int32_t)g.obs.size());
      w.put(g.obs.data(), g.obs.size());
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    std::fclose(w.f);
    return 1;
  }
  std::fclose(w.f);
  std::printf("capi_kf_check ok\n");
  return 0;
}
