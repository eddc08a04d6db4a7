// adapter_check.cpp -- drives include/slamgpu_adapters.hpp (the OpenCV-free graph gathering and
// write-back of Optimizer / both per-frame OrbMatcher::SearchByProjection) on a map read from a file, and writes every record the
// helpers produce, for tests/test_adapters.py to compare with its own restatement of
// optimizer.cpp / orb_matcher.cpp. Test infrastructure; CPU only (the one library call,
// slamgpu_orb_scale_tables, touches no device).
//
//   adapter_check <scenario.bin> <out.bin>     (layouts: tests/test_adapters.py write_scenario /
//                                               read_outputs)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "slamgpu_adapters.hpp"

namespace {

namespace A = slamgpu_adapter;

std::vector<char> slurp(const char* path) {
  std::vector<char> v;
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", path);
    std::exit(2);
  }
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}

struct Reader {
  const std::vector<char>& b;
  size_t off = 0;
  template <typename T>
  const T* take(size_t count) {
    const size_t bytes = sizeof(T) * count;
    if (off + bytes > b.size()) {
      std::fprintf(stderr, "truncated scenario\n");
      std::exit(2);
    }
    const T* p = reinterpret_cast<const T*>(b.data() + off);
    off += (bytes + 3) & ~size_t(3);  // every array padded to 4 bytes
    return p;
  }
  int32_t i32() { return *take<int32_t>(1); }
};

struct Writer {
  std::vector<char> out;
  template <typename T>
  void put(const T* p, size_t count) {
    const char* c = reinterpret_cast<const char*>(p);
    out.insert(out.end(), c, c + sizeof(T) * count);
    while (out.size() & 3) out.push_back(0);
  }
  void i32(int32_t v) { put(&v, 1); }
};

A::FrameView read_frame(Reader& r) {
  A::FrameView f;
  f.Tcw = r.take<float>(16);
  f.n_kps = r.i32();
  f.kps = r.take<slamgpu_keypoint>(f.n_kps);
  f.undist_kps = r.take<slamgpu_keypoint>(f.n_kps);
  f.right_coords = r.take<float>(f.n_kps);
  f.map_points = r.take<int32_t>(f.n_kps);
  f.outlier = r.take<uint8_t>(f.n_kps);
  return f;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: adapter_check <scenario.bin> <out.bin>\n");
    return 2;
  }
  const std::vector<char> buf = slurp(argv[1]);
  Reader r{buf};
  const int n_kf = r.i32(), n_mp = r.i32(), current = r.i32();
  std::vector<A::KeyFrameView> kfs(n_kf);
  for (auto& k : kfs) {
    k.id = *r.take<int64_t>(1);
    k.bad = r.i32() != 0;
    k.Tcw = r.take<float>(16);
    k.n_kps = r.i32();
    k.undist_kps = r.take<slamgpu_keypoint>(k.n_kps);
    k.right_coords = r.take<float>(k.n_kps);
    k.map_points = r.take<int32_t>(k.n_kps);
    k.n_covisible = r.i32();
    k.covisible = r.take<int32_t>(k.n_covisible);
  }
  std::vector<A::MapPointView> mps(n_mp);
  for (auto& m : mps) {
    m.id = *r.take<int64_t>(1);
    m.bad = r.i32() != 0;
    const float* x = r.take<float>(3);
    m.xyz[0] = x[0];
    m.xyz[1] = x[1];
    m.xyz[2] = x[2];
    m.desc = r.take<uint8_t>(32);
    m.n_obs = r.i32();
    m.obs = r.take<A::ObsRef>(m.n_obs);
  }
  const A::FrameView cur = read_frame(r), last = read_frame(r);
  const float baseline = *r.take<float>(1), th = *r.take<float>(1);
  const bool mono = r.i32() != 0, check_ori = r.i32() != 0;
  slamgpu_orb_params op;
  op.nfeatures = r.i32();
  op.scale_factor = *r.take<float>(1);
  op.nlevels = r.i32();
  op.ini_th_fast = r.i32();
  op.min_th_fast = r.i32();
  // Tracker::SearchLocalPoints' local map point list and every map point's track_* fields
  const int n_local = r.i32();
  const int32_t* local = r.take<int32_t>(n_local);
  std::vector<A::TrackView> track(n_mp);
  for (auto& t : track) {
    t.in_view = r.i32() != 0;
    const float* f = r.take<float>(4);
    t.proj_x = f[0];
    t.proj_y = f[1];
    t.proj_xr = f[2];
    t.view_cos = f[3];
    t.level = r.i32();
  }

  Writer w;
  // Optimizer::PoseOptimization on the current frame; then an outlier per odd edge
  const A::PoseGraph pg = A::gather_pose_optimization(cur, mps.data());
  w.i32((int32_t)pg.edges.size());
  w.put(pg.edges.data(), pg.edges.size());
  w.put(pg.keypoint.data(), pg.keypoint.size());
  std::vector<uint8_t> edge_out(pg.edges.size()), frame_out(cur.outlier, cur.outlier + cur.n_kps);
  for (size_t k = 0; k < edge_out.size(); ++k) edge_out[k] = k & 1;
  A::apply_pose_optimization(pg, edge_out.data(), frame_out.data());
  w.put(frame_out.data(), frame_out.size());
  // Optimizer::LocalBundleAdjustment around `current`; then every third edge erased
  const A::LocalBaGraph g = A::gather_local_bundle_adjustment(kfs.data(), n_kf, mps.data(), n_mp,
                                                              current);
  w.i32((int32_t)g.keyframe.size());
  w.put(g.keyframe.data(), g.keyframe.size());
  w.put(g.kf_Tcw.data(), g.kf_Tcw.size());
  w.put(g.kf_mode.data(), g.kf_mode.size());
  w.i32(g.n_local);
  w.i32((int32_t)g.map_point.size());
  w.put(g.map_point.data(), g.map_point.size());
  w.put(g.points.data(), g.points.size());
  w.put(g.point_obs_start.data(), g.point_obs_start.size());
  w.i32((int32_t)g.obs.size());
  w.put(g.obs.data(), g.obs.size());
  w.put(g.obs_ref.data(), g.obs_ref.size());
  std::vector<uint8_t> erase(g.obs.size());
  for (size_t e = 0; e < erase.size(); ++e) erase[e] = e % 3 == 0;
  const A::LocalBaResult res = A::local_bundle_adjustment_result(g, erase.data());
  w.i32((int32_t)res.erase_match.size());
  w.put(res.erase_match.data(), res.erase_match.size());
  w.put(res.erase_obs_point.data(), res.erase_obs_point.size());
  w.i32((int32_t)res.pose_keyframe.size());
  w.put(res.pose_keyframe.data(), res.pose_keyframe.size());
  w.put(res.pose.data(), res.pose.size());
  // OrbMatcher::SearchByProjection(current, last, th, mono); then a synthetic claim pattern
  const A::F2FInput in = A::gather_search_by_projection_frame(cur, last, mps.data(), baseline, th,
                                                              mono, check_ori);
  w.i32((int32_t)in.queries.size());
  w.put(in.queries.data(), in.queries.size());
  w.put(in.query_map_point.data(), in.query_map_point.size());
  w.put(&in.pose, 1);
  std::vector<int32_t> slot(cur.n_kps);
  std::vector<uint8_t> blocked(cur.n_kps);
  A::f2f_current_state(cur, mps.data(), slot.data(), blocked.data());
  w.put(slot.data(), slot.size());
  w.put(blocked.data(), blocked.size());
  const int nq = (int)in.queries.size();
  for (int i = 0; i < cur.n_kps; ++i) slot[i] = (nq > 0 && i % 5 == 0) ? i % nq : -1;
  std::vector<int32_t> after(cur.map_points, cur.map_points + cur.n_kps);
  w.i32(A::apply_search_by_projection_frame(in, slot.data(), after.data(), cur.n_kps));
  w.put(after.data(), after.size());
  // OrbMatcher::SearchByProjection(current, local map points, th); then a synthetic claim pattern
  const A::MpsInput mi = A::gather_search_by_projection_mps(local, n_local, mps.data(),
                                                            track.data());
  w.i32((int32_t)mi.queries.size());
  w.put(mi.queries.data(), mi.queries.size());
  w.put(mi.query_map_point.data(), mi.query_map_point.size());
  const int nmq = (int)mi.queries.size();
  for (int i = 0; i < cur.n_kps; ++i) slot[i] = (nmq > 0 && i % 3 == 1) ? (7 * i) % nmq : -1;
  std::vector<int32_t> after_mps(cur.map_points, cur.map_points + cur.n_kps);
  w.i32(A::apply_search_by_projection_mps(mi, slot.data(), after_mps.data(), cur.n_kps));
  w.put(after_mps.data(), after_mps.size());
  // ORBextractor's getters without a device context
  const A::OrbTables t = A::orb_scale_tables(op);
  w.i32(t.rc);
  for (const std::vector<float>* v : {&t.scale, &t.inv_scale, &t.sigma2, &t.inv_sigma2})
    w.put(v->data(), v->size());
  w.put(t.features_per_level.data(), t.features_per_level.size());

  FILE* f = std::fopen(argv[2], "wb");
  if (!f || std::fwrite(w.out.data(), 1, w.out.size(), f) != w.out.size()) return 2;
  std::fclose(f);
  return 0;
}
