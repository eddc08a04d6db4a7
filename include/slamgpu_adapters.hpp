// slamgpu_adapters.hpp -- the graph gathering and write-back of the reference's Optimizer and
// OrbMatcher entry points, as OpenCV- and g2o-free C++17 over plain views of the map (header only).
//
// The reference builds its g2o graphs and matcher inputs from Frame / KeyFrame / MapPoint objects
// (src/optimizer/optimizer.cpp, src/orb_features/orb_matcher.cpp). The C ABI (slamgpu.h,
// slamgpu_optimizer.h) takes arrays instead. These helpers turn plain views of those objects into
// the ABI records in exactly the order optimizer.cpp creates its vertices and edges, and apply the
// results back as the reference does, so a reference-side adapter is a loop that fills the views
// (Frame::GetMapPoint, KeyFrame::GetMapPointMatches, MapPoint::GetObservations, ...) and calls
// one function. tests/adapter_check.cpp drives them against an independent restatement of the
// reference's gathering (tests/test_adapters.py), and tests/capi_check.cpp feeds their output to
// the device.
#pragma once
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "slamgpu.h"
#include "slamgpu_optimizer.h"

namespace slamgpu_adapter {

// ---- views of the reference's objects (indices into caller-owned arrays, -1 = none) ---------

// One observation of a map point: MapPoint::GetObservations()'s (KeyFrame*, keypoint index),
// the keyframe given as its index in the keyframe array.
struct ObsRef {
  int32_t keyframe;
  int32_t keypoint;
};

struct MapPointView {
  int64_t id;                // MapPoint::GetId()
  bool bad;                  // isBad()
  float xyz[3];              // GetWorldPos()
  const uint8_t* desc;       // GetDescriptor() (32 B)
  const ObsRef* obs;         // GetObservations(), in the std::map's iteration order
  int n_obs;                 // NumObservations() counts these
};

struct KeyFrameView {
  int64_t id;                          // KeyFrame::Id()
  bool bad;                            // isBad()
  const float* Tcw;                    // GetPose(): 4x4 row-major f32
  const slamgpu_keypoint* undist_kps;  // undistorted_keypoints
  const float* right_coords;           // right_coords (< 0: monocular)
  const int32_t* map_points;           // GetMapPointMatches(): map point index per keypoint
  int n_kps;
  const int32_t* covisible;            // GetVectorCovisibleKeyFrames(): keyframe indices
  int n_covisible;
};

struct FrameView {
  const float* Tcw;                    // GetPose(): 4x4 row-major f32
  const slamgpu_keypoint* kps;         // GetKeys()
  const slamgpu_keypoint* undist_kps;  // GetUndistortedKeys()
  const float* right_coords;           // StereoCoordRight()
  const int32_t* map_points;           // GetMapPoint(i): map point index or -1
  const uint8_t* outlier;              // IsOutlier(i)
  int n_kps;
};

// ---- ORBextractor (orb_extractor.h:25-93) without OpenCV ----------------------------------------

// The ctor's tables (orb_extractor.cpp:351-387), host-side: what GetScaleFactors /
// GetInverseScaleFactors / GetScaleSigmaSquares / GetInverseScaleSigmaSquares return.
struct OrbTables {
  int rc = SLAMGPU_EINVAL;
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> features_per_level;
};

inline OrbTables orb_scale_tables(const slamgpu_orb_params& p) {
  OrbTables t;
  const int n = p.nlevels > 0 && p.nlevels <= 12 ? p.nlevels : 0;
  t.scale.resize(n);
  t.inv_scale.resize(n);
  t.sigma2.resize(n);
  t.inv_sigma2.resize(n);
  t.features_per_level.resize(n);
  t.rc = slamgpu_orb_scale_tables(&p, t.scale.data(), t.inv_scale.data(), t.sigma2.data(),
                                  t.inv_sigma2.data(), t.features_per_level.data());
  return t;
}

// The ORBextractor surface over plain buffers: the device context is created on the first
// Compute (and again when the image size changes); the tables never need one. The OpenCV class
// (slamgpu_orb_adapter.hpp) is a thin shell over this one.
class OrbExtractorCore {
 public:
  OrbExtractorCore(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                   int device = 0)
      : params_{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST}, device_(device),
        tables_(orb_scale_tables(params_)) {
    if (tables_.rc != SLAMGPU_OK) throw std::invalid_argument("slamgpu: invalid ORB parameters");
  }
  ~OrbExtractorCore() { slamgpu_destroy(ctx_); }
  OrbExtractorCore(const OrbExtractorCore&) = delete;
  OrbExtractorCore& operator=(const OrbExtractorCore&) = delete;

  // orb_extractor.cpp:985-1049 on an 8-bit image: kps / desc (N x 32) replaced; returns N. An
  // empty image (rows or cols 0) leaves the outputs untouched and returns -1 (:990-991).
  int Compute(const uint8_t* image, int rows, int cols, size_t step,
              std::vector<slamgpu_keypoint>& kps, std::vector<uint8_t>& desc) {
    if (!image || rows <= 0 || cols <= 0) return -1;
    ensure(cols, rows);
    const int cap = slamgpu_kp_capacity(ctx_);
    kps.resize(cap);
    desc.resize((size_t)cap * 32);
    int n = 0;
    check(slamgpu_extract(ctx_, image, step, kps.data(), desc.data(), cap, &n));
    kps.resize(n);
    desc.resize((size_t)n * 32);
    pyramid_valid_ = false;
    return n;
  }

  int GetLevels() const { return params_.nlevels; }
  float GetScaleFactor() const { return params_.scale_factor; }
  const std::vector<float>& GetScaleFactors() const { return tables_.scale; }
  const std::vector<float>& GetInverseScaleFactors() const { return tables_.inv_scale; }
  const std::vector<float>& GetScaleSigmaSquares() const { return tables_.sigma2; }
  const std::vector<float>& GetInverseScaleSigmaSquares() const { return tables_.inv_sigma2; }

  // GetImagePyramid (orb_extractor.h:62) of the last Compute, downloaded on first use: level l is
  // pyramid_size(l) = (cols, rows), rows of `cols` bytes.
  const std::vector<std::vector<uint8_t>>& GetImagePyramid() {
    if (!pyramid_valid_) {
      if (!ctx_) throw std::logic_error("slamgpu: GetImagePyramid before Compute");
      pyramid_.assign(params_.nlevels, {});
      sizes_.assign(params_.nlevels, {0, 0});
      for (int l = 0; l < params_.nlevels; l++) {
        int w = 0, h = 0;
        check(slamgpu_get_pyramid_level(ctx_, 0, l, nullptr, 0, &w, &h));
        pyramid_[l].resize((size_t)w * h);
        check(slamgpu_get_pyramid_level(ctx_, 0, l, pyramid_[l].data(), (size_t)w, &w, &h));
        sizes_[l] = {w, h};
      }
      pyramid_valid_ = true;
    }
    return pyramid_;
  }
  std::pair<int, int> pyramid_size(int level) const { return sizes_.at(level); }

  slamgpu_ctx* context() { return ctx_; }

 private:
  void ensure(int cols, int rows) {
    if (ctx_ && cols == cols_ && rows == rows_) return;
    slamgpu_destroy(ctx_);
    ctx_ = nullptr;
    check(slamgpu_create(device_, &params_, cols, rows, 1, &ctx_));
    cols_ = cols;
    rows_ = rows;
  }
  void check(int rc) const {
    if (rc != SLAMGPU_OK) throw std::runtime_error(std::string("slamgpu: ") +
                                                   slamgpu_last_error(ctx_));
  }

  slamgpu_orb_params params_;
  int device_;
  OrbTables tables_;
  slamgpu_ctx* ctx_ = nullptr;
  int cols_ = 0, rows_ = 0;
  bool pyramid_valid_ = false;
  std::vector<std::vector<uint8_t>> pyramid_;
  std::vector<std::pair<int, int>> sizes_;
};

// ---- Optimizer::PoseOptimization (optimizer.cpp:209-411) ---------------------------------------

struct PoseGraph {
  std::vector<slamgpu_pose_edge> edges;  // one per keypoint with a map point, keypoint order
  std::vector<int32_t> keypoint;         // the keypoint of each edge (vnIndexEdgeMono/Stereo)
};

// optimizer.cpp:247-327: an edge for every keypoint that has a map point (no isBad test there),
// monocular when StereoCoordRight()[i] < 0, with the undistorted keypoint as the measurement.
inline PoseGraph gather_pose_optimization(const FrameView& f, const MapPointView* mps) {
  PoseGraph g;
  for (int i = 0; i < f.n_kps; ++i) {
    const int m = f.map_points[i];
    if (m < 0) continue;
    const slamgpu_keypoint& k = f.undist_kps[i];
    slamgpu_pose_edge e;
    std::memcpy(e.xw, mps[m].xyz, sizeof e.xw);
    e.u = k.x;
    e.v = k.y;
    e.ur = f.right_coords[i];
    e.octave = k.octave;
    g.edges.push_back(e);
    g.keypoint.push_back(i);
  }
  return g;
}

// optimizer.cpp:262,289 + :349-397: the frame's outlier flags after the call (every keypoint with
// an edge is (re)classified; the others keep theirs).
inline void apply_pose_optimization(const PoseGraph& g, const uint8_t* edge_outlier,
                                    uint8_t* frame_outlier) {
  for (size_t k = 0; k < g.keypoint.size(); ++k) frame_outlier[g.keypoint[k]] = edge_outlier[k];
}

// ---- Optimizer::LocalBundleAdjustment (optimizer.cpp:413-716) ----------------------------------

struct LocalBaGraph {
  std::vector<int32_t> keyframe;      // keyframe index of each vertex: local keyframes, then fixed
  std::vector<float> kf_Tcw;          // [n][16]
  std::vector<uint8_t> kf_mode;       // SLAMGPU_KF_*
  std::vector<int32_t> map_point;     // map point index of each point vertex
  std::vector<float> points;          // [n][3]
  std::vector<int32_t> point_obs_start;
  std::vector<slamgpu_ba_obs> obs;    // edges, per point in observation order
  std::vector<ObsRef> obs_ref;        // (keyframe index, keypoint index) of each edge
  int n_local = 0;
};

// The graph gathering of optimizer.cpp:416-605. Local keyframes: the current one and its
// covisible keyframes that are not bad (every covisible one is marked local, bad or not,
// :422-427); local map points: the local keyframes' map point matches in order, not bad, each
// once (:431-442); fixed cameras: keyframes observing a local point that are neither marked
// local nor already fixed, in observation order, kept if not bad (:445-461). Vertices: local
// keyframes (fixed when Id() == 0), fixed cameras, then the points; edges per point in
// GetObservations() order, skipping bad keyframes (:537-605).
inline LocalBaGraph gather_local_bundle_adjustment(const KeyFrameView* kfs, int n_kf,
                                                   const MapPointView* mps, int n_mp,
                                                   int current) {
  LocalBaGraph g;
  std::vector<uint8_t> kf_local(n_kf, 0), kf_fixed(n_kf, 0), mp_local(n_mp, 0);
  std::vector<int32_t> local_kfs, fixed_kfs, vertex_of(n_kf, -1);
  kf_local[current] = 1;
  local_kfs.push_back(current);
  const KeyFrameView& cur = kfs[current];
  for (int c = 0; c < cur.n_covisible; ++c) {
    const int k = cur.covisible[c];
    kf_local[k] = 1;
    if (!kfs[k].bad) local_kfs.push_back(k);
  }
  for (int k : local_kfs) {
    const KeyFrameView& kf = kfs[k];
    for (int i = 0; i < kf.n_kps; ++i) {
      const int m = kf.map_points[i];
      if (m >= 0 && !mps[m].bad && !mp_local[m]) {
        mp_local[m] = 1;
        g.map_point.push_back(m);
      }
    }
  }
  for (int m : g.map_point) {
    for (int o = 0; o < mps[m].n_obs; ++o) {
      const int k = mps[m].obs[o].keyframe;
      if (!kf_local[k] && !kf_fixed[k]) {
        kf_fixed[k] = 1;
        if (!kfs[k].bad) fixed_kfs.push_back(k);
      }
    }
  }
  auto add_kf = [&](int k, uint8_t mode) {
    vertex_of[k] = (int32_t)g.keyframe.size();
    g.keyframe.push_back(k);
    g.kf_Tcw.insert(g.kf_Tcw.end(), kfs[k].Tcw, kfs[k].Tcw + 16);
    g.kf_mode.push_back(mode);
  };
  for (int k : local_kfs) add_kf(k, kfs[k].id == 0 ? SLAMGPU_KF_LOCAL_FIXED : SLAMGPU_KF_LOCAL);
  g.n_local = (int)local_kfs.size();
  for (int k : fixed_kfs) add_kf(k, SLAMGPU_KF_FIXED);
  g.point_obs_start.push_back(0);
  for (int m : g.map_point) {
    g.points.insert(g.points.end(), mps[m].xyz, mps[m].xyz + 3);
    for (int o = 0; o < mps[m].n_obs; ++o) {
      const ObsRef r = mps[m].obs[o];
      if (kfs[r.keyframe].bad) continue;
      const slamgpu_keypoint& kp = kfs[r.keyframe].undist_kps[r.keypoint];
      slamgpu_ba_obs e;
      e.keyframe = vertex_of[r.keyframe];
      e.u = kp.x;
      e.v = kp.y;
      e.ur = kfs[r.keyframe].right_coords[r.keypoint];
      e.octave = kp.octave;
      g.obs.push_back(e);
      g.obs_ref.push_back(r);
    }
    g.point_obs_start.push_back((int32_t)g.obs.size());
  }
  return g;
}

// The write-back of optimizer.cpp:667-716 as a list of changes for the caller to apply under
// map->map_update_mutex: the (keyframe, keypoint) / (map point, keyframe) pairs to erase
// (EraseMapPointMatch + EraseObservation for every erase[e]), the local keyframes' poses
// (SetPose), every point's position (SetWorldPos + UpdateNormalAndDepth).
struct LocalBaResult {
  std::vector<ObsRef> erase_match;      // KeyFrame::EraseMapPointMatch(keypoint)
  std::vector<int32_t> erase_obs_point; // MapPoint::EraseObservation(keyframe) of these points
  std::vector<int32_t> pose_keyframe;   // SetPose(pose[16 k]) of these keyframes
  std::vector<float> pose;
};

inline LocalBaResult local_bundle_adjustment_result(const LocalBaGraph& g, const uint8_t* erase) {
  LocalBaResult r;
  for (size_t p = 0; p + 1 < g.point_obs_start.size(); ++p)
    for (int e = g.point_obs_start[p]; e < g.point_obs_start[p + 1]; ++e)
      if (erase[e]) {
        r.erase_match.push_back(g.obs_ref[e]);
        r.erase_obs_point.push_back(g.map_point[p]);
      }
  for (int v = 0; v < g.n_local; ++v) {
    r.pose_keyframe.push_back(g.keyframe[v]);
    r.pose.insert(r.pose.end(), g.kf_Tcw.begin() + 16 * v, g.kf_Tcw.begin() + 16 * v + 16);
  }
  return r;
}

// ---- OrbMatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (orb_matcher.cpp:1312) ----

struct F2FInput {
  std::vector<slamgpu_f2f_query> queries;  // one per last-frame map point that is not an outlier
  std::vector<int32_t> query_map_point;    // map point index of each query (mp_id = position)
  slamgpu_f2f_pose pose;
};

// tlc = Rlw * (-Rcw^T tcw) + tlw in f32, as the cv::Mat expressions of :1326-1333.
inline float f2f_tlc_z(const float* Tcw_cur, const float* Tcw_last) {
  float twc[3];
  for (int k = 0; k < 3; ++k)
    twc[k] = -(Tcw_cur[0 * 4 + k] * Tcw_cur[3] + Tcw_cur[1 * 4 + k] * Tcw_cur[7] +
               Tcw_cur[2 * 4 + k] * Tcw_cur[11]);
  return Tcw_last[8] * twc[0] + Tcw_last[9] * twc[1] + Tcw_last[10] * twc[2] + Tcw_last[11];
}

// The queries of :1337-1341 (a last-frame keypoint with a map point, not an outlier) in
// last-frame keypoint order, and the pose record. A query's `blocks` is NumObservations() > 0
// (the claim it makes on a current-frame keypoint blocks later queries, :1389-1393).
inline F2FInput gather_search_by_projection_frame(const FrameView& current, const FrameView& last,
                                                  const MapPointView* mps, float baseline,
                                                  float th, bool mono, bool check_ori) {
  F2FInput in;
  for (int i = 0; i < last.n_kps; ++i) {
    const int m = last.map_points[i];
    if (m < 0 || last.outlier[i]) continue;
    slamgpu_f2f_query q{};
    std::memcpy(q.xyz, mps[m].xyz, sizeof q.xyz);
    q.last_angle = last.undist_kps[i].angle;
    q.last_octave = last.kps[i].octave;
    q.mp_id = (int32_t)in.queries.size();
    q.blocks = mps[m].n_obs > 0;
    std::memcpy(q.desc, mps[m].desc, 32);
    in.queries.push_back(q);
    in.query_map_point.push_back(m);
  }
  slamgpu_f2f_pose& p = in.pose;
  std::memset(&p, 0, sizeof p);
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) p.Rcw[3 * r + c] = current.Tcw[4 * r + c];
    p.tcw[r] = current.Tcw[4 * r + 3];
  }
  p.tlc_z = f2f_tlc_z(current.Tcw, last.Tcw);
  p.baseline = baseline;
  p.th = th;
  p.mono = mono ? 1 : 0;
  p.check_ori = check_ori ? 1 : 0;
  return in;
}

// The current frame's claim state before either SearchByProjection: slot[i] = -1 (no query has
// claimed keypoint i yet); blocked[i] = its map point has observations -- both overloads skip
// such keypoints (:1389-1393, :59-63), including the ones claimed earlier in the same call.
inline void current_claim_state(const FrameView& current, const MapPointView* mps,
                                int32_t* slot, uint8_t* blocked) {
  for (int i = 0; i < current.n_kps; ++i) {
    const int m = current.map_points[i];
    slot[i] = -1;
    blocked[i] = m >= 0 && mps[m].n_obs > 0;
  }
}
inline void f2f_current_state(const FrameView& current, const MapPointView* mps,
                              int32_t* slot, uint8_t* blocked) {
  current_claim_state(current, mps, slot, blocked);
}

// After a call: the current frame's map point per keypoint -- the queried map point a slot was
// given (F.SetMapPoint(bestIdx, pMP): :1414-1415, :99-100), the previous one elsewhere.
// Returns the number of slots the search assigned.
inline int apply_claims(const std::vector<int32_t>& query_map_point, const int32_t* slot,
                        int32_t* current_map_points, int n) {
  int assigned = 0;
  for (int i = 0; i < n; ++i)
    if (slot[i] >= 0) {
      current_map_points[i] = query_map_point[slot[i]];
      ++assigned;
    }
  return assigned;
}
inline int apply_search_by_projection_frame(const F2FInput& in, const int32_t* slot,
                                            int32_t* current_map_points, int n) {
  return apply_claims(in.query_map_point, slot, current_map_points, n);
}

// The whole call on frame `frame` of the context's last frame / frontend call: gather, claim
// state, slamgpu_search_by_projection_frame, write-back into current_map_points (the frame's
// map point indices, in/out). Returns the reference's nmatches; throws on a device error.
inline int search_by_projection_frame(slamgpu_ctx* ctx, int frame, const FrameView& current,
                                      const FrameView& last, const MapPointView* mps,
                                      float baseline, float th, bool mono, bool check_ori,
                                      int32_t* current_map_points) {
  const F2FInput in = gather_search_by_projection_frame(current, last, mps, baseline, th, mono,
                                                        check_ori);
  std::vector<int32_t> slot(current.n_kps);
  std::vector<uint8_t> blocked(current.n_kps);
  current_claim_state(current, mps, slot.data(), blocked.data());
  int nm = 0;
  const int rc = slamgpu_search_by_projection_frame(ctx, frame, in.queries.data(),
                                                    (int)in.queries.size(), &in.pose, slot.data(),
                                                    blocked.data(), current.n_kps, &nm);
  if (rc != SLAMGPU_OK) throw std::runtime_error(std::string("slamgpu: ") + slamgpu_last_error(ctx));
  apply_search_by_projection_frame(in, slot.data(), current_map_points, current.n_kps);
  return nm;
}

// ---- OrbMatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (orb_matcher.cpp:13) --

// A map point's tracking fields, MapPoint::track_* as Frame::IsInFrustum (frame.cpp:277-337)
// left them when Tracker::SearchLocalPoints (tracker.cpp:1176-1227) ran it on the current frame.
struct TrackView {
  bool in_view;             // track_is_in_view
  float proj_x, proj_y;     // track_projected_x / _y
  float proj_xr;            // track_projected_x_right
  float view_cos;           // track_view_cos
  int32_t level;            // track_scale_level
};

struct MpsInput {
  std::vector<slamgpu_mps_query> queries;  // one per in-view, not-bad point of vpMapPoints
  std::vector<int32_t> query_map_point;    // map point index of each query (mp_id = position)
};

// The queries of :18-26 in vpMapPoints order (a point that is not in view or is bad does nothing
// in the reference's loop, so it is left out), with the fields the loop reads: the track_*
// values, NumObservations() > 0 (the claim it makes blocks later points, :59-63) and
// GetDescriptor(). `track` is indexed like `mps` (the fields live on the MapPoint).
inline MpsInput gather_search_by_projection_mps(const int32_t* map_points, int n,
                                                const MapPointView* mps, const TrackView* track) {
  MpsInput in;
  for (int i = 0; i < n; ++i) {
    const int m = map_points[i];
    const TrackView& t = track[m];
    if (!t.in_view || mps[m].bad) continue;
    slamgpu_mps_query q{};
    q.proj_x = t.proj_x;
    q.proj_y = t.proj_y;
    q.proj_xr = t.proj_xr;
    q.view_cos = t.view_cos;
    q.level = t.level;
    q.in_view = 1;
    q.is_bad = 0;
    q.mp_id = (int32_t)in.queries.size();
    q.blocks = mps[m].n_obs > 0;
    std::memcpy(q.desc, mps[m].desc, 32);
    in.queries.push_back(q);
    in.query_map_point.push_back(m);
  }
  return in;
}

inline int apply_search_by_projection_mps(const MpsInput& in, const int32_t* slot,
                                          int32_t* current_map_points, int n) {
  return apply_claims(in.query_map_point, slot, current_map_points, n);
}

// The whole call (SearchLocalPoints' matcher.SearchByProjection(current_frame_,
// local_map_points_, th) with OrbMatcher(nnratio)): gather, claim state,
// slamgpu_search_by_projection_mps, write-back. Returns nmatches; throws on a device error.
inline int search_by_projection_mps(slamgpu_ctx* ctx, int frame, const FrameView& current,
                                    const MapPointView* mps, const int32_t* map_points, int n,
                                    const TrackView* track, float nnratio, int th,
                                    int32_t* current_map_points) {
  const MpsInput in = gather_search_by_projection_mps(map_points, n, mps, track);
  std::vector<int32_t> slot(current.n_kps);
  std::vector<uint8_t> blocked(current.n_kps);
  current_claim_state(current, mps, slot.data(), blocked.data());
  int nm = 0;
  const int rc = slamgpu_search_by_projection_mps(ctx, frame, in.queries.data(),
                                                  (int)in.queries.size(), nnratio, th,
                                                  slot.data(), blocked.data(), current.n_kps, &nm);
  if (rc != SLAMGPU_OK) throw std::runtime_error(std::string("slamgpu: ") + slamgpu_last_error(ctx));
  apply_search_by_projection_mps(in, slot.data(), current_map_points, current.n_kps);
  return nm;
}

// ---- the stereo Frame ctor (frame.cpp:61-111) ----------------------------------------------------

// What the stereo ctor leaves in the Frame: both views' keypoints and descriptors (ExtractORB
// :86-89), the undistorted left keypoints (:96), StereoCoordRight / StereoDepth
// (ComputeStereoMatches :97), map points all null and no outliers (:99-100).
struct StereoFrame {
  int N = 0;                                     // num_keypoints_ (left view)
  std::vector<slamgpu_keypoint> keys, keys_right, undist_keys;
  std::vector<uint8_t> desc, desc_right;         // N x 32, N_right x 32
  std::vector<float> right_coords, depth;        // N each, -1 = no stereo match
  std::vector<int32_t> map_points;               // N x -1
  std::vector<uint8_t> outlier;                  // N x 0
};

// One device context per tracker holding the current frame (frame 0): Make() runs
// slamgpu_frame_stereo (extraction of both views + ComputeStereoMatches + undistortion + the
// grid) and downloads what the Frame keeps; the matchers above then run on the same context
// (frame 0) against the frame's device-resident grid. The context is created on the first call
// and again when the image size changes; the distortion is set once per context.
class StereoFrameCore {
 public:
  StereoFrameCore(const slamgpu_orb_params& params, const slamgpu_camera& cam,
                  const float* dist_coef = nullptr, int n_dist = 0, int device = 0)
      : params_(params), cam_(cam), dist_(dist_coef, dist_coef + (dist_coef ? n_dist : 0)),
        device_(device) {}
  ~StereoFrameCore() { slamgpu_destroy(ctx_); }
  StereoFrameCore(const StereoFrameCore&) = delete;
  StereoFrameCore& operator=(const StereoFrameCore&) = delete;

  // frame.cpp:61-111 on two 8-bit images of the same size and row step. An empty left view
  // leaves N = 0 and the rest empty (:91-94).
  void Make(const uint8_t* left, const uint8_t* right, int rows, int cols, size_t step,
            StereoFrame& f) {
    f = StereoFrame();
    if (!left || !right || rows <= 0 || cols <= 0) return;
    ensure(cols, rows);
    check(slamgpu_frame_stereo(ctx_, left, right, step, &cam_));
    const int cap = slamgpu_kp_capacity(ctx_);
    int n = 0, nr = 0, ns = 0, nu = 0;
    f.keys.resize(cap);
    f.desc.resize((size_t)cap * 32);
    check(slamgpu_download_keypoints(ctx_, 0, f.keys.data(), f.desc.data(), cap, &n));
    f.keys_right.resize(cap);
    f.desc_right.resize((size_t)cap * 32);
    check(slamgpu_download_keypoints(ctx_, 1, f.keys_right.data(), f.desc_right.data(), cap, &nr));
    f.keys.resize(n);
    f.desc.resize((size_t)n * 32);
    f.keys_right.resize(nr);
    f.desc_right.resize((size_t)nr * 32);
    f.N = n;
    if (n == 0) return;
    f.right_coords.resize(n);
    f.depth.resize(n);
    check(slamgpu_download_stereo(ctx_, 0, f.right_coords.data(), f.depth.data(), n, &ns));
    f.undist_keys.resize(n);
    check(slamgpu_download_undistorted_keypoints(ctx_, 0, f.undist_keys.data(), n, &nu));
    if (ns != n || nu != n) throw std::logic_error("slamgpu: inconsistent frame downloads");
    f.map_points.assign(n, -1);
    f.outlier.assign(n, 0);
  }

  // A FrameView of `f` (pose Tcw: 4x4 row-major, caller-owned) for the matchers and
  // PoseOptimization above.
  static FrameView view(const StereoFrame& f, const float* Tcw) {
    FrameView v;
    v.Tcw = Tcw;
    v.kps = f.keys.data();
    v.undist_kps = f.undist_keys.data();
    v.right_coords = f.right_coords.data();
    v.map_points = f.map_points.data();
    v.outlier = f.outlier.data();
    v.n_kps = f.N;
    return v;
  }

  slamgpu_ctx* context() { return ctx_; }

 private:
  void ensure(int cols, int rows) {
    if (ctx_ && cols == cols_ && rows == rows_) return;
    slamgpu_destroy(ctx_);
    ctx_ = nullptr;
    check(slamgpu_create(device_, &params_, cols, rows, 1, &ctx_));
    if (!dist_.empty()) check(slamgpu_set_distortion(ctx_, dist_.data(), (int)dist_.size()));
    cols_ = cols;
    rows_ = rows;
  }
  void check(int rc) const {
    if (rc != SLAMGPU_OK) throw std::runtime_error(std::string("slamgpu: ") +
                                                   slamgpu_last_error(ctx_));
  }

  slamgpu_orb_params params_;
  slamgpu_camera cam_;
  std::vector<float> dist_;
  int device_;
  slamgpu_ctx* ctx_ = nullptr;
  int cols_ = 0, rows_ = 0;
};

}  // namespace slamgpu_adapter
