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
#include "slamgpu_bow.h"
#include "slamgpu_kfmatch.h"
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


// =================================================================================================
// The keyframe-rate surfaces: SearchByBoW, SearchForTriangulation, Fuse,
// OptimizeSim3 and the global BundleAdjustment, gathered from the same views, called, written back.

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned>>) as arrays: node ids ascending,
// each node's feature indices in insertion order.
struct FeatureVecView {
  const uint32_t* nodes = nullptr;
  const int32_t* node_start = nullptr;  // [n_nodes + 1]
  const uint32_t* node_feats = nullptr;
  int n_nodes = 0;
};

// What the keyframe-rate matchers read of a KeyFrame beyond KeyFrameView: its descriptors
// (KeyFrame::descriptors), feature_vec, and GetCameraCenter() (the stored Ow).
struct KeyFrameFeatures {
  const uint8_t* desc = nullptr;
  FeatureVecView fv;
  const float* Ow = nullptr;
};

inline void throw_if(int rc, const char* (*msg)(void)) {
  if (rc != SLAMGPU_OK) throw std::runtime_error(std::string("slamgpu: ") + msg());
}

inline slamgpu_bow_set bow_set(const uint8_t* desc, const slamgpu_keypoint* kps, const uint8_t* valid,
                               int n, const FeatureVecView& fv) {
  slamgpu_bow_set b;
  b.desc = desc;
  b.kps = kps;
  b.valid = valid;
  b.nodes = fv.nodes;
  b.node_start = fv.node_start;
  b.node_feats = fv.node_feats;
  b.n = n;
  b.n_nodes = fv.n_nodes;
  return b;
}

// A keyframe's features whose map point exists and is not bad (the `if(!pMP) continue; if
// (pMP->isBad()) continue;` of both SearchByBoW overloads).
inline std::vector<uint8_t> good_map_point_mask(const KeyFrameView& kf, const MapPointView* mps) {
  std::vector<uint8_t> v(kf.n_kps);
  for (int i = 0; i < kf.n_kps; ++i) v[i] = kf.map_points[i] >= 0 && !mps[kf.map_points[i]].bad;
  return v;
}

// ---- OrbMatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>&) (orb_matcher.cpp:
// 133-262): Tracker::TrackReferenceKeyFrame (tracker.cpp:666, OrbMatcher(0.7, true)) and the
// relocalisation (:860, 0.75). map_point_matches[j] = the keyframe map point matched to frame
// keypoint j, or -1 (the vpMapPointMatches the caller then gives to Frame::SetMapPoints).
inline int search_by_bow(const KeyFrameView& kf, const KeyFrameFeatures& kff,
                         const MapPointView* mps, const slamgpu_keypoint* f_keys,
                         const uint8_t* f_desc, int f_n, const FeatureVecView& f_fv,
                         float nnratio, bool check_ori, std::vector<int32_t>& map_point_matches) {
  const std::vector<uint8_t> valid = good_map_point_mask(kf, mps);
  const slamgpu_bow_set a = bow_set(kff.desc, kf.undist_kps, valid.data(), kf.n_kps, kff.fv);
  const slamgpu_bow_set b = bow_set(f_desc, f_keys, nullptr, f_n, f_fv);
  std::vector<int32_t> match(kf.n_kps > 0 ? kf.n_kps : 1);
  int nm = 0;
  throw_if(slamgpu_search_by_bow(&a, &b, 0, nnratio, check_ori ? 1 : 0, match.data(), &nm),
           slamgpu_bow_last_error);
  map_point_matches.assign(f_n, -1);
  for (int i = 0; i < kf.n_kps; ++i)
    if (match[i] >= 0) map_point_matches[match[i]] = kf.map_points[i];
  return nm;
}

// ---- OrbMatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
// (orb_matcher.cpp:499-632): LoopCloser::ComputeSim3 (loop_closer.cpp:327, OrbMatcher(0.75,
// true)). matches12[i] = pKF2's map point matched to pKF1 feature i, or -1.
inline int search_by_bow(const KeyFrameView& kf1, const KeyFrameFeatures& f1,
                         const KeyFrameView& kf2, const KeyFrameFeatures& f2,
                         const MapPointView* mps, float nnratio, bool check_ori,
                         std::vector<int32_t>& matches12) {
  const std::vector<uint8_t> v1 = good_map_point_mask(kf1, mps), v2 = good_map_point_mask(kf2, mps);
  const slamgpu_bow_set a = bow_set(f1.desc, kf1.undist_kps, v1.data(), kf1.n_kps, f1.fv);
  const slamgpu_bow_set b = bow_set(f2.desc, kf2.undist_kps, v2.data(), kf2.n_kps, f2.fv);
  std::vector<int32_t> match(kf1.n_kps > 0 ? kf1.n_kps : 1);
  int nm = 0;
  throw_if(slamgpu_search_by_bow(&a, &b, 1, nnratio, check_ori ? 1 : 0, match.data(), &nm),
           slamgpu_bow_last_error);
  matches12.assign(kf1.n_kps, -1);
  for (int i = 0; i < kf1.n_kps; ++i)
    if (match[i] >= 0) matches12[i] = kf2.map_points[match[i]];
  return nm;
}

// The matchers' record of one keyframe (pose split as KeyFrame::GetRotation / GetTranslation
// return it; has_mp[i] = GetMapPoint(i) != NULL, bad or not, as SearchForTriangulation tests it).
struct KfRecord {
  slamgpu_kf kf;
  std::vector<uint8_t> has_mp;
};
inline KfRecord kf_record(const KeyFrameView& v, const KeyFrameFeatures& f) {
  KfRecord r;
  r.has_mp.resize(v.n_kps > 0 ? v.n_kps : 1);
  for (int i = 0; i < v.n_kps; ++i) r.has_mp[i] = v.map_points[i] >= 0;
  slamgpu_kf& k = r.kf;
  std::memset(&k, 0, sizeof(k));
  k.kps = v.undist_kps;
  k.desc = f.desc;
  k.u_right = v.right_coords;
  k.has_mp = r.has_mp.data();
  k.nodes = f.fv.nodes;
  k.node_start = f.fv.node_start;
  k.node_feats = f.fv.node_feats;
  k.n = v.n_kps;
  k.n_nodes = f.fv.n_nodes;
  for (int r0 = 0; r0 < 3; ++r0) {
    for (int c = 0; c < 3; ++c) k.Rcw[3 * r0 + c] = v.Tcw[4 * r0 + c];
    k.tcw[r0] = v.Tcw[4 * r0 + 3];
    k.Ow[r0] = f.Ow[r0];
  }
  return r;
}

// ---- OrbMatcher::SearchForTriangulation (orb_matcher.cpp:634-802) as LocalMapper::
// CreateNewMapPoints calls it (local_mapper.cpp:312, OrbMatcher(0.6, false), only_stereo =
// false): F12 from LocalMapper::ComputeFundamentalMatrix; cam / lv = pKF2's calibration and
// level tables. Returns vMatchedPairs: (pKF1 index, pKF2 index), ascending pKF1 index.
inline std::vector<std::pair<int, int>> search_for_triangulation(
    const KeyFrameView& kf1, const KeyFrameFeatures& f1, const KeyFrameView& kf2,
    const KeyFrameFeatures& f2, const float F12[9], const slamgpu_camera& cam,
    const slamgpu_levels& lv, bool only_stereo, bool check_ori) {
  const KfRecord r1 = kf_record(kf1, f1), r2 = kf_record(kf2, f2);
  std::vector<int32_t> match(kf1.n_kps > 0 ? kf1.n_kps : 1);
  int nm = 0;
  throw_if(slamgpu_search_for_triangulation(&r1.kf, &r2.kf, F12, &cam, &lv, only_stereo ? 1 : 0,
                                            check_ori ? 1 : 0, match.data(), &nm),
           slamgpu_kfmatch_last_error);
  std::vector<std::pair<int, int>> pairs;
  for (int i = 0; i < kf1.n_kps; ++i)
    if (match[i] >= 0) pairs.emplace_back(i, match[i]);
  return pairs;
}

// ---- OrbMatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th)
// (orb_matcher.cpp:804-954), LocalMapper::SearchInNeighbors (local_mapper.cpp:521, 540).
// What Fuse reads of a map point beyond MapPointView: GetNormal(), min_dist_ / max_dist_ and
// NumObservations() (the stereo-weighted count AddObservation keeps, map_point.cpp:114-125).
struct MapPointGeometry {
  float normal[3];
  float min_dist, max_dist;
  int32_t num_observations;
};

// The object-graph changes of one Fuse call, in the reference's order, for the caller to apply
// to its MapPoints / KeyFrame:
//   kReplaceByKf:  point->Replace(other)   (other = the keyframe's map point, more observations)
//   kReplaceKf:    other->Replace(point)
//   kAdd:          point->AddObservation(pKF, keypoint); pKF->AddMapPoint(point, keypoint)
//   kNone:         the keyframe's map point at keypoint is bad: nothing (still counted as fused)
struct FuseAction {
  enum Kind : int32_t { kNone = 0, kReplaceByKf = 1, kReplaceKf = 2, kAdd = 3 };
  int32_t kind, point, other, keypoint;
};
struct FuseResult {
  int nfused = 0;
  std::vector<FuseAction> actions;
};

// The reference checks isBad() and IsInKeyFrame(pKF) of each offered point when the loop reaches
// it, after the Replace / AddObservation calls of earlier points (:821-828). The device search
// of a point does not depend on those calls (it reads the keyframe's keypoints, not its map
// points), so the candidates are searched once with the skip state at the start, and the walk
// below replays the loop on a model of the state those calls change: bad flags, the keyframe's
// slots, each touched point's keyframes and observation count (Replace, map_point.cpp:190-226:
// the survivor takes the other's observations in keyframes it is not in and the other's slot
// there; where both were, the keyframe drops the replaced point's slot).
inline FuseResult fuse(int kf_index, const KeyFrameView* kfs, const KeyFrameFeatures& kff,
                       const MapPointView* mps, const MapPointGeometry* geom, int n_mp,
                       const int32_t* points, int n_points, float th, const slamgpu_camera& cam,
                       const slamgpu_levels& lv, const slamgpu_kf_grid& grid) {
  const KeyFrameView& kf = kfs[kf_index];
  auto in_kf0 = [&](int m) {
    for (int o = 0; o < mps[m].n_obs; ++o)
      if (mps[m].obs[o].keyframe == kf_index) return true;
    return false;
  };
  std::vector<slamgpu_fuse_point> pts(n_points > 0 ? n_points : 1);
  for (int i = 0; i < n_points; ++i) {
    slamgpu_fuse_point& q = pts[i];
    std::memset(&q, 0, sizeof(q));
    const int m = points[i];
    q.skip = m < 0 || mps[m].bad || in_kf0(m);
    if (m < 0) continue;
    std::memcpy(q.xyz, mps[m].xyz, sizeof(q.xyz));
    std::memcpy(q.normal, geom[m].normal, sizeof(q.normal));
    q.min_dist = geom[m].min_dist;
    q.max_dist = geom[m].max_dist;
    std::memcpy(q.desc, mps[m].desc, 32);
  }
  const KfRecord rec = kf_record(kf, kff);
  std::vector<int32_t> best(n_points > 0 ? n_points : 1), dist(n_points > 0 ? n_points : 1);
  int nf = 0;
  throw_if(slamgpu_fuse(&rec.kf, pts.data(), n_points, th, &cam, &lv, &grid, best.data(),
                        dist.data(), &nf),
           slamgpu_kfmatch_last_error);
  // the model: touched points' keyframe -> keypoint maps, counts and bad flags
  std::vector<uint8_t> bad(n_mp);
  std::vector<int32_t> nobs(n_mp);
  std::vector<std::vector<ObsRef>> obs(n_mp);
  std::vector<uint8_t> loaded(n_mp, 0);
  for (int m = 0; m < n_mp; ++m) {
    bad[m] = mps[m].bad;
    nobs[m] = geom[m].num_observations;
  }
  auto load = [&](int m) -> std::vector<ObsRef>& {
    if (!loaded[m]) {
      obs[m].assign(mps[m].obs, mps[m].obs + mps[m].n_obs);
      loaded[m] = 1;
    }
    return obs[m];
  };
  std::vector<int32_t> slot(kf.map_points, kf.map_points + kf.n_kps);  // pKF->GetMapPoint(i)
  auto find = [](const std::vector<ObsRef>& o, int k) {
    for (size_t j = 0; j < o.size(); ++j)
      if (o[j].keyframe == k) return (int)j;
    return -1;
  };
  auto weight = [&](int k, int idx) { return kfs[k].right_coords[idx] >= 0 ? 2 : 1; };
  // this->Replace(point): map_point.cpp:190-226, on the model
  auto replace = [&](int victim, int survivor) {
    if (victim == survivor) return;
    bad[victim] = 1;
    std::vector<ObsRef>& vo = load(victim);
    std::vector<ObsRef>& so = load(survivor);
    for (const ObsRef& r : vo) {
      if (find(so, r.keyframe) < 0) {  // ReplaceMapPointMatch + AddObservation
        if (r.keyframe == kf_index) slot[r.keypoint] = survivor;
        so.push_back(r);
        nobs[survivor] += weight(r.keyframe, r.keypoint);
      } else if (r.keyframe == kf_index) {  // EraseMapPointMatch
        slot[r.keypoint] = -1;
      }
    }
    vo.clear();
  };
  FuseResult res;
  for (int i = 0; i < n_points; ++i) {
    const int m = points[i];
    if (m < 0 || bad[m] || find(load(m), kf_index) >= 0) continue;  // :821-828
    if (best[i] < 0) continue;                                       // bestDist > TH_LOW
    const int j = best[i], cur = slot[j];
    FuseAction a{FuseAction::kNone, m, cur, j};
    if (cur >= 0) {
      if (!bad[cur]) {
        if (nobs[cur] > nobs[m]) {
          a.kind = FuseAction::kReplaceByKf;
          replace(m, cur);
        } else {
          a.kind = FuseAction::kReplaceKf;
          replace(cur, m);
        }
      }
    } else {
      a.kind = FuseAction::kAdd;
      load(m).push_back(ObsRef{kf_index, j});
      nobs[m] += weight(kf_index, j);
      slot[j] = m;
    }
    res.actions.push_back(a);
    res.nfused++;
  }
  return res;
}

// ---- Optimizer::OptimizeSim3 (optimizer.cpp:962-1152), LoopCloser::ComputeSim3
// (loop_closer.cpp:393): the correspondences of :1020-1096 -- match i kept when both map points
// exist, are not bad and pKF2 observes the second (GetIndexInKeyFrame(pKF2) >= 0) -- with the
// points in their keyframes' camera frames as the f32 cv::Mat expression R*X + t forms them
// (one gemm: float dot, then (float)((double)dot + (double)t)).
struct Sim3Problem {
  std::vector<slamgpu_sim3_match> matches;
  std::vector<int32_t> match_index;  // i of each correspondence
};
inline float cv_gemm_row(const float* T, int r, const float* x) {
  const float dot = T[4 * r] * x[0] + T[4 * r + 1] * x[1] + T[4 * r + 2] * x[2];
  return (float)((double)dot + (double)T[4 * r + 3]);
}
inline Sim3Problem gather_optimize_sim3(int kf1_index, int kf2_index, const KeyFrameView* kfs,
                                        const MapPointView* mps, const int32_t* matches1, int n) {
  const KeyFrameView& kf1 = kfs[kf1_index];
  const KeyFrameView& kf2 = kfs[kf2_index];
  Sim3Problem p;
  for (int i = 0; i < n; ++i) {
    const int m2 = matches1[i];
    if (m2 < 0) continue;
    const int m1 = kf1.map_points[i];
    if (m1 < 0) continue;
    int i2 = -1;
    for (int o = 0; o < mps[m2].n_obs; ++o)
      if (mps[m2].obs[o].keyframe == kf2_index) i2 = mps[m2].obs[o].keypoint;
    if (mps[m1].bad || mps[m2].bad || i2 < 0) continue;
    slamgpu_sim3_match c;
    for (int r = 0; r < 3; ++r) {
      c.x1c[r] = cv_gemm_row(kf1.Tcw, r, mps[m1].xyz);
      c.x2c[r] = cv_gemm_row(kf2.Tcw, r, mps[m2].xyz);
    }
    c.u1 = kf1.undist_kps[i].x;
    c.v1 = kf1.undist_kps[i].y;
    c.u2 = kf2.undist_kps[i2].x;
    c.v2 = kf2.undist_kps[i2].y;
    c.octave1 = kf1.undist_kps[i].octave;
    c.octave2 = kf2.undist_kps[i2].octave;
    p.matches.push_back(c);
    p.match_index.push_back(i);
  }
  return p;
}
// The whole call: matches1 (vpMatches1: pKF2's map point per pKF1 feature, -1 none) is updated
// as the reference nulls its outliers (:1103-1106, :1135-1140; also on the early return); S12
// (qx, qy, qz, qw, tx, ty, tz, s) is updated unless the reference returns early. Returns nIn.
inline int optimize_sim3(int kf1_index, int kf2_index, const KeyFrameView* kfs,
                         const MapPointView* mps, int32_t* matches1, int n, const float K1[4],
                         const float K2[4], const float* inv_sigma2_1, const float* inv_sigma2_2,
                         int nlevels, double S12[8], float th2, bool fix_scale) {
  const Sim3Problem p = gather_optimize_sim3(kf1_index, kf2_index, kfs, mps, matches1, n);
  std::vector<uint8_t> inl(p.matches.size() + 1, 1);
  int n_in = 0;
  throw_if(slamgpu_optimize_sim3(K1, K2, inv_sigma2_1, inv_sigma2_2, nlevels, p.matches.data(),
                                 (int)p.matches.size(), th2, fix_scale ? 1 : 0, S12, inl.data(),
                                 &n_in),
           slamgpu_optimizer_last_error);
  for (size_t c = 0; c < p.matches.size(); ++c)
    if (!inl[c]) matches1[p.match_index[c]] = -1;
  return n_in;
}

// ---- Optimizer::BundleAdjustment (optimizer.cpp:33-207), GlobalBundleAdjustemnt (:18-31) ----
// Vertices: every keyframe that is not bad (fixed when Id() == 0), every map point that is not
// bad with its observations in GetObservations() order, skipping bad keyframes. A point left
// with no edge is still a vertex here and stays where it is (the device leaves points without
// observations out of the system, as :149-152 does).
inline LocalBaGraph gather_global_bundle_adjustment(const KeyFrameView* kfs, int n_kf,
                                                    const MapPointView* mps, int n_mp) {
  LocalBaGraph g;
  std::vector<int32_t> vertex_of(n_kf, -1);
  for (int k = 0; k < n_kf; ++k) {
    if (kfs[k].bad) continue;
    vertex_of[k] = (int32_t)g.keyframe.size();
    g.keyframe.push_back(k);
    g.kf_Tcw.insert(g.kf_Tcw.end(), kfs[k].Tcw, kfs[k].Tcw + 16);
    g.kf_mode.push_back(kfs[k].id == 0 ? SLAMGPU_KF_LOCAL_FIXED : SLAMGPU_KF_LOCAL);
  }
  g.n_local = (int)g.keyframe.size();
  g.point_obs_start.push_back(0);
  for (int m = 0; m < n_mp; ++m) {
    if (mps[m].bad) continue;
    g.map_point.push_back(m);
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
// The whole call: gather, solve (optimised keyframe poses and point positions written into the
// graph: the caller stores them as the reference's :170-206 does), LM iterations run.
inline int global_bundle_adjustment(LocalBaGraph& g, const slamgpu_camera& cam,
                                    const float* inv_sigma2, int nlevels, int n_iterations,
                                    bool robust, const volatile bool* stop_flag) {
  int its = 0;
  throw_if(slamgpu_global_bundle_adjustment(&cam, inv_sigma2, nlevels, g.kf_Tcw.data(),
                                            g.kf_mode.data(), (int)g.keyframe.size(),
                                            g.points.data(), (int)g.map_point.size(),
                                            g.point_obs_start.data(), g.obs.data(), n_iterations,
                                            robust ? 1 : 0, stop_flag, &its),
           slamgpu_optimizer_last_error);
  return its;
}

}  // namespace slamgpu_adapter
