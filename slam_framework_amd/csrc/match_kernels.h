// match_kernels.h -- device buffers and launchers of the batched matchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_kernels.h"

namespace slamgpu {

constexpr int kGridCols = 64, kGridRows = 48;  // Frame::grid_cols / grid_rows (frame.h:104-105)
constexpr int kGridCells = kGridCols * kGridRows;
// candidates kept per query for claim resolution: 6 (r5) -- a query whose kept candidates are all
// claimed by earlier queries is rescanned alone on the resolve chain (4: 0.153 ms/step of
// search_resolve, 6: 0.095, 8: 0.062 against search_cand 0.19 / 0.215 / 0.23)
constexpr int kTopK = 6;

struct Camera {
  float fx, fy, cx, cy, bf;
  float min_x, max_x, min_y, max_y;  // Frame image bounds (k1 == 0: 0..cols, 0..rows)
  float cell_w, cell_h;              // grid_element_width_/height_
};

// Keypoints of a set of frames: frame f's arrays start at f * stride (in keypoints).
struct FrameKps {
  const KeyPoint* kps;
  const uint8_t* desc;
  const int* n;        // n[f] (indexed with n_stride)
  int64_t stride;
  int n_stride;        // n[f * n_stride] is frame f's count
};

struct StereoWorkspace {
  int* row_start;      // [frame][rows + 1]
  uint2* row_items;    // [frame][row_cap]: (right keypoint | octave << 16, its x as float bits)
  int row_cap;
  int* sad;            // [frame][kp_cap] SAD score of accepted matches (-1 otherwise)
};

struct StereoOut {
  float* u_right;      // [frame][kp_cap]
  float* depth;        // [frame][kp_cap]
};

// Stereo: frame f uses image 2f (left) and 2f+1 (right) of the extractor batch.
// Stereo frame 0 of ext (images 0 / 1) packed in the host mirror's layout (runtime.cpp
// ResMirror: [nkps x2][err][pad] | kps 2 x kp_cap | desc 2 x kp_cap | u_right kp_cap | depth
// kp_cap) at dst, valid entries only: one DMA then brings the frame's results to the host.
// An empty kernel with a 1 x id grid: a mark in a profiler's kernel trace (slamgpu_trace_marker).
void launch_trace_marker(int id, hipStream_t st);

void launch_frame_pack(const FrameKps& ext, const float* u_right, const float* depth,
                       const uint32_t* err, int kp_cap, uint8_t* dst, hipStream_t st,
                       int parts = 3);
// pack: the single-frame call's packed record (frame 0's u_right / depth go there too), or null
void launch_stereo(const ImageBatch& b, const OrbGeomDev& g, const Camera& cam, int n_frames,
                   const StereoWorkspace& ws, const StereoOut& out, hipStream_t st,
                   uint8_t* pack = nullptr, bool rows_done = false);

// Frame::UndistortKeyPoints of n_sets keypoint sets (set f: src.kps + f * src.stride, count
// src.n[f * src.n_stride]) into dst + f * dst_stride.
struct Distortion;
void launch_undistort(const FrameKps& src, KeyPoint* dst, int64_t dst_stride, const Camera& cam,
                      const Distortion& dc, int n_sets, int kp_cap, hipStream_t st);

// Per-frame keypoint grid (AssignFeaturesToGrid), CSR over the 64x48 cells.
struct GridWorkspace {
  int* cell_start;     // [frame][kGridCells + 1]
  uint4* cell_items;   // [frame][kp_cap]: (keypoint index | octave << 16, x, y as float bits, 0)
  int* cell_fill;      // [frame][kGridCells] scratch
};

// One query of SearchByProjection(Frame&, const Frame&, th, bMono): a last-frame map point.
struct F2FQuery {
  float xyz[3];        // MapPoint::GetWorldPos
  float last_angle;    // LastFrame.GetUndistortedKeys()[i].angle
  int last_octave;     // LastFrame.GetKeys()[i].octave
  int mp_id;           // identity written into the current frame's map point slots
  int blocks;          // MapPoint::NumObservations() > 0
  int pad;
  uint8_t desc[32];    // MapPoint::GetDescriptor
};
static_assert(sizeof(F2FQuery) == 64, "F2FQuery layout");

struct F2FPose {
  float Rcw[9];        // current frame, row major
  float tcw[3];
  float tlc_z;         // (Rlw * twc + tlw).z
  float baseline;      // CurrentFrame.GetBaseline()
  float th;            // search radius factor (7 for stereo, 14 on retry)
  int mono;            // bMono
  int check_ori;       // OrbMatcher::mbCheckOrientation
  int pad;
};

// One query of SearchByProjection(Frame&, vector<MapPoint*>, th): a local map point with its
// IsInFrustum results (track_*).
struct MpsQuery {
  float proj_x, proj_y, proj_xr, view_cos;
  int level;           // track_scale_level
  int in_view;         // track_is_in_view
  int is_bad;
  int mp_id;
  int blocks;          // NumObservations() > 0
  int pad[3];
  uint8_t desc[32];
};
static_assert(sizeof(MpsQuery) == 80, "MpsQuery layout");
static_assert(sizeof(F2FPose) == 72, "F2FPose layout");

struct MatchWorkspace {
  uint64_t* topk;      // [query][kTopK] (dist, grid order) keys
  int* ncand;          // [query]
  int* rot_bin;        // [query] rotation-histogram bin of the accepted match (-1 none)
  int* best_idx;       // [query]
};

struct MatchIO {
  const int* q_start;  // [frame] first query of the frame
  const int* q_count;  // [frame]
  int* map_point;      // [frame][kp_cap] in/out: map point id per keypoint (-1 none)
  uint8_t* blocked;    // [frame][kp_cap] in/out: slot holds a map point with observations
  int* nmatches;       // [frame]
  int64_t mp_stride;   // stride of map_point/blocked between frames (keypoints)
};

void launch_grid(const FrameKps& cur, const Camera& cam, int n_frames, int kp_cap,
                 const GridWorkspace& gw, hipStream_t st);
// One frame (the single-frame call): the stereo row tables, the left view's grid and the packing
// of counts / keypoints / descriptors into `pack`, as three work-groups of one launch; then
// launch_stereo(..., rows_done = true).
void launch_frame_aux(const OrbGeomDev& g, const FrameKps& left, const Camera& cam,
                      const GridWorkspace& gw, const StereoWorkspace& ws, uint8_t* pack,
                      hipStream_t st);

void launch_search_frame(const FrameKps& cur, const float* u_right, int64_t ur_stride,
                         const Camera& cam, const OrbGeomDev& g, const F2FQuery* queries,
                         const F2FPose* poses, int n_frames, int max_queries_per_frame,
                         const GridWorkspace& gw, const MatchWorkspace& mw, const MatchIO& io,
                         hipStream_t st);

void launch_search_mps(const FrameKps& cur, const float* u_right, int64_t ur_stride,
                       const Camera& cam, const OrbGeomDev& g, const MpsQuery* queries,
                       float nnratio, int th, int n_frames, int max_queries_per_frame,
                       const GridWorkspace& gw, const MatchWorkspace& mw, const MatchIO& io,
                       hipStream_t st);

// Queries for frame f from frame f-1's stereo keypoints (frame 0 gets none); queries of frame f
// occupy queries[f * kp_cap ...].
void launch_vo_queries(const FrameKps& src, const float* depth, int64_t depth_stride,
                       const Camera& cam, const F2FPose* poses, int blocks, int kp_cap,
                       F2FQuery* queries, int* q_start, int* q_count, int n_frames,
                       hipStream_t st);

}  // namespace slamgpu
