// orb_kernels.h -- device buffers and launchers of the batched ORB extractor.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_geometry.h"

namespace slamgpu {

// Byte-identical to cv::KeyPoint (28 bytes): pt.x, pt.y, size, angle, response, octave, class_id.
struct KeyPoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
};
static_assert(sizeof(KeyPoint) == 28, "cv::KeyPoint layout");

// A batch of u8 images already in device memory. Image 2f is the left view of frame f at
// in_l + f * in_stride, image 2f+1 the right view at in_r + f * in_stride; rows are in_pitch
// bytes apart. (n mono images at base + i*s: in_l = base, in_r = base + s, in_stride = 2s.)
// pyr is the per-image pyramid (levels >= 1).
struct ImageBatch {
  const uint8_t* in_l;
  const uint8_t* in_r;
  int64_t in_stride;
  int in_pitch;
  uint8_t* pyr;
};

__device__ __forceinline__ const uint8_t* batch_image(const ImageBatch& b, int img) {
  return ((img & 1) ? b.in_r : b.in_l) + (int64_t)(img >> 1) * b.in_stride;
}

struct ExtractWorkspace {
  uint32_t* cell_keys;     // [img][cell][cell_cap] FAST survivors
  int* cell_count;         // [img][cell]
  uint32_t* key_scratch;   // [img][keys_per_image] octree ping-pong key buffers
  OctNode* node_scratch;   // [img][nodes_per_image]
  uint32_t* oct_keys;      // [img][out_per_image] octree output (list order per level)
  int* oct_count;          // [img][nlevels]
  uint32_t* err;           // error bits (kErr*)
};

struct ExtractOutput {
  KeyPoint* kps;           // [img][kp_cap]
  uint8_t* desc;           // [img][kp_cap][32]
  int* nkps;               // [img]
};

struct OrbGeomDev {
  const OrbGeom* host;
  const OrbGeom* dev;
  const ResizeX* rx;
  const ResizeY* ry;
  const CellDesc* cells;   // FAST cell views, cells_per_image entries (build_cells)
  ExtractWorkspace ws;
  ExtractOutput out;
};

// Optional side streams of the extraction (all null: everything on `st`):
//   side0: FAST of level 0 (reads only the caller's images) beside the pyramid, joined before
//          the octree; after the extraction, the left views' undistortion + grid beside the
//          stereo matching (fork1 / join1, runtime.cpp run_frontend).
struct ExtractStreams {
  hipStream_t side0 = nullptr;
  hipEvent_t fork0 = nullptr, join0 = nullptr;
  hipEvent_t fork1 = nullptr, join1 = nullptr;
};
void launch_extract(const ImageBatch& b, const OrbGeomDev& g, int n_images, hipStream_t st,
                    const ExtractStreams& fx = ExtractStreams());

// Dynamic LDS the octree kernels may take on `device`: the device's per-work-group limit less
// each kernel's static LDS (octree_img_kernel, octree_lvl_kernel); compute_geometry sizes their
// key capacities within these.
hipError_t octree_lds_limits(int device, int* img_bytes, int* lvl_bytes);
// The geometry was laid out with the kernels' own build constants (ring strip, FAST key group):
// false when orb_geometry.cpp and orb_kernels.hip were built with different -D flags.
bool extract_build_matches(const OrbGeom& g);

}  // namespace slamgpu
