// orb_geometry.h -- host-computed, device-consumed description of one ORB configuration.
//
// Everything here is a pure function of the ORBextractor ctor arguments and the image size
// (src/orb_features/orb_extractor.cpp:351-411 for the tables, :706-733 for the FAST cell grid,
// :480-488 for the octree's initial split, :1051-1057 for the level sizes). It is computed once
// on the host (orb_geometry.cpp) and passed by value to the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>


namespace slamgpu {

constexpr int kMaxLevels = 12;
// fast_cells writes the FAST survivors of each aligned group of kCellGroup cells (a wave's cells)
// (FAST_CELLS_PER_WAVE: the cells one fast_cells wave runs)
// contiguously from the group's first slot; every level's cell range is padded to a multiple of
// kCellGroup with empty cells, so groups never straddle levels or launches.
#ifndef FAST_CELLS_PER_WAVE
#define FAST_CELLS_PER_WAVE 8
#endif
constexpr int kCellGroup = FAST_CELLS_PER_WAVE;
static_assert(kCellGroup > 0 && (kCellGroup & (kCellGroup - 1)) == 0,
              "kCellGroup masks (i & ~(kCellGroup - 1)) need a power of two");
constexpr int kPyrMaxBands = 32;
constexpr int kCascR0 = 8, kCascDepth = 6, kCascSlots = 4;  // pyr_cascade_kernel (OrbGeom)
constexpr int kEdgeThreshold = 19;
constexpr int kMinBorder = kEdgeThreshold - 3;  // minBorderX/Y (:712)
constexpr int kPatchSize = 31;
constexpr int kHalfPatch = 15;

// One FAST cell's view (ComputeKeyPointsOctTree :735-749), precomputed per configuration so a
// cell costs one 16-byte load instead of a chain of level lookups. vw = vh = 0: empty cell.
struct CellDesc {
  int16_t level, ini_x, ini_y, vw, vh, pad0, pad1, pad2;
};
static_assert(sizeof(CellDesc) == 16, "CellDesc is one dwordx4");

#ifndef PYR_STRIP
#define PYR_STRIP 16  // pyr_down output rows per wave (batches)
#endif
#ifndef PYR_RING_STRIP
#define PYR_RING_STRIP 16  // pyr_ring_kernel output rows per wave (batches)
#endif

struct LevelGeom {
  int w, h;             // level image size
  int pitch;            // row pitch of this level in the pyramid buffers (level >= 1)
  int64_t offset;       // byte offset of this level inside one image's pyramid buffer
  // FAST cell grid (ComputeKeyPointsOctTree :712-733)
  int max_bx, max_by;   // maxBorderX/Y
  int ncols, nrows;     // cells
  int wcell, hcell;
  int cell_base;        // first cell of this level in the per-image cell list
  // DistributeOctTree (:480-488)
  int budget;           // mnFeaturesPerLevel[level]
  int n_ini;
  float hx;
  int node_cap;         // max list length: max(4*n_ini, budget + 3)
  int key_cap;          // max FAST candidates per (image, level) kept in scratch
  int64_t key_base;     // offset (in keys) of this level in the per-image key scratch
  int64_t node_base;    // offset (in nodes) of this level in the per-image node scratch
  int out_base;         // offset (in keypoints) of this level in the per-image octree output
  int out_cap;          // max keypoints this level can emit
  int oct_nc;           // octree_img_kernel: LDS node capacity (node_cap rounded to 64)
  int oct_list_off;     //   byte offset of the two node lists in the work-group's LDS
  int oct_work_off;     //   byte offset of sort keys / prefix arrays / flags
  // resize tables (level >= 1) in the shared table buffer
  int rx_base, ry_base; // offsets into the x (per dst column) / y (per dst row) tables
  int xmax;             // first dst column that copies S[sx] * 2048 (resize HResizeLinear)
  // pyr_ring_kernel (level >= 1): a strip's source rows staged in LDS by 16-byte buffer-to-LDS
  // loads, pyr_rpi rows of pyr_lpr chunks per 1 KiB slot (0: the row segment needs > 1 KiB);
  // pyr_slots slots hold the largest strip's rows; pyr_inv_rpi = ceil(2^16 / pyr_rpi),
  // pyr_inv_lpr = ceil(2^16 / pyr_lpr) (quotients of values < 64 by a multiply)
  int pyr_lpr, pyr_rpi, pyr_inv_rpi, pyr_inv_lpr, pyr_slots;
  double rsx;           // resize scale_x = 1 / (w / w_prev) (level >= 1; pyr_band_kernel
                        // derives the column coefficients from it exactly as the host tables)
  float scale, inv_scale;
  float patch_size;     // (float)(int)(PATCH_SIZE * scale) (:778)
};

struct OrbGeom {
  // the build constants this geometry was laid out with (orb_geometry.cpp's translation unit):
  // the kernels' own must agree (extract_build_matches), or a -D flag passed to one source only
  // would size LDS slots / key groups for another strip or group than the kernels use
  int pyr_ring_strip, cell_group;
  int nlevels, cols, rows;
  int nfeatures, ini_th, min_th;
  int cells_per_image;
  int cell_cap;          // max FAST survivors stored per cell
  // fast_cells LDS layout per wave (sized from the largest cell of this configuration)
  int fast_tile_stride, fast_tile_rows;    // cell view + 3 alignment bytes
  int fast_score_stride, fast_score_rows;  // detect area
  int fast_lds_per_wave;                   // bytes (tile + score + u16 candidate list)
  int64_t pyr_bytes;     // bytes of one image's pyramid (levels >= 1) buffer
  int gauss[7];          // GaussianBlur 7x7 sigma 2 integer kernel (x256)
  int64_t keys_per_image;
  int64_t nodes_per_image;
  int oct_lds_bytes;     // octree_img_kernel dynamic LDS (keys + per-level lists and arrays)
  int oct_kcap;          // keys of all levels of one image that fit in that LDS (0: no room)
  // octree_lvl_kernel (one work-group per level): one layout for every level
  // [keys u32 x oct2_kcap][gather staging u32 x oct2_kcap][cell prefix int x oct2_ccap]
  // [two node lists x oct2_nc][sort keys u32, pt / pe / pu / vnext i16, processed + candidate
  // u8, two scan prefixes (uint2), first-child index i16 x oct2_nc]
  int oct2_lds_bytes, oct2_kcap, oct2_ccap, oct2_nc;
  int oct2_tmp_off, oct2_cpre_off, oct2_list_off, oct2_work_off;
  int out_per_image;     // sum of out_cap
  int kp_cap;            // max keypoints per image after Compute (== out_per_image)
  int umax[16];
  LevelGeom lv[kMaxLevels];
  // pyr_band_kernel (small launches: levels 2 .. nlevels - 1 in one launch): band s computes
  // rows [pyr_band[s][l][0], pyr_band[s][l][1]) of level l -- its share of the level plus every
  // source row its own next level needs (so a band reads only rows it wrote itself)
  int pyr_bands;
  int pyr_ring_slots;  // pyr_ring_kernel: 1 KiB LDS slots per wave (max over levels; 0: unusable)
  int pyr_band_lds;  // bytes of one of its two LDS row buffers (the largest band level)
  int16_t pyr_band[kPyrMaxBands][kMaxLevels][2];
  // pyr_cascade_kernel (batches): one work-group per image streams level 0 top to bottom
  // through every level at once; per barrier step level 1 consumes one level-0 row and level l
  // the rows level l - 1 emitted in the step before. casc_waves compute waves (lane task k of
  // level l: columns 8 (k - casc_task_base[l]) .. + 7) + one loader wave; casc_steps steps;
  // LDS: level-0 rows (kCascR0 slots, loaded kCascDepth rows ahead by buffer-to-LDS loads), the
  // rows of levels 1 .. nlevels - 2 (kCascSlots slots), the packed row table of levels >= 1
  // (uint2 {y1 | (y0 == y1) << 16, b0 | b1 << 16} from lv[1].ry_base on), the per-level produced
  // row counters (int [2][kMaxLevels]). casc_waves == 0: not usable for this geometry.
  int casc_waves, casc_steps, casc_lds;
  int casc_task_base[kMaxLevels + 1];
  int casc_ring_off[kMaxLevels], casc_ring_stride[kMaxLevels];
  int casc_ry_off, casc_p_off;
  // orient_desc per-lane constants (host-built from gauss / umax, read once per wave):
  // od_band[tj][lane]: the v_mfma_i32_16x16x64_i8 B operand of tile column tj -- byte b of lane
  // (n = lane & 15, g = lane >> 4) is gauss[16 g + b - 16 tj - n] inside the 7 taps, else 0;
  // od_ic[lane]: the IC_Angle circle weights of the lane's two patch slots, {wt[0][0..1],
  // wt[1][0..1], one[0][0..1], one[1][0..1]} (see orient_desc_kernel)
  uint32_t od_band[3][64][4];
  uint32_t od_ic[64][8];
};

// Resize tables (HResizeLinear / VResizeLinear coefficients, 11-bit fixed point).
struct ResizeX { int32_t sx; int16_t a0, a1; };
struct ResizeY { int32_t y0, y1; int16_t b0, b1; };

// One FAST survivor / octree key: x_rel (12 b) | y_rel (11 b) << 12 | score (8 b) << 23,
// coordinates relative to (minBorderX, minBorderY).
__host__ __device__ inline uint32_t pack_key(int x, int y, int score) {
  return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 23);
}
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 0xfff); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 12) & 0x7ff); }
__host__ __device__ inline int key_score(uint32_t k) { return (int)(k >> 23); }

// Octree list node: rectangle [x0,x1] x [y0,y1] (UL/UR/BL/BR of ExtractorNode), keys
// [kbeg, kbeg+n) in key buffer `buf`, creation sequence number (the pointer-order proxy).
struct OctNode {
  int16_t x0, x1, y0, y1;
  int32_t kbeg;
  int32_t n;
  int32_t seq;
  int32_t buf;
};

// Error bits raised on the device (slamgpu_last_error reports them).
enum : uint32_t {
  kErrKeyOverflow = 1u << 0,   // more FAST candidates than key_cap for some level
  kErrNodeOverflow = 1u << 1,  // octree list exceeded node_cap
  kErrCellOverflow = 1u << 2,  // FAST survivors exceeded cell_cap
  kErrSortOverflow = 1u << 3,  // octree inner-loop set exceeded the LDS sort capacity
  kErrRowOverflow = 1u << 4,   // stereo row table overflow
  kErrCandOverflow = 1u << 5,  // matcher candidate list overflow
};

}  // namespace slamgpu
