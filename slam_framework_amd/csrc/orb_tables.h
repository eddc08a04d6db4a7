// orb_tables.h -- ORBextractor parameters and ctor-derived tables (host side).
#pragma once
#include <vector>

#include "orb_geometry.h"

namespace slamgpu {

// ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
// (src/orb_features/orb_extractor.h:35-39).
struct OrbParams {
  int nfeatures;
  float scale_factor;
  int nlevels;
  int ini_th_fast;
  int min_th_fast;
};

struct OrbTables {
  int nlevels;
  float scale[kMaxLevels], inv_scale[kMaxLevels];
  float sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
  int features_per_level[kMaxLevels];
  int umax[16];
};

void compute_tables(const OrbParams& p, OrbTables* t);
// Returns 0 on success, <0 if the configuration is outside what the kernels support.
// oct_img_lds / oct_lvl_lds: the dynamic LDS the octree kernels may take on the device
// (octree_lds_limits); the key capacities are sized within min(these, the gfx950 budgets).
int compute_geometry(const OrbParams& p, int cols, int rows, OrbGeom* g,
                     std::vector<ResizeX>* rx, std::vector<ResizeY>* ry,
                     int oct_img_lds = 1 << 30, int oct_lvl_lds = 1 << 30);
// FAST cell views of all levels, in the kernels' per-image cell order (cells_per_image entries).
void build_cells(const OrbGeom& g, std::vector<CellDesc>* cells);

}  // namespace slamgpu
