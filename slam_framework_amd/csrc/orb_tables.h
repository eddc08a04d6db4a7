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
int compute_geometry(const OrbParams& p, int cols, int rows, OrbGeom* g,
                     std::vector<ResizeX>* rx, std::vector<ResizeY>* ry);
// FAST cell views of all levels, in the kernels' per-image cell order (cells_per_image entries).
void build_cells(const OrbGeom& g, std::vector<CellDesc>* cells);
// pyr_band_kernel's column table: one 16-byte entry per 4-column group of every level >= 1
// (word k: a0 | a1 << 12 | (sx_k - sx_0) << 24 | xmax flag << 27 | nibble k of sx_0 << 28);
// sets g->lv[l].pc_base.
void build_pyr_columns(OrbGeom* g, const std::vector<ResizeX>& rx, std::vector<uint32_t>* pc);
// nb row bands of every level (nb * kMaxLevels entries, band-major); max_rows[l] = the longest
// need range of level l over the bands (the work-group's LDS is sized from it).
void build_pyr_bands(const OrbGeom& g, const std::vector<ResizeY>& ry, int nb,
                     std::vector<PyrBand>* bands, int max_rows[kMaxLevels]);

}  // namespace slamgpu
