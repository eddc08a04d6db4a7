// orb_geometry.cpp -- ORBextractor ctor tables and per-level launch geometry (host side).
//
// Mirrors src/orb_features/orb_extractor.cpp:351-411 (scale tables, per-level budget, umax),
// :706-733 (cell grid), :480-488 (octree initial split) and :1051-1057 (level sizes), plus
// OpenCV 3.3.1 resize's coefficient tables (imgproc resize.cpp, INTER_LINEAR, CV_8U).
// Compiled with -ffp-contract=off so float arithmetic matches the reference expression by
// expression.
#include "orb_geometry.h"
#include "orb_tables.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace slamgpu {

static inline int cv_round_h(float v) { return (int)std::lrintf(v); }
static inline int16_t sat_short(float v) {
  int i = (int)std::lrintf(v);
  return (int16_t)std::min(32767, std::max(-32768, i));
}

void compute_tables(const OrbParams& p, OrbTables* t) {
  std::memset(t, 0, sizeof(*t));
  t->nlevels = p.nlevels;
  const double sf = (double)p.scale_factor;  // ORBextractor::scaleFactor is a double
  t->scale[0] = 1.0f;
  t->sigma2[0] = 1.0f;
  for (int i = 1; i < p.nlevels; i++) {
    t->scale[i] = (float)((double)t->scale[i - 1] * sf);
    t->sigma2[i] = t->scale[i] * t->scale[i];
  }
  for (int i = 0; i < p.nlevels; i++) {
    t->inv_scale[i] = 1.0f / t->scale[i];
    t->inv_sigma2[i] = 1.0f / t->sigma2[i];
  }
  const float factor = (float)(1.0f / sf);
  float nDesired = (float)p.nfeatures * (1 - factor) /
                   (1 - (float)std::pow((double)factor, (double)p.nlevels));
  int sum = 0;
  for (int l = 0; l < p.nlevels - 1; l++) {
    t->features_per_level[l] = cv_round_h(nDesired);
    sum += t->features_per_level[l];
    nDesired *= factor;
  }
  t->features_per_level[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
  int v, v0;
  const int vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
  const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
  const double hp2 = kHalfPatch * kHalfPatch;
  for (v = 0; v <= vmax; ++v) t->umax[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
  for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
    while (t->umax[v0] == t->umax[v0 + 1]) ++v0;
    t->umax[v] = v0;
    ++v0;
  }
}

// getGaussianKernel(7, 2, CV_32F) then convertTo(CV_32S, 256) (OpenCV 3.3.1 smooth.cpp /
// filter.cpp createSeparableLinearFilter for 8U): {18, 34, 49, 55, 49, 34, 18}, sum 257.
static void gauss_kernel_int(int k[7]) {
  float cf[7];
  double sum = 0;
  const double sigma = 2.0, scale2X = -0.5 / (sigma * sigma);
  for (int i = 0; i < 7; i++) {
    double x = i - 3.0;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = (int)std::lrint((double)cf[i] * 256.0);
  }
}

static inline int round_up(int v, int a) { return (v + a - 1) / a * a; }

int compute_geometry(const OrbParams& p, int cols, int rows, OrbGeom* g,
                     std::vector<ResizeX>* rx, std::vector<ResizeY>* ry, int oct_img_lds,
                     int oct_lvl_lds) {
  if (p.nlevels < 1 || p.nlevels > kMaxLevels || cols < 64 || rows < 64 || cols > 4095 ||
      rows > 2047 || p.nfeatures < 1)
    return -1;
  OrbTables t;
  compute_tables(p, &t);
  std::memset(g, 0, sizeof(*g));
  g->pyr_ring_strip = PYR_RING_STRIP;
  g->cell_group = kCellGroup;
  g->nlevels = p.nlevels;
  g->cols = cols;
  g->rows = rows;
  g->nfeatures = p.nfeatures;
  g->ini_th = p.ini_th_fast;
  g->min_th = p.min_th_fast;
  std::memcpy(g->umax, t.umax, sizeof(g->umax));
  rx->clear();
  ry->clear();
  int64_t pyr_off = 0;
  int cell_base = 0, max_wcell = 0, max_hcell = 0;
  for (int l = 0; l < p.nlevels; l++) {
    LevelGeom& L = g->lv[l];
    L.scale = t.scale[l];
    L.inv_scale = t.inv_scale[l];
    L.w = cv_round_h((float)cols * t.inv_scale[l]);
    L.h = cv_round_h((float)rows * t.inv_scale[l]);
    if (L.w < 2 * kEdgeThreshold + 8 || L.h < 2 * kEdgeThreshold + 8) return -2;
    L.pitch = round_up(L.w, 64);
    if (l == 0) {
      L.offset = 0;  // level 0 lives in the caller's image buffer
    } else {
      L.offset = pyr_off;
      pyr_off += (int64_t)L.pitch * L.h;
      pyr_off = (pyr_off + 255) & ~(int64_t)255;
    }
    // FAST cell grid (:712-733); float arithmetic as in the reference.
    const float W = 30;
    L.max_bx = L.w - kEdgeThreshold + 3;
    L.max_by = L.h - kEdgeThreshold + 3;
    const float width = (float)(L.max_bx - kMinBorder);
    const float height = (float)(L.max_by - kMinBorder);
    L.ncols = (int)(width / W);
    L.nrows = (int)(height / W);
    L.wcell = (int)std::ceil(width / L.ncols);
    L.hcell = (int)std::ceil(height / L.nrows);
    L.cell_base = cell_base;
    cell_base += round_up(L.ncols * L.nrows, kCellGroup);  // padding cells are empty (vh 0)
    max_wcell = std::max(max_wcell, L.wcell);
    max_hcell = std::max(max_hcell, L.hcell);
    // octree (:484-486)
    L.budget = t.features_per_level[l];
    L.n_ini = (int)std::round((float)(L.max_bx - kMinBorder) / (L.max_by - kMinBorder));
    if (L.n_ini < 1) return -3;
    L.hx = (float)(L.max_bx - kMinBorder) / L.n_ini;
    L.node_cap = std::max(4 * L.n_ini, L.budget + 3);
    L.out_cap = L.node_cap;
    L.patch_size = (float)(int)(kPatchSize * t.scale[l]);
    // resize tables for level l from level l-1 (OpenCV resize.cpp resize/resizeGeneric_)
    if (l > 0) {
      const LevelGeom& S = g->lv[l - 1];
      const double inv_scale_x = (double)L.w / S.w, inv_scale_y = (double)L.h / S.h;
      const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
      L.rsx = scale_x;
      L.rx_base = (int)rx->size();
      L.xmax = L.w;
      for (int dx = 0; dx < L.w; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= S.w) {
          L.xmax = std::min(L.xmax, dx);
          if (sx >= S.w - 1) { fx = 0; sx = S.w - 1; }
        }
        ResizeX e;
        e.sx = sx;
        e.a0 = sat_short((1.f - fx) * 2048);
        e.a1 = sat_short(fx * 2048);
        rx->push_back(e);
      }
      L.ry_base = (int)ry->size();
      for (int dy = 0; dy < L.h; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        ResizeY e;
        e.y0 = std::min(std::max(sy, 0), S.h - 1);
        e.y1 = std::min(std::max(sy + 1, 0), S.h - 1);
        e.b0 = sat_short((1.f - fy) * 2048);
        e.b1 = sat_short(fy * 2048);
        ry->push_back(e);
      }
    }
  }
  g->cells_per_image = cell_base;
  // pyr_ring_kernel's row segments: lane k of a 256-column tile reads source dwords q0 .. q0 + 2
  // of columns 4k .. 4k + 3 (unclamped: bytes past the row's end have zero weight); the segment
  // starts at the tile's first dword rounded down to 16 bytes
  int ring_slots = 0;
  bool ring_ok = true;
  for (int l = 1; l < p.nlevels; l++) {
    LevelGeom& L = g->lv[l];
    const LevelGeom& S = g->lv[l - 1];
    const int qmax = (S.w - 1) >> 2;
    auto q0 = [&](int x) { return std::min((*rx)[L.rx_base + std::min(x, L.w - 1)].sx >> 2, qmax); };
    int span = 0;
    for (int x0 = 0; x0 < L.w; x0 += 256) {
      const int lo = (4 * q0(x0)) & ~15;
      int hi = 0;
      for (int k = 0; k < 64; k++) hi = std::max(hi, 4 * (q0(x0 + 4 * k) + 2) + 4);
      span = std::max(span, hi - lo);
    }
    int nsrc = 0;
    for (int dy0 = 0; dy0 < L.h; dy0 += PYR_RING_STRIP) {
      const int dy1 = std::min(dy0 + PYR_RING_STRIP, L.h) - 1;
      nsrc = std::max(nsrc, (*ry)[L.ry_base + dy1].y1 - (*ry)[L.ry_base + dy0].y0 + 1);
    }
    L.pyr_lpr = (span + 15) / 16;
    L.pyr_rpi = L.pyr_lpr <= 64 ? 64 / L.pyr_lpr : 0;
    L.pyr_inv_rpi = L.pyr_rpi ? (65536 + L.pyr_rpi - 1) / L.pyr_rpi : 0;
    L.pyr_inv_lpr = (65536 + L.pyr_lpr - 1) / L.pyr_lpr;
    L.pyr_slots = L.pyr_rpi ? (nsrc + L.pyr_rpi - 1) / L.pyr_rpi : 0;
    ring_ok = ring_ok && L.pyr_rpi > 0;
    ring_slots = std::max(ring_slots, L.pyr_slots);
  }
  g->pyr_ring_slots = ring_ok ? ring_slots : 0;
  {  // pyr_band_kernel's row bands, top-down from the last level
    const int nb = p.nlevels > 2 ? std::min(std::max(g->lv[2].h / 12, 1), kPyrMaxBands) : 0;
    g->pyr_bands = nb;
    std::memset(g->pyr_band, 0, sizeof(g->pyr_band));
    for (int s = 0; s < nb; s++) {
      for (int l = p.nlevels - 1; l >= 2; l--) {
        const int h = g->lv[l].h;
        int lo = (int)((int64_t)s * h / nb), hi = (int)((int64_t)(s + 1) * h / nb);
        if (l + 1 < p.nlevels) {
          const int a = g->pyr_band[s][l + 1][0], b = g->pyr_band[s][l + 1][1];
          if (b > a) {
            const LevelGeom& N = g->lv[l + 1];
            lo = std::min(lo, (*ry)[N.ry_base + a].y0);
            hi = std::max(hi, (*ry)[N.ry_base + b - 1].y1 + 1);
          }
        }
        g->pyr_band[s][l][0] = (int16_t)lo;
        g->pyr_band[s][l][1] = (int16_t)hi;
      }
    }
    int lds = 0;
    for (int s = 0; s < nb; s++)
      for (int l = 2; l < p.nlevels; l++)
        lds = std::max(lds, (g->pyr_band[s][l][1] - g->pyr_band[s][l][0]) * g->lv[l].pitch);
    g->pyr_band_lds = (lds + 15) & ~15;
    if (2 * g->pyr_band_lds > 64 * 1024) g->pyr_bands = 0;  // per-level launches instead
  }
  {  // pyr_cascade_kernel: lane tasks, LDS layout and the step count (simulated here)
    g->casc_waves = 0;
    int tasks = 0;
    for (int l = 1; l <= p.nlevels; l++) {
      g->casc_task_base[l] = tasks;
      if (l < p.nlevels) tasks += (g->lv[l].w + 7) / 8;
    }
    const int waves = (tasks + 63) / 64;
    int off = 0;
    for (int l = 0; l + 1 < p.nlevels; l++) {  // rows read by level l + 1: 16-byte chunks + over-read
      g->casc_ring_stride[l] = ((g->lv[l].w + 15) & ~15) + 16;
      g->casc_ring_off[l] = off;
      off += (l == 0 ? kCascR0 : kCascSlots) * g->casc_ring_stride[l];
    }
    g->casc_ry_off = off;
    if (p.nlevels > 1)
      off += 8 * (g->lv[p.nlevels - 1].ry_base + g->lv[p.nlevels - 1].h - g->lv[1].ry_base);
    g->casc_p_off = off;
    off += 2 * kMaxLevels * 4;
    g->casc_lds = off;
    // the schedule: level l's next source row ns[l] / next output row nd[l]; level l consumes at
    // step t every row level l - 1 had emitted by step t - 1 (level 1: level-0 rows 0 .. t)
    bool ok = p.nlevels > 1 && waves + 1 <= 16 && off <= 64 * 1024 &&
              ((g->lv[0].w + 15) >> 4) <= 128;
    int ns[kMaxLevels] = {0}, nd[kMaxLevels] = {0}, prev[kMaxLevels] = {0};
    int t = 0;
    for (; ok; t++) {
      bool done = true;
      for (int l = 1; l < p.nlevels; l++) {
        const LevelGeom& L = g->lv[l];
        const int avail = l == 1 ? std::min(t + 1, g->lv[0].h) : prev[l - 1];
        const int before = nd[l];
        for (; ns[l] < avail; ns[l]++)
          while (nd[l] < L.h && (*ry)[L.ry_base + nd[l]].y1 == ns[l]) nd[l]++;
        // two rows per step at most: a level's consumer reads the rows of the step before while
        // it writes the next two (kCascSlots = 4)
        if (nd[l] - before > 2) ok = false;
        done = done && nd[l] == L.h;
      }
      for (int l = 1; l < p.nlevels; l++) prev[l] = nd[l];
      if (done || t > 4 * g->lv[0].h) break;
    }
    if (ok && t <= 4 * g->lv[0].h) {
      g->casc_waves = waves;
      g->casc_steps = t + 1;
    }
  }
  gauss_kernel_int(g->gauss);
  {  // orient_desc packs taps into bytes and row sums into u16 (sum of taps <= 257)
    int sum = 0;
    for (int i = 0; i < 7; i++) {
      if (g->gauss[i] < 0 || g->gauss[i] > 255 || g->gauss[i] != g->gauss[6 - i]) return -6;
      sum += g->gauss[i];
    }
    if (sum > 257) return -6;
    // the MFMA band is signed int8
    for (int i = 0; i < 7; i++)
      if (g->gauss[i] > 127) return -6;
  }
  for (int lane = 0; lane < 64; lane++) {  // orient_desc's per-lane constants (orb_geometry.h)
    const int n = lane & 15, gq = lane >> 4;
    for (int tj = 0; tj < 3; tj++)
      for (int w = 0; w < 4; w++) {
        uint32_t v = 0;
        for (int bb = 0; bb < 4; bb++) {
          const int t = 16 * gq + 4 * w + bb - 16 * tj - n;
          if (t >= 0 && t <= 6) v |= (uint32_t)g->gauss[t] << (8 * bb);
        }
        g->od_band[tj][lane][w] = v;
      }
    const int ick = lane & 3;
    for (int q = 0; q < 2; q++) {
      const int r = 16 * q + (lane >> 2), vv = r - 15;
      const int hd = r < 31 ? g->umax[vv < 0 ? -vv : vv] : -1;
      for (int jj = 0; jj < 2; jj++) {
        uint32_t wt = 0, one = 0;
        for (int bb = 0; bb < 4; bb++) {
          const int u = 8 * ick + 4 * jj + bb - 15;
          if (u >= -hd && u <= hd) {
            wt |= (uint32_t)(u + 20) << (8 * bb);
            one |= 1u << (8 * bb);
          }
        }
        g->od_ic[lane][2 * q + jj] = wt;
        g->od_ic[lane][4 + 2 * q + jj] = one;
      }
    }
  }
  // strict 8-neighbour NMS keeps at most one pixel per 2x2 block of the detect area
  g->cell_cap = ((max_wcell + 1) / 2) * ((max_hcell + 1) / 2);
  // tile: dwords covering the cell view from iniX & ~3, plus one spare dword per row for the
  // prefilter's right-neighbour reads
  // fast_cells_kernel is compiled for row strides 64 and 128 (tile and score map share it; the
  // score map is indexed by tile column). A row holds the cell view from iniX & ~3 plus the
  // prefilter's spare right-neighbour dword.
  // A tile row starts at iniX & ~15 (16-byte global_load_lds chunks; up to 15 lead bytes).
  // One tile buffer per wave holding exactly the view's rows (the last glds block lane-masked):
  // LDS, not VGPRs, bounds the kernel's occupancy (double-buffered tiles of whole 1 KiB blocks,
  // 10.3 KB per wave, were slower than 6.6 KB single: 0.966 -> 0.84 ms per step, round 2).
  g->fast_tile_stride = max_wcell + 6 + 15 + 4 <= 64 ? 64 : 128;
  g->fast_tile_rows = max_hcell + 6;
  g->fast_score_stride = g->fast_tile_stride;
  g->fast_score_rows = max_hcell + 2;  // detect rows + a zero row above and below
  g->fast_lds_per_wave = round_up(g->fast_tile_stride * g->fast_tile_rows, 16) +
                         round_up(g->fast_score_stride * g->fast_score_rows, 16) +
                         round_up(2 * max_wcell * max_hcell, 16);  // u16 candidate list
  if (max_wcell > 64) return -4;
  // pyr_down reads the source bytes of 4 adjacent output columns as one 8-byte window
  // starting at sx(x0): sx(x0 + 3) + 1 - sx(x0) <= 7 (any scale factor up to ~2).
  for (int l = 1; l < p.nlevels; l++) {
    const LevelGeom& L = g->lv[l];
    for (int x0 = 0; x0 < L.w; x0 += 4) {
      const int x3 = std::min(x0 + 3, L.w - 1);
      if ((*rx)[L.rx_base + x3].sx - (*rx)[L.rx_base + x0].sx > 6) return -5;
    }
  }
  g->pyr_bytes = pyr_off;
  int64_t key_off = 0, node_off = 0;
  int out_off = 0;
  for (int l = 0; l < p.nlevels; l++) {
    LevelGeom& L = g->lv[l];
    const int64_t ncell = (int64_t)L.ncols * L.nrows;
    L.key_cap = (int)std::min<int64_t>(ncell * g->cell_cap, 65536);
    L.key_base = key_off;
    key_off += 2 * (int64_t)L.key_cap;           // ping-pong
    L.node_base = node_off;
    node_off += 3 * (int64_t)L.node_cap * 4 + 64;  // two lists + speculative children
    L.out_base = out_off;
    out_off += L.out_cap;
  }
  g->keys_per_image = key_off;
  g->nodes_per_image = node_off;
  {  // octree_img_kernel LDS: [keys u32 x kcap][per level: 2 node lists][per level: arrays]
    // gfx950: 156 KB of the 160 KB; a device with less LDS per work-group gets its own limit
    const int kLdsBudget = std::min(156 * 1024, oct_img_lds);
    constexpr int kNodeBytes = 12, kWorkBytesPerNode = 4 + 4 * 2 + 1;
    int off = 0;
    for (int l = 0; l < p.nlevels; l++) {
      LevelGeom& L = g->lv[l];
      L.oct_nc = round_up(L.node_cap, 64);
      L.oct_list_off = off;
      off += 2 * L.oct_nc * kNodeBytes;
    }
    for (int l = 0; l < p.nlevels; l++) {
      LevelGeom& L = g->lv[l];
      L.oct_work_off = off;
      off += round_up(L.oct_nc * kWorkBytesPerNode, 16);
    }
    // every level's node lists live in LDS at once: a large nfeatures (the monocular
    // initialiser's 2 * nFeatures extractor, tracker.cpp:84-89) leaves no room for keys, and
    // such a geometry runs every batch through octree_lvl_kernel (oct_kcap 0)
    const int kcap = std::min((kLdsBudget - off) / 4, 65535);
    g->oct_kcap = kcap >= 1024 ? kcap : 0;
    for (int l = 0; l < p.nlevels; l++) {  // keys go first
      g->lv[l].oct_list_off += 4 * g->oct_kcap;
      g->lv[l].oct_work_off += 4 * g->oct_kcap;
    }
    g->oct_lds_bytes = g->oct_kcap ? off + 4 * g->oct_kcap : 0;
  }
  {  // octree_lvl_kernel LDS (one work-group per CU: the small launches have <= 128 of them)
    // per node: sort key, pt / pe / pu / vnext, processed + candidate flags, the two scan
    // prefixes, the first child's push index (+16 B alignment)
    const int kLdsBudget = std::min(144 * 1024, oct_lvl_lds);
    constexpr int kNodeBytes = 12, kWorkBytesPerNode = 4 + 4 * 2 + 2 + 16 + 2;
    int nc = 64, ccap = 0;
    for (int l = 0; l < p.nlevels; l++) {
      nc = std::max(nc, g->lv[l].oct_nc);
      ccap = std::max(ccap, g->lv[l].ncols * g->lv[l].nrows + 1);
    }
    ccap = round_up(ccap, 4);
    const int fixed = ccap * 4 + 2 * nc * kNodeBytes + round_up(nc * kWorkBytesPerNode + 16, 16);
    const int kcap = std::min((kLdsBudget - fixed) / 8 / 4 * 4, 8192);
    if (kcap < 1024) return -7;
    g->oct2_kcap = kcap;
    g->oct2_ccap = ccap;
    g->oct2_nc = nc;
    g->oct2_tmp_off = 4 * kcap;
    g->oct2_cpre_off = 8 * kcap;
    g->oct2_list_off = g->oct2_cpre_off + 4 * ccap;
    g->oct2_work_off = g->oct2_list_off + 2 * nc * kNodeBytes;
    g->oct2_lds_bytes = g->oct2_work_off + round_up(nc * kWorkBytesPerNode + 16, 16);
  }
  g->out_per_image = out_off;
  g->kp_cap = out_off;
  return 0;
}

void build_cells(const OrbGeom& g, std::vector<CellDesc>* cells) {
  cells->assign(g.cells_per_image, CellDesc{});
  for (int l = 0; l < g.nlevels; l++) {
    const LevelGeom& L = g.lv[l];
    for (int c = 0; c < L.ncols * L.nrows; c++) {
      CellDesc& d = (*cells)[L.cell_base + c];
      const int ci = c / L.ncols, cj = c % L.ncols;
      const int iniY = kMinBorder + ci * L.hcell, iniX = kMinBorder + cj * L.wcell;
      d.level = (int16_t)l;
      d.ini_x = (int16_t)iniX;
      d.ini_y = (int16_t)iniY;
      if (iniY >= L.max_by - 3 || iniX >= L.max_bx - 6) continue;  // :737, :745
      const int maxY = std::min(iniY + L.hcell + 6, L.max_by);
      const int maxX = std::min(iniX + L.wcell + 6, L.max_bx);
      d.vh = (int16_t)(maxY - iniY);
      d.vw = (int16_t)(maxX - iniX);
    }
  }
}

}  // namespace slamgpu
