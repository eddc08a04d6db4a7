/*
 * oracle/matcher_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Restatement of the matching half of the hot path:
 *   Frame::ComputeStereoMatches      src/data/frame.cpp:406-577
 *   Frame::AssignFeaturesToGrid etc. src/data/frame.cpp:211-248, 339-403, 678-703
 *   OrbMatcher::DescriptorDistance   src/orb_features/orb_matcher.cpp:1630-1646
 *   OrbMatcher::SearchByProjection   src/orb_features/orb_matcher.cpp:13-103 and 1312-1453
 *   OrbMatcher::ComputeThreeMaxima   src/orb_features/orb_matcher.cpp:1584-1625
 * Release-build contractions (g++ -O3 -march=native) are explicit fmaf(): u = fma(fx*xc, invz,
 * cx), v likewise, ur = fma(-bf, invz, u). OpenCV's small float gemm (Rcw*x + tcw) is written
 * as a float dot product followed by (float)((double)dot + (double)t).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

enum { TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30, GRID_COLS = 64, GRID_ROWS = 48 };

int oc_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t pa, pb;
    memcpy(&pa, a + 4 * i, 4);
    memcpy(&pb, b + 4 * i, 4);
    uint32_t v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

typedef struct { int first, second; } ipair;

static int cmp_ipair(const void* a, const void* b) {
  const ipair* x = (const ipair*)a;
  const ipair* y = (const ipair*)b;
  if (x->first != y->first) return x->first < y->first ? -1 : 1;
  return x->second < y->second ? -1 : (x->second > y->second ? 1 : 0);
}

/* Frame::ComputeStereoMatches (frame.cpp:406-577). maxD: the reference reads baseline_ before
 * assigning it (:436 vs :108, UB); we use the ORB-SLAM2 value baseline = bf/fx, maxD = bf/baseline.
 * Rows outside the image in the right-keypoint row table are skipped (never hit: keypoints lie
 * >= 19 px inside every level). An empty vDistIdx skips the median filter (:565-566 reads [0]). */
void oc_stereo_match(const oc_orb_tables* t, const oc_keypoint* kl, const uint8_t* dl, int nl,
                     const oc_keypoint* kr, const uint8_t* dr, int nr, const oc_pyramid* pl,
                     const oc_pyramid* pr, float fx, float bf, float* u_right, float* depth,
                     int* sad_best) {
  for (int i = 0; i < nl; i++) {
    u_right[i] = -1.0f;
    depth[i] = -1.0f;
    if (sad_best) sad_best[i] = -1;
  }
  const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
  const int nRows = pl->h[0];
  /* row table: CSR of right keypoints per row, in iR order */
  int* cnt = (int*)calloc((size_t)nRows + 1, sizeof(int));
  for (int iR = 0; iR < nr; iR++) {
    const float kpY = kr[iR].y;
    const float r = 2.0f * t->scale[kr[iR].octave];
    const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
    for (int yi = minr; yi <= maxr; ++yi)
      if (yi >= 0 && yi < nRows) cnt[yi + 1]++;
  }
  for (int y = 0; y < nRows; y++) cnt[y + 1] += cnt[y];
  int* rowidx = (int*)malloc(sizeof(int) * (cnt[nRows] + 1));
  int* fill = (int*)malloc(sizeof(int) * (nRows + 1));
  memcpy(fill, cnt, sizeof(int) * (nRows + 1));
  for (int iR = 0; iR < nr; iR++) {
    const float kpY = kr[iR].y;
    const float r = 2.0f * t->scale[kr[iR].octave];
    const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
    for (int yi = minr; yi <= maxr; ++yi)
      if (yi >= 0 && yi < nRows) rowidx[fill[yi]++] = iR;
  }
  free(fill);

  const float baseline = bf / fx;
  const float minZ = baseline;
  const float minD = 0;
  const float maxD = bf / minZ;
  ipair* vDistIdx = (ipair*)malloc(sizeof(ipair) * (nl + 1));
  int nDist = 0;
  for (int iL = 0; iL < nl; ++iL) {
    const oc_keypoint* kpL = &kl[iL];
    const int levelL = kpL->octave;
    const float vL = kpL->y, uL = kpL->x;
    const int row = (int)vL;
    if (row < 0 || row >= nRows) continue;
    const int c0 = cnt[row], c1 = cnt[row + 1];
    if (c0 == c1) continue;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = TH_HIGH;
    int bestIdxR = 0;
    const uint8_t* dL = dl + 32 * (size_t)iL;
    for (int c = c0; c < c1; c++) {
      const int iR = rowidx[c];
      const oc_keypoint* kpR = &kr[iR];
      if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
      const float uR = kpR->x;
      if (uR >= minU && uR <= maxU) {
        const int dist = oc_descriptor_distance(dL, dr + 32 * (size_t)iR);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist < thOrbDist) {
      const float uR0 = kr[bestIdxR].x;
      const float scaleFactor = t->inv_scale[kpL->octave];
      const float scaleduL = roundf(kpL->x * scaleFactor);
      const float scaledvL = roundf(kpL->y * scaleFactor);
      const float scaleduR0 = roundf(uR0 * scaleFactor);
      const int w = 5, L = 5;
      const int lev = kpL->octave;
      const uint8_t* IL = pl->data[lev];
      const uint8_t* IR = pr->data[lev];
      const size_t sL = pl->step[lev], sR = pr->step[lev];
      const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
      const float iniu = scaleduR0 + L - w;
      const float endu = scaleduR0 + L + w + 1;
      if (iniu < 0 || endu >= pr->w[lev]) continue;
      int bestSad = 2147483647;
      int bestincR = 0;
      float vDists[11];
      const int cl = IL[(size_t)(yl0 + w) * sL + xl0 + w];
      for (int incR = -L; incR <= L; ++incR) {
        const int xr0 = (int)scaleduR0 + incR - w;
        const int cr = IR[(size_t)(yl0 + w) * sR + xr0 + w];
        double acc = 0;
        for (int yy = 0; yy < 2 * w + 1; yy++)
          for (int xx = 0; xx < 2 * w + 1; xx++) {
            float a = (float)IL[(size_t)(yl0 + yy) * sL + xl0 + xx] - (float)cl;
            float b = (float)IR[(size_t)(yl0 + yy) * sR + xr0 + xx] - (float)cr;
            acc += fabs((double)a - (double)b);
          }
        float dist = (float)acc;
        if (dist < (float)bestSad) {
          bestSad = (int)dist;
          bestincR = incR;
        }
        vDists[L + incR] = dist;
      }
      if (bestincR == -L || bestincR == L) continue;
      const float dist1 = vDists[L + bestincR - 1];
      const float dist2 = vDists[L + bestincR];
      const float dist3 = vDists[L + bestincR + 1];
      const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
      if (deltaR < -1 || deltaR > 1) continue;
      float bestuR = t->scale[kpL->octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
      float disparity = (uL - bestuR);
      if (disparity >= minD && disparity < maxD) {
        if (disparity <= 0) {
          disparity = 0.01f;
          bestuR = uL - 0.01f;
        }
        depth[iL] = bf / disparity;
        u_right[iL] = bestuR;
        if (sad_best) sad_best[iL] = bestSad;
        vDistIdx[nDist].first = bestSad;
        vDistIdx[nDist].second = iL;
        nDist++;
      }
    }
  }
  if (nDist > 0) {
    qsort(vDistIdx, nDist, sizeof(ipair), cmp_ipair);
    const float median = (float)vDistIdx[nDist / 2].first;
    const float thDist = (1.5f * 1.4f) * median;
    for (int i = nDist - 1; i >= 0; --i) {
      if ((float)vDistIdx[i].first < thDist) break;
      u_right[vDistIdx[i].second] = -1.0f;
      depth[vDistIdx[i].second] = -1.0f;
      if (sad_best) sad_best[vDistIdx[i].second] = -1;
    }
  }
  free(vDistIdx);
  free(cnt);
  free(rowidx);
}

/* Frame::ComputeImageBounds (k1 == 0 branch) + MakeInitialComputations grid sizes. */
void oc_grid_geom_init(oc_grid_geom* g, int cols, int rows) {
  g->min_x = 0.0f;
  g->max_x = (float)cols;
  g->min_y = 0.0f;
  g->max_y = (float)rows;
  g->cell_w = (float)(g->max_x - g->min_x) / (GRID_COLS);
  g->cell_h = (float)(g->max_y - g->min_y) / (GRID_ROWS);
}

/* Frame::PosInGrid (frame.cpp:339-346). */
static int pos_in_grid(const oc_grid_geom* g, const oc_keypoint* kp, int* px, int* py) {
  *px = (int)roundf((kp->x - g->min_x) / g->cell_w);
  *py = (int)roundf((kp->y - g->min_y) / g->cell_h);
  return (*px >= 0 && *px < GRID_COLS && *py >= 0 && *py < GRID_ROWS);
}

/* Frame::GetFeaturesInArea (frame.cpp:348-403) over the grid built by AssignFeaturesToGrid
 * (:234-248): cells visited x-major, each cell in ascending keypoint index. */
int oc_features_in_area(const oc_grid_geom* g, const oc_keypoint* kps, int n, float x, float y,
                        float r, int minLevel, int maxLevel, int* out, int cap) {
  int nout = 0;
  const int nMinCellX0 = (int)floorf((x - g->min_x - r) / g->cell_w);
  const int nMinCellX = nMinCellX0 > 0 ? nMinCellX0 : 0;
  const int nMaxCellX0 = (int)ceilf((x - g->min_x + r) / g->cell_w);
  const int nMaxCellX = nMaxCellX0 < GRID_COLS - 1 ? nMaxCellX0 : GRID_COLS - 1;
  if (nMaxCellX < 0 || nMinCellX >= GRID_COLS) return 0;
  const int nMinCellY0 = (int)floorf((y - g->min_y - r) / g->cell_h);
  const int nMinCellY = nMinCellY0 > 0 ? nMinCellY0 : 0;
  const int nMaxCellY0 = (int)ceilf((y - g->min_y + r) / g->cell_h);
  const int nMaxCellY = nMaxCellY0 < GRID_ROWS - 1 ? nMaxCellY0 : GRID_ROWS - 1;
  if (nMaxCellY < 0 || nMinCellY >= GRID_ROWS) return 0;
  const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  /* bucket keypoints once per call (AssignFeaturesToGrid order = ascending index) */
  int* cellOf = (int*)malloc(sizeof(int) * (n + 1));
  for (int i = 0; i < n; i++) {
    int px, py;
    cellOf[i] = pos_in_grid(g, &kps[i], &px, &py) ? px * GRID_ROWS + py : -1;
  }
  for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
    for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
      const int cell = ix * GRID_ROWS + iy;
      for (int j = 0; j < n; j++) {
        if (cellOf[j] != cell) continue;
        const oc_keypoint* kpUn = &kps[j];
        if (bCheckLevels) {
          if (kpUn->octave < minLevel) continue;
          if (maxLevel >= 0 && kpUn->octave > maxLevel) continue;
        }
        const float distx = kpUn->x - x, disty = kpUn->y - y;
        if (fabsf(distx) < r && fabsf(disty) < r) {
          if (nout < cap) out[nout] = j;
          nout++;
        }
      }
    }
  }
  free(cellOf);
  return nout;
}

/* OrbMatcher::ComputeThreeMaxima (orb_matcher.cpp:1584-1625). */
static void three_maxima(const int* sizes, int L, int* ind1, int* ind2, int* ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = sizes[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      *ind3 = *ind2; *ind2 = i;
    } else if (s > max3) {
      max3 = s;
      *ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    *ind2 = -1;
    *ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    *ind3 = -1;
  }
}

static inline int blocked(const oc_frame_view* F, const int* mp_nobs, int idx) {
  const int mp = F->map_point[idx];
  return mp >= 0 && mp_nobs[mp] > 0;
}

/* OpenCV small gemm: d = (float)((double)(float dot) + (double)c). */
static inline float mat3_row(const float* R, int r, const float* x, float c) {
  float dot = R[3 * r] * x[0] + R[3 * r + 1] * x[1] + R[3 * r + 2] * x[2];
  return (float)((double)dot + (double)c);
}

int oc_search_by_projection_frame(const oc_grid_geom* g, const oc_orb_tables* t,
                                  oc_frame_view* cur, const oc_keypoint* last_kps,
                                  const int* last_mp, const uint8_t* last_outlier, int n_last,
                                  const float* mp_xyz, const uint8_t* mp_desc,
                                  const int* mp_nobs, const float* Rcw, const float* tcw,
                                  float tlc_z, float baseline, float fx, float fy, float cx,
                                  float cy, float bf, float th, int mono, int check_ori) {
  int nmatches = 0;
  int* rotHist[HISTO_LENGTH];
  int rotN[HISTO_LENGTH];
  for (int i = 0; i < HISTO_LENGTH; i++) {
    rotHist[i] = (int*)malloc(sizeof(int) * (n_last + 1));
    rotN[i] = 0;
  }
  const float factor = 1.0f / HISTO_LENGTH;
  const int bForward = tlc_z > baseline && !mono;
  const int bBackward = -tlc_z > baseline && !mono;
  int* cand = (int*)malloc(sizeof(int) * (cur->n + 1));
  for (int i = 0; i < n_last; ++i) {
    const int mp = last_mp[i];
    if (mp < 0 || last_outlier[i]) continue;
    const float* X = mp_xyz + 3 * (size_t)mp;
    const float xc = mat3_row(Rcw, 0, X, tcw[0]);
    const float yc = mat3_row(Rcw, 1, X, tcw[1]);
    const float zc = mat3_row(Rcw, 2, X, tcw[2]);
    const float invzc = (float)(1.0 / (double)zc);
    if (invzc < 0) continue;
    const float u = fmaf(fx * xc, invzc, cx);
    const float v = fmaf(fy * yc, invzc, cy);
    if (u < g->min_x || u > g->max_x) continue;
    if (v < g->min_y || v > g->max_y) continue;
    const int nLastOctave = last_kps[i].octave;
    const float radius = th * t->scale[nLastOctave];
    int nc;
    if (bForward)
      nc = oc_features_in_area(g, cur->kps, cur->n, u, v, radius, nLastOctave, -1, cand, cur->n);
    else if (bBackward)
      nc = oc_features_in_area(g, cur->kps, cur->n, u, v, radius, 0, nLastOctave, cand, cur->n);
    else
      nc = oc_features_in_area(g, cur->kps, cur->n, u, v, radius, nLastOctave - 1,
                               nLastOctave + 1, cand, cur->n);
    if (nc == 0) continue;
    const uint8_t* dMP = mp_desc + 32 * (size_t)mp;
    int bestDist = 256, bestIdx2 = -1;
    for (int c = 0; c < nc; c++) {
      const int i2 = cand[c];
      if (blocked(cur, mp_nobs, i2)) continue;
      if (cur->u_right[i2] > 0) {
        const float ur = fmaf(-bf, invzc, u);
        const float er = fabsf(ur - cur->u_right[i2]);
        if (er > radius) continue;
      }
      const int dist = oc_descriptor_distance(dMP, cur->desc + 32 * (size_t)i2);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= TH_HIGH) {
      cur->map_point[bestIdx2] = mp;
      ++nmatches;
      if (check_ori) {
        float rot = last_kps[i].angle - cur->kps[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)roundf(rot * factor);
        if (bin == HISTO_LENGTH) bin = 0;
        rotHist[bin][rotN[bin]++] = bestIdx2;
      }
    }
  }
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotN, HISTO_LENGTH, &ind1, &ind2, &ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i != ind1 && i != ind2 && i != ind3) {
        for (int j = 0; j < rotN[i]; j++) {
          cur->map_point[rotHist[i][j]] = -1;
          --nmatches;
        }
      }
    }
  }
  for (int i = 0; i < HISTO_LENGTH; i++) free(rotHist[i]);
  free(cand);
  return nmatches;
}

/* OrbMatcher::RadiusByViewingCos (orb_matcher.cpp:105-111). */
static inline float radius_by_viewing_cos(float viewCos) {
  return ((double)viewCos > 0.998) ? 2.5f : 4.0f;
}

int oc_search_by_projection_mps(const oc_grid_geom* g, const oc_orb_tables* t,
                                oc_frame_view* F, int n_mp, const uint8_t* in_view,
                                const uint8_t* is_bad, const int* level, const float* view_cos,
                                const float* proj_x, const float* proj_y, const float* proj_xr,
                                const uint8_t* mp_desc, const int* mp_nobs, float nnratio,
                                int th) {
  int nmatches = 0;
  const int bFactor = (th != 1);
  int* cand = (int*)malloc(sizeof(int) * (F->n + 1));
  for (int iMP = 0; iMP < n_mp; iMP++) {
    if (!in_view[iMP]) continue;
    if (is_bad[iMP]) continue;
    const int nPredictedLevel = level[iMP];
    float r = radius_by_viewing_cos(view_cos[iMP]);
    if (bFactor) r *= (float)th;
    const float rs = r * t->scale[nPredictedLevel];
    const int nc = oc_features_in_area(g, F->kps, F->n, proj_x[iMP], proj_y[iMP], rs,
                                       nPredictedLevel - 1, nPredictedLevel, cand, F->n);
    if (nc == 0) continue;
    const uint8_t* MPdescriptor = mp_desc + 32 * (size_t)iMP;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int c = 0; c < nc; c++) {
      const int idx = cand[c];
      if (blocked(F, mp_nobs, idx)) continue;
      if (F->u_right[idx] > 0) {
        const float er = fabsf(proj_xr[iMP] - F->u_right[idx]);
        if (er > r * t->scale[nPredictedLevel]) continue;
      }
      const int dist = oc_descriptor_distance(MPdescriptor, F->desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = F->kps[idx].octave;
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = F->kps[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= TH_HIGH) {
      if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
      F->map_point[bestIdx] = iMP;
      nmatches++;
    }
  }
  free(cand);
  return nmatches;
}

/* ---- Frame::UndistortKeyPoints / ComputeImageBounds ------------------------------------------ */
/* OpenCV 3.3.1 cvUndistortPoints (imgproc/src/undistort.cpp) for the reference's call
 * cv::undistortPoints(mat, mat, K, DistCoef, cv::Mat(), K) (frame.cpp:630, :659): K and the
 * coefficients converted to double (k[14], unset entries 0); iters = 5 because D is given; the
 * tilt matrix for tau = 0 is the identity; RR = P * R = K * I. Evaluation order as written there
 * (left to right, no contraction: this file is built -ffp-contract=off). */
void oc_undistort_points(const float cam[4], const float* dist, int ndist, const float* xy_in,
                         float* xy_out, int n) {
  double k[14] = {0};
  for (int i = 0; i < ndist && i < 14; i++) k[i] = (double)dist[i];
  const double A00 = cam[0], A11 = cam[1], A02 = cam[2], A12 = cam[3];
  const double fx = A00, fy = A11, ifx = 1. / fx, ify = 1. / fy, cx = A02, cy = A12;
  /* RR = PP * I (cvMatMul of the 3x3 K with the identity): rows (fx 0 cx) (0 fy cy) (0 0 1) */
  const double RR[3][3] = {{A00, 0., A02}, {0., A11, A12}, {0., 0., 1.}};
  for (int i = 0; i < n; i++) {
    double x = xy_in[2 * i], y = xy_in[2 * i + 1], x0, y0;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    /* tilt compensation: vecUntilt = I * (x, y, 1), invProj = 1 */
    x0 = x;
    y0 = y;
    for (int j = 0; j < 5; j++) {
      double r2 = x * x + y * y;
      double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                      (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
      double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
      double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
      x = (x0 - deltaX) * icdist;
      y = (y0 - deltaY) * icdist;
    }
    double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
    double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
    double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
    xy_out[2 * i] = (float)(xx * ww);
    xy_out[2 * i + 1] = (float)(yy * ww);
  }
}

void oc_undistort_keypoints(const float cam[4], const float* dist, int ndist,
                            const oc_keypoint* in, oc_keypoint* out, int n) {
  for (int i = 0; i < n; i++) out[i] = in[i];
  if (dist[0] == 0.0f) return; /* frame.cpp:616-619 */
  for (int i = 0; i < n; i++) {
    float p[2] = {in[i].x, in[i].y};
    oc_undistort_points(cam, dist, ndist, p, p, 1);
    out[i].x = p[0];
    out[i].y = p[1];
  }
}

void oc_grid_geom_init_dist(oc_grid_geom* g, int cols, int rows, const float cam[4],
                            const float* dist, int ndist) {
  oc_grid_geom_init(g, cols, rows);
  if (dist[0] != 0.0) { /* frame.cpp:646-667: corners (0,0) (cols,0) (0,rows) (cols,rows) */
    float m[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
    oc_undistort_points(cam, dist, ndist, m, m, 4);
    g->min_x = fminf(m[0], m[4]);
    g->max_x = fmaxf(m[2], m[6]);
    g->min_y = fminf(m[1], m[3]);
    g->max_y = fmaxf(m[5], m[7]);
    g->cell_w = (float)(g->max_x - g->min_x) / (GRID_COLS);
    g->cell_h = (float)(g->max_y - g->min_y) / (GRID_ROWS);
  }
}
