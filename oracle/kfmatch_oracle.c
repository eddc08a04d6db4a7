/*
 * oracle/kfmatch_oracle.c -- CPU restatement of the keyframe-rate matchers the LocalMapper runs
 * before LocalBundleAdjustment (TEST INFRASTRUCTURE ONLY; see orb_oracle.h):
 *   src/orb_features/orb_matcher.cpp:634-802   SearchForTriangulation(pKF1, pKF2, F12, ...)
 *   src/orb_features/orb_matcher.cpp:114-131   CheckDistEpipolarLine
 *   src/orb_features/orb_matcher.cpp:804-954   Fuse(pKF, vpMapPoints, th) -- the candidate search
 *   src/data/map_point.cpp:356-381             Get{Min,Max}DistanceInvariance, PredictScale
 *   src/data/keyframe.cpp:442-476, :494-496     KeyFrame::GetFeaturesInArea, IsInImage
 *
 * Release-build contractions (g++ 11 -O3 -march=native on the same expressions, read from the
 * assembly): epipolar line a = fma(x1, F00, y1*F10) + F20 (b, c likewise), num = fma(a, x2,
 * b*y2) + c, den = fma(a, a, b*b), dsqr = num*num/den compared in double against 3.84*sigma2;
 * epipole distance fma(dx, dx, dy*dy) < 100.f*scale; projections fma(fx, x, cx), ur =
 * fma(-bf, invz, u), reprojection errors fma(er, er, fma(ex, ex, ey*ey)) (stereo) /
 * fma(ex, ex, ey*ey) (mono), (double)(e2*invSigma2) > 7.8 / 5.99. OpenCV (no contraction):
 * Rcw*X + tcw as a float dot + (double) add (see matcher_oracle.c), cv::norm of a 3-vector as a
 * double sum of squares, Mat::dot as a double sum of exact products. std::log(float) = glibc
 * logf (oc_logf, pinned exhaustively).
 *
 * SearchForTriangulation never sets vbMatched2 (the reference declares it, :656, and never
 * writes it), so every pKF1 feature is matched independently. Its inner loop keeps a candidate
 * when dist <= TH_LOW and dist <= the best so far (:717): the result is the LAST passing
 * candidate of minimal distance in node order.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary (OpenCV / DBoW2 absent; no
 * fixtures). Pinned by tests/test_kfmatch_oracle.py against an independent pure-Python
 * restatement.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

/* OpenCV small gemm row: (float)((double)(float dot) + (double)c) (matcher_oracle.c). */
static inline float gemm_row(const float* R, int r, const float* x, float c) {
  const float dot = R[3 * r] * x[0] + R[3 * r + 1] * x[1] + R[3 * r + 2] * x[2];
  return (float)((double)dot + (double)c);
}

static void three_maxima30(const int* hist, int* i1, int* i2, int* i3) {
  int m1 = 0, m2 = 0, m3 = 0;
  *i1 = *i2 = *i3 = -1;
  for (int i = 0; i < 30; i++) {
    const int s = hist[i];
    if (s > m1) {
      m3 = m2; m2 = m1; m1 = s;
      *i3 = *i2; *i2 = *i1; *i1 = i;
    } else if (s > m2) {
      m3 = m2; m2 = s;
      *i3 = *i2; *i2 = i;
    } else if (s > m3) {
      m3 = s;
      *i3 = i;
    }
  }
  if (m2 < 0.1f * (float)m1) {
    *i2 = -1;
    *i3 = -1;
  } else if (m3 < 0.1f * (float)m1) {
    *i3 = -1;
  }
}

/* CheckDistEpipolarLine (orb_matcher.cpp:114-131), F row-major. */
int oc_check_dist_epipolar(const oc_keypoint* kp1, const oc_keypoint* kp2, const float* F,
                           const float* sigma2) {
  const float a = fmaf(kp1->x, F[0], kp1->y * F[3]) + F[6];
  const float b = fmaf(kp1->x, F[1], kp1->y * F[4]) + F[7];
  const float c = fmaf(kp1->x, F[2], kp1->y * F[5]) + F[8];
  const float num = fmaf(a, kp2->x, b * kp2->y) + c;
  const float den = fmaf(a, a, b * b);
  if (den == 0) return 0;
  const float dsqr = num * num / den;
  return (double)dsqr < 3.84 * (double)sigma2[kp2->octave];
}

/* The epipole of pKF1's centre in pKF2 (orb_matcher.cpp:643-649): C2 = R2w*Cw + t2w. */
void oc_epipole(const float* C1w, const float* T2w, float fx, float fy, float cx, float cy,
                float* ex, float* ey) {
  const float c2x = gemm_row(T2w, 0, C1w, T2w[9]);
  const float c2y = gemm_row(T2w, 1, C1w, T2w[10]);
  const float c2z = gemm_row(T2w, 2, C1w, T2w[11]);
  const float invz = 1.0f / c2z;
  *ex = fmaf(fx * c2x, invz, cx);
  *ey = fmaf(fy * c2y, invz, cy);
}

static int node_find(const uint32_t* nodes, int nn, uint32_t key) {
  int lo = 0, hi = nn;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (nodes[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return (lo < nn && nodes[lo] == key) ? lo : -1;
}

/* SearchForTriangulation (orb_matcher.cpp:634-802). Keyframe i: keypoints k, descriptors d,
 * right coordinates ur (< 0 mono), has_mp (GetMapPoint(idx) != NULL), FeatureVector (nodes,
 * start, feats). T2w = pKF2's R (row-major) then t; C1w = pKF1->GetCameraCenter(). scale /
 * sigma2 = pKF2's scale_factors / level_sigma_sq. match12[idx1] = vMatches12; returns nmatches. */
int oc_search_for_triangulation(
    const oc_keypoint* k1, const uint8_t* d1, const float* ur1, const uint8_t* mp1, int n1,
    const uint32_t* nodes1, const int32_t* start1, const uint32_t* feats1, int nn1,
    const oc_keypoint* k2, const uint8_t* d2, const float* ur2, const uint8_t* mp2,
    const uint32_t* nodes2, const int32_t* start2, const uint32_t* feats2, int nn2,
    const float* C1w, const float* T2w, float fx, float fy, float cx, float cy,
    const float* scale, const float* sigma2, const float* F12, int only_stereo, int check_ori,
    int32_t* match12) {
  const int TH_LOW = 50;
  float ex, ey;
  oc_epipole(C1w, T2w, fx, fy, cx, cy, &ex, &ey);
  int nmatches = 0;
  int hist[30] = {0};
  int8_t* bin_of = (int8_t*)malloc((size_t)(n1 > 0 ? n1 : 1));
  memset(bin_of, -1, (size_t)(n1 > 0 ? n1 : 1));
  for (int i = 0; i < n1; i++) match12[i] = -1;
  const float factor = 1.0f / 30;
  for (int ia = 0; ia < nn1; ia++) { /* the merge visits the common nodes in ascending order */
    const int ib = node_find(nodes2, nn2, nodes1[ia]);
    if (ib < 0) continue;
    for (int p = start1[ia]; p < start1[ia + 1]; p++) {
      const int idx1 = (int)feats1[p];
      if (mp1[idx1]) continue;
      const int bStereo1 = ur1[idx1] >= 0;
      if (only_stereo && !bStereo1) continue;
      const oc_keypoint* kp1 = &k1[idx1];
      int bestDist = TH_LOW, bestIdx2 = -1;
      for (int q = start2[ib]; q < start2[ib + 1]; q++) {
        const int idx2 = (int)feats2[q];
        if (mp2[idx2]) continue;
        const int bStereo2 = ur2[idx2] >= 0;
        if (only_stereo && !bStereo2) continue;
        const int dist = oc_descriptor_distance(d1 + (size_t)idx1 * 32, d2 + (size_t)idx2 * 32);
        if (dist > TH_LOW || dist > bestDist) continue;
        const oc_keypoint* kp2 = &k2[idx2];
        if (!bStereo1 && !bStereo2) {
          const float distex = ex - kp2->x;
          const float distey = ey - kp2->y;
          if (fmaf(distex, distex, distey * distey) < 100 * scale[kp2->octave]) continue;
        }
        if (oc_check_dist_epipolar(kp1, kp2, F12, sigma2)) {
          bestIdx2 = idx2;
          bestDist = dist;
        }
      }
      if (bestIdx2 >= 0) {
        match12[idx1] = bestIdx2;
        nmatches++;
        if (check_ori) {
          float rot = kp1->angle - k2[bestIdx2].angle;
          if (rot < 0.0) rot += 360.0f;
          int bin = (int)roundf(rot * factor);
          if (bin == 30) bin = 0;
          bin_of[idx1] = (int8_t)bin;
          hist[bin]++;
        }
      }
    }
  }
  if (check_ori) {
    int i1, i2, i3;
    three_maxima30(hist, &i1, &i2, &i3);
    for (int i = 0; i < n1; i++) {
      const int b = bin_of[i];
      if (b >= 0 && b != i1 && b != i2 && b != i3) {
        match12[i] = -1;
        nmatches--;
      }
    }
  }
  free(bin_of);
  return nmatches;
}

/* MapPoint::PredictScale(dist, KeyFrame*) (map_point.cpp:366-381). */
int oc_predict_scale(float max_dist, float dist, float log_scale_factor, int nlevels) {
  const float ratio = max_dist / dist;
  int n = (int)ceilf(oc_logf(ratio) / log_scale_factor);
  if (n < 0) n = 0;
  else if (n >= nlevels) n = nlevels - 1;
  return n;
}

/* Fuse(pKF, vpMapPoints, th) (orb_matcher.cpp:804-954), the per-point candidate search at the
 * state the call starts from: pts[i].skip = !pMP || isBad() || IsInKeyFrame(pKF). best_idx[i] =
 * the keypoint the point fuses into (bestDist <= TH_LOW) or -1, best_dist[i] = bestDist (256 if
 * none). Returns the number of points with best_idx >= 0 (= nFused when the Replace /
 * AddObservation calls of earlier points do not change the skip state of later ones).
 * kf->Rcw row-major, tcw, Ow = GetCameraCenter(); g = the keyframe's grid and image bounds
 * (min_x_ .. max_y_ are ints in KeyFrame). */
int oc_fuse(const oc_keypoint* kps, const uint8_t* desc, const float* ur, int n,
            const oc_grid_geom* g, const float* Rcw, const float* tcw, const float* Ow, float fx,
            float fy, float cx, float cy, float bf, const float* scale, const float* inv_sigma2,
            int nlevels, float log_scale_factor, const oc_fuse_point* pts, int n_pts, float th,
            int32_t* best_idx, int32_t* best_dist) {
  const int TH_LOW = 50;
  int nfused = 0;
  int* cand = (int*)malloc(sizeof(int) * (size_t)(n + 1));
  for (int i = 0; i < n_pts; i++) {
    const oc_fuse_point* P = &pts[i];
    best_idx[i] = -1;
    best_dist[i] = 256;
    if (P->skip) continue;
    const float xc = gemm_row(Rcw, 0, P->xyz, tcw[0]);
    const float yc = gemm_row(Rcw, 1, P->xyz, tcw[1]);
    const float zc = gemm_row(Rcw, 2, P->xyz, tcw[2]);
    if (zc < 0.0f) continue;
    const float invz = 1 / zc;
    const float x = xc * invz, y = yc * invz;
    const float u = fmaf(fx, x, cx), v = fmaf(fy, y, cy);
    if (!(u >= g->min_x && u < g->max_x && v >= g->min_y && v < g->max_y)) continue;
    const float urp = fmaf(-bf, invz, u);
    const float maxDistance = 1.2f * P->max_dist, minDistance = 0.8f * P->min_dist;
    const float PO[3] = {P->xyz[0] - Ow[0], P->xyz[1] - Ow[1], P->xyz[2] - Ow[2]};
    double s = 0.0;
    for (int k = 0; k < 3; k++) s += (double)PO[k] * (double)PO[k];
    const float dist3D = (float)sqrt(s);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    double dot = 0.0;
    for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)P->normal[k];
    if (dot < 0.5 * (double)dist3D) continue;
    const int nPredictedLevel = oc_predict_scale(P->max_dist, dist3D, log_scale_factor, nlevels);
    const float radius = th * scale[nPredictedLevel];
    const int nc = oc_features_in_area(g, kps, n, u, v, radius, -1, -1, cand, n + 1);
    int bestDist = 256, bestIdx = -1;
    for (int c = 0; c < nc; c++) {
      const int idx = cand[c];
      const oc_keypoint* kp = &kps[idx];
      const int kpLevel = kp->octave;
      if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
      const float ex = u - kp->x, ey = v - kp->y;
      if (ur[idx] >= 0) {
        const float er = urp - ur[idx];
        const float e2 = fmaf(er, er, fmaf(ex, ex, ey * ey));
        if ((double)(e2 * inv_sigma2[kpLevel]) > 7.8) continue;
      } else {
        const float e2 = fmaf(ex, ex, ey * ey);
        if ((double)(e2 * inv_sigma2[kpLevel]) > 5.99) continue;
      }
      const int dist = oc_descriptor_distance(P->desc, desc + (size_t)idx * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    best_dist[i] = bestDist;
    if (bestDist <= TH_LOW) {
      best_idx[i] = bestIdx;
      nfused++;
    }
  }
  free(cand);
  return nfused;
}
