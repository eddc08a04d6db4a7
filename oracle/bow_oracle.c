/*
 * oracle/bow_oracle.c -- CPU restatement of the DBoW2 vocabulary transform, the two
 * OrbMatcher::SearchByBoW overloads, MapPoint::ComputeDistinctiveDescriptors and the colour ->
 * gray conversion of Tracker::GrabImageStereo (TEST INFRASTRUCTURE ONLY; see orb_oracle.h).
 *
 * Follows (paths relative to the reference repository root):
 *   third_party/DBoW2/DBoW2/TemplatedVocabulary.h
 *       :1335-1421  loadFromTextFile      (node creation order, children in file order, word ids
 *                                          = order of the leaf-flagged lines)
 *       :1214-1256  transform(feature, word_id, weight, nid, levelsup)
 *       :1123-1191  transform(features, BowVector, FeatureVector, levelsup)
 *   third_party/DBoW2/DBoW2/BowVector.cpp:34-84   addWeight / addIfNotExist / normalize
 *   third_party/DBoW2/DBoW2/FeatureVector.cpp:31-44 addFeature
 *   third_party/DBoW2/DBoW2/ScoringObject.h:53-89  mustNormalize per scoring type
 *   third_party/DBoW2/DBoW2/FORB.cpp:81-101        distance (== popcount of the xor)
 *   src/orb_features/orb_matcher.cpp:133-262        SearchByBoW(KeyFrame*, Frame&, ...)
 *   src/orb_features/orb_matcher.cpp:499-632        SearchByBoW(KeyFrame*, KeyFrame*, ...)
 *   src/data/map_point.cpp:249-304                  ComputeDistinctiveDescriptors
 *   src/core/tracker.cpp:110-127                    cv::cvtColor(*2GRAY) (OpenCV 3.3.1
 *                                                   RGB2Gray<uchar>, imgproc/color.cpp)
 *
 * The vocabulary is given as the arrays loadFromTextFile builds (node 0 = root). The vocabulary
 * text file itself (ORBvoc.txt) is not part of the reference repository; the parity tests use
 * seeded synthetic vocabularies of the same format.
 *
 * Release-build contraction: the reference compiles DBoW2 with -O3 -march=native (CMakeLists.txt
 * :11-13 applies to third_party/), so BowVector::normalize's L2 sum `norm += x * x` is an fma.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary (DBoW2 needs OpenCV; the
 * reference ships no vocabulary and no tests for this path). Pinned by tests/test_bow_oracle.py
 * against an independent pure-Python restatement and hand-checked trees.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

struct oc_vocab {
  int k, L, scoring, weighting;
  int n_nodes, n_words;
  int32_t* child_start; /* [n_nodes + 1] CSR of children in file order */
  int32_t* children;
  uint8_t* desc;        /* [n_nodes][32] */
  double* weight;       /* [n_nodes] */
  uint32_t* word_id;    /* [n_nodes] (0 for nodes without the leaf flag, Node() ctor :314) */
};

oc_vocab* oc_vocab_build(const oc_vocab_arrays* a) {
  if (a->n_nodes < 1) return NULL;
  for (int i = 1; i < a->n_nodes; i++)
    if (a->parent[i] < 0 || a->parent[i] >= i) return NULL;
  oc_vocab* v = (oc_vocab*)calloc(1, sizeof(oc_vocab));
  const int n = a->n_nodes;
  v->k = a->k;
  v->L = a->L;
  v->scoring = a->scoring;
  v->weighting = a->weighting;
  v->n_nodes = n;
  v->child_start = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
  v->children = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  v->desc = (uint8_t*)calloc((size_t)n, 32);
  v->weight = (double*)calloc((size_t)n, sizeof(double));
  v->word_id = (uint32_t*)calloc((size_t)n, sizeof(uint32_t));
  if (n > 1) memcpy(v->desc + 32, a->desc + 32, (size_t)(n - 1) * 32);
  /* m_nodes[pid].children.push_back(nid) in line order (:1389) */
  for (int i = 1; i < n; i++) v->child_start[a->parent[i] + 1]++;
  for (int i = 0; i < n; i++) v->child_start[i + 1] += v->child_start[i];
  int32_t* fill = (int32_t*)malloc((size_t)n * sizeof(int32_t));
  memcpy(fill, v->child_start, (size_t)n * sizeof(int32_t));
  for (int i = 1; i < n; i++) v->children[fill[a->parent[i]]++] = i;
  free(fill);
  int words = 0;
  for (int i = 1; i < n; i++) {
    v->weight[i] = a->weight[i];
    if (a->leaf_flag[i]) v->word_id[i] = (uint32_t)words++; /* :1405-1412 */
  }
  v->n_words = words;
  return v;
}

void oc_vocab_free(oc_vocab* v) {
  if (!v) return;
  free(v->child_start);
  free(v->children);
  free(v->desc);
  free(v->weight);
  free(v->word_id);
  free(v);
}

static int is_leaf(const oc_vocab* v, int node) {
  return v->child_start[node + 1] == v->child_start[node]; /* children.empty() :326 */
}

/* transform(feature, word_id, weight, nid, levelsup)  TemplatedVocabulary.h:1214-1256.
 * *leaf (optional) = the node the descent ends at. A level-`nid_level` node the descent never
 * reaches (a leaf above that level) leaves *nid at that leaf (declared semantics: the reference
 * leaves the caller's variable unassigned). Requires a root with children. */
void oc_vocab_transform_one(const oc_vocab* v, const uint8_t d[32], int levelsup, uint32_t* word,
                            double* weight, uint32_t* nid, uint32_t* leaf) {
  const int nid_level = v->L - levelsup;
  uint32_t node_at = 0; /* root when nid_level <= 0 (:1224) */
  int final_id = 0, level = 0;
  do {
    ++level;
    const int c0 = v->child_start[final_id], c1 = v->child_start[final_id + 1];
    int best_id = v->children[c0];
    int best_d = oc_descriptor_distance(d, v->desc + (size_t)best_id * 32);
    for (int c = c0 + 1; c < c1; c++) {
      const int id = v->children[c];
      const int dd = oc_descriptor_distance(d, v->desc + (size_t)id * 32);
      if (dd < best_d) { /* strict: the first child wins ties (:1241) */
        best_d = dd;
        best_id = id;
      }
    }
    final_id = best_id;
    if (level == nid_level) node_at = (uint32_t)final_id;
  } while (!is_leaf(v, final_id));
  if (nid_level > level) node_at = (uint32_t)final_id;
  *word = v->word_id[final_id];
  *weight = v->weight[final_id];
  if (nid) *nid = node_at;
  if (leaf) *leaf = (uint32_t)final_id;
}

typedef struct {
  uint32_t key;
  uint32_t idx;
  double w;
} kv_t;

static int kv_cmp(const void* a, const void* b) {
  const kv_t* x = (const kv_t*)a;
  const kv_t* y = (const kv_t*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* transform(features, BowVector, FeatureVector, levelsup)  TemplatedVocabulary.h:1123-1191.
 * BowVector = (words[], values[]) in ascending word order (std::map); FeatureVector = nodes[]
 * ascending with their feature indices node_feats[node_start[i] .. node_start[i + 1]). */
int oc_bow_transform(const oc_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* words,
                     double* values, int* n_words, uint32_t* nodes, int32_t* node_start,
                     uint32_t* node_feats, int* n_nodes) {
  *n_words = 0;
  *n_nodes = 0;
  node_start[0] = 0;
  if (v->n_words == 0 || is_leaf(v, 0)) return 0; /* empty() (:1131) */
  /* mustNormalize (ScoringObject.h:74-89): all but DOT_PRODUCT; the L2 norm only for L2_NORM */
  const int must = v->scoring != 5;
  const int l2 = v->scoring == 1;
  const int tf = v->weighting == 0 || v->weighting == 1;
  kv_t* bw = (kv_t*)malloc(sizeof(kv_t) * (size_t)(n > 0 ? n : 1));
  kv_t* fv = (kv_t*)malloc(sizeof(kv_t) * (size_t)(n > 0 ? n : 1));
  int m = 0;
  for (int i = 0; i < n; i++) {
    uint32_t w, nid;
    double wt;
    oc_vocab_transform_one(v, desc + (size_t)i * 32, levelsup, &w, &wt, &nid, NULL);
    if (wt > 0) { /* not stopped (:1154, :1182) */
      bw[m].key = w;
      bw[m].idx = (uint32_t)i;
      bw[m].w = wt;
      fv[m].key = nid;
      fv[m].idx = (uint32_t)i;
      fv[m].w = 0;
      m++;
    }
  }
  qsort(bw, (size_t)m, sizeof(kv_t), kv_cmp);
  qsort(fv, (size_t)m, sizeof(kv_t), kv_cmp);
  int nw = 0;
  for (int i = 0; i < m; i++) {
    if (i > 0 && bw[i].key == bw[i - 1].key) {
      if (tf) values[nw - 1] += bw[i].w; /* addWeight: += in feature order (BowVector.cpp:40) */
      continue;                          /* addIfNotExist keeps the first (:54-57) */
    }
    words[nw] = bw[i].key;
    values[nw] = bw[i].w;
    nw++;
  }
  if (tf && nw > 0 && !must) {
    const double nd = (double)nw; /* :1161-1167 */
    for (int i = 0; i < nw; i++) values[i] /= nd;
  }
  if (must) { /* BowVector::normalize (BowVector.cpp:62-84) */
    double norm = 0.0;
    if (!l2) {
      for (int i = 0; i < nw; i++) norm += fabs(values[i]);
    } else {
      for (int i = 0; i < nw; i++) norm = fma(values[i], values[i], norm);
      norm = sqrt(norm);
    }
    if (norm > 0.0)
      for (int i = 0; i < nw; i++) values[i] /= norm;
  }
  int nn = 0;
  for (int i = 0; i < m; i++) {
    if (i == 0 || fv[i].key != fv[i - 1].key) {
      nodes[nn] = fv[i].key;
      node_start[nn] = i;
      nn++;
    }
    node_feats[i] = fv[i].idx; /* addFeature appends in feature order (FeatureVector.cpp:31) */
  }
  node_start[nn] = m;
  *n_words = nw;
  *n_nodes = nn;
  free(bw);
  free(fv);
  return 0;
}

/* ComputeThreeMaxima (orb_matcher.cpp:1584-1625) over bin counts. */
static void three_maxima(const int* hist, int* i1, int* i2, int* i3) {
  int max1 = 0, max2 = 0, max3 = 0;
  *i1 = *i2 = *i3 = -1;
  for (int i = 0; i < 30; i++) {
    const int s = hist[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      *i3 = *i2; *i2 = *i1; *i1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      *i3 = *i2; *i2 = i;
    } else if (s > max3) {
      max3 = s;
      *i3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    *i2 = -1;
    *i3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    *i3 = -1;
  }
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

/* The two SearchByBoW overloads share one core (orb_matcher.cpp:133-262 and :499-632):
 * A = the keyframe whose features are iterated (pKF / pKF1), B = the other view (F / pKF2).
 * a_valid[i]: A's map point i exists and is not bad; b_valid NULL = every B feature is a
 * candidate (the Frame overload), else B's map point exists and is not bad (the KF-KF one).
 * strict_lt: bestDist1 < TH_LOW (KF-KF, :575) instead of <= TH_LOW (Frame, :202).
 * Output match_a[i] = the B feature matched to A feature i, or -1; returns nmatches. The Frame
 * overload's vpMapPointMatches[b] = A's map point of the i with match_a[i] == b; the KF-KF
 * overload's vpMatches12[i] = B's map point of match_a[i]. */
int oc_search_by_bow(const uint8_t* a_desc, const oc_keypoint* a_kps, const uint8_t* a_valid,
                     int n_a, const uint32_t* a_nodes, const int32_t* a_start,
                     const uint32_t* a_feats, int a_nn, const uint8_t* b_desc,
                     const oc_keypoint* b_kps, const uint8_t* b_valid, int n_b,
                     const uint32_t* b_nodes, const int32_t* b_start, const uint32_t* b_feats,
                     int b_nn, int strict_lt, float nnratio, int check_ori, int32_t* match_a) {
  const int TH_LOW = 50, HISTO_LENGTH = 30;
  for (int i = 0; i < n_a; i++) match_a[i] = -1;
  uint8_t* taken = (uint8_t*)calloc((size_t)(n_b > 0 ? n_b : 1), 1);
  int8_t* bin_of = (int8_t*)malloc((size_t)(n_a > 0 ? n_a : 1));
  memset(bin_of, -1, (size_t)(n_a > 0 ? n_a : 1));
  int hist[30] = {0};
  const float factor = 1.0f / HISTO_LENGTH;
  int nmatches = 0;
  /* the merge over both FeatureVectors visits exactly the common node ids, ascending */
  for (int ia = 0; ia < a_nn; ia++) {
    const int ib = node_find(b_nodes, b_nn, a_nodes[ia]);
    if (ib < 0) continue;
    for (int p = a_start[ia]; p < a_start[ia + 1]; p++) {
      const int idx_a = (int)a_feats[p];
      if (a_valid && !a_valid[idx_a]) continue;
      int best1 = 256, best2 = 256, best_b = -1;
      for (int q = b_start[ib]; q < b_start[ib + 1]; q++) {
        const int idx_b = (int)b_feats[q];
        if (taken[idx_b]) continue;
        if (b_valid && !b_valid[idx_b]) continue;
        const int dist = oc_descriptor_distance(a_desc + (size_t)idx_a * 32,
                                                b_desc + (size_t)idx_b * 32);
        if (dist < best1) {
          best2 = best1;
          best1 = dist;
          best_b = idx_b;
        } else if (dist < best2) {
          best2 = dist;
        }
      }
      const int pass = strict_lt ? (best1 < TH_LOW) : (best1 <= TH_LOW);
      if (pass && (float)best1 < nnratio * (float)best2) {
        match_a[idx_a] = best_b;
        taken[best_b] = 1;
        if (check_ori) {
          float rot = a_kps[idx_a].angle - b_kps[best_b].angle;
          if (rot < 0.0) rot += 360.0f;
          int bin = (int)roundf(rot * factor);
          if (bin == HISTO_LENGTH) bin = 0;
          bin_of[idx_a] = (int8_t)bin;
          hist[bin]++;
        }
        nmatches++;
      }
    }
  }
  if (check_ori) {
    int i1, i2, i3;
    three_maxima(hist, &i1, &i2, &i3);
    for (int i = 0; i < n_a; i++) {
      const int bin = bin_of[i];
      if (bin >= 0 && bin != i1 && bin != i2 && bin != i3) {
        match_a[i] = -1;
        nmatches--;
      }
    }
  }
  free(taken);
  free(bin_of);
  return nmatches;
}

/* MapPoint::ComputeDistinctiveDescriptors (src/data/map_point.cpp:249-304) over a batch of map
 * points: point p's observed descriptors are desc[start[p] .. start[p + 1]) (the observations
 * map's order, bad keyframes already dropped). best[p] = index (relative to start[p]) of the
 * descriptor with the least median distance to the others (first wins ties), -1 if none. */
void oc_distinctive_descriptors(const uint8_t* desc, const int32_t* start, int n_points,
                                int32_t* best) {
  for (int p = 0; p < n_points; p++) {
    const int s = start[p], n = start[p + 1] - start[p];
    if (n <= 0) {
      best[p] = -1; /* descriptors.empty() -> return (:270-272) */
      continue;
    }
    int* row = (int*)malloc(sizeof(int) * (size_t)n);
    const int half = (int)(0.5 * (n - 1)); /* :289 */
    int best_median = 0x7fffffff, best_idx = 0;
    for (int i = 0; i < n; i++) {
      for (int j = 0; j < n; j++)
        row[j] = (i == j) ? 0
                          : oc_descriptor_distance(desc + (size_t)(s + i) * 32,
                                                   desc + (size_t)(s + j) * 32);
      /* nth_element(half): the half-th smallest value (:291-293) */
      int median = 0;
      for (int c = 0; c < n; c++) {
        int less = 0, equal = 0;
        for (int j = 0; j < n; j++) {
          less += row[j] < row[c];
          equal += row[j] == row[c];
        }
        if (less <= half && half < less + equal) {
          median = row[c];
          break;
        }
      }
      if (median < best_median) { /* :294 */
        best_median = median;
        best_idx = i;
      }
    }
    best[p] = best_idx;
    free(row);
  }
}

/* cv::cvtColor(src, dst, CV_{RGB,BGR,RGBA,BGRA}2GRAY) on 8U data: OpenCV 3.3.1
 * RGB2Gray<uchar> (imgproc/color.cpp) -- tables tab[i] = i*db, tab[256+i] = i*dg,
 * tab[512+i] = i*dr + (1 << 13) with {R2Y, G2Y, B2Y} = {4899, 9617, 1868}, db = coeffs[bidx^2],
 * dr = coeffs[bidx], bidx = 2 for the RGB orders and 0 for BGR; Y = sum >> 14. */
void oc_cvt_gray(const uint8_t* src, size_t sstep, int cn, int rgb, int cols, int rows,
                 uint8_t* dst, size_t dstep) {
  const int coeffs[3] = {4899, 9617, 1868};
  const int bidx = rgb ? 2 : 0;
  const int db = coeffs[bidx ^ 2], dg = coeffs[1], dr = coeffs[bidx];
  int tab[768];
  int b = 0, g = 0, r = 1 << 13;
  for (int i = 0; i < 256; i++, b += db, g += dg, r += dr) {
    tab[i] = b;
    tab[i + 256] = g;
    tab[i + 512] = r;
  }
  for (int y = 0; y < rows; y++) {
    const uint8_t* s = src + (size_t)y * sstep;
    uint8_t* d = dst + (size_t)y * dstep;
    for (int x = 0; x < cols; x++, s += cn)
      d[x] = (uint8_t)((tab[s[0]] + tab[s[1] + 256] + tab[s[2] + 512]) >> 14);
  }
}
