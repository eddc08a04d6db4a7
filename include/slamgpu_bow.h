/*
 * slamgpu_bow.h -- C ABI of the bag-of-words and keyframe-rate matchers and the colour ingest
 * (libslamgpu.so). SURVEY.md section 8(f) rows 1-3, drop-in for (paths relative to the reference
 * repository root):
 *   DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (third_party/DBoW2/DBoW2/
 *     TemplatedVocabulary.h): loadFromTextFile :1335-1421 (called by SlamSystem,
 *     src/slam_system.cpp:35) and transform(features, BowVector, FeatureVector, levelsup)
 *     :1123-1191 (called by Frame::ComputeBoW src/data/frame.cpp:258-263 and
 *     KeyFrame::ComputeBoW src/data/keyframe.cpp:127-135, levelsup = 4)
 *   OrbMatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)  orb_matcher.cpp:133-262
 *     (callers tracker.cpp:666, :860) and SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)
 *     orb_matcher.cpp:499-632 (caller loop_closer.cpp:327)
 *   MapPoint::ComputeDistinctiveDescriptors  src/data/map_point.cpp:249-304
 *   cv::cvtColor(CV_{RGB,BGR,RGBA,BGRA}2GRAY) of Tracker::GrabImageStereo  tracker.cpp:110-127
 * Conventions as slamgpu.h: POD types, caller-owned buffers, 0 or a negative SLAMGPU_E* code with
 * the message in slamgpu_bow_last_error() (per thread). Synchronous host-buffer calls stage
 * through device buffers owned by the vocabulary (transform) or by the calling thread (the
 * others); the *_device calls take device pointers and a hipStream_t, never allocate and return
 * without synchronising.
 */
#ifndef SLAMGPU_BOW_H_
#define SLAMGPU_BOW_H_

#include <stddef.h>
#include <stdint.h>

#include "slamgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Largest descriptor set one transform / SearchByBoW call handles (LDS-resident sort). */
#define SLAMGPU_BOW_MAX_FEATURES 4096

/* DBoW2 enums (third_party/DBoW2/DBoW2/BowVector.h:36-53). */
enum { SLAMGPU_TF_IDF = 0, SLAMGPU_TF = 1, SLAMGPU_IDF = 2, SLAMGPU_BINARY = 3 };
enum {
  SLAMGPU_L1_NORM = 0, SLAMGPU_L2_NORM = 1, SLAMGPU_CHI_SQUARE = 2, SLAMGPU_KL = 3,
  SLAMGPU_BHATTACHARYYA = 4, SLAMGPU_DOT_PRODUCT = 5
};

typedef struct slamgpu_vocab slamgpu_vocab;

const char* slamgpu_bow_last_error(void);

/* ---- vocabulary --------------------------------------------------------------------------- */
/* Replaces TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1335-1421): header
 * "k L scoring weighting", then one line per node "parent isLeaf d0 .. d31 weight" (node ids in
 * line order from 1; node 0 is the root). Lines with nothing but blanks add no node (declared: the
 * reference appends a childless node with an unset descriptor for each, e.g. for the final
 * newline). */
int slamgpu_vocab_load_text(int device, const char* path, slamgpu_vocab** out);
/* The arrays loadFromTextFile builds, n_nodes entries each (entry 0 = the root, ignored):
 * parent[i] < i, leaf[i] = the line's isLeaf > 0, desc[i][32], weight[i]. */
int slamgpu_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes,
                         const int32_t* parent, const uint8_t* leaf, const uint8_t* desc,
                         const double* weight, slamgpu_vocab** out);
void slamgpu_vocab_destroy(slamgpu_vocab* v);
/* info[6] = k, L, scoring, weighting, #nodes (with the root), #words. */
int slamgpu_vocab_info(const slamgpu_vocab* v, int32_t* info);
/* The node arrays back (n_nodes entries each; any pointer may be NULL). */
int slamgpu_vocab_nodes(const slamgpu_vocab* v, int32_t* parent, uint8_t* leaf, uint8_t* desc,
                        double* weight);

/* Replaces TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
 * (TemplatedVocabulary.h:1123-1191) for one set of n descriptors (n x 32 bytes). BowVector:
 * words[*n_words] ascending with their values; FeatureVector: nodes[*n_nodes] ascending, node i's
 * features node_feats[node_start[i] .. node_start[i + 1]) ascending. Buffers hold n entries
 * (node_start n + 1). */
int slamgpu_bow_transform(slamgpu_vocab* v, const uint8_t* desc, int n, int levelsup,
                          uint32_t* words, double* values, int* n_words, uint32_t* nodes,
                          int32_t* node_start, uint32_t* node_feats, int* n_nodes);

/* Batched device outputs: set s's arrays start at s * cap (node_start at s * (cap + 1)). */
typedef struct {
  uint32_t* words;      /* [n_sets][cap] BowVector word ids                               */
  double* values;       /* [n_sets][cap] BowVector values                                 */
  int32_t* n_words;     /* [n_sets]                                                       */
  uint32_t* nodes;      /* [n_sets][cap] FeatureVector node ids                           */
  int32_t* node_start;  /* [n_sets][cap + 1]                                              */
  uint32_t* node_feats; /* [n_sets][cap]                                                  */
  int32_t* n_nodes;     /* [n_sets]                                                       */
  uint32_t* feat_leaf;  /* [n_sets][cap] per feature: the node its descent ends at        */
  uint32_t* feat_node;  /* [n_sets][cap] per feature: its node at level L - levelsup      */
  int32_t cap;          /* >= every set's count (larger counts are cut), <= 4096          */
  int32_t pad;
} slamgpu_bow_sets;

/* Set s = the d_counts[s * count_step] descriptors at d_desc + s * set_stride * 32 (with the
 * frontend's slamgpu_device_view: desc with set_stride = 2 * kp_cap and nkps with
 * count_step = 2 select the left views). */
int slamgpu_bow_transform_device(slamgpu_vocab* v, const uint8_t* d_desc, int64_t set_stride,
                                 const int32_t* d_counts, int count_step, int n_sets,
                                 int levelsup, const slamgpu_bow_sets* out, void* stream);

/* ---- SearchByBoW -------------------------------------------------------------------------- */
/* One side of a SearchByBoW call (host pointers). A = the keyframe whose features are iterated
 * (pKF / pKF1), B = the other view (F / pKF2). valid[i]: feature i's map point exists and is not
 * bad (NULL = every feature is a candidate). */
typedef struct {
  const uint8_t* desc;           /* [n][32]                                  */
  const slamgpu_keypoint* kps;   /* [n] undistorted keypoints (angle used)   */
  const uint8_t* valid;          /* [n] or NULL                              */
  const uint32_t* nodes;         /* FeatureVector: [n_nodes] ascending       */
  const int32_t* node_start;     /* [n_nodes + 1]                            */
  const uint32_t* node_feats;    /* [node_start[n_nodes]]                    */
  int32_t n;
  int32_t n_nodes;
} slamgpu_bow_set;

/* kf_kf = 0: SearchByBoW(KeyFrame* a, Frame& b) -- accept bestDist1 <= TH_LOW, b->valid ignored;
 * kf_kf = 1: SearchByBoW(KeyFrame* a, KeyFrame* b) -- accept bestDist1 < TH_LOW, B candidates
 * need b->valid. match_a[i] = B feature matched to A feature i, or -1 (Frame overload:
 * vpMapPointMatches[match_a[i]] = a's map point i; KF-KF: vpMatches12[i] = b's map point
 * match_a[i]). *nmatches = the reference's return value. */
int slamgpu_search_by_bow(const slamgpu_bow_set* a, const slamgpu_bow_set* b, int kf_kf,
                          float nnratio, int check_ori, int32_t* match_a, int* nmatches);

/* Device twin of slamgpu_bow_set; the counts are device pointers so that views can point at
 * slamgpu_bow_transform_device outputs without a round trip. */
typedef struct {
  const uint8_t* desc;
  const slamgpu_keypoint* kps;
  const uint8_t* valid;
  const int32_t* n;
  const uint32_t* nodes;
  const int32_t* node_start;
  const uint32_t* node_feats;
  const int32_t* n_nodes;
} slamgpu_bow_view;

/* n_pairs independent calls: A = d_a[p], B = d_b[p] (arrays of views in device memory), match of
 * pair p at d_match + p * match_stride, d_nmatches[p] (-1 if a set exceeds 4096 features). B's
 * valid pointer is used as given (NULL for the Frame overload). */
int slamgpu_search_by_bow_device(const slamgpu_bow_view* d_a, const slamgpu_bow_view* d_b,
                                 int n_pairs, int kf_kf, float nnratio, int check_ori,
                                 int32_t* d_match, int64_t match_stride, int32_t* d_nmatches,
                                 void* stream);

/* ---- MapPoint::ComputeDistinctiveDescriptors ----------------------------------------------- */
/* Map point p's observed descriptors (observation-map order, bad keyframes dropped) are
 * desc[start[p] .. start[p + 1]) (< 65536 each). best[p] = index relative to start[p] of the
 * descriptor with the least median distance to the others (first wins ties), -1 for none;
 * desc_out[p] (optional) = that descriptor (left untouched for none). */
int slamgpu_distinctive_descriptors(const uint8_t* desc, const int32_t* start, int n_points,
                                    int32_t* best, uint8_t* desc_out);
int slamgpu_distinctive_descriptors_device(const uint8_t* d_desc, const int32_t* d_start,
                                           int n_points, int32_t* d_best, uint8_t* d_desc_out,
                                           void* stream);

/* ---- ingest: colour -> gray ------------------------------------------------------------------ */
/* cv::cvtColor as Tracker::GrabImageStereo applies it (tracker.cpp:110-127): channels 3 or 4;
 * rgb != 0 -> CV_RGB2GRAY / CV_RGBA2GRAY (byte 0 weighted as red), rgb == 0 -> CV_BGR2GRAY /
 * CV_BGRA2GRAY. KITTI runs with is_rgb = true on BGR-decoded PNGs. */
int slamgpu_gray(const uint8_t* src, size_t src_pitch, int channels, int rgb, int cols, int rows,
                 uint8_t* dst, size_t dst_pitch);
/* n_images images: image i at d_src + i * src_stride (rows src_pitch bytes apart) into
 * d_dst + i * dst_stride (dst_pitch). */
int slamgpu_gray_device(const uint8_t* d_src, size_t src_pitch, size_t src_stride, int channels,
                        int rgb, int cols, int rows, int n_images, uint8_t* d_dst,
                        size_t dst_pitch, size_t dst_stride, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_BOW_H_ */
