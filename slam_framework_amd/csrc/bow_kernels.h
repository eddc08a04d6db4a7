// bow_kernels.h -- device layouts and launchers of the bag-of-words / keyframe-rate matchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_kernels.h"  // KeyPoint

namespace slamgpu {

constexpr int kBowMaxFeatures = 4096;  // == SLAMGPU_BOW_MAX_FEATURES

// The children of a vocabulary node are contiguous slots, in file order. A slot holds the child's
// node id and where the child's own children start / how many there are (0 = a leaf).
struct VocabSlot {
  uint32_t node, first, count, pad;
};

struct VocabDev {
  const uint4* slot_desc;     // [n_slots][2]: the slot node's 32-byte descriptor
  const VocabSlot* slot;      // [n_slots]
  const uint32_t* node_word;  // [n_nodes] word id (0 for nodes without the leaf flag)
  const double* node_weight;  // [n_nodes]
  uint32_t root_first, root_count;
  int nid_level;              // L - levelsup
  int empty;                  // no words: transform returns empty vectors
  int must, l2, tf;           // mustNormalize, L2 norm, TF / TF_IDF accumulation
};

struct BowSets {
  uint32_t* words;
  double* values;
  int32_t* n_words;
  uint32_t* nodes;
  int32_t* node_start;
  uint32_t* node_feats;
  int32_t* n_nodes;
  uint32_t* feat_leaf;
  uint32_t* feat_node;
  int32_t cap;
};

// == slamgpu_bow_view (include/slamgpu_bow.h)
struct BowView {
  const uint8_t* desc;
  const KeyPoint* kps;
  const uint8_t* valid;
  const int32_t* n;
  const uint32_t* nodes;
  const int32_t* node_start;
  const uint32_t* node_feats;
  const int32_t* n_nodes;
};

hipError_t launch_bow_transform(const VocabDev& v, const uint8_t* desc, int64_t set_stride,
                                const int32_t* counts, int count_step, int n_sets,
                                const BowSets& o, hipStream_t st);
hipError_t launch_search_bow(const BowView* a, const BowView* b, int n_pairs, int strict_lt,
                             float nnratio, int check_ori, int32_t* match, int64_t match_stride,
                             int32_t* nmatches, hipStream_t st);
hipError_t launch_distinctive(const uint8_t* desc, const int32_t* start, int n_points,
                              int32_t* best, uint8_t* desc_out, hipStream_t st);
hipError_t launch_gray(const uint8_t* src, size_t spitch, size_t sstride, int cn, int rgb,
                       int cols, int rows, int n_images, uint8_t* dst, size_t dpitch,
                       size_t dstride, hipStream_t st);

}  // namespace slamgpu
