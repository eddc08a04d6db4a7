// bow_kernels.hip -- bag-of-words and keyframe-rate matchers on gfx950, batched.
//
//   bow_descend   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
//                 (third_party/DBoW2/DBoW2/TemplatedVocabulary.h:1214-1256): one 16-lane row per
//                 descriptor, one child per lane per level. The children of a node are contiguous
//                 slots (file order), so a level is one coalesced read of k x 32 bytes; the first
//                 minimum (strict '<' in child order, :1241) is the row minimum of
//                 (distance << 16 | child position).
//   bow_vectors   transform(features, BowVector, FeatureVector, levelsup) (:1123-1191) with
//                 BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84) and
//                 FeatureVector::addFeature (FeatureVector.cpp:31-44): one workgroup per set,
//                 (word, feature) and (node, feature) keys bitonic-sorted in LDS, per-word sums in
//                 feature order and the norm summed serially in word order -- the reference's
//                 floating-point order, so the values are bit-identical.
//   search_bow    OrbMatcher::SearchByBoW, both overloads (src/orb_features/orb_matcher.cpp:
//                 133-262, 499-632): one workgroup per (A, B) pair, a wave per common node. A claim
//                 (vpMapPointMatches / vbMatched2) can only block a candidate of the same node, so
//                 nodes are independent; inside a node the A features run in order and the B
//                 candidates across lanes. The rotation histogram only counts, so its order is free.
//   distinctive   MapPoint::ComputeDistinctiveDescriptors (src/data/map_point.cpp:249-304): a wave
//                 per map point, a lane per row of the distance matrix; nth_element's median is the
//                 smallest d with #(row <= d) > (n - 1) / 2, found by bisection over [0, 256].
//   gray          cv::cvtColor(*2GRAY, 8U) as Tracker::GrabImageStereo applies it
//                 (tracker.cpp:110-127): OpenCV 3.3.1 RGB2Gray<uchar> fixed-point weights.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bow_kernels.h"
#include "device_math.h"
#include "timing.h"

namespace slamgpu {

namespace {

constexpr int kThLow = 50, kHisto = 30;  // OrbMatcher TH_LOW, HISTO_LENGTH (orb_matcher.cpp:5-7)

__device__ __forceinline__ int hamming_q(const uint4& a0, const uint4& a1, const uint4& b0,
                                         const uint4& b1) {
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ void load_desc(const uint8_t* p, uint4* d0, uint4* d1) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  *d0 = q[0];
  *d1 = q[1];
}

// ---------------------------------------------------------------------------------------
constexpr int kDescPerBlock = 16;  // 256 threads = 16 rows of 16 lanes

__global__ __launch_bounds__(256) void bow_descend_kernel(VocabDev v,
                                                          const uint8_t* __restrict__ desc,
                                                          int64_t set_stride,
                                                          const int32_t* __restrict__ counts,
                                                          int count_step, BowSets o) {
  const int set = blockIdx.y;
  const int f = blockIdx.x * kDescPerBlock + (int)(threadIdx.x >> 4);
  const uint32_t l16 = threadIdx.x & 15;
  const int n = min(counts[(int64_t)set * count_step], o.cap);
  if (f >= n) return;  // the whole row leaves together
  uint4 x0, x1;
  load_desc(desc + ((int64_t)set * set_stride + f) * 32, &x0, &x1);
  uint32_t first = v.root_first, cnt = v.root_count, node = 0, nid = 0;
  int level = 0;
  for (;;) {
    ++level;
    uint32_t best = 0xffffffffu;
    for (uint32_t c0 = 0; c0 < cnt; c0 += 16) {
      const uint32_t c = c0 + l16;
      if (c < cnt) {
        const uint4* s = v.slot_desc + 2 * (size_t)(first + c);
        best = min(best, (uint32_t)hamming_q(x0, x1, s[0], s[1]) << 16 | c);
      }
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1)
      best = min(best, (uint32_t)__shfl_xor((int)best, off, 16));
    const VocabSlot s = v.slot[first + (best & 0xffffu)];
    node = s.node;
    if (level == v.nid_level) nid = node;
    if (s.count == 0) break;
    first = s.first;
    cnt = s.count;
  }
  if (v.nid_level > level) nid = node;  // declared: a leaf above the FeatureVector level
  if (l16 == 0) {
    const int64_t i = (int64_t)set * o.cap + f;
    o.feat_leaf[i] = node;
    o.feat_node[i] = nid;
  }
}

// ---------------------------------------------------------------------------------------
constexpr int kVecThreads = 1024;
constexpr int kVecPer = kBowMaxFeatures / kVecThreads;  // consecutive keys per thread

__device__ void lds_bitonic(uint64_t* a, int P) {
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kVecThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t x = a[i], y = a[ixj];
          if ((x > y) == ((i & k) == 0)) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
}

// Exclusive prefix of one int per thread over the workgroup; *total = the sum.
__device__ int block_scan(int x, int* s_w, int* total) {
  const int lane = lane_id(), wid = wave_id();
  int inc = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < kVecThreads / 64; w++) {
    const int s = s_w[w];
    if (w < wid) base += s;
    tot += s;
  }
  *total = tot;
  __syncthreads();  // s_w is reused by the next call
  return base + inc - x;
}

__global__ __launch_bounds__(kVecThreads) void bow_vectors_kernel(VocabDev v,
                                                                  const int32_t* __restrict__ counts,
                                                                  int count_step, BowSets o) {
  __shared__ uint64_t s_key[kBowMaxFeatures];
  __shared__ double s_val[kBowMaxFeatures];
  __shared__ int s_w[kVecThreads / 64];
  __shared__ int s_m;
  __shared__ double s_norm;
  const int set = blockIdx.x, tid = threadIdx.x;
  const int n = v.empty ? 0 : min(counts[(int64_t)set * count_step], o.cap);
  const int64_t base = (int64_t)set * o.cap;
  int32_t* nstart = o.node_start + (int64_t)set * (o.cap + 1);
  int P = 2;
  while (P < n) P <<= 1;
  // pass 0: BowVector from (word, feature) keys; pass 1: FeatureVector from (node, feature) keys.
  // Stopped words (weight <= 0, :1154) take part in neither.
  for (int pass = 0; pass < 2; pass++) {
    if (tid == 0) s_m = 0;
    for (int i = tid; i < P; i += kVecThreads) {
      uint64_t k = ~0ull;
      if (i < n) {
        const uint32_t leaf = o.feat_leaf[base + i];
        if (v.node_weight[leaf] > 0)
          k = (uint64_t)(pass == 0 ? v.node_word[leaf] : o.feat_node[base + i]) << 32 |
              (uint32_t)i;
      }
      s_key[i] = k;
    }
    __syncthreads();
    lds_bitonic(s_key, P);
    for (int i = tid; i < P; i += kVecThreads)
      if (s_key[i] != ~0ull && (i + 1 == P || s_key[i + 1] == ~0ull)) s_m = i + 1;
    __syncthreads();
    const int m = s_m;
    int heads = 0;
#pragma unroll
    for (int j = 0; j < kVecPer; j++) {
      const int i = kVecPer * tid + j;
      if (i < m && (i == 0 || (s_key[i] >> 32) != (s_key[i - 1] >> 32))) heads++;
    }
    int total;
    int u = block_scan(heads, s_w, &total);
    for (int j = 0; j < kVecPer; j++) {
      const int i = kVecPer * tid + j;
      if (i >= m) break;
      const uint32_t key = (uint32_t)(s_key[i] >> 32);
      if (pass == 1) o.node_feats[base + i] = (uint32_t)s_key[i];
      if (i > 0 && (uint32_t)(s_key[i - 1] >> 32) == key) continue;
      if (pass == 0) {
        double w = v.node_weight[o.feat_leaf[base + (uint32_t)s_key[i]]];
        if (v.tf)  // addWeight: += in feature order (BowVector.cpp:40); else addIfNotExist
          for (int r = i + 1; r < m && (uint32_t)(s_key[r] >> 32) == key; r++)
            w += v.node_weight[o.feat_leaf[base + (uint32_t)s_key[r]]];
        o.words[base + u] = key;
        s_val[u] = w;
      } else {
        o.nodes[base + u] = key;
        nstart[u] = i;
      }
      u++;
    }
    if (pass == 0) {
      __syncthreads();
      const int nw = total;
      if (tid == 0) {
        double norm = 0.0;
        if (v.must) {  // BowVector::normalize (BowVector.cpp:62-84), serially in word order
          if (v.l2) {
            for (int i = 0; i < nw; i++) norm = fma(s_val[i], s_val[i], norm);
            norm = sqrt(norm);
          } else {
            for (int i = 0; i < nw; i++) norm += fabs(s_val[i]);
          }
        } else {
          norm = (double)nw;  // TF / TF_IDF without normalisation: / v.size() (:1161-1167)
        }
        s_norm = norm;
        o.n_words[set] = nw;
      }
      __syncthreads();
      const double norm = s_norm;
      const bool divide = v.must ? norm > 0.0 : (v.tf != 0);
      for (int i = tid; i < nw; i += kVecThreads) {
        double x = s_val[i];
        if (divide) x /= norm;
        o.values[base + i] = x;
      }
    } else if (tid == 0) {
      nstart[total] = m;
      o.n_nodes[set] = total;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
constexpr int kSbWaves = 4;

__global__ __launch_bounds__(64 * kSbWaves) void search_bow_kernel(
    const BowView* __restrict__ av, const BowView* __restrict__ bv, int strict_lt, float nnratio,
    int check_ori, int32_t* __restrict__ match, int64_t match_stride,
    int32_t* __restrict__ nmatches) {
  __shared__ int8_t s_bin[kBowMaxFeatures];
  __shared__ int s_hist[kHisto];
  __shared__ int s_acc[kSbWaves];
  __shared__ int s_rem[kSbWaves];
  __shared__ int s_ind[3];
  const int pair = blockIdx.x;
  const BowView A = av[pair], B = bv[pair];
  const int na = *A.n, nb = *B.n, ann = *A.n_nodes, bnn = *B.n_nodes;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  if (na > kBowMaxFeatures || nb > kBowMaxFeatures || na < 0 || nb < 0) {
    if (tid == 0) nmatches[pair] = -1;
    return;
  }
  int32_t* out = match + (int64_t)pair * match_stride;
  for (int i = tid; i < na; i += 64 * kSbWaves) {
    out[i] = -1;
    s_bin[i] = -1;
  }
  if (tid < kHisto) s_hist[tid] = 0;
  __syncthreads();
  int acc = 0;
  for (int ia = wid; ia < ann; ia += kSbWaves) {
    const uint32_t key = A.nodes[ia];
    int lo = 0, hi = bnn;  // the same node in B's FeatureVector (the merge of :154-238)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (B.nodes[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    if (lo >= bnn || B.nodes[lo] != key) continue;
    const int b0 = B.node_start[lo], nbn = min(B.node_start[lo + 1] - b0, 64 * 64);
    uint64_t taken = 0;  // bit c: this lane's candidate b0 + 64 c + lane is claimed
    for (int p = A.node_start[ia]; p < A.node_start[ia + 1]; p++) {
      const int fa = (int)A.node_feats[p];
      if (A.valid && !A.valid[fa]) continue;
      uint4 x0, x1;
      load_desc(A.desc + (int64_t)fa * 32, &x0, &x1);
      // this lane's best (distance << 16 | position) and second-best distance
      uint32_t m1 = 0xffffffffu, m2 = 256;
      for (int c = 0; c * 64 < nbn; c++) {
        const int pos = c * 64 + lane;
        if (pos < nbn && !((taken >> c) & 1)) {
          const int fb = (int)B.node_feats[b0 + pos];
          if (!B.valid || B.valid[fb]) {
            uint4 y0, y1;
            load_desc(B.desc + (int64_t)fb * 32, &y0, &y1);
            const uint32_t d = (uint32_t)hamming_q(x0, x1, y0, y1);
            const uint32_t k = d << 16 | (uint32_t)pos;
            if (k < m1) {
              if (m1 != 0xffffffffu) m2 = min(m2, m1 >> 16);
              m1 = k;
            } else {
              m2 = min(m2, d);
            }
          }
        }
      }
      // bestDist1 / bestIdx: the first strict minimum in node order; bestDist2: the second
      // smallest distance of the multiset (:190-199)
      const uint32_t g1 = wave_min(m1);
      if (g1 == 0xffffffffu) continue;
      const uint32_t best1 = g1 >> 16;
      const uint32_t best2 = wave_min(m1 == g1 ? m2 : (m1 == 0xffffffffu ? 256u : m1 >> 16));
      const bool pass = strict_lt ? best1 < (uint32_t)kThLow : best1 <= (uint32_t)kThLow;
      if (pass && (float)best1 < nnratio * (float)best2) {
        const int pos = (int)(g1 & 0xffffu);
        if (lane == (pos & 63)) taken |= 1ull << (pos >> 6);
        if (lane == 0) {
          const int fb = (int)B.node_feats[b0 + pos];
          out[fa] = fb;
          if (check_ori) {
            float rot = A.kps[fa].angle - B.kps[fb].angle;
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * (1.0f / kHisto));
            if (bin == kHisto) bin = 0;
            s_bin[fa] = (int8_t)bin;
            atomicAdd(&s_hist[bin], 1);
          }
        }
        acc++;
      }
    }
  }
  if (lane == 0) s_acc[wid] = acc;
  __syncthreads();
  if (tid == 0) {  // ComputeThreeMaxima (orb_matcher.cpp:1584-1625)
    int max1 = 0, max2 = 0, max3 = 0, i1 = -1, i2 = -1, i3 = -1;
    for (int i = 0; i < kHisto; i++) {
      const int s = s_hist[i];
      if (s > max1) {
        max3 = max2; max2 = max1; max1 = s;
        i3 = i2; i2 = i1; i1 = i;
      } else if (s > max2) {
        max3 = max2; max2 = s;
        i3 = i2; i2 = i;
      } else if (s > max3) {
        max3 = s;
        i3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) {
      i2 = -1;
      i3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
      i3 = -1;
    }
    s_ind[0] = i1;
    s_ind[1] = i2;
    s_ind[2] = i3;
  }
  __syncthreads();
  int removed = 0;
  if (check_ori) {
    const int i1 = s_ind[0], i2 = s_ind[1], i3 = s_ind[2];
    for (int i = tid; i < na; i += 64 * kSbWaves) {
      const int bin = s_bin[i];
      if (bin >= 0 && bin != i1 && bin != i2 && bin != i3) {
        out[i] = -1;
        removed++;
      }
    }
  }
  removed = wave_sum(removed);
  if (lane == 0) s_rem[wid] = removed;
  __syncthreads();
  if (tid == 0) {
    int nm = 0;
    for (int w = 0; w < kSbWaves; w++) nm += s_acc[w] - s_rem[w];
    nmatches[pair] = nm;
  }
}

// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void distinctive_kernel(const uint8_t* __restrict__ desc,
                                                          const int32_t* __restrict__ start,
                                                          int n_points, int32_t* __restrict__ best,
                                                          uint8_t* __restrict__ desc_out) {
  const int p = blockIdx.x * 4 + wave_id();
  if (p >= n_points) return;
  const int lane = lane_id();
  const int s = start[p], n = start[p + 1] - s;
  if (n <= 0) {
    if (lane == 0) best[p] = -1;
    return;
  }
  const int half = (int)(0.5 * (double)(n - 1));  // map_point.cpp:289
  const uint8_t* D = desc + (int64_t)s * 32;
  uint32_t bk = 0xffffffffu;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    if (i < n) {
      uint4 x0, x1;
      load_desc(D + (int64_t)i * 32, &x0, &x1);
      int lo = 0, hi = 256;  // the half-th smallest of row i (0 on the diagonal)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        int cnt = 0;
        for (int j = 0; j < n; j++) {
          uint4 y0, y1;
          load_desc(D + (int64_t)j * 32, &y0, &y1);
          cnt += (j == i ? 0 : hamming_q(x0, x1, y0, y1)) <= mid;
        }
        if (cnt > half) hi = mid;
        else lo = mid + 1;
      }
      bk = min(bk, (uint32_t)lo << 16 | (uint32_t)i);  // strict '<' over rows in order (:294)
    }
  }
  bk = wave_min(bk);
  const int bi = (int)(bk & 0xffffu);
  if (lane == 0) best[p] = bi;
  if (desc_out && lane < 8)
    reinterpret_cast<uint32_t*>(desc_out + (int64_t)p * 32)[lane] =
        reinterpret_cast<const uint32_t*>(D + (int64_t)bi * 32)[lane];
}

// ---------------------------------------------------------------------------------------
// A thread converts 4 pixels of one row. Y = (s0 c0 + s1 9617 + s2 c2 + 8192) >> 14 with
// (c0, c2) = (4899, 1868) for the RGB orders and (1868, 4899) for BGR (R2Y, G2Y, B2Y, yuv_shift 14).
__global__ __launch_bounds__(256) void gray_kernel(const uint8_t* __restrict__ src, size_t spitch,
                                                   size_t sstride, int cn, uint32_t c0,
                                                   uint32_t c2, int cols, int rows,
                                                   uint8_t* __restrict__ dst, size_t dpitch,
                                                   size_t dstride) {
  const int img = blockIdx.z, y = blockIdx.y;
  const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (x0 >= cols) return;
  const uint8_t* s = src + (int64_t)img * sstride + (int64_t)y * spitch + (int64_t)x0 * cn;
  uint8_t* d = dst + (int64_t)img * dstride + (int64_t)y * dpitch + x0;
  const int nx = min(4, cols - x0);
  uint32_t w[5] = {0, 0, 0, 0, 0};
  // dword path: the 4 aligned dwords around 12 (16) bytes, cut with alignbyte; never past the
  // image's last byte (that group takes the byte path)
  const bool vec = nx == 4 && !(y == rows - 1 && x0 + 4 >= cols);
  if (vec) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(s);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t r[5];
    const int nd = cn + (sh ? 1 : 0);  // dwords covering [s, s + 4 cn)
#pragma unroll
    for (int i = 0; i < 5; i++) r[i] = i < nd ? sw[i] : 0u;
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
  } else {
    for (int b = 0; b < nx * cn; b++) w[b >> 2] |= (uint32_t)s[b] << (8 * (b & 3));
  }
  auto byte = [&](int b) { return (w[b >> 2] >> (8 * (b & 3))) & 0xffu; };
  uint32_t out = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k < nx) {
      const uint32_t v = (byte(k * cn) * c0 + byte(k * cn + 1) * 9617u + byte(k * cn + 2) * c2 +
                          8192u) >> 14;
      out |= v << (8 * k);
    }
  }
  if (nx == 4 && (reinterpret_cast<uintptr_t>(d) & 3) == 0) {
    *reinterpret_cast<uint32_t*>(d) = out;
  } else {
    for (int k = 0; k < nx; k++) d[k] = (uint8_t)(out >> (8 * k));
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------
hipError_t launch_bow_transform(const VocabDev& v, const uint8_t* desc, int64_t set_stride,
                                const int32_t* counts, int count_step, int n_sets,
                                const BowSets& o, hipStream_t st) {
  if (n_sets <= 0) return hipSuccess;
  if (!v.empty)
    SLAMGPU_LAUNCH("bow_descend", st, bow_descend_kernel,
                   dim3((o.cap + kDescPerBlock - 1) / kDescPerBlock, n_sets), dim3(256), 0, st, v,
                   desc, set_stride, counts, count_step, o);
  SLAMGPU_LAUNCH("bow_vectors", st, bow_vectors_kernel, dim3(n_sets), dim3(kVecThreads), 0, st, v,
                 counts, count_step, o);
  return hipGetLastError();
}

hipError_t launch_search_bow(const BowView* a, const BowView* b, int n_pairs, int strict_lt,
                             float nnratio, int check_ori, int32_t* match, int64_t match_stride,
                             int32_t* nmatches, hipStream_t st) {
  if (n_pairs <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("search_bow", st, search_bow_kernel, dim3(n_pairs), dim3(64 * kSbWaves), 0, st, a,
                 b, strict_lt, nnratio, check_ori, match, match_stride, nmatches);
  return hipGetLastError();
}

hipError_t launch_distinctive(const uint8_t* desc, const int32_t* start, int n_points,
                              int32_t* best, uint8_t* desc_out, hipStream_t st) {
  if (n_points <= 0) return hipSuccess;
  SLAMGPU_LAUNCH("distinctive", st, distinctive_kernel, dim3((n_points + 3) / 4), dim3(256), 0, st,
                 desc, start, n_points, best, desc_out);
  return hipGetLastError();
}

hipError_t launch_gray(const uint8_t* src, size_t spitch, size_t sstride, int cn, int rgb,
                       int cols, int rows, int n_images, uint8_t* dst, size_t dpitch,
                       size_t dstride, hipStream_t st) {
  if (n_images <= 0 || cols <= 0 || rows <= 0) return hipSuccess;
  const uint32_t c0 = rgb ? 4899u : 1868u, c2 = rgb ? 1868u : 4899u;
  SLAMGPU_LAUNCH("gray", st, gray_kernel, dim3((cols + 1023) / 1024, rows, n_images), dim3(256), 0,
                 st, src, spitch, sstride, cn, c0, c2, cols, rows, dst, dpitch, dstride);
  return hipGetLastError();
}

}  // namespace slamgpu
