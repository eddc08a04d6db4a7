// bow_runtime.cpp -- host side of include/slamgpu_bow.h: vocabulary loading and its device
// layout, the synchronous per-frame calls (staged through device buffers owned by the vocabulary
// or by the calling thread) and the batched *_device calls (validate, launch on the caller's
// stream, never allocate).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/slamgpu_bow.h"
#include "bow_kernels.h"

using namespace slamgpu;

static_assert(sizeof(slamgpu_bow_view) == sizeof(BowView), "slamgpu_bow_view layout");
static_assert(sizeof(slamgpu_keypoint) == sizeof(KeyPoint), "keypoint layout");

struct slamgpu_vocab {
  int device = 0;
  int k = 0, L = 0, scoring = 0, weighting = 0, n_words = 0;
  std::vector<int32_t> parent;
  std::vector<uint8_t> leaf, desc;
  std::vector<double> weight;
  uint4* d_slot_desc = nullptr;
  VocabSlot* d_slot = nullptr;
  uint32_t* d_node_word = nullptr;
  double* d_node_weight = nullptr;
  uint32_t root_first = 0, root_count = 0;
  hipStream_t stream = nullptr;
  char* stage = nullptr;  // slamgpu_bow_transform's staging buffer (grown on demand)
  size_t stage_bytes = 0;
};

namespace {

thread_local std::string t_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

#define BOW_HIPCHECK(x)                                                                 \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(SLAMGPU_EHIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

void release(slamgpu_vocab* v) {
  if (!v) return;
  (void)hipSetDevice(v->device);
  if (v->d_slot_desc) (void)hipFree(v->d_slot_desc);
  if (v->d_slot) (void)hipFree(v->d_slot);
  if (v->d_node_word) (void)hipFree(v->d_node_word);
  if (v->d_node_weight) (void)hipFree(v->d_node_weight);
  if (v->stage) (void)hipFree(v->stage);
  if (v->stream) (void)hipStreamDestroy(v->stream);
  delete v;
}

// Device layout: the children of every node, in file order, are contiguous slots (slot s = entry
// s of the parent-grouped child list), so one descent level reads one contiguous run of slots.
int upload(slamgpu_vocab* v) {
  const int n = (int)v->parent.size();
  std::vector<int32_t> cstart(n + 1, 0), child(n > 1 ? n - 1 : 1, 0);
  for (int i = 1; i < n; i++) cstart[v->parent[i] + 1]++;
  for (int i = 0; i < n; i++) cstart[i + 1] += cstart[i];
  std::vector<int32_t> fill(cstart.begin(), cstart.end() - 1);
  for (int i = 1; i < n; i++) child[fill[v->parent[i]]++] = i;
  const int ns = n > 1 ? n - 1 : 1;
  std::vector<uint8_t> sdesc((size_t)ns * 32, 0);
  std::vector<VocabSlot> slot(ns, VocabSlot{0, 0, 0, 0});
  for (int s = 0; s < n - 1; s++) {
    const int node = child[s];
    std::memcpy(&sdesc[(size_t)s * 32], &v->desc[(size_t)node * 32], 32);
    const int cnt = cstart[node + 1] - cstart[node];
    if (cnt > 0xffff) return fail(SLAMGPU_EINVAL, "node %d has %d children (max 65535)", node, cnt);
    slot[s] = VocabSlot{(uint32_t)node, (uint32_t)cstart[node], (uint32_t)cnt, 0u};
  }
  if (cstart[1] > 0xffff) return fail(SLAMGPU_EINVAL, "the root has %d children (max 65535)", cstart[1]);
  v->root_first = 0;
  v->root_count = (uint32_t)cstart[1];
  std::vector<uint32_t> word(n, 0);
  int words = 0;
  for (int i = 1; i < n; i++)
    if (v->leaf[i]) word[i] = (uint32_t)words++;  // TemplatedVocabulary.h:1405-1412
  v->n_words = words;
  BOW_HIPCHECK(hipSetDevice(v->device));
  BOW_HIPCHECK(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
  BOW_HIPCHECK(hipMalloc(&v->d_slot_desc, sdesc.size()));
  BOW_HIPCHECK(hipMalloc(&v->d_slot, sizeof(VocabSlot) * slot.size()));
  BOW_HIPCHECK(hipMalloc(&v->d_node_word, sizeof(uint32_t) * n));
  BOW_HIPCHECK(hipMalloc(&v->d_node_weight, sizeof(double) * n));
  BOW_HIPCHECK(hipMemcpy(v->d_slot_desc, sdesc.data(), sdesc.size(), hipMemcpyHostToDevice));
  BOW_HIPCHECK(hipMemcpy(v->d_slot, slot.data(), sizeof(VocabSlot) * slot.size(),
                         hipMemcpyHostToDevice));
  BOW_HIPCHECK(hipMemcpy(v->d_node_word, word.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice));
  BOW_HIPCHECK(hipMemcpy(v->d_node_weight, v->weight.data(), sizeof(double) * n,
                         hipMemcpyHostToDevice));
  return 0;
}

VocabDev device_view(const slamgpu_vocab* v, int levelsup) {
  VocabDev d;
  d.slot_desc = v->d_slot_desc;
  d.slot = v->d_slot;
  d.node_word = v->d_node_word;
  d.node_weight = v->d_node_weight;
  d.root_first = v->root_first;
  d.root_count = v->root_count;
  d.nid_level = v->L - levelsup;
  d.empty = (v->n_words == 0 || v->root_count == 0) ? 1 : 0;  // empty() (:1131)
  d.must = v->scoring != SLAMGPU_DOT_PRODUCT;  // ScoringObject.h:74-89
  d.l2 = v->scoring == SLAMGPU_L2_NORM;
  d.tf = (v->weighting == SLAMGPU_TF_IDF || v->weighting == SLAMGPU_TF) ? 1 : 0;
  return d;
}

int check_header(int k, int L, int scoring, int weighting) {
  // loadFromTextFile's header check (TemplatedVocabulary.h:1356-1360)
  if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
      weighting > 3)
    return fail(SLAMGPU_EINVAL,
                "Vocabulary loading failure: not a correct vocabulary (k %d, L %d, scoring %d, "
                "weighting %d)", k, L, scoring, weighting);
  return 0;
}

slamgpu_vocab* new_vocab(int device, int k, int L, int scoring, int weighting) {
  slamgpu_vocab* v = new slamgpu_vocab();
  v->device = device;
  v->k = k;
  v->L = L;
  v->scoring = scoring;
  v->weighting = weighting;
  v->parent.assign(1, 0);  // node 0 = the root (:1373-1374)
  v->leaf.assign(1, 0);
  v->desc.assign(32, 0);
  v->weight.assign(1, 0.0);
  return v;
}

int finish(slamgpu_vocab* v, slamgpu_vocab** out) {
  if (int r = upload(v)) {
    release(v);
    return r;
  }
  *out = v;
  return 0;
}

// Per-thread staging of the synchronous SearchByBoW / distinctive / gray calls.
struct Stage {
  int device = -1;
  hipStream_t stream = nullptr;
  char* buf = nullptr;
  size_t bytes = 0;
  ~Stage() {
    if (buf) (void)hipFree(buf);
    if (stream) (void)hipStreamDestroy(stream);
  }
};
thread_local Stage t_stage;

int stage_reserve(Stage& S, size_t need) {
  int dev = 0;
  BOW_HIPCHECK(hipGetDevice(&dev));
  if (S.device != dev) {
    if (S.buf) (void)hipFree(S.buf);
    if (S.stream) (void)hipStreamDestroy(S.stream);
    S.buf = nullptr;
    S.stream = nullptr;
    S.bytes = 0;
    BOW_HIPCHECK(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
    S.device = dev;
  }
  if (need > S.bytes) {
    if (S.buf) BOW_HIPCHECK(hipFree(S.buf));
    S.buf = nullptr;
    S.bytes = 0;
    const size_t cap = need < (1u << 20) ? (1u << 20) : need;
    BOW_HIPCHECK(hipMalloc(&S.buf, cap));
    S.bytes = cap;
  }
  return 0;
}

// A host FeatureVector must be well formed before its indices reach the device.
int check_set(const slamgpu_bow_set* s, const char* name) {
  if (!s) return fail(SLAMGPU_EINVAL, "%s is NULL", name);
  if (s->n < 0 || s->n > SLAMGPU_BOW_MAX_FEATURES)
    return fail(SLAMGPU_EINVAL, "%s: n %d outside [0, %d]", name, s->n, SLAMGPU_BOW_MAX_FEATURES);
  if (s->n_nodes < 0 || s->n_nodes > s->n)
    return fail(SLAMGPU_EINVAL, "%s: n_nodes %d outside [0, n]", name, s->n_nodes);
  if (s->n > 0 && (!s->desc || !s->kps)) return fail(SLAMGPU_EINVAL, "%s: NULL desc/kps", name);
  if (s->n_nodes > 0 && (!s->nodes || !s->node_start || !s->node_feats))
    return fail(SLAMGPU_EINVAL, "%s: NULL FeatureVector", name);
  if (s->n_nodes > 0) {
    if (s->node_start[0] != 0) return fail(SLAMGPU_EINVAL, "%s: node_start[0] != 0", name);
    for (int i = 0; i < s->n_nodes; i++) {
      if (s->node_start[i + 1] < s->node_start[i] || s->node_start[i + 1] > s->n)
        return fail(SLAMGPU_EINVAL, "%s: node_start not ascending within [0, n]", name);
      if (i > 0 && s->nodes[i] <= s->nodes[i - 1])
        return fail(SLAMGPU_EINVAL, "%s: nodes not strictly ascending", name);
    }
    for (int j = 0; j < s->node_start[s->n_nodes]; j++)
      if (s->node_feats[j] >= (uint32_t)s->n)
        return fail(SLAMGPU_EINVAL, "%s: feature index %u >= n", name, s->node_feats[j]);
  }
  return 0;
}

}  // namespace

extern "C" {

const char* slamgpu_bow_last_error(void) { return t_err.c_str(); }

int slamgpu_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes,
                         const int32_t* parent, const uint8_t* leaf, const uint8_t* desc,
                         const double* weight, slamgpu_vocab** out) {
  if (!out) return fail(SLAMGPU_EINVAL, "out is NULL");
  *out = nullptr;
  if (int r = check_header(k, L, scoring, weighting)) return r;
  if (n_nodes < 1) return fail(SLAMGPU_EINVAL, "n_nodes %d < 1 (the root)", n_nodes);
  if (n_nodes > 1 && (!parent || !leaf || !desc || !weight))
    return fail(SLAMGPU_EINVAL, "NULL node array");
  for (int i = 1; i < n_nodes; i++)
    if (parent[i] < 0 || parent[i] >= i)
      return fail(SLAMGPU_EINVAL, "node %d: parent %d is not an earlier node", i, parent[i]);
  slamgpu_vocab* v = new_vocab(device, k, L, scoring, weighting);
  for (int i = 1; i < n_nodes; i++) {
    v->parent.push_back(parent[i]);
    v->leaf.push_back(leaf[i] ? 1 : 0);
    v->desc.insert(v->desc.end(), desc + (size_t)i * 32, desc + (size_t)i * 32 + 32);
    v->weight.push_back(weight[i]);
  }
  return finish(v, out);
}

int slamgpu_vocab_load_text(int device, const char* path, slamgpu_vocab** out) {
  if (!out || !path) return fail(SLAMGPU_EINVAL, "NULL argument");
  *out = nullptr;
  std::ifstream f(path);
  if (!f.is_open()) return fail(SLAMGPU_EINVAL, "cannot open %s", path);
  std::string s;
  std::getline(f, s);
  std::stringstream ss(s);
  int k = -1, L = -1, n1 = -1, n2 = -1;
  ss >> k >> L >> n1 >> n2;
  if (int r = check_header(k, L, n1, n2)) return r;
  slamgpu_vocab* v = new_vocab(device, k, L, n1, n2);
  std::string line;
  while (std::getline(f, line)) {
    if (line.find_first_not_of(" \t\r") == std::string::npos) continue;  // declared: no node
    std::stringstream ls(line);
    int pid = 0, is_leaf = 0;
    ls >> pid >> is_leaf;
    // the 32 descriptor fields are read as strings and re-parsed (F::fromString, FORB.cpp:120)
    std::stringstream ssd;
    for (int i = 0; i < 32; i++) {
      std::string e;
      ls >> e;
      ssd << e << " ";
    }
    uint8_t d[32] = {0};
    for (int i = 0; i < 32; i++) {
      int x = 0;
      ssd >> x;
      if (!ssd.fail()) d[i] = (uint8_t)x;
    }
    double w = 0.0;
    ls >> w;
    const int nid = (int)v->parent.size();
    if (pid < 0 || pid >= nid) {
      release(v);
      return fail(SLAMGPU_EINVAL, "%s: node %d names parent %d", path, nid, pid);
    }
    v->parent.push_back(pid);
    v->leaf.push_back(is_leaf > 0 ? 1 : 0);
    v->desc.insert(v->desc.end(), d, d + 32);
    v->weight.push_back(w);
  }
  return finish(v, out);
}

void slamgpu_vocab_destroy(slamgpu_vocab* v) { release(v); }

int slamgpu_vocab_info(const slamgpu_vocab* v, int32_t* info) {
  if (!v || !info) return fail(SLAMGPU_EINVAL, "NULL argument");
  info[0] = v->k;
  info[1] = v->L;
  info[2] = v->scoring;
  info[3] = v->weighting;
  info[4] = (int32_t)v->parent.size();
  info[5] = v->n_words;
  return 0;
}

int slamgpu_vocab_nodes(const slamgpu_vocab* v, int32_t* parent, uint8_t* leaf, uint8_t* desc,
                        double* weight) {
  if (!v) return fail(SLAMGPU_EINVAL, "NULL vocabulary");
  const size_t n = v->parent.size();
  if (parent) std::memcpy(parent, v->parent.data(), n * sizeof(int32_t));
  if (leaf) std::memcpy(leaf, v->leaf.data(), n);
  if (desc) std::memcpy(desc, v->desc.data(), n * 32);
  if (weight) std::memcpy(weight, v->weight.data(), n * sizeof(double));
  return 0;
}

int slamgpu_bow_transform_device(slamgpu_vocab* v, const uint8_t* d_desc, int64_t set_stride,
                                 const int32_t* d_counts, int count_step, int n_sets,
                                 int levelsup, const slamgpu_bow_sets* out, void* stream) {
  if (!v || !out) return fail(SLAMGPU_EINVAL, "NULL argument");
  if (n_sets < 0 || n_sets > 65535) return fail(SLAMGPU_EINVAL, "n_sets %d outside [0, 65535]", n_sets);
  if (n_sets == 0) return 0;
  if (out->cap < 1 || out->cap > SLAMGPU_BOW_MAX_FEATURES)
    return fail(SLAMGPU_EINVAL, "cap %d outside [1, %d]", out->cap, SLAMGPU_BOW_MAX_FEATURES);
  if (count_step < 1 || set_stride < 0) return fail(SLAMGPU_EINVAL, "bad set_stride/count_step");
  if (!d_desc || !d_counts || !out->words || !out->values || !out->n_words || !out->nodes ||
      !out->node_start || !out->node_feats || !out->n_nodes || !out->feat_leaf || !out->feat_node)
    return fail(SLAMGPU_EINVAL, "NULL device buffer");
  BOW_HIPCHECK(hipSetDevice(v->device));
  BowSets o;
  o.words = out->words;
  o.values = out->values;
  o.n_words = out->n_words;
  o.nodes = out->nodes;
  o.node_start = out->node_start;
  o.node_feats = out->node_feats;
  o.n_nodes = out->n_nodes;
  o.feat_leaf = out->feat_leaf;
  o.feat_node = out->feat_node;
  o.cap = out->cap;
  BOW_HIPCHECK(launch_bow_transform(device_view(v, levelsup), d_desc, set_stride, d_counts,
                                    count_step, n_sets, o, static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_bow_transform(slamgpu_vocab* v, const uint8_t* desc, int n, int levelsup,
                          uint32_t* words, double* values, int* n_words, uint32_t* nodes,
                          int32_t* node_start, uint32_t* node_feats, int* n_nodes) {
  if (!v || !n_words || !n_nodes || !node_start) return fail(SLAMGPU_EINVAL, "NULL argument");
  if (n < 0 || n > SLAMGPU_BOW_MAX_FEATURES)
    return fail(SLAMGPU_ECAP, "n %d outside [0, %d]", n, SLAMGPU_BOW_MAX_FEATURES);
  if (n > 0 && (!desc || !words || !values || !nodes || !node_feats))
    return fail(SLAMGPU_EINVAL, "NULL buffer");
  const int cap = n > 0 ? n : 1;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += al256(bytes); return o; };
  const size_t o_desc = take((size_t)cap * 32), o_cnt = take(4), o_words = take((size_t)cap * 4),
               o_vals = take((size_t)cap * 8), o_nw = take(4), o_nodes = take((size_t)cap * 4),
               o_start = take((size_t)(cap + 1) * 4), o_feats = take((size_t)cap * 4),
               o_nn = take(4), o_leaf = take((size_t)cap * 4), o_nid = take((size_t)cap * 4);
  BOW_HIPCHECK(hipSetDevice(v->device));
  if (off > v->stage_bytes) {
    if (v->stage) BOW_HIPCHECK(hipFree(v->stage));
    v->stage = nullptr;
    v->stage_bytes = 0;
    BOW_HIPCHECK(hipMalloc(&v->stage, off));
    v->stage_bytes = off;
  }
  char* b = v->stage;
  const int32_t cnt = n;
  if (n > 0)
    BOW_HIPCHECK(hipMemcpyAsync(b + o_desc, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
  BOW_HIPCHECK(hipMemcpyAsync(b + o_cnt, &cnt, 4, hipMemcpyHostToDevice, v->stream));
  BowSets o;
  o.words = reinterpret_cast<uint32_t*>(b + o_words);
  o.values = reinterpret_cast<double*>(b + o_vals);
  o.n_words = reinterpret_cast<int32_t*>(b + o_nw);
  o.nodes = reinterpret_cast<uint32_t*>(b + o_nodes);
  o.node_start = reinterpret_cast<int32_t*>(b + o_start);
  o.node_feats = reinterpret_cast<uint32_t*>(b + o_feats);
  o.n_nodes = reinterpret_cast<int32_t*>(b + o_nn);
  o.feat_leaf = reinterpret_cast<uint32_t*>(b + o_leaf);
  o.feat_node = reinterpret_cast<uint32_t*>(b + o_nid);
  o.cap = cap;
  BOW_HIPCHECK(launch_bow_transform(device_view(v, levelsup), reinterpret_cast<uint8_t*>(b + o_desc),
                                    0, reinterpret_cast<int32_t*>(b + o_cnt), 1, 1, o, v->stream));
  int32_t nw = 0, nn = 0;
  BOW_HIPCHECK(hipMemcpyAsync(&nw, b + o_nw, 4, hipMemcpyDeviceToHost, v->stream));
  BOW_HIPCHECK(hipMemcpyAsync(&nn, b + o_nn, 4, hipMemcpyDeviceToHost, v->stream));
  BOW_HIPCHECK(hipStreamSynchronize(v->stream));
  if (nw > 0) {
    BOW_HIPCHECK(hipMemcpyAsync(words, b + o_words, (size_t)nw * 4, hipMemcpyDeviceToHost, v->stream));
    BOW_HIPCHECK(hipMemcpyAsync(values, b + o_vals, (size_t)nw * 8, hipMemcpyDeviceToHost, v->stream));
  }
  BOW_HIPCHECK(hipMemcpyAsync(node_start, b + o_start, (size_t)(nn + 1) * 4, hipMemcpyDeviceToHost,
                              v->stream));
  if (nn > 0)
    BOW_HIPCHECK(hipMemcpyAsync(nodes, b + o_nodes, (size_t)nn * 4, hipMemcpyDeviceToHost, v->stream));
  BOW_HIPCHECK(hipStreamSynchronize(v->stream));
  if (nn > 0 && node_start[nn] > 0)
    BOW_HIPCHECK(hipMemcpy(node_feats, b + o_feats, (size_t)node_start[nn] * 4,
                           hipMemcpyDeviceToHost));
  *n_words = nw;
  *n_nodes = nn;
  return 0;
}

int slamgpu_search_by_bow_device(const slamgpu_bow_view* d_a, const slamgpu_bow_view* d_b,
                                 int n_pairs, int kf_kf, float nnratio, int check_ori,
                                 int32_t* d_match, int64_t match_stride, int32_t* d_nmatches,
                                 void* stream) {
  if (n_pairs < 0) return fail(SLAMGPU_EINVAL, "n_pairs %d < 0", n_pairs);
  if (n_pairs == 0) return 0;
  if (!d_a || !d_b || !d_match || !d_nmatches) return fail(SLAMGPU_EINVAL, "NULL device buffer");
  if (match_stride < 0) return fail(SLAMGPU_EINVAL, "match_stride < 0");
  BOW_HIPCHECK(launch_search_bow(reinterpret_cast<const BowView*>(d_a),
                                 reinterpret_cast<const BowView*>(d_b), n_pairs, kf_kf ? 1 : 0,
                                 nnratio, check_ori ? 1 : 0, d_match, match_stride, d_nmatches,
                                 static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_search_by_bow(const slamgpu_bow_set* a, const slamgpu_bow_set* b, int kf_kf,
                          float nnratio, int check_ori, int32_t* match_a, int* nmatches) {
  if (int r = check_set(a, "a")) return r;
  if (int r = check_set(b, "b")) return r;
  if (!nmatches || (a->n > 0 && !match_a)) return fail(SLAMGPU_EINVAL, "NULL output");
  const uint8_t* b_valid = kf_kf ? b->valid : nullptr;
  Stage& S = t_stage;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += al256(bytes); return o; };
  struct Placed {
    size_t desc, kps, valid, cnt, nodes, start, feats;
  } pa, pb;
  auto place = [&](const slamgpu_bow_set* s, Placed* p) {
    p->desc = take((size_t)s->n * 32);
    p->kps = take((size_t)s->n * sizeof(slamgpu_keypoint));
    p->valid = take((size_t)s->n);
    p->cnt = take(8);
    p->nodes = take((size_t)s->n_nodes * 4);
    p->start = take((size_t)(s->n_nodes + 1) * 4);
    p->feats = take((size_t)s->n * 4);
  };
  place(a, &pa);
  place(b, &pb);
  const size_t o_views = take(2 * sizeof(slamgpu_bow_view)), o_match = take((size_t)a->n * 4 + 4),
               o_nm = take(4);
  if (int r = stage_reserve(S, off)) return r;
  char* base = S.buf;
  slamgpu_bow_view views[2];
  auto upload_set = [&](const slamgpu_bow_set* s, const Placed& p, const uint8_t* valid,
                        slamgpu_bow_view* vw) -> int {
    const int32_t cnt[2] = {s->n, s->n_nodes};
    if (s->n > 0) {
      BOW_HIPCHECK(hipMemcpyAsync(base + p.desc, s->desc, (size_t)s->n * 32, hipMemcpyHostToDevice, S.stream));
      BOW_HIPCHECK(hipMemcpyAsync(base + p.kps, s->kps, (size_t)s->n * sizeof(slamgpu_keypoint),
                                  hipMemcpyHostToDevice, S.stream));
      if (valid)
        BOW_HIPCHECK(hipMemcpyAsync(base + p.valid, valid, (size_t)s->n, hipMemcpyHostToDevice, S.stream));
    }
    BOW_HIPCHECK(hipMemcpyAsync(base + p.cnt, cnt, 8, hipMemcpyHostToDevice, S.stream));
    if (s->n_nodes > 0) {
      BOW_HIPCHECK(hipMemcpyAsync(base + p.nodes, s->nodes, (size_t)s->n_nodes * 4,
                                  hipMemcpyHostToDevice, S.stream));
      BOW_HIPCHECK(hipMemcpyAsync(base + p.start, s->node_start, (size_t)(s->n_nodes + 1) * 4,
                                  hipMemcpyHostToDevice, S.stream));
      if (s->node_start[s->n_nodes] > 0)
        BOW_HIPCHECK(hipMemcpyAsync(base + p.feats, s->node_feats, (size_t)s->node_start[s->n_nodes] * 4,
                                    hipMemcpyHostToDevice, S.stream));
    }
    vw->desc = reinterpret_cast<const uint8_t*>(base + p.desc);
    vw->kps = reinterpret_cast<const slamgpu_keypoint*>(base + p.kps);
    vw->valid = valid ? reinterpret_cast<const uint8_t*>(base + p.valid) : nullptr;
    vw->n = reinterpret_cast<const int32_t*>(base + p.cnt);
    vw->n_nodes = reinterpret_cast<const int32_t*>(base + p.cnt + 4);
    vw->nodes = reinterpret_cast<const uint32_t*>(base + p.nodes);
    vw->node_start = reinterpret_cast<const int32_t*>(base + p.start);
    vw->node_feats = reinterpret_cast<const uint32_t*>(base + p.feats);
    return 0;
  };
  // the pair's hipMemcpyAsync sources must outlive the copies: synchronise before returning
  if (int r = upload_set(a, pa, a->valid, &views[0])) return r;
  if (int r = upload_set(b, pb, b_valid, &views[1])) return r;
  BOW_HIPCHECK(hipMemcpyAsync(base + o_views, views, sizeof(views), hipMemcpyHostToDevice, S.stream));
  const slamgpu_bow_view* dv = reinterpret_cast<const slamgpu_bow_view*>(base + o_views);
  BOW_HIPCHECK(launch_search_bow(reinterpret_cast<const BowView*>(dv),
                                 reinterpret_cast<const BowView*>(dv + 1), 1, kf_kf ? 1 : 0, nnratio,
                                 check_ori ? 1 : 0, reinterpret_cast<int32_t*>(base + o_match), 0,
                                 reinterpret_cast<int32_t*>(base + o_nm), S.stream));
  int32_t nm = 0;
  BOW_HIPCHECK(hipMemcpyAsync(&nm, base + o_nm, 4, hipMemcpyDeviceToHost, S.stream));
  if (a->n > 0)
    BOW_HIPCHECK(hipMemcpyAsync(match_a, base + o_match, (size_t)a->n * 4, hipMemcpyDeviceToHost,
                                S.stream));
  BOW_HIPCHECK(hipStreamSynchronize(S.stream));
  *nmatches = nm;
  return 0;
}

int slamgpu_distinctive_descriptors_device(const uint8_t* d_desc, const int32_t* d_start,
                                           int n_points, int32_t* d_best, uint8_t* d_desc_out,
                                           void* stream) {
  if (n_points < 0) return fail(SLAMGPU_EINVAL, "n_points %d < 0", n_points);
  if (n_points == 0) return 0;
  if (!d_desc || !d_start || !d_best) return fail(SLAMGPU_EINVAL, "NULL device buffer");
  BOW_HIPCHECK(launch_distinctive(d_desc, d_start, n_points, d_best, d_desc_out,
                                  static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_distinctive_descriptors(const uint8_t* desc, const int32_t* start, int n_points,
                                    int32_t* best, uint8_t* desc_out) {
  if (n_points < 0 || !start || (n_points > 0 && !best))
    return fail(SLAMGPU_EINVAL, "bad arguments");
  if (n_points == 0) return 0;
  const int32_t s0 = start[0];
  for (int p = 0; p < n_points; p++)
    if (start[p + 1] < start[p] || start[p + 1] - start[p] > 65535 || start[p] < 0)
      return fail(SLAMGPU_EINVAL, "start not ascending (or a point with > 65535 descriptors)");
  const int total = start[n_points] - s0;
  if (total > 0 && !desc) return fail(SLAMGPU_EINVAL, "NULL desc");
  Stage& S = t_stage;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += al256(bytes); return o; };
  const size_t o_desc = take((size_t)total * 32 + 4), o_start = take((size_t)(n_points + 1) * 4),
               o_best = take((size_t)n_points * 4), o_out = take((size_t)n_points * 32);
  if (int r = stage_reserve(S, off)) return r;
  char* b = S.buf;
  std::vector<int32_t> rel(n_points + 1);
  for (int p = 0; p <= n_points; p++) rel[p] = start[p] - s0;
  if (total > 0)
    BOW_HIPCHECK(hipMemcpyAsync(b + o_desc, desc + (size_t)s0 * 32, (size_t)total * 32,
                                hipMemcpyHostToDevice, S.stream));
  BOW_HIPCHECK(hipMemcpyAsync(b + o_start, rel.data(), rel.size() * 4, hipMemcpyHostToDevice, S.stream));
  BOW_HIPCHECK(launch_distinctive(reinterpret_cast<uint8_t*>(b + o_desc),
                                  reinterpret_cast<int32_t*>(b + o_start), n_points,
                                  reinterpret_cast<int32_t*>(b + o_best),
                                  desc_out ? reinterpret_cast<uint8_t*>(b + o_out) : nullptr, S.stream));
  BOW_HIPCHECK(hipMemcpyAsync(best, b + o_best, (size_t)n_points * 4, hipMemcpyDeviceToHost, S.stream));
  BOW_HIPCHECK(hipStreamSynchronize(S.stream));
  if (desc_out) {
    std::vector<uint8_t> tmp((size_t)n_points * 32);
    BOW_HIPCHECK(hipMemcpy(tmp.data(), b + o_out, tmp.size(), hipMemcpyDeviceToHost));
    for (int p = 0; p < n_points; p++)
      if (best[p] >= 0) std::memcpy(desc_out + (size_t)p * 32, &tmp[(size_t)p * 32], 32);
  }
  return 0;
}

int slamgpu_gray_device(const uint8_t* d_src, size_t src_pitch, size_t src_stride, int channels,
                        int rgb, int cols, int rows, int n_images, uint8_t* d_dst,
                        size_t dst_pitch, size_t dst_stride, void* stream) {
  if (channels != 3 && channels != 4) return fail(SLAMGPU_EINVAL, "channels %d not 3 or 4", channels);
  if (cols < 0 || rows < 0 || n_images < 0 || rows > 65535 || n_images > 65535)
    return fail(SLAMGPU_EINVAL, "bad image geometry");
  if (src_pitch < (size_t)cols * channels || dst_pitch < (size_t)cols)
    return fail(SLAMGPU_EINVAL, "pitch smaller than a row");
  if ((size_t)cols * rows * n_images > 0 && (!d_src || !d_dst))
    return fail(SLAMGPU_EINVAL, "NULL device buffer");
  BOW_HIPCHECK(launch_gray(d_src, src_pitch, src_stride, channels, rgb, cols, rows, n_images,
                           d_dst, dst_pitch, dst_stride, static_cast<hipStream_t>(stream)));
  return 0;
}

int slamgpu_gray(const uint8_t* src, size_t src_pitch, int channels, int rgb, int cols, int rows,
                 uint8_t* dst, size_t dst_pitch) {
  if (channels != 3 && channels != 4) return fail(SLAMGPU_EINVAL, "channels %d not 3 or 4", channels);
  if (cols < 0 || rows < 0 || rows > 65535) return fail(SLAMGPU_EINVAL, "bad image geometry");
  if (cols == 0 || rows == 0) return 0;
  if (!src || !dst || src_pitch < (size_t)cols * channels || dst_pitch < (size_t)cols)
    return fail(SLAMGPU_EINVAL, "bad buffers");
  Stage& S = t_stage;
  const size_t sp = (size_t)cols * channels, dp = (size_t)cols;
  const size_t o_src = 0, o_dst = al256(sp * rows);
  if (int r = stage_reserve(S, o_dst + al256(dp * rows))) return r;
  char* b = S.buf;
  BOW_HIPCHECK(hipMemcpy2DAsync(b + o_src, sp, src, src_pitch, sp, rows, hipMemcpyHostToDevice, S.stream));
  BOW_HIPCHECK(launch_gray(reinterpret_cast<uint8_t*>(b + o_src), sp, 0, channels, rgb, cols, rows, 1,
                           reinterpret_cast<uint8_t*>(b + o_dst), dp, 0, S.stream));
  BOW_HIPCHECK(hipMemcpy2DAsync(dst, dst_pitch, b + o_dst, dp, dp, rows, hipMemcpyDeviceToHost, S.stream));
  BOW_HIPCHECK(hipStreamSynchronize(S.stream));
  return 0;
}

}  // extern "C"
