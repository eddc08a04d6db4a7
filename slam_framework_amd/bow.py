"""Bag of words, SearchByBoW, ComputeDistinctiveDescriptors and the colour-to-gray ingest on the
device: ctypes binding of include/slamgpu_bow.h with reference-shaped names.

  ORBVocabulary             DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
                            (third_party/DBoW2/DBoW2/TemplatedVocabulary.h): loadFromTextFile
                            (:1335-1421); transform(features, BowVector, FeatureVector, levelsup)
                            (:1123-1191) as Frame::ComputeBoW (frame.cpp:258-263) calls it
  search_by_bow             OrbMatcher::SearchByBoW, both overloads (orb_matcher.cpp:133-262,
                            :499-632); slamgpu.OrbMatcher.SearchByBoW wraps it
  distinctive_descriptors   MapPoint::ComputeDistinctiveDescriptors (map_point.cpp:249-304)
  cvt_gray                  cv::cvtColor(*2GRAY) of Tracker::GrabImageStereo (tracker.cpp:110-127)

libslamgpu.so is the only compute path (no CPU fallback); errors raise SlamGpuError.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import slamgpu as G

MAX_FEATURES = 4096
TF_IDF, TF, IDF, BINARY = range(4)                                        # BowVector.h:36-42
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)  # BowVector.h:45-53


class BowSet(C.Structure):
    """slamgpu_bow_set: one side of a SearchByBoW call (host pointers)."""
    _fields_ = [("desc", C.c_void_p), ("kps", C.c_void_p), ("valid", C.c_void_p),
                ("nodes", C.c_void_p), ("node_start", C.c_void_p), ("node_feats", C.c_void_p),
                ("n", C.c_int32), ("n_nodes", C.c_int32)]


VIEW_FIELDS = ("desc", "kps", "valid", "n", "nodes", "node_start", "node_feats", "n_nodes")
# slamgpu_bow_view: device addresses, 8 x u64
VIEW_DTYPE = np.dtype([(f, "<u8") for f in VIEW_FIELDS])


class BowSets(C.Structure):
    """slamgpu_bow_sets: device outputs of slamgpu_bow_transform_device."""
    _fields_ = [(f, C.c_void_p) for f in ("words", "values", "n_words", "nodes", "node_start",
                                          "node_feats", "n_nodes", "feat_leaf", "feat_node")] + [
        ("cap", C.c_int32), ("pad", C.c_int32)]


_bound = False


def lib():
    global _bound
    L = G.lib()
    if not _bound:
        vp, ip, sz, i64 = C.c_void_p, C.c_int, C.c_size_t, C.c_int64
        L.slamgpu_bow_last_error.argtypes = []
        L.slamgpu_bow_last_error.restype = C.c_char_p
        L.slamgpu_vocab_load_text.argtypes = [ip, C.c_char_p, C.POINTER(vp)]
        L.slamgpu_vocab_create.argtypes = [ip, ip, ip, ip, ip, ip, vp, vp, vp, vp, C.POINTER(vp)]
        L.slamgpu_vocab_destroy.argtypes = [vp]
        L.slamgpu_vocab_destroy.restype = None
        L.slamgpu_vocab_info.argtypes = [vp, vp]
        L.slamgpu_vocab_nodes.argtypes = [vp, vp, vp, vp, vp]
        L.slamgpu_bow_transform.argtypes = [vp, vp, ip, ip, vp, vp, C.POINTER(ip), vp, vp, vp,
                                            C.POINTER(ip)]
        L.slamgpu_bow_transform_device.argtypes = [vp, vp, i64, vp, ip, ip, ip,
                                                   C.POINTER(BowSets), vp]
        L.slamgpu_search_by_bow.argtypes = [C.POINTER(BowSet), C.POINTER(BowSet), ip, C.c_float,
                                            ip, vp, C.POINTER(ip)]
        L.slamgpu_search_by_bow_device.argtypes = [vp, vp, ip, ip, C.c_float, ip, vp, i64, vp, vp]
        L.slamgpu_distinctive_descriptors.argtypes = [vp, vp, ip, vp, vp]
        L.slamgpu_distinctive_descriptors_device.argtypes = [vp, vp, ip, vp, vp, vp]
        L.slamgpu_gray.argtypes = [vp, sz, ip, ip, ip, ip, vp, sz]
        L.slamgpu_gray_device.argtypes = [vp, sz, sz, ip, ip, ip, ip, ip, vp, sz, sz, vp]
        _bound = True
    return L


def _check(rc):
    if rc != 0:
        raise G.SlamGpuError(f"slamgpu error {rc}: {lib().slamgpu_bow_last_error().decode()}")


_p = G._ptr


def _dev(x):
    """Device address (torch tensor or int) as a c_void_p (NULL for None)."""
    if x is None:
        return None
    return C.c_void_p(x if isinstance(x, int) else int(x.data_ptr()))


class BowVector:
    """DBoW2::BowVector (std::map<WordId, WordValue>): ascending word ids, f64 values."""

    def __init__(self, words, values):
        self.words, self.values = words, values

    def __len__(self):
        return len(self.words)

    def items(self):
        return zip(self.words.tolist(), self.values.tolist())


class FeatureVector:
    """DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned>>) in CSR form."""

    def __init__(self, nodes, node_start, node_feats):
        self.nodes = np.ascontiguousarray(nodes, np.uint32)
        self.node_start = np.ascontiguousarray(node_start, np.int32)
        self.node_feats = np.ascontiguousarray(node_feats, np.uint32)

    def __len__(self):
        return len(self.nodes)

    def __getitem__(self, node):
        i = int(np.searchsorted(self.nodes, node))
        if i >= len(self.nodes) or self.nodes[i] != node:
            raise KeyError(node)
        return self.node_feats[self.node_start[i]:self.node_start[i + 1]]

    def items(self):
        for i, nd in enumerate(self.nodes.tolist()):
            yield nd, self.node_feats[self.node_start[i]:self.node_start[i + 1]]

    def arrays(self):
        return self.nodes, self.node_start, self.node_feats


class ORBVocabulary:
    """A DBoW2 ORB vocabulary resident on one device (TemplatedVocabulary's surface)."""

    def __init__(self, device=0):
        self.device = device
        self.h = None
        self.error = ""

    @classmethod
    def from_arrays(cls, V, device=0):
        """V: dict with k, L, scoring, weighting and the node arrays parent, leaf, desc, weight
        (node 0 = root), e.g. synthetic.vocabulary()."""
        self = cls(device)
        parent = np.ascontiguousarray(V["parent"], np.int32)
        leaf = np.ascontiguousarray(V["leaf"], np.uint8)
        desc = np.ascontiguousarray(V["desc"], np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(V["weight"], np.float64)
        h = C.c_void_p()
        _check(lib().slamgpu_vocab_create(device, int(V["k"]), int(V["L"]), int(V["scoring"]),
                                          int(V["weighting"]), len(parent), _p(parent), _p(leaf),
                                          _p(desc), _p(weight), C.byref(h)))
        self.h = h
        return self

    def loadFromTextFile(self, path) -> bool:
        """TemplatedVocabulary::loadFromTextFile; False (self.error says why) on a bad file."""
        self.close()
        h = C.c_void_p()
        rc = lib().slamgpu_vocab_load_text(self.device, str(path).encode(), C.byref(h))
        if rc != 0:
            self.error = lib().slamgpu_bow_last_error().decode()
            return False
        self.h = h
        return True

    def info(self):
        a = np.zeros(6, np.int32)
        _check(lib().slamgpu_vocab_info(self.h, _p(a)))
        return dict(zip(("k", "L", "scoring", "weighting", "n_nodes", "n_words"), a.tolist()))

    def nodes(self):
        n = self.info()["n_nodes"]
        parent, leaf = np.zeros(n, np.int32), np.zeros(n, np.uint8)
        desc, weight = np.zeros((n, 32), np.uint8), np.zeros(n, np.float64)
        _check(lib().slamgpu_vocab_nodes(self.h, _p(parent), _p(leaf), _p(desc), _p(weight)))
        return parent, leaf, desc, weight

    def transform(self, desc, levelsup=4):
        """Frame::ComputeBoW: (BowVector, FeatureVector) of an N x 32 u8 descriptor set."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        words, values = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        nodes, feats = np.zeros(m, np.uint32), np.zeros(m, np.uint32)
        start = np.zeros(m + 1, np.int32)
        nw, nn = C.c_int(), C.c_int()
        _check(lib().slamgpu_bow_transform(self.h, _p(d), n, levelsup, _p(words), _p(values),
                                           C.byref(nw), _p(nodes), _p(start), _p(feats),
                                           C.byref(nn)))
        nw, nn = nw.value, nn.value
        return (BowVector(words[:nw].copy(), values[:nw].copy()),
                FeatureVector(nodes[:nn].copy(), start[:nn + 1].copy(),
                              feats[:start[nn]].copy()))

    def transform_device(self, d_desc, set_stride, d_counts, count_step, n_sets, levelsup, sets,
                         stream=None):
        """Batched transform of device-resident descriptor sets into DeviceBowSets `sets`."""
        _check(lib().slamgpu_bow_transform_device(self.h, _dev(d_desc), set_stride,
                                                  _dev(d_counts), count_step, n_sets, levelsup,
                                                  C.byref(sets.struct), C.c_void_p(stream or 0)))

    def close(self):
        if getattr(self, "h", None):
            lib().slamgpu_vocab_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBowSets:
    """Torch-owned device outputs of ORBVocabulary.transform_device for n_sets sets."""

    def __init__(self, n_sets, cap, device):
        import torch
        i32 = torch.int32
        self.cap = cap
        self.words = torch.zeros((n_sets, cap), dtype=i32, device=device)
        self.values = torch.zeros((n_sets, cap), dtype=torch.float64, device=device)
        self.n_words = torch.zeros(n_sets, dtype=i32, device=device)
        self.nodes = torch.zeros((n_sets, cap), dtype=i32, device=device)
        self.node_start = torch.zeros((n_sets, cap + 1), dtype=i32, device=device)
        self.node_feats = torch.zeros((n_sets, cap), dtype=i32, device=device)
        self.n_nodes = torch.zeros(n_sets, dtype=i32, device=device)
        self.feat_leaf = torch.zeros((n_sets, cap), dtype=i32, device=device)
        self.feat_node = torch.zeros((n_sets, cap), dtype=i32, device=device)
        self.struct = BowSets(*[C.c_void_p(int(t.data_ptr())) for t in (
            self.words, self.values, self.n_words, self.nodes, self.node_start, self.node_feats,
            self.n_nodes, self.feat_leaf, self.feat_node)], cap, 0)

    def view_of(self, s):
        """Device addresses of set s's FeatureVector (for a slamgpu_bow_view)."""
        return {"nodes": int(self.nodes.data_ptr()) + 4 * s * self.cap,
                "node_start": int(self.node_start.data_ptr()) + 4 * s * (self.cap + 1),
                "node_feats": int(self.node_feats.data_ptr()) + 4 * s * self.cap,
                "n_nodes": int(self.n_nodes.data_ptr()) + 4 * s}

    def host(self, s):
        """(BowVector, FeatureVector) of set s, downloaded."""
        nw, nn = int(self.n_words[s]), int(self.n_nodes[s])
        start = self.node_start[s, :nn + 1].cpu().numpy()
        return (BowVector(self.words[s, :nw].cpu().numpy().view(np.uint32),
                          self.values[s, :nw].cpu().numpy()),
                FeatureVector(self.nodes[s, :nn].cpu().numpy().view(np.uint32), start,
                              self.node_feats[s, :start[nn]].cpu().numpy().view(np.uint32)))


def _host_set(desc, kps, valid, fv):
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    k = np.ascontiguousarray(kps)
    if len(k) and k.dtype != G.KP_DTYPE:
        k = k.view(G.KP_DTYPE)
    v = None if valid is None else np.ascontiguousarray(valid, np.uint8)
    nodes, start, feats = (np.ascontiguousarray(fv.nodes, np.uint32),
                           np.ascontiguousarray(fv.node_start, np.int32),
                           np.ascontiguousarray(fv.node_feats, np.uint32))
    s = BowSet(_p(d), _p(k), _p(v), _p(nodes), _p(start), _p(feats), len(d), len(nodes))
    return s, (d, k, v, nodes, start, feats)


def search_by_bow(a_desc, a_kps, a_valid, a_fv, b_desc, b_kps, b_fv, b_valid=None, kf_kf=False,
                  nnratio=0.6, check_ori=True):
    """OrbMatcher::SearchByBoW core. A = the keyframe (its map-point validity a_valid), B = the
    frame (kf_kf False) or the second keyframe (kf_kf True, b_valid). Returns (nmatches, match_a)
    with match_a[i] = B feature matched to A feature i or -1."""
    sa, keep_a = _host_set(a_desc, a_kps, a_valid, a_fv)
    sb, keep_b = _host_set(b_desc, b_kps, b_valid, b_fv)
    match = np.full(max(sa.n, 1), -1, np.int32)
    nm = C.c_int()
    _check(lib().slamgpu_search_by_bow(C.byref(sa), C.byref(sb), int(bool(kf_kf)), float(nnratio),
                                       int(bool(check_ori)), _p(match), C.byref(nm)))
    del keep_a, keep_b
    return nm.value, match[:sa.n]


def search_by_bow_device(d_a_views, d_b_views, n_pairs, kf_kf, nnratio, check_ori, d_match,
                         match_stride, d_nmatches, stream=None):
    _check(lib().slamgpu_search_by_bow_device(_dev(d_a_views), _dev(d_b_views), n_pairs,
                                              int(bool(kf_kf)), float(nnratio),
                                              int(bool(check_ori)), _dev(d_match), match_stride,
                                              _dev(d_nmatches), C.c_void_p(stream or 0)))


def distinctive_descriptors(desc, start):
    """ComputeDistinctiveDescriptors for every map point p (descriptors desc[start[p]:start[p+1]])
    -> (best index per point or -1, the chosen descriptors)."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    st = np.ascontiguousarray(start, np.int32)
    n = len(st) - 1
    best = np.zeros(max(n, 1), np.int32)
    out = np.zeros((max(n, 1), 32), np.uint8)
    _check(lib().slamgpu_distinctive_descriptors(_p(d), _p(st), n, _p(best), _p(out)))
    return best[:n], out[:n]


def distinctive_descriptors_device(d_desc, d_start, n_points, d_best, d_desc_out=None,
                                   stream=None):
    _check(lib().slamgpu_distinctive_descriptors_device(_dev(d_desc), _dev(d_start), n_points,
                                                        _dev(d_best), _dev(d_desc_out),
                                                        C.c_void_p(stream or 0)))


def cvt_gray(img, rgb=True):
    """cv::cvtColor(img, gray, rgb ? CV_RGB2GRAY : CV_BGR2GRAY) (4 channels: *A2GRAY)."""
    a = np.asarray(img, np.uint8)
    if a.strides[1] != a.shape[2] or a.strides[2] != 1:
        a = np.ascontiguousarray(a)
    rows, cols, cn = a.shape
    out = np.zeros((rows, cols), np.uint8)
    _check(lib().slamgpu_gray(_p(a), a.strides[0], cn, int(bool(rgb)), cols, rows, _p(out), cols))
    return out


def cvt_gray_device(d_src, src_pitch, src_stride, channels, rgb, cols, rows, n_images, d_dst,
                    dst_pitch, dst_stride, stream=None):
    _check(lib().slamgpu_gray_device(_dev(d_src), src_pitch, src_stride, channels, int(bool(rgb)),
                                     cols, rows, n_images, _dev(d_dst), dst_pitch, dst_stride,
                                     C.c_void_p(stream or 0)))
