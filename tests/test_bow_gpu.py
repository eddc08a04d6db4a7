"""GPU parity of the BoW rows (SURVEY.md section 8(f) rows 1-3 + the colour ingest) against the
oracle (oracle/bow_oracle.c, itself pinned by tests/test_bow_oracle.py), through the C ABI
(include/slamgpu_bow.h). Bit-exact on every output: word ids, f64 word values, FeatureVector
nodes and feature lists, SearchByBoW assignments and counts, distinctive-descriptor indices, gray
pixels.

Vocabularies are seeded synthetic trees in ORBvoc.txt's format and shape (k = 10, L = 6, L1 /
TF-IDF, top levels drawn from real ORB descriptors): the reference ships no vocabulary."""
import types

import numpy as np
import pytest

import test_bow_oracle as T
from slam_framework_amd import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B(gpu_lib):
    from slam_framework_amd import bow
    return bow


@pytest.fixture(scope="module")
def torch_dev(gpu_lib):
    import torch
    return torch, torch.device("cuda", 0)


@pytest.fixture(scope="module")
def frames(oracle):
    """Oracle ORB features (keypoints, descriptors) of 2 consecutive frames of one sequence."""
    t = oracle.tables()
    L, _ = S.sequence(3100, 2)
    return [oracle.extract(t, L[i]) for i in range(2)]


@pytest.fixture(scope="module")
def orbvoc(frames):
    return S.vocabulary(31, k=10, L=6, pool=frames[0][1])


@pytest.fixture(scope="module")
def orbvoc_pair(oracle, B, orbvoc):
    return oracle.OracleVocab(orbvoc), B.ORBVocabulary.from_arrays(orbvoc)


def _eq_transform(got, want):
    bv, fv = got
    words, vals, nodes, start, feats = want
    np.testing.assert_array_equal(bv.words, words)
    assert bv.values.tobytes() == vals.tobytes()
    np.testing.assert_array_equal(fv.nodes, nodes)
    np.testing.assert_array_equal(fv.node_start, start)
    np.testing.assert_array_equal(fv.node_feats, feats)


@pytest.mark.parametrize("name,make", T.VOCABS, ids=[v[0] for v in T.VOCABS])
@pytest.mark.parametrize("levelsup", [0, 2, 4])
def test_transform_small_vocabularies(oracle, B, name, make, levelsup):
    V = make()
    ov, gv = oracle.OracleVocab(V), B.ORBVocabulary.from_arrays(V)
    for n in (0, 1, 150, 700):
        feats = T.descs(11 + n, n, V)
        _eq_transform(gv.transform(feats, levelsup), oracle.bow_transform(ov, feats, levelsup))


def test_transform_orbvoc_frames(oracle, frames, orbvoc_pair):
    ov, gv = orbvoc_pair
    info = gv.info()
    assert info["n_nodes"] == 1111111 and info["n_words"] == 10 ** 6
    for _, d in frames:
        want = oracle.bow_transform(ov, d, 4)
        _eq_transform(gv.transform(d, 4), want)
        assert len(want[0]) > 500 and len(want[2]) > 20


def test_transform_device_batched(oracle, B, frames, orbvoc_pair, torch_dev):
    torch, dev = torch_dev
    ov, gv = orbvoc_pair
    rng = np.random.default_rng(5)
    sets = [frames[0][1], frames[1][1], frames[0][1][:1], frames[0][1][:0],
            rng.integers(0, 256, (700, 32), dtype=np.uint8), frames[1][1][::-1]]
    cap = 2200
    host = np.zeros((len(sets), cap, 32), np.uint8)
    counts = np.zeros(2 * len(sets), np.int32)  # count_step 2: the odd entries are decoys
    for s, d in enumerate(sets):
        host[s, :len(d)] = d
        counts[2 * s], counts[2 * s + 1] = len(d), 12345
    d_desc = torch.from_numpy(host).to(dev)
    d_cnt = torch.from_numpy(counts).to(dev)
    out = B.DeviceBowSets(len(sets), cap, dev)
    gv.transform_device(d_desc, cap, d_cnt, 2, len(sets), 4, out,
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for s, d in enumerate(sets):
        _eq_transform(out.host(s), oracle.bow_transform(ov, d, 4))


def _kf(kps, desc, fv, mps):
    return types.SimpleNamespace(keypoints=kps, descriptors=desc, feature_vec=fv, map_points=mps)


@pytest.mark.parametrize("kf_kf", [False, True])
@pytest.mark.parametrize("check_ori", [True, False])
@pytest.mark.parametrize("nnratio", [0.6, 0.75])
def test_search_by_bow_frames(oracle, B, frames, orbvoc_pair, kf_kf, check_ori, nnratio):
    """Keyframe = frame 0 (80% of its keypoints carry a map point), Frame / KeyFrame 2 = frame 1."""
    ov, gv = orbvoc_pair
    (ka, da), (kb, db) = frames
    fa, fb = gv.transform(da, 4)[1], gv.transform(db, 4)[1]
    rng = np.random.default_rng(7)
    va = (rng.random(len(da)) < 0.8).astype(np.uint8)
    vb = (rng.random(len(db)) < 0.8).astype(np.uint8) if kf_kf else None
    nm_o, m_o = oracle.search_by_bow(da, ka, va, fa.arrays(), db, kb, vb, fb.arrays(), kf_kf,
                                     nnratio, check_ori)
    nm_g, m_g = B.search_by_bow(da, ka, va, fa, db, kb, fb, b_valid=vb, kf_kf=kf_kf,
                                nnratio=nnratio, check_ori=check_ori)
    assert nm_g == nm_o
    np.testing.assert_array_equal(m_g, m_o)
    assert nm_o > 30, "consecutive frames should share vocabulary nodes and match"
    # the reference-shaped surface (OrbMatcher::SearchByBoW, both overloads)
    from slam_framework_amd.slamgpu import OrbMatcher
    mtch = OrbMatcher(nnratio, check_ori)
    mp_a = np.where(va > 0, np.arange(len(da)) + 1000, -1)
    if kf_kf:
        mp_b = np.where(vb > 0, np.arange(len(db)) + 5000, -1)
        nm, v12 = mtch.SearchByBoWKeyFrames(_kf(ka, da, fa, mp_a), _kf(kb, db, fb, mp_b))
        want = np.where(m_o >= 0, mp_b[np.maximum(m_o, 0)], -1)
    else:
        nm, v12 = mtch.SearchByBoW(_kf(ka, da, fa, mp_a), _kf(kb, db, fb, None))
        want = np.full(len(db), -1)
        want[m_o[m_o >= 0]] = mp_a[m_o >= 0]
    assert nm == nm_o
    np.testing.assert_array_equal(v12, want)


@pytest.mark.parametrize("kf_kf", [False, True])
def test_search_by_bow_synthetic_views(oracle, B, kf_kf):
    V = S.vocabulary(21, k=4, L=4)
    ov, gv = oracle.OracleVocab(V), B.ORBVocabulary.from_arrays(V)
    da, aa, db, ab = T.two_views(5, V, 1500, 1900)
    rng = np.random.default_rng(2)
    va = (rng.random(len(da)) < 0.85).astype(np.uint8)
    vb = (rng.random(len(db)) < 0.85).astype(np.uint8) if kf_kf else None
    ka, kb = T.kp_angles(oracle, aa), T.kp_angles(oracle, ab)
    fa, fb = gv.transform(da, 2)[1], gv.transform(db, 2)[1]
    nm_o, m_o = oracle.search_by_bow(da, ka, va, fa.arrays(), db, kb, vb, fb.arrays(), kf_kf, 0.8,
                                     True)
    nm_g, m_g = B.search_by_bow(da, ka, va, fa, db, kb, fb, b_valid=vb, kf_kf=kf_kf, nnratio=0.8)
    assert nm_g == nm_o and nm_o > 100
    np.testing.assert_array_equal(m_g, m_o)


def test_search_by_bow_one_big_node(oracle, B):
    """Every feature in one vocabulary node: > 64 candidates per lane row, the claimed-bitmask
    across candidate blocks, and identical descriptors (first-index ties)."""
    rng = np.random.default_rng(9)
    na, nb = 3000, 4096
    base = rng.integers(0, 256, (600, 32), dtype=np.uint8)
    da = base[rng.integers(0, 600, na)]
    db = base[rng.integers(0, 600, nb)].copy()
    flip = rng.integers(0, 256, db.shape, dtype=np.uint8)
    for _ in range(5):
        flip &= rng.integers(0, 256, db.shape, dtype=np.uint8)
    db ^= flip
    ka = T.kp_angles(oracle, rng.uniform(0, 360, na).astype(np.float32))
    kb = T.kp_angles(oracle, rng.uniform(0, 360, nb).astype(np.float32))
    fva = B.FeatureVector([77], [0, na], rng.permutation(na))
    fvb = B.FeatureVector([77], [0, nb], rng.permutation(nb))
    for check_ori in (False, True):
        nm_o, m_o = oracle.search_by_bow(da, ka, None, fva.arrays(), db, kb, None, fvb.arrays(),
                                         False, 1.0, check_ori)
        nm_g, m_g = B.search_by_bow(da, ka, None, fva, db, kb, fvb, nnratio=1.0,
                                    check_ori=check_ori)
        assert nm_g == nm_o and nm_o > 100
        np.testing.assert_array_equal(m_g, m_o)


def test_search_by_bow_device_batched(oracle, B, frames, orbvoc_pair, torch_dev):
    """Transform on the device, then SearchByBoW over device views of its outputs, no round trip."""
    torch, dev = torch_dev
    ov, gv = orbvoc_pair
    cap = 2200
    descs = [frames[0][1], frames[1][1]]
    kps = [frames[0][0], frames[1][0]]
    host = np.zeros((2, cap, 32), np.uint8)
    for s in range(2):
        host[s, :len(descs[s])] = descs[s]
    d_desc = torch.from_numpy(host).to(dev)
    d_cnt = torch.tensor([len(d) for d in descs], dtype=torch.int32, device=dev)
    out = B.DeviceBowSets(2, cap, dev)
    st = torch.cuda.current_stream().cuda_stream
    gv.transform_device(d_desc, cap, d_cnt, 1, 2, 4, out, st)
    rng = np.random.default_rng(3)
    valid = [(rng.random(len(d)) < 0.8).astype(np.uint8) for d in descs]
    keep = []

    def view(s, with_valid):
        k = torch.from_numpy(np.ascontiguousarray(kps[s]).view(np.uint8).copy()).to(dev)
        v = torch.from_numpy(valid[s]).to(dev)
        keep.extend([k, v])
        rec = {"desc": int(d_desc.data_ptr()) + s * cap * 32, "kps": int(k.data_ptr()),
               "valid": int(v.data_ptr()) if with_valid else 0,
               "n": int(d_cnt.data_ptr()) + 4 * s}
        rec.update(out.view_of(s))
        return rec

    pairs = [(0, 1), (1, 0), (0, 0)]
    for kf_kf in (False, True):
        va = np.zeros(len(pairs), B.VIEW_DTYPE)
        vb = np.zeros(len(pairs), B.VIEW_DTYPE)
        for p, (a, b) in enumerate(pairs):
            ra, rb = view(a, True), view(b, kf_kf)
            for f in B.VIEW_FIELDS:
                va[f][p], vb[f][p] = ra[f], rb[f]
        d_va = torch.from_numpy(va.view(np.uint8).copy()).to(dev)
        d_vb = torch.from_numpy(vb.view(np.uint8).copy()).to(dev)
        d_match = torch.full((len(pairs), cap), -7, dtype=torch.int32, device=dev)
        d_nm = torch.zeros(len(pairs), dtype=torch.int32, device=dev)
        B.search_by_bow_device(d_va, d_vb, len(pairs), kf_kf, 0.75, True, d_match, cap, d_nm, st)
        torch.cuda.synchronize()
        nm, match = d_nm.cpu().numpy(), d_match.cpu().numpy()
        for p, (a, b) in enumerate(pairs):
            fa, fb = out.host(a)[1], out.host(b)[1]
            nm_o, m_o = oracle.search_by_bow(descs[a], kps[a], valid[a], fa.arrays(), descs[b],
                                             kps[b], valid[b] if kf_kf else None, fb.arrays(),
                                             kf_kf, 0.75, True)
            assert nm[p] == nm_o
            np.testing.assert_array_equal(match[p, :len(descs[a])], m_o)


def test_distinctive_descriptors(oracle, B, torch_dev):
    torch, dev = torch_dev
    desc, start = T.distinctive_case(4)
    want = oracle.distinctive(desc, start)
    best, chosen = B.distinctive_descriptors(desc, start)
    np.testing.assert_array_equal(best, want)
    for p in np.nonzero(want >= 0)[0]:
        np.testing.assert_array_equal(chosen[p], desc[start[p] + want[p]])
    # device twin, with a point of 300 observations (> 64 rows per lane)
    rng = np.random.default_rng(6)
    big = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    d2 = np.concatenate([desc, big])
    s2 = np.concatenate([start, [start[-1] + 300]]).astype(np.int32)
    want2 = oracle.distinctive(d2, s2)
    d_best = torch.zeros(len(s2) - 1, dtype=torch.int32, device=dev)
    d_out = torch.zeros((len(s2) - 1, 32), dtype=torch.uint8, device=dev)
    B.distinctive_descriptors_device(torch.from_numpy(d2).to(dev), torch.from_numpy(s2).to(dev),
                                     len(s2) - 1, d_best, d_out,
                                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_best.cpu().numpy(), want2)


@pytest.mark.parametrize("shape", [(376, 1241), (37, 53), (5, 3), (1, 1)])
@pytest.mark.parametrize("cn", [3, 4])
@pytest.mark.parametrize("rgb", [True, False])
def test_cvt_gray(oracle, B, shape, cn, rgb):
    rng = np.random.default_rng(shape[1] + cn + rgb)
    img = rng.integers(0, 256, shape + (cn,), dtype=np.uint8)
    np.testing.assert_array_equal(B.cvt_gray(img, rgb), oracle.cvt_gray(img, rgb))
    # a row-padded source view (pitch > cols * cn)
    padded = np.zeros((shape[0], shape[1] + 7, cn), np.uint8)
    padded[:, :shape[1]] = img
    np.testing.assert_array_equal(B.cvt_gray(padded[:, :shape[1]], rgb), oracle.cvt_gray(img, rgb))


def test_cvt_gray_device_batch(oracle, B, torch_dev):
    """KITTI ingest: a batch of colour stereo images (BGR-decoded, is_rgb = true) into the
    frontend's pitched gray buffers."""
    torch, dev = torch_dev
    rows, cols, n = 376, 1241, 4
    rng = np.random.default_rng(12)
    src = rng.integers(0, 256, (n, rows, cols * 3 + 5), dtype=np.uint8)
    d_src = torch.from_numpy(src).to(dev)
    dpitch = 1280
    d_dst = torch.zeros((n, rows, dpitch), dtype=torch.uint8, device=dev)
    B.cvt_gray_device(d_src, cols * 3 + 5, rows * (cols * 3 + 5), 3, True, cols, rows, n, d_dst,
                      dpitch, rows * dpitch, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy()
    for i in range(n):
        img = src[i, :, :cols * 3].reshape(rows, cols, 3)
        np.testing.assert_array_equal(got[i, :, :cols], oracle.cvt_gray(img, True))
        assert (got[i, :, cols:] == 0).all()


def test_vocab_text_roundtrip(oracle, B, tmp_path):
    """loadFromTextFile on saveToTextFile's layout (TemplatedVocabulary.h:1335-1446)."""
    V = S.vocabulary(13, k=5, L=4, scoring=1, weighting=0)  # the header allows L <= 10 (:1356)
    V["leaf"][np.random.default_rng(1).choice(len(V["leaf"]), 40)] = 0  # unflagged nodes
    p = tmp_path / "voc.txt"
    p.write_text(S.vocabulary_text(V) + "\n  \n")  # trailing blank lines add no node
    gv = B.ORBVocabulary()
    assert gv.loadFromTextFile(p)
    parent, leaf, desc, weight = gv.nodes()
    np.testing.assert_array_equal(parent, V["parent"])
    np.testing.assert_array_equal(leaf, V["leaf"])
    np.testing.assert_array_equal(desc, V["desc"])
    assert weight.tobytes() == np.asarray(V["weight"], np.float64).tobytes()
    info = gv.info()
    assert (info["k"], info["L"], info["scoring"], info["weighting"]) == (
        V["k"], V["L"], 1, 0)
    feats = T.descs(2, 300, V)
    _eq_transform(gv.transform(feats, 2), oracle.bow_transform(oracle.OracleVocab(V), feats, 2))
    bad = tmp_path / "bad.txt"
    bad.write_text("10 6 9 0\n")  # scoring 9: "not a correct vocabulary"
    assert not gv.loadFromTextFile(bad) and "vocabulary" in gv.error
    assert not gv.loadFromTextFile(tmp_path / "missing.txt")


def test_errors_are_loud(B, orbvoc_pair):
    _, gv = orbvoc_pair
    with pytest.raises(B.G.SlamGpuError):
        gv.transform(np.zeros((B.MAX_FEATURES + 1, 32), np.uint8))
    fv = B.FeatureVector([3, 2], [0, 1, 2], [0, 1])  # nodes not ascending
    d = np.zeros((2, 32), np.uint8)
    k = np.zeros(2, B.G.KP_DTYPE)
    with pytest.raises(B.G.SlamGpuError):
        B.search_by_bow(d, k, None, fv, d, k, fv)
