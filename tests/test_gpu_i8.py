"""The int8 single pass for one-buyer searches (tt_i8_image + tt_scan_topk_i8f32,
DESIGN 4.1c): the image against its numpy restatement, and the search bit-exact against the
canonical f32 oracle -- the bound and the exact-score certification make it exact; a query the
final cannot certify takes the exact f32 fallback (clustered and adversarial cases below)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from twotower import kernels

    return kernels


def dev_rows(x, ep=None):
    from twotower import _lib

    x = np.ascontiguousarray(x, np.float32)
    ep = ep or _lib.padded_dim(x.shape[1])
    t = torch.zeros((x.shape[0], ep), dtype=torch.float32, device="cuda")
    t[:, : x.shape[1]] = torch.from_numpy(x).cuda()
    return t


@pytest.mark.parametrize("n,d", [(1000, 384), (129, 700), (64, 384), (5, 768)])
def test_i8_image_vs_numpy(K, oracle_mod, n, d):
    from oracle import oracle as O

    rng = np.random.default_rng(n + d)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    x[3 % n] = 0.0  # a zero row (its tile scale stays that of the other rows)
    if n >= 64:
        x[64:] *= 0.5  # tiles of different magnitude
    db = dev_rows(x)
    codes, scales, b3 = K.i8_image(db, d)
    c_ref, s_ref, b_ref = O.i8_image(x)
    assert np.array_equal(scales.cpu().numpy(), s_ref)
    got = codes.cpu().numpy()
    assert np.array_equal(got[:, :d], c_ref) and np.all(got[:, d:] == 0)
    b = b3.cpu().numpy().astype(np.float64)
    for i in range(3):  # upper bounds, tight to f64 rounding + the x1.000001 margin
        assert b_ref[i] <= b[i] <= b_ref[i] * 1.00001 + 1e-30, (i, b[i], b_ref[i])


def _i8_search(K, db, x16_ref, n, d, q, k):
    codes, scales, b3 = K.i8_image(db, d)
    return K.scan_topk_i8(db, codes, scales, n, d, q, k, b3.tolist())


@pytest.mark.parametrize("n,d,nq,k", [(100_000, 384, 1, 100), (300_001, 384, 4, 128),
                                      (1000, 384, 2, 10), (50_000, 700, 3, 100),
                                      (70_000, 768, 1, 1), (257, 384, 1, 128),
                                      (1_000_000, 384, 1, 100), (200_000, 384, 5, 100),
                                      (1_000_000, 384, 8, 100), (30_001, 700, 7, 64),
                                      (100_000, 768, 8, 128)])
def test_scan_topk_i8_bit_exact_vs_oracle(K, oracle_mod, n, d, nq, k):
    rng = np.random.default_rng(n + nq + k)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    db, qd = dev_rows(x), dev_rows(q)
    s, i = _i8_search(K, db, None, n, d, qd, k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("n,d", [(1000, 384), (37, 300), (16, 384), (129, 768)])
def test_i8_tile_vs_numpy(K, oracle_mod, n, d):
    """The tiled int8 image (tt_i8_tile) is the numpy restatement's permutation of the codes:
    per 16-row block, piece s, lane l = 16 g + col -> row col's bytes 64 s + 16 g .. + 15."""
    from oracle import oracle as O

    rng = np.random.default_rng(n * 3 + d)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    db = dev_rows(x)
    codes, _, _ = K.i8_image(db, d)
    tiled = K.i8_tile(codes, n, d)
    ref = O.i8_tile(codes.cpu().numpy(), n)
    assert tiled.numel() == ref.size
    assert np.array_equal(tiled.cpu().numpy(), ref)


@pytest.mark.parametrize("n,nq,k", [(100_000, 1, 100), (300_001, 4, 128), (1000, 2, 10),
                                    (5, 1, 3), (257, 1, 128), (70_001, 3, 1),
                                    (1_000_000, 1, 100), (200_000, 5, 100), (1_000_000, 8, 100),
                                    (100_000, 9, 100), (1_000_000, 16, 100), (33_333, 17, 64),
                                    (1_000_000, 32, 100), (4097, 31, 128), (20, 32, 20)])
def test_scan_topk_i8_tiled_bit_exact(K, oracle_mod, n, nq, k):
    """The register-fed stream over the tiled image (tt_scan_topk_i8t_f32, padded dim 384):
    bit-exact against the oracle and, for nq <= 8, identical to the LDS-ring stream over the
    row-major image, fallback counts included; tiny catalogs leave most waves without a block
    (n = 5: one block in one wave of the whole grid), at 1M rows the last slabs hold no rows,
    and 9-32 queries run as one or two 16-query MFMA blocks."""
    d = 384
    rng = np.random.default_rng(n + 7 * nq + k)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    db, qd = dev_rows(x), dev_rows(q)
    codes, scales, b3 = K.i8_image(db, d)
    tiled = K.i8_tile(codes, n, d)
    ws = torch.empty(K.filter_workspace_bytes(n, d, nq, k), dtype=torch.uint8, device="cuda")
    out = {}
    for name, t in (("tiled", tiled), ("ring", None)):
        if t is None and nq > K.I8_NQ_MAX:
            continue
        s, i = K.scan_topk_i8(db, codes, scales, n, d, qd, k, b3.tolist(), workspace=ws, tiled=t)
        out[name] = (s.cpu().numpy(), i.cpu().numpy(), K.filter_fallback_count(ws, n, d, nq, k))
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(out["tiled"][1], ri) and np.array_equal(out["tiled"][0], rs)
    if "ring" in out:
        assert out["tiled"][2] == out["ring"][2]
        assert np.array_equal(out["tiled"][1], out["ring"][1])
        assert np.array_equal(out["tiled"][0], out["ring"][0])
    if n >= 100_000:  # iid rows: every query certifies
        assert out["tiled"][2] == 0


def test_scan_topk_i8_tiled_32_queries_nan_clustered_mode_b(K, oracle_mod):
    """32 queries over the tiled image (two 16-query blocks) on the hard cases at once: Mode B
    buyers, a NaN query in the second block, and one query with 400 near-copies in one slab
    (cannot certify: falls back alone); every result bit-exact."""
    n, d, k = 300_000, 384, 100
    rng = np.random.default_rng(21)
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = np.empty((32, d), np.float32)
    h = rng.integers(0, n, (32, 20))
    w = np.where(rng.random((32, 20)) < 0.75, 1.0, 5.0).astype(np.float32)
    xn = oracle_mod.l2norm_rows(x, 0)
    q[:] = oracle_mod.weighted_avg_l2(xn[h], w)
    x[5000:5400] = q[7] + 0.05 * rng.standard_normal((400, d)).astype(np.float32)
    x = oracle_mod.l2norm_rows(x, 0)
    q = oracle_mod.l2norm_rows(q, 0)
    q[20, 3] = np.nan
    db = dev_rows(x)
    codes, scales, b3 = K.i8_image(db, d)
    ws = torch.empty(K.filter_workspace_bytes(n, d, 32, k), dtype=torch.uint8, device="cuda")
    s, i = K.scan_topk_i8(db, codes, scales, n, d, dev_rows(q), k, b3.tolist(), workspace=ws,
                          tiled=K.i8_tile(codes, n, d))
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert 1 <= K.filter_fallback_count(ws, n, d, 32, k) <= 2  # query 7 (and the NaN query)


def test_scan_topk_i8_tiled_nan_and_clustered(K, oracle_mod):
    """The tiled stream on the adversarial cases: a NaN row and a NaN query (bit-exact), and a
    clustered slab the final cannot certify (falls back, bit-exact)."""
    d, k = 384, 100
    rng = np.random.default_rng(11)
    n = 20_000
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    x[77, 5] = np.nan
    q = oracle_mod.l2norm_rows(rng.standard_normal((2, d)).astype(np.float32), 0)
    q[1, 0] = np.nan
    db = dev_rows(x)
    codes, scales, b3 = K.i8_image(db, d)
    s, i = K.scan_topk_i8(db, codes, scales, n, d, dev_rows(q), 50, b3.tolist(),
                          tiled=K.i8_tile(codes, n, d))
    rs, ri = oracle_mod.scan_topk(x, q, 50)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    n = 200_000
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((1, d)).astype(np.float32)
    x[1000:1400] = q + 0.05 * rng.standard_normal((400, d)).astype(np.float32)
    x = oracle_mod.l2norm_rows(x, 0)
    q = oracle_mod.l2norm_rows(q, 0)
    db = dev_rows(x)
    codes, scales, b3 = K.i8_image(db, d)
    ws = torch.empty(K.filter_workspace_bytes(n, d, 1, k), dtype=torch.uint8, device="cuda")
    s, i = K.scan_topk_i8(db, codes, scales, n, d, dev_rows(q), k, b3.tolist(), workspace=ws,
                          tiled=K.i8_tile(codes, n, d))
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert K.filter_fallback_count(ws, n, d, 1, k) == 1


def test_scan_topk_i8_mode_b_buyers_no_fallback(K, oracle_mod):
    """Mode B buyers (weighted averages of 20 catalog rows, as bench.py's) over 1M x 384: every
    result bit-exact, and the certification holds (no query falls back)."""
    n, d, k = 1_000_000, 384, 100
    rng = np.random.default_rng(5)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    db = dev_rows(x)
    codes, scales, b3 = K.i8_image(db, d)
    ws = torch.empty(K.filter_workspace_bytes(n, d, 8, k), dtype=torch.uint8, device="cuda")
    fb = 0
    for rep, nq in enumerate((4, 4, 1, 8, 8)):  # both buffer layouts (4 and 8 queries)
        h = rng.integers(0, n, (nq, 20))
        w = np.where(rng.random((nq, 20)) < 0.75, 1.0, 5.0).astype(np.float32)
        q = oracle_mod.l2norm_rows(oracle_mod.weighted_avg_l2(x[h], w), 0)
        s, i = K.scan_topk_i8(db, codes, scales, n, d, dev_rows(q), k, b3.tolist(), workspace=ws)
        fb += K.filter_fallback_count(ws, n, d, nq, k)
        rs, ri = oracle_mod.scan_topk(x, q, k)
        assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert fb == 0, fb


def test_scan_topk_i8_clustered_slab_falls_back_exactly(K, oracle_mod):
    """400 near-copies of the query inside one slab: that slab's 16th approximate score is far
    above the 100th exact score, so the final cannot certify and the exact fallback serves the
    query -- bit-exact either way; duplicates tie to the lower row."""
    n, d, k = 200_000, 384, 100
    rng = np.random.default_rng(9)
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((1, d)).astype(np.float32)
    x[1000:1400] = q + 0.05 * rng.standard_normal((400, d)).astype(np.float32)
    x[5000] = x[1001]  # an exact duplicate
    x = oracle_mod.l2norm_rows(x, 0)
    q = oracle_mod.l2norm_rows(q, 0)
    db = dev_rows(x)
    codes, scales, b3 = K.i8_image(db, d)
    ws = torch.empty(K.filter_workspace_bytes(n, d, 1, k), dtype=torch.uint8, device="cuda")
    s, i = K.scan_topk_i8(db, codes, scales, n, d, dev_rows(q), k, b3.tolist(), workspace=ws)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert K.filter_fallback_count(ws, n, d, 1, k) == 1


def test_scan_topk_i8_nan_row_and_nan_query(K, oracle_mod):
    n, d, k = 20_000, 384, 50
    rng = np.random.default_rng(4)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    x[77, 5] = np.nan  # a NaN row: never returned
    q = oracle_mod.l2norm_rows(rng.standard_normal((2, d)).astype(np.float32), 0)
    q[1, 0] = np.nan  # a NaN query: every slot (-inf, -1)
    db = dev_rows(x)
    s, i = _i8_search(K, db, None, n, d, dev_rows(q), k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)


def test_retrieve_one_buyer_takes_the_i8_pass(K):
    """VectorDatabase.retrieve (the serving path) at d = 384 builds the int8 image with the
    index and serves one-buyer calls through it: same answers as the bf16 path."""
    from twotower import VectorDatabase

    rng = np.random.default_rng(21)
    n, d, k = 60_000, 384, 100
    vdb = VectorDatabase(d)
    vdb.build_index(rng.standard_normal((n, d)).astype(np.float32), [f"p{j}" for j in range(n)])
    assert vdb.index.i8 is not None
    q = rng.standard_normal((3, d)).astype(np.float32)
    qd = vdb.normalize_queries(torch.from_numpy(q).cuda())
    s16, i16 = vdb.index.search_device(qd, k, method="bf16")
    for b in range(3):
        got = vdb.retrieve(q[b], k=k)
        assert [p for p, _ in got] == [f"p{j}" for j in i16[b].tolist()]
        assert [v for _, v in got] == s16[b].tolist()


def test_retrieve_falls_back_when_the_i8_pass_is_unsupported(K, oracle_mod):
    """A shape the int8 single pass refuses (TT_ERR_UNSUPPORTED: > 16.7M rows on 256 CUs, a
    GPU with more than 256 CUs, TT_FILTER_TOPM=0 -- forced here by the test hook) is served by
    the bf16 filter on every one-buyer path: retrieve (serving slot), search_device and
    PreparedSearch, with the oracle's exact answers; the int8 image is built lazily (on the
    first search after build_index) and add() marks it stale instead of rebuilding it."""
    from twotower import VectorDatabase, kernels

    rng = np.random.default_rng(41)
    n, d, k = 30_000, 384, 100
    x = rng.standard_normal((n, d)).astype(np.float32)
    vdb = VectorDatabase(d)
    vdb.build_index(x, [f"p{j}" for j in range(n)])
    assert vdb.index._i8_stale and vdb.index._i8 is None  # lazy: not built by build_index
    q = rng.standard_normal((2, d)).astype(np.float32)
    xn = oracle_mod.vector_db_normalize(x)
    qn = oracle_mod.vector_db_normalize(q)
    rs, ri = oracle_mod.scan_topk(xn, qn, k)
    assert K.i8_single_pass_ok(n, d, 1, k, 384)
    first = vdb.retrieve(q[0], k=k)  # builds the image, runs the int8 pass
    assert vdb.index._i8 is not None and not vdb.index._i8_stale
    try:
        K.debug_i8_force_unsupported(True)
        assert not K.i8_single_pass_ok(n, d, 1, k, 384)
        for b in range(2):
            got = vdb.retrieve(q[b], k=k)
            assert [p for p, _ in got] == [f"p{j}" for j in ri[b].tolist()]
            assert [v for _, v in got] == rs[b].tolist()
        assert got == vdb.retrieve(q[1], k=k) and first == vdb.retrieve(q[0], k=k)
        qd = vdb.normalize_queries(torch.from_numpy(q).cuda())
        s, i = vdb.index.search_device(qd, k)
        assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
        ix = vdb.index
        ps = K.PreparedSearch(ix.xb, ix.xb16, n, d, 2, k, ix.bounds, i8=ix.i8)
        assert not ps.i8
        s, i = ps(qd)
        assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    finally:
        K.debug_i8_force_unsupported(False)
    assert vdb.retrieve(q[0], k=k) == first  # back on the int8 pass, same answers
    vdb.index.add(np.zeros((1, d), np.float32))  # add(): image marked stale, not rebuilt
    assert vdb.index._i8_stale and vdb.index._i8 is None


def test_i8_abi_rejects_more_than_8_queries(K):
    """The ABI's batch limit (nq <= 8, the 8-query buffer layout): nq = 9 is refused with
    TT_ERR_UNSUPPORTED before any launch, and the Python wrapper raises."""
    import ctypes

    from twotower import _lib

    n, d, k = 4096, 384, 10
    db = torch.randn((n, d), device="cuda")
    K.l2norm_rows(db, d, _lib.TT_NORM_ADD_EPS, out=db)
    codes, scales, b3 = K.i8_image(db, d)
    q = torch.randn((9, d), device="cuda")
    with pytest.raises(ValueError):
        K.scan_topk_i8(db, codes, scales, n, d, q, k, b3.tolist())
    ws = torch.empty(K.filter_workspace_bytes(n, d, 9, k), dtype=torch.uint8, device="cuda")
    out_s = torch.empty((9, k), device="cuda")
    out_i = torch.empty((9, k), dtype=torch.int64, device="cuda")
    X, R, S = (ctypes.c_float(v) for v in b3.tolist())
    rc = _lib.lib().tt_scan_topk_i8f32(
        db.data_ptr(), codes.data_ptr(), scales.data_ptr(), n, d, db.stride(0), codes.stride(0),
        0, q.data_ptr(), 9, q.stride(0), k, X, R, S, out_s.data_ptr(), out_i.data_ptr(),
        ws.data_ptr(), ws.numel(), None, None, None)
    assert rc == _lib.TT_ERR_UNSUPPORTED


def test_retrieve_batch_large_takes_the_i8_sample_level(K, oracle_mod):
    """VectorDatabase.retrieve_batch with 2100 queries at d = 384 (the serving slot's large
    batch) runs its sample level on the index's int8 image (tt_scan_topk_bf16f32_i8s) and
    returns the C oracle's exact top k."""
    from twotower import VectorDatabase, _lib

    rng = np.random.default_rng(33)
    n, d, k, nq = 40_000, 384, 50, 2100
    x = rng.standard_normal((n, d)).astype(np.float32)
    vdb = VectorDatabase(d)
    vdb.build_index(x, [f"p{j}" for j in range(n)])
    assert vdb.index.i8 is not None
    q = rng.standard_normal((nq, d)).astype(np.float32)
    got = vdb.retrieve_batch(q, k=k)
    assert _lib.lib().tt_debug_last_sample_i8() == 1
    xn = oracle_mod.vector_db_normalize(x)
    qn = oracle_mod.vector_db_normalize(q)
    rs, ri = oracle_mod.scan_topk(xn, qn, k)
    for b in (0, 1, 777, 2099):
        assert [p for p, _ in got[b]] == [f"p{j}" for j in ri[b].tolist()]
        assert [v for _, v in got[b]] == rs[b].tolist()
