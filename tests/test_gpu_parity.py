"""Parity of the HIP kernels (through the C ABI) with the CPU oracle and the reference
fixtures.  Bar: bit-exact for ids and for scores / normalised rows where the
oracle restates the kernel's canonical order; stated tolerances elsewhere."""
import numpy as np
import pytest
import torch

import inputs as gi

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


# ------------------------------------------------------------------ normalisation
@pytest.mark.parametrize("d", [1, 7, 64, 100, 128, 200, 257, 384, 768, 1000, 1536])
@pytest.mark.parametrize("mode", [0, 1])
def test_l2norm_bit_exact(K, oracle_mod, d, mode):
    rng = np.random.default_rng(d + 7 * mode)
    x = (rng.standard_normal((257, d)) * rng.uniform(1e-3, 1e3, (257, 1))).astype(np.float32)
    x[5] = 0.0  # zero row: mode 0 -> 0/(0+1e-8) = 0, mode 1 -> 0/1e-12 = 0
    xt = torch.from_numpy(x).cuda()
    ld = d + 3
    out = torch.full((257, ld), 7.0, device="cuda")
    K.l2norm_rows(xt, d, mode, out=out)
    got = out.cpu().numpy()
    assert np.array_equal(got[:, :d], oracle_mod.l2norm_rows(x, mode))
    assert np.all(got[:, d:] == 0)  # padding invariant
    if mode == 0:
        assert np.array_equal(got[:, :d], oracle_mod.vector_db_normalize(x))


def test_l2norm_bf16_copy(K):
    x = torch.randn(100, 384, device="cuda")
    out = torch.empty_like(x)
    ob = torch.empty((100, 384), dtype=torch.bfloat16, device="cuda")
    K.l2norm_rows(x, 384, 0, out=out, out_bf16=ob)
    assert torch.equal(ob, out.to(torch.bfloat16))


# ------------------------------------------------------------------ scan + top-k
SCAN_CASES = [
    # n, d, nq, k
    (1, 384, 3, 1),
    (33, 64, 3, 1),
    (100, 384, 16, 100),
    (101, 384, 16, 100),
    (1000, 384, 5, 10),
    (4096, 384, 16, 100),
    (4096, 384, 70, 128),
    (3000, 100, 7, 50),
    (5000, 768, 8, 100),
    (20000, 384, 130, 100),
    (70000, 384, 2, 100),
    (200000, 384, 1, 100),
    (4096, 384, 8, 129),
    (4096, 384, 8, 1000),
    (2048, 256, 17, 1024),
]


@pytest.mark.parametrize("n,d,nq,k", SCAN_CASES)
def test_scan_bit_exact_vs_oracle(K, oracle_mod, n, d, nq, k):
    rng = np.random.default_rng(n * 31 + d + k)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    s, i = K.scan_topk(dev_rows(x), n, d, dev_rows(q), k)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i, ri)
    assert np.array_equal(s, rs)


@pytest.mark.parametrize("n,d,nq,k", [(20000, 384, 3, 1025), (5000, 128, 2, 5000),
                                      (3000, 768, 5, 2999)])
def test_scan_large_k_bit_exact_vs_oracle(K, oracle_mod, n, d, nq, k):
    """k > 1024 (faiss takes any k <= ntotal): every canonical score by the f32 MFMA GEMM, a
    stable sort -- bit-exact ids and scores vs the oracle; a NaN row is never returned."""
    rng = np.random.default_rng(n + k)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    x[7] = np.nan
    x[11] = x[12]  # an exact tie: the lower row first
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    s, i = K.scan_topk_large(dev_rows(x), n, d, dev_rows(q), k, row_base=5)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    rs, ri = oracle_mod.scan_topk(x, q, k, row_base=5)
    assert np.array_equal(i, ri)
    assert np.array_equal(s, rs)
    assert not np.any(i == 7 + 5)


@pytest.mark.parametrize("n,d,nq,k", [(3000, 384, 1, 129), (20000, 384, 5, 500),
                                      (20000, 768, 17, 1000), (4096, 64, 70, 1024),
                                      (1024, 128, 3, 1024), (50000, 384, 2, 1000)])
def test_scan_select_bit_exact_vs_oracle(K, oracle_mod, n, d, nq, k):
    """128 < k <= 1024 (the /retrieve cap is 1000, server.py:46): scores-then-radix-select,
    bit-exact ids and scores vs the oracle and vs the per-slab-list scan -- one query tile
    (rows split over waves), several (shared rows), k == n, a NaN row never returned, exact
    ties (lower row first, also where the k-th score itself is tied), a NaN query (all slots
    (-inf, -1))."""
    rng = np.random.default_rng(n + d + k)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    x[7] = np.nan
    x[11] = x[12]  # an exact tie
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    # the k-th best of query 0 tied with a later duplicate row: the tie at the threshold
    # must be resolved by the row word (lower row in, higher row out)
    s0 = x @ q[0]
    order = np.argsort(-np.where(np.isnan(s0), -np.inf, s0), kind="stable")
    if k < n - 2:
        x[order[k + 1]] = x[order[k - 1]]
    if nq > 2:
        q[2] = np.nan
    dx, dq = dev_rows(x), dev_rows(q)
    s, i = K.scan_topk_select(dx, n, d, dq, k, row_base=3)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    rs, ri = oracle_mod.scan_topk(x, q, k, row_base=3)
    assert np.array_equal(i, ri)
    assert np.array_equal(s, rs)
    assert not np.any(i == 7 + 3)
    ss, si = K.scan_topk(dx, n, d, dq, k, row_base=3)
    assert np.array_equal(si.cpu().numpy(), i) and np.array_equal(ss.cpu().numpy(), s)


@pytest.mark.parametrize("k", [1000, 129])
def test_scan_select_heavy_duplicates_tail(K, oracle_mod, k):
    """3000 identical rows at the top score (more than SL_CAP keys share the k-th key's
    bucket after two digits): the per-query tail resolves the remaining digits on the row word
    -- the lowest rows win, bit-exact vs the oracle; a second query without duplicates in the
    same call takes the short path."""
    rng = np.random.default_rng(k)
    n, d = 20000, 128
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((2, d)).astype(np.float32), 0)
    x[100:3100] = q[0]  # score ~1.0 for query 0, 3000 exact ties
    dx, dq = dev_rows(x), dev_rows(q)
    s, i = K.scan_topk_select(dx, n, d, dq, k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert np.array_equal(ri[0], np.arange(100, 100 + k))
    s1, i1 = K.scan_topk_select(dx, n, d, dq[:1], k)  # one query: the fused first histogram
    assert np.array_equal(i1.cpu().numpy(), ri[:1]) and np.array_equal(s1.cpu().numpy(), rs[:1])


def test_scan_select_query_chunks_bit_exact(K, oracle_mod):
    """More queries than one chunk of score rows (the chunk is sized by a 256 MB budget: 64
    queries at 1M rows) -- chunks reuse the workspace, results bit-exact vs the scan."""
    rng = np.random.default_rng(5)
    n, d, nq, k = 1_000_000, 128, 80, 300
    x = torch.from_numpy(oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0))
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    dx, dq = dev_rows(x.numpy()), dev_rows(q)
    s, i = K.scan_topk_select(dx, n, d, dq, k)
    ss, si = K.scan_topk(dx, n, d, dq, k)
    assert torch.equal(i, si) and torch.equal(s, ss)
    sub = [0, 63, 64, 79]
    rs, ri = oracle_mod.scan_topk(x.numpy(), q[sub], k)
    assert np.array_equal(i.cpu().numpy()[sub], ri)


@pytest.mark.parametrize("d,k", [(1000, 100), (1024, 10), (1536, 1100)])
def test_vector_db_dims_above_768_bit_exact(K, oracle_mod, d, k):
    """Embedding dims past the scan kernels' 768 (the reference accepts any embedding_dim,
    vector_db.py:13,48): VectorDatabase builds, normalises and retrieves through the generic
    exact path (f32 MFMA GEMM scores + key top-k) -- ids and scores bit-exact vs the oracle,
    through retrieve_batch, retrieve and the device search."""
    from twotower import VectorDatabase

    rng = np.random.default_rng(d + k)
    n, nq = 5000, 6
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    ids = [f"p{i}" for i in range(n)]
    vdb = VectorDatabase(d)
    vdb.build_index(x, ids)
    assert vdb.index.ep % 64 == 0 and vdb.index.ep >= d and not vdb.index.scan_dim
    xn = oracle_mod.vector_db_normalize(x)
    assert np.array_equal(vdb.index.xb[:, :d].cpu().numpy(), xn)
    rs, ri = oracle_mod.scan_topk(xn, oracle_mod.vector_db_normalize(q), k)
    res = vdb.retrieve_batch(q, k=k)
    assert [[p for p, _ in r] for r in res] == [[ids[j] for j in row] for row in ri]
    assert np.array_equal(np.array([[sc for _, sc in r] for r in res], np.float32), rs)
    assert vdb.retrieve(q[2], k=k) == res[2]


BF16_CASES = [c for c in SCAN_CASES if c[3] <= 128] + [
    (2049, 384, 5, 128),     # two filter levels, k at the filter's maximum
    (300000, 384, 40, 100),  # tile-max first level at stride 16; 1024 full-level slabs
    (1000000, 384, 1, 100),  # one buyer at the bench catalog size (grouped k_select_reg)
    (150000, 384, 3, 10),    # 585 slabs: ragged groups of 10 per lane
    (70000, 128, 2, 50),     # E = 128, 273 slabs
    (60000, 768, 33, 100),   # E = 768 (one query block per wave)
    (60000, 768, 300, 100),  # E = 768 mid-size batch: two query blocks per wave (LVL 4)
    (30000, 500, 129, 64),   # E = 512, one query past a 128-query tile
    (20000, 384, 300, 100),  # several query tiles
    (40000, 512, 9, 64),
    # small batches (block-per-query selection): ragged sizes, every E
    (65600, 384, 1, 100),
    (250001, 768, 7, 128),   # E = 768, k at the maximum
    (130000, 64, 256, 100),  # the largest coarse batch
    (99999, 512, 2, 1),
    # the single-pass path (nq <= 4): one slab per CU, ragged / tiny slabs, every E shape
    (1000, 384, 3, 10),      # slabs of 4 rows: first tiles partly out of range
    (4096, 384, 4, 100),     # 16 rows per slab: the tile-max bound never fills
    (3000, 100, 2, 50),      # E padded to 128
    (5000, 768, 4, 100),     # E = 768: one compute wave per tile
    (40000, 64, 4, 100),     # E = 64: two k-steps per tile
    (250001, 768, 3, 128),   # k at the maximum, ragged last slab
]


def bounds(K, db, db16, d):
    return K.bf16_image_bounds(db, db16, d).tolist()


def test_bf16_image_bounds_vs_torch(K):
    """tt_bf16_image_bounds: upper bounds, tight to ~1e-6, NaN rows skipped."""
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn((5000, 384), generator=g, device="cuda") * 3
    x[17] = float("nan")
    x16 = x.to(torch.bfloat16)
    X, R = K.bf16_image_bounds(x, x16, 384).tolist()
    ok = ~torch.isnan(x).any(dim=1)
    nx = torch.linalg.vector_norm(x[ok].double(), dim=1).max().item()
    nr = torch.linalg.vector_norm((x[ok].double() - x16[ok].double()), dim=1).max().item()
    assert nx <= X <= nx * (1 + 1e-4) and nr <= R <= nr * (1 + 1e-4)
    out2 = torch.zeros(2, device="cuda")  # max-combine across batches
    K.bf16_image_bounds(x[:2500], x16[:2500], 384, out2=out2)
    K.bf16_image_bounds(x[2500:], x16[2500:], 384, out2=out2)
    assert out2.tolist() == [X, R]


@pytest.mark.parametrize("n,d,nq,k", BF16_CASES)
def test_bf16_filter_bit_exact_vs_oracle(K, oracle_mod, n, d, nq, k):
    """bf16 MFMA filter + exact f32 re-rank == canonical f32 top-k, bit for bit."""
    from twotower import _lib

    rng = np.random.default_rng(n * 17 + d + k)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    db = dev_rows(x)
    db16 = db.to(torch.bfloat16)
    s, i = K.scan_topk_bf16(db, db16, n, d, dev_rows(q), k, bounds(K, db, db16, d))
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)


def test_bf16_filter_exact_under_biased_rounding(K, oracle_mod):
    """Every catalog/query component sits just past a bf16 rounding midpoint, so all products
    round the same way (the case a worst-case-u bound of 2^-8 misses): still bit-exact."""
    rng = np.random.default_rng(79)
    n, d, nq, k = 50000, 384, 24, 100

    def biased(a):
        u = a.astype(np.float32).view(np.uint32)
        return ((u & np.uint32(0xFFFF0000)) | np.uint32(0x8001)).view(np.float32)

    x = biased(rng.standard_normal((n, d)).astype(np.float32) / np.sqrt(d))
    q = biased(rng.standard_normal((nq, d)).astype(np.float32) / np.sqrt(d))
    db = dev_rows(x)
    db16 = db.to(torch.bfloat16)
    s, i = K.scan_topk_bf16(db, db16, n, d, dev_rows(q), k, bounds(K, db, db16, d))
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)


def test_bf16_single_pass_clustered_slab_takes_fallback(K, oracle_mod):
    """The single-pass small-batch path keeps 16 rows per slab (one slab per CU): a catalog
    whose best rows crowd into ONE slab (40 near-copies of the query, consecutive) breaks its
    certification (that slab's 16th kept row is inside the band), so the query must take the
    exact fallback -- and still come out bit-exact."""
    rng = np.random.default_rng(83)
    n, d, k = 200000, 384, 100
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((1, d)).astype(np.float32)
    x[5000:5040] = q + 0.05 * rng.standard_normal((40, d)).astype(np.float32)
    x = oracle_mod.l2norm_rows(x, 0)
    q = oracle_mod.l2norm_rows(q, 0)
    db = dev_rows(x)
    db16 = db.to(torch.bfloat16)
    ws = torch.empty(K.filter_workspace_bytes(n, d, 1, k), dtype=torch.uint8, device="cuda")
    s, i = K.scan_topk_bf16(db, db16, n, d, dev_rows(q), k, bounds(K, db, db16, d),
                            workspace=ws)
    torch.cuda.synchronize()
    assert K.filter_fallback_count(ws, n, d, 1, k) == 1
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("nq", [1, 4, 16, 256, 300])
def test_bf16_filter_no_fallback_on_iid_data(K, nq):
    """The optimistic threshold must hold on iid data: no query may need the exact fallback
    (a performance property: fallbacks are correct but slow).  nq <= 256: the small path."""
    from twotower import _lib

    n, d, k = 1000000, 384, 100
    g = torch.Generator(device="cuda").manual_seed(5)
    db = torch.randn((n, d), generator=g, device="cuda")
    K.l2norm_rows(db, d, 0, out=db)
    q = torch.randn((nq, d), generator=g, device="cuda")
    K.l2norm_rows(q, d, 0, out=q)
    ws = torch.empty(K.filter_workspace_bytes(n, d, nq, k), dtype=torch.uint8, device="cuda")
    db16 = db.to(torch.bfloat16)
    K.scan_topk_bf16(db, db16, n, d, q, k, bounds(K, db, db16, d), workspace=ws)
    torch.cuda.synchronize()
    assert K.filter_fallback_count(ws, n, d, nq, k) == 0


@pytest.mark.parametrize("nq", [20, 150, 2100])
@pytest.mark.parametrize("resid", [0.5, 4.0])
def test_bf16_filter_fallback_is_exact(K, oracle_mod, resid, nq):
    """A loose bound overflows the candidate lists: every query then takes the exact
    fallback launch, and the results must not change.  nq = 20: one 64-query tile, its slab
    lists merged inside the scan launch by the last slab block (run twice on one workspace:
    the arrival counter is re-zeroed by each search); nq = 150 (the small path) and 2100 (the
    batched > 2048 path): the adaptive fallback (k_scan_fallback: 16-query tiles spread over
    the chip on the device, then k_merge_fallback), ragged last tiles."""
    rng = np.random.default_rng(77)
    n, d, k = 30000, 384, 100
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    db = dev_rows(x)
    ws = torch.empty(K.filter_workspace_bytes(n, d, nq, k), dtype=torch.uint8, device="cuda")
    rs, ri = oracle_mod.scan_topk(x, q, k)
    for _ in range(2):
        s, i = K.scan_topk_bf16(db, db.to(torch.bfloat16), n, d, dev_rows(q), k, (1.0, resid),
                                workspace=ws)
        assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
        assert K.filter_fallback_count(ws, n, d, nq, k) == nq  # every query fell back


@pytest.mark.parametrize("nq", [1, 5, 64])
def test_bf16_filter_small_batch_clustered(K, oracle_mod, nq):
    """Small batches on clustered data: tight clusters can push a query's full level past the
    small path's candidate cap -> exact fallback; the results stay bit-exact either way."""
    rng = np.random.default_rng(90 + nq)
    base = oracle_mod.l2norm_rows(rng.standard_normal((300, 384)).astype(np.float32), 0)
    x = np.repeat(base, 400, axis=0) + rng.standard_normal((120000, 384)).astype(np.float32) * 0.05
    x = oracle_mod.l2norm_rows(x, 0)
    q = oracle_mod.l2norm_rows(base[:nq] + rng.standard_normal((nq, 384)).astype(np.float32) * 0.02, 0)
    db = dev_rows(x)
    db16 = db.to(torch.bfloat16)
    s, i = K.scan_topk_bf16(db, db16, x.shape[0], 384, dev_rows(q), 100, bounds(K, db, db16, 384))
    rs, ri = oracle_mod.scan_topk(x, q, 100)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)


def test_bf16_filter_clusters_and_ties(K, oracle_mod):
    """Near-duplicate clusters (band overflow) and exact duplicates (ties on both scores)."""
    rng = np.random.default_rng(78)
    base = oracle_mod.l2norm_rows(rng.standard_normal((400, 384)).astype(np.float32), 0)
    noise = rng.standard_normal((12000, 384)).astype(np.float32) * 1e-4
    x = oracle_mod.l2norm_rows(np.repeat(base, 30, axis=0) + noise, 0)
    x[:1200] = np.repeat(base[:40], 30, axis=0)  # exact duplicates
    q = np.concatenate([base[:6], oracle_mod.l2norm_rows(
        rng.standard_normal((6, 384)).astype(np.float32), 0), np.zeros((1, 384), np.float32)])
    db = dev_rows(x)
    db16 = db.to(torch.bfloat16)
    s, i = K.scan_topk_bf16(db, db16, x.shape[0], 384, dev_rows(q), 128, bounds(K, db, db16, 384))
    rs, ri = oracle_mod.scan_topk(x, q, 128)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)


def test_scan_ties_and_duplicates(K, oracle_mod):
    rng = np.random.default_rng(9)
    base = oracle_mod.l2norm_rows(rng.standard_normal((700, 384)).astype(np.float32), 0)
    x = np.concatenate([base] * 5)  # every score appears 5x; the lower row must win
    q = np.concatenate([base[:8], np.zeros((2, 384), np.float32)])  # zero query: all scores 0
    s, i = K.scan_topk(dev_rows(x), x.shape[0], 384, dev_rows(q), 128)
    rs, ri = oracle_mod.scan_topk(x, q, 128)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert np.array_equal(ri[-1], np.arange(128))  # all-equal scores -> rows 0..127


def test_scan_nan_rows_never_returned(K, oracle_mod):
    rng = np.random.default_rng(10)
    x = oracle_mod.l2norm_rows(rng.standard_normal((300, 384)).astype(np.float32), 0)
    x[[3, 50, 299]] = np.nan
    q = oracle_mod.l2norm_rows(rng.standard_normal((4, 384)).astype(np.float32), 0)
    s, i = K.scan_topk(dev_rows(x), 300, 384, dev_rows(q), 299)
    rs, ri = oracle_mod.scan_topk(x, q, 299)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)
    assert not np.isin(i.cpu().numpy()[:, :297], [3, 50, 299]).any()
    assert np.all(i.cpu().numpy()[:, 297:] == -1)


def test_scan_row_base_and_merge_equal_single_shard(K, oracle_mod):
    rng = np.random.default_rng(11)
    n, d, nq, k = 50000, 384, 40, 100
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = dev_rows(oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0))
    cuts = [0, 7000, 19000, 33333, n]
    parts = [K.scan_topk(dev_rows(x[a:b]), b - a, d, q, k, row_base=a)
             for a, b in zip(cuts[:-1], cuts[1:])]
    ms, mi = K.merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]), k)
    fs, fi = K.scan_topk(dev_rows(x), n, d, q, k)
    assert torch.equal(mi, fi) and torch.equal(ms, fs)


@pytest.mark.parametrize("case", list(gi.FLATIP_CASES))
def test_vector_db_matches_f64_flatip_restatement(golden, oracle_mod, case):
    """Full reference API path: build_index -> retrieve_batch / retrieve vs the f64
    restatement of faiss IndexFlatIP over the reference's numpy-normalised catalog."""
    from twotower import VectorDatabase

    g = golden("flatip.npz")
    spec = gi.FLATIP_CASES[case]
    x, q = gi.flatip_inputs(spec)
    E = x.shape[1]
    ids = [f"p{j}" for j in range(x.shape[0])]
    vdb = VectorDatabase(E)
    vdb.build_index(x, ids)
    xn = vdb.index.xb[:, :E].cpu().numpy()
    assert gi.sha(np.ascontiguousarray(xn)) == bytes(g[case + "__xn_sha"]).decode()
    res = vdb.retrieve_batch(q, k=spec["k"])
    ref_i, ref_s = g[case + "__i"], g[case + "__s64"]
    k = ref_i.shape[1]
    got_i = np.array([[int(pid[1:]) for pid, _ in r] for r in res])
    got_s = np.array([[sc for _, sc in r] for r in res])
    assert got_i.shape == (q.shape[0], k)
    np.testing.assert_allclose(got_s, ref_s, rtol=0, atol=1e-5)
    assert oracle_mod.topk_parity_f64(got_s.astype(np.float32), got_i, xn, g[case + "__qn"], k) == []
    one = vdb.retrieve(q[0], k=spec["k"])
    assert one == res[0]


def test_vector_db_errors_and_clamp():
    from twotower import VectorDatabase

    vdb = VectorDatabase(384)
    with pytest.raises(ValueError, match="Index not built"):
        vdb.retrieve(np.ones(384, np.float32))
    with pytest.raises(ValueError, match="Embedding dimension mismatch: expected 384, got 128"):
        vdb.build_index(np.ones((3, 128), np.float32), ["a", "b", "c"])
    vdb.build_index(np.eye(5, 384, dtype=np.float32), list("abcde"))
    r = vdb.retrieve(np.eye(5, 384, dtype=np.float32)[2], k=50)
    assert len(r) == 5 and r[0] == ("c", pytest.approx(1.0, abs=1e-6))


def test_vector_db_save_load_roundtrip(tmp_path):
    from twotower import VectorDatabase

    rng = np.random.default_rng(0)
    x = rng.standard_normal((500, 384)).astype(np.float32)
    ids = [f"prod_{i}" for i in range(500)]
    a = VectorDatabase(384)
    a.build_index(x, ids)
    a.save_index(str(tmp_path / "i.faiss"), str(tmp_path / "ids.npy"), str(tmp_path / "m.json"))
    b = VectorDatabase(384)
    b.load_index(str(tmp_path / "i.faiss"), str(tmp_path / "ids.npy"), str(tmp_path / "m.json"))
    assert torch.equal(a.index.xb, b.index.xb) and b.product_ids == ids
    q = rng.standard_normal((5, 384)).astype(np.float32)
    assert a.retrieve_batch(q, 20) == b.retrieve_batch(q, 20)


# ------------------------------------------------------------------ buyer tower
@pytest.mark.parametrize("case", [c for c, s in gi.BUYER_CASES.items()
                                  if s["method"] == "weighted_avg"])
def test_weighted_avg_bit_exact_and_vs_reference(K, oracle_mod, golden, case):
    spec = gi.BUYER_CASES[case]
    items, w = gi.buyer_inputs(spec)
    got = K.weighted_avg_l2(torch.from_numpy(items).cuda(), torch.from_numpy(w).cuda()).cpu().numpy()
    assert np.array_equal(got, oracle_mod.weighted_avg_l2(items, w))
    np.testing.assert_allclose(got, golden("buyer.npz")[case], rtol=0, atol=1e-6)


def test_gather_weighted_avg_bit_exact(K, oracle_mod):
    rng = np.random.default_rng(12)
    table = oracle_mod.l2norm_rows(rng.standard_normal((5000, 384)).astype(np.float32), 1)
    hist = rng.integers(0, 5000, (300, 20))
    hist[:, 15:] = -1
    w = gi.event_weights(rng, (300, 20))
    w[:, 15:] = 0
    out = K.gather_weighted_avg_l2(dev_rows(table), 384, torch.from_numpy(hist).cuda(),
                                   torch.from_numpy(w).cuda()).cpu().numpy()
    assert np.array_equal(out[:, :384], oracle_mod.gather_weighted_avg_l2(table, hist, w))


@pytest.mark.parametrize("d,s", [(64, 3), (128, 70), (640, 5), (1000, 9), (1024, 66)])
def test_weighted_avg_register_shapes_bit_exact(K, oracle_mod, d, s):
    """Every per-lane register shape of k_weighted_avg_l2 (PER 2/6/12/16 elements, 4/2/1 rows
    read ahead), history lengths that are not a multiple of the read-ahead and span two
    64-row chunks, invalid history ids; dense and gathered forms bit-exact vs the oracle."""
    rng = np.random.default_rng(d + s)
    b = 37
    items = rng.standard_normal((b, s, d)).astype(np.float32)
    w = gi.event_weights(rng, (b, s))
    got = K.weighted_avg_l2(torch.from_numpy(items).cuda(), torch.from_numpy(w).cuda()).cpu().numpy()
    assert np.array_equal(got, oracle_mod.weighted_avg_l2(items, w))
    table = rng.standard_normal((500, d)).astype(np.float32)
    hist = rng.integers(-1, 500, (b, s))
    out = K.gather_weighted_avg_l2(torch.from_numpy(table).cuda(), d,  # ld = d (up to 1024)
                                   torch.from_numpy(hist).cuda(),
                                   torch.from_numpy(w).cuda()).cpu().numpy()
    assert np.array_equal(out[:, :d], oracle_mod.gather_weighted_avg_l2(table, hist, w))


@pytest.mark.parametrize("case", [c for c, s in gi.BUYER_CASES.items()
                                  if s["method"] == "attention"])
def test_attention_vs_oracle_and_reference(K, oracle_mod, golden, case):
    spec = gi.BUYER_CASES[case]
    items, w = gi.buyer_inputs(spec)
    W1, b1, W2, b2 = gi.attn_weights(spec)
    t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    got = K.attn_agg_l2(t(items), t(w), t(W1), t(b1), t(W2), t(b2)).cpu().numpy()
    # expf on the device and in libm may differ by an ulp: tolerance, not bit-exact
    np.testing.assert_allclose(got, oracle_mod.attn_agg_l2(items, w, W1, b1, W2, b2),
                               rtol=0, atol=1e-6)
    np.testing.assert_allclose(got, golden("buyer.npz")[case], rtol=0, atol=2e-6)


def test_buyer_tower_module_drop_in(golden):
    """The reference's own unit test (tests/test_buyer_tower.py) run against our module."""
    from twotower import BuyerTower

    for method in ("weighted_avg", "attention"):
        bt = BuyerTower(384, method).eval()
        items = torch.randn(2, 5, 384)
        weights = torch.tensor([[1.0, 5.0, 10.0, 1.0, 1.0], [1.0, 1.0, 5.0, 5.0, 1.0]])
        with torch.no_grad():
            y = bt(items, weights)
        assert y.shape == (2, 384) and y.device.type == "cpu"
        assert torch.allclose(y.norm(dim=1), torch.ones(2), atol=1e-5)
    with pytest.raises(ValueError, match="Unknown aggregation method: mean"):
        BuyerTower(384, "mean")


# ------------------------------------------------------------------ full-size properties
@pytest.mark.slow
def test_scan_full_size_properties(K, oracle_mod):
    """BASELINE config[2] size (1M x 384, k=100): sortedness, exact recomputed scores for the
    returned rows, and completeness against an fp64 GPU GEMV for a query subset."""
    n, d, nq, k = 1_000_000, 384, 64, 100
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn((n, d), generator=g, device="cuda")
    K.l2norm_rows(x, d, 0, out=x)
    q = torch.randn((nq, d), generator=g, device="cuda")
    K.l2norm_rows(q, d, 0, out=q)
    s, i = K.scan_topk(x, n, d, q, k)
    assert torch.all(s[:, :-1] >= s[:, 1:])
    assert torch.all((i >= 0) & (i < n))
    assert all(len(set(r)) == k for r in i.cpu().numpy().tolist())
    xs = x[i.reshape(-1)].cpu().numpy().reshape(nq, k, d)
    qs = q.cpu().numpy()
    for a in range(0, nq, 8):
        for b in range(0, k, 9):
            assert oracle_mod.dot(xs[a, b], qs[a]) == s[a, b].item()
    full = (q[:8].double() @ x.double().T)
    kth = s[:8, -1].double()
    missing = (full > kth[:, None] + 1e-6)
    missing.scatter_(1, i[:8], False)
    assert not missing.any()


def _sharded_search_emulated(K, x, q, W, k, owners=None, between=None):
    """The row-sharded protocol with W shards on one GPU: per-owner begin on the global
    sample, stats 'all-gathered' by concatenation, probe counts 'all-reduced' by summing.
    x, q: host arrays or device row tensors [rows, ep]; between(r, workspace) runs after
    the full stages, before shard r's finish (fault injection)."""
    from twotower.sharded import shard_range

    if isinstance(x, torch.Tensor):
        xd, qd, d = x, q, x.shape[1]
    else:
        xd, qd, d = dev_rows(x), dev_rows(q), x.shape[1]
    n = xd.shape[0]
    nq = qd.shape[0]
    x16 = xd.to(torch.bfloat16)
    sample = K.sharded_sample(x16, n)
    groups = owners or [(r * nq // W, (r + 1) * nq // W) for r in range(W)]
    stats = torch.cat([K.sharded_begin(sample, d, qd[a:b], k) for a, b in groups])
    shards = []
    bmax = torch.zeros(2)
    for r in range(W):
        lo, hi = shard_range(n, r, W)
        bd = torch.tensor(bounds(K, xd[lo:hi], x16[lo:hi], d))
        bmax = torch.maximum(bmax, bd)
        shards.append((lo, hi))
    pcs = [torch.empty((nq, 16), dtype=torch.int32, device="cuda") for _ in range(W)]
    wss = [None] * W
    outs = [None] * W
    # stage 2 on every shard, then the SUM, then stage 3 (split sharded_search by hand)
    from twotower import _lib
    import ctypes

    L, st = _lib.lib(), _lib.stream_ptr()
    for r, (lo, hi) in enumerate(shards):
        wss[r] = torch.empty(K.sharded_workspace_bytes(hi - lo, d, nq, k), dtype=torch.uint8,
                             device="cuda")
        _lib.check(L.tt_sharded_filter_full(
            x16[lo:].data_ptr(), hi - lo, d, x16.stride(0), qd.data_ptr(), nq, qd.stride(0), k,
            ctypes.c_float(bmax[0]), ctypes.c_float(bmax[1]), stats.data_ptr(), pcs[r].data_ptr(),
            wss[r].data_ptr(), wss[r].numel(), st, None, None), "full")
    total = torch.stack(pcs).sum(0, dtype=torch.int32)
    for r, (lo, hi) in enumerate(shards):
        if between is not None:
            between(r, wss[r])
        s_ = torch.empty((nq, k), device="cuda")
        i_ = torch.empty((nq, k), device="cuda", dtype=torch.int64)
        _lib.check(L.tt_sharded_filter_finish(
            xd[lo:].data_ptr(), x16[lo:].data_ptr(), hi - lo, d, xd.stride(0), lo, qd.data_ptr(),
            nq, qd.stride(0), k, stats.data_ptr(), total.data_ptr(), s_.data_ptr(), i_.data_ptr(),
            wss[r].data_ptr(), wss[r].numel(), st), "finish")
        outs[r] = (s_, i_)
    fb = [K.filter_fallback_count(wss[r], hi - lo, d, nq, k, sharded=True)
          for r, (lo, hi) in enumerate(shards)]
    ms, mi = K.merge_topk(torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs]), k)
    return ms.cpu().numpy(), mi.cpu().numpy(), fb


@pytest.mark.parametrize("W,n,nq,k", [(2, 300000, 64, 100), (8, 1000000, 40, 100),
                                      (3, 5000, 17, 64), (4, 2000, 9, 10), (8, 70000, 33, 128)])
def test_sharded_filter_protocol_bit_exact(K, oracle_mod, W, n, nq, k):
    """tt_sharded_filter_* on W row shards of one catalog (collectives done by hand on one
    GPU) + merge == the single-catalog exact top-k, bit for bit; few fallbacks on iid data."""
    rng = np.random.default_rng(W * 1000 + nq)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, 384)).astype(np.float32), 0)
    x[n // 2: n // 2 + 50] = x[:50]  # duplicates across shards
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, 384)).astype(np.float32), 0)
    ms, mi, fb = _sharded_search_emulated(K, x, q, W, k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(mi, ri) and np.array_equal(ms, rs)
    if n >= 100000:
        assert max(fb) <= nq // 10, fb


def test_sharded_filter_clustered_and_nan(K, oracle_mod):
    """Near-duplicate clusters (tiny score gaps: probes land inside eps) and a NaN query:
    still bit-exact (fallbacks allowed)."""
    rng = np.random.default_rng(7)
    n, W, k = 60000, 4, 100
    c = rng.standard_normal((30, 384)).astype(np.float32)
    x = c[rng.integers(0, 30, n)] + 1e-3 * rng.standard_normal((n, 384)).astype(np.float32)
    x = oracle_mod.l2norm_rows(x, 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((12, 384)).astype(np.float32), 0)
    q[3] = np.nan
    ms, mi, _ = _sharded_search_emulated(K, x, q, W, k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    ok = np.arange(12) != 3
    assert np.array_equal(mi[ok], ri[ok]) and np.array_equal(ms[ok], rs[ok])


def test_sharded_finish_wave_list_overflow_is_reduced(K, oracle_mod):
    """A shard keeping more band rows for a query than the wave re-rank's list (k_rerank_wave,
    256 keys) scores the list and keeps its top k, then goes on appending (was: the query took
    the shard's exact f32 fallback): ~600 near-copies of query 0 in shard 0 all land within
    2 eps of the k-th score -- three reductions.  Results stay bit-exact and no shard falls
    back."""
    rng = np.random.default_rng(31)
    n, W, k, nq = 40000, 2, 100, 6
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, 384)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, 384)).astype(np.float32), 0)
    # scattered over shard 0 (rows < n / W) so that no (query, slab) candidate list overflows
    rows = rng.choice(n // W, 600, replace=False)
    x[rows] = oracle_mod.l2norm_rows(
        q[:1] + 1e-4 * rng.standard_normal((600, 384)).astype(np.float32), 0)
    ms, mi, fb = _sharded_search_emulated(K, x, q, W, k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(mi, ri) and np.array_equal(ms, rs)
    assert sum(fb) == 0, fb


def test_sharded_finish_corrupt_band_row_falls_back(K, oracle_mod):
    """Bounds check of decoded candidate rows (k_rerank_wave): a band key whose row decodes
    past the shard (here row 0xffffffff, planted in the workspace between the full and finish
    stages) is never read -- the query takes that shard's exact f32 fallback instead, and the
    merged result stays bit-exact with no fault."""
    rng = np.random.default_rng(41)
    n, W, k, nq = 50000, 2, 100, 8
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, 384)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, 384)).astype(np.float32), 0)
    from twotower.sharded import shard_range

    planted = {}

    def corrupt(r, ws):
        if r != 0:
            return
        lo, hi = shard_range(n, 0, W)
        lay = K.filter_workspace_layout(hi - lo, 384, nq, k, sharded=True)
        band_n = ws[lay["band_n"]:lay["band_n"] + 4 * nq].view(torch.int32)
        qi = int(torch.argmax(band_n).item())
        assert int(band_n[qi]) > 0
        keys = ws[lay["band"]:lay["band"] + 8 * nq * lay["band_cap"]].view(torch.int64)
        e0 = qi * lay["band_cap"]
        # the band is unordered and entries below the cut are dropped undecoded: corrupt the
        # best-scoring entry (always kept)
        mine = keys[e0:e0 + int(band_n[qi])].cpu().numpy().view(np.uint64)
        e = e0 + int(np.argmax(mine))
        keys[e] = keys[e] & ~0xFFFFFFFF  # low word 0 -> row ~0 = 0xffffffff
        planted["q"] = qi

    ms, mi, fb = _sharded_search_emulated(K, x, q, W, k, between=corrupt)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(mi, ri) and np.array_equal(ms, rs)
    assert fb[0] >= 1 and "q" in planted


@pytest.mark.parametrize("where,n,nq", [(1, 100000, 300), (1, 300000, 2100), (2, 100000, 1),
                                         (2, 1000000, 3)])
def test_bf16_filter_corrupt_key_falls_back(K, oracle_mod, where, n, nq):
    """Bounds check of decoded candidate rows on the single-GPU paths (tt_debug_plant_bad_row
    corrupts one query's best candidate key on the device so that its row decodes to
    0xffffffff): where 1 = a band key between the full level and k_rerank (the large-batch
    path), 2 = an exact key between k_filter_topm and k_final_topm (the one-buyer single pass).
    The row is never read: the query takes the exact f32 fallback, every result stays
    bit-exact, nothing faults; the hook is one-shot (the next call takes no fallback)."""
    from twotower import _lib

    rng = np.random.default_rng(n + nq + where)
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, 384)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, 384)).astype(np.float32), 0)
    db, qd = dev_rows(x), dev_rows(q)
    db16 = db.to(torch.bfloat16)
    b = bounds(K, db, db16, 384)
    k = 100
    ws = torch.empty(K.filter_workspace_bytes(n, 384, nq, k), dtype=torch.uint8, device="cuda")
    sub = np.unique(np.linspace(0, nq - 1, min(nq, 64)).round().astype(int))
    qi = int(sub[len(sub) // 2])
    rs, ri = oracle_mod.scan_topk(x, q[sub], k)
    for planted in (True, False):
        if planted:
            _lib.check(_lib.lib().tt_debug_plant_bad_row(where, qi), "plant")
        s, i = K.scan_topk_bf16(db, db16, n, 384, qd, k, b, workspace=ws)
        fb = K.filter_fallback_count(ws, n, 384, nq, k)
        assert np.array_equal(i.cpu().numpy()[sub], ri)
        assert np.array_equal(s.cpu().numpy()[sub], rs)
        assert fb == (1 if planted else 0), (planted, fb)


def test_plant_hook_disarmed_by_a_call_on_another_path(K, oracle_mod):
    """The hook armed for the single pass (where 2) but spent on a call that takes the
    multi-level path (nq > 4) is disarmed by that call: a later one-buyer search takes no
    fallback (an armed hook must not outlive the call it was meant for)."""
    from twotower import _lib

    rng = np.random.default_rng(77)
    n, k = 100000, 100
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, 384)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((40, 384)).astype(np.float32), 0)
    db, qd = dev_rows(x), dev_rows(q)
    db16 = db.to(torch.bfloat16)
    b = bounds(K, db, db16, 384)
    ws = torch.empty(K.filter_workspace_bytes(n, 384, 40, k), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.lib().tt_debug_plant_bad_row(2, 0), "plant")
    K.scan_topk_bf16(db, db16, n, 384, qd, k, b, workspace=ws)      # multi-level path
    assert K.filter_fallback_count(ws, n, 384, 40, k) == 0
    s, i = K.scan_topk_bf16(db, db16, n, 384, qd[:1], k, b, workspace=ws)  # single pass
    assert K.filter_fallback_count(ws, n, 384, 1, k) == 0
    rs, ri = oracle_mod.scan_topk(x, q[:1], k)
    assert np.array_equal(i.cpu().numpy(), ri) and np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("E,S", [(384, 20), (768, 20), (768, 100), (1024, 20)])
def test_attn_agg_batched_gemm_form_vs_oracle(K, oracle_mod, E, S):
    """tt_attn_agg_l2_f32_ws (the batched form: first MLP layer on the f32 MFMA GEMM, then the
    per-buyer softmax / weighted sum / F.normalize) vs the C oracle and the one-kernel form:
    within 1e-6 (only the first layer's summation order differs), buyer_tower.py:70-101."""
    rng = np.random.default_rng(E + S)
    B, H = 300, 128
    items = oracle_mod.l2norm_rows(rng.standard_normal((B * S, E)).astype(np.float32),
                                   1).reshape(B, S, E)
    w = np.where(rng.random((B, S)) < 0.75, 1.0, np.where(rng.random((B, S)) < 0.7, 5.0, 10.0))
    w = w.astype(np.float32)
    w[3, S // 2:] = 0.0  # zero-weight padding positions
    W1 = (rng.standard_normal((H, E)) / np.sqrt(E)).astype(np.float32)
    b1 = (0.1 * rng.standard_normal(H)).astype(np.float32)
    W2 = (rng.standard_normal((1, H)) / np.sqrt(H)).astype(np.float32)
    b2 = (0.1 * rng.standard_normal(1)).astype(np.float32)
    t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    got = K.attn_agg_l2(t(items), t(w), t(W1), t(b1), t(W2), t(b2), fused=False).cpu().numpy()
    one = K.attn_agg_l2(t(items), t(w), t(W1), t(b1), t(W2), t(b2), fused=True).cpu().numpy()
    ref = oracle_mod.attn_agg_l2(items, w, W1, b1, W2, b2)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6)
    np.testing.assert_allclose(got, one, rtol=0, atol=1e-6)
