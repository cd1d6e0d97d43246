"""Parity of the large-batch bf16 filter path: more than RG_SMALL_NQ = 2048 queries per launch,
so the full-catalog level is the k_filter_ring<EP, 1> instantiation (tt_filter.hip:1717) that
bench.py's headline number runs -- the retrieve_batch pattern of configs[2]
(reference src/inference/vector_db.py:171-209, 10k buyers per batch).

Bar: bit-exact ids and scores.  Oracles: the C restatement (oracle.scan_topk, canonical f32,
threaded over queries) for every query where that finishes in seconds, and the exact f32
MFMA scan (tt_scan_topk_f32, itself bit-exact vs the C oracle in test_gpu_parity.py) for
every query of the full-size case, plus a C-oracle subset there."""
import numpy as np
import pytest
import torch

from test_gpu_parity import _sharded_search_emulated, bounds, dev_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from twotower import kernels

    return kernels


def _bf16_search(K, xd, n, d, qd, k, i8=False):
    """i8: the catalog also holds its int8 image, so a large batch at padded dim 384 runs its
    sample level on it (k_sample_i8; tt_scan_topk_bf16f32_i8s) -- asserted taken."""
    from twotower import _lib

    x16 = xd.to(torch.bfloat16)
    ws = torch.empty(K.filter_workspace_bytes(n, d, qd.shape[0], k), dtype=torch.uint8,
                     device="cuda")
    img = K.i8_image(xd, d) if i8 else None
    s, i = K.scan_topk_bf16(xd, x16, n, d, qd, k, bounds(K, xd, x16, d), workspace=ws, i8=img)
    torch.cuda.synchronize()
    if i8:
        assert _lib.lib().tt_debug_last_sample_i8() == int(_lib.padded_dim(d) == 384)
    return s, i, K.filter_fallback_count(ws, n, d, qd.shape[0], k)


def _iid(oracle_mod, rng, n, nq, d=384):
    x = oracle_mod.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    return x, q


def test_large_batch_threshold_is_crossed():
    """The cases below only test the LVL-1 kernel if they exceed its batch threshold."""
    import re
    import os

    src = open(os.path.join(os.path.dirname(__file__), "..", "two-tower-model-v2_amd", "csrc",
                            "tt_filter.hip")).read()
    assert int(re.search(r"constexpr int RG_SMALL_NQ = (\d+);", src).group(1)) == 2048


@pytest.mark.parametrize("i8", [False, True])
@pytest.mark.parametrize("nq", [2049, 4096])
def test_large_batch_iid_bit_exact_vs_oracle(K, oracle_mod, nq, i8):
    """n = 100k, k = 100: every query bit-exact vs the C oracle (2049 = one query past the
    threshold, a 1-query ragged last tile; 4096 = 16 full 256-query tiles); with and without
    the int8 sample level."""
    rng = np.random.default_rng(nq)
    n, d, k = 100_000, 384, 100
    x, q = _iid(oracle_mod, rng, n, nq)
    s, i, fb = _bf16_search(K, dev_rows(x), n, d, dev_rows(q), k, i8=i8)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)
    assert fb == 0  # iid data: the optimistic thresholds hold


@pytest.mark.parametrize("i8", [False, True])
def test_large_batch_clustered_bit_exact(K, oracle_mod, i8):
    """Near-duplicate clusters (tiny score gaps, band overflow -> exact fallback for some
    queries) and queries that sit on a cluster centre, nq = 4096 (ragged n)."""
    rng = np.random.default_rng(101)
    n, d, nq, k = 100_003, 384, 4096, 100
    c = rng.standard_normal((200, d)).astype(np.float32)
    x = c[rng.integers(0, 200, n)] + 2e-3 * rng.standard_normal((n, d)).astype(np.float32)
    x = oracle_mod.l2norm_rows(x, 0)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    q[::3] = c[rng.integers(0, 200, len(q[::3]))]
    q = oracle_mod.l2norm_rows(q, 0)
    s, i, fb = _bf16_search(K, dev_rows(x), n, d, dev_rows(q), k, i8=i8)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("i8", [False, True])
def test_large_batch_duplicates_and_special_queries(K, oracle_mod, i8):
    """Exact duplicate rows (ties on both scores -> lower row first), zero queries (all scores
    0: rows 0..k-1), a NaN catalog row, a NaN query, nq = 4096."""
    rng = np.random.default_rng(102)
    n, d, nq, k = 60_000, 384, 4096, 128
    base = oracle_mod.l2norm_rows(rng.standard_normal((n // 4, d)).astype(np.float32), 0)
    x = np.concatenate([base] * 4)
    x[777] = np.nan
    q = oracle_mod.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    q[::5] = base[rng.integers(0, n // 4, len(q[::5]))]
    q[17] = 0.0
    q[4095] = 0.0
    q[2222, 3] = np.nan  # every slot (-inf, -1), as the f32 scan
    s, i, fb = _bf16_search(K, dev_rows(x), n, d, dev_rows(q), k, i8=i8)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    gi = i.cpu().numpy()
    assert np.array_equal(gi, ri)
    assert np.array_equal(s.cpu().numpy(), rs)
    assert np.array_equal(gi[17], np.arange(k)) and not np.isin(777, gi).any()


@pytest.mark.parametrize("d,k", [(128, 50), (500, 64), (700, 128), (768, 100)])
def test_large_batch_other_dims(K, oracle_mod, d, k):
    """Other padded widths of the same instantiation family (E = 128 32-row tiles; E = 512 and
    768 16-row tiles with two query blocks per wave, d = 500 / 700 zero-padded to them)."""
    rng = np.random.default_rng(d + 7)
    n, nq = 50_000, 2500
    x, q = _iid(oracle_mod, rng, n, nq, d)
    s, i, _ = _bf16_search(K, dev_rows(x), n, d, dev_rows(q), k)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.slow
@pytest.mark.parametrize("i8", [False, True])
def test_configs2_full_size_bit_exact(K, oracle_mod, i8):
    """configs[2] exactly as bench.py runs it: 1M x 384 catalog, 10k queries, k = 100 (with and
    without the int8 sample level).  Every query bit-exact vs the exact f32 MFMA scan; 64
    queries (spread over all 40 query tiles, incl. the 16-query last tile) bit-exact vs the C
    oracle; no fallbacks."""
    n, d, nq, k = 1_000_000, 384, 10_000, 100
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn((n, d), generator=g, device="cuda")
    K.l2norm_rows(x, d, 0, out=x)
    q = torch.randn((nq, d), generator=g, device="cuda")
    K.l2norm_rows(q, d, 0, out=q)
    s, i, fb = _bf16_search(K, x, n, d, q, k, i8=i8)
    fs, fi = K.scan_topk(x, n, d, q, k)
    assert fb == 0
    assert torch.equal(i, fi), int((i != fi).any(dim=1).sum())
    assert torch.equal(s, fs)
    sub = np.unique(np.concatenate([np.linspace(0, nq - 1, 60).astype(int),
                                    [255, 256, 9983, 9999]]))
    rs, ri = oracle_mod.scan_topk(x.cpu().numpy(), q[sub].cpu().numpy(), k)
    assert np.array_equal(i[sub].cpu().numpy(), ri)
    assert np.array_equal(s[sub].cpu().numpy(), rs)


def _flagged_scenario(K, n_picked):
    """1M x 384, 10k queries, k = 100; n_picked queries (spread over the batch) each sit on a
    cluster of 1500 near-copies, so their band overflows BAND_CAP and exactly those take the
    exact f32 fallback.  Every other query is orthogonal to the picked ones (a cluster of 1500
    equal scores inside a query's top-k band overflows it too; iid queries reach it at ~1e-3
    per query), and the picked queries are orthonormal."""
    n, d, nq = 1_000_000, 384, 10_000
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn((n, d), generator=g, device="cuda")
    q = torch.randn((nq, d), generator=g, device="cuda")
    K.l2norm_rows(q, d, 0, out=q)
    picked = np.unique(np.linspace(17, nq - 2, n_picked).astype(int)).tolist()
    basis = torch.linalg.qr(q[picked].T.cpu())[0].cuda()
    q[picked] = basis.T.contiguous()  # picked queries orthonormal: no cross-cluster bands
    rest = torch.ones(nq, dtype=torch.bool, device="cuda")
    rest[picked] = False
    q[rest] -= (q[rest] @ basis) @ basis.T
    K.l2norm_rows(q, d, 0, out=q)
    step = (n - 100_000) // len(picked)
    for j, qi in enumerate(picked):
        rows = torch.arange(100_000 + step * j, 100_000 + step * j + 1500, device="cuda")
        x[rows] = q[qi] + 1e-3 * torch.randn((1500, d), generator=g, device="cuda")
    K.l2norm_rows(x, d, 0, out=x)
    x16 = x.to(torch.bfloat16)
    # the same batch with the clustered queries replaced by iid ones (orthogonal already)
    q2 = q.clone()
    q2[picked] = q[[1, 2, 3] * (len(picked) // 3) + [1, 2, 3][:len(picked) % 3]]
    return x, x16, q, q2, picked


@pytest.mark.slow
@pytest.mark.parametrize("n_picked", [3, 40])
def test_configs2_flagged_queries_fallback_bit_exact(K, oracle_mod, n_picked):
    """A few (3: one 16-query tile of the adaptive fallback) or more (40: three tiles) flagged
    queries of a 10k batch (tt_scan.hip k_scan_fallback / k_merge_fallback: the flagged slots
    are spread over the whole chip on the device): exactly those fall back, bit-exact."""
    n, d, k = 1_000_000, 384, 100
    x, x16, q, q2, picked = _flagged_scenario(K, n_picked)
    ws = torch.empty(K.filter_workspace_bytes(n, d, q.shape[0], k), dtype=torch.uint8,
                     device="cuda")
    bnd = bounds(K, x, x16, d)
    s, i = K.scan_topk_bf16(x, x16, n, d, q, k, bnd, workspace=ws)
    torch.cuda.synchronize()
    assert K.filter_fallback_count(ws, n, d, q.shape[0], k) == len(picked)
    fs, fi = K.scan_topk(x, n, d, q, k)
    assert torch.equal(i, fi) and torch.equal(s, fs)
    sub = picked[:8] + [0, 5000, 9999]
    rs, ri = oracle_mod.scan_topk(x.cpu().numpy(), q[sub].cpu().numpy(), k)
    assert np.array_equal(i[sub].cpu().numpy(), ri)
    assert np.array_equal(s[sub].cpu().numpy(), rs)
    K.scan_topk_bf16(x, x16, n, d, q2, k, bnd, workspace=ws)
    torch.cuda.synchronize()
    assert K.filter_fallback_count(ws, n, d, q.shape[0], k) == 0


@pytest.mark.slow
def test_sharded_protocol_large_batch_w8(K, oracle_mod):
    """The W = 8 staged sharded filter with W.B = 4096 queries per rank launch (> 2048: the
    per-shard full level is the large-batch instantiation), 1M rows: merged results bit-exact
    vs the single-catalog f32 scan (all queries) and the C oracle (a subset)."""
    rng = np.random.default_rng(8)
    n, nq, k, W = 1_000_000, 4096, 100, 8
    x, q = _iid(oracle_mod, rng, n, nq)
    x[n // 2: n // 2 + 50] = x[:50]  # duplicates across shards
    ms, mi, fb = _sharded_search_emulated(K, x, q, W, k)
    fs, fi = K.scan_topk(dev_rows(x), n, 384, dev_rows(q), k)
    assert np.array_equal(mi, fi.cpu().numpy())
    assert np.array_equal(ms, fs.cpu().numpy())
    assert max(fb) <= nq // 100, fb
    sub = np.arange(0, nq, 97)
    rs, ri = oracle_mod.scan_topk(x, q[sub], k)
    assert np.array_equal(mi[sub], ri) and np.array_equal(ms[sub], rs)


@pytest.mark.slow
@pytest.mark.parametrize("nq", [1, 4096])
def test_10m_rows_single_gpu_bit_exact(K, oracle_mod, nq):
    """configs[3]'s whole 10M x 384 catalog resident on ONE MI355X (15.4 GB f32 + 7.7 GB bf16
    image): the bf16 filter path bit-exact vs the f32 scan for every query, and vs the C
    oracle for a 16-query subset."""
    n, d, k = 10_000_000, 384, 100
    g = torch.Generator(device="cuda").manual_seed(10)
    x = torch.randn((n, d), generator=g, device="cuda")
    K.l2norm_rows(x, d, 0, out=x)
    q = torch.randn((nq, d), generator=g, device="cuda")
    K.l2norm_rows(q, d, 0, out=q)
    s, i, fb = _bf16_search(K, x, n, d, q, k)
    fs, fi = K.scan_topk(x, n, d, q, k)
    assert fb == 0
    assert torch.equal(i, fi) and torch.equal(s, fs)
    sub = np.unique(np.linspace(0, nq - 1, 16).astype(int))
    rs, ri = oracle_mod.scan_topk(x.cpu().numpy(), q[sub].cpu().numpy(), k)
    assert np.array_equal(i[sub].cpu().numpy(), ri)
    assert np.array_equal(s[sub].cpu().numpy(), rs)


@pytest.mark.slow
def test_sharded_protocol_10m_w8(K, oracle_mod):
    """configs[3] layout emulated on one GPU: 10M rows in 8 row shards (1.25M each), the
    staged protocol for W.B = 2048 queries, merged == the single-catalog f32 scan."""
    n, nq, k, W = 10_000_000, 2048, 100, 8
    g = torch.Generator(device="cuda").manual_seed(11)
    xd = torch.randn((n, 384), generator=g, device="cuda")
    K.l2norm_rows(xd, 384, 0, out=xd)
    qd = torch.randn((nq, 384), generator=g, device="cuda")
    K.l2norm_rows(qd, 384, 0, out=qd)
    x, q = xd.cpu().numpy(), qd.cpu().numpy()
    fs, fi = K.scan_topk(xd, n, 384, qd, k)
    del xd
    torch.cuda.empty_cache()
    ms, mi, fb = _sharded_search_emulated(K, x, q, W, k)
    assert np.array_equal(mi, fi.cpu().numpy())
    assert np.array_equal(ms, fs.cpu().numpy())
    assert max(fb) <= nq // 100, fb
