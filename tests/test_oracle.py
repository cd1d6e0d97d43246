"""Pin the CPU oracle (oracle/) against the reference's own outputs (tests/golden/).

The oracle is trusted only after these pass: the HIP parity tests compare against it.
"""
import json
import os

import numpy as np
import pytest

import inputs as gi


# ------------------------------------------------------------------ numpy norm (vector_db)
@pytest.mark.parametrize("d", [1, 3, 7, 8, 13, 64, 100, 128, 129, 200, 257, 384, 768, 1000, 1536])
def test_oracle_norm_bit_exact_vs_numpy(oracle_mod, d):
    rng = np.random.default_rng(d)
    x = (rng.standard_normal((64, d)) * rng.uniform(0.01, 100, (64, 1))).astype(np.float32)
    ref = oracle_mod.vector_db_normalize(x)  # the reference's numpy expression
    got = oracle_mod.l2norm_rows(x, 0)
    assert np.array_equal(got, ref)


def test_oracle_fnormalize_close_to_torch(oracle_mod):
    import torch
    import torch.nn.functional as F

    rng = np.random.default_rng(0)
    x = rng.standard_normal((128, 384)).astype(np.float32)
    ref = F.normalize(torch.from_numpy(x), p=2, dim=1).numpy()
    got = oracle_mod.l2norm_rows(x, 1)
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-7)
    z = oracle_mod.l2norm_rows(np.zeros((2, 384), np.float32), 1)  # F.normalize(0) == 0
    assert np.all(z == 0)


# ------------------------------------------------------------------ flat IP (faiss restatement)
@pytest.mark.parametrize("case", list(gi.FLATIP_CASES))
def test_oracle_scan_vs_f64_fixture(oracle_mod, golden, case):
    g = golden("flatip.npz")
    spec = gi.FLATIP_CASES[case]
    x, q = gi.flatip_inputs(spec)
    xn = oracle_mod.l2norm_rows(x, 0)
    assert gi.sha(xn) == bytes(g[case + "__xn_sha"]).decode()  # normalisation == reference's
    qn = g[case + "__qn"]
    assert np.array_equal(oracle_mod.l2norm_rows(q, 0), qn)
    k = min(spec["k"], x.shape[0])
    s, i = oracle_mod.scan_topk(xn, qn, k)
    ref_s, ref_i = g[case + "__s64"], g[case + "__i"]
    assert s.shape == ref_s.shape
    np.testing.assert_allclose(s, ref_s, rtol=0, atol=1e-5)
    assert oracle_mod.topk_parity_f64(s, i, xn, qn, k) == []
    if spec.get("dups"):
        # exact ties: lower row first -> identical ids to the f64 lexsort order
        assert np.array_equal(i, ref_i)


def test_oracle_dot_is_canonical_fma_chain(oracle_mod):
    rng = np.random.default_rng(3)
    for d in (16, 100, 384):
        x = rng.standard_normal(d).astype(np.float32)
        q = rng.standard_normal(d).astype(np.float32)
        acc = np.float32(0)
        dp = (d + 15) // 16 * 16
        xp = np.zeros(dp, np.float32); xp[:d] = x
        qp = np.zeros(dp, np.float32); qp[:d] = q
        for t in range(dp // 16):
            for i in range(4):
                for g in range(4):
                    e = 16 * t + 4 * g + i
                    acc = np.float32(np.float64(xp[e]) * np.float64(qp[e]) + np.float64(acc))
        # fp64 fma emulation is exact for f32 operands (product exact in f64, one rounding)
        assert oracle_mod.dot(x, q) == acc


# ------------------------------------------------------------------ buyer tower
@pytest.mark.parametrize("case", [c for c, s in gi.BUYER_CASES.items()
                                  if s["method"] == "weighted_avg"])
def test_oracle_weighted_avg_vs_reference(oracle_mod, golden, case):
    g = golden("buyer.npz")
    spec = gi.BUYER_CASES[case]
    items, w = gi.buyer_inputs(spec)
    assert gi.sha(items, w) == bytes(g[case + "__sha"]).decode()
    got = oracle_mod.weighted_avg_l2(items, w)
    ref = g[case]
    # torch's CPU reduction order differs from the canonical sequential one: a few ulp
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6)
    if spec.get("w") != "zero":
        np.testing.assert_allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-5)
    else:
        assert np.all(got == 0) and np.all(ref == 0)


@pytest.mark.parametrize("case", [c for c, s in gi.BUYER_CASES.items()
                                  if s["method"] == "attention"])
def test_oracle_attention_vs_reference(oracle_mod, golden, case):
    g = golden("buyer.npz")
    spec = gi.BUYER_CASES[case]
    items, w = gi.buyer_inputs(spec)
    assert gi.sha(items, w) == bytes(g[case + "__sha"]).decode()
    W1, b1, W2, b2 = gi.attn_weights(spec)
    got = oracle_mod.attn_agg_l2(items, w, W1, b1, W2, b2)
    np.testing.assert_allclose(got, g[case], rtol=0, atol=2e-6)


@pytest.mark.parametrize("case", list(gi.BUYER_CASES))
def test_oracle_buyer_f64_vs_reference(golden, case):
    """The float64 buyer restatements (the Mode A / encode_buyer envelope tests' reference)
    against the reference BuyerTower's own float32 outputs: within its f32 rounding."""
    from oracle import oracle as O

    g = golden("buyer.npz")
    spec = gi.BUYER_CASES[case]
    items, w = gi.buyer_inputs(spec)
    if spec["method"] == "weighted_avg":
        got = O.weighted_avg_l2_f64(items, w)
    else:
        got = O.attn_agg_l2_f64(items, w, *gi.attn_weights(spec))
    np.testing.assert_allclose(got, g[case], rtol=0, atol=1e-6)


def test_oracle_gather_equals_dense(oracle_mod):
    rng = np.random.default_rng(5)
    table = rng.standard_normal((500, 384)).astype(np.float32)
    hist = rng.integers(0, 500, (6, 20))
    hist[:, -3:] = -1  # padding
    w = gi.event_weights(rng, (6, 20))
    w[:, -3:] = 0
    dense = np.where(hist[..., None] >= 0, table[np.maximum(hist, 0)], 0).astype(np.float32)
    assert np.array_equal(oracle_mod.gather_weighted_avg_l2(table, hist, w),
                          oracle_mod.weighted_avg_l2(dense, w))


# ------------------------------------------------------------------ host logic vs reference
def test_event_weights_match_reference(golden):
    from twotower.config import DEFAULT_CONFIG, get_event_weight

    with open(os.path.join(os.path.dirname(__file__), "golden", "event_weights.json")) as f:
        table = json.load(f)
    for name, wgt in table.items():
        assert get_event_weight(name, DEFAULT_CONFIG) == wgt, name


def test_oracle_i8_tile_layout():
    """oracle.i8_tile against the layout's definition chunk by chunk (the tiled int8 image of
    tt_i8_tile: piece s of 16-row block b holds, at byte 16 l, row 16 b + l % 16's codes
    64 s + 16 (l // 16) .. + 15; rows past n zero)."""
    from oracle import oracle as O

    rng = np.random.default_rng(0)
    for n, e in ((37, 384), (16, 768), (1, 64)):
        c = rng.integers(-127, 128, (n, e)).astype(np.int8)
        t = O.i8_tile(c, n)
        nb = (n + 15) // 16
        assert t.size == nb * 16 * e
        for ch in range(nb * e):
            b, wi = divmod(ch, e)
            s, lane = wi >> 6, wi & 63
            row, off = 16 * b + (lane & 15), 64 * s + 16 * (lane >> 4)
            exp = c[row, off:off + 16] if row < n else np.zeros(16, np.int8)
            assert np.array_equal(t[16 * ch:16 * ch + 16], exp), (n, e, ch)
