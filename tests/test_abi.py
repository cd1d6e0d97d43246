"""C-ABI checks that need no GPU: the library loads, exports every symbol the header
declares, and rejects bad arguments before touching the device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "twotower_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tt_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def L():
    from twotower import _lib

    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ("tt_scan_topk_f32", "tt_topk_merge_f32", "tt_l2norm_rows_f32",
                 "tt_weighted_avg_l2_f32", "tt_gather_weighted_avg_l2_f32", "tt_attn_agg_l2_f32",
                 "tt_scan_workspace_bytes", "tt_padded_dim", "tt_last_error", "tt_version",
                 "tt_scan_topk_bf16f32", "tt_bf16_image_bounds", "tt_bert_encode", "tt_gemm_f32",
                 "tt_gemm_bf16", "tt_gemm_ln_bf16", "tt_layernorm_f32", "tt_attention_varlen_f32", "tt_item_concat"):
        assert name in fns


def test_library_exports_every_header_symbol(L):
    from twotower import _lib

    for name in header_functions():
        assert hasattr(L, name), f"{name} declared in include/twotower_hip.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature in _lib.py"


def test_version_and_padded_dim(L):
    assert L.tt_version() >= 100
    assert [L.tt_padded_dim(d) for d in (1, 64, 65, 100, 384, 385, 768, 769)] == \
        [64, 64, 128, 128, 384, 512, 768, -1]


def test_i8_tiled_bytes(L):
    """tt_i8_tiled_bytes: whole 16-row blocks of the padded dim (host arithmetic only)."""
    assert [L.tt_i8_tiled_bytes(n, 384) for n in (1, 16, 17, 1_000_000)] == \
        [16 * 384, 16 * 384, 32 * 384, 1_000_000 * 384]
    assert L.tt_i8_tiled_bytes(5, 768) == 16 * 768
    assert L.tt_i8_tiled_bytes(5, 900) == -1 and L.tt_i8_tiled_bytes(-1, 384) == -1


def test_invalid_arguments_rejected_without_device(L):
    from twotower._lib import check

    rc = L.tt_scan_topk_f32(None, 0, 384, 384, 0, None, 1, 384, 10, None, None, None, 0, None)
    assert rc == -1 and b"empty catalog" in L.tt_last_error()
    rc = L.tt_scan_topk_f32(None, 100, 384, 384, 0, None, 1, 384, 101, None, None, None, 0, None)
    assert rc == -1 and b"k <= n" in L.tt_last_error()
    rc = L.tt_scan_topk_f32(None, 100, 900, 900, 0, None, 1, 900, 10, None, None, None, 0, None)
    assert rc == -3
    rc = L.tt_l2norm_rows_f32(None, 10, 384, 100, None, 384, None, 0, None)
    assert rc == -1
    rc = L.tt_weighted_avg_l2_f32(None, 4, 0, 384, None, None, 384, None)
    assert rc == -1
    with pytest.raises(RuntimeError, match="status -1"):
        check(L.tt_l2norm_rows_f32(None, 1, 384, 100, None, 384, None, 0, None), "norm")
    b = ctypes.c_int64(0)
    assert L.tt_scan_workspace_bytes(1_000_000, 384, 10_000, 100, ctypes.byref(b)) == 0
    assert b.value > 10_000 * 100 * 8


def test_product_path_has_no_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import numpy as np
    from twotower import BuyerTower, HipUnavailable, VectorDatabase

    db = VectorDatabase(384)
    with pytest.raises(HipUnavailable):
        db.build_index(np.ones((4, 384), np.float32), ["a", "b", "c", "d"])
    bt = BuyerTower(384, "weighted_avg")
    with pytest.raises(HipUnavailable):
        bt(torch.ones(1, 3, 384), torch.ones(1, 3))


def test_shipped_library_reads_no_ab_switches():
    """The A/B kernel switches are read from the environment only in timing builds
    (-DTT_TIMING_BUILD): the shipped library always runs the path the GPU suite tests."""
    from twotower import _lib

    raw = open(_lib.LIB_PATH, "rb").read()
    for name in (b"TT_GEMM_LN", b"TT_GEMM_LN96", b"TT_ATTN_FAST", b"TT_GEMM_WIDE", b"TT_GEMM_BIG",
                 b"TT_SELECT_REG", b"TT_FILTER_TMAX_FIRST"):
        assert name not in raw, name
