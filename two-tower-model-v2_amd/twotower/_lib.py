"""Loader for libtwotower_hip.so (the C ABI declared in include/twotower_hip.h).

The library is built in-tree (two-tower-model-v2_amd/lib/) by csrc/Makefile and bound with
ctypes.  ``import torch`` happens first so the library's libamdhip64.so.7 dependency
resolves to the HIP runtime torch already loaded.  There is no CPU fallback:
if the library is missing or no HIP device is visible, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("TWOTOWER_HIP_LIB") or os.path.join(_PKG_ROOT, "lib", "libtwotower_hip.so")
CSRC = os.path.join(_PKG_ROOT, "csrc")

TT_OK = 0
TT_ERR_INVALID, TT_ERR_LAUNCH, TT_ERR_UNSUPPORTED, TT_ERR_WORKSPACE = -1, -2, -3, -4
TT_SHARD_PROBES = 16  # include/twotower_hip.h
TT_SHARD_SAMPLE_STRIDE = 16
TT_NORM_ADD_EPS = 0
TT_NORM_MAX_EPS = 1

_lock = threading.Lock()
_lib = None

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32

TT_PREC_F32 = 0
TT_PREC_BF16 = 1
TT_PREC_X3 = 2  # f32 operands, split-bf16 (hi + lo) MFMA products
TT_ACT_NONE, TT_ACT_GELU, TT_ACT_RELU = 0, 1, 2


class BertLayer(ctypes.Structure):
    """tt_bert_layer (include/twotower_hip.h): device pointers of one BertLayer."""
    _fields_ = [(n, _vp) for n in (
        "wqkv", "bqkv", "wo", "bo", "ln1_g", "ln1_b", "w1", "b1", "w2", "b2", "ln2_g", "ln2_b",
        "wqkv_bf16", "wo_bf16", "w1_bf16", "w2_bf16", "wqkv_x3", "wo_x3", "w1_x3", "w2_x3",
        "wqkv_x3i", "wo_x3i", "w1_x3i", "w2_x3i")]


class BertModel(ctypes.Structure):
    """tt_bert_model (include/twotower_hip.h)."""
    _fields_ = [("vocab", _i32), ("hidden", _i32), ("heads", _i32), ("intermediate", _i32),
                ("layers", _i32), ("max_positions", _i32), ("ln_eps", ctypes.c_float),
                ("word_emb", _vp), ("pos_emb", _vp), ("type_emb", _vp), ("emb_ln_g", _vp),
                ("emb_ln_b", _vp), ("layer", ctypes.POINTER(BertLayer))]


class ConvertJob(ctypes.Structure):
    """tt_convert_job (include/twotower_hip.h): one operand copy of tt_convert_batch."""
    _fields_ = [("src", _vp), ("ld_src", _i64), ("rows", _i32), ("cols", _i32), ("dst", _vp),
                ("ld_dst", _i64), ("transpose", _i32), ("to_bf16", _i32), ("row_ids", _vp)]


class TnPending(ctypes.Structure):
    """tt_tn_pending (include/twotower_hip.h): one deferred tt_gemm_tn_partial reduce."""
    _fields_ = [("workspace", _vp), ("M", _i64), ("N", _i32), ("K", _i32), ("C", _vp),
                ("ldc", _i64), ("db", _vp)]


# name -> (restype, argtypes); mirrors include/twotower_hip.h
SIGNATURES = {
    "tt_version": (ctypes.c_int, []),
    "tt_last_error": (ctypes.c_char_p, []),
    "tt_padded_dim": (_i32, [_i32]),
    "tt_l2norm_rows_f32": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i64, _vp, _i32, _vp]),
    "tt_scan_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_scan_topk_f32": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i64, _vp, _i32, _i64, _i32, _vp,
                                        _vp, _vp, _i64, _vp]),
    "tt_scan_topk_f32_timed": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i64, _vp, _i32, _i64, _i32,
                                              _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "tt_scan_topk_f32_select": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i64, _vp, _i32, _i64,
                                               _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "tt_select_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_scan_topk_select_f32": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i64, _vp, _i32, _i64,
                                               _i32, _vp, _vp, _vp, _i64, _vp]),
    "tt_filter_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, _i32,
                                                 ctypes.POINTER(_i64)]),
    "tt_filter_fallback_offset": (ctypes.c_int, [_i64, _i32, _i32, _i32,
                                                 ctypes.POINTER(_i64)]),
    "tt_scan_topk_bf16f32": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i64, _i64, _vp, _i32, _i64,
                                            _i32, ctypes.c_float, ctypes.c_float, _vp, _vp, _vp,
                                            _i64, _vp, _vp, _vp]),
    "tt_scan_topk_bf16f32_i8s": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, _i64, _i64, _i64,
                                                _vp, _i32, _i64, _i32, ctypes.c_float,
                                                ctypes.c_float, _vp, _vp, _vp, _i64, _vp, _vp,
                                                _vp]),
    "tt_sharded_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_sharded_fallback_offset": (ctypes.c_int, [_i64, _i32, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_filter_workspace_layout": (ctypes.c_int, [_i64, _i32, _i32, _i32, _i32,
                                                  ctypes.POINTER(_i64)]),
    "tt_sharded_filter_begin": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _i64, _i32, _vp,
                                               _vp, _i64, _vp]),
    "tt_sharded_filter_full": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _i64, _i32,
                                              ctypes.c_float, ctypes.c_float, _vp, _vp, _vp, _i64,
                                              _vp, _vp, _vp]),
    "tt_sharded_filter_finish": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i64, _i64, _vp, _i32,
                                                _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "tt_bf16_image_bounds": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i64, _vp, _vp]),
    "tt_i8_image": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i64, _vp, _vp, _vp]),
    "tt_scan_topk_i8f32": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i64, _i64, _i64, _vp, _i32,
                                          _i64, _i32, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_float, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "tt_scan_topk_i8t_f32": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i64, _i64, _vp, _i32,
                                            _i64, _i32, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "tt_i8_tiled_bytes": (ctypes.c_int64, [_i64, _i32]),
    "tt_i8t_single_pass_ok": (ctypes.c_int, [_i64, _i32, _i32, _i32]),
    "tt_i8_tile": (ctypes.c_int, [_vp, _i64, _i64, _i32, _vp, _vp]),
    "tt_topk_merge_f32": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp]),
    "tt_weighted_avg_l2_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _i64, _vp]),
    "tt_gather_weighted_avg_l2_f32": (ctypes.c_int, [_vp, _i64, _i64, _i32, _vp, _vp, _i64,
                                                     _i32, _vp, _i64, _vp]),
    "tt_attn_agg_l2_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp,
                                          _vp, _i64, _vp]),
    "tt_attn_agg_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_attn_agg_l2_f32_ws": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp,
                                             _vp, _i64, _vp, _i64, _vp]),
    "tt_bert_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_bert_encode": (ctypes.c_int, [ctypes.POINTER(BertModel), _vp, _vp, _i32, _i64, _i32, _i32,
                                      _vp, _i64, _vp, _i64, _vp]),
    "tt_gemm_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64,
                                   _i32, _i32, _i32, _i32, _vp]),
    "tt_gemm_x3": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64,
                                  _i32, _i32, _i32, _i32, _vp]),
    "tt_gemm_x3w": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64,
                                   _i32, _i32, _i32, _i32, _vp]),
    "tt_x3_split_weights": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _i64, _vp]),
    "tt_debug_plant_bad_row": (ctypes.c_int, [_i32, _i32]),
    "tt_debug_last_sample_i8": (ctypes.c_int, []),
    "tt_i8_single_pass_ok": (ctypes.c_int, [_i64, _i32, _i32, _i32, _i64]),
    "tt_debug_i8_force_unsupported": (ctypes.c_int, [_i32]),
    "tt_attention_varlen_x3i": (ctypes.c_int, [_vp, _i64, _vp, _i32, _i32, _i32, _i32, _vp, _i64,
                                               _vp]),
    "tt_x3i_weights": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _i64, _vp]),
    "tt_gemm_x3i": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32, _i32, _i32, _i32,
                                   _vp]),
    "tt_gemm_ln_x3i": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, ctypes.c_float, _vp,
                                       _i64, _vp, _i64, _i32, _i32, _i32, _vp]),
    "tt_gemm_bf16": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64,
                                    _i32, _i32, _i32, _i32, _vp]),
    "tt_gemm_ln_bf16": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, ctypes.c_float, _vp,
                                        _i64, _vp, _i64, _i32, _i32, _i32, _vp]),
    "tt_layernorm_f32": (ctypes.c_int, [_vp, _i64, _vp, _vp, ctypes.c_float, _vp, _i64, _vp, _i64,
                                        _i64, _i32, _vp]),
    "tt_attention_varlen": (ctypes.c_int, [_vp, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i64,
                                           _vp, _vp]),
    "tt_attention_varlen_bf16": (ctypes.c_int, [_vp, _i64, _vp, _i32, _i32, _i32, _i32, _vp, _i64,
                                                _vp, _vp]),
    "tt_attention_varlen_f32": (ctypes.c_int, [_vp, _i64, _vp, _i32, _i32, _i32, _i32, _vp, _i64,
                                               _vp, _vp]),
    "tt_infonce_workspace_bytes": (ctypes.c_int, [_i32, _i32, _i32, _i32, _i32,
                                                  ctypes.POINTER(_i64)]),
    "tt_infonce_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32,
                                      ctypes.c_float, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "tt_l2norm_backward_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _vp,
                                              _i64, _vp]),
    "tt_transpose_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _i32, _vp]),
    "tt_col_sum_f32": (ctypes.c_int, [_vp, _i64, _i64, _i32, _vp, _i32, _vp]),
    "tt_relu_backward_f32": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "tt_dropout_apply_f32": (ctypes.c_int, [_vp, _vp, ctypes.c_float, _i64, _vp]),
    "tt_attn_pool_fwd_f32": (ctypes.c_int, [_vp, _i32, _vp, ctypes.c_float, _vp, _vp, _i64, _i32,
                                            _i32, _vp, _vp, _vp, _i64, _vp]),
    "tt_attn_pool_bwd_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _i32,
                                            _i32, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "tt_embedding_backward_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i32, _vp, _vp]),
    "tt_adam_f32": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_float, ctypes.c_float, _i32, _vp]),
    "tt_f32_to_bf16": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _i64, _vp]),
    "tt_attn_pool_fwd_f32_dev": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i64, _i32, _i32,
                                                _vp, _vp, _vp, _i64, _vp, _vp]),
    "tt_dropout_rng_f32": (ctypes.c_int, [_vp, _i64, ctypes.c_float, ctypes.c_uint64, _vp, _vp,
                                          _vp]),
    "tt_embedding_backward2_f32": (ctypes.c_int, [_vp, _i64, _vp, _vp, _i64, _i32, _vp, _vp,
                                                  _vp]),
    "tt_infonce_ex": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32,
                                     ctypes.c_float, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                     _i64, _vp, _i64, _vp]),
    "tt_attn_pool_bwd_relu_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64,
                                                 _i32, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _vp,
                                                 _vp]),
    "tt_gemm_tn_workspace_bytes": (ctypes.c_int, [_i64, _i32, _i32, ctypes.POINTER(_i64)]),
    "tt_gemm_tn_partial": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _vp,
                                          _i64, _vp, _vp, _i64, _vp]),
    "tt_gemm_tn_reduce_many": (ctypes.c_int, [_vp, _i32, _vp]),
    "tt_train_bwd_tail": (ctypes.c_int, [_vp, _i32, _vp, _i64, _i32, _vp, _vp, _vp, _i64, _vp,
                                         _vp, _i64, _i32, _vp, _vp, _vp]),
    "tt_attn_pool_bwd_relu_parts_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp,
                                                       _i64, _i32, _i32, _vp, _vp, _i32, _vp,
                                                       _vp, _vp]),
    "tt_gemm_tn": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _vp, _i64, _vp,
                                  _vp, _i64, _vp]),
    "tt_dropout_apply_ex": (ctypes.c_int, [_vp, _vp, ctypes.c_float, _i64, _vp, _vp]),
    "tt_relu_dropout_backward_f32": (ctypes.c_int, [_vp, _vp, ctypes.c_float, _i64, _vp, _vp,
                                                    _vp]),
    "tt_l2norm_backward_ex": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32, _vp,
                                             _i64, _vp, _i64, _vp]),
    "tt_convert_batch": (ctypes.c_int, [ctypes.POINTER(ConvertJob), _i32, _vp]),
    "tt_item_concat": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _i64,
                                      _vp, _vp]),
}


class HipUnavailable(RuntimeError):
    """Raised when the HIP library or a HIP device is missing (no silent fallback)."""


def build(verbose: bool = False) -> str:
    """Compile csrc/ for gfx950 into lib/libtwotower_hip.so (hipcc cross-compiles on CPU)."""
    subprocess.run(["make", "-C", CSRC] + ([] if verbose else ["-s"]), check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipUnavailable(
                    f"{LIB_PATH} not built; run `make -C {CSRC}` (or __graft_entry__.build())")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != TT_OK:
        msg = lib().tt_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def require_device(t: "torch.Tensor", name: str) -> None:
    if not t.is_cuda:
        raise HipUnavailable(f"{name} must be a HIP device tensor (got {t.device})")


def device() -> "torch.device":
    if not torch.cuda.is_available():
        raise HipUnavailable("no HIP device visible: the two-tower hot path runs only on MI355X")
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def padded_dim(d: int) -> int:
    """Row length of the device catalog / query layout: tt_padded_dim(d) (64 ... 768, the scan
    and bf16-filter kernels' instantiations), or for d > 768 the next multiple of 64 -- rows
    that only the generic exact path (kernels.scan_topk_large: f32 MFMA GEMM + key top-k)
    searches.  The reference accepts any embedding_dim (vector_db.py:13,48)."""
    if int(d) < 1:
        raise ValueError(f"embedding dim must be >= 1, got {d}")
    ep = lib().tt_padded_dim(int(d))
    return ep if ep > 0 else (int(d) + 63) // 64 * 64


def scan_kernel_dim(d: int) -> bool:
    """True when the scan / bf16-filter kernels take dimension d (<= 768)."""
    return lib().tt_padded_dim(int(d)) > 0


class StreamWorkspaces:
    """Device scratch buffers keyed by the current HIP stream, least-recently-used first out
    (at most ``maxsize`` kept).  Kernels on one stream are ordered, so a workspace per stream
    never races; an evicted buffer returns to torch's caching allocator, whose blocks are
    reused on the stream that freed them only, so in-flight work on it stays safe."""

    def __init__(self, maxsize: int = 4):
        import collections

        self._d = collections.OrderedDict()
        self.maxsize = maxsize

    def get(self, need: int, device) -> "torch.Tensor":
        st = stream_ptr()
        ws = self._d.pop(st, None)
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 1), dtype=torch.uint8, device=device)
        self._d[st] = ws
        while len(self._d) > self.maxsize:
            self._d.popitem(last=False)
        return ws

    def __len__(self) -> int:
        return len(self._d)
