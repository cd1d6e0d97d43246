"""Tensor-level wrappers over the C ABI (include/twotower_hip.h).

Every function takes/returns HIP device tensors, launches on torch's current stream and
never synchronises.  Shapes and dtypes are validated here so that a bad call raises a
Python exception instead of reaching a kernel with inconsistent sizes.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check, lib, require_device, stream_ptr

_f32 = torch.float32


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _check_2d(t, name, dtype=_f32):
    require_device(t, name)
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be 2-D with unit column stride, got {tuple(t.shape)}")


def alloc_rows(n: int, d: int, device=None) -> torch.Tensor:
    """[n, tt_padded_dim(d)] zero-initialised float32 (the scan's row layout)."""
    ep = _lib.padded_dim(d)
    return torch.zeros((n, ep), dtype=_f32, device=device or _lib.device())


def l2norm_rows(x: torch.Tensor, d: int, mode: int, out: torch.Tensor = None,
                out_bf16: torch.Tensor = None) -> torch.Tensor:
    """Row-normalise the first d columns of x; padding columns of out are zeroed."""
    _check_2d(x, "x")
    if out is None:
        out = torch.empty_like(x)
    _check_2d(out, "out")
    if out.shape[0] != x.shape[0] or out.shape[1] < d or x.shape[1] < d:
        raise ValueError("l2norm_rows: shape mismatch")
    if out_bf16 is not None:
        if out_bf16.shape != out.shape or out_bf16.dtype != torch.bfloat16:
            raise ValueError("out_bf16 must be bf16 with out's shape")
    check(lib().tt_l2norm_rows_f32(_ptr(x), x.shape[0], d, x.stride(0), _ptr(out), out.stride(0),
                                   _ptr(out_bf16), mode, stream_ptr()), "tt_l2norm_rows_f32")
    return out


def scan_workspace_bytes(n: int, d: int, nq: int, k: int) -> int:
    b = ctypes.c_int64(0)
    check(lib().tt_scan_workspace_bytes(n, d, nq, k, ctypes.byref(b)), "tt_scan_workspace_bytes")
    return b.value


def scan_topk(db: torch.Tensor, n: int, d: int, q: torch.Tensor, k: int, row_base: int = 0,
              workspace: torch.Tensor = None, out=None):
    """Exact top-k of q @ db[:n].T -> (scores [nq,k] f32, rows [nq,k] int64 = row_base + row)."""
    _check_2d(db, "db")
    _check_2d(q, "q")
    nq = q.shape[0]
    if not (1 <= k <= n <= db.shape[0]):
        raise ValueError(f"scan_topk: need 1 <= k ({k}) <= n ({n}) <= rows ({db.shape[0]})")
    if out is None:
        out = (torch.empty((nq, k), dtype=_f32, device=q.device),
               torch.empty((nq, k), dtype=torch.int64, device=q.device))
    if nq == 0:
        return out
    need = scan_workspace_bytes(n, d, nq, k)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    check(lib().tt_scan_topk_f32(_ptr(db), n, d, db.stride(0), row_base, _ptr(q), nq, q.stride(0),
                                 k, _ptr(out[0]), _ptr(out[1]), _ptr(workspace), workspace.numel(),
                                 stream_ptr()), "tt_scan_topk_f32")
    return out


def select_workspace_bytes(n: int, nq: int, k: int) -> int:
    b = ctypes.c_int64(0)
    check(lib().tt_select_workspace_bytes(n, nq, k, ctypes.byref(b)), "tt_select_workspace_bytes")
    return b.value


def scan_topk_select(db: torch.Tensor, n: int, d: int, q: torch.Tensor, k: int, row_base: int = 0,
                     workspace: torch.Tensor = None, out=None):
    """scan_topk's results (bit-identical) by scores-then-radix-select (tt_scan_topk_select_f32):
    the path for FILTER_KMAX < k <= SCAN_KMAX, ~25x the per-slab-list scan at k = 1000."""
    _check_2d(db, "db")
    _check_2d(q, "q")
    nq = q.shape[0]
    if not (1 <= k <= n <= db.shape[0]):
        raise ValueError(f"scan_topk_select: need 1 <= k ({k}) <= n ({n}) <= rows ({db.shape[0]})")
    if out is None:
        out = (torch.empty((nq, k), dtype=_f32, device=q.device),
               torch.empty((nq, k), dtype=torch.int64, device=q.device))
    if nq == 0:
        return out
    need = select_workspace_bytes(n, nq, k)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    check(lib().tt_scan_topk_select_f32(_ptr(db), n, d, db.stride(0), row_base, _ptr(q), nq,
                                        q.stride(0), k, _ptr(out[0]), _ptr(out[1]),
                                        _ptr(workspace), workspace.numel(), stream_ptr()),
          "tt_scan_topk_select_f32")
    return out


FILTER_KMAX = 128
SCAN_KMAX = 1024  # tt_scan_topk_f32's / tt_scan_topk_select_f32's largest k; larger: scan_topk_large


def scan_topk_large(db: torch.Tensor, n: int, d: int, q: torch.Tensor, k: int, row_base: int = 0,
                    chunk_elems: int = 1 << 25):
    """Generic exact top-k: any k (faiss' IndexFlatIP takes any k <= ntotal; the reference's
    /retrieve caps k at 1000, server.py:46, VectorDatabase.retrieve does not) and any dimension
    (rows past 768 dims, which the scan kernels do not instantiate; vector_db.py:13,48 accept
    any embedding_dim).  Every score by tt_gemm_f32 -- the f32 MFMA GEMM whose k order IS the
    canonical fma order of the scan, so the scores are the scan's bits --
    then a top-k over 64-bit keys (orderable(score) << 32 | ~row: score descending, ties to
    the lower row, exactly the scan's order).  NaN scores are never returned: their slots read
    (-inf, -1) at the end of the list, as in the scan.  Queries in chunks of at most
    chunk_elems scores: a chunk holds its f32 scores plus ~4 int64 temporaries of the same
    shape (bits, orderable, key, the where result), ~36 B per score -- 1.2 GB at 2^25.  Not the serving path (k <= 128, d <= 768 take the bf16 filter)."""
    _check_2d(db, "db")
    _check_2d(q, "q")
    nq, ep = q.shape[0], db.shape[1]
    if not (1 <= k <= n <= db.shape[0]) or q.shape[1] != ep or ep % 32 != 0:
        raise ValueError(f"scan_topk_large: need 1 <= k ({k}) <= n ({n}), q [nq, {ep}], "
                         "row length % 32 == 0")
    out_s = torch.empty((nq, k), dtype=_f32, device=q.device)
    out_i = torch.empty((nq, k), dtype=torch.int64, device=q.device)
    step = max(1, min(nq, chunk_elems // max(n, 1)))
    rows = torch.arange(n, device=q.device, dtype=torch.int64)
    low = 0xFFFFFFFF - rows  # ~row in the low word: ties -> the lower row first
    for a in range(0, nq, step):
        b = min(nq, a + step)
        sc = torch.empty((b - a, n), dtype=_f32, device=q.device)
        check(lib().tt_gemm_f32(_ptr(q[a:b]), q.stride(0), _ptr(db), db.stride(0), None, None, 0,
                                _ptr(sc), sc.stride(0), None, 0, b - a, n, ep, 0, stream_ptr()),
              "tt_gemm_f32")
        bits = sc.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        # orderable: negative floats flipped, positive with the sign bit set; NaN -> 0 (last)
        orderable = torch.where(bits >= 0x80000000, 0xFFFFFFFF - bits, bits + 0x80000000)
        nan = torch.isnan(sc)
        orderable = orderable.masked_fill(nan, 0)
        key = ((orderable - 0x80000000) << 32) | low  # signed: the order of (orderable, ~row)
        top = torch.topk(key, k, dim=1, largest=True, sorted=True).values
        r = 0xFFFFFFFF - (top & 0xFFFFFFFF)
        bad = torch.gather(nan, 1, r)
        out_s[a:b] = torch.gather(sc, 1, r).masked_fill(bad, float("-inf"))
        out_i[a:b] = (r + row_base).masked_fill(bad, -1)
        del sc, bits, orderable, key
    return out_s, out_i


def bf16_image_bounds(x: torch.Tensor, x16: torch.Tensor, d: int, out2: torch.Tensor = None):
    """Max-combine (max ||x_r||, max ||x_r - x16_r||) upper bounds into out2 (device [2] f32).

    These catalog bounds set the bf16 filter's per-query error bound (tt_scan_topk_bf16f32)."""
    _check_2d(x, "x")
    _check_2d(x16, "x16", torch.bfloat16)
    if x16.shape != x.shape or x16.stride(0) != x.stride(0):
        raise ValueError("x16 must be the bf16 image of x (same shape and leading dim)")
    if out2 is None:
        out2 = torch.zeros(2, dtype=_f32, device=x.device)
    check(lib().tt_bf16_image_bounds(_ptr(x), _ptr(x16), x.shape[0], d, x.stride(0), _ptr(out2),
                                     stream_ptr()), "tt_bf16_image_bounds")
    return out2


def filter_workspace_bytes(n: int, d: int, nq: int, k: int) -> int:
    b = ctypes.c_int64(0)
    check(lib().tt_filter_workspace_bytes(n, d, nq, k, ctypes.byref(b)),
          "tt_filter_workspace_bytes")
    return b.value


def filter_fallback_count(workspace: torch.Tensor, n: int, d: int, nq: int, k: int,
                          sharded: bool = False) -> int:
    """Queries of the last scan_topk_bf16 (sharded=True: sharded_search) call with this
    workspace that took the exact fallback.  Diagnostic: synchronises."""
    off = ctypes.c_int64(0)
    fn = lib().tt_sharded_fallback_offset if sharded else lib().tt_filter_fallback_offset
    check(fn(n, d, nq, k, ctypes.byref(off)), "fallback_offset")
    return int(workspace[off.value:off.value + 4].view(torch.int32).item())


def filter_workspace_layout(n: int, d: int, nq: int, k: int, sharded: bool = False) -> dict:
    """Byte offsets of the band keys / counts, fallback flags and fallback count inside a
    filter workspace (tt_filter_workspace_layout; diagnostic, for tests)."""
    off = (ctypes.c_int64 * 5)()
    check(lib().tt_filter_workspace_layout(n, d, nq, k, int(sharded), off),
          "tt_filter_workspace_layout")
    return {"band": off[0], "band_n": off[1], "flags": off[2], "fallback_count": off[3],
            "band_cap": off[4]}


def scan_topk_bf16(db: torch.Tensor, db16: torch.Tensor, n: int, d: int, q: torch.Tensor,
                   k: int, bounds, row_base: int = 0, workspace: torch.Tensor = None,
                   out=None, events=(None, None), i8=None):
    """Exact top-k (bit-identical to scan_topk) via the bf16 filter + f32 re-rank (k <= 128).

    bounds = (x_norm_max, x_resid_max) host floats, e.g. bf16_image_bounds(...).tolist().
    i8 = (codes, tile scales[, bounds]) from i8_image: a large batch at padded dim 384 then runs
    its sample level on the int8 image (tt_scan_topk_bf16f32_i8s; same results)."""
    x_norm_max, x_resid_max = (float(v) for v in bounds)
    _check_2d(db, "db")
    _check_2d(db16, "db16", torch.bfloat16)
    _check_2d(q, "q")
    if db16.shape[0] < n or db16.stride(0) != db.stride(0):
        raise ValueError("db16 must be the bf16 image of db (same rows and leading dim)")
    nq = q.shape[0]
    if not (1 <= k <= min(n, FILTER_KMAX)) or n > db.shape[0]:
        raise ValueError(f"scan_topk_bf16: need 1 <= k ({k}) <= min(n, 128), n <= rows")
    if out is None:
        out = (torch.empty((nq, k), dtype=_f32, device=q.device),
               torch.empty((nq, k), dtype=torch.int64, device=q.device))
    if nq == 0:
        return out
    need = filter_workspace_bytes(n, d, nq, k)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    e0, e1 = events
    ev = (e0.cuda_event if e0 is not None else None, e1.cuda_event if e1 is not None else None)
    if i8 is not None:
        codes, scales = i8[0], i8[1]
        if codes.dtype != torch.int8 or codes.dim() != 2 or codes.shape[0] < n:
            raise ValueError("i8 codes must be the int8 image [n, ep] of db (i8_image)")
        check(lib().tt_scan_topk_bf16f32_i8s(
            _ptr(db), _ptr(db16), _ptr(codes), _ptr(scales), n, d, db.stride(0),
            codes.stride(0), row_base, _ptr(q), nq, q.stride(0), k, ctypes.c_float(x_norm_max),
            ctypes.c_float(x_resid_max), _ptr(out[0]), _ptr(out[1]), _ptr(workspace),
            workspace.numel(), stream_ptr(), *ev), "tt_scan_topk_bf16f32_i8s")
        return out
    check(lib().tt_scan_topk_bf16f32(
        _ptr(db), _ptr(db16), n, d, db.stride(0), row_base, _ptr(q), nq, q.stride(0), k,
        ctypes.c_float(x_norm_max), ctypes.c_float(x_resid_max), _ptr(out[0]), _ptr(out[1]), _ptr(workspace), workspace.numel(),
        stream_ptr(), *ev), "tt_scan_topk_bf16f32")
    return out


I8_DIMS = (384, 768)  # padded dims of the int8 single pass (tt_scan_topk_i8f32)
I8_NQ_MAX = 8  # nq 5-8: the 8-query buffer layout (still ahead of the multi-level path)
_i8_ok_cache = {}


def i8_single_pass_ok(n: int, d: int, nq: int, k: int, ld_i8: int = 0) -> bool:
    """Whether tt_scan_topk_i8f32 runs this shape (tt_i8_single_pass_ok: nq <= 8, k <= 128,
    padded dim 384 / 768, rows per CU <= 65536, <= 256 CUs) -- else the caller takes the bf16
    filter (tt_scan_topk_bf16f32), which it would otherwise return TT_ERR_UNSUPPORTED for."""
    key = (n, d, nq, k, ld_i8)
    v = _i8_ok_cache.get(key)
    if v is None:
        if len(_i8_ok_cache) > 4096:
            _i8_ok_cache.clear()
        v = _i8_ok_cache[key] = bool(lib().tt_i8_single_pass_ok(n, d, nq, k, ld_i8))
    return v


def debug_i8_force_unsupported(on: bool) -> None:
    """Test hook (tt_debug_i8_force_unsupported): make the int8 single pass report every shape
    unsupported, as on a > 256-CU GPU or past its row limit."""
    check(lib().tt_debug_i8_force_unsupported(1 if on else 0), "tt_debug_i8_force_unsupported")
    _i8_ok_cache.clear()
    _i8t_ok_cache.clear()


def i8_image(x: torch.Tensor, d: int, out3: torch.Tensor = None):
    """The int8 image of a normalised catalog x [n, ep] f32 (tt_i8_image): codes [n, ep] int8,
    per-64-row-tile scales [ceil(n / 64)] f32 and the bounds (max ||x||, max ||x - s n||,
    max s ||n||) max-combined into out3 (device [3] f32)."""
    _check_2d(x, "x")
    n, ep = x.shape
    codes = torch.empty((n, ep), dtype=torch.int8, device=x.device)
    scales = torch.empty(max((n + 63) // 64, 1), dtype=_f32, device=x.device)
    if out3 is None:
        out3 = torch.zeros(3, dtype=_f32, device=x.device)
    check(lib().tt_i8_image(_ptr(x), n, d, x.stride(0), _ptr(codes), codes.stride(0),
                            _ptr(scales), _ptr(out3), stream_ptr()), "tt_i8_image")
    return codes, scales, out3


I8T_DIMS = (384,)  # padded dims of the tiled int8 image's register-fed stream
I8T_NQ_MAX = 32  # queries of the tiled int8 single pass (two 16-query MFMA blocks)
_i8t_ok_cache = {}


def i8t_single_pass_ok(n: int, d: int, nq: int, k: int) -> bool:
    """Whether tt_scan_topk_i8t_f32 (the tiled image, nq <= 32) runs this shape."""
    key = (n, d, nq, k)
    v = _i8t_ok_cache.get(key)
    if v is None:
        if len(_i8t_ok_cache) > 4096:
            _i8t_ok_cache.clear()
        v = _i8t_ok_cache[key] = bool(lib().tt_i8t_single_pass_ok(n, d, nq, k))
    return v


def i8_pass_ok(n: int, d: int, nq: int, k: int, i8) -> bool:
    """Whether an int8 single pass serves nq queries with this int8 image tuple (codes, scales,
    bounds[, tiled]): the tiled stream for nq <= 32 at padded dim 384, else the ring one for
    nq <= 8 at 384 / 768."""
    if i8 is None:
        return False
    if len(i8) > 3 and i8[3] is not None and _lib.padded_dim(d) in I8T_DIMS:
        return nq <= I8T_NQ_MAX and i8t_single_pass_ok(n, d, nq, k)
    return nq <= I8_NQ_MAX and i8_single_pass_ok(n, d, nq, k, i8[0].stride(0))


def i8_tile(codes: torch.Tensor, n: int, d: int) -> torch.Tensor:
    """The tiled int8 image (tt_i8_tile) of i8_image's codes: per 16-row block E / 64 pieces of
    1 KB in MFMA operand order, for scan_topk_i8(tiled=...) / PreparedSearch at padded dim 384."""
    if codes.dtype != torch.int8 or codes.dim() != 2 or codes.shape[0] < n:
        raise ValueError("codes must be the int8 image [n, ep] (i8_image)")
    nbytes = lib().tt_i8_tiled_bytes(n, d)
    if nbytes < 0:
        raise ValueError(f"i8_tile: padded dim of d = {d} is not a multiple of 64")
    tiled = torch.empty(max(nbytes, 16), dtype=torch.int8, device=codes.device)
    check(lib().tt_i8_tile(_ptr(codes), codes.stride(0), n, d, _ptr(tiled), stream_ptr()),
          "tt_i8_tile")
    return tiled


def scan_topk_i8(db: torch.Tensor, codes: torch.Tensor, scales: torch.Tensor, n: int, d: int,
                 q: torch.Tensor, k: int, bounds3, row_base: int = 0,
                 workspace: torch.Tensor = None, out=None, events=(None, None), tiled=None):
    """Exact top-k (bit-identical to scan_topk) for nq <= 8 through the int8 single pass
    (tt_scan_topk_i8f32): padded dim 384 / 768, k <= 128.  bounds3 = i8_image's out3 as host
    floats.  tiled = i8_tile(codes, ...) at padded dim 384: the register-fed stream over the
    tiled image (tt_scan_topk_i8t_f32, same results)."""
    _check_2d(db, "db")
    _check_2d(q, "q")
    if codes.dtype != torch.int8 or codes.dim() != 2 or codes.shape[0] < n:
        raise ValueError("codes must be the int8 image [n, ep] of db (i8_image)")
    nq = q.shape[0]
    nq_max = I8T_NQ_MAX if tiled is not None and _lib.padded_dim(d) in I8T_DIMS else I8_NQ_MAX
    if not (1 <= k <= min(n, FILTER_KMAX)) or nq > nq_max:
        raise ValueError(f"scan_topk_i8: need 1 <= k ({k}) <= min(n, 128) and nq <= {nq_max}")
    if out is None:
        out = (torch.empty((nq, k), dtype=_f32, device=q.device),
               torch.empty((nq, k), dtype=torch.int64, device=q.device))
    if nq == 0:
        return out
    need = filter_workspace_bytes(n, d, nq, k)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    X, R, S = (float(v) for v in bounds3)
    e0, e1 = events
    ev = (e0.cuda_event if e0 is not None else None, e1.cuda_event if e1 is not None else None)
    if tiled is not None and _lib.padded_dim(d) in I8T_DIMS:
        if tiled.dtype != torch.int8 or tiled.numel() < lib().tt_i8_tiled_bytes(n, d):
            raise ValueError("tiled must be i8_tile(codes, n, d)")
        check(lib().tt_scan_topk_i8t_f32(
            _ptr(db), _ptr(tiled), _ptr(scales), n, d, db.stride(0), row_base, _ptr(q), nq,
            q.stride(0), k, ctypes.c_float(X), ctypes.c_float(R), ctypes.c_float(S),
            _ptr(out[0]), _ptr(out[1]), _ptr(workspace), workspace.numel(), stream_ptr(), *ev),
            "tt_scan_topk_i8t_f32")
        return out
    check(lib().tt_scan_topk_i8f32(
        _ptr(db), _ptr(codes), _ptr(scales), n, d, db.stride(0), codes.stride(0), row_base,
        _ptr(q), nq, q.stride(0), k, ctypes.c_float(X), ctypes.c_float(R), ctypes.c_float(S),
        _ptr(out[0]), _ptr(out[1]), _ptr(workspace), workspace.numel(), stream_ptr(), *ev),
        "tt_scan_topk_i8f32")
    return out


class PreparedSearch:
    """scan_topk_bf16 for a fixed (catalog, nq, k): validation, workspace, output buffers and
    the C arguments are set up once, so a call is one ctypes call (the serving pattern: the
    /retrieve path searches one buyer at a time, server.py:241-244 -> vector_db.py:160).

    Returns the same (scores, ids) tensors on every call (overwritten in place)."""

    def __init__(self, db: torch.Tensor, db16: torch.Tensor, n: int, d: int, nq: int, k: int,
                 bounds, row_base: int = 0, i8=None):
        """i8 = (codes, scales, bounds3[, tiled]) from i8_image (+ i8_tile): nq <= 8 at padded
        dim 384 / 768 then runs the int8 single pass (tt_scan_topk_i8f32; with the tiled image
        at 384, tt_scan_topk_i8t_f32 -- same results)."""
        _check_2d(db, "db")
        _check_2d(db16, "db16", torch.bfloat16)
        if db16.shape[0] < n or db16.stride(0) != db.stride(0):
            raise ValueError("db16 must be the bf16 image of db (same rows and leading dim)")
        if not (1 <= k <= min(n, FILTER_KMAX)) or n > db.shape[0] or nq < 1:
            raise ValueError(f"PreparedSearch: need nq >= 1, 1 <= k ({k}) <= min(n, 128)")
        self.db, self.db16, self.nq, self.d = db, db16, nq, d
        dev = db.device
        self.out = (torch.empty((nq, k), dtype=_f32, device=dev),
                    torch.empty((nq, k), dtype=torch.int64, device=dev))
        self.ws = torch.empty(filter_workspace_bytes(n, d, nq, k), dtype=torch.uint8, device=dev)
        self.ld_q = _lib.padded_dim(d)
        self._fn = lib().tt_scan_topk_bf16f32
        x_norm_max, x_resid_max = (float(v) for v in bounds)
        self._head = (_ptr(db), _ptr(db16), n, d, db.stride(0), row_base)
        self._tail = (k, ctypes.c_float(x_norm_max), ctypes.c_float(x_resid_max),
                      _ptr(self.out[0]), _ptr(self.out[1]), _ptr(self.ws), self.ws.numel())
        self.i8 = self.ld_q in I8_DIMS and i8_pass_ok(n, d, nq, k, i8)
        if self.i8:
            codes, scales, b3 = i8[:3]
            tiled = i8[3] if len(i8) > 3 else None
            X, R, S = (float(v) for v in b3)
            self._keep = (codes, scales, tiled)
            if tiled is not None and self.ld_q in I8T_DIMS:
                self._fn = lib().tt_scan_topk_i8t_f32
                self._head = (_ptr(db), _ptr(tiled), _ptr(scales), n, d, db.stride(0), row_base)
            else:
                self._fn = lib().tt_scan_topk_i8f32
                self._head = (_ptr(db), _ptr(codes), _ptr(scales), n, d, db.stride(0),
                              codes.stride(0), row_base)
            self._tail = (k, ctypes.c_float(X), ctypes.c_float(R), ctypes.c_float(S),
                          _ptr(self.out[0]), _ptr(self.out[1]), _ptr(self.ws), self.ws.numel())

    def __call__(self, q: torch.Tensor):
        if (q.shape != (self.nq, self.ld_q) or q.dtype != _f32 or q.device != self.db.device
                or not q.is_contiguous()):
            raise ValueError(f"PreparedSearch: q must be a contiguous f32 [{self.nq}, "
                             f"{self.ld_q}] tensor on {self.db.device}")
        rc = self._fn(*self._head, q.data_ptr(), self.nq, self.ld_q, *self._tail,
                      torch.cuda.current_stream().cuda_stream, None, None)
        if rc:
            check(rc, "tt_scan_topk_bf16f32")
        return self.out


def sharded_sample(x16: torch.Tensor, n: int) -> torch.Tensor:
    """Rows 0, 16, 32, ... of a bf16 catalog image (the replicated sample of the sharded search)."""
    return x16[:n:_lib.TT_SHARD_SAMPLE_STRIDE].contiguous()


def sharded_begin(sample16: torch.Tensor, d: int, q: torch.Tensor, k: int, stats=None,
                  workspace: torch.Tensor = None) -> torch.Tensor:
    """Stage 1 of the row-sharded search (tt_sharded_filter_begin): this rank's queries
    against the global catalog sample -> stats [nq, 2] f32 (threshold, probe top)."""
    _check_2d(sample16, "sample16", torch.bfloat16)
    _check_2d(q, "q")
    nq, ns = q.shape[0], sample16.shape[0]
    if stats is None:
        stats = torch.empty((nq, 2), dtype=_f32, device=q.device)
    if nq == 0:
        return stats
    need = filter_workspace_bytes(ns, d, nq, min(k, ns))
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    check(lib().tt_sharded_filter_begin(_ptr(sample16), ns, d, sample16.stride(0), _ptr(q), nq,
                                        q.stride(0), k, _ptr(stats), _ptr(workspace),
                                        workspace.numel(), stream_ptr()),
          "tt_sharded_filter_begin")
    return stats


def sharded_workspace_bytes(n: int, d: int, nq: int, k: int) -> int:
    v = ctypes.c_int64(0)
    check(lib().tt_sharded_workspace_bytes(n, d, nq, k, ctypes.byref(v)),
          "tt_sharded_workspace_bytes")
    return v.value


def sharded_full(db16: torch.Tensor, n: int, d: int, q: torch.Tensor, k: int, bounds,
                 stats: torch.Tensor, workspace: torch.Tensor, pcount: torch.Tensor = None,
                 events=(None, None)) -> torch.Tensor:
    """Stage 2 of the row-sharded search (tt_sharded_filter_full): all ranks' queries q
    [nq, ep] with their gathered stats [nq, 2] against this rank's shard -> probe counts
    [nq, TT_SHARD_PROBES] int32, to be all-reduced (SUM) over the ranks before
    sharded_finish with the SAME workspace.  bounds: the whole catalog's (MAX over shards)."""
    _check_2d(db16, "db16", torch.bfloat16)
    _check_2d(q, "q")
    nq = q.shape[0]
    if not (1 <= k <= min(n, FILTER_KMAX)) or n > db16.shape[0]:
        raise ValueError(f"sharded_full: need 1 <= k ({k}) <= min(n, 128)")
    if tuple(stats.shape) != (nq, 2) or stats.dtype != _f32 or not stats.is_contiguous():
        raise ValueError("sharded_full: stats must be contiguous float32 [nq, 2]")
    if workspace is None or workspace.numel() < sharded_workspace_bytes(n, d, nq, k):
        raise ValueError("sharded_full: workspace smaller than sharded_workspace_bytes")
    if pcount is None or pcount.numel() < nq * _lib.TT_SHARD_PROBES:
        pcount = torch.empty((nq, _lib.TT_SHARD_PROBES), dtype=torch.int32, device=q.device)
    pcount = pcount.view(-1)[: nq * _lib.TT_SHARD_PROBES]
    x_norm_max, x_resid_max = (float(v) for v in bounds)
    e0, e1 = events
    check(lib().tt_sharded_filter_full(_ptr(db16), n, d, db16.stride(0), _ptr(q), nq, q.stride(0),
                                       k, ctypes.c_float(x_norm_max), ctypes.c_float(x_resid_max),
                                       _ptr(stats), _ptr(pcount), _ptr(workspace),
                                       workspace.numel(), stream_ptr(),
                                       e0.cuda_event if e0 is not None else None,
                                       e1.cuda_event if e1 is not None else None),
          "tt_sharded_filter_full")
    return pcount


def sharded_finish(db: torch.Tensor, db16: torch.Tensor, n: int, d: int, q: torch.Tensor, k: int,
                   row_base: int, stats: torch.Tensor, pcount: torch.Tensor,
                   workspace: torch.Tensor, out=None):
    """Stage 3 (tt_sharded_filter_finish) with the all-reduced probe counts: this shard's part
    of the global top-k [nq, k] (global row ids), merged across ranks with merge_topk."""
    _check_2d(db, "db")
    nq = q.shape[0]
    if out is None:
        out = (torch.empty((nq, k), dtype=_f32, device=q.device),
               torch.empty((nq, k), dtype=torch.int64, device=q.device))
    check(lib().tt_sharded_filter_finish(_ptr(db), _ptr(db16), n, d, db.stride(0), row_base,
                                         _ptr(q), nq, q.stride(0), k, _ptr(stats), _ptr(pcount),
                                         out[0].data_ptr(), out[1].data_ptr(), _ptr(workspace),
                                         workspace.numel(), stream_ptr()),
          "tt_sharded_filter_finish")
    return out


def sharded_search(db: torch.Tensor, db16: torch.Tensor, n: int, d: int, q: torch.Tensor, k: int,
                   bounds, row_base: int, stats: torch.Tensor, allreduce_sum,
                   workspace: torch.Tensor = None, out=None, pcount: torch.Tensor = None,
                   events=(None, None)):
    """Stages 2-3 of the row-sharded search (sharded_full, allreduce_sum(probe counts) in
    place, sharded_finish).  Returns this shard's part of the global top-k; merge the ranks'
    parts with merge_topk.  bounds must hold for the whole catalog (MAX over the shards)."""
    _check_2d(db, "db")
    nq = q.shape[0]
    if out is None:
        out = (torch.empty((nq, k), dtype=_f32, device=q.device),
               torch.empty((nq, k), dtype=torch.int64, device=q.device))
    if nq == 0:
        return out
    need = sharded_workspace_bytes(n, d, nq, k)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
    pcount = sharded_full(db16, n, d, q, k, bounds, stats, workspace, pcount, events)
    allreduce_sum(pcount)
    return sharded_finish(db, db16, n, d, q, k, row_base, stats, pcount, workspace, out)


def merge_topk(scores: torch.Tensor, idx: torch.Tensor, k: int):
    """[L, nq, k_in] per-shard sorted lists (global ids) -> [nq, k]."""
    require_device(scores, "scores")
    if scores.dim() != 3 or idx.shape != scores.shape or idx.dtype != torch.int64:
        raise ValueError("merge_topk: expected [L, nq, k_in] f32 scores and int64 ids")
    scores, idx = scores.contiguous(), idx.contiguous()
    L, nq, k_in = scores.shape
    out_s = torch.empty((nq, k), dtype=_f32, device=scores.device)
    out_i = torch.empty((nq, k), dtype=torch.int64, device=scores.device)
    check(lib().tt_topk_merge_f32(_ptr(scores), _ptr(idx), L, nq, k_in, k, _ptr(out_s),
                                  _ptr(out_i), stream_ptr()), "tt_topk_merge_f32")
    return out_s, out_i


def weighted_avg_l2(items: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None):
    require_device(items, "item_embeddings")
    if items.dim() != 3 or w.shape != items.shape[:2]:
        raise ValueError("weighted_avg_l2: items [B,S,E] and weights [B,S] required")
    items = items.contiguous().to(_f32)
    w = w.contiguous().to(_f32)
    b, s, d = items.shape
    if out is None:
        out = torch.empty((b, d), dtype=_f32, device=items.device)
    check(lib().tt_weighted_avg_l2_f32(_ptr(items), b, s, d, _ptr(w), _ptr(out), out.stride(0),
                                       stream_ptr()), "tt_weighted_avg_l2_f32")
    return out


def gather_weighted_avg_l2(table: torch.Tensor, d: int, hist: torch.Tensor, w: torch.Tensor,
                           out: torch.Tensor = None):
    """Mode B buyer encode: rows table[hist[b, s]] aggregated with weights w[b, s]."""
    _check_2d(table, "table")
    require_device(hist, "hist")
    if hist.dtype != torch.int64 or hist.dim() != 2 or w.shape != hist.shape:
        raise ValueError("gather_weighted_avg_l2: hist [B,S] int64 and w [B,S] required")
    hist = hist.contiguous()
    w = w.contiguous().to(_f32)
    b, s = hist.shape
    if out is None:
        out = torch.empty((b, table.shape[1]), dtype=_f32, device=table.device)
    check(lib().tt_gather_weighted_avg_l2_f32(_ptr(table), table.shape[0], table.stride(0), d,
                                              _ptr(hist), _ptr(w), b, s, _ptr(out),
                                              out.stride(0), stream_ptr()),
          "tt_gather_weighted_avg_l2_f32")
    return out


ATTN_WS_MIN_ROWS = 256  # b*s from which the GEMM-based form (tt_attn_agg_l2_f32_ws) runs


def attn_agg_l2(items, w, W1, b1, W2, b2, out=None, fused: bool = None):
    """BuyerTower.attention_aggregation + F.normalize (buyer_tower.py:70-101).  Batches of
    >= ATTN_WS_MIN_ROWS history rows take the two-stage form (first MLP layer as an f32 MFMA
    GEMM, tt_attn_agg_l2_f32_ws); smaller ones (e.g. one /retrieve buyer) the one-kernel form.
    fused=True/False forces one of them.  The two forms sum the first MLP layer's dot products
    in different orders, so the same buyer's embedding can differ in the last bits (measured
    <= 1e-6) between a call with >= 256 history rows (batch encode) and a smaller one (one
    /retrieve buyer); near-tied items may then swap ranks between the two.  Both are within the
    reference-fixture tolerance (2e-6); pass the same ``fused`` everywhere when identical bits
    across batch sizes matter."""
    require_device(items, "item_embeddings")
    if items.dim() != 3 or w.shape != items.shape[:2]:
        raise ValueError("attn_agg_l2: items [B,S,E] and weights [B,S] required")
    items = items.contiguous().to(_f32)
    w = w.contiguous().to(_f32)
    W1, b1, W2, b2 = (t.detach().contiguous().to(_f32) for t in (W1, b1, W2, b2))
    b, s, d = items.shape
    h = W1.shape[0]
    if out is None:
        out = torch.empty((b, d), dtype=_f32, device=items.device)
    if fused is None:
        fused = b * s < ATTN_WS_MIN_ROWS or d % 32 != 0
    if fused:
        check(lib().tt_attn_agg_l2_f32(_ptr(items), b, s, d, _ptr(w), _ptr(W1), _ptr(b1), h,
                                       _ptr(W2), _ptr(b2), _ptr(out), out.stride(0),
                                       stream_ptr()), "tt_attn_agg_l2_f32")
        return out
    need = ctypes.c_int64(0)
    check(lib().tt_attn_agg_workspace_bytes(b, s, h, ctypes.byref(need)),
          "tt_attn_agg_workspace_bytes")
    ws = torch.empty(need.value, dtype=torch.uint8, device=items.device)
    check(lib().tt_attn_agg_l2_f32_ws(_ptr(items), b, s, d, _ptr(w), _ptr(W1), _ptr(b1), h,
                                      _ptr(W2), _ptr(b2), _ptr(out), out.stride(0), _ptr(ws),
                                      ws.numel(), stream_ptr()), "tt_attn_agg_l2_f32_ws")
    return out
