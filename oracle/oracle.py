"""CPU oracle for the two-tower hot path -- TEST INFRASTRUCTURE, never the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  It wraps oracle/tt_oracle.c (canonical float32 restatement, bit-exact with the HIP
kernels) and adds float64 restatements of the reference semantics:

* ``flatip_search_f64``  faiss.IndexFlatIP.search as used by VectorDatabase.retrieve /
  retrieve_batch (reference src/inference/vector_db.py:159-160, 196-197): exact inner
  product, k clamped by the caller, descending scores.  faiss-cpu (>=1.7.4,
  requirements.txt:26) is not installed offline; this restates its published semantics.
* ``vector_db_normalize``  the reference's own numpy expression (vector_db.py:44-45):
  ``x / (np.linalg.norm(x, axis=1, keepdims=True) + 1e-8)`` -- executed with numpy itself.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libtt_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.tto_norm.restype = ctypes.c_float
        L.tto_norm.argtypes = [_f32p, _i64]
        L.tto_dot.restype = ctypes.c_float
        L.tto_dot.argtypes = [_f32p, _f32p, _i32]
        L.tto_l2norm_rows.restype = None
        L.tto_l2norm_rows.argtypes = [_f32p, _i64, _i32, _i64, _f32p, _i64, _i32]
        L.tto_scan_topk.restype = None
        L.tto_scan_topk.argtypes = [_f32p, _i64, _i32, _i64, _i64, _f32p, _i32, _i64, _i32,
                                    _f32p, _i64p]
        L.tto_weighted_avg_l2.restype = None
        L.tto_weighted_avg_l2.argtypes = [_f32p, _f32p, _i64, _i64p, _i64, _i32, _i32, _f32p,
                                          _f32p, _i64]
        L.tto_attn_agg_l2.restype = None
        L.tto_attn_agg_l2.argtypes = [_f32p, _i64, _i32, _i32, _f32p, _f32p, _f32p, _i32,
                                      _f32p, _f32p, _f32p, _i64]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(_f32p) if a is not None else None


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# --------------------------------------------------------------------------- canonical f32
def l2norm_rows(x: np.ndarray, mode: int) -> np.ndarray:
    """mode 0: x/(||x||+1e-8) (vector_db.py:44-45); mode 1: F.normalize (item_tower.py:209)."""
    x = _c32(x)
    n, d = x.shape
    y = np.empty_like(x)
    lib().tto_l2norm_rows(_fp(x), n, d, d, _fp(y), d, mode)
    return y


def dot(x: np.ndarray, q: np.ndarray) -> float:
    x, q = _c32(x), _c32(q)
    return float(lib().tto_dot(_fp(x), _fp(q), x.shape[0]))


def scan_topk(db: np.ndarray, q: np.ndarray, k: int, row_base: int = 0, threads: int = 0):
    """Canonical-f32 exact top-k; bit-exact reference for tt_scan_topk_f32.

    threads > 1 splits the queries over a thread pool (ctypes drops the GIL; queries are
    independent, so the result does not depend on the split).  0 = min(16, cpu count)."""
    db, q = _c32(db), _c32(q)
    n, d = db.shape
    nq = q.shape[0]
    s = np.empty((nq, k), np.float32)
    i = np.empty((nq, k), np.int64)
    L = lib()

    def run(a, b):
        if b > a:
            L.tto_scan_topk(_fp(db), n, d, d, row_base, _fp(q[a:b]), b - a, d, k, _fp(s[a:b]),
                            i[a:b].ctypes.data_as(_i64p))

    t = threads or min(16, os.cpu_count() or 1)
    if t <= 1 or nq * n < (1 << 22):
        run(0, nq)
        return s, i
    from concurrent.futures import ThreadPoolExecutor

    t = min(t, nq)
    cuts = [nq * j // t for j in range(t + 1)]
    with ThreadPoolExecutor(t) as ex:
        list(ex.map(lambda j: run(cuts[j], cuts[j + 1]), range(t)))
    return s, i


def weighted_avg_l2(items: np.ndarray, w: np.ndarray) -> np.ndarray:
    items, w = _c32(items), _c32(w)
    b, s, d = items.shape
    out = np.empty((b, d), np.float32)
    lib().tto_weighted_avg_l2(_fp(items), None, 0, None, b, s, d, _fp(w), _fp(out), d)
    return out


def gather_weighted_avg_l2(table: np.ndarray, hist: np.ndarray, w: np.ndarray) -> np.ndarray:
    table, w = _c32(table), _c32(w)
    hist = np.ascontiguousarray(hist, dtype=np.int64)
    b, s = hist.shape
    d = table.shape[1]
    out = np.empty((b, d), np.float32)
    lib().tto_weighted_avg_l2(None, _fp(table), d, hist.ctypes.data_as(_i64p), b, s, d, _fp(w),
                              _fp(out), d)
    return out


def attn_agg_l2(items, w, W1, b1, W2, b2) -> np.ndarray:
    items, w, W1, b1, W2, b2 = map(_c32, (items, w, W1, b1, W2, b2))
    b, s, d = items.shape
    h = W1.shape[0]
    out = np.empty((b, d), np.float32)
    lib().tto_attn_agg_l2(_fp(items), b, s, d, _fp(w), _fp(W1), _fp(b1), h,
                          _fp(W2.reshape(-1)), _fp(b2.reshape(-1)), _fp(out), d)
    return out


# --------------------------------------------------------------------------- reference f64
def vector_db_normalize(x: np.ndarray) -> np.ndarray:
    """The reference's expression, vector_db.py:44-45 / 152-153 / 189-190, run by numpy."""
    norms = np.linalg.norm(x, axis=1, keepdims=True)
    return (x / (norms + 1e-8)).astype(np.float32)


def i8_tile(codes: np.ndarray, n: int) -> np.ndarray:
    """numpy restatement of tt_i8_tile (test infrastructure; the layout is this framework's,
    not the reference's): codes [n, E] int8 (E % 64 == 0) -> per 16-row block b, E / 64 pieces
    of 1 KB, piece s holding at byte 16 l (l = 16 g + col) row 16 b + col's codes
    64 s + 16 g .. + 15; rows past n zero.  Flat int8 [ceil(n / 16) * 16 * E]."""
    e = codes.shape[1]
    nb = (n + 15) // 16
    c = np.zeros((nb * 16, e), np.int8)
    c[:n] = codes[:n]
    # [b, col, s, g, 16] -> [b, s, g, col, 16]
    t = c.reshape(nb, 16, e // 64, 4, 16).transpose(0, 2, 3, 1, 4)
    return np.ascontiguousarray(t).reshape(-1)


def i8_image(x: np.ndarray):
    """numpy restatement of tt_i8_image (test infrastructure): per 64-row tile s = max|x| / 127
    over finite values (float32 division), codes rint(x / s) clamped to [-127, 127] (0 where
    s == 0 or x is not finite); bounds (max ||x||, max ||x - s n||, max s ||n||) in float64 over
    rows without a non-finite value."""
    x = np.asarray(x, np.float32)
    n, d = x.shape
    codes = np.zeros((n, d), np.int8)
    scales = np.zeros((n + 63) // 64, np.float32)
    bx = br = bs = 0.0
    fin = np.isfinite(x)
    for t in range(scales.size):
        blk, f = x[64 * t:64 * t + 64], fin[64 * t:64 * t + 64]
        m = np.float32(np.abs(np.where(f, blk, 0)).max()) if blk.size else np.float32(0)
        s = np.float32(m / np.float32(127.0))
        scales[t] = s
        if s > 0:
            with np.errstate(invalid="ignore", divide="ignore"):
                c = np.clip(np.rint(np.where(f, blk, 0) / s), -127, 127)
            c = np.where(f, c, 0).astype(np.int8)
        else:
            c = np.zeros(blk.shape, np.int8)
        codes[64 * t:64 * t + 64] = c
        ok = f.all(axis=1)
        if ok.any():
            b64, c64 = blk[ok].astype(np.float64), c[ok].astype(np.float64)
            bx = max(bx, float(np.sqrt((b64 ** 2).sum(1)).max()))
            br = max(br, float(np.sqrt(((b64 - float(s) * c64) ** 2).sum(1)).max()))
            bs = max(bs, float(s) * float(np.sqrt((c64 ** 2).sum(1)).max()))
    return codes, scales, (bx, br, bs)


def weighted_avg_l2_f64(items: np.ndarray, w: np.ndarray) -> np.ndarray:
    """BuyerTower.weighted_average in float64 (buyer_tower.py:43-68): w / (sum w + 1e-8),
    weighted sum over the history, F.normalize (x / max(||x||, 1e-12))."""
    items = np.asarray(items, np.float64)
    w = np.asarray(w, np.float64)[..., None]
    z = (items * (w / (w.sum(axis=1, keepdims=True) + 1e-8))).sum(axis=1)
    return z / np.maximum(np.linalg.norm(z, axis=1, keepdims=True), 1e-12)


def attn_agg_l2_f64(items, w, W1, b1, W2, b2) -> np.ndarray:
    """BuyerTower.attention_aggregation in float64 (buyer_tower.py:70-101, MLP :32-36):
    scores = Linear(ReLU(Linear(x))) * w, softmax over the history, weighted sum, F.normalize."""
    items = np.asarray(items, np.float64)
    f = lambda a: np.asarray(a, np.float64)  # noqa: E731
    h = np.maximum(items @ f(W1).T + f(b1), 0.0)
    a = (h @ f(W2).T + f(b2))[..., 0] * f(w)
    a = np.exp(a - a.max(axis=1, keepdims=True))
    a /= a.sum(axis=1, keepdims=True)
    z = (items * a[..., None]).sum(axis=1)
    return z / np.maximum(np.linalg.norm(z, axis=1, keepdims=True), 1e-12)


def flatip_search_f64(db: np.ndarray, q: np.ndarray, k: int):
    """fp64 restatement of IndexFlatIP.search: scores desc, ties -> lower row."""
    s = np.asarray(q, np.float64) @ np.asarray(db, np.float64).T
    order = np.lexsort((np.broadcast_to(np.arange(db.shape[0]), s.shape), -s), axis=1)[:, :k]
    return np.take_along_axis(s, order, 1), order.astype(np.int64)


def topk_parity_f64(gpu_s, gpu_i, db, q, k, score_tol=1e-5, gap=1e-6):
    """SURVEY.md H0 parity rule (ii) against the fp64 oracle.  Returns list of problems."""
    ref_s, ref_i = flatip_search_f64(db, q, k)
    full = np.asarray(q, np.float64) @ np.asarray(db, np.float64).T
    problems = []
    for qi in range(q.shape[0]):
        got = full[qi, gpu_i[qi]]
        if np.max(np.abs(gpu_s[qi].astype(np.float64) - got)) > score_tol:
            problems.append((qi, "score"))
            continue
        # ids must match at every rank whose fp64 gap to neighbours exceeds `gap`
        rs = ref_s[qi]
        kth = rs[-1]
        nxt = np.sort(full[qi])[::-1][k] if full.shape[1] > k else -np.inf
        for r in range(k):
            lo = rs[r + 1] if r + 1 < k else nxt
            hi = rs[r - 1] if r > 0 else np.inf
            if hi - rs[r] > gap and rs[r] - lo > gap and gpu_i[qi, r] != ref_i[qi, r]:
                problems.append((qi, f"id@{r}"))
                break
        # set equality outside the near-tie band at the k/k+1 boundary
        sure = set(ref_i[qi][rs > kth + gap].tolist())
        if not sure.issubset(set(gpu_i[qi].tolist())):
            problems.append((qi, "set"))
    return problems
