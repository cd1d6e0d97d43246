"""configs[4] training step on MI355X: item-tower head + buyer-tower attention + InfoNCE.

What the reference's Trainer does per batch (src/training/trainer.py:74-243 with
TwoTowerModel.forward_simplified, two_tower.py:155-218, InfoNCELoss, losses.py:20-79, Adam,
trainer.py:49-52), with the trainable parameters of the default configuration: the item
tower's projection head + brand/category embeddings and the buyer tower's attention MLP (the
sentence-transformer is frozen, item_tower.py:40-42, so the step takes the text embeddings of
the positive/negative products as inputs; `BertEncoder` produces them).

Every arithmetic step is a HIP kernel (C ABI in include/twotower_hip.h): forward and backward
GEMMs on MFMA (tt_gemm_f32 / tt_gemm_bf16), F.normalize and its backward, the attention
pooling forward/backward, InfoNCE forward+backward, embedding scatter-add, fused Adam.
Python only sequences the launches and owns the buffers.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from . import _lib, kernels
from ._lib import check, lib, stream_ptr
from .losses import infonce


def _p(t):
    return t.data_ptr() if t is not None else None


def dropout_keep(shape, p: float, device) -> torch.Tensor:
    """Keep mask of nn.Dropout(p) (uint8, 1 = keep), drawn from torch's device RNG."""
    return (torch.rand(shape, device=device) >= p).to(torch.uint8)


def apply_dropout(x: torch.Tensor, keep: torch.Tensor, p: float) -> torch.Tensor:
    """In place x = x * keep / (1 - p) (tt_dropout_apply_f32); also the backward on a grad."""
    if keep.shape != x.shape or keep.dtype != torch.uint8 or not x.is_contiguous():
        raise ValueError("dropout: keep must be a uint8 mask of x's shape, x contiguous")
    check(lib().tt_dropout_apply_f32(x.data_ptr(), keep.contiguous().data_ptr(),
                                     1.0 / (1.0 - p), x.numel(), stream_ptr()), "dropout")
    return x


class GemmOps:
    """GEMM-shaped pieces of the backward passes on the HIP kernels (f32 or bf16 MFMA)."""

    def __init__(self, prec: str = "f32", device=None):
        if prec not in ("f32", "bf16"):
            raise ValueError("prec must be 'f32' or 'bf16'")
        self.prec = prec
        self.dev = device or _lib.device()

    def gemm(self, A, W, bias=None, act=0, res=None):
        """C = act(A W^T + bias) (+ res): A [M,K], W [N,K] f32 device (K % 32 / 64 == 0)."""
        M, K = A.shape
        N = W.shape[0]
        C = torch.empty((M, N), dtype=torch.float32, device=self.dev)
        if self.prec == "bf16":
            A16 = torch.empty((M, K), dtype=torch.bfloat16, device=self.dev)
            W16 = torch.empty((N, K), dtype=torch.bfloat16, device=self.dev)
            check(lib().tt_f32_to_bf16(A.data_ptr(), A.stride(0), M, K, A16.data_ptr(), K,
                                       stream_ptr()), "bf16 A")
            check(lib().tt_f32_to_bf16(W.data_ptr(), W.stride(0), N, K, W16.data_ptr(), K,
                                       stream_ptr()), "bf16 W")
            check(lib().tt_gemm_bf16(A16.data_ptr(), K, W16.data_ptr(), K, _p(bias), _p(res),
                                     res.stride(0) if res is not None else 0, C.data_ptr(), N,
                                     None, 0, M, N, K, act, stream_ptr()), "gemm_bf16")
        else:
            check(lib().tt_gemm_f32(A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0),
                                    _p(bias), _p(res), res.stride(0) if res is not None else 0,
                                    C.data_ptr(), N, None, 0, M, N, K, act, stream_ptr()),
                  "gemm_f32")
        return C

    def kpad(self, k: int) -> int:
        q = 64 if self.prec == "bf16" else 32
        return (k + q - 1) // q * q

    def T(self, x, ld=None):
        """x [r, c] -> [c, ld] with zero columns r..ld-1 (ld = K padding of the GEMM)."""
        r, c = x.shape
        ld = ld or self.kpad(r)
        t = torch.empty((c, ld), dtype=torch.float32, device=self.dev)
        check(lib().tt_transpose_f32(x.data_ptr(), x.stride(0), r, c, t.data_ptr(), ld,
                                     stream_ptr()), "transpose")
        return t

    def dW(self, dY, X):
        """dY^T X : [N, M] x [M, K] -> [N, K] (dY [M, N], X [M, K])."""
        ldk = self.kpad(dY.shape[0])
        return self.gemm(self.T(dY, ldk), self.T(X, ldk))

    def colsum(self, x):
        out = torch.empty(x.shape[1], dtype=torch.float32, device=self.dev)
        check(lib().tt_col_sum_f32(x.data_ptr(), x.stride(0), x.shape[0], x.shape[1],
                                   out.data_ptr(), 0, stream_ptr()), "col_sum")
        return out


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _Bufs:
    """Every intermediate of one step shape (preallocated once: a replayed HIP graph and the
    eager launch sequence read and write the same addresses)."""


class TwoTowerTrainStep:
    """One optimizer step of the item head + buyer attention under InfoNCE (Adam).

    Layout: the trained parameters live in ONE flat f32 buffer (the modules' parameters are
    views of it), beside flat gradient / Adam-moment buffers, so Adam is one launch and the
    data-parallel gradient average one all-reduce.  Every intermediate of a step shape is
    preallocated; the launch sequence per step is:

      forward   concat(+bf16 copy) | operand prep (ONE tt_convert_batch: bf16 weights,
                transposed weights, bf16 history rows) | head GEMM + ReLU | dropout (+bf16) |
                head GEMM | F.normalize | attention GEMM + ReLU | attention pooling | InfoNCE
      backward  F.normalize bwd (+bf16) | dW3, db3 (tt_gemm_tn: A^T B, bias fused) | dh GEMM |
                ReLU + dropout bwd (+bf16) | dW0, db0 (tt_gemm_tn) | embedding-row grads |
                attention pooling bwd (+ReLU) | dWa0, dba0 (tt_gemm_tn)
      then      all-reduce (multi-GPU) | Adam (one launch over the flat buffers)

    ``graph=True`` captures forward + backward of each step shape in a HIP graph (torch's
    CUDAGraph over the same launches) after one eager warm-up call, and replays it: the ~35
    launches cost one graph launch of host time.  Inputs are copied into the graph's static
    buffers (``input_buffers`` hands them out to write in place instead)."""

    def __init__(self, item_tower, buyer_tower, temperature: float = 0.07, lr: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, prec: str = "f32", graph: bool = False):
        if buyer_tower.aggregation_method not in ("attention", "weighted_avg"):
            raise ValueError(f"Unknown aggregation method: {buyer_tower.aggregation_method}")
        self.attention = buyer_tower.aggregation_method == "attention"
        if prec not in ("f32", "bf16"):
            raise ValueError("prec must be 'f32' or 'bf16'")
        self.it, self.bt = item_tower, buyer_tower
        self.tau, self.lr, self.betas, self.eps, self.prec = temperature, lr, betas, eps, prec
        self.dev = _lib.device()
        self.ops = GemmOps(prec, self.dev)
        self.it.to(self.dev)
        self.bt.to(self.dev)
        self._flatten()
        self.t = 0
        self.last_loss = None
        # nn.Dropout(0.1) of the projection (item_tower.py:61): active when the item tower is
        # in train mode, as under the reference Trainer (model.train(), trainer.py:167)
        self.keep_fn = dropout_keep
        self.graph = graph
        # projection dropout drawn in-kernel (tt_dropout_rng_f32) from (seed, draw counter): the
        # counter lives on the device and advances every step, so graph replays draw new masks
        self._drop_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self._drop_ctr = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._bufs = {}    # shape key -> _Bufs
        self._graphs = {}  # shape key -> torch.cuda.CUDAGraph (graph=True)
        self._pool = None

    # ------------------------------------------------------------------ flat parameters
    def _param_objs(self) -> Dict[str, torch.nn.Parameter]:
        it, bt = self.it, self.bt
        p = {"proj0.w": it.projection[0].weight, "proj0.b": it.projection[0].bias,
             "proj3.w": it.projection[3].weight, "proj3.b": it.projection[3].bias}
        if self.attention:  # weighted_avg has no parameters (buyer_tower.py:43-68)
            p.update({"att0.w": bt.attention[0].weight, "att0.b": bt.attention[0].bias,
                      "att2.w": bt.attention[2].weight, "att2.b": bt.attention[2].bias})
        if it.use_categorical_features and it.brand_embedding is not None:
            p["brand"] = it.brand_embedding.weight  # brand and cat adjacent: one zero-fill
            p["cat"] = it.category_embedding.weight
        return p

    def _flatten(self) -> None:
        """Move the trained parameters into one flat buffer (module parameters become views)
        and lay out the matching gradient / moment buffers.  Moments carry over by name."""
        objs = self._param_objs()
        total = sum(v.numel() for v in objs.values())
        flat = torch.empty(total, dtype=torch.float32, device=self.dev)
        old_m, old_v = getattr(self, "m", None), getattr(self, "v", None)
        fm = torch.zeros(total, dtype=torch.float32, device=self.dev)
        fv = torch.zeros(total, dtype=torch.float32, device=self.dev)
        self.flat_g = torch.zeros(total, dtype=torch.float32, device=self.dev)
        self.params, self.m, self.v, self.g, self._span = {}, {}, {}, {}, {}
        off = 0
        for k, prm in objs.items():
            n = prm.numel()
            view = flat[off:off + n].view(prm.shape)
            view.copy_(prm.data)
            prm.data = view
            self.params[k] = prm.data
            self.m[k] = fm[off:off + n].view(prm.shape)
            self.v[k] = fv[off:off + n].view(prm.shape)
            self.g[k] = self.flat_g[off:off + n].view(prm.shape)
            if old_m is not None and k in old_m:
                self.m[k].copy_(old_m[k])
                self.v[k].copy_(old_v[k])
            self._span[k] = (off, n)
            off += n
        self.flat_p, self.flat_m, self.flat_v = flat, fm, fv
        self._objs = objs
        self._bufs = {}
        self._graphs = {}

    def _check_layout(self) -> None:
        # model.to() / parameter re-assignment after construction: rebuild the flat layout
        for k, prm in self._objs.items():
            if prm.data.data_ptr() != self.params[k].data_ptr():
                self._flatten()
                return

    # kept for autograd_ops-style callers
    def _gemm(self, A, W, bias=None, act=0, res=None):
        return self.ops.gemm(A, W, bias, act, res)

    # ------------------------------------------------------------------ buffers
    def _key(self, B, S, N, E, Ht, use_cat, has_b, has_c, pdrop):
        return (B, S, N, E, Ht, use_cat, has_b, has_c, pdrop)

    def _alloc(self, key) -> "_Bufs":
        B, S, N, E, Ht, use_cat, has_b, has_c, pdrop = key
        dev, f32, bf = self.dev, torch.float32, torch.bfloat16
        P = self.params
        b = _Bufs()
        R = B + B * N
        C = self.it.categorical_embedding_dim if use_cat else 0
        width = Ht + 2 * C
        hid = P["proj0.w"].shape[0]
        b.R, b.C, b.width, b.hid = R, C, width, hid
        e = lambda *shape, dt=f32: torch.empty(shape, dtype=dt, device=dev)  # noqa: E731
        # inputs (static in graph mode)
        b.items, b.w = e(B, S, E), e(B, S)
        b.text = e(R, Ht)
        b.bids = torch.zeros(R, dtype=torch.int32, device=dev) if has_b else None
        b.cids = torch.zeros(R, dtype=torch.int32, device=dev) if has_c else None
        bf16 = self.prec == "bf16"
        b.x = e(R, width)
        b.x16 = e(R, width, dt=bf) if bf16 else None
        b.h = e(R, hid)
        b.h16 = e(R, hid, dt=bf) if bf16 else None
        b.y, b.z = e(R, E), e(R, E)
        b.zb = e(B, E)
        b.z16 = e(R, E, dt=bf) if bf16 else None  # the bf16 InfoNCE GEMM's operand copies
        b.zb16 = e(B, E, dt=bf) if (bf16 and self.attention) else None
        if self.attention:
            Hd = P["att0.w"].shape[0]
            b.Hd = Hd
            b.Hb = e(B * S, Hd)
            b.X16 = e(B * S, E, dt=bf) if bf16 else None
            b.alpha, b.onorm = e(B, S), e(B)
            b.dHb = e(B * S, Hd)
            b.da = e((B * S + 63) // 64 * 64 + B * (Hd + 1))  # da, then per-buyer dW2 parts
        b.loss = torch.empty((), dtype=f32, device=dev)
        need = ctypes.c_int64(0)
        check(lib().tt_infonce_workspace_bytes(B, N, E, _lib.TT_PREC_BF16 if bf16 else
                                               _lib.TT_PREC_F32, 1, ctypes.byref(need)),
              "tt_infonce_workspace_bytes")
        b.nce_ws = torch.empty(need.value, dtype=torch.uint8, device=dev)
        b.gb = e(B, E)
        b.dz = e(R, E)        # [gp; gn]: InfoNCE writes the item rows' gradient in place
        b.dy = e(R, E)
        b.dy16 = e(R, E, dt=bf) if bf16 else None
        b.dh = e(R, hid)
        b.dh16 = e(R, hid, dt=bf) if (bf16 and use_cat) else None
        b.dxc = e(R, 2 * C) if use_cat else None
        # one workspace per weight-gradient GEMM: their split sums wait for ONE reduce launch
        # at the end of the backward (tt_gemm_tn_partial + tt_gemm_tn_reduce_many)
        G = self.g
        tn_jobs = [((R, E, hid), "proj3"), ((R, hid, width), "proj0")]
        if self.attention:
            tn_jobs.append(((B * S, b.Hd, E), "att0"))
        b.tn_ws, pend = [], []
        for (M_, N_, K_), name in tn_jobs:
            v = ctypes.c_int64(0)
            check(lib().tt_gemm_tn_workspace_bytes(M_, N_, K_, ctypes.byref(v)), "tn ws")
            ws_ = torch.empty(max(v.value, 256), dtype=torch.uint8, device=dev)
            b.tn_ws.append(ws_)
            pend.append(_lib.TnPending(ctypes.c_void_p(ws_.data_ptr()), M_, N_, K_,
                                       ctypes.c_void_p(G[name + ".w"].data_ptr()), K_,
                                       ctypes.c_void_p(G[name + ".b"].data_ptr())))
        b.tn_pend = (_lib.TnPending * len(pend))(*pend)
        b.n_pend = len(pend)
        # weight-derived GEMM operands, refreshed by ONE tt_convert_batch per step
        W0, W3 = P["proj0.w"], P["proj3.w"]
        jobs = []

        def job(src, rows, cols, ld_src, dst, ld_dst, transpose, to_bf16, ids=None, dst_off=0):
            jobs.append(_lib.ConvertJob(ctypes.c_void_p(src), ld_src, rows, cols,
                                        ctypes.c_void_p(dst.data_ptr() + dst_off), ld_dst,
                                        transpose, to_bf16,
                                        ctypes.c_void_p(ids.data_ptr()) if ids is not None
                                        else None))
        if use_cat:  # the item head's input [text | brand[bid] | cat[cid]] (+ its bf16 copy)
            for dst, sz, bf_ in ((b.x, 4, 0),) + (((b.x16, 2, 1),) if bf16 else ()):
                job(b.text.data_ptr(), R, Ht, Ht, dst, width, 0, bf_)
                job(P["brand"].data_ptr() if has_b else None, R, C, C, dst, width, 0, bf_,
                    ids=b.bids, dst_off=sz * Ht)
                job(P["cat"].data_ptr() if has_c else None, R, C, C, dst, width, 0, bf_,
                    ids=b.cids, dst_off=sz * (Ht + C))
        b.W3T = e(hid, E, dt=bf if bf16 else f32)
        job(W3.data_ptr(), E, hid, hid, b.W3T, E, 1, int(bf16))
        b.W0cT = e(2 * C, hid, dt=bf if bf16 else f32) if use_cat else None
        if use_cat:
            job(W0.data_ptr() + 4 * Ht, hid, 2 * C, width, b.W0cT, hid, 1, int(bf16))
        if bf16:
            b.W0_16, b.W3_16 = e(hid, width, dt=bf), e(E, hid, dt=bf)
            job(W0.data_ptr(), hid, width, width, b.W0_16, width, 0, 1)
            job(W3.data_ptr(), E, hid, hid, b.W3_16, hid, 0, 1)
            if self.attention:
                Wa = P["att0.w"]
                b.Wa16 = e(b.Hd, E, dt=bf)
                job(Wa.data_ptr(), b.Hd, E, E, b.Wa16, E, 0, 1)
                job(b.items.data_ptr(), B * S, E, E, b.X16, E, 0, 1)
            if not use_cat:
                job(b.text.data_ptr(), R, Ht, Ht, b.x16, width, 0, 1)
        # gradients the step accumulates with atomics, zeroed by the same launch
        if use_cat:
            o0, o1 = self._span["brand"][0], self._span["cat"][0] + self._span["cat"][1]
            jobs.append(_lib.ConvertJob(None, 0, 1, o1 - o0, ctypes.c_void_p(
                self.flat_g.data_ptr() + 4 * o0), o1 - o0, 0, 0))
        b.jobs = (_lib.ConvertJob * len(jobs))(*jobs)
        b.njobs = len(jobs)
        return b

    def input_buffers(self, B, S, N, E=None, Ht=None, use_cat=None, has_b=True, has_c=True):
        """The static input buffers of a step shape (graph mode): (items [B,S,E], w [B,S],
        text [B + B N, Ht] = positives then negatives row-major, brand ids [B + B N] int32,
        cat ids [B + B N] int32).  Write a batch there and call step(...) with the SAME tensors
        to skip the copies."""
        E = E or self.params["proj3.w"].shape[0]
        Ht = Ht or (self.params["proj0.w"].shape[1] - 2 * (self.it.categorical_embedding_dim
                    if "brand" in self.params else 0))
        use_cat = "brand" in self.params if use_cat is None else use_cat
        pdrop = self.it.projection[2].p if self.it.training else 0.0
        key = self._key(B, S, N, E, Ht, use_cat, has_b and use_cat, has_c and use_cat, pdrop)
        if key not in self._bufs:
            self._bufs[key] = self._alloc(key)
        bb = self._bufs[key]
        return bb.items, bb.w, bb.text, bb.bids, bb.cids

    # ------------------------------------------------------------------ the step
    def forward_loss(self, *args, **kw) -> torch.Tensor:
        """The loss alone (the reference's validate: forward + criterion under no_grad,
        trainer.py:245-319): no backward GEMMs, no gradients."""
        return self.forward_backward(*args, grads=False, **kw)[0]

    def forward_backward(self, buyer_items, weights, pos_text, neg_text, pos_brand=None,
                         pos_cat=None, neg_brand=None, neg_cat=None, grads: bool = True):
        """buyer_items [B,S,E], weights [B,S], pos_text [B,Ht], neg_text [B,N,Ht] (device f32);
        *_brand / *_cat: int32 id tensors (vocab ids, 0 = <UNK>) or None.
        Returns (loss tensor, grads dict keyed like self.params; {} when grads=False).  The
        returned tensors are this step shape's buffers: read them before the next call."""
        self._check_layout()
        P = self.params
        B, S, E = buyer_items.shape
        N = neg_text.shape[1]
        Ht = pos_text.shape[1]
        use_cat = "brand" in P
        has_b = use_cat and (pos_brand is not None or neg_brand is not None)
        has_c = use_cat and (pos_cat is not None or neg_cat is not None)
        pdrop = self.it.projection[2].p if self.it.training else 0.0
        key = self._key(B, S, N, E, Ht, use_cat, has_b, has_c, pdrop)
        bb = self._bufs.get(key)
        if bb is None:
            bb = self._bufs[key] = self._alloc(key)
        # inputs into the static buffers (no-ops when the caller wrote them in place)
        bb_R = bb.R

        def put(dst, src):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src.reshape(dst.shape))
        put(bb.items, buyer_items.to(torch.float32))
        put(bb.w, weights.to(torch.float32))
        if pos_text.data_ptr() != bb.text.data_ptr():
            bb.text[:B].copy_(pos_text)
            bb.text[B:].copy_(neg_text.reshape(B * N, Ht))
        for buf, a, c in ((bb.bids, pos_brand, neg_brand), (bb.cids, pos_cat, neg_cat)):
            if buf is None or (a is not None and a.data_ptr() == buf.data_ptr()):
                continue
            if a is not None:
                buf[:B].copy_(a.reshape(-1))
            else:
                buf[:B].zero_()
            if c is not None:
                buf[B:].copy_(c.reshape(-1))
            else:
                buf[B:].zero_()
        del bb_R
        if not grads:
            self._launch(bb, key, grads=False)
            return bb.loss, {}
        if self.graph:
            g = self._graphs.get(key)
            if g is None:
                self._launch(bb, key, grads=True)  # eager warm-up (lazy inits, pool sizes)
                torch.cuda.current_stream().synchronize()
                g = torch.cuda.CUDAGraph()
                if self._pool is None:
                    self._pool = torch.cuda.graph_pool_handle()
                with torch.cuda.graph(g, pool=self._pool):
                    self._launch(bb, key, grads=True)
                self._graphs[key] = g
            g.replay()
        else:
            self._launch(bb, key, grads=True)
        return bb.loss, {k: self.g[k] for k in P}

    def _launch(self, bb: "_Bufs", key, grads: bool) -> None:
        B, S, N, E, Ht, use_cat, has_b, has_c, pdrop = key
        P, L, st = self.params, lib(), stream_ptr()
        bf16 = self.prec == "bf16"
        R, C, width, hid = bb.R, bb.C, bb.width, bb.hid
        # forward: [text | brand | cat] (+ bf16 copy for the bf16 GEMM) -- jobs of the step's
        # one tt_convert_batch launch, with the weight-derived GEMM operands
        x_in = bb.x if use_cat else bb.text
        if bb.njobs:
            check(L.tt_convert_batch(bb.jobs, bb.njobs, st), "convert_batch")
        rng_drop = pdrop > 0 and self.keep_fn is dropout_keep  # (a custom keep_fn: its mask)
        keep = self.keep_fn((R, hid), pdrop, self.dev) if pdrop > 0 and not rng_drop else None
        h16 = bb.h16 if pdrop == 0 else None
        if bf16:
            xa = bb.x16
            check(L.tt_gemm_bf16(xa.data_ptr(), width, bb.W0_16.data_ptr(), width,
                                 _p(P["proj0.b"]), None, 0, bb.h.data_ptr(), hid, _p(h16), hid,
                                 R, hid, width, _lib.TT_ACT_RELU, st), "gemm h")
        else:
            check(L.tt_gemm_f32(x_in.data_ptr(), x_in.stride(0), P["proj0.w"].data_ptr(), width,
                                _p(P["proj0.b"]), None, 0, bb.h.data_ptr(), hid, None, 0, R, hid,
                                width, _lib.TT_ACT_RELU, st), "gemm h")
        scale = 1.0
        if rng_drop:
            scale = 1.0 / (1.0 - pdrop)
            check(L.tt_dropout_rng_f32(bb.h.data_ptr(), bb.h.numel(), ctypes.c_float(pdrop),
                                       self._drop_seed, self._drop_ctr.data_ptr(), _p(bb.h16),
                                       st), "dropout")
        elif keep is not None:
            scale = 1.0 / (1.0 - pdrop)
            check(L.tt_dropout_apply_ex(bb.h.data_ptr(), keep.data_ptr(), scale, bb.h.numel(),
                                        _p(bb.h16), st), "dropout")
        if bf16:
            check(L.tt_gemm_bf16(bb.h16.data_ptr(), hid, bb.W3_16.data_ptr(), hid,
                                 _p(P["proj3.b"]), None, 0, bb.y.data_ptr(), E, None, 0, R, E,
                                 hid, 0, st), "gemm y")
        else:
            check(L.tt_gemm_f32(bb.h.data_ptr(), hid, P["proj3.w"].data_ptr(), hid,
                                _p(P["proj3.b"]), None, 0, bb.y.data_ptr(), E, None, 0, R, E,
                                hid, 0, st), "gemm y")
        check(L.tt_l2norm_rows_f32(bb.y.data_ptr(), R, E, E, bb.z.data_ptr(), E, _p(bb.z16),
                                   _lib.TT_NORM_MAX_EPS, st), "normalize")
        X = bb.items.view(B * S, E)
        if not self.attention:  # weighted average + F.normalize: no trainable parameters
            check(L.tt_weighted_avg_l2_f32(bb.items.data_ptr(), B, S, E, bb.w.data_ptr(),
                                           bb.zb.data_ptr(), E, st), "weighted_avg")
        else:
            Hd = bb.Hd
            if bf16:
                check(L.tt_gemm_bf16(bb.X16.data_ptr(), E, bb.Wa16.data_ptr(), E,
                                     _p(P["att0.b"]), None, 0, bb.Hb.data_ptr(), Hd, None, 0,
                                     B * S, Hd, E, _lib.TT_ACT_RELU, st), "gemm att")
            else:
                check(L.tt_gemm_f32(X.data_ptr(), E, P["att0.w"].data_ptr(), E, _p(P["att0.b"]),
                                    None, 0, bb.Hb.data_ptr(), Hd, None, 0, B * S, Hd, E,
                                    _lib.TT_ACT_RELU, st), "gemm att")
            check(L.tt_attn_pool_fwd_f32_dev(bb.Hb.data_ptr(), Hd, P["att2.w"].data_ptr(),
                                             P["att2.b"].data_ptr(), bb.w.data_ptr(),
                                             X.data_ptr(), B, S, E, bb.alpha.data_ptr(),
                                             bb.onorm.data_ptr(), bb.zb.data_ptr(), E,
                                             _p(bb.zb16), st), "attn_pool_fwd")
        # InfoNCE forward (+ backward): item-row gradients straight into dz = [gp; gn]
        pr = _lib.TT_PREC_BF16 if bf16 else _lib.TT_PREC_F32
        zp, zn = bb.z.data_ptr(), bb.z.data_ptr() + 4 * B * E
        dzp, dzn = bb.dz.data_ptr(), bb.dz.data_ptr() + 4 * B * E
        check(L.tt_infonce_ex(bb.zb.data_ptr(), E, zp, E, zn if N else None, N * E, E, B, N, E,
                              ctypes.c_float(self.tau), pr, bb.loss.data_ptr(),
                              bb.gb.data_ptr() if grads else None, dzp if grads else None,
                              (dzn if N else None) if grads else None, bb.nce_ws.data_ptr(),
                              bb.nce_ws.numel(), _p(bb.zb16), E, _p(bb.z16), E, st),
              "tt_infonce_ex")
        if not grads:
            return
        G, ws3, ws0 = self.g, bb.tn_ws[0], bb.tn_ws[1]
        # item head backward
        check(L.tt_l2norm_backward_ex(bb.y.data_ptr(), E, bb.z.data_ptr(), E, dzp, E, R, E,
                                      bb.dy.data_ptr(), E, _p(bb.dy16), E, st), "norm_bwd")
        check(L.tt_gemm_tn_partial(bb.dy.data_ptr(), E, bb.h.data_ptr(), hid, R, E, hid, pr,
                                   G["proj3.w"].data_ptr(), hid, G["proj3.b"].data_ptr(),
                                   ws3.data_ptr(), ws3.numel(), st), "dW3")
        if bf16:  # dh = dy W3 (A W^T form with W = W3^T)
            check(L.tt_gemm_bf16(bb.dy16.data_ptr(), E, bb.W3T.data_ptr(), E, None, None, 0,
                                 bb.dh.data_ptr(), hid, None, 0, R, hid, E, 0, st), "gemm dh")
        else:
            check(L.tt_gemm_f32(bb.dy.data_ptr(), E, bb.W3T.data_ptr(), E, None, None, 0,
                                bb.dh.data_ptr(), hid, None, 0, R, hid, E, 0, st), "gemm dh")
        check(L.tt_relu_dropout_backward_f32(bb.dh.data_ptr(), bb.h.data_ptr(), scale,
                                             bb.dh.numel(), _p(bb.dh16),
                                             _p(self._drop_ctr) if rng_drop else None, st),
              "relu_bwd")
        check(L.tt_gemm_tn_partial(bb.dh.data_ptr(), hid, x_in.data_ptr(), x_in.stride(0), R,
                                   hid, width, pr, G["proj0.w"].data_ptr(), width,
                                   G["proj0.b"].data_ptr(), ws0.data_ptr(), ws0.numel(), st),
              "dW0")
        if use_cat:  # embedding-row gradients through dxc = dh W0[:, Ht:]
            if bf16:
                check(L.tt_gemm_bf16(bb.dh16.data_ptr(), hid, bb.W0cT.data_ptr(), hid, None,
                                     None, 0, bb.dxc.data_ptr(), 2 * C, None, 0, R, 2 * C, hid,
                                     0, st), "gemm dxc")
            else:
                check(L.tt_gemm_f32(bb.dh.data_ptr(), hid, bb.W0cT.data_ptr(), hid, None, None,
                                    0, bb.dxc.data_ptr(), 2 * C, None, 0, R, 2 * C, hid, 0, st),
                      "gemm dxc")
            # (brand / cat gradients zeroed by the step's tt_convert_batch; scattered by the
            # backward tail below)
        emb = ((bb.dxc.data_ptr(), 2 * C, _p(bb.bids), _p(bb.cids), R, C, G["brand"].data_ptr(),
                G["cat"].data_ptr()) if use_cat else (None, 0, None, None, 0, 0, None, None))
        if not self.attention:  # the backward tail: weight-gradient reduces + embedding rows
            check(L.tt_train_bwd_tail(bb.tn_pend, bb.n_pend, None, 0, 0, None, None, *emb, st),
                  "bwd tail")
            return
        Hd = bb.Hd
        check(L.tt_attn_pool_bwd_relu_parts_f32(bb.gb.data_ptr(), E, bb.zb.data_ptr(), E,
                                                bb.onorm.data_ptr(), bb.alpha.data_ptr(),
                                                bb.w.data_ptr(), X.data_ptr(), B, S, E,
                                                bb.Hb.data_ptr(), P["att2.w"].data_ptr(), Hd,
                                                bb.dHb.data_ptr(), bb.da.data_ptr(), st),
              "attn_pool_bwd")
        wsa = bb.tn_ws[2]
        check(L.tt_gemm_tn_partial(bb.dHb.data_ptr(), Hd, X.data_ptr(), E, B * S, Hd, E, pr,
                                   G["att0.w"].data_ptr(), E, G["att0.b"].data_ptr(),
                                   wsa.data_ptr(), wsa.numel(), st), "dWa0")
        # the backward tail, one launch: the three weight gradients' split sums, dW2 / db2
        # from the attention pooling's per-buyer parts, the embedding-row gradients
        parts = bb.da.data_ptr() + 4 * ((B * S + 63) // 64 * 64)
        check(L.tt_train_bwd_tail(bb.tn_pend, bb.n_pend, ctypes.c_void_p(parts), B, Hd,
                                  G["att2.w"].data_ptr(), G["att2.b"].data_ptr(), *emb, st),
              "bwd tail")

    # torch.optim.Adam state dict (the reference saves optimizer.state_dict(), trainer.py:330):
    # 'state' indexed by the position of the parameter in model.parameters(), 'param_groups'
    # with Adam's defaults.  Parameters the fused step does not train (the frozen text
    # encoder) have no state entry, as under torch Adam when they never received a gradient.
    def optimizer_state_dict(self, model) -> Dict:
        pos = {p.data_ptr(): i for i, p in enumerate(model.parameters())}
        state = {}
        for k, p in self.params.items():
            if self.t > 0:
                state[pos[p.data_ptr()]] = {"step": torch.tensor(float(self.t)),
                                            "exp_avg": self.m[k].detach().cpu().clone(),
                                            "exp_avg_sq": self.v[k].detach().cpu().clone()}
        group = {"lr": self.lr, "betas": tuple(self.betas), "eps": self.eps, "weight_decay": 0,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "decoupled_weight_decay": False,
                 "params": list(range(len(pos)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, model, sd: Dict) -> None:
        """Restore Adam's step count and moments from optimizer_state_dict's format (or a
        torch.optim.Adam state dict over THIS model's model.parameters()).

        Compatibility is with this module's own parameter order: the reference's Adam state
        indexes the SentenceTransformer's ~200 frozen parameters first (item_tower.py:38,
        trainer.py:49-50), so its indices do not line up here.  A state dict whose entries do
        not match the trained parameters' shapes, or none of whose entries lands on a trained
        parameter, raises instead of silently leaving Adam at step 0."""
        pos = {p.data_ptr(): i for i, p in enumerate(model.parameters())}
        st = sd["state"]
        steps = set()
        matched = 0
        for k, p in self.params.items():
            i = pos[p.data_ptr()]
            e = st.get(i)
            if e is None:
                continue
            ea, es = torch.as_tensor(e["exp_avg"]), torch.as_tensor(e["exp_avg_sq"])
            if ea.numel() != self.m[k].numel() or es.numel() != self.v[k].numel():
                raise ValueError(
                    f"optimizer state entry {i} holds {tuple(ea.shape)} moments, parameter {k} "
                    f"needs {tuple(self.m[k].shape)}: the state dict indexes a different parameter "
                    "list (e.g. a reference checkpoint, whose frozen text-encoder parameters come "
                    "first)")
            self.m[k].copy_(ea.view_as(self.m[k]))
            self.v[k].copy_(es.view_as(self.v[k]))
            steps.add(int(float(e["step"])))
            matched += 1
        if st and matched == 0:
            raise ValueError("no optimizer state entry matches a trained parameter: the state dict "
                             "indexes a different parameter list")
        if len(steps) > 1:
            raise ValueError(f"inconsistent Adam step counts in the state dict: {sorted(steps)}")
        self.t = steps.pop() if steps else 0
        g = sd.get("param_groups", [{}])[0]
        self.lr = g.get("lr", self.lr)
        self.betas = tuple(g.get("betas", self.betas))
        self.eps = g.get("eps", self.eps)

    def adam(self, grads: Dict[str, torch.Tensor]) -> None:
        """One Adam launch over the flat parameter / gradient / moment buffers (gradients not
        already in the flat gradient buffer are copied there first)."""
        self._check_layout()
        self.t += 1
        b1, b2 = self.betas
        for k in self.params:
            if grads[k].data_ptr() != self.g[k].data_ptr():
                self.g[k].copy_(grads[k].reshape(self.g[k].shape))
        check(lib().tt_adam_f32(self.flat_p.data_ptr(), self.flat_g.data_ptr(),
                                self.flat_m.data_ptr(), self.flat_v.data_ptr(),
                                self.flat_p.numel(), self.lr, b1, b2, self.eps, self.t,
                                stream_ptr()), "adam")

    def step(self, *args, group=None, **kw) -> torch.Tensor:
        """One optimiser step.  With an initialised process group (one process per GPU, the
        configs[4] 8-GPU layout) every rank runs its own batch and the gradients are averaged
        over ranks before Adam (data parallel, like DistributedDataParallel around the
        reference's model)."""
        loss, g = self.forward_backward(*args, **kw)
        allreduce_mean(g, group, flat=self.flat_g)
        self.adam(g)
        self.last_loss = loss
        return loss


def allreduce_mean(grads: Dict[str, torch.Tensor], group=None, flat: torch.Tensor = None) -> None:
    """Average gradient tensors over the ranks of ``group`` in place with ONE all-reduce of a
    flat bucket (the parameters of the trainable towers are ~0.5 M floats: one RCCL call over
    xGMI instead of one per tensor).  ``flat``: a buffer the gradients already are views of
    (TwoTowerTrainStep.flat_g) -- reduced in place, no packing.  No-op without an initialised
    multi-rank group."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    if flat is not None:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        flat.mul_(1.0 / world)
        return
    keys = sorted(grads)  # same order on every rank
    flat = torch.cat([grads[k].reshape(-1) for k in keys])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.mul_(1.0 / world)
    off = 0
    for k in keys:
        n = grads[k].numel()
        grads[k].copy_(flat[off:off + n].view_as(grads[k]))
        off += n
