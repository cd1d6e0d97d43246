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


class TwoTowerTrainStep:
    """One optimizer step of the item head + buyer attention under InfoNCE (Adam)."""

    def __init__(self, item_tower, buyer_tower, temperature: float = 0.07, lr: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, prec: str = "f32"):
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
        self.params = self._params()
        self.m = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.t = 0
        self.last_loss = None
        # nn.Dropout(0.1) of the projection (item_tower.py:61): active when the item tower is
        # in train mode, as under the reference Trainer (model.train(), trainer.py:167)
        self.keep_fn = dropout_keep

    def _params(self) -> Dict[str, torch.Tensor]:
        it, bt = self.it, self.bt
        p = {"proj0.w": it.projection[0].weight, "proj0.b": it.projection[0].bias,
             "proj3.w": it.projection[3].weight, "proj3.b": it.projection[3].bias}
        if self.attention:  # weighted_avg has no parameters (buyer_tower.py:43-68)
            p.update({"att0.w": bt.attention[0].weight, "att0.b": bt.attention[0].bias,
                      "att2.w": bt.attention[2].weight, "att2.b": bt.attention[2].bias})
        if it.use_categorical_features and it.brand_embedding is not None:
            p["brand"] = it.brand_embedding.weight
            p["cat"] = it.category_embedding.weight
        for v in p.values():
            if not v.is_contiguous():
                raise ValueError("parameters must be contiguous")
        return {k: v.data for k, v in p.items()}

    def _gemm(self, A, W, bias=None, act=0, res=None):
        return self.ops.gemm(A, W, bias, act, res)

    def _kpad(self, k):
        return self.ops.kpad(k)

    def _T(self, x, ld=None):
        return self.ops.T(x, ld)

    def _dW(self, dY, X):
        return self.ops.dW(dY, X)

    def _colsum(self, x):
        return self.ops.colsum(x)

    # ------------------------------------------------------------------ the step
    def forward_loss(self, *args, **kw) -> torch.Tensor:
        """The loss alone (the reference's validate: forward + criterion under no_grad,
        trainer.py:245-319): no backward GEMMs, no gradients."""
        return self.forward_backward(*args, grads=False, **kw)[0]

    def forward_backward(self, buyer_items, weights, pos_text, neg_text, pos_brand=None,
                         pos_cat=None, neg_brand=None, neg_cat=None, grads: bool = True):
        """buyer_items [B,S,E], weights [B,S], pos_text [B,Ht], neg_text [B,N,Ht] (device f32);
        *_brand / *_cat: int32 id tensors (vocab ids, 0 = <UNK>) or None.
        Returns (loss tensor, grads dict keyed like self.params; {} when grads=False)."""
        P = self.params
        B, S, E = buyer_items.shape
        N = neg_text.shape[1]
        Ht = pos_text.shape[1]
        R = B + B * N
        use_cat = "brand" in P
        C = self.it.categorical_embedding_dim if use_cat else 0
        text = torch.cat([pos_text, neg_text.reshape(B * N, Ht)]).contiguous()
        width = Ht + 2 * C
        x = torch.empty((R, width), dtype=torch.float32, device=self.dev)
        bids = cids = None
        if use_cat:
            def ids(a, b_):
                if a is None and b_ is None:
                    return None
                a = a if a is not None else torch.zeros(B, dtype=torch.int32, device=self.dev)
                b_ = b_ if b_ is not None else torch.zeros(B * N, dtype=torch.int32, device=self.dev)
                return torch.cat([a.reshape(-1), b_.reshape(-1)]).to(torch.int32).contiguous()
            bids, cids = ids(pos_brand, neg_brand), ids(pos_cat, neg_cat)
            check(lib().tt_item_concat(text.data_ptr(), Ht, Ht, _p(bids),
                                       _p(P["brand"]) if bids is not None else None, _p(cids),
                                       _p(P["cat"]) if cids is not None else None, C, R,
                                       x.data_ptr(), width, None, stream_ptr()), "concat")
        else:
            x.copy_(text)
        # item head forward (Linear -> ReLU -> Dropout -> Linear)
        h = self._gemm(x, P["proj0.w"], P["proj0.b"], _lib.TT_ACT_RELU)
        pdrop = self.it.projection[2].p if self.it.training else 0.0
        keep = self.keep_fn(h.shape, pdrop, self.dev) if pdrop > 0 else None
        if keep is not None:
            apply_dropout(h, keep, pdrop)
        y = self._gemm(h, P["proj3.w"], P["proj3.b"])
        z = kernels.l2norm_rows(y, E, _lib.TT_NORM_MAX_EPS, out=torch.empty_like(y))
        w = weights.contiguous().to(torch.float32)
        if not self.attention:  # weighted average + F.normalize: no trainable parameters
            zb = kernels.weighted_avg_l2(buyer_items, w)
        else:  # buyer attention forward
            X = buyer_items.reshape(B * S, E).contiguous()
            Hb = self._gemm(X, P["att0.w"], P["att0.b"], _lib.TT_ACT_RELU)
            Hd = Hb.shape[1]
            alpha = torch.empty((B, S), dtype=torch.float32, device=self.dev)
            onorm = torch.empty(B, dtype=torch.float32, device=self.dev)
            zb = torch.empty((B, E), dtype=torch.float32, device=self.dev)
            b2 = float(P["att2.b"].item())
            check(lib().tt_attn_pool_fwd_f32(Hb.data_ptr(), Hd, P["att2.w"].data_ptr(), b2,
                                             w.data_ptr(), X.data_ptr(), B, S, E,
                                             alpha.data_ptr(), onorm.data_ptr(), zb.data_ptr(),
                                             E, stream_ptr()), "attn_pool_fwd")
        # InfoNCE forward + backward
        if not grads:
            return infonce(zb, z[:B], z[B:].view(B, N, E), self.tau, self.prec, grads=False)[0], {}
        loss, (gb, gp, gn) = infonce(zb, z[:B], z[B:].view(B, N, E), self.tau, self.prec)
        g = {}
        # item head backward
        dz = torch.cat([gp, gn.reshape(B * N, E)]).contiguous()
        dy = torch.empty_like(y)
        check(lib().tt_l2norm_backward_f32(y.data_ptr(), E, z.data_ptr(), E, dz.data_ptr(), E,
                                           R, E, dy.data_ptr(), E, stream_ptr()), "norm_bwd")
        g["proj3.b"] = self._colsum(dy)
        g["proj3.w"] = self._dW(dy, h)
        dh = self._gemm(dy, self._T(P["proj3.w"], self._kpad(E)))       # dy W3
        if keep is not None:  # dropout backward; h is post-dropout (dropped entries 0)
            apply_dropout(dh, keep, pdrop)
        check(lib().tt_relu_backward_f32(dh.data_ptr(), h.data_ptr(), dh.numel(), stream_ptr()),
              "relu_bwd")
        g["proj0.b"] = self._colsum(dh)
        g["proj0.w"] = self._dW(dh, x)
        if use_cat:
            W0cat = P["proj0.w"][:, Ht:].contiguous()                     # [hid, 2C]
            dxc = self._gemm(dh, self._T(W0cat, self._kpad(dh.shape[1])))  # [R, 2C]
            for key, idsv, off in (("brand", bids, 0), ("cat", cids, C)):
                gt = torch.zeros_like(P[key])
                if idsv is not None:
                    check(lib().tt_embedding_backward_f32(dxc[:, off:].data_ptr(), dxc.stride(0),
                                                          idsv.data_ptr(), R, C, gt.data_ptr(),
                                                          stream_ptr()), "emb_bwd")
                g[key] = gt
        if not self.attention:
            return loss, g
        # buyer attention backward
        dW2 = torch.empty(Hd, dtype=torch.float32, device=self.dev)
        db2 = torch.empty(1, dtype=torch.float32, device=self.dev)
        dHb = torch.empty_like(Hb)
        da = torch.empty(B * S, dtype=torch.float32, device=self.dev)
        check(lib().tt_attn_pool_bwd_f32(gb.data_ptr(), E, zb.data_ptr(), E, onorm.data_ptr(),
                                         alpha.data_ptr(), w.data_ptr(), X.data_ptr(), B, S, E,
                                         Hb.data_ptr(), P["att2.w"].data_ptr(), Hd,
                                         dW2.data_ptr(), db2.data_ptr(), dHb.data_ptr(),
                                         da.data_ptr(), stream_ptr()), "attn_pool_bwd")
        check(lib().tt_relu_backward_f32(dHb.data_ptr(), Hb.data_ptr(), dHb.numel(),
                                         stream_ptr()), "relu_bwd")
        g["att2.w"] = dW2.view_as(P["att2.w"])
        g["att2.b"] = db2.view_as(P["att2.b"])
        g["att0.b"] = self._colsum(dHb)
        g["att0.w"] = self._dW(dHb, X)
        return loss, g

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
        self.t += 1
        b1, b2 = self.betas
        for k, p in self.params.items():
            gk = grads[k].contiguous()
            check(lib().tt_adam_f32(p.data_ptr(), gk.data_ptr(), self.m[k].data_ptr(),
                                    self.v[k].data_ptr(), p.numel(), self.lr, b1, b2, self.eps,
                                    self.t, stream_ptr()), "adam")

    def step(self, *args, group=None, **kw) -> torch.Tensor:
        """One optimiser step.  With an initialised process group (one process per GPU, the
        configs[4] 8-GPU layout) every rank runs its own batch and the gradients are averaged
        over ranks before Adam (data parallel, like DistributedDataParallel around the
        reference's model)."""
        loss, g = self.forward_backward(*args, **kw)
        allreduce_mean(g, group)
        self.adam(g)
        self.last_loss = loss
        return loss


def allreduce_mean(grads: Dict[str, torch.Tensor], group=None) -> None:
    """Average gradient tensors over the ranks of ``group`` in place with ONE all-reduce of a
    flat bucket (the parameters of the trainable towers are ~0.5 M floats: one RCCL call over
    xGMI instead of one per tensor).  No-op without an initialised multi-rank group."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
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
