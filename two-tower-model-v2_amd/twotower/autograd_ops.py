"""torch.autograd Functions over the HIP kernels, so the mirrored modules train under the
reference's own loop (loss.backward(); torch.optim.Adam(model.parameters()).step(),
src/training/trainer.py:49-52,74-243).

  AttnAggFn   BuyerTower.attention_aggregation (buyer_tower.py:70-101): gradients for the
              attention MLP (Linear(E,H) -> ReLU -> Linear(H,1)); item embeddings and event
              weights are inputs without gradient (pre-encoded history, two_tower.py:212).
  ItemHeadFn  ItemTower.forward after the text encoder (item_tower.py:194-209): concat with the
              brand/category embedding rows, projection, F.normalize; gradients for the
              projection, the embedding tables and (if required) the text embeddings.
"""
from __future__ import annotations

import torch

from . import _lib, kernels
from ._lib import check, lib, stream_ptr
from .train import GemmOps, _p, apply_dropout


class AttnAggFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, items, w, W1, b1, W2, b2):
        B, S, E = items.shape
        ops = GemmOps("f32", items.device)
        X = items.reshape(B * S, E).contiguous().float()
        w = w.contiguous().float()
        Hb = ops.gemm(X, W1.contiguous(), b1.contiguous(), _lib.TT_ACT_RELU)
        Hd = Hb.shape[1]
        alpha = torch.empty((B, S), dtype=torch.float32, device=items.device)
        onorm = torch.empty(B, dtype=torch.float32, device=items.device)
        z = torch.empty((B, E), dtype=torch.float32, device=items.device)
        W2c = W2.contiguous()
        check(lib().tt_attn_pool_fwd_f32(Hb.data_ptr(), Hd, W2c.data_ptr(), float(b2.item()),
                                         w.data_ptr(), X.data_ptr(), B, S, E, alpha.data_ptr(),
                                         onorm.data_ptr(), z.data_ptr(), E, stream_ptr()),
              "attn_pool_fwd")
        ctx.save_for_backward(X, w, Hb, alpha, onorm, z, W2c)
        ctx.shape = (B, S, E)
        return z

    @staticmethod
    def backward(ctx, dz):
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            raise NotImplementedError("gradients w.r.t. item embeddings / weights are not "
                                      "computed (the reference feeds pre-encoded history)")
        X, w, Hb, alpha, onorm, z, W2 = ctx.saved_tensors
        B, S, E = ctx.shape
        Hd = Hb.shape[1]
        ops = GemmOps("f32", X.device)
        dz = dz.contiguous()
        dW2 = torch.empty(Hd, dtype=torch.float32, device=X.device)
        db2 = torch.empty(1, dtype=torch.float32, device=X.device)
        dHb = torch.empty_like(Hb)
        da = torch.empty(B * S, dtype=torch.float32, device=X.device)
        check(lib().tt_attn_pool_bwd_f32(dz.data_ptr(), E, z.data_ptr(), E, onorm.data_ptr(),
                                         alpha.data_ptr(), w.data_ptr(), X.data_ptr(), B, S, E,
                                         Hb.data_ptr(), W2.data_ptr(), Hd, dW2.data_ptr(),
                                         db2.data_ptr(), dHb.data_ptr(), da.data_ptr(),
                                         stream_ptr()), "attn_pool_bwd")
        check(lib().tt_relu_backward_f32(dHb.data_ptr(), Hb.data_ptr(), dHb.numel(),
                                         stream_ptr()), "relu_bwd")
        return None, None, ops.dW(dHb, X), ops.colsum(dHb), dW2.view(1, Hd), db2


class ItemHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, text, bids, cids, brand_tab, cat_tab, W0, b0, W3, b3, keep=None, pdrop=0.0):
        dev = text.device
        ops = GemmOps("f32", dev)
        R, Ht = text.shape
        C = brand_tab.shape[1] if brand_tab is not None else 0
        width = Ht + 2 * C
        te = text.contiguous().float()
        x = torch.empty((R, width), dtype=torch.float32, device=dev)
        if brand_tab is not None:
            check(lib().tt_item_concat(te.data_ptr(), Ht, Ht, _p(bids),
                                       _p(brand_tab) if bids is not None else None, _p(cids),
                                       _p(cat_tab) if cids is not None else None, C, R,
                                       x.data_ptr(), width, None, stream_ptr()), "concat")
        else:
            x.copy_(te)
        if W0.shape[1] != width:
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({R}x{width} and "
                               f"{W0.shape[1]}x{W0.shape[0]})")
        h = ops.gemm(x, W0.contiguous(), b0.contiguous(), _lib.TT_ACT_RELU)
        if keep is not None:  # nn.Dropout (item_tower.py:61) in train mode
            apply_dropout(h, keep, pdrop)
        y = ops.gemm(h, W3.contiguous(), b3.contiguous())
        E = y.shape[1]
        z = kernels.l2norm_rows(y, E, _lib.TT_NORM_MAX_EPS, out=torch.empty_like(y))
        ctx.save_for_backward(x, h, y, z, W0, W3, bids, cids, keep)
        ctx.pdrop = pdrop
        ctx.dims = (Ht, C, brand_tab is not None,
                    tuple(brand_tab.shape) if brand_tab is not None else None,
                    tuple(cat_tab.shape) if cat_tab is not None else None)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, h, y, z, W0, W3, bids, cids, keep = ctx.saved_tensors
        Ht, C, use_cat, bshape, cshape = ctx.dims
        ops = GemmOps("f32", x.device)
        R, E = y.shape
        dz = dz.contiguous()
        dy = torch.empty_like(y)
        check(lib().tt_l2norm_backward_f32(y.data_ptr(), E, z.data_ptr(), E, dz.data_ptr(), E,
                                           R, E, dy.data_ptr(), E, stream_ptr()), "norm_bwd")
        db3, dW3 = ops.colsum(dy), ops.dW(dy, h)
        dh = ops.gemm(dy, ops.T(W3.contiguous(), ops.kpad(E)))
        if keep is not None:  # dropout backward (h is post-dropout: dropped entries are 0)
            apply_dropout(dh, keep, ctx.pdrop)
        check(lib().tt_relu_backward_f32(dh.data_ptr(), h.data_ptr(), dh.numel(), stream_ptr()),
              "relu_bwd")
        db0, dW0 = ops.colsum(dh), ops.dW(dh, x)
        need_x = ctx.needs_input_grad[0] or (use_cat and (ctx.needs_input_grad[3] or
                                                          ctx.needs_input_grad[4]))
        dtext = dbt = dct = None
        if need_x:
            dx = ops.gemm(dh, ops.T(W0.contiguous(), ops.kpad(dh.shape[1])))  # [R, width]
            if ctx.needs_input_grad[0]:
                dtext = dx[:, :Ht].contiguous()
            if use_cat:
                for key, ids, off, shape in (("b", bids, Ht, bshape), ("c", cids, Ht + C, cshape)):
                    gt = torch.zeros(shape, dtype=torch.float32, device=x.device)
                    if ids is not None:
                        check(lib().tt_embedding_backward_f32(dx[:, off:].data_ptr(), dx.stride(0),
                                                              ids.data_ptr(), R, C, gt.data_ptr(),
                                                              stream_ptr()), "emb_bwd")
                    if key == "b":
                        dbt = gt
                    else:
                        dct = gt
        return dtext, None, None, dbt, dct, dW0, db0, dW3, db3, None, None
