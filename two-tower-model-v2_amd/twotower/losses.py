"""InfoNCELoss on MI355X: drop-in for src/training/losses.py (class InfoNCELoss :8).

Same constructor (temperature=0.07) and forward(buyer_embeddings, positive_embeddings,
negative_embeddings) -> scalar loss.  Forward and backward run in one HIP call
(tt_infonce_f32, csrc/tt_loss.hip): the in-batch logits are one MFMA GEMM instead of the
reference's expanded [B, B, E] bmm (:55-61), and the gradients are two more GEMMs; autograd
receives the precomputed input gradients.  ``prec="bf16"`` runs the GEMMs on bf16 MFMA
(configs[4]'s "MFMA bf16" training step); the default "f32" matches the reference to ~1e-6.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib
from ._lib import check, lib, require_device, stream_ptr


def infonce(b: torch.Tensor, p: torch.Tensor, n: torch.Tensor, temperature: float = 0.07,
            prec: str = "f32", grads: bool = True):
    """Device tensors b [B,E], p [B,E], n [B,N,E] -> (loss [] f32, (gb, gp, gn) or None)."""
    for t, name in ((b, "buyer_embeddings"), (p, "positive_embeddings"),
                    (n, "negative_embeddings")):
        require_device(t, name)
    b, p, n = (t.detach().contiguous().to(torch.float32) for t in (b, p, n))
    B, E = b.shape
    if p.shape != (B, E) or n.dim() != 3 or n.shape[0] != B or n.shape[2] != E:
        raise ValueError("InfoNCE: expected b [B,E], p [B,E], n [B,N,E]")
    N = n.shape[1]
    pr = _lib.TT_PREC_BF16 if prec == "bf16" else _lib.TT_PREC_F32
    need = ctypes.c_int64(0)
    check(lib().tt_infonce_workspace_bytes(B, N, E, pr, int(grads), ctypes.byref(need)),
          "tt_infonce_workspace_bytes")
    ws = torch.empty(need.value, dtype=torch.uint8, device=b.device)
    loss = torch.empty((), dtype=torch.float32, device=b.device)
    g = tuple(torch.empty_like(t) for t in (b, p, n)) if grads else (None, None, None)
    check(lib().tt_infonce_f32(b.data_ptr(), b.stride(0), p.data_ptr(), p.stride(0),
                               n.data_ptr(), n.stride(0), n.stride(1), B, N, E,
                               ctypes.c_float(temperature), pr, loss.data_ptr(),
                               *(t.data_ptr() if t is not None else None for t in g),
                               ws.data_ptr(), ws.numel(), stream_ptr()), "tt_infonce_f32")
    return loss, (g if grads else None)


class _InfoNCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, b, p, n, temperature, prec):
        need = any(ctx.needs_input_grad[:3])
        loss, g = infonce(b, p, n, temperature, prec, grads=need)
        if need:
            ctx.save_for_backward(*g)
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        gb, gp, gn = ctx.saved_tensors
        return grad_out * gb, grad_out * gp, grad_out * gn, None, None


class InfoNCELoss(nn.Module):
    """Mirror of reference ``InfoNCELoss`` (src/training/losses.py:8-79)."""

    def __init__(self, temperature: float = 0.07, prec: str = "f32"):
        super().__init__()
        self.temperature = temperature
        self.prec = prec

    def forward(self, buyer_embeddings: torch.Tensor, positive_embeddings: torch.Tensor,
                negative_embeddings: torch.Tensor) -> torch.Tensor:
        return _InfoNCEFn.apply(buyer_embeddings, positive_embeddings, negative_embeddings,
                                self.temperature, self.prec)
