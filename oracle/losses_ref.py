"""torch float64/float32 restatement of InfoNCELoss (TEST INFRASTRUCTURE ONLY).

Follows src/training/losses.py:20-79 term by term (positive, explicit negatives, in-batch
negatives with the diagonal masked to -inf, cross-entropy against column 0); autograd gives
the reference gradients.  Pinned to the reference's own outputs in tests/golden/infonce.npz.
"""
import torch
import torch.nn.functional as F


def infonce(b, p, n, tau):
    B = b.shape[0]
    pos = (b * p).sum(dim=1) / tau
    neg = torch.bmm(b.unsqueeze(1), n.transpose(1, 2)).squeeze(1) / tau
    inb = (b @ p.T) / tau
    inb = inb.masked_fill(torch.eye(B, dtype=torch.bool, device=b.device), float("-inf"))
    logits = torch.cat([pos.unsqueeze(1), neg, inb], dim=1)
    return F.cross_entropy(logits, torch.zeros(B, dtype=torch.long, device=b.device))
