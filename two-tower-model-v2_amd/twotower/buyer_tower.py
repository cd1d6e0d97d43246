"""BuyerTower on MI355X: drop-in for the reference module.

Reference: src/models/buyer_tower.py (class BuyerTower :9).  Same constructor, submodule
names (``attention`` = Linear(E,H) -> ReLU -> Linear(H,1), so checkpoint keys
``buyer_tower.attention.{0,2}.{weight,bias}`` load unchanged), methods and errors.  The
forward arithmetic is the HIP kernels of csrc/tt_buyer.hip; inputs on the host are moved
to the HIP device and results moved back, so CPU-tensor callers keep working on an MI355X
box.  There is no CPU compute path: without a HIP device the forward raises.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib, kernels


class BuyerTower(nn.Module):
    """Mirror of reference ``BuyerTower`` (buyer_tower.py:9-146)."""

    def __init__(self, embedding_dim: int = 384, aggregation_method: str = "attention",
                 attention_hidden_dim: int = 128):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.aggregation_method = aggregation_method
        if aggregation_method == "attention":
            self.attention = nn.Sequential(
                nn.Linear(embedding_dim, attention_hidden_dim),
                nn.ReLU(),
                nn.Linear(attention_hidden_dim, 1),
            )
        elif aggregation_method == "weighted_avg":
            pass
        else:
            raise ValueError(f"Unknown aggregation method: {aggregation_method}")

    @staticmethod
    def _on_device(t: torch.Tensor) -> torch.Tensor:
        return t if t.is_cuda else t.to(_lib.device())

    def weighted_average(self, item_embeddings: torch.Tensor,
                         weights: torch.Tensor) -> torch.Tensor:
        """reference :43-68 -> tt_weighted_avg_l2_f32"""
        home = item_embeddings.device
        out = kernels.weighted_avg_l2(self._on_device(item_embeddings), self._on_device(weights))
        return out.to(home)

    def attention_aggregation(self, item_embeddings: torch.Tensor,
                              weights: torch.Tensor) -> torch.Tensor:
        """reference :70-101 -> tt_attn_agg_l2_f32"""
        home = item_embeddings.device
        l0, l2 = self.attention[0], self.attention[2]
        dev = _lib.device()
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from .autograd_ops import AttnAggFn  # training: HIP forward + backward

            out = AttnAggFn.apply(self._on_device(item_embeddings), self._on_device(weights),
                                  l0.weight.to(dev), l0.bias.to(dev), l2.weight.to(dev),
                                  l2.bias.to(dev))
            return out.to(home)
        out = kernels.attn_agg_l2(self._on_device(item_embeddings), self._on_device(weights),
                                  l0.weight.to(dev), l0.bias.to(dev), l2.weight.to(dev),
                                  l2.bias.to(dev))
        return out.to(home)

    def forward(self, item_embeddings: torch.Tensor, weights: torch.Tensor) -> torch.Tensor:
        """reference :103-122"""
        if self.aggregation_method == "weighted_avg":
            return self.weighted_average(item_embeddings, weights)
        elif self.aggregation_method == "attention":
            return self.attention_aggregation(item_embeddings, weights)
        else:
            raise ValueError(f"Unknown aggregation method: {self.aggregation_method}")

    def encode_from_sequence(self, item_embeddings: torch.Tensor,
                             weights: torch.Tensor) -> torch.Tensor:
        """reference :124-144"""
        if item_embeddings.dim() == 2:
            item_embeddings = item_embeddings.unsqueeze(0)
        if weights.dim() == 1:
            weights = weights.unsqueeze(0)
        return self.forward(item_embeddings, weights)
