"""TwoTowerModel on MI355X: drop-in for src/models/two_tower.py (class TwoTowerModel :10).

Composition only: the item tower (twotower.item_tower.ItemTower, HIP encoder + head) and
the buyer tower (twotower.buyer_tower.BuyerTower, HIP aggregation kernels).  Same methods,
arguments and output dictionaries as the reference (:33-218).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib


class TwoTowerModel(nn.Module):
    def __init__(self, item_tower, buyer_tower):
        super().__init__()
        self.item_tower = item_tower
        self.buyer_tower = buyer_tower
        assert item_tower.embedding_dim == buyer_tower.embedding_dim, \
            "Item and Buyer towers must have the same embedding dimension"

    def encode_items(self, texts: List[str], brands: Optional[List[str]] = None,
                     categories: Optional[List[str]] = None) -> torch.Tensor:
        return self.item_tower(texts, brands, categories)

    def encode_buyer(self, item_embeddings: torch.Tensor, weights: torch.Tensor) -> torch.Tensor:
        return self.buyer_tower(item_embeddings, weights)

    def _encode_products(self, positive_texts, negative_texts, positive_brands,
                         positive_categories, negative_brands, negative_categories, batch_size):
        pos = self.item_tower(positive_texts, positive_brands, positive_categories)
        all_neg = [t for lst in negative_texts for t in lst]
        nb = [b for lst in negative_brands for b in lst] if negative_brands else None
        nc = [c for lst in negative_categories for c in lst] if negative_categories else None
        neg = self.item_tower(all_neg, nb, nc)
        nneg = len(negative_texts[0]) if negative_texts else 0
        return pos, neg.view(batch_size, nneg, -1)

    # reference :67-153
    def forward(self, buyer_sequences: List[List[Tuple[str, int]]], positive_texts: List[str],
                negative_texts: List[List[str]], positive_brands=None, positive_categories=None,
                negative_brands=None, negative_categories=None,
                product_embeddings_cache: Optional[Dict[str, torch.Tensor]] = None):
        batch_size = len(buyer_sequences)
        dev = _lib.device()
        pos, neg = self._encode_products(positive_texts, negative_texts, positive_brands,
                                         positive_categories, negative_brands,
                                         negative_categories, batch_size)
        E = self.item_tower.embedding_dim
        out = []
        for seq in buyer_sequences:
            w = torch.tensor([wt for _, wt in seq], dtype=torch.float32, device=dev)
            if product_embeddings_cache:
                x = torch.stack([product_embeddings_cache.get(pid, torch.zeros(E, device=dev))
                                 .to(dev) for pid, _ in seq])
            else:  # the reference's placeholder (:138-141)
                x = torch.zeros(len(seq), E, device=dev)
            out.append(self.buyer_tower(x.unsqueeze(0), w.unsqueeze(0)).squeeze(0))
        return {"buyer_embeddings": torch.stack(out), "positive_embeddings": pos,
                "negative_embeddings": neg}

    # reference :155-218
    def forward_simplified(self, buyer_item_embeddings: torch.Tensor, buyer_weights: torch.Tensor,
                           positive_texts: List[str], negative_texts: List[List[str]],
                           positive_brands=None, positive_categories=None, negative_brands=None,
                           negative_categories=None) -> Dict[str, torch.Tensor]:
        batch_size = buyer_item_embeddings.shape[0]
        pos, neg = self._encode_products(positive_texts, negative_texts, positive_brands,
                                         positive_categories, negative_brands,
                                         negative_categories, batch_size)
        buyers = self.buyer_tower(buyer_item_embeddings, buyer_weights)
        return {"buyer_embeddings": buyers, "positive_embeddings": pos,
                "negative_embeddings": neg}
