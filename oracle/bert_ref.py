"""CPU float32 restatement of the item-tower text encoder (TEST INFRASTRUCTURE ONLY).

Follows Hugging Face BertModel (the architecture SentenceTransformer
"paraphrase-multilingual-MiniLM-L12-v2" wraps, reference src/models/item_tower.py:116) and
sentence-transformers mean pooling, over PACKED sequences (cu_seqlens), in plain torch:

  BertEmbeddings      (word[id] + token_type[0]) + position[p] -> LayerNorm(eps)
  BertSelfAttention   softmax(q k^T / sqrt(dh)) v per head, keys of the same sequence only
  BertSelfOutput      LayerNorm(dense(ctx) + x)
  BertIntermediate    gelu(dense(x))  (exact erf GELU)
  BertOutput          LayerNorm(dense(h) + x)
  Pooling (mean)      sum_t h_t / max(L, 1e-9)

Pinned against transformers.BertModel itself (tests/golden/bert.npz, made by
tests/golden/make_bert_golden.py, and directly when transformers is importable).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _ln(x, g, b, eps):
    return F.layer_norm(x, (x.shape[-1],), g, b, eps)


def bert_mean_pool(sd, cfg, ids, cu_seqlens, dtype=torch.float32, device="cpu"):
    """sd: HF BertModel state dict; ids [T] int; cu_seqlens [n+1] -> pooled [n, H] (computed on
    `device`: a float64 run of a 12-layer configs[1] batch is minutes on the CPU, a second on a
    GPU's torch -- still this restatement, not the product path)."""
    H, nh = cfg["hidden"], cfg["heads"]
    dh = H // nh
    ids = torch.as_tensor(ids, dtype=torch.long).to(device)
    cu = [int(v) for v in cu_seqlens]
    n = len(cu) - 1
    W = {k: v.to(device=device, dtype=dtype) for k, v in sd.items()}
    pos = torch.cat([torch.arange(cu[i + 1] - cu[i]) for i in range(n)]).to(device)
    x = (W["embeddings.word_embeddings.weight"][ids]
         + W["embeddings.token_type_embeddings.weight"][0]) \
        + W["embeddings.position_embeddings.weight"][pos]
    x = _ln(x, W["embeddings.LayerNorm.weight"], W["embeddings.LayerNorm.bias"], cfg["ln_eps"])
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."
        q = F.linear(x, W[p + "attention.self.query.weight"], W[p + "attention.self.query.bias"])
        k = F.linear(x, W[p + "attention.self.key.weight"], W[p + "attention.self.key.bias"])
        v = F.linear(x, W[p + "attention.self.value.weight"], W[p + "attention.self.value.bias"])
        ctx = torch.empty_like(x)
        for i in range(n):
            a, b = cu[i], cu[i + 1]
            qs = q[a:b].view(b - a, nh, dh).transpose(0, 1)
            ks = k[a:b].view(b - a, nh, dh).transpose(0, 1)
            vs = v[a:b].view(b - a, nh, dh).transpose(0, 1)
            att = torch.softmax(qs @ ks.transpose(1, 2) / math.sqrt(dh), dim=-1)
            ctx[a:b] = (att @ vs).transpose(0, 1).reshape(b - a, H)
        y = F.linear(ctx, W[p + "attention.output.dense.weight"],
                     W[p + "attention.output.dense.bias"]) + x
        x = _ln(y, W[p + "attention.output.LayerNorm.weight"],
                W[p + "attention.output.LayerNorm.bias"], cfg["ln_eps"])
        h = F.gelu(F.linear(x, W[p + "intermediate.dense.weight"], W[p + "intermediate.dense.bias"]))
        y = F.linear(h, W[p + "output.dense.weight"], W[p + "output.dense.bias"]) + x
        x = _ln(y, W[p + "output.LayerNorm.weight"], W[p + "output.LayerNorm.bias"], cfg["ln_eps"])
    return torch.stack([x[cu[i]:cu[i + 1]].sum(0) / max(cu[i + 1] - cu[i], 1e-9)
                        for i in range(n)])


def item_head(text_emb, sd_head, brand_ids=None, cat_ids=None):
    """ItemTower.forward after the text encoder (item_tower.py:194-209), float32 torch."""
    x = text_emb
    if brand_ids is not None or cat_ids is not None:
        parts = [x]
        for ids, key in ((brand_ids, "brand_embedding.weight"), (cat_ids, "category_embedding.weight")):
            tab = sd_head[key]
            parts.append(tab[torch.as_tensor(ids)] if ids is not None
                         else torch.zeros(x.shape[0], tab.shape[1]))
        x = torch.cat(parts, 1)
    h = torch.relu(F.linear(x, sd_head["projection.0.weight"], sd_head["projection.0.bias"]))
    y = F.linear(h, sd_head["projection.3.weight"], sd_head["projection.3.bias"])
    return F.normalize(y, p=2, dim=1)
