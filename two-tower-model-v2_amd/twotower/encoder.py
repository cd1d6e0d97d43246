"""EmbeddingEncoder on MI355X: drop-in for src/inference/encoder.py (class EmbeddingEncoder :15).

The inference caller of the hot path: ``encode_items`` (catalog encode, scripts/
generate_embeddings.py:42-60) and ``encode_buyer`` (the /retrieve request, src/api/server.py:
241-244), over the HIP item tower (twotower.item_tower) and buyer tower (twotower.buyer_tower).
Same constructor, checkpoint format (trainer.py:327-340: ``model_state_dict``, ``config``,
``brand_vocab``, ``category_vocab``), metadata handling, history rules (timestamp sort iff every
interaction has one, last ``max_interaction_history``, ``get_event_weight``) and errors.

Differences, all on paths where the reference fails or cannot run here:
  * checkpoint ``brand_vocab`` / ``category_vocab`` dicts are used as saved.  The reference
    passes them back through ``initialize_categorical_embeddings`` (encoder.py:80-102), which
    prepends a second '<UNK>' and builds a table one row larger than the checkpoint's, so its
    ``load_state_dict`` raises a size mismatch for every checkpoint the trainer writes.
  * the text encoder's weights are read from the checkpoint's sentence-transformers keys
    (``item_tower.text_encoder.0.auto_model.*`` = Hugging Face BertModel names); a checkpoint
    without them gets the seeded stand-in weights (the real MiniLM is not available offline).
  * checkpoints are read with ``torch.load(weights_only=True)`` (tensors and plain containers
    only, nothing executed from the file).
  * ``encode_buyers`` (batched, one item-tower pass for every history text of a batch) and the
    Mode B path (``set_item_embeddings``: history rows gathered from the resident catalog
    embeddings instead of re-encoded) are additions for throughput; ``encode_buyer`` keeps the
    reference's one-buyer Mode A semantics.
There is no CPU compute path: without a HIP device the towers raise.
"""
from __future__ import annotations

import copy
import json
import warnings
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from . import _lib, kernels
from .buyer_tower import BuyerTower
from .config import DEFAULT_CONFIG, get_event_weight, load_config
from .item_tower import MINILM_L12, ItemTower
from .two_tower import TwoTowerModel

ST_PREFIX = "item_tower.text_encoder.0.auto_model."  # SentenceTransformer module 0 = BertModel


def encoder_cfg_from_state_dict(sd: Dict[str, torch.Tensor]) -> Dict[str, Any]:
    """BertModel hyper-parameters from its weights (heads: MiniLM's 32-wide heads)."""
    word = sd["embeddings.word_embeddings.weight"]
    layers = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("encoder.layer."))
    hidden = word.shape[1]
    return dict(vocab=word.shape[0], hidden=hidden, layers=layers, heads=hidden // 32,
                intermediate=sd["encoder.layer.0.intermediate.dense.weight"].shape[0],
                max_positions=sd["embeddings.position_embeddings.weight"].shape[0],
                type_vocab=sd["embeddings.token_type_embeddings.weight"].shape[0],
                ln_eps=MINILM_L12["ln_eps"])


class EmbeddingEncoder:
    """Mirror of reference ``EmbeddingEncoder`` (src/inference/encoder.py:15-335)."""

    def __init__(self, model_path: Optional[str], config_path: Optional[str] = "configs/config.yaml",
                 device: Optional[str] = None, model: Optional[TwoTowerModel] = None,
                 tokenizer=None, prec: str = "x3", text_encoder=None):
        """reference :18-43.  ``config_path=None`` uses the reference's shipped config;
        ``model`` skips the checkpoint (an already-built TwoTowerModel); ``prec`` is the text
        encoder's GEMM precision: "x3" (default: split-bf16 products, the f32 fixture tolerance
        at 2x the f32 MFMA path's throughput), "f32" (f32 MFMA), "bf16" (throughput mode);
        ``text_encoder`` replaces the HIP MiniLM (any object with the SentenceTransformer
        surface ItemTower uses: ``encode``, ``get_sentence_embedding_dimension``)."""
        self.config = (load_config(config_path) if config_path is not None
                       else copy.deepcopy(DEFAULT_CONFIG))
        if device is not None and not str(device).startswith("cuda"):
            raise _lib.HipUnavailable(f"device {device!r}: the MI355X path has no CPU compute")
        self.device = _lib.device()
        self.model = (model if model is not None
                      else self._load_model(model_path, tokenizer, prec, text_encoder))
        self.model.eval()
        self.model.to(self.device)
        self.product_metadata = None
        self._table: Optional[torch.Tensor] = None  # Mode B: resident item embeddings
        self._table_rows: Optional[Dict[str, int]] = None

    # reference :45-130
    def _load_model(self, model_path: str, tokenizer=None, prec: str = "x3",
                    text_encoder=None) -> TwoTowerModel:
        checkpoint = torch.load(model_path, map_location="cpu", weights_only=True)
        model_config = (checkpoint["config"]["model"] if "config" in checkpoint
                        else self.config["model"])
        state_dict = dict(checkpoint["model_state_dict"])
        enc_sd = {k[len(ST_PREFIX):]: v.float() for k, v in state_dict.items()
                  if k.startswith(ST_PREFIX)}
        for k in [k for k in state_dict if k.startswith("item_tower.text_encoder.")]:
            del state_dict[k]
        it = model_config["item_tower"]
        if enc_sd:
            enc_cfg = encoder_cfg_from_state_dict(enc_sd)
        elif text_encoder is not None:
            enc_cfg = MINILM_L12
        else:
            warnings.warn("checkpoint holds no text-encoder weights: seeded stand-in MiniLM")
            enc_cfg = MINILM_L12
        item_tower = ItemTower(
            text_encoder_name=it["text_encoder"], embedding_dim=model_config["embedding_dim"],
            use_categorical_features=it["use_categorical_features"],
            categorical_embedding_dim=it["categorical_embedding_dim"],
            projection_hidden_dim=it["projection_hidden_dim"],
            freeze_text_encoder=self.config["training"]["freeze_text_encoder"],
            text_encoder=text_encoder, tokenizer=tokenizer, encoder_state_dict=enc_sd or None,
            encoder_cfg=enc_cfg, prec=prec)
        if it["use_categorical_features"]:
            for kind in ("brand", "category"):
                key = f"item_tower.{kind}_embedding.weight"
                saved = checkpoint.get(f"{kind}_vocab")
                if saved is not None:  # the saved string -> row mapping, as saved
                    rows = state_dict[key].shape[0] if key in state_dict else len(saved)
                    setattr(item_tower, f"{kind}_embedding",
                            nn.Embedding(rows, it["categorical_embedding_dim"], padding_idx=0))
                    setattr(item_tower, f"{kind}_vocab", dict(saved))
                elif key in state_dict:  # reference :104-116: dummy vocab of the saved size
                    dummy = [f"{kind}_{i}" for i in range(1, state_dict[key].shape[0])]
                    item_tower.initialize_categorical_embeddings(**{f"{kind}_vocab": dummy})
        bt = model_config["buyer_tower"]
        buyer_tower = BuyerTower(embedding_dim=model_config["embedding_dim"],
                                 aggregation_method=bt["aggregation_method"],
                                 attention_hidden_dim=bt["attention_hidden_dim"])
        model = TwoTowerModel(item_tower, buyer_tower)
        model.load_state_dict(state_dict)
        return model

    # reference :132-204
    def set_product_metadata(self, product_metadata: Dict):
        self.product_metadata = product_metadata
        item_tower = self.model.item_tower
        if not (item_tower.use_categorical_features
                and getattr(item_tower, "brand_embedding", None) is not None):
            return
        vocab_list = sorted(k for k in getattr(item_tower, "brand_vocab", {}) if k != "<UNK>")
        if not (vocab_list and vocab_list[0].startswith("brand_")):
            return
        for kind in ("brand", "category"):
            values = [p.get(kind) for p in product_metadata.values() if p.get(kind)]
            emb = getattr(item_tower, f"{kind}_embedding", None)
            size = emb.num_embeddings if emb is not None else None
            if not values or not size:
                continue
            uniq = sorted(set(values))
            if len(uniq) + 1 <= size:
                vocab = ["<UNK>"] + uniq
                while len(vocab) < size:
                    vocab.append(f"{kind}_dummy_{len(vocab)}")
            else:
                vocab = ["<UNK>"] + uniq[: size - 1]
            assert len(vocab) == size, f"{kind} vocab size mismatch: {len(vocab)} != {size}"
            setattr(item_tower, f"{kind}_vocab", {v: i for i, v in enumerate(vocab)})

    def _use_cat(self) -> bool:
        return bool(self.config["model"]["item_tower"]["use_categorical_features"])

    def _item_inputs(self, product_ids: Sequence[str]):
        texts, brands, categories = [], [], []
        meta = self.product_metadata or {}
        for pid in product_ids:
            m = meta.get(pid, {})
            texts.append(m.get("text", ""))
            brands.append(m.get("brand"))
            categories.append(m.get("category"))
        if not self._use_cat():
            return texts, None, None
        return texts, brands, categories

    # reference :206-242
    def encode_items(self, product_ids: List[str], batch_size: int = 32) -> np.ndarray:
        if self.product_metadata is None:
            raise ValueError("Product metadata must be set before encoding items")
        texts, brands, categories = self._item_inputs(product_ids)
        return self.model.item_tower.encode_batch(texts, brands, categories,
                                                  batch_size=batch_size)

    def _history(self, interactions: List[Dict[str, Any]]):
        """reference :262-273: timestamp sort iff all present, last max_history, weights."""
        if all(i.get("timestamp") is not None for i in interactions):
            interactions = sorted(interactions, key=lambda x: x["timestamp"])
        max_history = self.config["model"]["buyer_tower"]["max_interaction_history"]
        interactions = interactions[-max_history:]
        pids = [i["product_id"] for i in interactions]
        weights = [get_event_weight(i["event_type"], self.config) for i in interactions]
        return pids, weights

    # reference :244-305
    def encode_buyer(self, interactions: List[Dict[str, Any]]) -> np.ndarray:
        if self.product_metadata is None:
            raise ValueError("Product metadata must be set before encoding buyers")
        pids, weights = self._history(interactions)
        texts, brands, categories = self._item_inputs(pids)
        with torch.no_grad():
            items = self.model.item_tower(texts, brands, categories)
            w = torch.tensor(weights, dtype=torch.float32, device=self.device)
            buyer = self.model.buyer_tower(items.unsqueeze(0), w.unsqueeze(0))
        return buyer.squeeze(0).cpu().numpy()

    # ------------------------------------------------------------------ additions
    def set_item_embeddings(self, product_ids: Sequence[str], embeddings) -> None:
        """Mode B: keep the catalog's item embeddings (ItemTower outputs, e.g. the
        product_embeddings.npy of encode_items) resident in HBM; encode_buyers(mode="B")
        then gathers history rows instead of re-encoding their texts."""
        emb = torch.as_tensor(np.asarray(embeddings, dtype=np.float32))
        E = emb.shape[1]
        table = kernels.alloc_rows(emb.shape[0], E, self.device)
        table[:, :E].copy_(emb)
        self._table, self._table_rows = table, {p: i for i, p in enumerate(product_ids)}

    def encode_buyers(self, histories: Sequence[List[Dict[str, Any]]], mode: str = "A",
                      as_numpy: bool = True):
        """Batched encode_buyer: [B, E].  Mode "A" re-encodes every history text (one item
        tower pass for the whole batch), mode "B" gathers rows of set_item_embeddings.
        Histories are zero-weight padded to the longest one (weighted_avg: identical to the
        per-buyer result; attention: padded scores are 0, not -inf, as in the reference's
        own padded training path, which shifts the result at the 1e-7 level)."""
        if mode == "A" and self.product_metadata is None:
            raise ValueError("Product metadata must be set before encoding buyers")
        if mode == "B" and self._table is None:
            raise ValueError("set_item_embeddings must be called before mode='B'")
        E = self.model.item_tower.embedding_dim
        hist = [self._history(h) for h in histories]
        B, S = len(hist), max((len(p) for p, _ in hist), default=0)
        w = torch.zeros((B, max(S, 1)), dtype=torch.float32)
        for b, (_, wt) in enumerate(hist):
            w[b, : len(wt)] = torch.tensor(wt, dtype=torch.float32)
        w = w.to(self.device)
        unknown = []
        if mode == "B":  # ids outside the resident table: encoded like the reference does
            unknown = sorted({x for p, _ in hist for x in p if x not in self._table_rows})
        with torch.no_grad():
            if (mode == "B" and not unknown
                    and self.model.buyer_tower.aggregation_method == "weighted_avg"):
                rows = torch.zeros((B, max(S, 1)), dtype=torch.int64)
                for b, (p, _) in enumerate(hist):
                    rows[b, : len(p)] = torch.tensor([self._table_rows[x] for x in p],
                                                     dtype=torch.int64)
                out = kernels.gather_weighted_avg_l2(self._table, E, rows.to(self.device), w)
                out = out[:, :E]
            else:
                items = torch.zeros((B, max(S, 1), E), dtype=torch.float32, device=self.device)
                flat = [x for p, _ in hist for x in p]
                if flat:
                    if mode == "B":
                        enc = self._mode_b_rows(flat, unknown, E)
                    else:
                        enc = self.model.item_tower(*self._item_inputs(flat))
                    o = 0
                    for b, (p, _) in enumerate(hist):
                        items[b, : len(p)] = enc[o: o + len(p)]
                        o += len(p)
                out = self.model.buyer_tower(items, w)
        return out.cpu().numpy() if as_numpy else out

    def _mode_b_rows(self, flat, unknown, E):
        """History rows for Mode B: table rows for resident ids; an id missing from the table
        gets what encode_buyer would compute for it (its metadata, {} if unknown: text ' ',
        no brand / category, encoder.py:280-292), so Mode B never fails where Mode A works."""
        rows = [self._table_rows.get(x, -1) for x in flat]
        enc = torch.empty((len(flat), E), dtype=torch.float32, device=self.device)
        have = [i for i, r in enumerate(rows) if r >= 0]
        if have:
            enc[have] = self._table[torch.tensor([rows[i] for i in have], device=self.device), :E]
        if unknown:
            extra = self.model.item_tower(*self._item_inputs(unknown))
            pos = {x: j for j, x in enumerate(unknown)}
            miss = [i for i, r in enumerate(rows) if r < 0]
            enc[miss] = extra[torch.tensor([pos[flat[i]] for i in miss], device=self.device)]
        return enc

    # reference :307-335
    def save_item_embeddings(self, product_ids: List[str], embeddings: np.ndarray,
                             output_dir: str):
        output_dir = Path(output_dir)
        output_dir.mkdir(parents=True, exist_ok=True)
        np.save(output_dir / "product_embeddings.npy", embeddings)
        np.save(output_dir / "product_ids.npy", np.array(product_ids))
        with open(output_dir / "product_id_to_index.json", "w", encoding="utf-8") as f:
            json.dump({pid: idx for idx, pid in enumerate(product_ids)}, f, ensure_ascii=False,
                      indent=2)
        print(f"Saved {len(product_ids)} item embeddings to {output_dir}")
