"""Trainer on MI355X: drop-in for the reference's configs[4] training loop.

Reference: src/training/trainer.py (class Trainer :20).  Same constructor, attributes,
batch format (src/data/dataset.py collate_fn: buyer_ids, positive_product_ids,
negative_product_ids, buyer_sequences, positive_product_texts, negative_product_texts,
weights) and loop structure:

  _encode_buyer_sequences_batched  (:74-159)  history texts -> ONE text-encoder pass (the HIP
      MiniLM encoder) -> per buyer [max_interaction_history, H] zero-padded with weight 0;
      empty histories fall back to the positive text with weight 1; the last
      max_interaction_history items are kept.
  graph=True: each batch shape's forward + backward is captured once in a HIP graph and
      replayed (TwoTowerTrainStep(graph=True)).
  train_epoch (:161-243)  model.train(); per batch: the sequence encode above, brand /
      category lookups from the product metadata (:190-209), then ONE fused HIP step
      (twotower.train.TwoTowerTrainStep: item head incl. its train-mode Dropout + buyer
      attention + InfoNCE forward/backward + Adam) instead of forward_simplified ->
      criterion -> backward -> optimizer.step (:211-231).  The sentence encoder is frozen
      (freeze_text_encoder, item_tower.py:40-42), so the positive / negative text embeddings
      are inputs of the step, like the history rows.
  validate (:245-319)  the same forward in eval mode, loss only (no backward work).
  save_checkpoint / train (:321-378)  the reference's checkpoint dict (optimizer_state_dict
      in torch.optim.Adam's format) and epoch loop; load_checkpoint resumes from it.

The trainable parameters are those the reference's Adam updates with a frozen text encoder
(projection, brand / category embeddings, attention MLP); the fused step keeps Adam's moments
in HBM and writes the module parameters in place, so ``model.state_dict()`` is the trained
model.  The default pads every history to max_interaction_history (100) as the reference
does; ``pad_to_batch_max=True`` pads to the batch's longest history instead (the padded
positions carry weight 0 and contribute exactly nothing after the L2 normalisation, SURVEY.md
a5/a6, at a fraction of the work for S ~ 20).
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, List, Optional

import torch

from .config import DEFAULT_CONFIG, load_config
from .train import TwoTowerTrainStep


class Trainer:
    """Mirror of reference ``Trainer`` (src/training/trainer.py:20-380)."""

    def __init__(self, model, train_loader, val_loader=None,
                 config_path: Optional[str] = "configs/config.yaml", prec: str = "f32",
                 pad_to_batch_max: bool = False, graph: bool = False):
        self.model = model
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.config = load_config(config_path) if config_path else DEFAULT_CONFIG
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.model.to(self.device)
        tc = self.config["training"]
        self.step = TwoTowerTrainStep(model.item_tower, model.buyer_tower,
                                      temperature=tc["temperature"], lr=tc["learning_rate"],
                                      prec=prec, graph=graph)
        self.optimizer = self.step  # Adam lives in the fused step (moments resident in HBM)
        self.current_epoch = 0
        self.start_epoch = 0  # first epoch train() runs (load_checkpoint: saved epoch + 1)
        self.best_val_loss = float("inf")
        self.checkpoint_dir = Path(tc["checkpoint_dir"])
        self.product_metadata = None
        self.pad_to_batch_max = pad_to_batch_max

    def set_product_metadata(self, product_metadata: Dict):
        self.product_metadata = product_metadata

    # reference :74-159
    def _encode_buyer_sequences_batched(self, buyer_sequences, weights, positive_texts):
        max_seq_len = self.config["model"]["buyer_tower"]["max_interaction_history"]
        all_seq_texts: List[str] = []
        seq_lengths: List[int] = []
        seq_weights_all: List[List[float]] = []
        for seq, _ in zip(buyer_sequences, weights):
            seq_texts, seq_w = [], []
            for item in seq:
                if len(item) == 3:
                    product_id, weight, _ = item
                elif len(item) == 2:
                    product_id, weight = item
                else:
                    continue
                if self.product_metadata and product_id in self.product_metadata:
                    seq_texts.append(self.product_metadata[product_id]["text"])
                    seq_w.append(weight)
            if len(seq_texts) == 0:  # fallback: the positive product's text
                seq_texts = [positive_texts[len(seq_lengths)]]
                seq_w = [1.0]
            if len(seq_texts) > max_seq_len:
                seq_texts = seq_texts[-max_seq_len:]
                seq_w = seq_w[-max_seq_len:]
            seq_lengths.append(len(seq_texts))
            all_seq_texts.extend(seq_texts)
            seq_weights_all.append(seq_w)
        with torch.no_grad():  # ONE encoder pass for the whole batch (:128-131)
            all_emb = self.model.item_tower.encode_text(all_seq_texts).to(self.device)
        S = max(seq_lengths) if self.pad_to_batch_max else max_seq_len
        B, H = len(seq_lengths), all_emb.shape[1]
        items = torch.zeros((B, S, H), dtype=torch.float32, device=self.device)
        w = torch.zeros((B, S), dtype=torch.float32)
        o = 0
        for i, (n, sw) in enumerate(zip(seq_lengths, seq_weights_all)):
            items[i, :n] = all_emb[o:o + n]
            w[i, :n] = torch.tensor(sw, dtype=torch.float32)
            o += n
        return items, w.to(self.device)

    def _batch_inputs(self, batch):
        buyer_items, buyer_w = self._encode_buyer_sequences_batched(
            batch["buyer_sequences"], batch["weights"], batch["positive_product_texts"])
        it = self.model.item_tower
        pos_t = batch["positive_product_texts"]
        neg_t = batch["negative_product_texts"]
        B, N = len(pos_t), len(neg_t[0]) if neg_t else 0
        with torch.no_grad():  # frozen sentence encoder (item_tower.py:40-42)
            text = it.encode_text(list(pos_t) + [t for row in neg_t for t in row])
        pos_text, neg_text = text[:B], text[B:].view(B, N, -1)
        ids = [None] * 4
        if self.product_metadata and it.use_categorical_features \
                and it.brand_embedding is not None:
            md = self.product_metadata
            pb = [md.get(p, {}).get("brand") for p in batch["positive_product_ids"]]
            pc = [md.get(p, {}).get("category") for p in batch["positive_product_ids"]]
            nb = [md.get(p, {}).get("brand") for row in batch["negative_product_ids"] for p in row]
            nc = [md.get(p, {}).get("category") for row in batch["negative_product_ids"]
                  for p in row]
            dev = self.device
            ids = [torch.tensor(it._categorical_ids(b, c)[j], dtype=torch.int32, device=dev)
                   for b, c in ((pb, pc), (nb, nc)) for j in (0, 1)]
            ids[2], ids[3] = ids[2].view(B, N), ids[3].view(B, N)
        return buyer_items, buyer_w, pos_text, neg_text, ids

    # reference :161-243
    def train_epoch(self) -> float:
        self.model.train()
        total, n = 0.0, 0
        for batch in self.train_loader:
            items, w, pos, neg, (pb, pc, nb, nc) = self._batch_inputs(batch)
            loss = self.step.step(items, w, pos, neg, pb, pc, nb, nc)
            total += loss.item()
            n += 1
        return total / n if n > 0 else 0.0

    # reference :245-319
    def validate(self) -> float:
        if self.val_loader is None:
            return 0.0
        self.model.eval()
        total, n = 0.0, 0
        with torch.no_grad():
            for batch in self.val_loader:
                items, w, pos, neg, (pb, pc, nb, nc) = self._batch_inputs(batch)
                loss = self.step.forward_loss(items, w, pos, neg, pb, pc, nb, nc)
                total += loss.item()
                n += 1
        return total / n if n > 0 else 0.0

    # reference :321-352
    def save_checkpoint(self, is_best: bool = False):
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        checkpoint = {"epoch": self.current_epoch, "model_state_dict": self.model.state_dict(),
                      "optimizer_state_dict": self.step.optimizer_state_dict(self.model),
                      "best_val_loss": self.best_val_loss, "config": self.config}
        it = self.model.item_tower
        if getattr(it, "brand_vocab", None) is not None:
            checkpoint["brand_vocab"] = it.brand_vocab
        if getattr(it, "category_vocab", None) is not None:
            checkpoint["category_vocab"] = it.category_vocab
        torch.save(checkpoint, self.checkpoint_dir / f"checkpoint_epoch_{self.current_epoch + 1}.pt")
        if is_best:
            torch.save(checkpoint, self.checkpoint_dir / "best_model.pt")
            print(f"Saved best model with validation loss: {self.best_val_loss:.4f}")

    def load_checkpoint(self, path) -> Dict:
        """Resume from a save_checkpoint file (the reference saves but never reloads): model
        weights, Adam moments / step (torch.optim.Adam's state-dict format), epoch and best
        validation loss.  Read with weights_only=True."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(ck["model_state_dict"])
        self.model.to(self.device)
        if "optimizer_state_dict" in ck:
            self.step.load_optimizer_state_dict(self.model, ck["optimizer_state_dict"])
        self.current_epoch = int(ck.get("epoch", 0)) + 1
        self.start_epoch = self.current_epoch  # train() continues from here
        self.best_val_loss = float(ck.get("best_val_loss", float("inf")))
        return ck

    # reference :354-378 (a resumed Trainer continues at start_epoch: the checkpoint's epochs
    # are not re-run, and the epoch labels of later checkpoints continue from it)
    def train(self):
        num_epochs = self.config["training"]["num_epochs"]
        save_every = self.config["training"]["save_every_n_epochs"]
        for epoch in range(self.start_epoch, num_epochs):
            self.current_epoch = epoch
            train_loss = self.train_epoch()
            print(f"Epoch {epoch + 1}/{num_epochs} - Train Loss: {train_loss:.4f}")
            val_loss = self.validate()
            print(f"Epoch {epoch + 1}/{num_epochs} - Val Loss: {val_loss:.4f}")
            is_best = val_loss < self.best_val_loss
            if is_best:
                self.best_val_loss = val_loss
            if (epoch + 1) % save_every == 0 or is_best:
                self.save_checkpoint(is_best=is_best)
        print("Training completed!")
