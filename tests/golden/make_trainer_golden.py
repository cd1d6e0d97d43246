"""Fixture of the REFERENCE Trainer._encode_buyer_sequences_batched (trainer.py:74-159), run in
the build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_trainer_golden.py

The reference method is called unbound on a minimal `self` (config, product_metadata, device
cpu, model.item_tower.encode_text = a stand-in whose row for text j carries j + 1 in column 0),
so the padded [B, 100, 384] output reduces to which text sits in every slot (0 = padding)
plus the padded weights.  Inputs come from tests/golden/inputs.py (trainer_batch).
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs as gi  # noqa: E402

REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
sys.path.insert(0, REF)


def main():
    if "sentence_transformers" not in sys.modules:
        st = types.ModuleType("sentence_transformers")
        st.SentenceTransformer = object
        sys.modules["sentence_transformers"] = st
    if "faiss" not in sys.modules:
        sys.modules["faiss"] = types.ModuleType("faiss")
    if "tqdm" not in sys.modules:
        try:
            import tqdm  # noqa: F401
        except ImportError:
            tq = types.ModuleType("tqdm")
            tq.tqdm = lambda x, **k: x
            sys.modules["tqdm"] = tq
    from src.training.trainer import Trainer  # reference module

    meta, seqs, pos_texts = gi.trainer_batch()
    texts = gi.trainer_texts()
    tid = {t: j for j, t in enumerate(texts)}

    def encode_text(batch_texts):
        out = torch.zeros((len(batch_texts), 384))
        out[:, 0] = torch.tensor([tid[t] + 1 for t in batch_texts], dtype=torch.float32)
        return out

    fake = types.SimpleNamespace(
        config={"model": {"buyer_tower": {"max_interaction_history": 100}}},
        product_metadata=meta, device=torch.device("cpu"),
        model=types.SimpleNamespace(item_tower=types.SimpleNamespace(encode_text=encode_text)))
    weights = torch.ones(len(seqs))
    emb, w = Trainer._encode_buyer_sequences_batched(fake, seqs, weights, pos_texts)
    assert emb.shape == (len(seqs), 100, 384) and float(emb[:, :, 1:].abs().sum()) == 0.0
    np.savez_compressed(os.path.join(HERE, "trainer_seq.npz"),
                        slot_text=emb[:, :, 0].numpy().astype(np.int16), weights=w.numpy())
    print("trainer_seq.npz", os.path.getsize(os.path.join(HERE, "trainer_seq.npz")))


if __name__ == "__main__":
    main()
