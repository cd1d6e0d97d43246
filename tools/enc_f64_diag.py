"""Encoder error vs the float64 BertModel fixture (tests/golden/bert.npz pooled64), per
precision, beside the reference's own f32 deviation (f32_vs_f64_max); and the projection head
in f32 / x3 vs the reference ItemTower fixture (item_head.npz).  Diagnostic, prints JSON."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)

import make_bert_golden as mbg  # noqa: E402
import inputs as gi  # noqa: E402
from twotower.item_tower import BertEncoder, ItemTower, random_bert_state_dict  # noqa: E402


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "bert.npz"))
    sd = random_bert_state_dict(mbg.CFG, mbg.SEED)
    ids = torch.from_numpy(g["ids"]).cuda()
    cu = torch.from_numpy(g["cu_seqlens"]).cuda()
    mx = int(np.diff(g["cu_seqlens"]).max())
    out = {"f32_fixture_vs_f64_max": float(g["f32_vs_f64_max"])}
    for prec in ("f32", "x3", "bf16"):
        y = BertEncoder(sd, mbg.CFG, prec=prec).encode_packed(ids, cu, mx).cpu().double().numpy()
        d = np.abs(y - g["pooled64"])
        out[prec] = {"max_vs_f64": float(d.max()), "mean_vs_f64": float(d.mean()),
                     "ratio_to_f32_fixture": float(d.max() / g["f32_vs_f64_max"]),
                     "max_vs_f32_fixture": float(np.abs(y - g["pooled"]).max())}
    h = np.load(os.path.join(ROOT, "tests", "golden", "item_head.npz"))
    emb = gi.item_text_embeddings()

    class Stub:
        def get_sentence_embedding_dimension(self):
            return 384

        def encode(self, texts, **kw):
            return torch.from_numpy(emb[[int(t.split("#")[1]) for t in texts]])

    for use_cat in (False, True):
        for hp in ("f32", "x3"):
            it = ItemTower(use_categorical_features=use_cat, text_encoder=Stub())
            if use_cat:
                it.initialize_categorical_embeddings(gi.BRANDS, gi.CATEGORIES)
            with torch.no_grad():
                for k, v in gi.item_head_weights(use_cat).items():
                    dict(it.named_parameters())[k].copy_(torch.from_numpy(v))
            it.eval()
            it.head_prec = hp
            texts, brands, cats = gi.item_batch()
            with torch.no_grad():
                y = it(texts, brands if use_cat else None, cats if use_cat else None)
            tag = "cat" if use_cat else "nocat"
            out[f"head_{tag}_{hp}_max_vs_fixture"] = float(
                np.abs(y.cpu().numpy() - h[f"{tag}__out"]).max())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
