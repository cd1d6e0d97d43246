"""configs[0] pipeline fixtures produced by the REFERENCE scripts (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_pipeline_golden.py

BASELINE.json configs[0] is the reference's CPU workload: 1k products in its CSV schema,
100 buyers x 20 events, k = 10, run as
    scripts/generate_embeddings.py:17-64  (DataProcessor.load_products -> get_product_metadata
                                           -> EmbeddingEncoder.encode_items(batch 64) ->
                                           save_item_embeddings)
    scripts/build_index.py:16-63          (VectorDatabase.build_index -> save_index)
    scripts/evaluate.py:86-207            (prepare_test_data -> load_index -> Evaluator.evaluate_all,
                                           --k-values 1 5 10)
This script runs those three mains AS WRITTEN from /root/reference (read-only; never shipped,
never on the GPU box) in a scratch working directory holding synthetic CSVs
(tests/golden/inputs.py pipeline_products / pipeline_events), a config.yaml copied from the
reference with device cpu, and a checkpoint in the trainer's format (trainer.py:327-340) whose
weights come from inputs.pipeline_weights and which carries no vocab dicts (the dummy-vocab
path encoder.py:104-116 + set_product_metadata's reconstruction :132-204: the path on which the
reference loader works -- with saved vocab dicts it adds a second '<UNK>' and cannot load).

Stand-ins for the two third-party modules absent offline:
  * sentence_transformers.SentenceTransformer: encode() returns inputs.stub_text_embedding
    (deterministic per text) -- the MiniLM arithmetic is pinned separately (bert.npz);
  * faiss.IndexFlatIP: exact inner products (float64 accumulate, float32 out, ties to the lower
    row); write_index / read_index keep the stand-in's vectors (the .faiss bytes are not a
    fixture).
It also captures EmbeddingEncoder.encode_buyer's host rules (encoder.py:244-305) on
adversarial interaction lists: what reaches ItemTower.forward (texts, brands, categories)
and BuyerTower.forward (weights), and the buyer embedding.

Outputs: pipeline.json (metadata in index order, test pairs, evaluation results, encode_buyer
captures, vocab sizes) and pipeline.npz (reference embeddings of 128 rows, the side files of
both scripts byte for byte, encode_buyer outputs).
"""
from __future__ import annotations

import contextlib
import io
import json
import math
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs as gi  # noqa: E402

REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
sys.path.insert(0, REF)

K_VALUES = [1, 5, 10]
EMB_ROWS = 128  # reference embedding rows kept in the fixture (every n/128-th row)


class _IndexFlatIP:
    """Test-only stand-in for faiss.IndexFlatIP (exact search, module docstring)."""

    def __init__(self, d):
        self.d = int(d)
        self.xb = np.zeros((0, self.d), np.float32)
        self.ntotal = 0
        self.is_trained = True

    def add(self, x):
        x = np.ascontiguousarray(x)
        assert x.dtype == np.float32 and x.shape[1] == self.d
        self.xb = np.concatenate([self.xb, x])
        self.ntotal = self.xb.shape[0]

    def search(self, q, k):
        q = np.ascontiguousarray(q)
        assert q.dtype == np.float32 and q.shape[1] == self.d
        s = q.astype(np.float64) @ self.xb.astype(np.float64).T
        rows = np.broadcast_to(np.arange(self.ntotal), s.shape)
        order = np.lexsort((rows, -s), axis=1)[:, :k]
        return np.take_along_axis(s, order, 1).astype(np.float32), order.astype(np.int64)


def _install_stubs():
    import torch

    fa = types.ModuleType("faiss")
    fa.IndexFlatIP = _IndexFlatIP

    def write_index(index, path):
        with open(path, "wb") as f:
            np.save(f, index.xb)

    def read_index(path):
        with open(path, "rb") as f:
            xb = np.load(f)
        idx = _IndexFlatIP(xb.shape[1])
        idx.add(xb)
        return idx

    fa.write_index, fa.read_index = write_index, read_index
    sys.modules["faiss"] = fa

    class SentenceTransformer(torch.nn.Module):
        def __init__(self, name, *a, **k):
            super().__init__()

        def get_sentence_embedding_dimension(self):
            return 384

        def encode(self, texts, convert_to_tensor=True, show_progress_bar=False,
                   normalize_embeddings=False, device=None, **k):
            return torch.from_numpy(gi.stub_text_embedding(list(texts)))

    st = types.ModuleType("sentence_transformers")
    st.SentenceTransformer = SentenceTransformer
    sys.modules["sentence_transformers"] = st


def _clean(v):
    """pandas cell -> JSON value (NaN -> None, numpy scalars -> Python)."""
    if v is None:
        return None
    if isinstance(v, float) and math.isnan(v):
        return None
    if hasattr(v, "item"):
        v = v.item()
        if isinstance(v, float) and math.isnan(v):
            return None
    return v


def _write_inputs(work):
    import pandas as pd
    import yaml

    os.makedirs(os.path.join(work, "data"))
    os.makedirs(os.path.join(work, "configs"))
    os.makedirs(os.path.join(work, "checkpoints"))
    prows = gi.pipeline_products()
    pd.DataFrame(prows, columns=["id", "title", "description", "metadata"]).to_csv(
        os.path.join(work, "data", "products.csv"), index=False)
    erows = gi.pipeline_events([r["id"] for r in prows])
    pd.DataFrame(erows, columns=["distinct_id", "product_id", "event_name", "created_at"]).to_csv(
        os.path.join(work, "data", "events.csv"), index=False)
    with open(os.path.join(REF, "configs", "config.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["inference"]["device"] = "cpu"
    with open(os.path.join(work, "configs", "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    return cfg


def _write_checkpoint(cfg):
    import torch

    from src.data.processor import DataProcessor
    from src.models.buyer_tower import BuyerTower
    from src.models.item_tower import ItemTower
    from src.models.two_tower import TwoTowerModel

    proc = DataProcessor()
    meta = proc.get_product_metadata(proc.load_products())
    brands = [m["brand"] for m in meta.values() if m.get("brand")]
    cats = [m["category"] for m in meta.values() if m.get("category")]
    mc = cfg["model"]
    it = ItemTower(mc["item_tower"]["text_encoder"], mc["embedding_dim"], True,
                   mc["item_tower"]["categorical_embedding_dim"],
                   mc["item_tower"]["projection_hidden_dim"], True)
    it.initialize_categorical_embeddings(brands, cats)
    model = TwoTowerModel(it, BuyerTower(mc["embedding_dim"], mc["buyer_tower"]["aggregation_method"],
                                         mc["buyer_tower"]["attention_hidden_dim"]))
    n_brand, n_cat = len(it.brand_vocab), len(it.category_vocab)
    w = gi.pipeline_weights(n_brand, n_cat)
    sd = model.state_dict()
    assert set(sd) == set(w), sorted(set(sd) ^ set(w))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    torch.save({"epoch": 0, "model_state_dict": model.state_dict(), "best_val_loss": 0.0,
                "config": cfg}, os.path.join("checkpoints", "best_model.pt"))
    return n_brand, n_cat


def _run_main(module_name, argv):
    import importlib

    mod = importlib.import_module(module_name)
    old = sys.argv
    sys.argv = argv
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            mod.main()
    finally:
        sys.argv = old


def _encode_buyer_captures(product_ids):
    import torch

    from src.data.processor import DataProcessor
    from src.inference.encoder import EmbeddingEncoder

    enc = EmbeddingEncoder("checkpoints/best_model.pt")
    proc = DataProcessor()
    enc.set_product_metadata(proc.get_product_metadata(proc.load_products()))
    it, bt = enc.model.item_tower, enc.model.buyer_tower
    it_fwd, bt_fwd = it.forward, bt.forward
    cap = {}

    def it_capture(texts, brands=None, categories=None):
        cap["texts"], cap["brands"], cap["categories"] = list(texts), brands, categories
        return it_fwd(texts, brands, categories)

    def bt_capture(item_embeddings, weights):
        cap["weights"] = weights[0].tolist()
        return bt_fwd(item_embeddings, weights)

    it.forward, bt.forward = it_capture, bt_capture
    cases, outs = [], []
    for inter in gi.encoder_buyer_cases(product_ids):
        cap.clear()
        with torch.no_grad():
            y = enc.encode_buyer(inter)
        cases.append({"interactions": inter, "texts": cap["texts"],
                      "brands": [_clean(b) for b in cap["brands"]] if cap["brands"] else None,
                      "categories": [_clean(c) for c in cap["categories"]] if cap["categories"]
                      else None, "weights": cap["weights"]})
        outs.append(y.astype(np.float32))
    return cases, np.stack(outs)


def main():
    _install_stubs()
    np.random.seed(0)
    here_out = {}
    with tempfile.TemporaryDirectory() as work:
        cwd = os.getcwd()
        os.chdir(work)
        try:
            cfg = _write_inputs(work)
            n_brand, n_cat = _write_checkpoint(cfg)
            _run_main("scripts.generate_embeddings", ["generate_embeddings.py"])
            _run_main("scripts.build_index", ["build_index.py"])
            _run_main("scripts.evaluate", ["evaluate.py", "--k-values"] +
                      [str(k) for k in K_VALUES] + ["--output", "outputs/eval.json"])
            from scripts.evaluate import prepare_test_data
            from src.data.processor import DataProcessor

            proc = DataProcessor()
            products = proc.load_products()
            meta = proc.get_product_metadata(products)
            with contextlib.redirect_stdout(io.StringIO()):
                pairs = prepare_test_data(proc.load_events(), products)
            emb = np.load("outputs/embeddings/product_embeddings.npy")
            ids = np.load("outputs/embeddings/product_ids.npy").tolist()
            assert ids == list(meta)
            raw = lambda p: np.frombuffer(open(p, "rb").read(), np.uint8)  # noqa: E731
            rows = np.linspace(0, len(ids) - 1, EMB_ROWS).astype(np.int64)
            here_out.update({
                "emb_rows": rows, "emb": emb[rows], "emb_norm_sum": np.float64(
                    np.linalg.norm(emb.astype(np.float64), axis=1).sum()),
                "emb_ids_npy": raw("outputs/embeddings/product_ids.npy"),
                "emb_map_json": raw("outputs/embeddings/product_id_to_index.json"),
                "index_ids_npy": raw("outputs/index/product_ids.npy"),
                "index_map_json": raw("outputs/index/product_id_to_index.json"),
            })
            with open("outputs/eval.json", encoding="utf-8") as f:
                results = json.load(f)
            cases, outs = _encode_buyer_captures(ids)
            here_out["encode_buyer_out"] = outs
            doc = {
                "k_values": K_VALUES, "n_brand": n_brand, "n_cat": n_cat,
                "config": cfg,
                "metadata": [[pid, {"text": _clean(m.get("text")), "brand": _clean(m.get("brand")),
                                    "category": _clean(m.get("category"))}]
                             for pid, m in meta.items()],
                "test_pairs": [[b, inter, sorted(rel)] for b, inter, rel in pairs],
                "results": results,
                "encode_buyer_cases": cases,
            }
        finally:
            os.chdir(cwd)
    with open(os.path.join(HERE, "pipeline.json"), "w", encoding="utf-8") as f:
        json.dump(doc, f, ensure_ascii=False, indent=0)
    np.savez_compressed(os.path.join(HERE, "pipeline.npz"), **here_out)
    for name in ("pipeline.json", "pipeline.npz"):
        print(name, os.path.getsize(os.path.join(HERE, name)))


if __name__ == "__main__":
    main()
