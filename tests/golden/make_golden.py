"""Generate golden fixtures from the REFERENCE implementation (run in the build container).

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python tests/golden/make_golden.py

What is imported from the reference (read-only at /root/reference; never shipped):
  src.models.buyer_tower.BuyerTower      (buyer_tower.py:9)   -> buyer_*.npz
  src.training.losses.InfoNCELoss        (losses.py:8)        -> infonce.npz
  src.utils.config.get_event_weight      (config.py:27)       -> event_weights.json
  src.evaluation.metrics (functions + Evaluator, stub encoder / index) -> metrics.json
  src.models.item_tower.ItemTower        (item_tower.py:10)   -> item_head.npz; the module
      imports sentence_transformers (absent offline), so a test-only stand-in module supplies
      a SentenceTransformer whose encode() returns fixed, seeded 384-d "text embeddings": the
      reference's own categorical / projection / normalize code (:126-211) is what runs.
faiss (vector_db.py) is not installed: flatip.npz holds an fp64 restatement of
IndexFlatIP.search (oracle/oracle.py) plus the reference's numpy normalisation expression.

Fixtures hold seeds, expected outputs and a sha256 of the regenerated inputs (inputs are
re-created from the seeds by tests/golden/inputs.py, so the files stay small).
"""
from __future__ import annotations

import json
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


def buyer_fixtures():
    from src.models.buyer_tower import BuyerTower  # reference module

    out = {}
    for name, spec in gi.BUYER_CASES.items():
        items, w = gi.buyer_inputs(spec)
        with torch.no_grad():
            if spec["method"] == "weighted_avg":
                bt = BuyerTower(spec["E"], "weighted_avg")
                y = bt(torch.from_numpy(items), torch.from_numpy(w)).numpy()
            else:
                bt = BuyerTower(spec["E"], "attention", spec.get("H", 128))
                W1, b1, W2, b2 = gi.attn_weights(spec)
                bt.attention[0].weight.copy_(torch.from_numpy(W1))
                bt.attention[0].bias.copy_(torch.from_numpy(b1))
                bt.attention[2].weight.copy_(torch.from_numpy(W2))
                bt.attention[2].bias.copy_(torch.from_numpy(b2))
                y = bt(torch.from_numpy(items), torch.from_numpy(w)).numpy()
        out[name] = y.astype(np.float32)
        out[name + "__sha"] = np.frombuffer(gi.sha(items, w).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "buyer.npz"), **out)


def infonce_fixtures():
    from src.training.losses import InfoNCELoss

    out = {}
    for name, spec in gi.INFONCE_CASES.items():
        b, p, n = gi.infonce_inputs(spec)
        bt, pt, nt = (torch.from_numpy(a).requires_grad_(True) for a in (b, p, n))
        loss = InfoNCELoss(spec["tau"])(bt, pt, nt)
        loss.backward()
        out[name + "__loss"] = np.array([loss.item()], np.float64)
        if spec["B"] <= 8:  # keep the fixture small: gradients only for the small case
            out[name + "__gb"] = bt.grad.numpy()
            out[name + "__gp"] = pt.grad.numpy()
            out[name + "__gn"] = nt.grad.numpy()
        else:
            out[name + "__gnorm"] = np.array([bt.grad.norm().item(), pt.grad.norm().item(),
                                              nt.grad.norm().item()], np.float64)
    np.savez_compressed(os.path.join(HERE, "infonce.npz"), **out)


def event_weight_fixtures():
    from src.utils.config import get_event_weight

    cfg = {"event_weights": {"view": 1, "add_to_cart": 5, "purchase": 10}}
    names = ["view", "View", "VIEW", "add_to_cart", "AddToCart", "addtocart", "purchase",
             "Purchase", "buy", "BUY", "wishlist", "", "click", "add-to-cart"]
    table = {n: get_event_weight(n, cfg) for n in names}
    with open(os.path.join(HERE, "event_weights.json"), "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)


def item_head_fixtures():
    """ItemTower projection/categorical/normalize path with a stand-in text encoder."""
    text_emb = gi.item_text_embeddings()

    class _StubST(torch.nn.Module):  # test-only stand-in for sentence_transformers
        def __init__(self, name):
            super().__init__()
            self._p = torch.nn.Parameter(torch.zeros(1))

        def get_sentence_embedding_dimension(self):
            return 384

        def encode(self, texts, **kw):
            idx = [int(t.split("#")[1]) if "#" in t else 0 for t in texts]
            return torch.from_numpy(text_emb[idx])

    mod = types.ModuleType("sentence_transformers")
    mod.SentenceTransformer = _StubST
    sys.modules["sentence_transformers"] = mod
    from src.models.item_tower import ItemTower  # reference module

    out = {}
    for use_cat in (False, True):
        it = ItemTower(use_categorical_features=use_cat)
        if use_cat:
            it.initialize_categorical_embeddings(gi.BRANDS, gi.CATEGORIES)
        with torch.no_grad():  # seeded weights (regenerated by the tests, not stored)
            for kname, v in gi.item_head_weights(use_cat).items():
                dict(it.named_parameters())[kname].copy_(torch.from_numpy(v))
        it.eval()
        texts, brands, cats = gi.item_batch()
        with torch.no_grad():
            y = it(texts, brands if use_cat else None, cats if use_cat else None).numpy()
        tag = "cat" if use_cat else "nocat"
        out[f"{tag}__out"] = y
        out[f"{tag}__keys"] = np.array(sorted(k for k in it.state_dict()
                                              if not k.startswith("text_encoder")))
        if use_cat:
            out[f"{tag}__brand_vocab"] = np.array(sorted(it.brand_vocab, key=it.brand_vocab.get))
            out[f"{tag}__category_vocab"] = np.array(
                sorted(it.category_vocab, key=it.category_vocab.get))
    np.savez_compressed(os.path.join(HERE, "item_head.npz"), **out)


def flatip_fixtures():
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from oracle import oracle as orc

    out = {}
    for name, spec in gi.FLATIP_CASES.items():
        x, q = gi.flatip_inputs(spec)
        xn = orc.vector_db_normalize(x)          # the reference's numpy expression
        qn = orc.vector_db_normalize(q)
        k = min(spec["k"], x.shape[0])           # reference clamp, vector_db.py:159
        s, i = orc.flatip_search_f64(xn, qn, k)
        out[name + "__xn_sha"] = np.frombuffer(gi.sha(xn).encode(), np.uint8)
        out[name + "__qn"] = qn
        out[name + "__s64"] = s
        out[name + "__i"] = i
    np.savez_compressed(os.path.join(HERE, "flatip.npz"), **out)


def _stub_sentence_transformers():
    """test-only stand-in module so that reference modules importing it load (see item_head)."""
    if "sentence_transformers" in sys.modules:
        return

    class _StubST(torch.nn.Module):
        def __init__(self, name):
            super().__init__()

        def get_sentence_embedding_dimension(self):
            return 384

    mod = types.ModuleType("sentence_transformers")
    mod.SentenceTransformer = _StubST
    sys.modules["sentence_transformers"] = mod


def metrics_fixtures():
    """src/evaluation/metrics.py: every metric function on seeded cases, and
    Evaluator.evaluate_retrieval / evaluate_diversity / evaluate_coverage driven by stub
    encoder / index objects that return the cases' retrieved lists."""
    _stub_sentence_transformers()
    if "faiss" not in sys.modules:  # imported by vector_db.py at module level; never called here
        sys.modules["faiss"] = types.ModuleType("faiss")
    from src.evaluation import metrics as M  # reference module

    pids, meta, cases = gi.eval_cases()
    per_case = []
    for _, hist, rel, ret in cases:
        h = [i["product_id"] for i in hist]
        row = {"mrr": M.compute_mrr(ret, rel)}
        for k in gi.EVAL_K:
            row[f"recall@{k}"] = M.compute_recall_at_k(ret, rel, k)
            row[f"precision@{k}"] = M.compute_precision_at_k(ret, rel, k)
            row[f"ndcg@{k}"] = M.compute_ndcg_at_k(ret, rel, k)
            row[f"hit@{k}"] = M.compute_hit_rate_at_k(ret, rel, k)
            row[f"cat@{k}"] = M.compute_category_overlap(ret[:k], h, meta)
            row[f"brand@{k}"] = M.compute_brand_overlap(ret[:k], h, meta)
            row[f"rel@{k}"] = M.compute_relevance_score(ret[:k], h, meta)
        for attr in ("category", "brand"):
            row[f"div_{attr}"] = M.compute_diversity(ret, meta, attr)
        per_case.append(row)

    index_of = {}

    class StubEncoder:  # encode_buyer -> a one-hot of the case index
        def encode_buyer(self, interactions):
            return np.array([float(index_of[id(interactions)])], np.float32)

    class StubDB:
        def retrieve(self, emb, k=10):
            ret = cases[int(emb[0])][3]
            return [(p, 1.0 - 0.01 * r) for r, p in enumerate(ret[:k])]

    test_pairs = []
    for c, (bid, hist, rel, _) in enumerate(cases):
        index_of[id(hist)] = c
        test_pairs.append((bid, hist, rel))
    ev = M.Evaluator(StubEncoder(), StubDB(), config_path=os.path.join(REF, "configs/config.yaml"))
    ev.set_product_metadata(meta)
    out = {"per_case": per_case,
           "retrieval": ev.evaluate_retrieval(test_pairs, gi.EVAL_K, verbose=False),
           "div_category": ev.evaluate_diversity(test_pairs, 20, "category"),
           "div_brand": ev.evaluate_diversity(test_pairs, 20, "brand"),
           "coverage": ev.evaluate_coverage(test_pairs, 20),
           "coverage@5": M.compute_coverage(set().union(*[set(c[3][:5]) for c in cases]),
                                            set(pids))}
    with open(os.path.join(HERE, "metrics.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["metrics"]:
        metrics_fixtures()
        sys.exit(0)
    buyer_fixtures()
    infonce_fixtures()
    event_weight_fixtures()
    item_head_fixtures()
    flatip_fixtures()
    metrics_fixtures()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
