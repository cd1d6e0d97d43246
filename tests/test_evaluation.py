"""twotower.evaluation (batched Evaluator) vs the reference src/evaluation/metrics.py:
every metric function per case and the Evaluator aggregates, against tests/golden/metrics.json
(made by tests/golden/make_golden.py from the reference module)."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import inputs as gi  # noqa: E402


@pytest.fixture(scope="module")
def fixture():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "metrics.json")))


def test_metric_functions_match_reference(fixture):
    from twotower import evaluation as E

    _, meta, cases = gi.eval_cases()
    for (_, hist, rel, ret), want in zip(cases, fixture["per_case"]):
        h = [i["product_id"] for i in hist]
        got = {"mrr": E.compute_mrr(ret, rel)}
        for k in gi.EVAL_K:
            got[f"recall@{k}"] = E.compute_recall_at_k(ret, rel, k)
            got[f"precision@{k}"] = E.compute_precision_at_k(ret, rel, k)
            got[f"ndcg@{k}"] = E.compute_ndcg_at_k(ret, rel, k)
            got[f"hit@{k}"] = E.compute_hit_rate_at_k(ret, rel, k)
            got[f"cat@{k}"] = E.compute_category_overlap(ret[:k], h, meta)
            got[f"brand@{k}"] = E.compute_brand_overlap(ret[:k], h, meta)
            got[f"rel@{k}"] = E.compute_relevance_score(ret[:k], h, meta)
        for attr in ("category", "brand"):
            got[f"div_{attr}"] = E.compute_diversity(ret, meta, attr)
        assert got == want


class _Enc:
    """batched stub: one-hot of the case index (what the reference run's stub returned)."""

    def __init__(self, index_of):
        self.index_of, self.calls = index_of, 0

    def encode_buyers(self, histories, mode="A"):
        self.calls += 1
        for h in histories:
            if any(i["product_id"] == "boom" for i in h):
                raise RuntimeError("bad buyer")
        return np.array([[float(self.index_of[id(h)])] for h in histories], np.float32)


class _DB:
    def __init__(self, cases):
        self.cases, self.calls = cases, 0

    def retrieve_batch(self, embs, k=10):
        self.calls += 1
        return [[(p, 1.0 - 0.01 * r) for r, p in enumerate(self.cases[int(e[0])][3][:k])]
                for e in embs]


def test_evaluator_matches_reference_with_one_batched_pass(fixture):
    from twotower.evaluation import Evaluator

    pids, meta, cases = gi.eval_cases()
    index_of, pairs = {}, []
    for c, (bid, hist, rel, _) in enumerate(cases):
        index_of[id(hist)] = c
        pairs.append((bid, hist, rel))
    enc, db = _Enc(index_of), _DB(cases)
    ev = Evaluator(enc, db, config_path=None, batch_size=16)
    ev.set_product_metadata(meta)
    assert ev.evaluate_retrieval(pairs, gi.EVAL_K, verbose=False) == fixture["retrieval"]
    assert ev.evaluate_diversity(pairs, 20, "category") == fixture["div_category"]
    assert ev.evaluate_diversity(pairs, 20, "brand") == fixture["div_brand"]
    assert ev.evaluate_coverage(pairs, 20) == fixture["coverage"]
    # one batched pass (3 batches of <= 16 buyers) served all four evaluations
    assert enc.calls == 3 and db.calls == 3


def test_evaluator_skips_failing_buyers_like_reference():
    from twotower.evaluation import Evaluator

    _, meta, cases = gi.eval_cases()
    index_of, pairs = {}, []
    for c, (bid, hist, rel, _) in enumerate(cases[:10]):
        hist = list(hist) + ([{"product_id": "boom", "event_type": "view"}] if c == 4 else [])
        index_of[id(hist)] = c
        pairs.append((bid, hist, rel))
    ev = Evaluator(_Enc(index_of), _DB(cases), config_path=None)
    ev.set_product_metadata(meta)
    r = ev.evaluate_retrieval(pairs, [5], verbose=False)
    assert r["diagnostics"]["total_buyers_evaluated"] == 9
    with pytest.raises(ValueError, match="Product metadata must be set"):
        Evaluator(_Enc({}), _DB(cases), config_path=None).evaluate_retrieval(pairs)
