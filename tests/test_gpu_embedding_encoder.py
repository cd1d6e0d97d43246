"""EmbeddingEncoder (twotower.encoder, reference src/inference/encoder.py) end to end on the
GPU: a checkpoint in the reference trainer's format (trainer.py:327-340, sentence-transformers
text-encoder keys) -> encode_items / encode_buyer vs the float32 oracle composition
(bert_ref encoder -> item head -> oracle buyer aggregation); history rules; batched and
Mode B encodes; the dummy-vocab checkpoint path."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

pytestmark = pytest.mark.gpu

CFG = dict(vocab=1000, hidden=384, layers=2, heads=12, intermediate=1536, max_positions=512,
           type_vocab=2, ln_eps=1e-12)
BRANDS = ["Damas", "Acme", "Lazurde", "Zed"]
CATS = ["rings", "necklaces", "bracelets", "engine-oil"]


def _metadata(n=30, seed=0):
    rng = np.random.default_rng(seed)
    words = ["خاتم", "ذهب", "عيار", "21", "سلسال", "gold", "ring", "زيت", "محرك", "5W-30"]
    meta = {}
    for i in range(n):
        text = " ".join(rng.choice(words, rng.integers(0, 9)))
        meta[f"p{i}"] = {"text": text,
                         "brand": BRANDS[i % 5] if i % 5 < 4 else None,
                         "category": CATS[i % 4]}
    return meta


def _checkpoint(tmp_path, aggregation, with_vocab=True, seed=3):
    from twotower.buyer_tower import BuyerTower
    from twotower.config import DEFAULT_CONFIG
    from twotower.item_tower import ItemTower, random_bert_state_dict
    from twotower.two_tower import TwoTowerModel

    torch.manual_seed(seed)
    enc_sd = random_bert_state_dict(CFG, seed)
    it = ItemTower(use_categorical_features=True, encoder_state_dict=enc_sd, encoder_cfg=CFG,
                   prec="f32")
    it.initialize_categorical_embeddings(BRANDS, CATS)
    model = TwoTowerModel(it, BuyerTower(384, aggregation, 128))
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    sd.update({"item_tower.text_encoder.0.auto_model." + k: v for k, v in enc_sd.items()})
    cfg = {k: (dict(v) if isinstance(v, dict) else v) for k, v in DEFAULT_CONFIG.items()}
    cfg["model"] = {**DEFAULT_CONFIG["model"],
                    "buyer_tower": {**DEFAULT_CONFIG["model"]["buyer_tower"],
                                    "aggregation_method": aggregation}}
    ck = {"epoch": 0, "model_state_dict": sd, "best_val_loss": 1.0, "config": cfg}
    if with_vocab:
        ck["brand_vocab"], ck["category_vocab"] = it.brand_vocab, it.category_vocab
    path = tmp_path / "best_model.pt"
    torch.save(ck, path)
    return path, enc_sd, sd, it


def _oracle_items(enc, enc_sd, sd, pids, meta, dtype=torch.float32):
    from oracle import bert_ref

    it = enc.model.item_tower
    texts = [meta.get(p, {}).get("text", "") for p in pids]
    seqs = it.text_encoder.tokenizer([t if t and t.strip() else " " for t in texts])
    cu = np.concatenate([[0], np.cumsum([len(s) for s in seqs])])
    te = bert_ref.bert_mean_pool(enc_sd, CFG, torch.tensor([t for s in seqs for t in s]), cu,
                                 dtype=dtype)
    head = {k[len("item_tower."):]: v.to(dtype) for k, v in sd.items()
            if k.startswith("item_tower.") and "text_encoder" not in k}
    bid = [it.brand_vocab.get(meta[p].get("brand"), 0) if meta.get(p, {}).get("brand") else 0
           for p in pids]
    cid = [it.category_vocab.get(meta[p].get("category"), 0)
           if meta.get(p, {}).get("category") else 0 for p in pids]
    return bert_ref.item_head(te, head, bid, cid)


@pytest.mark.parametrize("prec", ["f32", "x3"])
@pytest.mark.parametrize("aggregation", ["weighted_avg", "attention"])
def test_encode_items_and_buyer_vs_oracle(tmp_path, oracle_mod, aggregation, prec):
    """encode_items / encode_buyer (f32 and the default x3 encoder) vs the float64 composition
    (bert_ref in float64 -> head in float64 -> float64 buyer aggregation): unit rows within 2e-6,
    the bar of the f32 head against the reference ItemTower fixture."""
    from oracle import oracle as O
    from twotower.encoder import EmbeddingEncoder

    path, enc_sd, sd, _ = _checkpoint(tmp_path, aggregation)
    enc = EmbeddingEncoder(str(path), config_path=None, prec=prec)
    meta = _metadata()
    with pytest.raises(ValueError, match="Product metadata must be set"):
        enc.encode_items(["p0"])
    enc.set_product_metadata(meta)
    pids = list(meta)
    y = enc.encode_items(pids, batch_size=7)
    ref = _oracle_items(enc, enc_sd, sd, pids, meta, torch.float64).numpy()
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)

    # encode_buyer: timestamps sort, event weights (aliases, unknown -> 1), unknown product
    inter = [{"product_id": "p3", "event_type": "purchase", "timestamp": "2024-01-03"},
             {"product_id": "p1", "event_type": "view", "timestamp": "2024-01-01"},
             {"product_id": "p7", "event_type": "AddToCart", "timestamp": "2024-01-02"},
             {"product_id": "nope", "event_type": "share", "timestamp": "2024-01-04"}]
    b = enc.encode_buyer(inter)
    order = ["p1", "p7", "p3", "nope"]
    w = np.array([[1, 5, 10, 1]], np.float32)
    items = _oracle_items(enc, enc_sd, sd, order, meta, torch.float64).numpy()[None]
    if aggregation == "weighted_avg":
        rb = O.weighted_avg_l2_f64(items, w)
    else:
        a = {k: v.numpy() for k, v in sd.items() if k.startswith("buyer_tower.attention")}
        rb = O.attn_agg_l2_f64(items, w, a["buyer_tower.attention.0.weight"],
                               a["buyer_tower.attention.0.bias"],
                               a["buyer_tower.attention.2.weight"],
                               a["buyer_tower.attention.2.bias"])
    assert b.shape == (384,)
    np.testing.assert_allclose(b, rb[0], rtol=0, atol=2e-6)


def test_history_truncation_and_missing_timestamp(tmp_path):
    from twotower.encoder import EmbeddingEncoder

    path, *_ = _checkpoint(tmp_path, "weighted_avg")
    enc = EmbeddingEncoder(str(path), config_path=None)
    enc.config["model"]["buyer_tower"]["max_interaction_history"] = 3
    enc.set_product_metadata(_metadata())
    inter = [{"product_id": f"p{i}", "event_type": "view", "timestamp": f"t{9 - i}"}
             for i in range(6)]
    # sorted by timestamp -> p5..p0, last 3 = p2, p1, p0
    pids, w = enc._history(inter)
    assert pids == ["p2", "p1", "p0"] and w == [1, 1, 1]
    inter[2]["timestamp"] = None  # one missing -> input order kept
    pids, _ = enc._history(inter)
    assert pids == ["p3", "p4", "p5"]


@pytest.mark.parametrize("aggregation", ["weighted_avg", "attention"])
def test_encode_buyers_batched_and_mode_b(tmp_path, aggregation):
    from twotower.encoder import EmbeddingEncoder

    path, *_ = _checkpoint(tmp_path, aggregation)
    enc = EmbeddingEncoder(str(path), config_path=None)
    meta = _metadata()
    enc.set_product_metadata(meta)
    rng = np.random.default_rng(1)
    ev = ["view", "add_to_cart", "purchase"]
    hists = [[{"product_id": f"p{rng.integers(0, 30)}", "event_type": ev[rng.integers(0, 3)]}
              for _ in range(rng.integers(1, 9))] for _ in range(6)]
    single = np.stack([enc.encode_buyer(h) for h in hists])
    tol = 0 if aggregation == "weighted_avg" else 1e-6
    np.testing.assert_allclose(enc.encode_buyers(hists, mode="A"), single, rtol=0, atol=tol)
    pids = list(meta)
    enc.set_item_embeddings(pids, enc.encode_items(pids))
    np.testing.assert_allclose(enc.encode_buyers(hists, mode="B"), single, rtol=0,
                               atol=max(tol, 1e-6))


def test_dummy_vocab_checkpoint_and_reconstruction(tmp_path):
    """A checkpoint without vocab dicts (reference :104-116) loads with dummy vocabs of the
    saved sizes; set_product_metadata rebuilds the mapping from metadata (:132-204)."""
    from twotower.encoder import EmbeddingEncoder

    path, _, sd, it = _checkpoint(tmp_path, "weighted_avg", with_vocab=False)
    enc = EmbeddingEncoder(str(path), config_path=None)
    t = enc.model.item_tower
    assert t.brand_embedding.num_embeddings == sd["item_tower.brand_embedding.weight"].shape[0]
    assert sorted(k for k in t.brand_vocab if k != "<UNK>")[0].startswith("brand_")
    enc.set_product_metadata(_metadata())
    assert t.brand_vocab == it.brand_vocab and t.category_vocab == it.category_vocab


def test_save_item_embeddings_layout(tmp_path):
    import json

    from twotower.encoder import EmbeddingEncoder

    path, *_ = _checkpoint(tmp_path, "weighted_avg")
    enc = EmbeddingEncoder(str(path), config_path=None)
    emb = np.arange(12, dtype=np.float32).reshape(3, 4)
    enc.save_item_embeddings(["a", "b", "c"], emb, str(tmp_path / "out"))
    assert np.array_equal(np.load(tmp_path / "out" / "product_embeddings.npy"), emb)
    assert list(np.load(tmp_path / "out" / "product_ids.npy")) == ["a", "b", "c"]
    assert json.load(open(tmp_path / "out" / "product_id_to_index.json")) == \
        {"a": 0, "b": 1, "c": 2}


def test_batched_evaluator_equals_reference_per_buyer_loop(tmp_path):
    """twotower.evaluation.Evaluator (one batched encode + retrieve_batch) == the reference's
    per-buyer loop (encode_buyer + retrieve, metrics.py:419-429) on the HIP towers + index."""
    from twotower import evaluation as E
    from twotower.encoder import EmbeddingEncoder
    from twotower.vector_db import VectorDatabase

    path, *_ = _checkpoint(tmp_path, "weighted_avg")
    enc = EmbeddingEncoder(str(path), config_path=None)
    meta = _metadata()
    enc.set_product_metadata(meta)
    pids = list(meta)
    db = VectorDatabase(384)
    db.build_index(enc.encode_items(pids), pids)
    rng = np.random.default_rng(4)
    ev_types = ["view", "add_to_cart", "purchase"]
    pairs = []
    for b in range(12):
        hist = [{"product_id": f"p{rng.integers(0, 30)}", "event_type": ev_types[rng.integers(0, 3)]}
                for _ in range(rng.integers(1, 6))]
        pairs.append((f"u{b}", hist, {f"p{j}" for j in rng.integers(0, 30, 3)}))
    ev = E.Evaluator(enc, db, config_path=None)
    ev.set_product_metadata(meta)
    got = ev.evaluate_retrieval(pairs, [1, 5, 10], verbose=False)
    # the reference loop, restated
    ref = {}
    for _, inter, rel in pairs:
        ret = [p for p, _ in db.retrieve(enc.encode_buyer(inter), k=10)]
        for k in [1, 5, 10]:
            ref.setdefault(f"recall@{k}", []).append(E.compute_recall_at_k(ret, rel, k))
            ref.setdefault(f"ndcg@{k}", []).append(E.compute_ndcg_at_k(ret, rel, k))
        ref.setdefault("mrr", []).append(E.compute_mrr(ret, rel))
    for key, vals in ref.items():
        assert got[f"{key}_mean"] == float(np.mean(vals)), key


@pytest.mark.parametrize("aggregation", ["weighted_avg", "attention"])
def test_mode_b_unknown_ids_match_encode_buyer(tmp_path, aggregation):
    """History ids missing from the resident table (and from the metadata) are encoded as
    encode_buyer encodes them (metadata {} -> text ' ', encoder.py:280-292): Mode B equals
    the per-buyer reference path instead of raising KeyError."""
    from twotower.encoder import EmbeddingEncoder

    path, *_ = _checkpoint(tmp_path, aggregation)
    enc = EmbeddingEncoder(str(path), config_path=None)
    meta = _metadata()
    enc.set_product_metadata(meta)
    pids = list(meta)[:20]  # p20..p29 known to the metadata but not in the table
    enc.set_item_embeddings(pids, enc.encode_items(pids))
    hists = [[{"product_id": "p3", "event_type": "view"},
              {"product_id": "p25", "event_type": "purchase"},
              {"product_id": "not-a-product", "event_type": "add_to_cart"}],
             [{"product_id": "p1", "event_type": "view"}],
             [{"product_id": "ghost", "event_type": "view"}]]
    single = np.stack([enc.encode_buyer(h) for h in hists])
    np.testing.assert_allclose(enc.encode_buyers(hists, mode="B"), single, rtol=0, atol=1e-6)
