"""BASELINE.json configs[0] as ONE workload through twotower, against the reference scripts' own
outputs (tests/golden/pipeline.{json,npz}, made by make_pipeline_golden.py running
scripts/generate_embeddings.py:17-64 -> scripts/build_index.py:16-63 -> scripts/evaluate.py:86-207
as written, with stand-in text embeddings and a stand-in exact IndexFlatIP).

The same sequence here: the reference's product metadata in its index order (H3: processor.py:272
dedup-sort -> product_ids.npy, consumed, not re-derived) and the same checkpoint (trainer format,
no vocab dicts: dummy vocabs rebuilt by set_product_metadata) -> EmbeddingEncoder.encode_items
(batch 64; the stand-in text embeddings feed the HIP projection head) -> save_item_embeddings ->
VectorDatabase.build_index / save_index / load_index (HIP index) -> Evaluator.evaluate_all at
k in {1, 5, 10} (batched HIP buyer encode + retrieve_batch).

Bars: item embeddings within 2e-6 of the reference's CPU float32 (a different GEMM summation
order); the side files of both scripts byte-identical; every retrieval / diversity / coverage
aggregate equal to the reference's (they are functions of the retrieved id lists, so equality
means every buyer's top-k list matched); embedding-quality statistics within 1e-6."""
import json
import os

import numpy as np
import pytest
import torch
import yaml

import inputs as gi

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(GOLD, "pipeline.json"), encoding="utf-8") as f:
        doc = json.load(f)
    return doc, np.load(os.path.join(GOLD, "pipeline.npz"))


class StubTextEncoder:
    """The generator's sentence_transformers stand-in, on the device."""

    def get_sentence_embedding_dimension(self):
        return 384

    def encode(self, texts, **kw):
        return torch.from_numpy(gi.stub_text_embedding(list(texts))).cuda()


def _encoder(tmp_path, doc):
    from twotower.encoder import EmbeddingEncoder

    cfg_path = tmp_path / "config.yaml"
    with open(cfg_path, "w") as f:
        yaml.safe_dump(doc["config"], f)
    w = gi.pipeline_weights(doc["n_brand"], doc["n_cat"])
    ck = {"epoch": 0, "model_state_dict": {k: torch.from_numpy(v) for k, v in w.items()},
          "best_val_loss": 0.0, "config": doc["config"]}
    path = tmp_path / "best_model.pt"
    torch.save(ck, path)
    enc = EmbeddingEncoder(str(path), config_path=str(cfg_path), text_encoder=StubTextEncoder())
    meta = {pid: m for pid, m in doc["metadata"]}
    enc.set_product_metadata(meta)
    return enc, meta, str(cfg_path)


def _raw(p):
    return np.frombuffer(open(p, "rb").read(), np.uint8)


def test_configs0_pipeline_matches_reference_scripts(tmp_path, fx):
    from twotower.evaluation import Evaluator
    from twotower.vector_db import VectorDatabase

    doc, z = fx
    enc, meta, cfg_path = _encoder(tmp_path, doc)
    ids = list(meta)
    # scripts/generate_embeddings.py:48-60
    emb = enc.encode_items(ids, batch_size=64)
    np.testing.assert_allclose(emb[z["emb_rows"]], z["emb"], rtol=0, atol=2e-6)
    assert abs(np.linalg.norm(emb.astype(np.float64), axis=1).sum() - float(z["emb_norm_sum"])) < 1e-3
    enc.save_item_embeddings(ids, emb, str(tmp_path / "emb"))
    assert np.array_equal(_raw(tmp_path / "emb" / "product_ids.npy"), z["emb_ids_npy"])
    assert np.array_equal(_raw(tmp_path / "emb" / "product_id_to_index.json"), z["emb_map_json"])
    # scripts/build_index.py:35-59
    e2 = np.load(tmp_path / "emb" / "product_embeddings.npy")
    ids2 = np.load(tmp_path / "emb" / "product_ids.npy", allow_pickle=False).tolist()
    db = VectorDatabase(embedding_dim=doc["config"]["model"]["embedding_dim"])
    db.build_index(e2, ids2)
    idx = tmp_path / "index"
    idx.mkdir()
    db.save_index(str(idx / "product_index.faiss"), str(idx / "product_ids.npy"),
                  str(idx / "product_id_to_index.json"))
    assert np.array_equal(_raw(idx / "product_ids.npy"), z["index_ids_npy"])
    assert np.array_equal(_raw(idx / "product_id_to_index.json"), z["index_map_json"])
    # scripts/evaluate.py:170-203 (test pairs: the reference's prepare_test_data output)
    db2 = VectorDatabase(embedding_dim=doc["config"]["model"]["embedding_dim"])
    db2.load_index(str(idx / "product_index.faiss"), str(idx / "product_ids.npy"),
                   str(idx / "product_id_to_index.json"))
    ev = Evaluator(enc, db2, config_path=cfg_path)
    ev.set_product_metadata(meta)
    pairs = [(b, inter, set(rel)) for b, inter, rel in doc["test_pairs"]]
    got = ev.evaluate_all(pairs, k_values=doc["k_values"], all_product_ids=ids)
    ref = doc["results"]
    assert got["retrieval"] == ref["retrieval"]
    assert got["diversity"] == ref["diversity"]
    assert got["coverage"] == ref["coverage"]
    for key, v in ref["embedding_quality"].items():
        assert abs(got["embedding_quality"][key] - v) < 1e-6, key


def test_configs0_encode_buyer_matches_reference(tmp_path, fx):
    """EmbeddingEncoder.encode_buyer (encoder.py:244-305) on the generator's adversarial
    interaction lists: the same texts / brands / categories reach the item tower and the same
    weights reach the buyer tower as in the reference run, and the buyer embedding (attention
    aggregation over the re-encoded history) agrees within 5e-6."""
    doc, z = fx
    enc, meta, _ = _encoder(tmp_path, doc)
    for c, ref in zip(doc["encode_buyer_cases"], z["encode_buyer_out"]):
        pids, weights = enc._history(c["interactions"])
        texts, brands, cats = enc._item_inputs(pids)
        assert texts == c["texts"] and weights == c["weights"]
        assert brands == c["brands"] and cats == c["categories"]
        np.testing.assert_allclose(enc.encode_buyer(c["interactions"]), ref, rtol=0, atol=5e-6)
