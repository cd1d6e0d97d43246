"""Item-tower oracle checks (CPU): the float32 restatement in oracle/bert_ref.py against
transformers.BertModel outputs (tests/golden/bert.npz) and the reference ItemTower head
(tests/golden/item_head.npz, made by importing src/models/item_tower.py)."""
import hashlib

import numpy as np
import pytest
import torch

import make_bert_golden as mbg
import inputs as gi


def _sd():
    from twotower.item_tower import random_bert_state_dict

    return random_bert_state_dict(mbg.CFG, mbg.SEED)


def test_bert_weights_regenerate_identically(golden):
    g = golden("bert.npz")
    assert mbg.weights_sha(_sd()) == bytes(g["weights_sha256"]).decode()


def test_bert_oracle_vs_transformers_fixture(golden):
    from oracle import bert_ref

    g = golden("bert.npz")
    with torch.no_grad():
        y = bert_ref.bert_mean_pool(_sd(), mbg.CFG, torch.from_numpy(g["ids"]), g["cu_seqlens"])
    np.testing.assert_allclose(y.numpy(), g["pooled"], rtol=0, atol=2e-5)


def test_bert_oracle_f64_vs_transformers_f64_fixture(golden):
    """The float64 restatement (the envelope the GPU encoder tests measure against) equals
    transformers.BertModel run in float64 on the same weights; and the reference's own f32
    arithmetic sits within the stored f32_vs_f64_max of it."""
    from oracle import bert_ref

    g = golden("bert.npz")
    with torch.no_grad():
        y = bert_ref.bert_mean_pool(_sd(), mbg.CFG, torch.from_numpy(g["ids"]), g["cu_seqlens"],
                                    dtype=torch.float64)
    np.testing.assert_allclose(y.numpy(), g["pooled64"], rtol=0, atol=1e-11)
    dev = np.abs(g["pooled"].astype(np.float64) - g["pooled64"]).max()
    assert dev == pytest.approx(float(g["f32_vs_f64_max"]), rel=1e-12) and 1e-7 < dev < 1e-5


def test_bert_oracle_vs_transformers_live():
    transformers = pytest.importorskip("transformers")
    from oracle import bert_ref
    from twotower.item_tower import random_bert_state_dict

    cfg = dict(mbg.CFG, layers=2, vocab=300)
    sd = random_bert_state_dict(cfg, 3, std=0.05)
    bc = transformers.BertConfig(vocab_size=300, hidden_size=384, num_hidden_layers=2,
                                 num_attention_heads=12, intermediate_size=1536, hidden_act="gelu",
                                 layer_norm_eps=1e-12, type_vocab_size=2,
                                 max_position_embeddings=512)
    m = transformers.BertModel(bc, add_pooling_layer=False).eval()
    m.load_state_dict(sd, strict=False)
    lens = [5, 31, 1, 12]
    rng = np.random.default_rng(0)
    seqs = [rng.integers(0, 300, L).tolist() for L in lens]
    ids = torch.zeros((4, 31), dtype=torch.long)
    mask = torch.zeros((4, 31), dtype=torch.long)
    for i, s in enumerate(seqs):
        ids[i, :len(s)], mask[i, :len(s)] = torch.tensor(s), 1
    with torch.no_grad():
        h = m(input_ids=ids, attention_mask=mask).last_hidden_state
        mm = mask.unsqueeze(-1).float()
        ref = (h * mm).sum(1) / mm.sum(1)
        cu = np.concatenate([[0], np.cumsum(lens)])
        y = bert_ref.bert_mean_pool(sd, cfg, torch.tensor([t for s in seqs for t in s]), cu)
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=0, atol=2e-5)


@pytest.mark.parametrize("use_cat", [False, True])
def test_item_head_oracle_vs_reference_fixture(golden, use_cat):
    from oracle import bert_ref

    g = golden("item_head.npz")
    tag = "cat" if use_cat else "nocat"
    sd = {k: torch.from_numpy(v) for k, v in gi.item_head_weights(use_cat).items()}
    texts, brands, cats = gi.item_batch()
    emb = torch.from_numpy(gi.item_text_embeddings()[[int(t.split("#")[1]) for t in texts]])
    if use_cat:
        bv = {b: i for i, b in enumerate(g["cat__brand_vocab"].tolist())}
        cv = {c: i for i, c in enumerate(g["cat__category_vocab"].tolist())}
        bid = [bv.get(b, 0) if b else 0 for b in brands]
        cid = [cv.get(c, 0) if c else 0 for c in cats]
        y = bert_ref.item_head(emb, sd, bid, cid)
    else:
        y = bert_ref.item_head(emb, sd)
    np.testing.assert_allclose(y.numpy(), g[f"{tag}__out"], rtol=0, atol=1e-6)


def test_item_tower_mirror_state_dict_and_vocab(golden):
    """Same parameter names and categorical vocab order as the reference module."""
    from twotower.item_tower import ItemTower

    class Stub:
        def get_sentence_embedding_dimension(self):
            return 384

    g = golden("item_head.npz")
    for use_cat in (False, True):
        it = ItemTower(use_categorical_features=use_cat, text_encoder=Stub())
        tag = "cat" if use_cat else "nocat"
        if use_cat:
            it.initialize_categorical_embeddings(gi.BRANDS, gi.CATEGORIES)
            assert sorted(it.brand_vocab, key=it.brand_vocab.get) == g["cat__brand_vocab"].tolist()
            assert (sorted(it.category_vocab, key=it.category_vocab.get)
                    == g["cat__category_vocab"].tolist())
        assert sorted(it.state_dict()) == g[f"{tag}__keys"].tolist()


def test_hash_tokenizer_deterministic():
    from twotower.item_tower import HashTokenizer

    tok = HashTokenizer(vocab=1000, max_length=8)
    a = tok(["hello world", " ", "a b c d e f g h i j"])
    assert a == tok(["hello world", " ", "a b c d e f g h i j"])
    assert a[0][0] == 0 and a[0][-1] == 2 and len(a[2]) == 8 and a[1] == [0, 2]
    assert all(3 <= t < 1000 for s in a for t in s[1:-1])


@pytest.mark.parametrize("case", list(gi.INFONCE_CASES))
def test_infonce_oracle_vs_reference_fixture(golden, case):
    from oracle import losses_ref

    g = golden("infonce.npz")
    spec = gi.INFONCE_CASES[case]
    b, p, n = (torch.from_numpy(a).requires_grad_(True) for a in gi.infonce_inputs(spec))
    loss = losses_ref.infonce(b, p, n, spec["tau"])
    loss.backward()
    assert abs(loss.item() - g[case + "__loss"][0]) < 1e-6
    if case + "__gb" in g:
        for t, k in ((b, "gb"), (p, "gp"), (n, "gn")):
            np.testing.assert_allclose(t.grad.numpy(), g[f"{case}__{k}"], rtol=0, atol=1e-7)
    else:
        gn = [t.grad.norm().item() for t in (b, p, n)]
        np.testing.assert_allclose(gn, g[case + "__gnorm"], rtol=1e-5)


def test_encoder_cfg_from_checkpoint_weights():
    """EmbeddingEncoder infers the BertModel shape from the checkpoint's text-encoder weights
    (sentence-transformers keys, reference item_tower.py:29 model; 32-wide heads)."""
    from twotower.encoder import encoder_cfg_from_state_dict
    from twotower.item_tower import random_bert_state_dict

    cfg = dict(vocab=777, hidden=384, layers=3, heads=12, intermediate=1536, max_positions=512,
               type_vocab=2, ln_eps=1e-12)
    assert encoder_cfg_from_state_dict(random_bert_state_dict(cfg, 0)) == cfg
