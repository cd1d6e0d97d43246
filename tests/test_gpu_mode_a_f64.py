"""Mode A end to end against the float64 composition (north_star: cosine scores within 1e-5).

EmbeddingEncoder.encode_buyer as the reference writes it (src/inference/encoder.py:286-303):
each buyer's S history texts re-encoded by the item tower (MiniLM-shape BertModel + mean pool,
item_tower.py:100-124; projection head + F.normalize, :174-211), aggregated by the buyer tower
(buyer_tower.py:43-101), then VectorDatabase.retrieve_batch (vector_db.py:171-209:
q / (||q|| + 1e-8), IndexFlatIP top-k).  Here: the HIP encoder (f32 and the default x3), the
HIP head at ItemTower's own precision for that encoder, the HIP aggregation, the HIP exact
top-100 over a 50k x 384 catalog.  Against: the same arithmetic in float64 (oracle/bert_ref.py
pinned to BertModel in float64, tests/test_encoder_oracle.py; the float64 buyer restatements
in oracle/oracle.py) with the f32-normalised catalog rows widened to float64.

Bars: every rank's score within 1e-5 of the float64 list at that rank; the score the GPU
reports for a row within 1e-5 of that row's float64 score; ids equal at every rank whose
float64 neighbours are more than 2e-5 away (a pair closer than the combined score error may
legitimately swap); the float64 top-k set outside the boundary band contained in the GPU's."""
import os
import sys

import numpy as np
import pytest
import torch

import make_bert_golden as mbg

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

B, S, K, N_CAT = 12, 20, 100, 50_000
SCORE_TOL, GAP = 1e-5, 2e-5


def _inputs():
    rng = np.random.default_rng(42)
    seqs = []
    for _ in range(B * S):
        L = int(rng.integers(8, 65))
        seqs.append([0] + (3 + rng.zipf(1.2, L - 2) % (mbg.CFG["vocab"] - 3)).tolist() + [2])
    bid = rng.integers(0, 5, B * S).tolist()
    cid = rng.integers(0, 5, B * S).tolist()
    w = np.where(rng.random((B, S)) < 0.75, 1.0, np.where(rng.random((B, S)) < 0.7, 5.0, 10.0))
    cat = rng.standard_normal((N_CAT, 384)).astype(np.float32)
    return seqs, bid, cid, w.astype(np.float32), cat


@pytest.fixture(scope="module")
def case():
    from oracle import bert_ref
    from twotower.item_tower import ItemTower, random_bert_state_dict

    sd = random_bert_state_dict(mbg.CFG, 5)
    seqs, bid, cid, w, cat = _inputs()
    torch.manual_seed(1)
    it = ItemTower(use_categorical_features=True, encoder_state_dict=sd, encoder_cfg=mbg.CFG,
                   prec="f32")
    it.initialize_categorical_embeddings(["b1", "b2", "b3", "b4"], ["c1", "c2", "c3", "c4"])
    head = {k: v.detach().cpu() for k, v in it.state_dict().items()}
    cu = np.concatenate([[0], np.cumsum([len(s) for s in seqs])])
    with torch.no_grad():
        te64 = bert_ref.bert_mean_pool(sd, mbg.CFG, torch.tensor([t for s in seqs for t in s]),
                                       cu, dtype=torch.float64)
        items64 = bert_ref.item_head(te64, {k: v.double() for k, v in head.items()}, bid, cid)
    g = torch.Generator().manual_seed(3)
    att = {"W1": torch.randn((128, 384), generator=g) / 384 ** 0.5,
           "b1": 0.1 * torch.randn(128, generator=g),
           "W2": torch.randn((1, 128), generator=g) / 128 ** 0.5,
           "b2": 0.1 * torch.randn(1, generator=g)}
    return dict(sd=sd, seqs=seqs, bid=bid, cid=cid, w=w, cat=cat, head=head, att=att,
                items64=items64.numpy().reshape(B, S, 384))


def _hip_items(case, prec):
    from twotower.item_tower import BertEncoder, ItemTower, pack_sequences

    it = ItemTower(use_categorical_features=True, text_encoder=_Dim())
    it.initialize_categorical_embeddings(["b1", "b2", "b3", "b4"], ["c1", "c2", "c3", "c4"])
    it.load_state_dict(case["head"])
    it.cuda().eval()
    it.head_prec = "f32" if prec == "f32" else "x3"  # ItemTower's choice with that encoder
    enc = BertEncoder(case["sd"], mbg.CFG, prec=prec)
    ids, cu, mx = pack_sequences(case["seqs"], "cuda")
    with torch.no_grad():
        pooled = enc.encode_packed(ids, cu, mx)
        return it.head(pooled, case["bid"], case["cid"], use_cat=True)


class _Dim:
    def get_sentence_embedding_dimension(self):
        return 384


def _check(gs, gi, q64, cat64):
    full = q64 @ cat64.T
    problems = []
    for b in range(q64.shape[0]):
        order = np.lexsort((np.arange(full.shape[1]), -full[b]))
        rs = full[b, order[:K + 1]]
        if np.abs(gs[b] - rs[:K]).max() > SCORE_TOL:
            problems.append((b, "rank scores", float(np.abs(gs[b] - rs[:K]).max())))
        if np.abs(gs[b] - full[b, gi[b]]).max() > SCORE_TOL:
            problems.append((b, "id scores"))
        for r in range(K):
            hi = rs[r - 1] if r else np.inf
            if hi - rs[r] > GAP and rs[r] - rs[r + 1] > GAP and gi[b, r] != order[r]:
                problems.append((b, f"id@{r}"))
                break
        sure = set(order[:K][rs[:K] > rs[K - 1] + GAP].tolist())
        if not sure.issubset(set(gi[b].tolist())):
            problems.append((b, "set"))
    return problems


@pytest.mark.parametrize("aggregation", ["weighted_avg", "attention"])
@pytest.mark.parametrize("prec", ["f32", "x3"])
def test_mode_a_scores_vs_f64_composition(case, prec, aggregation):
    from oracle import oracle as O
    from twotower import kernels
    from twotower.vector_db import VectorDatabase

    items = _hip_items(case, prec)
    dev_items = float(np.abs(items.cpu().double().numpy().reshape(B, S, 384)
                             - case["items64"]).max())
    assert dev_items <= 2e-6, dev_items  # unit rows: the reference head fixture's bar
    w = torch.from_numpy(case["w"]).cuda()
    a = case["att"]
    if aggregation == "weighted_avg":
        q = kernels.weighted_avg_l2(items.view(B, S, 384), w)
        q64 = O.weighted_avg_l2_f64(case["items64"], case["w"])
    else:
        q = kernels.attn_agg_l2(items.view(B, S, 384), w, *(a[k].cuda() for k in
                                                            ("W1", "b1", "W2", "b2")))
        q64 = O.attn_agg_l2_f64(case["items64"], case["w"], *(a[k].numpy() for k in
                                                             ("W1", "b1", "W2", "b2")))
    q64 = q64 / (np.linalg.norm(q64, axis=1, keepdims=True) + 1e-8)  # vector_db.py:189-190
    db = VectorDatabase(384)
    db.build_index(case["cat"], [f"p{i}" for i in range(N_CAT)])
    s, i = db.search(q, k=K)  # device retrieve_batch: the normalisation + exact top-k on HIP
    cat64 = O.vector_db_normalize(case["cat"]).astype(np.float64)  # the index's own f32 rows
    assert np.array_equal(db.index.xb[:N_CAT, :384].cpu().numpy(), cat64.astype(np.float32))
    problems = _check(s.cpu().double().numpy(), i.cpu().numpy(), q64, cat64)
    assert not problems, problems[:5]
