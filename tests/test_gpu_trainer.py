"""configs[4] trainer glue (twotower.trainer.Trainer, reference src/training/trainer.py) and
the bf16 training step at the configs[4] shape.

* _encode_buyer_sequences_batched vs the reference method itself (fixture
  tests/golden/trainer_seq.npz: slot -> text and padded weights for tuple formats, malformed
  and unknown entries, empty-history fallback, truncation to the last 100).
* TwoTowerTrainStep bf16 (bf16 MFMA GEMMs, f32 accumulate) vs the f32 step at B = 512,
  E = 768, S = 20, N = 4: loss within 1e-2 relative, every gradient tensor within 3e-2
  relative Frobenius error (bf16 unit roundoff 2^-9 on both GEMM operands, K <= 768).
* Trainer.train over reference-format batches: loss decreases, checkpoints in the
  reference layout, eval-mode validate() is deterministic."""
import numpy as np
import pytest
import torch

import inputs as gi

pytestmark = pytest.mark.gpu


def _model(E=384, aggregation="attention", seed=0):
    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower, random_bert_state_dict
    from twotower.two_tower import TwoTowerModel

    cfg = dict(vocab=1000, hidden=384, layers=2, heads=12, intermediate=1536, max_positions=512,
               type_vocab=2, ln_eps=1e-12)
    torch.manual_seed(seed)
    it = ItemTower(embedding_dim=E, use_categorical_features=True,
                   encoder_state_dict=random_bert_state_dict(cfg, seed), encoder_cfg=cfg)
    it.initialize_categorical_embeddings(["Damas", "Acme", "Lazurde"], ["rings", "oil"])
    return TwoTowerModel(it, BuyerTower(E, aggregation, 128))


def test_encode_buyer_sequences_matches_reference(golden):
    from twotower.config import DEFAULT_CONFIG
    from twotower.trainer import Trainer

    g = golden("trainer_seq.npz")
    meta, seqs, pos = gi.trainer_batch()
    texts = gi.trainer_texts()
    tid = {t: j for j, t in enumerate(texts)}
    model = _model()
    tr = Trainer(model, [], config_path=None)
    tr.set_product_metadata(meta)

    def encode_text(batch_texts):  # the fixture's stand-in encoder
        out = torch.zeros((len(batch_texts), 384), device="cuda")
        out[:, 0] = torch.tensor([tid[t] + 1 for t in batch_texts], dtype=torch.float32)
        return out

    model.item_tower.encode_text = encode_text
    assert DEFAULT_CONFIG["model"]["buyer_tower"]["max_interaction_history"] == 100
    emb, w = tr._encode_buyer_sequences_batched(seqs, torch.ones(len(seqs)), pos)
    assert emb.shape == (len(seqs), 100, 384) and emb.is_cuda
    assert np.array_equal(emb[:, :, 0].cpu().numpy().astype(np.int16), g["slot_text"])
    assert float(emb[:, :, 1:].abs().sum()) == 0.0
    assert np.array_equal(w.cpu().numpy(), g["weights"])
    tr.pad_to_batch_max = True  # same rows, padding trimmed to the longest history
    emb2, w2 = tr._encode_buyer_sequences_batched(seqs, torch.ones(len(seqs)), pos)
    S = emb2.shape[1]
    assert S == int((g["weights"] != 0).sum(1).max()) or S == 100
    assert torch.equal(emb2, emb[:, :S]) and torch.equal(w2, w[:, :S])


def _torch_grads(it, bt, items, w, pos, neg, pb, pc, nb, nc, tau, autocast):
    """The same step as torch modules on the GPU (f32, or under torch.autocast bf16): the
    yardstick for what bf16 GEMMs do to these gradients."""
    import copy

    import torch.nn.functional as F
    from oracle import losses_ref

    it, bt = copy.deepcopy(it).cuda(), copy.deepcopy(bt).cuda()
    B, N = neg.shape[:2]
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        def head(t, b, c):
            x = torch.cat([t, it.brand_embedding(b.long()), it.category_embedding(c.long())], 1)
            return F.normalize(it.projection(x).float(), p=2, dim=1)

        p = head(pos, pb, pc)
        n = head(neg.reshape(B * N, -1), nb.reshape(-1), nc.reshape(-1)).view(B, N, -1)
        a = bt.attention(items).squeeze(-1).float() * w
        zb = F.normalize((torch.softmax(a, 1).unsqueeze(-1) * items).sum(1), p=2, dim=1)
        loss = losses_ref.infonce(zb, p, n, tau)
    loss.backward()
    g = {"proj0.w": it.projection[0].weight, "proj0.b": it.projection[0].bias,
         "proj3.w": it.projection[3].weight, "proj3.b": it.projection[3].bias,
         "att0.w": bt.attention[0].weight, "att0.b": bt.attention[0].bias,
         "att2.w": bt.attention[2].weight, "att2.b": bt.attention[2].bias,
         "brand": it.brand_embedding.weight, "cat": it.category_embedding.weight}
    return loss.item(), {k: v.grad.detach().double() for k, v in g.items()}


def test_bf16_step_vs_f32_step_configs4_shape():
    """bf16 step (bf16 MFMA GEMMs, f32 accumulate) vs the f32 step at configs[4]'s shape.
    Tolerance: loss within 1e-2 relative; per gradient tensor, the relative Frobenius error
    of our bf16 step vs our f32 step at most max(2 x torch-autocast-bf16's error on the same
    step, 1e-2) -- bf16's 2^-9 unit roundoff, amplified in cancelling sums such as the bias
    gradients, bounds what any bf16 step can do here."""
    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower
    from twotower.train import TwoTowerTrainStep

    class Dim:
        def get_sentence_embedding_dimension(self):
            return 384

    B, N, S, E, tau = 512, 4, 20, 768, 0.07
    rng = np.random.default_rng(12)
    items = torch.from_numpy(rng.standard_normal((B, S, E)).astype(np.float32)).cuda()
    w = torch.from_numpy(rng.choice([0.0, 1.0, 5.0, 10.0], (B, S)).astype(np.float32)).cuda()
    w[:, 0] = 1.0
    pos = torch.from_numpy(rng.standard_normal((B, 384)).astype(np.float32)).cuda()
    neg = torch.from_numpy(rng.standard_normal((B, N, 384)).astype(np.float32)).cuda()
    ids = lambda *sh: torch.from_numpy(rng.integers(0, 4, sh).astype(np.int32)).cuda()  # noqa
    pb, pc, nb, nc = ids(B), ids(B), ids(B, N), ids(B, N)
    res = {}
    for prec in ("f32", "bf16"):
        torch.manual_seed(3)
        it = ItemTower(embedding_dim=E, use_categorical_features=True, text_encoder=Dim())
        it.initialize_categorical_embeddings(["a", "b", "c"], ["x", "y", "z"])
        it.eval()  # dropout off: the two precisions must see the same network
        bt = BuyerTower(E, "attention")
        if prec == "f32":
            t32 = _torch_grads(it, bt, items, w, pos, neg, pb, pc, nb, nc, tau, False)
            t16 = _torch_grads(it, bt, items, w, pos, neg, pb, pc, nb, nc, tau, True)
        step = TwoTowerTrainStep(it, bt, temperature=tau, prec=prec)
        loss, g = step.forward_backward(items, w, pos, neg, pb, pc, nb, nc)
        res[prec] = (loss.item(), {k: v.detach().double() for k, v in g.items()})
    l32, g32 = res["f32"]
    l16, g16 = res["bf16"]
    assert abs(l32 - t32[0]) <= 1e-5 * abs(l32)
    assert abs(l16 - l32) <= 1e-2 * abs(l32), (l16, l32)
    report = {}
    for k, v in g32.items():
        rel = (g16[k] - v).norm().item() / (v.norm().item() + 1e-30)
        vt = t32[1][k].reshape(v.shape)
        rel_t = (t16[1][k].reshape(v.shape) - vt).norm().item() / (vt.norm().item() + 1e-30)
        report[k] = (round(rel, 4), round(rel_t, 4))
        assert rel <= max(2 * rel_t, 1e-2), (k, rel, rel_t)
    print("bf16 rel grad error (ours, torch autocast):", report)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("aggregation", ["attention", "weighted_avg"])
def test_trainer_epochs_reference_batches(tmp_path, aggregation, graph):
    from twotower.config import DEFAULT_CONFIG
    from twotower.trainer import Trainer

    rng = np.random.default_rng(5)
    n_prod, B, N = 60, 16, 4
    meta = {f"p{i}": {"text": f"منتج {i} " + " ".join(f"w{int(x)}" for x in
                                                       rng.integers(0, 200, 6)),
                      "brand": ["Damas", "Acme", None][i % 3], "category": ["rings", "oil"][i % 2]}
            for i in range(n_prod)}

    def batch():
        pos = [f"p{int(x)}" for x in rng.integers(0, n_prod, B)]
        negs = [[f"p{int(x)}" for x in rng.integers(0, n_prod, N)] for _ in range(B)]
        seqs = [[(f"p{int(x)}", float(rng.choice([1, 5, 10]))) for x in
                 rng.integers(0, n_prod, rng.integers(0, 12))] for _ in range(B)]
        return {"buyer_ids": [f"b{j}" for j in range(B)], "positive_product_ids": pos,
                "negative_product_ids": negs, "buyer_sequences": seqs,
                "positive_product_texts": [meta[p]["text"] for p in pos],
                "negative_product_texts": [[meta[p]["text"] for p in r] for r in negs],
                "weights": torch.ones(B)}

    train = [batch() for _ in range(4)]
    val = [batch() for _ in range(2)]
    cfg = {k: (dict(v) if isinstance(v, dict) else v) for k, v in DEFAULT_CONFIG.items()}
    cfg["training"] = dict(DEFAULT_CONFIG["training"], checkpoint_dir=str(tmp_path),
                           num_epochs=4, save_every_n_epochs=2, learning_rate=3e-3)
    import yaml

    cp = tmp_path / "config.yaml"
    cp.write_text(yaml.safe_dump(cfg, allow_unicode=True))
    model = _model(aggregation=aggregation, seed=1)
    tr = Trainer(model, train, val, config_path=str(cp), pad_to_batch_max=True, graph=graph)
    tr.set_product_metadata(meta)
    v0 = tr.validate()
    assert v0 == tr.validate()  # eval mode: deterministic
    losses = [tr.train_epoch() for _ in range(3)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]
    if graph:  # one captured HIP graph per batch shape (histories padded to the batch max)
        assert 1 <= len(tr.step._graphs) <= len(train)
    tr.train()
    assert (tmp_path / "best_model.pt").exists()
    ck = torch.load(tmp_path / "checkpoint_epoch_4.pt", weights_only=True)
    assert set(ck) >= {"epoch", "model_state_dict", "optimizer_state_dict", "best_val_loss",
                       "config", "brand_vocab", "category_vocab"}
    assert ck["epoch"] == 3
    sd = model.state_dict()  # the fused step trained the module parameters in place
    assert torch.equal(ck["model_state_dict"]["item_tower.projection.0.weight"].cpu(),
                       sd["item_tower.projection.0.weight"].cpu())
    # optimizer_state_dict is torch.optim.Adam's (reference trainer.py:330): a torch Adam over
    # model.parameters() loads it and holds the fused step's moments
    osd = ck["optimizer_state_dict"]
    assert set(osd) == {"state", "param_groups"}
    assert {int(float(e["step"])) for e in osd["state"].values()} == {7 * 4}
    ref = {k: v.clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=3e-3)
    opt.load_state_dict(osd)
    params = list(model.parameters())
    w0 = model.item_tower.projection[0].weight
    i0 = next(i for i, p in enumerate(params) if p is w0)
    assert torch.equal(opt.state_dict()["state"][i0]["exp_avg"].cpu(), tr.step.m["proj0.w"].cpu())
    # resume: a fresh Trainer restores weights, Adam moments and step count
    model2 = _model(aggregation=aggregation, seed=9)
    tr2 = Trainer(model2, train, val, config_path=str(cp), pad_to_batch_max=True)
    tr2.load_checkpoint(tmp_path / "checkpoint_epoch_4.pt")
    assert tr2.step.t == 7 * 4 and tr2.current_epoch == 4
    for k in tr.step.m:
        assert torch.equal(tr2.step.m[k], tr.step.m[k]) and torch.equal(tr2.step.v[k], tr.step.v[k])
    assert all(torch.equal(v.cpu(), ref[k].cpu()) for k, v in model2.state_dict().items())
    # resume INTO train(): it continues at the checkpoint's next epoch -- the saved epochs are
    # not re-run and later checkpoints keep the epoch / Adam step numbering
    tr3 = Trainer(_model(aggregation=aggregation, seed=9), train, val, config_path=str(cp),
                  pad_to_batch_max=True)
    tr3.set_product_metadata(meta)
    tr3.load_checkpoint(tmp_path / "checkpoint_epoch_2.pt")
    t_ck = tr3.step.t
    assert tr3.start_epoch == 2 and t_ck == 3 * 4 + 2 * 4
    calls = []
    run_epoch = tr3.train_epoch
    tr3.train_epoch = lambda: (calls.append(tr3.current_epoch), run_epoch())[1]
    tr3.train()
    assert calls == [2, 3] and tr3.step.t == t_ck + 2 * len(train)
    ck4 = torch.load(tmp_path / "checkpoint_epoch_4.pt", weights_only=True)
    assert ck4["epoch"] == 3
    assert {int(float(e["step"])) for e in ck4["optimizer_state_dict"]["state"].values()} == {7 * 4}
    # a state dict indexed over a different parameter list (the reference's Adam state puts
    # the frozen SentenceTransformer parameters first) is refused, not silently ignored
    shifted = {"state": {int(i) + 200: e for i, e in osd["state"].items()},
               "param_groups": osd["param_groups"]}
    with pytest.raises(ValueError, match="different parameter"):
        tr2.step.load_optimizer_state_dict(model2, shifted)
    first = sorted(osd["state"])[0]
    wrong = {"state": {first: dict(osd["state"][first], exp_avg=torch.zeros(3),
                                   exp_avg_sq=torch.zeros(3))},
             "param_groups": osd["param_groups"]}
    with pytest.raises(ValueError, match="different parameter"):
        tr2.step.load_optimizer_state_dict(model2, wrong)
