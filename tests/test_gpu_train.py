"""configs[4] training step (twotower.train) vs torch autograd + torch.optim.Adam on CPU.

The reference step: item-tower head on positive/negative text embeddings, buyer-tower
attention aggregation, InfoNCE, backward, Adam (trainer.py:49-52,74-243).  Tolerances: f32
MFMA path differs from the CPU by summation order only (rtol 1e-4 on gradients, which span
several orders of magnitude; parameters after the Adam step 1e-6 absolute)."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import inputs as gi

pytestmark = pytest.mark.gpu


def _setup(E=384, use_cat=True, seed=0):
    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower

    class Dim:
        def get_sentence_embedding_dimension(self):
            return 384

    torch.manual_seed(seed)
    it = ItemTower(embedding_dim=E, use_categorical_features=use_cat, text_encoder=Dim())
    if use_cat:
        it.initialize_categorical_embeddings(gi.BRANDS, gi.CATEGORIES)
    bt = BuyerTower(E, "attention")
    return it, bt


def _reference_step(it, bt, items, w, pos, neg, pb, pc, nb, nc, tau, lr):
    from oracle import losses_ref

    it, bt = copy.deepcopy(it).cpu(), copy.deepcopy(bt).cpu()
    B, N = neg.shape[:2]

    def head(text, bid, cid):
        x = text
        if it.use_categorical_features:
            x = torch.cat([text, it.brand_embedding(bid.long()), it.category_embedding(cid.long())], 1)
        return F.normalize(it.projection(x), p=2, dim=1)

    it.eval()  # dropout off (the HIP step has no dropout either)
    p = head(pos, pb, pc)
    n = head(neg.reshape(B * N, -1), nb.reshape(-1), nc.reshape(-1)).view(B, N, -1)
    a = bt.attention(items).squeeze(-1) * w
    zb = F.normalize((torch.softmax(a, 1).unsqueeze(-1) * items).sum(1), p=2, dim=1)
    loss = losses_ref.infonce(zb, p, n, tau)
    params = list(it.projection.parameters()) + list(bt.attention.parameters())
    if it.use_categorical_features:
        params += [it.brand_embedding.weight, it.category_embedding.weight]
    opt = torch.optim.Adam(params, lr=lr)
    opt.zero_grad()
    loss.backward()
    grads = {"proj0.w": it.projection[0].weight.grad, "proj0.b": it.projection[0].bias.grad,
             "proj3.w": it.projection[3].weight.grad, "proj3.b": it.projection[3].bias.grad,
             "att0.w": bt.attention[0].weight.grad, "att0.b": bt.attention[0].bias.grad,
             "att2.w": bt.attention[2].weight.grad, "att2.b": bt.attention[2].bias.grad}
    if it.use_categorical_features:
        grads["brand"] = it.brand_embedding.weight.grad
        grads["cat"] = it.category_embedding.weight.grad
    grads = {k: v.clone() for k, v in grads.items()}
    opt.step()
    after = {"proj0.w": it.projection[0].weight, "att0.w": bt.attention[0].weight,
             "proj3.b": it.projection[3].bias, "att2.b": bt.attention[2].bias}
    if it.use_categorical_features:
        after["brand"] = it.brand_embedding.weight
    return loss.item(), grads, {k: v.detach().clone() for k, v in after.items()}


@pytest.mark.parametrize("E,use_cat", [(384, True), (768, True), (384, False)])
def test_train_step_matches_torch_autograd_and_adam(E, use_cat):
    from twotower.train import TwoTowerTrainStep

    B, N, S, tau, lr = 8, 4, 5, 0.07, 1e-3
    it, bt = _setup(E, use_cat)
    rng = np.random.default_rng(E)
    items = torch.from_numpy(rng.standard_normal((B, S, E)).astype(np.float32))
    w = torch.from_numpy(rng.integers(1, 11, (B, S)).astype(np.float32))
    w[0, 3:] = 0.0  # padded history positions
    pos = torch.from_numpy(rng.standard_normal((B, 384)).astype(np.float32) * 0.3)
    neg = torch.from_numpy(rng.standard_normal((B, N, 384)).astype(np.float32) * 0.3)
    pb = torch.from_numpy(rng.integers(0, 6, B).astype(np.int32))
    pc = torch.from_numpy(rng.integers(0, 5, B).astype(np.int32))
    nb = torch.from_numpy(rng.integers(0, 6, (B, N)).astype(np.int32))
    nc = torch.from_numpy(rng.integers(0, 5, (B, N)).astype(np.int32))
    ref_loss, ref_g, ref_after = _reference_step(it, bt, items, w, pos, neg, pb, pc, nb, nc, tau, lr)

    step = TwoTowerTrainStep(it, bt, temperature=tau, lr=lr, prec="f32")
    cu = lambda t: t.cuda()  # noqa: E731
    loss, g = step.forward_backward(cu(items), cu(w), cu(pos), cu(neg), cu(pb), cu(pc), cu(nb),
                                    cu(nc))
    assert abs(loss.item() - ref_loss) < 1e-5 * max(1, abs(ref_loss))
    for k, v in ref_g.items():
        got = g[k].detach().cpu().reshape(v.shape)
        scale = v.abs().max().item() + 1e-12
        assert (got - v).abs().max().item() <= 1e-4 * scale + 1e-6, k  # + cancellation in sums
    # Adam: the fused kernel == torch.optim.Adam applied to the same gradients (Adam's first
    # step is ~lr * sign(g), so comparing against the CPU gradients would only measure the
    # sign of near-zero gradient entries)
    before = {k: v.detach().cpu().clone() for k, v in step.params.items()}
    step.adam(g)
    for k, p0 in before.items():
        ref_p = torch.nn.Parameter(p0.clone())
        ref_p.grad = g[k].detach().cpu().reshape(p0.shape).clone()
        torch.optim.Adam([ref_p], lr=lr).step()
        torch.testing.assert_close(step.params[k].cpu(), ref_p.detach(), rtol=0, atol=2e-7)
    # and the parameters end up where the reference step put them, except where Adam's
    # first step amplifies sub-ulp gradient differences of near-zero entries
    names = {"proj0.w": it.projection[0].weight, "att0.w": bt.attention[0].weight,
             "proj3.b": it.projection[3].bias, "att2.b": bt.attention[2].bias}
    if use_cat:
        names["brand"] = it.brand_embedding.weight
    for k, ref in ref_after.items():
        diff = (names[k].detach().cpu() - ref).abs()
        assert (diff > 1e-6).float().mean().item() < 1e-3, k


def test_train_step_bf16_loss_decreases():
    from twotower.train import TwoTowerTrainStep

    B, N, S, E = 64, 4, 20, 768
    it, bt = _setup(E, True, seed=3)
    rng = np.random.default_rng(1)
    items = torch.from_numpy(rng.standard_normal((B, S, E)).astype(np.float32)).cuda()
    w = torch.from_numpy(rng.integers(1, 11, (B, S)).astype(np.float32)).cuda()
    pos = torch.from_numpy(rng.standard_normal((B, 384)).astype(np.float32)).cuda()
    neg = torch.from_numpy(rng.standard_normal((B, N, 384)).astype(np.float32)).cuda()
    step = TwoTowerTrainStep(it, bt, lr=1e-3, prec="bf16")
    losses = [step.step(items, w, pos, neg).item() for _ in range(20)]
    assert losses[-1] < losses[0] and all(np.isfinite(losses))


def test_modules_train_under_torch_autograd():
    """The mirrored modules are drop-ins for the reference's own training loop:
    forward_simplified -> InfoNCELoss -> loss.backward() -> torch.optim.Adam, gradients by the
    HIP backward kernels (autograd_ops), equal to the CPU reference's."""
    from twotower.losses import InfoNCELoss
    from twotower.two_tower import TwoTowerModel

    B, N, S, E, tau = 6, 4, 5, 384, 0.07
    it, bt = _setup(E, True, seed=5)
    emb = torch.from_numpy(np.random.default_rng(2).standard_normal((16, 384)).astype(np.float32))

    class Stub:
        def get_sentence_embedding_dimension(self):
            return 384

        def encode(self, texts, **kw):
            return emb[[int(t.split("#")[1]) for t in texts]]

    rng = np.random.default_rng(6)
    items = torch.from_numpy(rng.standard_normal((B, S, E)).astype(np.float32))
    w = torch.from_numpy(rng.integers(1, 11, (B, S)).astype(np.float32))
    pos_i = rng.integers(0, 16, B)
    neg_i = rng.integers(0, 16, (B, N))
    pb = [gi.BRANDS[i % 5] if i % 3 else None for i in range(B)]
    nb = [[gi.BRANDS[(i + j) % 5] for j in range(N)] for i in range(B)]
    ids = lambda names: torch.tensor([it.brand_vocab.get(x, 0) if x else 0 for x in names],  # noqa
                                     dtype=torch.int32)
    ref_loss, ref_g, _ = _reference_step(
        it, bt, items, w, emb[pos_i], emb[neg_i], ids(pb), torch.zeros(B, dtype=torch.int32),
        ids([x for l in nb for x in l]).view(B, N), torch.zeros((B, N), dtype=torch.int32),
        tau, 1e-3)
    it.text_encoder = Stub()
    model = TwoTowerModel(it, bt).cuda()
    model.item_tower.eval()
    out = model.forward_simplified(items.cuda(), w.cuda(), [f"p#{i}" for i in pos_i],
                                   [[f"p#{j}" for j in row] for row in neg_i], pb, None, nb, None)
    loss = InfoNCELoss(tau)(out["buyer_embeddings"], out["positive_embeddings"],
                            out["negative_embeddings"])
    loss.backward()
    assert abs(loss.item() - ref_loss) < 1e-5 * max(1, abs(ref_loss))
    got = {"proj0.w": it.projection[0].weight.grad, "proj3.b": it.projection[3].bias.grad,
           "att0.w": bt.attention[0].weight.grad, "att2.b": bt.attention[2].bias.grad,
           "brand": it.brand_embedding.weight.grad, "cat": it.category_embedding.weight.grad}
    for k, g in got.items():
        v = ref_g[k]
        scale = v.abs().max().item() + 1e-12
        assert (g.cpu().reshape(v.shape) - v).abs().max().item() <= 1e-4 * scale + 1e-6, k
    torch.optim.Adam(model.parameters(), lr=1e-3).step()  # torch's own optimizer on top
