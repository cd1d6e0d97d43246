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


def _reference_step(it, bt, items, w, pos, neg, pb, pc, nb, nc, tau, lr, keep=None):
    """keep (None: eval mode, dropout off): the [B + B*N, hidden] keep mask of the
    projection's nn.Dropout(0.1) in train mode, rows = positives then negatives."""
    from oracle import losses_ref

    it, bt = copy.deepcopy(it).cpu(), copy.deepcopy(bt).cpu()
    B, N = neg.shape[:2]

    def head(text, bid, cid, kp):
        x = text
        if it.use_categorical_features:
            x = torch.cat([text, it.brand_embedding(bid.long()), it.category_embedding(cid.long())], 1)
        if kp is None:
            return F.normalize(it.projection(x), p=2, dim=1)
        h = torch.relu(it.projection[0](x)) * kp.float() / (1.0 - it.projection[2].p)
        return F.normalize(it.projection[3](h), p=2, dim=1)

    it.eval()
    p = head(pos, pb, pc, keep[:B] if keep is not None else None)
    n = head(neg.reshape(B * N, -1), nb.reshape(-1), nc.reshape(-1),
             keep[B:] if keep is not None else None).view(B, N, -1)
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

    it.eval()  # dropout off here; train mode: test_train_step_dropout_fixed_mask
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


def test_train_step_dropout_fixed_mask():
    """Train mode (the reference Trainer calls model.train(), trainer.py:167): the
    projection's nn.Dropout(0.1) (item_tower.py:61) is applied with the step's keep mask and
    scaled 1/(1-p), in the forward and the backward -- checked with a fixed mask against
    torch autograd applying the same mask."""
    from twotower.train import TwoTowerTrainStep

    B, N, S, E, tau, lr = 8, 4, 5, 384, 0.07, 1e-3
    it, bt = _setup(E, True, seed=4)
    it.train()
    rng = np.random.default_rng(44)
    items = torch.from_numpy(rng.standard_normal((B, S, E)).astype(np.float32))
    w = torch.from_numpy(rng.integers(1, 11, (B, S)).astype(np.float32))
    pos = torch.from_numpy(rng.standard_normal((B, 384)).astype(np.float32) * 0.3)
    neg = torch.from_numpy(rng.standard_normal((B, N, 384)).astype(np.float32) * 0.3)
    z = lambda *sh: torch.zeros(sh, dtype=torch.int32)  # noqa: E731
    keep = torch.from_numpy((rng.random((B + B * N, 256)) >= 0.1).astype(np.uint8))
    ref_loss, ref_g, _ = _reference_step(it, bt, items, w, pos, neg, z(B), z(B), z(B, N),
                                         z(B, N), tau, lr, keep=keep)
    step = TwoTowerTrainStep(it, bt, temperature=tau, lr=lr, prec="f32")
    seen = []

    def fixed(shape, p, dev):
        assert tuple(shape) == tuple(keep.shape) and p == 0.1
        seen.append(1)
        return keep.to(dev)

    step.keep_fn = fixed
    cu = lambda t: t.cuda()  # noqa: E731
    loss, g = step.forward_backward(cu(items), cu(w), cu(pos), cu(neg), cu(z(B)), cu(z(B)),
                                    cu(z(B, N)), cu(z(B, N)))
    assert seen == [1]
    assert abs(loss.item() - ref_loss) < 1e-5 * max(1, abs(ref_loss))
    for k, v in ref_g.items():
        got = g[k].detach().cpu().reshape(v.shape)
        scale = v.abs().max().item() + 1e-12
        assert (got - v).abs().max().item() <= 1e-4 * scale + 1e-6, k
    # eval mode: no mask is drawn
    it.eval()
    step.forward_backward(cu(items), cu(w), cu(pos), cu(neg))
    assert seen == [1]


def test_item_head_autograd_dropout_train_mode():
    """ItemTower.head under autograd in train mode: the HIP ItemHeadFn with the keep mask the
    module drew == torch applying that mask; eval mode is deterministic (no dropout)."""
    import twotower.train as T

    it, _ = _setup(384, True, seed=6)
    it.cuda().train()
    rng = np.random.default_rng(7)
    text = torch.from_numpy(rng.standard_normal((10, 384)).astype(np.float32)).cuda()
    text.requires_grad_(True)
    masks = []
    orig = T.dropout_keep

    def rec(shape, p, dev):
        m = orig(shape, p, dev)
        masks.append(m)
        return m

    T.dropout_keep = rec
    try:
        y = it.head(text, [1] * 10, [2] * 10, use_cat=True)
    finally:
        T.dropout_keep = orig
    assert len(masks) == 1 and masks[0].shape == (10, 256)
    y.square().sum().backward()
    ref_it = copy.deepcopy(it).cpu()
    tx = text.detach().cpu().requires_grad_(True)
    x = torch.cat([tx, ref_it.brand_embedding(torch.ones(10, dtype=torch.long)),
                   ref_it.category_embedding(torch.full((10,), 2, dtype=torch.long))], 1)
    h = torch.relu(ref_it.projection[0](x)) * masks[0].cpu().float() / 0.9
    ry = F.normalize(ref_it.projection[3](h), p=2, dim=1)
    ry.square().sum().backward()
    torch.testing.assert_close(y.detach().cpu(), ry.detach(), rtol=0, atol=2e-6)
    torch.testing.assert_close(text.grad.cpu(), tx.grad, rtol=0, atol=1e-5)
    g0, r0 = it.projection[0].weight.grad.cpu(), ref_it.projection[0].weight.grad
    assert (g0 - r0).abs().max().item() <= 1e-4 * r0.abs().max().item() + 1e-6
    it.eval()
    with torch.no_grad():
        a, b = it.head(text, [1] * 10, [2] * 10, use_cat=True), it.head(text, [1] * 10, [2] * 10, use_cat=True)
    assert torch.equal(a, b)


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
