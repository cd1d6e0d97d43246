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


@pytest.mark.parametrize("M,N,K", [(2560, 768, 256), (2560, 256, 512), (10240, 128, 768),
                                   (512, 512, 768), (37, 70, 33), (64, 64, 64), (1000, 5, 300),
                                   (0, 16, 16)])
@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("with_db", [True, False])
def test_gemm_tn_vs_float64(M, N, K, prec, with_db):
    """tt_gemm_tn (the weight-gradient GEMM C = A^T B without transposed copies, bias column
    sums fused): vs float64 of the same (bf16-rounded for prec bf16) operands.  f32 MFMA: only
    the summation order differs (relative 1e-5 of the |A|^T |B| scale); bf16: operands rounded
    RNE, f32 accumulation.  Deterministic: two calls give the same bits."""
    import ctypes

    from twotower import _lib

    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
    A = torch.randn((M, N), generator=g, device="cuda")
    Bm = torch.randn((M, K), generator=g, device="cuda")
    C = torch.full((N, K), float("nan"), device="cuda")
    db = torch.full((N,), float("nan"), device="cuda") if with_db else None
    need = ctypes.c_int64(0)
    _lib.check(L.tt_gemm_tn_workspace_bytes(M, N, K, ctypes.byref(need)), "ws")
    ws = torch.zeros(max(need.value, 256), dtype=torch.uint8, device="cuda")
    pr = _lib.TT_PREC_BF16 if prec == "bf16" else _lib.TT_PREC_F32

    def run():
        _lib.check(L.tt_gemm_tn(A.data_ptr(), N, Bm.data_ptr(), K, M, N, K, pr, C.data_ptr(), K,
                                db.data_ptr() if with_db else None, ws.data_ptr(), ws.numel(),
                                _lib.stream_ptr()), "tt_gemm_tn")
        return C.clone(), (db.clone() if with_db else None)

    c1, d1 = run()
    c2, d2 = run()  # deterministic: the same bits again
    assert torch.equal(c1, c2) and (not with_db or torch.equal(d1, d2))
    a64, b64 = A.double(), Bm.double()
    if prec == "bf16":
        a64, b64 = A.bfloat16().double(), Bm.bfloat16().double()
    ref = (a64.T @ b64) if M else torch.zeros((N, K), dtype=torch.float64, device="cuda")
    scale = (a64.abs().T @ b64.abs()) if M else torch.ones((N, K), dtype=torch.float64,
                                                           device="cuda")
    err = ((c1.double() - ref).abs() / (scale + 1e-30)).max().item()
    assert err <= 1e-5, err
    if with_db:
        rdb = A.double().sum(0) if M else torch.zeros(N, dtype=torch.float64, device="cuda")
        dscale = A.double().abs().sum(0) + 1e-30 if M else torch.ones(N, dtype=torch.float64,
                                                                       device="cuda")
        assert ((d1.double() - rdb).abs() / dscale).max().item() <= 1e-5


@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("use_cat", [True, False])
def test_graph_step_matches_eager_step(prec, use_cat):
    """TwoTowerTrainStep(graph=True) (forward + backward captured once per step shape in a HIP
    graph, then replayed) trains like the eager launch sequence: same losses and parameters over
    6 Adam steps within float-reordering noise (the embedding / attention-bias gradient sums use
    atomics), and inputs written in place through input_buffers give the same step."""
    from twotower.train import TwoTowerTrainStep

    B, N, S, E = 128, 4, 20, 768
    it0, bt0 = _setup(E, use_cat, seed=9)
    rng = np.random.default_rng(9)
    cu = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    items = cu(rng.standard_normal((B, S, E)).astype(np.float32))
    w = cu(rng.integers(1, 11, (B, S)).astype(np.float32))
    pos = cu(rng.standard_normal((B, 384)).astype(np.float32))
    neg = cu(rng.standard_normal((B, N, 384)).astype(np.float32))
    nv = (len(gi.BRANDS) + 1, len(gi.CATEGORIES) + 1)  # vocab sizes incl. <UNK> = 0
    ids = [cu(rng.integers(0, nv[j % 2], s).astype(np.int32))
           for j, s in enumerate(((B,), (B,), (B, N), (B, N)))]  # brand, cat, brand, cat
    batch = (items, w, pos, neg, *ids) if use_cat else (items, w, pos, neg)
    res = {}
    for mode in ("eager", "graph"):
        it, bt = copy.deepcopy(it0).cuda().eval(), copy.deepcopy(bt0).cuda()
        st = TwoTowerTrainStep(it, bt, lr=1e-3, prec=prec, graph=mode == "graph")
        l0, g0 = st.forward_backward(*batch)  # graph: warm-up, capture, replay
        g0 = {k: v.clone() for k, v in g0.items()}
        losses = [float(l0)] + [float(st.step(*batch)) for _ in range(6)]
        res[mode] = (losses, g0, st)
    (le, ge, _), (lg, gg, st) = res["eager"], res["graph"]
    assert len(st._graphs) == 1
    # the first forward + backward: same gradients up to float reordering (embedding-row and
    # attention-bias gradient sums use atomics); then the loss trajectory over 6 Adam steps
    # (parameters are not compared: Adam's first step is lr x sign(g), which an ulp of
    # reordering flips for near-zero gradient elements)
    for k in ge:
        d = (gg[k] - ge[k]).abs().max().item()
        assert d <= 1e-5 * max(ge[k].abs().max().item(), 1e-12), (k, d)
    np.testing.assert_allclose(lg, le, rtol=1e-4, atol=0)
    # inputs written in place: the same next step as the copying call
    if use_cat:
        bi = st.input_buffers(B, S, N)
        bi[0].copy_(items)
        bi[1].copy_(w)
        bi[2][:B].copy_(pos)
        bi[2][B:].copy_(neg.reshape(B * N, -1))
        bi[3][:B].copy_(ids[0])
        bi[3][B:].copy_(ids[2].reshape(-1))
        bi[4][:B].copy_(ids[1])
        bi[4][B:].copy_(ids[3].reshape(-1))
        l1, g1 = st.forward_backward(*batch)
        l1, g1 = float(l1), {k: v.clone() for k, v in g1.items()}
        l2, g2 = st.forward_backward(bi[0], bi[1], bi[2][:B], bi[2][B:].view(B, N, -1),
                                     bi[3][:B], bi[4][:B], bi[3][B:].view(B, N),
                                     bi[4][B:].view(B, N))
        assert abs(float(l2) - l1) <= 1e-6 * abs(l1)
        for k in g1:
            assert torch.allclose(g2[k], g1[k], rtol=1e-5, atol=1e-7), k


def test_gemm_tn_one_workspace_many_shapes():
    """One workspace serves tt_gemm_tn calls of different shapes in stream order (the training
    step's dW3 / dW0 / dWa0): each result is complete."""
    import ctypes

    from twotower import _lib

    L = _lib.lib()
    shapes = [(2560, 768, 256), (2560, 256, 512), (10240, 128, 768), (2560, 768, 256),
              (300, 40, 700)]
    need = 0
    for M, N, K in shapes:
        v = ctypes.c_int64(0)
        _lib.check(L.tt_gemm_tn_workspace_bytes(M, N, K, ctypes.byref(v)), "ws")
        need = max(need, v.value)
    ws = torch.empty(need, dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    outs = []
    for M, N, K in shapes:
        A = torch.randn((M, N), generator=g, device="cuda")
        Bm = torch.randn((M, K), generator=g, device="cuda")
        C = torch.full((N, K), float("nan"), device="cuda")
        db = torch.full((N,), float("nan"), device="cuda")
        _lib.check(L.tt_gemm_tn(A.data_ptr(), N, Bm.data_ptr(), K, M, N, K, _lib.TT_PREC_F32,
                                C.data_ptr(), K, db.data_ptr(), ws.data_ptr(), ws.numel(),
                                _lib.stream_ptr()), "tt_gemm_tn")
        outs.append((A, Bm, C, db))
    for A, Bm, C, db in outs:
        ref = A.double().T @ Bm.double()
        scale = A.double().abs().T @ Bm.double().abs()
        assert ((C.double() - ref).abs() / scale).max().item() <= 1e-5
        assert ((db.double() - A.double().sum(0)).abs()
                / A.double().abs().sum(0)).max().item() <= 1e-5
