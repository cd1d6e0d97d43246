"""InfoNCE forward + backward on the GPU (csrc/tt_loss.hip) vs the reference's own outputs
(tests/golden/infonce.npz) and the float64 restatement (oracle/losses_ref.py)."""
import numpy as np
import pytest
import torch

import inputs as gi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", list(gi.INFONCE_CASES))
def test_infonce_f32_vs_reference_fixture(golden, case):
    from twotower.losses import InfoNCELoss

    g = golden("infonce.npz")
    spec = gi.INFONCE_CASES[case]
    b, p, n = (torch.from_numpy(a).cuda().requires_grad_(True) for a in gi.infonce_inputs(spec))
    loss = InfoNCELoss(spec["tau"])(b, p, n)
    loss.backward()
    assert abs(loss.item() - g[case + "__loss"][0]) < 2e-6 * max(1.0, abs(g[case + "__loss"][0]))
    if case + "__gb" in g:
        for t, k in ((b, "gb"), (p, "gp"), (n, "gn")):
            np.testing.assert_allclose(t.grad.cpu().numpy(), g[f"{case}__{k}"], rtol=0, atol=2e-7)
    else:
        gn = [t.grad.norm().item() for t in (b, p, n)]
        np.testing.assert_allclose(gn, g[case + "__gnorm"], rtol=1e-5)


@pytest.mark.parametrize("B,N,E,tau", [(1, 4, 384, 0.07), (37, 0, 64, 0.2), (512, 4, 768, 0.07),
                                       (130, 7, 384, 1.0)])
@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_infonce_vs_f64(B, N, E, tau, prec):
    from oracle import losses_ref
    from twotower.losses import infonce

    if prec == "bf16" and E % 64:
        pytest.skip("bf16 GEMM needs E % 64 == 0")
    gen = torch.Generator().manual_seed(B + N + E)
    b, p, n = (torch.nn.functional.normalize(torch.randn(s, generator=gen), dim=-1)
               for s in ((B, E), (B, E), (B, N, E)))
    bd, pd, nd = (t.double().requires_grad_(True) for t in (b, p, n))
    ref = losses_ref.infonce(bd, pd, nd, tau)
    ref.backward()
    loss, (gb, gp, gn) = infonce(b.cuda(), p.cuda(), n.cuda(), tau, prec)
    tol = 1e-5 if prec == "f32" else 2e-2
    assert abs(loss.item() - ref.item()) <= tol * max(1.0, abs(ref.item()))
    for got, want in ((gb, bd.grad), (gp, pd.grad), (gn, nd.grad)):
        if want.numel() == 0:
            continue
        scale = want.abs().max().item() + 1e-30
        assert (got.cpu().double() - want).abs().max().item() <= tol * scale


def test_infonce_no_grad_path_and_errors():
    from twotower.losses import infonce

    b = torch.randn(8, 96, device="cuda")
    loss, g = infonce(b, b, b.view(8, 1, 96), 0.07, grads=False)
    assert g is None and torch.isfinite(loss)
    with pytest.raises(RuntimeError):
        infonce(b[:, :40].contiguous(), b[:, :40].contiguous(), b[:, :40].contiguous().view(8, 1, 40))


def test_two_tower_forward_simplified_and_loss():
    """TwoTowerModel.forward_simplified (two_tower.py:155-218) + InfoNCE on the device ==
    oracle item head / buyer attention / loss."""
    from oracle import bert_ref, losses_ref
    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower
    from twotower.losses import InfoNCELoss
    from twotower.two_tower import TwoTowerModel

    emb = gi.item_text_embeddings()

    class Stub:
        def get_sentence_embedding_dimension(self):
            return 384

        def encode(self, texts, **kw):
            return torch.from_numpy(emb[[int(t.split("#")[1]) for t in texts]])

    torch.manual_seed(0)
    it = ItemTower(text_encoder=Stub())
    it.initialize_categorical_embeddings(gi.BRANDS, gi.CATEGORIES)
    bt = BuyerTower(384, "attention")
    m = TwoTowerModel(it, bt).eval()
    B, N, S = 3, 4, 5
    rng = np.random.default_rng(4)
    items = torch.from_numpy(rng.standard_normal((B, S, 384)).astype(np.float32))
    w = torch.from_numpy(rng.integers(1, 11, (B, S)).astype(np.float32))
    pos = [f"p#{i}" for i in range(B)]
    neg = [[f"p#{(i + j + 3) % 16}" for j in range(N)] for i in range(B)]
    pb = ["Acme", None, "Damas"]
    nb = [["Tiffany", None, "x", "Acme"]] * B
    with torch.no_grad():  # attention-aggregation backward is not implemented (forward only)
        out = m.forward_simplified(items.cuda(), w.cuda(), pos, neg, pb, None, nb, None)
    head = {k: v.detach() for k, v in it.state_dict().items()}
    bid = lambda names: [it.brand_vocab.get(x, 0) if x else 0 for x in names]  # noqa: E731
    ref_pos = bert_ref.item_head(torch.from_numpy(emb[[0, 1, 2]]), head, bid(pb), None)
    ref_neg = bert_ref.item_head(torch.from_numpy(emb[[int(t.split("#")[1]) for l in neg for t in l]]),
                                 head, bid([x for l in nb for x in l]), None).view(B, N, 384)
    with torch.no_grad():
        import torch.nn.functional as F
        a = bt.attention(items.view(-1, 384)).view(B, S) * w
        ref_b = F.normalize((torch.softmax(a, 1).unsqueeze(-1) * items).sum(1), dim=1)
    torch.testing.assert_close(out["positive_embeddings"].cpu(), ref_pos, rtol=0, atol=2e-6)
    torch.testing.assert_close(out["negative_embeddings"].cpu(), ref_neg, rtol=0, atol=2e-6)
    torch.testing.assert_close(out["buyer_embeddings"].cpu(), ref_b, rtol=0, atol=5e-6)
    loss = InfoNCELoss(0.07)(out["buyer_embeddings"], out["positive_embeddings"],
                             out["negative_embeddings"])
    ref = losses_ref.infonce(ref_b.double(), ref_pos.double(), ref_neg.double(), 0.07)
    assert abs(loss.item() - ref.item()) < 1e-5
