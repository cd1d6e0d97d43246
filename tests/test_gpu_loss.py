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
