"""How many rows does the exact re-rank need per query?  (CPU, numpy/torch; VERDICT r4 #3.)

The bf16 filter's band is {a >= A_k - 2 eps_q}, eps_q the per-query
Cauchy-Schwarz bound with the catalog-wide R = max ||x_r - bf16(x_r)||.  Variants measured:
  rowR     eps_r with each row's own residual norm R_r (4 B per row beside the bf16 image):
           band = {a_r + eps_r >= L_k}, L_k = k-th largest (a_r - eps_r)
  twophase exact scores of the k rows with the largest a first; s1 = their minimum is a lower
           bound of s_k, so the rest of the band needs a_r + eps_r >= s1 only
  both     the two together
Queries: iid unit vectors, and Mode B buyers (weighted averages of 20 catalog rows, as bench.py).
"""
import argparse
import json

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--e", type=int, default=384)
    ap.add_argument("--nq", type=int, default=24)
    ap.add_argument("--k", type=int, default=100)
    a = ap.parse_args()
    torch.manual_seed(0)
    n, E, k = a.n, a.e, a.k
    x = torch.randn(n, E)
    x /= x.norm(dim=1, keepdim=True) + 1e-8
    x16 = x.to(torch.bfloat16).float()
    Rr = (x - x16).norm(dim=1)
    X, R = float(x.norm(dim=1).max()), float(Rr.max())
    out = {"R_max": R, "R_mean": float(Rr.mean()), "R_p50": float(Rr.median())}
    qi = torch.randn(a.nq, E)
    hist = torch.randint(0, n, (a.nq, 20))
    w = torch.ones(a.nq, 20)
    w[torch.rand(a.nq, 20) > 0.75] = 5.0
    qb = (x[hist] * (w / w.sum(1, keepdim=True))[..., None]).sum(1)
    for name, q in (("iid", qi), ("mode_b", qb)):
        q = q / (q.norm(dim=1, keepdim=True) + 1e-8)
        q16 = q.to(torch.bfloat16).float()
        A = (q16.double() @ x16.double().T)           # the filter's bf16 products
        S = (q.double() @ x.double().T)               # exact scores
        qn, dq, qt = q.norm(dim=1), (q - q16).norm(dim=1), q16.norm(dim=1)
        tail = 2 * E * 2.0 ** -23 * (X + R) * qt + E * 2.0 ** -24 * X * qn
        eps = 1.001 * (R * qn + (X + R) * dq + tail)                      # [nq]
        eps_r = 1.001 * (Rr[None, :] * qn[:, None] + (X + Rr[None, :]) * dq[:, None]
                         + tail[:, None])                                 # [nq, n]
        res = {"eps_mean": float(eps.mean()), "actual_max_abs_err": float((A - S).abs().max())}
        cnt = {"global": [], "rowR": [], "twophase": [], "both": []}
        for i in range(a.nq):
            ai, si, e, er = A[i], S[i], float(eps[i]), eps_r[i].double()
            Ak = float(torch.topk(ai, k).values[-1])
            band = ai >= Ak - 2 * e
            cnt["global"].append(int(band.sum()))
            Lk = float(torch.topk(ai - er, k).values[-1])
            cnt["rowR"].append(int((ai + er >= Lk).sum()))
            top = ai >= Ak
            s1 = float(si[top].min())
            cnt["twophase"].append(int(top.sum() + ((~top) & band & (ai + e >= s1)).sum()))
            bandr = ai + er >= Lk
            cnt["both"].append(int(top.sum() + ((~top) & bandr & (ai + er >= s1)).sum()))
            assert torch.isin(torch.topk(si, k).indices, torch.nonzero(bandr).flatten()).all()
        res.update({kk: float(np.mean(v)) for kk, v in cnt.items()})
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
