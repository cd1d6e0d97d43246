"""Exact top-k for k in (128, 1024] at small batches: tt_scan_topk_f32 (per-slab lists +
merge) vs the scores-then-radix-select path (kernels.scan_topk_select), 1M x 384 catalog.

    python tools/bench_large_k.py [--n 1000000] [--ks 129,500,1000] [--nqs 1,8,32]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

import torch  # noqa: E402

from twotower import _lib, kernels  # noqa: E402


def timed(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2], r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=384)
    ap.add_argument("--ks", default="129,500,1000")
    ap.add_argument("--nqs", default="1,8,32")
    ap.add_argument("--paths", default="select,scan")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    ep = _lib.padded_dim(a.d)
    db = torch.zeros((a.n, ep), device=dev)
    db[:, :a.d] = torch.randn((a.n, a.d), generator=g, device=dev)
    kernels.l2norm_rows(db, a.d, _lib.TT_NORM_ADD_EPS, out=db)
    out = {"n": a.n, "d": a.d}
    for nq in (int(v) for v in a.nqs.split(",")):
        q = torch.zeros((nq, ep), device=dev)
        q[:, :a.d] = torch.randn((nq, a.d), generator=g, device=dev)
        kernels.l2norm_rows(q, a.d, _lib.TT_NORM_ADD_EPS, out=q)
        for k in (int(v) for v in a.ks.split(",")):
            res = {}
            outs = {}
            for p in a.paths.split(","):
                f = {"scan": lambda: kernels.scan_topk(db, a.n, a.d, q, k),
                     "select": lambda: kernels.scan_topk_select(db, a.n, a.d, q, k),
                     "large": lambda: kernels.scan_topk_large(db, a.n, a.d, q, k)}[p]
                ms, r = timed(f)
                res[p + "_ms"] = round(ms, 4)
                outs[p] = r
            if len(outs) >= 2:
                (s0, i0), *rest = outs.values()
                res["bit_exact"] = all(bool(torch.equal(i0, i1) and torch.equal(s0, s1))
                                       for s1, i1 in rest)
            out[f"nq{nq}_k{k}"] = res
            print(json.dumps({f"nq{nq}_k{k}": res}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
