"""One-buyer search latency: where the time between the host call and the result goes.

    python tools/bench_small_search.py [--catalog 1000000] [--nq 1]

Variants (1M x 384 catalog, k = 100, median of --reps synchronised calls unless noted):
  wrapper   kernels.scan_topk_bf16 as bench.py's single_buyer_search calls it
  b2b       the same call issued back to back (GPU time per search, host work overlapped)
  prepared  kernels.PreparedSearch (arguments, outputs and workspace bound once)
  graph     torch.cuda.CUDAGraph replay of one captured search (query copied in first)
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

import torch  # noqa: E402

from twotower import _lib, kernels  # noqa: E402


def timed(fn, reps, stream):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    gpu, host = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record(stream)
        fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        host.append((time.perf_counter() - t0) * 1e3)
        gpu.append(ev[0].elapsed_time(ev[1]))
    return {"events_ms": round(statistics.median(gpu), 4),
            "host_ms": round(statistics.median(host), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--catalog", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--nq", type=int, default=1)
    ap.add_argument("--reps", type=int, default=41)
    ap.add_argument("--modeb", action="store_true",
                    help="queries = L2-normalised means of 20 catalog rows (the bench's Mode B "
                         "buyers) instead of iid")
    a = ap.parse_args()
    N, E, K, NQ = a.catalog, a.dim, a.k, a.nq
    ep = _lib.padded_dim(E)
    g = torch.Generator(device="cuda").manual_seed(0)
    db = torch.zeros((N, ep), device="cuda")
    db[:, :E] = torch.randn((N, E), generator=g, device="cuda")
    db16 = torch.empty((N, ep), device="cuda", dtype=torch.bfloat16)
    kernels.l2norm_rows(db, E, 0, out=db, out_bf16=db16)
    bounds = kernels.bf16_image_bounds(db, db16, E).tolist()
    q = torch.zeros((NQ, ep), device="cuda")
    if a.modeb:
        hist = torch.randint(0, N, (NQ, 20), generator=g, device="cuda")
        q[:, :E] = db[hist, :E].mean(dim=1)
    else:
        q[:, :E] = torch.randn((NQ, E), generator=g, device="cuda")
    kernels.l2norm_rows(q, E, 0, out=q)
    stream = torch.cuda.current_stream()
    ws = torch.empty(kernels.filter_workspace_bytes(N, E, NQ, K), dtype=torch.uint8, device="cuda")
    ref = kernels.scan_topk_bf16(db, db16, N, E, q, K, bounds, workspace=ws)
    res = {"catalog": N, "dim": E, "k": K, "nq": NQ, "queries": "modeb" if a.modeb else "iid"}

    def wrapper():
        return kernels.scan_topk_bf16(db, db16, N, E, q, K, bounds, workspace=ws)

    for _ in range(5):
        wrapper()
    res["wrapper"] = timed(wrapper, a.reps, stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(50):
        wrapper()
    e1.record(stream)
    torch.cuda.synchronize()
    res["b2b_ms"] = round(e0.elapsed_time(e1) / 50, 4)

    if hasattr(kernels, "PreparedSearch"):
        ps = kernels.PreparedSearch(db, db16, N, E, NQ, K, bounds)
        for _ in range(5):
            ps(q)
        out = ps(q)
        torch.cuda.synchronize()
        assert torch.equal(out[1], ref[1]) and torch.equal(out[0], ref[0])
        res["prepared"] = timed(lambda: ps(q), a.reps, stream)

    qs = q.clone()
    outs = (torch.empty((NQ, K), device="cuda"), torch.empty((NQ, K), dtype=torch.int64, device="cuda"))
    side = torch.cuda.Stream()
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        for _ in range(3):
            kernels.scan_topk_bf16(db, db16, N, E, qs, K, bounds, workspace=ws, out=outs)
    stream.wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        kernels.scan_topk_bf16(db, db16, N, E, qs, K, bounds, workspace=ws, out=outs)

    def replay():
        qs.copy_(q)
        graph.replay()

    for _ in range(5):
        replay()
    torch.cuda.synchronize()
    assert torch.equal(outs[1], ref[1]) and torch.equal(outs[0], ref[0])
    res["graph"] = timed(replay, a.reps, stream)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
