"""/retrieve under concurrent callers: VectorDatabase.retrieve(host query, k=100) calls/s from 1,
4 and 8 threads over the configs[2] catalog (1M x 384, int8 single pass for nq <= 4), for
coalescing variants (FlatIPIndex.LEAD_EXTRA / COALESCE_MAX set per instance), in one process,
variant order rotated every repetition."""
import json
import os
import statistics
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

from twotower import _lib, kernels  # noqa: E402
from twotower.vector_db import FlatIPIndex, VectorDatabase  # noqa: E402

VARIANTS = [(0, 8), (0, 4), (0, 2), (0, 0)]  # (LEAD_EXTRA, COALESCE_MAX); 0: no coalescing


def main():
    N, E, K = 1_000_000, 384, 100
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn((N, E), generator=g, device=dev)
    x16 = torch.empty((N, E), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    idx = FlatIPIndex(E, device=dev)
    idx.xb, idx.xb16, idx.ntotal, idx.bounds = x, x16, N, tuple(bnd)
    idx.build_i8()
    vdb = VectorDatabase(E)
    vdb.index = idx
    vdb.product_ids = [f"product_{i}" for i in range(N)]
    qs = [torch.randn(E, generator=g, device=dev).cpu().numpy() for _ in range(64)]
    ref = [vdb.retrieve(q, k=K) for q in qs]

    def calls(n, off, bad):
        for c in range(n):
            j = (off + c) % len(qs)
            if vdb.retrieve(qs[j], k=K) != ref[j]:
                bad.append(j)

    def rate(threads, per=100):
        bad = []
        th = [threading.Thread(target=calls, args=(per, 7 * t, bad)) for t in range(threads)]
        st0 = list(idx.coalesce_stats)
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        nb, nr = idx.coalesce_stats[0] - st0[0], idx.coalesce_stats[1] - st0[1]
        assert not bad, bad
        return threads * per / dt, nr / max(nb, 1)

    res = {f"lead{le}_max{cm}": {"1": [], "4": [], "8": [], "batch4": [], "batch8": []}
           for le, cm in VARIANTS}
    def setv(le, cm):
        idx.LEAD_EXTRA, idx.COALESCE_MAX = le, max(cm, 1)
        idx.coalesce = cm > 0

    for v in VARIANTS:
        setv(*v)
        rate(1, 20)
        rate(4, 20)
    for rep in range(5):
        order = VARIANTS[rep % len(VARIANTS):] + VARIANTS[:rep % len(VARIANTS)]
        for le, cm in order:
            setv(le, cm)
            r = res[f"lead{le}_max{cm}"]
            r["1"].append(rate(1)[0])
            v4, b4 = rate(4)
            v8, b8 = rate(8)
            r["4"].append(v4)
            r["8"].append(v8)
            r["batch4"].append(b4)
            r["batch8"].append(b8)
    out = {name: {k: round(statistics.median(v), 2) for k, v in r.items()}
           for name, r in res.items()}
    print(json.dumps({"config": f"{N} x {E}, k={K}, calls/s (median of 5)", "variants": out},
                     indent=1))


if __name__ == "__main__":
    main()
