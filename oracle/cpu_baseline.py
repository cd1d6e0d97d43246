"""CPU baseline for bench.py (TEST/MEASUREMENT INFRASTRUCTURE -- never the product).

A CPU port of the reference's hot path for BASELINE.json configs[2] (Mode B buyer encode +
exact top-k), run on the host cores of the GPU box:
  buyer encode   BuyerTower.weighted_average   src/models/buyer_tower.py:58-66  (torch CPU)
  query norm     VectorDatabase.retrieve      src/inference/vector_db.py:151-153 (numpy)
  exact top-k    faiss IndexFlatIP.search     vector_db.py:160 -- faiss-cpu is absent on
                 this image, so the port is its algorithm: BLAS sgemm of the scores
                 (torch CPU matmul) + per-query top-k selection.
Two variants:
  (i)  reference-faithful: one buyer at a time, nq = 1, as /retrieve (server.py:241-244)
       and Evaluator (metrics.py:425-429) call it;
  (ii) batched: retrieve_batch over query blocks (vector_db.py:171-209; no caller in the repo).
If ``import faiss`` works on the host, the faiss IndexFlatIP itself is timed instead
(kind "reference").

``run_mode_a`` times Mode A (EmbeddingEncoder.encode_buyer as written, encoder.py:286-303:
the history texts are re-encoded by the item tower) one buyer at a time: the torch-CPU
restatement of the MiniLM encoder (oracle/bert_ref.py) + projection head + weighted average +
nq = 1 exact search.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.nn.functional as F


def _encode(table: torch.Tensor, hist: np.ndarray, w: np.ndarray) -> np.ndarray:
    x = table[torch.from_numpy(hist)]                      # [b, s, d] gathered history
    wt = torch.from_numpy(w).unsqueeze(-1)
    nw = wt / (wt.sum(dim=1, keepdim=True) + 1e-8)
    return F.normalize((x * nw).sum(dim=1), p=2, dim=1).numpy()


def _gemv_torch_mm(cat: torch.Tensor, q: np.ndarray) -> torch.Tensor:
    """catalog [n, d] . q [d] through torch's matmul (MKL sgemm with one column)."""
    return (cat @ torch.from_numpy(q)[:, None])[:, 0]


def _gemv_torch_mv(cat: torch.Tensor, q: np.ndarray) -> torch.Tensor:
    return torch.mv(cat, torch.from_numpy(q))


def _gemv_numpy(cat: torch.Tensor, q: np.ndarray) -> torch.Tensor:
    """numpy's BLAS sgemv (OpenBLAS in numpy's wheel)."""
    return torch.from_numpy(cat.numpy() @ q)


GEMVS = {"torch_matmul": _gemv_torch_mm, "torch_mv": _gemv_torch_mv, "numpy_sgemv": _gemv_numpy}
_gemv = _gemv_torch_mm  # replaced by the fastest (implementation, threads) pick in run()


def _thread_counts() -> list:
    """Host threads to try: the whole affinity mask and the box's CPU share (OMP_NUM_THREADS;
    on the GPU box the mask shows every CPU of the machine, the share is 16)."""
    try:
        allc = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        allc = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", allc))
    return sorted({allc, share})


def _set_threads(t: int):
    torch.set_num_threads(t)
    try:
        from threadpoolctl import threadpool_limits

        threadpool_limits(t)  # numpy's BLAS pool
    except Exception:  # pragma: no cover
        pass


def pick_gemv(cat: torch.Tensor, one_buyer, reps: int = 3) -> dict:
    """Time one reference-faithful buyer (encode + nq=1 GEMV + top-k: one_buyer()) with every
    GEMV implementation at every thread count (median of reps) and install the fastest as
    _gemv (timing the whole buyer, not the GEMV alone: numpy's BLAS pool and torch's OpenMP
    pool spin against each other).  Round 2 used torch matmul at OMP_NUM_THREADS only: 137 ms
    for the 1M x 384 GEMV (11 GB/s) on the GPU box's EPYC 9575F."""
    global _gemv
    table = {}
    best = None
    for t in _thread_counts():
        _set_threads(t)
        for name, fn in GEMVS.items():
            _gemv = fn
            one_buyer()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                one_buyer()
                ts.append(time.perf_counter() - t0)
            ms = float(np.median(ts)) * 1e3
            table[f"{name}@{t}"] = ms
            if best is None or ms < best[0]:
                best = (ms, name, t)
    ms, name, t = best
    _gemv = GEMVS[name]
    _set_threads(t)
    return {"ms_per_buyer_by_impl_threads": table, "picked": f"{name}@{t}", "threads": t}


def _norm(q: np.ndarray) -> np.ndarray:
    return (q / (np.linalg.norm(q, axis=1, keepdims=True) + 1e-8)).astype(np.float32)


def host_info(threads: int) -> dict:
    """lscpu-style host description (model name + cores used)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = os.cpu_count()
    return {"cpu_model": model, "threads_used": threads, "cpus_visible": os.cpu_count(),
            "cpus_in_affinity_mask": affinity}


def _median_rate(fn, units: int, reps: int):
    """Median over `reps` timed repetitions of fn() (each processing `units`) -> (rate, all)."""
    rates = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        rates.append(units / (time.perf_counter() - t0))
    return float(np.median(rates)), rates


def run(table_np: np.ndarray, catalog_np: np.ndarray, hist: np.ndarray, w: np.ndarray, k: int,
        single_buyers: int = 16, batch_buyers: int = 256, threads: int | None = None,
        reps: int = 5) -> dict:
    table = torch.from_numpy(table_np)
    cat = torch.from_numpy(catalog_np)
    try:
        import faiss  # noqa: F401
        index = faiss.IndexFlatIP(catalog_np.shape[1])
        index.add(catalog_np)
        search = lambda q, kk: index.search(q, kk)  # noqa: E731
        kind = "reference"
    except Exception:
        def search(q, kk):
            if q.shape[0] == 1:  # row-major GEMV + top-k
                v, i = torch.topk(_gemv(cat, q[0]), kk)
                return v[None].numpy(), i[None].numpy()
            s = torch.from_numpy(q) @ cat.T
            v, i = torch.topk(s, kk, dim=1)
            return v.numpy(), i.numpy()
        kind = "port"

    gemv = pick_gemv(cat, lambda: search(_norm(_encode(table, hist[:1], w[:1])), k))
    if threads:
        _set_threads(threads)
    threads = threads or gemv["threads"]
    # warm-up (one buyer each way)
    search(_norm(_encode(table, hist[:1], w[:1])), k)
    search(_norm(_encode(table, hist[:64], w[:64])), k)
    t_all = time.perf_counter()

    # (i) reference-faithful: encode_buyer + retrieve per buyer, nq = 1
    def single():
        for b in range(single_buyers):
            search(_norm(_encode(table, hist[b:b + 1], w[b:b + 1])), k)

    # (ii) batched retrieve_batch in blocks of 64 queries
    nb = batch_buyers

    def batched():
        q = _norm(_encode(table, hist[:nb], w[:nb]))
        for a in range(0, nb, 64):
            search(q[a:a + 64], k)

    v_single, r_single = _median_rate(single, single_buyers, reps)
    v_batch, r_batch = _median_rate(batched, nb, reps)
    # the other thread count(s), one repetition each, reported beside the value
    others = {}
    for t in _thread_counts():
        if t != threads:
            _set_threads(t)
            others[str(t)] = {"single_value": _median_rate(single, single_buyers, 1)[0],
                              "batched_value": _median_rate(batched, nb, 1)[0]}
    _set_threads(threads)
    # where the nq = 1 time goes: the catalog GEMV alone
    q1 = _norm(_encode(table, hist[:1], w[:1]))
    t0 = time.perf_counter()
    for _ in range(8):
        _gemv(cat, q1[0])
    gemv_ms = (time.perf_counter() - t0) / 8 * 1e3
    return {
        "value": v_single,
        "unit": "buyers/s",
        "cores": threads,
        "kind": kind,
        "sample": (f"(i) {single_buyers} buyers one at a time (nq=1) and (ii) {nb} buyers "
                   f"batched 64/query-block, Mode B weighted-avg encode, exact top-{k} over "
                   f"{catalog_np.shape[0]}x{catalog_np.shape[1]} f32, torch-CPU GEMV/sgemm + "
                   f"topk; median of {reps} repetitions of each; GEMV implementation and "
                   f"thread count = the fastest of a probe over both"),
        "batched_value": v_batch,
        "single_rates": r_single, "batched_rates": r_batch,
        "nq1_gemv_ms": gemv_ms,
        "gemv_probe": gemv,
        "other_thread_counts": others,
        "host": host_info(threads),
        "seconds": time.perf_counter() - t_all,
    }


def run_mode_a(sd, cfg, head_sd, seqs_per_buyer, brand_ids, cat_ids, w, catalog_np, k,
               n_buyers: int = 32, threads: int | None = None, reps: int = 5) -> dict:
    """Mode A per buyer: encode S history texts (bert_ref, torch CPU f32) -> head ->
    weighted average -> F.normalize -> q/(||q||+1e-8) -> exact top-k (nq = 1)."""
    from . import bert_ref

    threads = threads or torch.get_num_threads()  # run() left the fastest GEMV setting
    _set_threads(threads)
    cat = torch.from_numpy(catalog_np)

    def one(b):
        seqs = seqs_per_buyer[b]
        cu = np.concatenate([[0], np.cumsum([len(x) for x in seqs])])
        with torch.no_grad():
            te = bert_ref.bert_mean_pool(sd, cfg, torch.tensor([t for x in seqs for t in x]), cu)
            items = bert_ref.item_head(te, head_sd, brand_ids[b], cat_ids[b])
        wt = torch.from_numpy(w[b:b + 1]).unsqueeze(-1)
        nw = wt / (wt.sum(dim=1, keepdim=True) + 1e-8)
        q = _norm(F.normalize((items.unsqueeze(0) * nw).sum(dim=1), p=2, dim=1).numpy())
        torch.topk(_gemv(cat, q[0]), k)

    one(0)  # warm-up
    nb = min(n_buyers, len(seqs_per_buyer))
    t0 = time.perf_counter()
    v, rates = _median_rate(lambda: [one(b) for b in range(nb)], nb, reps)
    dt = time.perf_counter() - t0
    n_texts = sum(len(seqs_per_buyer[b]) for b in range(nb))
    return {"value": v, "unit": "buyers/s", "cores": threads, "kind": "port",
            "sample": f"{nb} buyers one at a time x {reps} repetitions (median; "
                      f"{nb * reps} buyer encodes, {n_texts} distinct history texts) re-encoded "
                      f"by a torch-CPU f32 MiniLM-L12 restatement + head + exact top-{k} "
                      f"(nq=1) over {catalog_np.shape[0]} rows",
            "rates": rates, "host": host_info(threads), "seconds": dt}
