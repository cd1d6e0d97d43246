#!/usr/bin/env python
"""Headline benchmark: buyers encoded+retrieved/sec @ k=100 over a 1M x 384 catalog
(BASELINE.json metric, configs[2]) on MI355X, with the HBM/MFMA roofline of the dominant
kernel and the CPU baseline beside it.

One step = one pass of the hot path over one batch of synthetic buyers, inputs resident in
HBM before the timed region:
  Mode B buyer encode (gather the 20 history rows of each buyer from the resident item
  table + weighted average + F.normalize; EmbeddingEncoder.encode_buyer with the item rows
  gathered instead of re-encoded)  ->  query re-normalisation (VectorDatabase.retrieve_batch)
  ->  exact inner-product top-k (fused HIP scan + top-k).
Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): the catalog is
row-sharded over the ranks (north_star / SURVEY 8(e)); each rank encodes its own buyers,
queries are all-gathered over RCCL, every rank scans its shard for all queries, per-shard
top-k lists go back to the buyer's owner with one all-to-all and are merged there.  Per-rank
work (buyers x catalog rows scanned) is constant in N: "scaling": "weak".
"""
from __future__ import annotations

import argparse
import json
import statistics
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from twotower import _lib, kernels  # noqa: E402
from twotower.sharded import PipelinedStagedExchange, TopkExchange, shard_range  # noqa: E402

F32_MFMA_PEAK_TFLOPS = 157.3   # MI355X dense f32 MFMA (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (no sparsity)
HBM_PEAK_GBPS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--catalog", type=int, default=1_000_000)
    p.add_argument("--buyers", type=int, default=10_000, help="buyers per rank per step")
    p.add_argument("--hist", type=int, default=20)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--dim", type=int, default=384)
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="gloo: rehearse N ranks on one GPU (functional check, not a measurement)")
    p.add_argument("--method", choices=["bf16", "f32"], default="bf16",
                   help="bf16: bf16 MFMA filter + exact f32 re-rank; f32: exact f32 MFMA scan "
                        "(identical results)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-single", type=int, default=32, help="per repetition (median of 5)")
    p.add_argument("--cpu-batch", type=int, default=512, help="per repetition (median of 5)")
    p.add_argument("--mode-a-buyers", type=int, default=256,
                   help="Mode A sample per rank (history texts re-encoded); 0 disables")
    p.add_argument("--mode-a-prec", choices=["bf16", "x3", "f32"], default="x3",
                   help="x3 (default): the reference's f32 precision class (split-bf16 "
                        "products); bf16 is reported beside it as a throughput mode")
    p.add_argument("--mode-a-steps", type=int, default=3)
    p.add_argument("--no-extra", action="store_true",
                   help="skip the configs[1] leg, the batch sweep and the f32 Mode A leg")
    p.add_argument("--configs1-texts", type=int, default=100_000)
    p.add_argument("--sweep", default="1,8,16,32,256")
    p.add_argument("--chunks", type=int, default=2,
                   help="multi-GPU staged search: query chunks whose collectives overlap the "
                        "next chunk's shard filter (PipelinedStagedExchange)")
    return p.parse_args()


def inflight_streams(n):
    """n fresh HIP streams created back to back for work kept in flight together.  HIP hands
    out hardware queues round-robin (4 on the box), so consecutively created streams sit on
    different queues, while a new stream paired with the default one shares its queue in about
    1 of 4 cases and then serialises with it (tools/stream_overlap.py: a spin kernel on the
    default stream and on a new one took 1.0x / 1.6x / 2.0x of one spin, varying by stream)."""
    return [torch.cuda.Stream() for _ in range(n)]


def event_mix(gen, shape, device):
    u = torch.rand(shape, generator=gen, device=device)
    w = torch.ones(shape, device=device)
    w[u > 0.75] = 5.0
    w[u > 0.92] = 10.0
    return w


def synth_text_ids(rng, n, vocab, lo=16, hi=128):
    """Synthetic 'Arabic-like' token sequences: <s>=0, Zipf(1.1) ids over a 30k sub-range,
    </s>=2; lengths ~ U[lo, hi] (SURVEY.md section 8(d), configs[1])."""
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        out.append([0] + (3 + (rng.zipf(1.1, size=L - 2) % 30000) % (vocab - 3)).tolist() + [2])
    return out


def synth_text_ids_fast(rng, n, vocab, lo=16, hi=128):
    """synth_text_ids in one vectorised draw (same distribution; for the 100k-text leg)."""
    lens = rng.integers(lo, hi + 1, n)
    body = 3 + (rng.zipf(1.1, size=int((lens - 2).sum())) % 30000) % (vocab - 3)
    cu = np.concatenate([[0], np.cumsum(lens - 2)])
    return [[0] + body[cu[i]:cu[i + 1]].tolist() + [2] for i in range(n)]


def encoder_flops(lens, E_out=384):
    """SURVEY.md 8(d) per text: L (42.47e6 + 18432 L) (12-layer MiniLM encoder, L tokens)
    + 0.46e6 (projection head)."""
    L = np.asarray(lens, np.float64)
    return float((L * (42.47e6 + 18432.0 * L)).sum() + 0.46e6 * len(L))


@torch.no_grad()  # inference, as ItemTower.encode_batch runs it
def configs1(a, dev, rank):
    """BASELINE.json configs[1]: 100k products x 384-d, item-tower encode at batch 256 +
    brute-force top-100 (scripts/generate_embeddings.py:52 -> ItemTower.encode_batch,
    item_tower.py:213-243; then VectorDatabase.retrieve_batch, vector_db.py:171-209).
    One step = one batch of 256 product texts: MiniLM-L12 encode (HIP, packed varlen) +
    projection head + F.normalize -> q/(||q||+1e-8) -> exact top-100 of the 256 new item
    embeddings over the 100k x 384 catalog.  The reported value is the x3 encoder (the
    reference's f32 precision class: ItemTower's default) over all 100k texts (the whole
    generate_embeddings pass); the bf16 encoder (throughput mode, below f32 precision) on a
    64-batch sample and the f32-MFMA encoder on a 16-batch sample beside it."""
    from twotower.item_tower import MINILM_L12, BertEncoder, ItemTower, pack_sequences, \
        random_bert_state_dict

    cfg, E, K, BS = MINILM_L12, 384, 100, 256
    n_txt = a.configs1_texts
    rng = np.random.default_rng(200 + rank)
    seqs = synth_text_ids_fast(rng, n_txt, cfg["vocab"])
    bid = rng.integers(0, 51, n_txt).tolist()
    cid = rng.integers(0, 21, n_txt).tolist()

    class _Dim:
        def get_sentence_embedding_dimension(self):
            return cfg["hidden"]

    torch.manual_seed(0)
    it = ItemTower(text_encoder=_Dim())
    it.initialize_categorical_embeddings([f"brand{i}" for i in range(50)],
                                         [f"cat{i}" for i in range(20)])
    it.to(dev).eval()
    sd = random_bert_state_dict(cfg, 0)
    ep = _lib.padded_dim(E)
    g = torch.Generator(device=dev).manual_seed(2)
    cat = torch.zeros((100_000, ep), device=dev)
    cat[:, :E] = torch.randn((100_000, E), generator=g, device=dev)
    cat16 = torch.empty_like(cat, dtype=torch.bfloat16)
    kernels.l2norm_rows(cat, E, _lib.TT_NORM_ADD_EPS, out=cat, out_bf16=cat16)
    bnd = kernels.bf16_image_bounds(cat, cat16, E).tolist()
    ws = torch.empty(kernels.filter_workspace_bytes(100_000, E, BS, K), dtype=torch.uint8,
                     device=dev)
    qn = torch.zeros((BS, ep), device=dev)
    batches = [pack_sequences(seqs[i:i + BS], dev) for i in range(0, n_txt, BS)]
    out = {"workload": "configs[1]: 100k products x 384-d, batch 256 item-tower encode "
                       "(MiniLM-L12 arch, seeded random weights, synthetic Zipf token ids, "
                       "L ~ U[16,128]) + exact top-100 over a 100k x 384 catalog",
           "texts": n_txt, "batch": BS}
    res, ys = {}, {}
    for prec, nb in (("x3", len(batches)), ("bf16", min(64, len(batches))),
                     ("f32", min(16, len(batches)))):
        enc = BertEncoder(sd, cfg, device=dev, prec=prec)
        it.head_prec = "f32" if prec == "f32" else "x3"  # ItemTower's choice with this encoder
        pooled = torch.empty((BS, cfg["hidden"]), device=dev)
        e_enc = [torch.cuda.Event(enable_timing=True) for _ in range(2 * nb)]
        e_srch = [torch.cuda.Event(enable_timing=True) for _ in range(nb)]

        def step(j, timed):
            ids, cu, mx = batches[j]
            nt = cu.numel() - 1
            if timed:
                e_enc[2 * j].record()
            enc.encode_packed(ids, cu, mx, out=pooled[:nt])
            y = it.head(pooled[:nt], bid[j * BS:j * BS + nt], cid[j * BS:j * BS + nt],
                        use_cat=True)
            if timed:
                e_enc[2 * j + 1].record()
            kernels.l2norm_rows(y, E, _lib.TT_NORM_ADD_EPS, out=qn[:nt])
            r = kernels.scan_topk_bf16(cat, cat16, 100_000, E, qn[:nt], K, bnd, workspace=ws)
            if timed:
                e_srch[j].record()
            return y, r

        step(0, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(nb):
            step(j, True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        enc_ms = sum(e_enc[2 * j].elapsed_time(e_enc[2 * j + 1]) for j in range(nb))
        srch_ms = sum(e_enc[2 * j + 1].elapsed_time(e_srch[j]) for j in range(nb))
        # the same batches of 256 with two in flight (alternating streams, each with its own
        # encoder workspace / outputs / search workspace): a batch's GEMMs fill under two
        # rounds of tiles on 256 CUs, the other batch's kernels fill the rest
        NS = getattr(a, "configs1_streams", 2)
        streams = inflight_streams(NS)
        bufs = [(torch.empty((BS, cfg["hidden"]), device=dev), torch.zeros((BS, ep), device=dev),
                 torch.empty_like(ws)) for _ in streams]

        def step2(j):
            pooled_s, qn_s, ws_s = bufs[j % NS]
            ids, cu, mx = batches[j]
            nt = cu.numel() - 1
            enc.encode_packed(ids, cu, mx, out=pooled_s[:nt])
            y = it.head(pooled_s[:nt], bid[j * BS:j * BS + nt], cid[j * BS:j * BS + nt],
                        use_cat=True)
            kernels.l2norm_rows(y, E, _lib.TT_NORM_ADD_EPS, out=qn_s[:nt])
            kernels.scan_topk_bf16(cat, cat16, 100_000, E, qn_s[:nt], K, bnd, workspace=ws_s)

        for j in range(NS):
            with torch.cuda.stream(streams[j % NS]):
                step2(j)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(nb):
            with torch.cuda.stream(streams[j % NS]):
                step2(j)
        torch.cuda.synchronize()
        dt2 = time.perf_counter() - t0
        lens = [len(x) for x in seqs[:nb * BS]]
        fl = encoder_flops(lens)
        peak = F32_MFMA_PEAK_TFLOPS if prec == "f32" else BF16_MFMA_PEAK_TFLOPS
        mf = 3.0 if prec == "x3" else 1.0  # x3: three bf16 MFMAs per product
        ntx = min(n_txt, nb * BS)
        res[prec] = {"texts_timed": ntx, "texts_per_s": ntx / min(dt, dt2),
                     "texts_per_s_two_streams": ntx / dt2, "texts_per_s_one_stream": ntx / dt,
                     "ms_per_batch": dt / nb * 1e3, "encode_ms_per_batch": enc_ms / nb,
                     "search_ms_per_batch": srch_ms / nb,
                     "encode_tflops": fl / (enc_ms * 1e-3) / 1e12,
                     "encode_mfma_frac": mf * fl / (enc_ms * 1e-3) / 1e12 / peak,
                     "encode_mfma_frac_two_streams": mf * fl / dt2 / 1e12 / peak,
                     "mfma_peak_tflops": peak,
                     "tokens_timed": int(sum(lens))}
        if prec == "x3":
            res[prec]["mfma_products_per_flop"] = 3
        ys[prec] = step(0, False)[0].clone().detach()
        del enc
        torch.cuda.empty_cache()
    # bf16 and x3 encoders vs the f32 (parity) encoder on the L2-normalised item embeddings
    # (item_tower.py:209): worst cosine distance / element difference over the first batch
    for prec in ("bf16", "x3"):
        cos = (ys[prec] * ys["f32"]).sum(dim=1)
        res[f"{prec}_vs_f32_item_cosine"] = {
            "min_cos": float(cos.min()), "max_1_minus_cos": float((1 - cos).max()),
            "max_abs_diff": float((ys[prec] - ys["f32"]).abs().max())}
    res["x3_over_f32_texts_per_s"] = res["x3"]["texts_per_s"] / res["f32"]["texts_per_s"]
    # the same 100k texts through the chunking the drop-in API runs: ItemTower.encode_batch(
    # texts, batch_size=256) encodes device chunks of device_batch = 4096 texts (same results
    # row for row, tests/test_gpu_encoder.py), then the top-100 of every 256 new embeddings
    # (pre-tokenized ids: the tokenizer is host-side and out of scope)
    DB = ItemTower.device_batch
    enc = BertEncoder(sd, cfg, device=dev, prec="x3")
    it.head_prec = "x3"
    chunks = [pack_sequences(seqs[i:i + DB], dev) for i in range(0, n_txt, DB)]
    pooled = torch.empty((DB, cfg["hidden"]), device=dev)
    qc = torch.zeros((DB, ep), device=dev)
    wsc = torch.empty(kernels.filter_workspace_bytes(100_000, E, DB, K), dtype=torch.uint8,
                      device=dev)

    def chunk_step(c):
        ids, cu, mx = chunks[c]
        nt = cu.numel() - 1
        enc.encode_packed(ids, cu, mx, out=pooled[:nt])
        y = it.head(pooled[:nt], bid[c * DB:c * DB + nt], cid[c * DB:c * DB + nt], use_cat=True)
        # the top-100 of the chunk's new embeddings in one batched search (each query's exact
        # top 100: the same answers as one search per 256)
        kernels.l2norm_rows(y, E, _lib.TT_NORM_ADD_EPS, out=qc[:nt])
        kernels.scan_topk_bf16(cat, cat16, 100_000, E, qc[:nt], K, bnd, workspace=wsc)

    chunk_step(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(len(chunks)):
        chunk_step(c)
    torch.cuda.synchronize()
    dtc = time.perf_counter() - t0
    res["x3_api_chunks"] = {
        "texts_per_s": n_txt / dtc, "device_batch": DB, "texts": n_txt,
        "is": ("ItemTower.encode_batch(texts, batch_size=256)'s device chunking (4096 texts per "
               "encoder call, x3) + the exact top-100 of each new embedding (one batched search "
               "per chunk)")}
    del enc
    out.update(res)
    out["value"] = res["x3"]["texts_per_s"]
    out["value_prec"] = "x3 (f32 precision class; bf16 throughput mode under 'bf16')"
    out["unit"] = "texts/s (encode + top-100 per batch of 256)"
    return out


def batch_sweep(a, shard, shard16, n, E, K, bounds, dev, i8=None):
    """SURVEY.md 8(d) query-batch sweep over the 1M x 384 catalog (vector_db.py:160,197):
    end-to-end search time per call (every launch of tt_scan_topk_bf16f32, queries resident;
    kernels.PreparedSearch as the serving path calls it, the per-call wrapper beside it) and
    the fraction of the HBM peak for the bytes the search streams: the bf16 image once (2NE),
    end to end and for the full-catalog level alone."""
    ep = _lib.padded_dim(E)
    g = torch.Generator(device=dev).manual_seed(9)
    res = {}
    stream = torch.cuda.current_stream()
    for B in (int(v) for v in a.sweep.split(",") if v):
        q = torch.zeros((B, ep), device=dev)
        q[:, :E] = torch.randn((B, E), generator=g, device=dev)
        kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
        ws = torch.empty(kernels.filter_workspace_bytes(n, E, B, K), dtype=torch.uint8,
                         device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for e in ev:
            e.record(stream)
        for _ in range(3):
            kernels.scan_topk_bf16(shard, shard16, n, E, q, K, bounds, workspace=ws)
        tot, lvl = [], []
        for _ in range(21):
            torch.cuda.synchronize()
            ev[2].record(stream)
            kernels.scan_topk_bf16(shard, shard16, n, E, q, K, bounds, workspace=ws,
                                   events=(ev[0], ev[1]))
            ev[3].record(stream)
            torch.cuda.synchronize()
            tot.append(ev[2].elapsed_time(ev[3]))
            lvl.append(ev[0].elapsed_time(ev[1]))
        tw, l_ = float(np.median(tot)), float(np.median(lvl))
        # end to end through the serving path (one PreparedSearch call per batch; nq <= 32
        # takes the int8 single pass over the tiled image when the catalog has it, same results)
        def prepared(i8_):
            ps = kernels.PreparedSearch(shard, shard16, n, E, B, K, bounds, i8=i8_)
            for _ in range(3):
                ps(q)
            prep = []
            for _ in range(21):
                torch.cuda.synchronize()
                ev[2].record(stream)
                ps(q)
                ev[3].record(stream)
                torch.cuda.synchronize()
                prep.append(ev[2].elapsed_time(ev[3]))
            return float(np.median(prep)), ps.i8, (ps.out[0].clone(), ps.out[1].clone())

        t16, _, o16 = prepared(None)
        t, extra = t16, {}
        if kernels.i8_pass_ok(n, E, B, K, i8):
            t8, used, o8 = prepared(i8)
            if used:
                assert torch.equal(o8[0], o16[0]) and torch.equal(o8[1], o16[1])
                b8 = float(n * ep + 4 * ((n + 63) // 64))  # codes + tile scales, read once
                t = t8
                extra = {"pass": "int8 single pass (bit-identical to the bf16 pass)",
                         "bf16_pass_ms_per_search": t16, "int8_pass_bytes": b8,
                         "int8_pass_frac_end_to_end": b8 / (t8 * 1e-3) / 1e9 / HBM_PEAK_GBPS}
        # bytes the bf16 pass streams: the bf16 image once (the full level; the sample level,
        # selection and re-rank add ~5% and are not counted), so frac <= 1
        res[str(B)] = {"ms_per_search": t, "queries_per_s": B / (t * 1e-3), **extra,
                       "wrapper_ms_per_search": tw, "full_level_ms": l_,
                       "bf16_pass_bytes": 2.0 * n * ep,
                       "bf16_pass_gbps_end_to_end": 2.0 * n * ep / (t16 * 1e-3) / 1e9,
                       "bf16_pass_frac_end_to_end":
                           2.0 * n * ep / (t16 * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                       "full_level_frac": 2.0 * n * ep / (l_ * 1e-3) / 1e9 / HBM_PEAK_GBPS}
        del ws
    # k in (128, 1000] (the /retrieve cap, server.py:46): nq = 1, 32 at k = 1000 through the
    # scores-then-radix-select path the index takes for k > 128 (FlatIPIndex.search_device),
    # the per-slab-list scan beside it at nq = 1
    k2 = 1000

    def time_k(fn, reps=21):
        for _ in range(3):
            fn()
        tk = []
        for _ in range(reps):
            torch.cuda.synchronize()
            ev[2].record(stream)
            fn()
            ev[3].record(stream)
            torch.cuda.synchronize()
            tk.append(ev[2].elapsed_time(ev[3]))
        return float(np.median(tk))

    k1000 = {}
    for nq_ in (1, 32):
        q = torch.zeros((nq_, ep), device=dev)
        q[:, :E] = torch.randn((nq_, E), generator=g, device=dev)
        kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
        ws = torch.empty(kernels.select_workspace_bytes(n, nq_, k2), dtype=torch.uint8,
                         device=dev)
        t = time_k(lambda: kernels.scan_topk_select(shard, n, E, q, k2, workspace=ws))
        k1000[f"nq{nq_}"] = {
            "nq": nq_, "k": k2, "ms_per_search": t,
            "kernel": "tt_scan_topk_select_f32 (exact f32 scores + radix select)",
            "f32_pass_bytes": 4.0 * n * ep,
            "f32_pass_frac_end_to_end": 4.0 * n * ep / (t * 1e-3) / 1e9 / HBM_PEAK_GBPS}
        if nq_ == 1:
            ws2 = torch.empty(kernels.scan_workspace_bytes(n, E, 1, k2), dtype=torch.uint8,
                              device=dev)
            k1000["nq1"]["per_slab_list_scan_ms"] = time_k(
                lambda: kernels.scan_topk(shard, n, E, q, k2, workspace=ws2), reps=5)
            del ws2
        del ws
    k1000.update(k1000.pop("nq1"))  # nq = 1 at the top level (the driver's key), nq = 32 nested
    return {"catalog": f"{n} x {E}", "k": K, "timing": "median of 21 synchronised calls",
            "by_batch": res, "k1000_nq1": k1000}


def catalog_10m(a, dev, nq=10_000, n=10_000_000):
    """configs[3]'s whole 10M x 384 catalog resident on ONE MI355X: the exact top-100 for a
    10k-query batch (bf16 filter + f32 re-rank), timed, with 64 queries re-checked against
    the exact f32 scan (bit-exact ids + scores)."""
    E, K = 384, 100
    ep = _lib.padded_dim(E)
    g = torch.Generator(device=dev).manual_seed(12)
    x = torch.randn((n, ep), generator=g, device=dev)
    x16 = torch.empty((n, ep), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    q = torch.randn((nq, ep), generator=g, device=dev)
    kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
    ws = torch.empty(kernels.filter_workspace_bytes(n, E, nq, K), dtype=torch.uint8, device=dev)
    kernels.scan_topk_bf16(x, x16, n, E, q, K, bnd, workspace=ws)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    stream = torch.cuda.current_stream()
    for e in ev:
        e.record(stream)
    tot, lvl = [], []
    for _ in range(3):
        torch.cuda.synchronize()
        ev[2].record(stream)
        s, i = kernels.scan_topk_bf16(x, x16, n, E, q, K, bnd, workspace=ws, events=(ev[0], ev[1]))
        ev[3].record(stream)
        torch.cuda.synchronize()
        tot.append(ev[2].elapsed_time(ev[3]))
        lvl.append(ev[0].elapsed_time(ev[1]))
    fb = kernels.filter_fallback_count(ws, n, E, nq, K)
    sub = torch.linspace(0, nq - 1, 64, device=dev).round().long()
    fs, fi = kernels.scan_topk(x, n, E, q[sub].contiguous(), K)
    bad = int(((i[sub] != fi) | (s[sub] != fs)).any(dim=1).sum())
    t = float(np.median(tot))
    fl = 2.0 * nq * n * E
    return {"workload": "10M x 384 catalog (configs[3]'s, unsharded) on one GPU, 10k queries, "
                        "k=100", "ms_per_search": t, "queries_per_s": nq / (t * 1e-3),
            "full_level_ms": float(np.median(lvl)),
            "full_level_tflops": fl / (float(np.median(lvl)) * 1e-3) / 1e12,
            "fallback_queries": fb,
            "self_check": {"queries": 64, "mismatched_queries": bad,
                           "vs": "tt_scan_topk_f32 (exact f32)"},
            "hbm_resident_gb": (x.numel() * 4 + x16.numel() * 2) / 1e9}


def catalog_10m_768(a, dev, nq=10_000, n=10_000_000):
    """configs[4]'s search workload on ONE MI355X: the whole 10M x 768 catalog resident (30.7 GB
    f32 + 15.4 GB bf16 image), 10k buyers x 20 history rows gathered from it (Mode B), encoded
    by BuyerTower.attention_aggregation (buyer_tower.py:70-101; tt_attn_agg_l2_f32, seeded MLP
    128 hidden), re-normalised (vector_db.py:189-190) and searched top-100 (bf16 filter + exact
    f32 re-rank).  The full level (k_filter_ring<768, 1>) is reported against the bf16 peak;
    64 queries are re-checked against the exact f32 scan."""
    E, K, S, Hd = 768, 100, 20, 128
    g = torch.Generator(device=dev).manual_seed(13)
    x = torch.randn((n, E), generator=g, device=dev)
    x16 = torch.empty((n, E), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    hist = torch.randint(0, n, (nq, S), generator=g, device=dev)
    w = event_mix(g, (nq, S), dev)
    W1 = torch.randn((Hd, E), generator=g, device=dev) / E ** 0.5
    b1 = 0.1 * torch.randn(Hd, generator=g, device=dev)
    W2 = torch.randn((1, Hd), generator=g, device=dev) / Hd ** 0.5
    b2 = 0.1 * torch.randn(1, generator=g, device=dev)
    items = torch.empty((nq, S, E), device=dev)
    b = torch.empty((nq, E), device=dev)
    q = torch.empty((nq, E), device=dev)
    ws = torch.empty(kernels.filter_workspace_bytes(n, E, nq, K), dtype=torch.uint8, device=dev)
    out = (torch.empty((nq, K), device=dev), torch.empty((nq, K), device=dev, dtype=torch.int64))
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    for e in ev:
        e.record(stream)

    def step(timed):
        if timed:
            ev[4].record(stream)
        torch.index_select(x, 0, hist.view(-1), out=items.view(-1, E))   # Mode B gather
        kernels.attn_agg_l2(items, w, W1, b1, W2, b2, out=b)                # BuyerTower
        kernels.l2norm_rows(b, E, _lib.TT_NORM_ADD_EPS, out=q)               # retrieve_batch
        if timed:
            ev[5].record(stream)
        kernels.scan_topk_bf16(x, x16, n, E, q, K, bnd, workspace=ws, out=out,
                               events=(ev[0], ev[1]) if timed else (None, None))

    step(False)
    tot, lvl, enc = [], [], []
    for _ in range(3):
        torch.cuda.synchronize()
        ev[2].record(stream)
        step(True)
        ev[3].record(stream)
        torch.cuda.synchronize()
        tot.append(ev[2].elapsed_time(ev[3]))
        lvl.append(ev[0].elapsed_time(ev[1]))
        enc.append(ev[4].elapsed_time(ev[5]))
    fb = kernels.filter_fallback_count(ws, n, E, nq, K)
    del ws
    sub = torch.linspace(0, nq - 1, 64, device=dev).round().long()
    fs, fi = kernels.scan_topk(x, n, E, q[sub].contiguous(), K)
    bad = int(((out[1][sub] != fi) | (out[0][sub] != fs)).any(dim=1).sum())
    t, tl = float(np.median(tot)), float(np.median(lvl))
    fl = 2.0 * nq * n * E
    return {"workload": "configs[4] search: 10M x 768 catalog on one GPU, 10k buyers x 20 "
                        "history rows, attention aggregation (MLP 768-128-1), k=100",
            "ms_per_step": t, "buyers_per_s": nq / (t * 1e-3),
            "encode_ms": float(np.median(enc)), "full_level_ms": tl,
            "full_level_kernel": "k_filter_ring<768, 1>",
            "full_level_tflops": fl / (tl * 1e-3) / 1e12,
            "full_level_frac_bf16_peak": fl / (tl * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS,
            "fallback_queries": fb,
            "self_check": {"queries": 64, "mismatched_queries": bad,
                           "vs": "tt_scan_topk_f32 (exact f32)"},
            "hbm_resident_gb": (x.numel() * 4 + x16.numel() * 2) / 1e9}


def train_step_leg(a, dev, steps=20, B=512, N=4, S=20, E=768):
    """configs[4]'s training step (BASELINE.json configs[4]; trainer.py:161-243 with
    forward_simplified, two_tower.py:155-218, InfoNCELoss, losses.py:20-79, Adam): item-tower
    projection head on the positive / 4 negative text embeddings, buyer-tower attention
    aggregation over S = 20 history rows, InfoNCE (in-batch + explicit negatives, tau 0.07),
    backward, Adam -- twotower.train.TwoTowerTrainStep, every GEMM on HIP MFMA, in bf16 (GEMM
    operands) and f32.  Reports ms per step (ms_per_step: forward + backward replayed as one HIP
    graph on a batch resident in the graph's input buffers, then the one-launch Adam;
    graph_copy_inputs_ms_per_step: the same with the batch copied in from the caller's tensors
    every step; eager_ms_per_step: the launches issued one by one), the
    MFMA fraction of the matching dense peak, and the bf16 step's loss / gradient deviation from
    the f32 step on the same weights and batch.  The frozen text encoder is NOT in this leg: the
    step takes text embeddings (see train_step_e2e for the step with the encoder inside).
    Synthetic batch (random-normal text and history embeddings, event-mix weights), random-init
    weights; projection Dropout active (train mode) in the timed steps, off for the deviation."""
    import copy

    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower
    from twotower.train import TwoTowerTrainStep

    class _Dim:
        def get_sentence_embedding_dimension(self):
            return 384

    torch.manual_seed(0)
    it0 = ItemTower(embedding_dim=E, text_encoder=_Dim())
    it0.initialize_categorical_embeddings([f"b{i}" for i in range(500)],
                                          [f"c{i}" for i in range(50)])
    bt0 = BuyerTower(E, "attention")
    g = torch.Generator(device=dev).manual_seed(17)
    items = torch.randn((B, S, E), generator=g, device=dev)
    w = event_mix(g, (B, S), dev)
    pos = torch.randn((B, 384), generator=g, device=dev)
    neg = torch.randn((B, N, 384), generator=g, device=dev)
    pb, pc = (torch.randint(0, m, (B,), generator=g, device=dev, dtype=torch.int32)
              for m in (501, 51))
    nb, nc = (torch.randint(0, m, (B, N), generator=g, device=dev, dtype=torch.int32)
              for m in (501, 51))
    batch = (items, w, pos, neg, pb, pc, nb, nc)
    # flops per step: head forward 2 B(1+N)(512*256 + 256 E), attention MLP 2 B S E 128,
    # in-batch logits 2 B B E; backward ~2x forward
    flops = 3.0 * (2 * B * (1 + N) * (512 * 256 + 256 * E) + 2 * B * S * E * 128 + 2 * B * B * E)
    stream = torch.cuda.current_stream()
    out = {"workload": f"configs[4] training step: B={B}, {N} negatives, S={S} history rows, "
                       f"E={E}, attention aggregation, InfoNCE tau 0.07, Adam",
           "flops_per_step": flops}
    grads = {}
    for prec in ("bf16", "f32"):
        it, bt = copy.deepcopy(it0).to(dev), copy.deepcopy(bt0).to(dev)
        st = TwoTowerTrainStep(it, bt, lr=1e-4, prec=prec)
        it.eval()  # deviation: same weights, same batch, no dropout
        loss, gr = st.forward_backward(*batch)
        grads[prec] = (float(loss), {k: v.detach().clone() for k, v in gr.items()})
        it.train()  # as under the reference Trainer (model.train(), trainer.py:167)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ms = {}
        for mode in ("eager", "graph", "graph_inplace"):
            args = batch
            if mode == "graph":  # the same step captured once in a HIP graph, then replayed
                st = TwoTowerTrainStep(it, bt, lr=1e-4, prec=prec, graph=True)
            if mode == "graph_inplace":  # the batch in the graph's static input buffers (as
                # train_step_e2e's encoder writes it): no input copies in the step
                bi = st.input_buffers(B, S, N)
                bi[0].copy_(items)
                bi[1].copy_(w)
                bi[2][:B].copy_(pos)
                bi[2][B:].copy_(neg.reshape(B * N, -1))
                bi[3][:B].copy_(pb)
                bi[3][B:].copy_(nb.reshape(-1))
                bi[4][:B].copy_(pc)
                bi[4][B:].copy_(nc.reshape(-1))
                args = (bi[0], bi[1], bi[2][:B], bi[2][B:].view(B, N, -1), bi[3][:B], bi[4][:B],
                        bi[3][B:].view(B, N), bi[4][B:].view(B, N))
            for _ in range(3):
                st.step(*args)
            torch.cuda.synchronize()
            ev[0].record(stream)
            for _ in range(steps):
                st.step(*args)
            ev[1].record(stream)
            torch.cuda.synchronize()
            ms[mode] = ev[0].elapsed_time(ev[1]) / steps
        peak = BF16_MFMA_PEAK_TFLOPS if prec == "bf16" else F32_MFMA_PEAK_TFLOPS
        t = ms["graph_inplace"]
        out[prec] = {"ms_per_step": t, "graph_copy_inputs_ms_per_step": ms["graph"],
                     "eager_ms_per_step": ms["eager"],
                     "samples_per_s": B / (t * 1e-3),
                     "tflops": flops / (t * 1e-3) / 1e12,
                     "mfma_frac": flops / (t * 1e-3) / 1e12 / peak,
                     "mfma_peak_tflops": peak, "loss_after": float(st.last_loss)}
        del st, it, bt
    l16, g16 = grads["bf16"]
    l32, g32 = grads["f32"]
    rel = {k: float((g16[k] - g32[k]).norm() / g32[k].norm().clamp_min(1e-30)) for k in g32}
    out["bf16_vs_f32"] = {
        "loss_abs_diff": abs(l16 - l32), "loss_f32": l32,
        "grad_max_rel_l2": max(rel.values()),
        "grad_rel_l2_per_param": rel,
        "is": ("one forward+backward on identical weights and batch, dropout off; relative "
               "Frobenius error per gradient tensor (tests/test_gpu_trainer.py bounds it by 2x "
               "torch autocast-bf16's own error on the same step)")}
    return out


def train_step_e2e(a, dev, steps=3, B=512, N=4, S=20):
    """configs[4]'s training step as the reference's Trainer runs it, encoder included
    (trainer.py:93-131 _encode_buyer_sequences_batched + :161-231 train_epoch with
    forward_simplified, two_tower.py:155-218): per step of B = 512 buyers
      1. the frozen MiniLM encoder over the B*S = 10,240 history texts (ONE pass, :128-131),
      2. the frozen MiniLM encoder over the B positive + 4B negative texts (two_tower.py:182,198;
         2,560 texts, written straight into the step's static text buffer),
      3. head + attention + InfoNCE forward/backward (HIP graph replay) + Adam (one launch).
    E = 384 is the reference's composition exactly (history rows = encode_text outputs, 384-d,
    into a BuyerTower(384)).  At configs[4]'s E = 768 the reference's Trainer cannot run as
    written (384-d encode_text rows into a Linear(768 -> 128)), so the history rows pass the
    frozen item-tower head first (no grad, the inference composition of encoder.py:288-292) to
    become 768-d.  Histories use S = 20 positions (the reference pads to 100 with weight 0:
    exactly zero contribution after the L2 normalisation).  Pre-tokenized
    synthetic ids (the tokenizer is host-side, out of scope), random-init weights, the encoder
    at x3 (the parity class) and bf16 (throughput mode)."""
    import copy

    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import MINILM_L12, BertEncoder, ItemTower, pack_sequences, \
        random_bert_state_dict
    from twotower.train import TwoTowerTrainStep

    cfg = MINILM_L12
    sd = random_bert_state_dict(cfg, 0)
    rng = np.random.default_rng(400)
    R = B + B * N
    nsteps = steps + 1  # one warm-up batch
    # per step: history texts and positive/negative texts, packed on the device up front
    batches = []
    for _ in range(nsteps):
        hs = synth_text_ids_fast(rng, B * S, cfg["vocab"])
        ps = synth_text_ids_fast(rng, R, cfg["vocab"])
        batches.append((pack_sequences(hs, dev), pack_sequences(ps, dev),
                        [len(x) for x in hs] + [len(x) for x in ps]))
    g = torch.Generator(device=dev).manual_seed(23)
    w = event_mix(g, (B, S), dev)
    hb = rng.integers(0, 501, B * S).tolist()
    hc = rng.integers(0, 51, B * S).tolist()
    pb = torch.from_numpy(rng.integers(0, 501, R).astype(np.int32)).to(dev)
    pc = torch.from_numpy(rng.integers(0, 51, R).astype(np.int32)).to(dev)

    class _Dim:
        def get_sentence_embedding_dimension(self):
            return cfg["hidden"]

    out = {"workload": f"configs[4] training step with the frozen text encoder inside: B={B}, "
                       f"{N} negatives, S={S}; {B * S} history + {R} positive/negative texts "
                       "per step through the MiniLM-L12 architecture (seeded random weights, "
                       "synthetic Zipf ids, L ~ U[16,128]), then head + attention + InfoNCE "
                       "fwd/bwd + Adam",
           "texts_per_step": B * S + R}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4 * nsteps)]
    for E in (768, 384):
        torch.manual_seed(0)
        it0 = ItemTower(embedding_dim=E, text_encoder=_Dim())
        it0.initialize_categorical_embeddings([f"b{i}" for i in range(500)],
                                              [f"c{i}" for i in range(50)])
        bt0 = BuyerTower(E, "attention")
        res_e = {}
        for prec in ("x3", "bf16"):
            enc = BertEncoder(sd, cfg, device=dev, prec=prec)
            it, bt = copy.deepcopy(it0).to(dev), copy.deepcopy(bt0).to(dev)
            it.head_prec = "x3"
            st = TwoTowerTrainStep(it, bt, lr=1e-4, prec="bf16", graph=True)
            it.train()
            items, wbuf, text, bids, cids = st.input_buffers(B, S, N)
            wbuf.copy_(w)
            bids.copy_(pb)
            cids.copy_(pc)
            args = (items, wbuf, text[:B], text[B:].view(B, N, -1), bids[:B], cids[:B],
                    bids[B:].view(B, N), cids[B:].view(B, N))
            pooled = torch.empty((B * S, cfg["hidden"]), device=dev)

            def step(j, timed):
                (hi, hcu, hmx), (pi, pcu, pmx), _ = batches[j]
                if timed:
                    ev[4 * j].record()
                with torch.no_grad():
                    if E == cfg["hidden"]:  # the reference's rows: encode_text outputs
                        enc.encode_packed(hi, hcu, hmx, out=items.view(B * S, E))
                    else:  # 768-d rows: the frozen head after the encoder (see docstring)
                        enc.encode_packed(hi, hcu, hmx, out=pooled)
                        it.eval()
                        items.view(B * S, E).copy_(it.head(pooled, hb, hc, use_cat=True))
                        it.train()
                    enc.encode_packed(pi, pcu, pmx, out=text)
                if timed:
                    ev[4 * j + 1].record()
                loss = st.step(*args)
                if timed:
                    ev[4 * j + 2].record()
                return loss

            step(0, False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j in range(1, nsteps):
                loss = step(j, True)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            enc_ms = sum(ev[4 * j].elapsed_time(ev[4 * j + 1]) for j in range(1, nsteps)) / steps
            post_ms = sum(ev[4 * j + 1].elapsed_time(ev[4 * j + 2])
                          for j in range(1, nsteps)) / steps
            lens = [L for j in range(1, nsteps) for L in batches[j][2]]
            fl_enc = encoder_flops(lens) / steps
            fl_step = 3.0 * (2 * B * (1 + N) * (512 * 256 + 256 * E) + 2 * B * S * E * 128
                             + 2 * B * B * E)
            mf = 3.0 if prec == "x3" else 1.0
            res_e[prec] = {"ms_per_step": dt * 1e3, "samples_per_s": B / dt,
                           "texts_per_s": (B * S + R) / dt, "encode_ms": enc_ms,
                           "post_encode_ms": post_ms, "encoder_share": enc_ms / (dt * 1e3),
                           "tflops": (fl_enc + fl_step) / dt / 1e12,
                           "mfma_frac": (mf * fl_enc + fl_step) / dt / 1e12 / BF16_MFMA_PEAK_TFLOPS,
                           "loss_last": float(loss)}
            del enc, st, it, bt
            torch.cuda.empty_cache()
        out[f"E{E}"] = res_e
    out["is"] = ("E768 = configs[4]; E384 = the reference Trainer's exact composition. "
                 "mfma_frac counts x3's three bf16 products per encoder flop; the step's GEMMs "
                 "are bf16 (TwoTowerTrainStep prec='bf16', HIP graph)")
    return out


def _sig(v, n=4):
    return float(f"{v:.{n}g}") if isinstance(v, float) else v


def summary(result):
    """Compact digest of every headline number, printed LAST in the JSON line so a reader
    that keeps only the line's tail (the driver) sees all of them."""
    s = {"value": _sig(result["value"]), "ms_per_step": _sig(result["ms_per_step"]),
         "filter_frac": _sig(result["roofline"]["frac"]),
         "filter_ms": _sig(result["roofline"]["kernel_ms"]),
         "search_minus_filter_ms": _sig(result["roofline"]["search_ms"]
                                        - result["roofline"]["kernel_ms"]),
         "fallbacks": result["roofline"]["fallback_queries_last_step"],
         "self_check_bad": result["self_check"]["mismatched_queries"]}
    ma = result.get("mode_a")
    if ma:
        s["mode_a_buyers_per_s"] = _sig(ma["value"])
        s["mode_a_prec"] = ma["encoder_prec"]
        if "cpu_baseline" in ma:
            s["mode_a_cpu_buyers_per_s"] = _sig(ma["cpu_baseline"]["value"])
    sb = result.get("single_buyer_search")
    if sb:
        s["one_buyer_ms"] = _sig(sb["ms_per_search"])
        if "bf16_pass_ms_per_search" in sb:
            s["one_buyer_bf16_pass_ms"] = _sig(sb["bf16_pass_ms_per_search"])
            s["one_buyer_int8_stream_frac"] = _sig(sb["int8_stream_frac"])
        s["one_buyer_api_ms"] = _sig(sb["api_ms_per_call"])
        s["one_buyer_api_e2e_ms"] = _sig(sb["api_e2e_ms_per_buyer"])
        s["one_buyer_api_k1000_ms"] = _sig(sb["api_k1000_ms_per_call"])
        s["api_calls_per_s_1_vs_4_threads"] = [_sig(sb["api_calls_per_s_1_thread"]),
                                               _sig(sb["api_calls_per_s_4_threads"])]
    bs = result.get("batch_sweep", {}).get("by_batch", {})
    if bs:
        s["batch_ms"] = {b: _sig(v["ms_per_search"]) for b, v in bs.items()}
    if "configs1" in result:
        s["configs1_texts_per_s"] = _sig(result["configs1"]["value"])
        s["configs1_api_chunks_texts_per_s"] = _sig(result["configs1"]["x3_api_chunks"]["texts_per_s"])
    if "catalog_10m" in result:
        s["catalog_10m_queries_per_s"] = _sig(result["catalog_10m"]["queries_per_s"])
    if "catalog_10m_768" in result:
        c = result["catalog_10m_768"]
        s["catalog_10m_768_buyers_per_s"] = _sig(c["buyers_per_s"])
        s["catalog_10m_768_frac"] = _sig(c["full_level_frac_bf16_peak"])
    if "train_step" in result:
        t = result["train_step"]
        s["train_ms"] = {p: _sig(t[p]["ms_per_step"]) for p in ("bf16", "f32")}
        s["train_mfma_frac"] = {p: _sig(t[p]["mfma_frac"]) for p in ("bf16", "f32")}
        s["train_bf16_grad_rel"] = _sig(t["bf16_vs_f32"]["grad_max_rel_l2"])
    if "train_step_e2e" in result:
        t = result["train_step_e2e"]
        s["train_e2e_ms"] = {f"{e}_{p}": _sig(t[e][p]["ms_per_step"])
                             for e in ("E768", "E384") for p in ("x3", "bf16")}
        s["train_e2e_encoder_share"] = _sig(t["E768"]["x3"]["encoder_share"])
    cb = result.get("cpu_baseline")
    if cb:
        s["cpu_buyers_per_s"] = _sig(cb["value"])
        s["cpu_cores"] = cb.get("cores")
    return s


CPU_MODE_A_BUYERS = 32


def single_buyer_api(a, dev, shard, shard16, n, E, K, bounds, table, hist, w, reps=21):
    """The reference's /retrieve chain as it calls the API (server.py:241-244): the buyer's
    embedding arrives as a host numpy vector (encode_buyer's output) and
    VectorDatabase.retrieve(q, k) returns a list of (product_id, score) -- host to host, through
    the drop-in class's prepared serving path (FlatIPIndex.search_host).  Also the same chain
    with the Mode B buyer encode of that one buyer in front (the GPU side of the one-at-a-time
    CPU comparison)."""
    from twotower.vector_db import FlatIPIndex, VectorDatabase

    idx = FlatIPIndex(E, device=dev)
    idx.xb, idx.xb16, idx.ntotal = shard, shard16, n
    idx.bounds = tuple(bounds)
    idx.build_i8()
    vdb = VectorDatabase(E)
    vdb.index = idx
    vdb.product_ids = [f"product_{i}" for i in range(n)]
    qb = torch.empty((1, table.shape[1]), device=dev)

    def encode_one(b):
        kernels.gather_weighted_avg_l2(table, E, hist[b:b + 1], w[b:b + 1], out=qb)
        return qb[0, :E].cpu().numpy()

    q_np = encode_one(0)
    for _ in range(3):
        res = vdb.retrieve(q_np, k=K)
    api, e2e = [], []
    for r in range(reps):
        t0 = time.perf_counter()
        res = vdb.retrieve(q_np, k=K)
        api.append((time.perf_counter() - t0) * 1e3)
    for r in range(reps):
        t0 = time.perf_counter()
        res = vdb.retrieve(encode_one(r % hist.shape[0]), k=K)
        e2e.append((time.perf_counter() - t0) * 1e3)
    assert len(res) == K
    # the /retrieve cap k = 1000 (server.py:46) through the same API: k > 128 takes the
    # scores-then-radix-select path (FlatIPIndex.search_device)
    for _ in range(3):
        res_k = vdb.retrieve(q_np, k=1000)
    api_k = []
    for r in range(reps):
        t0 = time.perf_counter()
        res_k = vdb.retrieve(q_np, k=1000)
        api_k.append((time.perf_counter() - t0) * 1e3)
    assert len(res_k) == 1000
    # concurrent callers (the reference's /retrieve under a threaded server): 4 threads, each
    # call on its own serving slot's stream, vs the same calls from one thread
    import threading

    def calls(n_calls, t_off=0):
        for c in range(n_calls):
            vdb.retrieve(q_np, k=K)

    def threads(n_threads, per):
        th = [threading.Thread(target=calls, args=(per,)) for _ in range(n_threads)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return n_threads * per / (time.perf_counter() - t0)

    calls(20)
    threads(4, 25)  # warm: the coalesced batch sizes' serving slots (streams, pinned buffers)
    t0 = time.perf_counter()
    calls(800)
    one = 800 / (time.perf_counter() - t0)
    st0 = list(idx.coalesce_stats)
    four = threads(4, 200)
    nb, nr = (idx.coalesce_stats[0] - st0[0], idx.coalesce_stats[1] - st0[1])
    return {"api_ms_per_call": statistics.median(api),
            "api_calls_per_s_1_thread": one, "api_calls_per_s_4_threads": four,
            "api_4_threads_mean_batch": nr / max(nb, 1),
            "api_k1000_ms_per_call": statistics.median(api_k),
            "api_ms_per_call_is": ("VectorDatabase.retrieve(host numpy query, k) -> list of "
                                   "(product_id, score), host to host, median of 21"),
            "api_e2e_ms_per_buyer": statistics.median(e2e),
            "api_e2e_is": "Mode B encode of one buyer (device) + .cpu() + VectorDatabase.retrieve"}


@torch.no_grad()  # inference, as ItemTower.encode_batch runs it
def mode_a(a, dev, world, rank, search_local, k, E):
    """Mode A: EmbeddingEncoder.encode_buyer as written (src/inference/encoder.py:286-303):
    each buyer's S history texts are re-encoded by the item tower (MiniLM encoder on HIP,
    projection head, F.normalize), then weighted-averaged and searched."""
    from twotower.item_tower import MINILM_L12, BertEncoder, ItemTower, pack_sequences, \
        random_bert_state_dict

    B, S = a.mode_a_buyers, a.hist
    cfg = MINILM_L12
    sd = random_bert_state_dict(cfg, 0)
    enc = BertEncoder(sd, cfg, device=dev, prec=a.mode_a_prec)

    class _Dim:
        def get_sentence_embedding_dimension(self):
            return cfg["hidden"]

    torch.manual_seed(0)
    it = ItemTower(text_encoder=_Dim(), embedding_dim=E)  # the catalog's dim (--dim)
    it.head_prec = "f32" if a.mode_a_prec == "f32" else "x3"  # as with the HIP text encoder
    it.initialize_categorical_embeddings([f"brand{i}" for i in range(50)],
                                         [f"cat{i}" for i in range(20)])
    it.to(dev).eval()
    rng = np.random.default_rng(100 + rank)
    seqs = synth_text_ids(rng, B * S, cfg["vocab"])
    ids, cu, mx = pack_sequences(seqs, dev)
    bid = rng.integers(0, 51, B * S).tolist()
    cid = rng.integers(0, 21, B * S).tolist()
    w = event_mix(torch.Generator(device=dev).manual_seed(7 + rank), (B, S), dev)
    pooled = torch.empty((B * S, cfg["hidden"]), device=dev)
    ex = TopkExchange(B, _lib.padded_dim(E), k, device=dev)

    def step():
        enc.encode_packed(ids, cu, mx, out=pooled)
        items = it.head(pooled, bid, cid, use_cat=True)            # [B*S, E] unit rows
        q = kernels.weighted_avg_l2(items.view(B, S, E), w)         # BuyerTower.forward
        qn = torch.zeros((B, _lib.padded_dim(E)), device=dev)
        kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=qn)      # retrieve :152-153
        return ex.search(qn, search_local, kernels.merge_topk)

    step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.mode_a_steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / a.mode_a_steps
    dt1 = dt2 = dt
    if world == 1:
        # consecutive steps (independent batches of 256 buyers) two in flight on alternating
        # streams, each with its own encoder workspace / outputs / exchange, as configs[1]
        streams = inflight_streams(2)
        slots = [(torch.empty_like(pooled), TopkExchange(B, _lib.padded_dim(E), k, device=dev))
                 for _ in streams]

        def step2(j):
            pooled_s, ex_s = slots[j % 2]
            enc.encode_packed(ids, cu, mx, out=pooled_s)
            items = it.head(pooled_s, bid, cid, use_cat=True)
            q = kernels.weighted_avg_l2(items.view(B, S, E), w)
            qn = torch.zeros((B, _lib.padded_dim(E)), device=dev)
            kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=qn)
            return ex_s.search(qn, search_local, kernels.merge_topk)

        for j in range(2):
            with torch.cuda.stream(streams[j % 2]):
                step2(j)
        torch.cuda.synchronize()
        n2 = max(4, 2 * a.mode_a_steps)
        t0 = time.perf_counter()
        for j in range(n2):
            with torch.cuda.stream(streams[j % 2]):
                step2(j)
        torch.cuda.synchronize()
        dt2 = (time.perf_counter() - t0) / n2
        dt = min(dt1, dt2)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    tokens = int(ids.numel())
    res = {"value": world * B / dt, "unit": "buyers/s", "ms_per_step": dt * 1e3,
           "buyers_per_s_one_stream": world * B / dt1,
           "buyers_per_s_two_streams": world * B / dt2,
           "buyers_per_rank": B, "texts_per_step_per_rank": B * S,
           "tokens_per_step_per_rank": tokens, "encoder_prec": a.mode_a_prec,
           "texts_per_s": world * B * S / dt,
           "model": "MiniLM-L12 architecture (12L/384h/12 heads/FFN 1536, vocab 250037), "
                    "seeded random weights; synthetic token ids, L ~ U[16,128]"}
    nc = min(CPU_MODE_A_BUYERS, B)  # the CPU baseline's sample (>= 32 buyers)
    cpu_inputs = (sd, cfg, {k2: v.detach().cpu() for k2, v in it.state_dict().items()},
                  [seqs[b * S:(b + 1) * S] for b in range(nc)],
                  [bid[b * S:(b + 1) * S] for b in range(nc)],
                  [cid[b * S:(b + 1) * S] for b in range(nc)], w[:nc].cpu().numpy())
    return res, cpu_inputs


def self_check(a, out, q, table, shard, dev, world, nsub=64):
    """The timed path checks its own results: nsub of this rank's buyers (spread over all
    query tiles) re-searched by the exact f32 MFMA scan (tt_scan_topk_f32, bit-exact vs the C
    oracle in tests/) over the WHOLE catalog; ids and scores must match bit for bit."""
    N, E, K, B = a.catalog, a.dim, a.k, q.shape[0]
    sub = torch.linspace(0, B - 1, min(nsub, B), device=dev).round().long().unique()
    if world == 1:
        full = shard
    else:  # the whole catalog, normalised exactly like the shards were
        full = torch.empty_like(table)
        kernels.l2norm_rows(table, E, _lib.TT_NORM_ADD_EPS, out=full)
    fs, fi = kernels.scan_topk(full, N, E, q[sub].contiguous(), K)
    bad = ((out[1][sub] != fi) | (out[0][sub] != fs)).any(dim=1).sum().to(torch.int64)
    n = torch.tensor([sub.numel()], device=dev, dtype=torch.int64)
    if world > 1:
        dist.all_reduce(bad)
        dist.all_reduce(n)
        del full
    return {"queries": int(n.item()), "mismatched_queries": int(bad.item()),
            "vs": "tt_scan_topk_f32 over the whole catalog (exact f32, bit-exact ids+scores)"}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    if a.backend == "gloo":  # rehearsal: ranks may share the visible GPU(s)
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    N, E, B, S, K = a.catalog, a.dim, a.buyers, a.hist, a.k
    ep = _lib.padded_dim(E)
    # ---- synthetic inputs (identical catalog on every rank; buyers differ per rank)
    g = torch.Generator(device=dev).manual_seed(2)
    table = torch.zeros((N, ep), device=dev)
    table[:, :E] = torch.randn((N, E), generator=g, device=dev)
    kernels.l2norm_rows(table, E, _lib.TT_NORM_MAX_EPS, out=table)  # ItemTower outputs (F.normalize)
    lo, hi = shard_range(N, rank, world)
    shard = torch.empty((hi - lo, ep), device=dev)
    shard16 = torch.empty((hi - lo, ep), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(table[lo:hi], E, _lib.TT_NORM_ADD_EPS, out=shard, out_bf16=shard16)
    bounds = kernels.bf16_image_bounds(shard, shard16, E).tolist()  # build-time statistic
    gb = torch.Generator(device=dev).manual_seed(3 + rank)
    hist = torch.randint(0, N, (B, S), generator=gb, device=dev, dtype=torch.int64)
    w = event_mix(gb, (B, S), dev)

    q = torch.empty((B, ep), device=dev)
    staged = a.method == "bf16" and world > 1
    # all-gather queries (+ their sharded-filter stats) / all-to-all top-k (RCCL); the staged
    # search runs in query chunks whose collectives overlap the next chunk's filter
    ex = TopkExchange(B, ep, K, device=dev)
    pipe = PipelinedStagedExchange(B, ep, K, a.chunks, device=dev) if staged else None
    nq = world * B
    if staged:
        # row-sharded bf16 filter (tt_sharded_filter_*): the replicated 1/16 catalog sample
        # (from the replicated item table, same rows as the shards' images) and the
        # whole-catalog bounds (MAX over ranks), both built once like the index
        sample16 = torch.empty(((N + 15) // 16, ep), device=dev, dtype=torch.bfloat16)
        kernels.l2norm_rows(table[::16].contiguous(), E, _lib.TT_NORM_ADD_EPS,
                            out=torch.empty_like(sample16, dtype=torch.float32),
                            out_bf16=sample16)
        gb_ = torch.tensor(bounds, device=dev)
        dist.all_reduce(gb_, op=dist.ReduceOp.MAX)
        bounds = gb_.tolist()
        bmax = max(c.b for c in pipe.ex)
        ws_begin = torch.empty(kernels.filter_workspace_bytes(sample16.shape[0], E, bmax, K),
                               dtype=torch.uint8, device=dev)
        ws_chunks = [torch.empty(kernels.sharded_workspace_bytes(hi - lo, E, world * c.b, K),
                                 dtype=torch.uint8, device=dev) for c in pipe.ex]
        pc_chunks = [torch.empty((world * c.b, _lib.TT_SHARD_PROBES), dtype=torch.int32,
                                 device=dev) for c in pipe.ex]
        ws_bytes = 256
    elif a.method == "bf16":
        ws_bytes = kernels.filter_workspace_bytes(hi - lo, E, nq, K)
    else:
        ws_bytes = kernels.scan_workspace_bytes(hi - lo, E, nq, K)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    # the catalog's int8 image (built once with the index, like the bf16 one): the one-buyer
    # single pass and the batched search's sample level run on it (same results)
    img8 = (kernels.i8_image(shard, E) if a.method == "bf16" and not staged
            and ep in kernels.I8_DIMS else None)
    if img8 is not None:  # + the tiled copy the register-fed stream reads (padded dim 384)
        img8 = (*img8, kernels.i8_tile(img8[0], hi - lo, E) if ep in kernels.I8T_DIMS else None)
    s_shard = torch.empty((nq, K), device=dev)
    i_shard = torch.empty((nq, K), dtype=torch.int64, device=dev)
    L = _lib.lib()
    stream = torch.cuda.current_stream()

    def local_search(qall, ev):
        e0, e1, p0, p1 = (ev[:4] if ev else (None, None, None, None))
        if p0 is not None:
            p0.record(stream)
        if a.method == "bf16":
            kernels.scan_topk_bf16(shard, shard16, hi - lo, E, qall, K, bounds, row_base=lo,
                                   workspace=ws, out=(s_shard, i_shard), events=(e0, e1),
                                   i8=img8)
        else:
            _lib.check(L.tt_scan_topk_f32_timed(
                shard.data_ptr(), hi - lo, E, shard.stride(0), lo,
                qall.data_ptr(), nq, qall.stride(0), K, s_shard.data_ptr(), i_shard.data_ptr(),
                ws.data_ptr(), ws.numel(), stream.cuda_stream,
                e0.cuda_event if e0 is not None else None,
                e1.cuda_event if e1 is not None else None), "scan")
        if p1 is not None:
            p1.record(stream)
        return s_shard, i_shard

    def step(ev=None):
        kernels.gather_weighted_avg_l2(table, E, hist, w, out=q)  # Mode B buyer encode
        kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)    # retrieve_batch :189-190
        if staged:  # per chunk: this rank's thresholds from the replicated sample (the query
            # all-gather runs async under them), shard filter, probe-count all-reduce and
            # result all-to-all overlapped with the next chunk's filter
            if ev:
                ev[2].record(stream)

            def full(c, qa, sa):
                evc = (ev[4 + 2 * c], ev[5 + 2 * c]) if ev else (None, None)
                return kernels.sharded_full(shard16, hi - lo, E, qa, K, bounds, sa, ws_chunks[c],
                                            pc_chunks[c], events=evc)

            out = pipe.search(
                q, lambda x: kernels.sharded_begin(sample16, E, x, K, workspace=ws_begin), full,
                lambda c, qa, sa, pc: kernels.sharded_finish(shard, shard16, hi - lo, E, qa, K,
                                                             lo, sa, pc, ws_chunks[c]),
                kernels.merge_topk)
            if ev:
                ev[3].record(stream)
            return out
        return ex.search(q, lambda qall: local_search(qall, ev), kernels.merge_topk)

    for _ in range(a.warmup):
        step()
    evs = []
    n_ev = 4 + (2 * len(pipe.ex) if staged else 0)
    for _ in range(a.steps):
        ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(n_ev))
        for e in ev:
            e.record(stream)  # materialise the hipEvent handles; the ABI re-records them
        evs.append(ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        out = step(evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    if staged:  # the shard filter of every chunk
        scan_ms = sum(e[4 + 2 * c].elapsed_time(e[5 + 2 * c]) for e in evs
                      for c in range(len(pipe.ex))) / a.steps
    else:
        scan_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / a.steps
    search_ms = sum(e[2].elapsed_time(e[3]) for e in evs) / a.steps
    if world > 1:
        t = torch.tensor([dt, scan_ms, search_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, scan_ms, search_ms = t.tolist()
    if staged:
        fallback = sum(kernels.filter_fallback_count(ws_chunks[c], hi - lo, E, world * x.b, K,
                                                     sharded=True)
                       for c, x in enumerate(pipe.ex))
    else:
        fallback = (kernels.filter_fallback_count(ws, hi - lo, E, nq, K)
                    if a.method == "bf16" else 0)
    check = self_check(a, out, q, table, shard, dev, world)
    ms_per_step = dt / a.steps * 1e3
    value = world * B / (dt / a.steps)

    # dominant kernel, per launch: nq queries x (hi-lo) rows x E multiply-adds
    #   bf16: k_filter_bf16 over the full shard (bf16 catalog image read once = 2*rows*ep B)
    #   f32:  k_scan_topk_f32 (f32 catalog read once = 4*rows*ep B)
    rows = hi - lo
    flops = 2.0 * nq * rows * E
    elem = 2.0 if a.method == "bf16" else 4.0
    alg_bytes = elem * rows * ep + 4.0 * nq * ep
    achieved_tf = flops / (scan_ms * 1e-3) / 1e12
    # (the instantiation for > 2048 queries per launch; Mode A's 256-query searches use
    # k_filter_ring<ep, 2>, so the profiled average of this name is this workload's)
    kname = f"k_filter_ring<{ep}, 1>" if a.method == "bf16" else "k_scan_topk_f32"
    peak = BF16_MFMA_PEAK_TFLOPS if a.method == "bf16" else F32_MFMA_PEAK_TFLOPS
    traffic = None
    tj = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tj) and world == 1:  # PMC pass is of the 1-GPU launch shape
        tk = json.load(open(tj)).get("kernels", {}).get(kname)
        if tk and tk.get("config", "").startswith(f"{N // 1000000}M x {E}"):
            traffic = tk["fetch_bytes"] + tk["write_bytes"]
    result = {
        "metric": "buyers encoded+retrieved/sec @ k=100, 1M x 384 catalog",
        "value": value,
        "unit": "buyers/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "self_check": check,
        "dtype": "bf16 filter + f32 exact scores" if a.method == "bf16" else "f32",
        "data": "synthetic (random-normal item embeddings, uniform 20-event histories, event mix 0.75/0.17/0.08)",
        "config": {
            "workload": "configs[2]: 1M x 384 catalog, 10k buyers/rank x 20 events, weighted-avg, "
                        "Mode B (history rows gathered), k=100",
            "catalog_rows": N, "dim": E, "buyers_per_rank": B, "history": S, "k": K,
            "sample_level": ("int8 image (k_sample_i8; the threshold it places is certified by "
                             "the exact re-rank)" if img8 is not None and ep == 384 else "bf16"),
            "backend": a.backend if world > 1 else None,
            "parallelism": f"catalog row-shard x{world}" + ((f" + RCCL all-gather(queries, filter stats), all-reduce(probe counts), all-to-all(top-k), {len(pipe.ex)} overlapped query chunks" if staged else " + RCCL all-gather(queries), all-to-all(top-k)") if world > 1 else ""),
        },
        "roofline": {
            "kernel": kname,
            "bound": "mfma",
            "achieved": achieved_tf,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved_tf / peak,
            "traffic": traffic,
            "kernel_ms": scan_ms,
            "search_ms": search_ms,
            "fallback_queries_last_step": fallback,
            "flops_per_launch": flops,
            "algorithmic_bytes_per_launch": alg_bytes,
            "achieved_hbm_gbps": alg_bytes / (scan_ms * 1e-3) / 1e9,
        },
    }
    def local_search_k(qall):
        # Mode A search: the same exact search as Mode B (bf16 filter + f32 re-rank; its
        # full-level launch for a 256-query batch is the separate k_filter_ring<ep, 2>
        # instantiation, so the roofline kernel's profiled average stays Mode B's)
        if a.method == "bf16":
            return kernels.scan_topk_bf16(shard, shard16, hi - lo, E, qall, K, bounds,
                                          row_base=lo)
        return kernels.scan_topk(shard, hi - lo, E, qall, K, row_base=lo)

    if world == 1 and a.method == "bf16":
        # the reference's /retrieve pattern: ONE buyer per search (server.py:241-244).  At
        # nq = 1 the full-catalog level is HBM-bound (bf16 image read once): its achieved
        # bandwidth against the 8 TB/s peak is the scan's HBM roofline.
        q1 = q[:1].clone()
        ws1 = torch.empty(kernels.filter_workspace_bytes(hi - lo, E, 1, K), dtype=torch.uint8,
                          device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        for e in ev:
            e.record(stream)
        for _ in range(3):
            kernels.scan_topk_bf16(shard, shard16, hi - lo, E, q1, K, bounds, workspace=ws1)
        n1, tot, lvl = 21, [], []
        for _ in range(n1):  # per-call wrapper (validation, output allocation every call)
            ev[2].record(stream)
            kernels.scan_topk_bf16(shard, shard16, hi - lo, E, q1, K, bounds, workspace=ws1,
                                   events=(ev[0], ev[1]))
            ev[3].record(stream)
            torch.cuda.synchronize()
            tot.append(ev[2].elapsed_time(ev[3]))
            lvl.append(ev[0].elapsed_time(ev[1]))
        lvl_ms = statistics.median(lvl)
        # the int8 single pass the serving path takes for nq <= 8 (tt_scan_topk_i8f32, same
        # results): its image is built once per catalog, like the bf16 one
        i8 = img8
        i8_lvl, ring_lvl = [], []
        if i8 is not None:
            # the stream the serving path takes (the register-fed one over the tiled image at
            # padded dim 384), and the LDS-ring stream over the row-major image beside it
            for r in range(n1 + 3):
                for tl, acc in ((i8[3], i8_lvl), (None, ring_lvl)):
                    kernels.scan_topk_i8(shard, i8[0], i8[1], hi - lo, E, q1, K, i8[2].tolist(),
                                         row_base=lo, workspace=ws1, events=(ev[0], ev[1]),
                                         tiled=tl)
                    torch.cuda.synchronize()
                    if r >= 3:
                        acc.append(ev[0].elapsed_time(ev[1]))
                    if tl is not None:
                        i8_fb = kernels.filter_fallback_count(ws1, hi - lo, E, 1, K)

        # the device search as the serving path binds it (kernels.PreparedSearch: one C call per
        # buyer, outputs / workspace bound once); median of 21 synchronised calls
        def prepared(i8_):
            ps = kernels.PreparedSearch(shard, shard16, hi - lo, E, 1, K, bounds, row_base=lo,
                                        i8=i8_)
            for _ in range(3):
                ps(q1)
            prep = []
            for _ in range(n1):
                ev[2].record(stream)
                ps(q1)
                ev[3].record(stream)
                torch.cuda.synchronize()
                prep.append(ev[2].elapsed_time(ev[3]))
            o = (ps.out[0].clone(), ps.out[1].clone())
            return statistics.median(prep), o

        bf16_ms, o16 = prepared(None)
        one_ms, o1 = prepared(i8) if i8 is not None else (bf16_ms, o16)
        assert torch.equal(o1[0], o16[0]) and torch.equal(o1[1], o16[1]), "int8 != bf16 pass"
        api = single_buyer_api(a, dev, shard, shard16, hi - lo, E, K, bounds, table, hist, w)
        i8_info = {}
        if i8 is not None:
            i8_ms = statistics.median(i8_lvl)
            i8_bytes = float((hi - lo) * ep + 4 * ((hi - lo + 63) // 64))
            ring_ms = statistics.median(ring_lvl)
            i8_info = {"bf16_pass_ms_per_search": bf16_ms, "int8_stream_ms": i8_ms,
                       "int8_stream_kernel": ("k_filter_topm_i8r<384, 4> (tiled image, "
                                              "register-fed)" if i8[3] is not None else
                                              f"k_filter_topm_i8<{ep}, 4> (LDS ring)"),
                       "int8_stream_bytes": i8_bytes,
                       "int8_stream_gbps": i8_bytes / (i8_ms * 1e-3) / 1e9,
                       "int8_stream_frac": i8_bytes / (i8_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                       "int8_ring_stream_ms": ring_ms,
                       "int8_ring_stream_frac": i8_bytes / (ring_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                       "int8_fallback_queries": int(i8_fb),
                       "int8_same_as_bf16_pass": True}
        result["single_buyer_search"] = {
            "nq": 1, "ms_per_search": one_ms,
            "ms_per_search_is": ("kernels.PreparedSearch device call (no host copies); the int8 "
                                 "single pass (tiled image at padded dim 384: nq <= 32; else "
                                 "nq <= 8), bit-identical to the bf16 pass"
                                 if i8 is not None else
                                 "kernels.PreparedSearch device call (no host copies)"),
            **i8_info,
            **api,
            "timing": "median of 21 synchronised calls, HIP events on the launch stream",
            "wrapper_ms_per_search": statistics.median(tot), "full_level_ms": lvl_ms,
            "full_level_bytes": 2.0 * (hi - lo) * ep,
            "achieved_hbm_gbps": 2.0 * (hi - lo) * ep / (lvl_ms * 1e-3) / 1e9,
            "hbm_peak_gbps": HBM_PEAK_GBPS,
            "frac": 2.0 * (hi - lo) * ep / (lvl_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "kernel": f"k_filter_topm<{ep}>"}
        del ws1

    cpu_a = None
    if a.mode_a_buyers > 0:
        result["mode_a"], cpu_a = mode_a(a, dev, world, rank, lambda qall: local_search_k(qall),
                                         K, E)
    if world == 1 and not a.no_extra:
        result["batch_sweep"] = batch_sweep(a, shard, shard16, hi - lo, E, K, bounds, dev,
                                            i8=i8 if a.method == "bf16" else None)
        if a.mode_a_buyers > 0 and a.mode_a_prec == "x3":
            # beside the parity-precision (x3) Mode A: the bf16 encoder (throughput mode, below
            # the reference's f32 precision) and one step of the f32 MFMA encoder
            for prec, steps in (("bf16", a.mode_a_steps), ("f32", 1)):
                a32 = argparse.Namespace(**vars(a))
                a32.mode_a_prec, a32.mode_a_steps = prec, steps
                m32, _ = mode_a(a32, dev, world, rank, lambda qall: local_search_k(qall), K, E)
                result[f"mode_a_{prec}"] = m32
        result["configs1"] = configs1(a, dev, rank)
        torch.cuda.empty_cache()
        result["catalog_10m"] = catalog_10m(a, dev)
        torch.cuda.empty_cache()
        result["catalog_10m_768"] = catalog_10m_768(a, dev)
        torch.cuda.empty_cache()
        result["train_step"] = train_step_leg(a, dev)
        torch.cuda.empty_cache()
        result["train_step_e2e"] = train_step_e2e(a, dev)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle import cpu_baseline

        del ws
        torch.cuda.empty_cache()
        hist_np = hist.cpu().numpy()
        w_np = w.cpu().numpy()
        table_np = table[:, :E].cpu().numpy()
        cat_np = shard[:, :E].cpu().numpy()
        result["cpu_baseline"] = cpu_baseline.run(table_np, cat_np, hist_np, w_np, K,
                                                  single_buyers=a.cpu_single,
                                                  batch_buyers=a.cpu_batch)
        cb = result["cpu_baseline"]
        sb = result.get("single_buyer_search", {})
        if "api_e2e_ms_per_buyer" in sb:
            # like for like: one buyer at a time on both sides (encode + search, host to host)
            cb["gpu_over_cpu_single"] = (1e3 / sb["api_e2e_ms_per_buyer"]) / cb["value"]
            cb["gpu_over_cpu_single_is"] = ("GPU /retrieve chain one buyer at a time (encode + "
                                            "VectorDatabase.retrieve, host to host) vs the CPU "
                                            "port one buyer at a time")
        cb["gpu_over_cpu_batched"] = value / cb["batched_value"]
        cb["gpu_over_cpu_batched_is"] = ("the GPU batched step (value) vs the CPU port batched "
                                         "(batched_value)")
        if cpu_a is not None:
            sd_, cfg_, head_, seqs_, bid_, cid_, w_ = cpu_a
            result["mode_a"]["cpu_baseline"] = cpu_baseline.run_mode_a(
                sd_, cfg_, head_, seqs_, bid_, cid_, w_, cat_np, K, n_buyers=CPU_MODE_A_BUYERS)
            result["mode_a"]["gpu_over_cpu_single"] = (
                result["mode_a"]["value"] / result["mode_a"]["cpu_baseline"]["value"])
    if rank == 0:
        result["summary"] = summary(result)  # last: the line's tail carries every headline
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
