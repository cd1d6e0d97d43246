"""Per-CU timeline of the batched full level (k_filter_ring<384, 1>) at configs[2].

Needs a timing build with -DTT_EXP_BLKTIME=1 (results unaffected, the kernel records per block
its start / end wall clock (100 MHz), HW_ID and XCC_ID):
    VARIANTS="blk:-DTT_EXP_BLKTIME=1" EXP_FILES=tt_filter bash tools/exp_build2.sh
    TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/exp/lib_blk.so python tools/blktime.py
Prints where the launch's CU time goes: blocks per CU, busy fraction, the idle head / tail
per CU, the gaps between a CU's consecutive blocks, block durations by query tile."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

from twotower import _lib, kernels  # noqa: E402


def main():
    N, E, B, S, K = 1_000_000, 384, 10_000, 20, 100
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    table = torch.zeros((N, E), device=dev)
    table[:] = torch.randn((N, E), generator=g, device=dev)
    kernels.l2norm_rows(table, E, _lib.TT_NORM_MAX_EPS, out=table)
    x = torch.empty_like(table)
    x16 = torch.empty((N, E), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(table, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    gb = torch.Generator(device=dev).manual_seed(3)
    hist = torch.randint(0, N, (B, S), generator=gb, device=dev)
    w = torch.ones((B, S), device=dev)
    q = kernels.gather_weighted_avg_l2(table, E, hist, w)
    kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
    ws = torch.empty(kernels.filter_workspace_bytes(N, E, B, K), dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record()
    for _ in range(4):
        kernels.scan_topk_bf16(x, x16, N, E, q, K, bnd, workspace=ws, events=(ev[0], ev[1]))
    torch.cuda.synchronize()
    lvl_ms = ev[0].elapsed_time(ev[1])
    L = _lib.lib()
    L.tt_debug_blktimes.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    buf = np.zeros((8192, 4), np.uint64)
    n = L.tt_debug_blktimes(buf.ctypes.data, 8192)
    rec = buf[:n]
    rec = rec[rec[:, 1] > 0]
    t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    hw, xcc = rec[:, 2].astype(np.int64), (rec[:, 3] & 0xF).astype(np.int64)
    lb = (rec[:, 3] >> 32).astype(np.int64)
    cu = xcc * 256 + ((hw >> 8) & 0xFF)
    base = t0.min()
    t0, t1 = (t0 - base) * 10e-3, (t1 - base) * 10e-3  # us
    span = t1.max()
    n_qt = (B + 383) // 384
    dur = t1 - t0
    part = (lb % n_qt) == n_qt - 1
    out = {"level_ms_hip_events": lvl_ms, "blocks": int(len(rec)), "span_us": float(span),
           "cus": int(len(np.unique(cu))),
           "block_us_full_tiles": [float(np.percentile(dur[~part], p)) for p in (0, 50, 100)],
           "block_us_partial_tile": [float(np.percentile(dur[part], p)) for p in (0, 50, 100)]
           if part.any() else None}
    heads, tails, gaps, busy, nblk = [], [], [], [], []
    for c in np.unique(cu):
        m = cu == c
        a, b = np.sort(t0[m]), np.sort(t1[m])
        heads.append(a[0])
        tails.append(span - b[-1])
        gaps.extend((a[1:] - b[:-1]).tolist())
        busy.append(float((b - a).sum()))
        nblk.append(int(m.sum()))
    out["blocks_per_cu"] = {int(k): int(v) for k, v in zip(*np.unique(nblk, return_counts=True))}
    out["busy_frac_mean"] = float(np.sum(busy) / (len(busy) * span))
    out["idle_head_us_mean"] = float(np.mean(heads))
    out["idle_tail_us_mean"] = float(np.mean(tails))
    out["idle_tail_us_max"] = float(np.max(tails))
    out["gap_us_mean"] = float(np.mean(gaps)) if gaps else 0.0
    out["gap_us_p90"] = float(np.percentile(gaps, 90)) if gaps else 0.0
    out["idle_us_per_cu_total_mean"] = float(span - np.mean(busy))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
