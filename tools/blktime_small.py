"""Block timeline of one launch of the small-batch ladder (sample level, full level or
k_final_small) at 1M x 384, nq queries (Mode B buyers), k = 100.

Needs a timing build with -DTT_EXP_BLKTIME=1 -DTT_EXP_BLKTIME_LVL=<0: sample level, 2: full
level, 9: k_final_small> (results unaffected):
    VARIANTS="s0:-DTT_EXP_BLKTIME=1,-DTT_EXP_BLKTIME_LVL=0" EXP_FILES=tt_filter bash tools/exp_build2.sh
    TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_s0.so python tools/blktime_small.py
Prints the launch span, the spread of block start times (dispatch) and block durations."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

from twotower import _lib, kernels  # noqa: E402


def pct(a):
    return [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 100)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--catalog", type=int, default=1_000_000)
    a = ap.parse_args()
    N, E, K = a.catalog, 384, 100
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn((N, E), generator=g, device=dev)
    x16 = torch.empty((N, E), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    hist = torch.randint(0, N, (a.nq, 20), generator=g, device=dev)
    q = x[hist].mean(1)
    kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
    ws = torch.empty(kernels.filter_workspace_bytes(N, E, a.nq, K), dtype=torch.uint8, device=dev)
    L = _lib.lib()
    L.tt_debug_blktimes.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    runs = []
    for it in range(6):
        buf = np.zeros((8192, 4), np.uint64)
        L.tt_debug_blktimes(buf.ctypes.data, 8192)  # (read clears nothing: zero by a fresh search)
        kernels.scan_topk_bf16(x, x16, N, E, q, K, bnd, workspace=ws)
        torch.cuda.synchronize()
        n = L.tt_debug_blktimes(buf.ctypes.data, 8192)
        ph = np.zeros((8192, 2), np.uint64)
        if hasattr(L, "tt_debug_blkph"):
            L.tt_debug_blkph.argtypes = [ctypes.c_void_p, ctypes.c_int32]
            L.tt_debug_blkph(ph.ctypes.data, 8192)
        keep = buf[:n, 1] > 0
        rec, ph = buf[:n][keep], ph[:n][keep]
        t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
        base = t0.min()
        s, e = (t0 - base) * 10e-3, (t1 - base) * 10e-3  # us (100 MHz)
        if it >= 2:
            r = {"blocks": int(len(rec)), "span_us": round(float(e.max()), 2),
                 "start_us_pct": pct(s), "dur_us_pct": pct(e - s), "end_us_pct": pct(e)}
            if ph[:, 0].min() > 0:  # ring levels: tile 0 landed / tile loop done, from the start
                p0 = (ph[:, 0].astype(np.int64) - t0) * 10e-3
                p1 = (ph[:, 1].astype(np.int64) - t0) * 10e-3
                r["first_tile_us_pct"] = pct(p0)
                r["loop_us_pct"] = pct(p1 - p0)
                r["tail_us_pct"] = pct((t1 - t0) * 10e-3 - p1)
            runs.append(r)
    print(json.dumps({"nq": a.nq, "catalog": N, "runs": runs}, indent=1))


if __name__ == "__main__":
    main()
