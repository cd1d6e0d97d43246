"""Phase split of the tiled int8 stream (k_filter_topm_i8r) from a TT_I8R_CLK timing build:
per block s_memrealtime stamps (100 MHz) at start, after the prologue (query coding, scales,
barrier), after the block loop, after the merge barrier, at the end (wave 0) -- one search at
1M x 384 (env N), nq = 1.  TWOTOWER_HIP_LIB=<timing build> python tools/i8r_clk.py"""
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
    N, E, K = int(os.environ.get("N", 1_000_000)), 384, 100
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn((N, E), generator=g, device=dev)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x)
    codes, scales, b3 = kernels.i8_image(x, E)
    tiled = kernels.i8_tile(codes, N, E)
    NQ = int(os.environ.get("NQ", 1))
    q = torch.randn((NQ, E), generator=g, device=dev)
    kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
    L = _lib.lib()
    buf = (ctypes.c_ulonglong * (256 * 8 + 8))()
    out = {}
    for rep in range(5):
        kernels.scan_topk_i8(x, codes, scales, N, E, q, K, b3.tolist(), tiled=tiled)
        torch.cuda.synchronize()
    assert L.tt_debug_i8r_clk(buf) == 0
    allv = np.frombuffer(buf, dtype=np.uint64)
    a = allv[:256 * 8].reshape(256, 8)[:, :5].astype(np.float64)
    cnts = allv[:256 * 8].reshape(256, 8)[:, 5:7]
    f = allv[256 * 8:256 * 8 + 5].astype(np.float64)
    t0 = a[:, 0].min()
    us = (a - t0) / 100.0  # 100 MHz -> us
    for i, name in enumerate(("start", "prologue_done", "loop_done", "merge_barrier", "end")):
        col = us[:, i]
        out[name] = {"min": round(col.min(), 2), "median": round(float(np.median(col)), 2),
                     "max": round(col.max(), 2)}
    d = np.diff(us, axis=1)
    for i, name in enumerate(("prologue", "loop", "merge_wait", "epilogue")):
        out["dur_" + name] = {"median": round(float(np.median(d[:, i])), 2),
                              "max": round(float(d[:, i].max()), 2)}
    t7 = allv[:256 * 8].reshape(256, 8)[:, 7].astype(np.float64)
    out["dur_merge"] = {"median": round(float(np.median((t7 - a[:, 3]) / 100.0)), 2)}
    out["dur_exact16"] = {"median": round(float(np.median((a[:, 4] - t7) / 100.0)), 2)}
    out["wave0_compactions_median"] = float(np.median(cnts[:, 0]))
    out["wave0_append_blocks_median"] = float(np.median(cnts[:, 1]))
    fd = np.diff(f) / 100.0
    out["final"] = {"start_after_stream_end_max_us": round((f[0] - a[:, 4].max()) / 100.0, 2),
                    "load_reduce": round(fd[0], 2), "select": round(fd[1], 2),
                    "cert_band": round(fd[2], 2), "rank_out": round(fd[3], 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
