"""Cycle split of the int8 single pass's tile loop (k_filter_topm_i8<384>, 1M x 384, nq = 1).
Needs a timing build with -DTT_I8_EXP_CLK=1 (results unaffected; s_memtime stamps, each one
waits for the wave's outstanding LDS / scalar loads, so segments 3-4 merge):
  TWOTOWER_HIP_LIB=.../lib_clk.so python tools/i8clk.py
Per wave class (compute waves 0-3, DMA-only waves 4-7): mean cycles per tile in
0 wait_tiles, 1 barrier, 2 DMA issue, 3 appends (8: fragment reads), 4 lds_wait, 5 MFMA + scale,
and the whole loop."""
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
    N, E, K = 1_000_000, 384, 100
    nq = int(os.environ.get("NQ", 1))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn((N, E), generator=g, device=dev)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x)
    codes, scales, b3 = kernels.i8_image(x, E)
    q = torch.randn((nq, E), generator=g, device=dev)
    kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
    ws = torch.empty(kernels.filter_workspace_bytes(N, E, nq, K), dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record()
    ms = []
    for _ in range(8):
        kernels.scan_topk_i8(x, codes, scales, N, E, q, K, b3.tolist(), workspace=ws,
                             events=(ev[0], ev[1]))
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    L = _lib.lib()
    L.tt_debug_i8clk.argtypes = [ctypes.c_void_p]
    buf = np.zeros((256, 8, 8), np.uint64)
    assert L.tt_debug_i8clk(buf.ctypes.data) == 0
    reads = (buf[:, :, 3] >> np.uint64(32)).astype(np.float64)
    n_any = (buf[:, :, 4] >> np.uint64(32)).astype(np.float64)
    n_cmp = (buf[:, :, 5] >> np.uint64(32)).astype(np.float64)
    buf[:, :, 3:6] &= np.uint64(0xFFFFFFFF)
    c = np.concatenate([buf.astype(np.float64), reads[..., None]], axis=2)
    c = c[c[:, 0, 7] > 0]  # blocks past the catalog's end have no tiles
    nt = c[:, :, 7]
    names = ["wait_tiles", "barrier", "issue", "appends", "lds_wait", "mfma_scale"]
    live = buf[:, 0, 7] > 0
    out = {"stream_ms_median": float(np.median(ms)), "tiles_per_block": float(nt[:, 0].mean()),
           "appends_run_tiles_per_wave": float(n_any[live][:, :4].mean()),
           "compactions_per_wave": float(n_cmp[live][:, :4].mean())}
    for cls, ws_ in (("compute_waves", slice(0, 4)), ("dma_waves", slice(4, 8))):
        per = c[:, ws_, :6] / nt[:, ws_, None]
        out[cls] = {nm: round(float(per[..., i].mean()), 1) for i, nm in enumerate(names)}
        out[cls]["fragment_reads"] = round(float((c[:, ws_, 8] / nt[:, ws_]).mean()), 1)
        out[cls]["loop_total_per_tile"] = round(float((c[:, ws_, 6] / nt[:, ws_]).mean()), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
