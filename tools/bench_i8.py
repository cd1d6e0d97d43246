"""One-buyer / small-batch latency (env NQS = batch sizes, default 1,2,4): bf16 single pass vs the int8 single pass (1M x 384, k=100),
kernels.PreparedSearch device calls, median of 51 synchronised calls (HIP events), plus the
stream kernel alone (ev_start/ev_stop around k_filter_topm / k_filter_topm_i8[r]).  I8VS = the
int8 streams to time in turn (ring: k_filter_topm_i8 over the row-major image; tiled:
k_filter_topm_i8r over kernels.i8_tile's image; default "ring,tiled,ring,tiled": an A/B x2 in
one process)."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

from twotower import _lib, kernels  # noqa: E402


def main():
    N, E, K = int(os.environ.get("N", 1_000_000)), int(os.environ.get("E", 384)), 100
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    ep = _lib.padded_dim(E)
    x = torch.zeros((N, ep), device=dev)
    x[:, :E] = torch.randn((N, E), generator=g, device=dev)
    x16 = torch.empty((N, ep), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(x, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    codes, scales, b3 = kernels.i8_image(x, E)
    tiled = kernels.i8_tile(codes, N, E) if ep in kernels.I8T_DIMS else None
    out = {"config": f"{N} x {E}, k={K}", "i8_bounds": b3.tolist()}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    st = torch.cuda.current_stream()
    for e in ev:
        e.record(st)
    kernels.I8_NQ_MAX = int(os.environ.get("I8MAX", kernels.I8_NQ_MAX))  # timing builds only
    for nq in (int(v) for v in os.environ.get("NQS", "1,2,4").split(",")):
        q = torch.zeros((nq, ep), device=dev)
        q[:, :E] = torch.randn((nq, E), generator=g, device=dev)
        kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
        res = {}
        ref = None
        runs = [("bf16", None, None)]
        for r, v in enumerate(os.environ.get("I8VS", "ring,tiled,ring,tiled").split(",")):
            if v == "tiled" and tiled is None:
                continue
            runs.append((f"i8_{v}" + ("" if r < 2 else f"_{r // 2 + 1}"),
                         (codes, scales, b3) + ((tiled,) if v == "tiled" else ()),
                         tiled if v == "tiled" else None))
        for name, i8, tl in runs:
            if i8 is not None and nq > (kernels.I8T_NQ_MAX if tl is not None else kernels.I8_NQ_MAX):
                continue
            ps = kernels.PreparedSearch(x, x16, N, E, nq, K, bnd, i8=i8)
            assert ps.i8 == (i8 is not None)
            for _ in range(5):
                ps(q)
            t = []
            for _ in range(51):
                torch.cuda.synchronize()
                ev[2].record(st)
                ps(q)
                ev[3].record(st)
                torch.cuda.synchronize()
                t.append(ev[2].elapsed_time(ev[3]))
            o = (ps.out[0].clone(), ps.out[1].clone())
            if ref is None:
                ref = o
            same = bool(torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]))
            ws = torch.empty(kernels.filter_workspace_bytes(N, E, nq, K), dtype=torch.uint8,
                             device=dev)
            lv = []
            for _ in range(21):
                torch.cuda.synchronize()
                if i8 is not None:
                    kernels.scan_topk_i8(x, codes, scales, N, E, q, K, b3.tolist(), workspace=ws,
                                         events=(ev[0], ev[1]), tiled=tl)
                else:
                    kernels.scan_topk_bf16(x, x16, N, E, q, K, bnd, workspace=ws,
                                           events=(ev[0], ev[1]))
                torch.cuda.synchronize()
                lv.append(ev[0].elapsed_time(ev[1]))
            fb = kernels.filter_fallback_count(ws, N, E, nq, K)
            res[name] = {"ms_per_search": statistics.median(t), "stream_ms": statistics.median(lv),
                         "same_as_bf16": same, "fallbacks_last": fb}
        out[f"nq{nq}"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
