"""In-process A/B of filter-library variants on the configs[2] search (1M x 384, 10k Mode B
buyers, k = 100): every variant's tt_scan_topk_bf16f32 is called in turn from ONE process on
the same device buffers, the order rotated every repetition, so clock and thermal drift hit
all variants alike (separate bench.py processes had shown a first-run bias of ~2-5%).
    python tools/ab_inproc.py --libs a.so,b.so,... [--reps 12]
Prints per variant the median full-level and whole-search times (HIP events on the launch
stream) and checks that all variants return identical results."""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

from twotower import _lib, kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--nq", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--i8", action="store_true",
                    help="call tt_scan_topk_bf16f32_i8s with the catalog's int8 image")
    a = ap.parse_args()
    N, E, B, S, K = a.n, a.dim, a.nq, 20, a.k
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(2)
    ep = _lib.padded_dim(E)
    table = torch.zeros((N, ep), device=dev)
    table[:, :E] = torch.randn((N, E), generator=g, device=dev)
    kernels.l2norm_rows(table, E, _lib.TT_NORM_MAX_EPS, out=table)
    x = torch.empty_like(table)
    x16 = torch.empty((N, ep), device=dev, dtype=torch.bfloat16)
    kernels.l2norm_rows(table, E, _lib.TT_NORM_ADD_EPS, out=x, out_bf16=x16)
    bnd = kernels.bf16_image_bounds(x, x16, E).tolist()
    img = kernels.i8_image(x, E) if a.i8 else None
    gb = torch.Generator(device=dev).manual_seed(3)
    hist = torch.randint(0, N, (B, S), generator=gb, device=dev)
    w = torch.ones((B, S), device=dev)
    w[torch.rand((B, S), generator=gb, device=dev) > 0.75] = 5.0
    q = kernels.gather_weighted_avg_l2(table, E, hist, w)
    kernels.l2norm_rows(q, E, _lib.TT_NORM_ADD_EPS, out=q)
    names = a.libs.split(",")
    libs = []
    for p in names:
        L = ctypes.CDLL(os.path.abspath(p), mode=os.RTLD_LOCAL | os.RTLD_NOW)
        L.tt_scan_topk_bf16f32.restype = ctypes.c_int
        L.tt_scan_topk_bf16f32.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
            ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
            ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        if a.i8:
            L.tt_scan_topk_bf16f32_i8s.restype = ctypes.c_int
            L.tt_scan_topk_bf16f32_i8s.argtypes = [
                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_float,
                ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.tt_filter_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
        need = ctypes.c_int64(0)
        assert L.tt_filter_workspace_bytes(N, E, B, K, ctypes.byref(need)) == 0
        ws = torch.empty(need.value, dtype=torch.uint8, device=dev)
        out = (torch.empty((B, K), device=dev), torch.empty((B, K), device=dev, dtype=torch.int64))
        libs.append((os.path.basename(p), L, ws, out))
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for e in ev:
        e.record(stream)

    def run(L, ws, out, timed):
        if timed:
            ev[2].record(stream)
        evs = (ev[0].cuda_event if timed else None, ev[1].cuda_event if timed else None)
        if a.i8:
            rc = L.tt_scan_topk_bf16f32_i8s(
                x.data_ptr(), x16.data_ptr(), img[0].data_ptr(), img[1].data_ptr(), N, E,
                x.stride(0), img[0].stride(0), 0, q.data_ptr(), B, q.stride(0), K, bnd[0],
                bnd[1], out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(), ws.numel(),
                stream.cuda_stream, *evs)
        else:
            rc = L.tt_scan_topk_bf16f32(x.data_ptr(), x16.data_ptr(), N, E, x.stride(0), 0,
                                        q.data_ptr(), B, q.stride(0), K, bnd[0], bnd[1],
                                        out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(),
                                        ws.numel(), stream.cuda_stream, *evs)
        assert rc == 0, rc
        if timed:
            ev[3].record(stream)

    for name, L, ws, out in libs:
        for _ in range(2):
            run(L, ws, out, False)
    torch.cuda.synchronize()
    res = {name: {"full": [], "total": []} for name, *_ in libs}
    for r in range(a.reps):
        order = libs[r % len(libs):] + libs[:r % len(libs)]
        for name, L, ws, out in order:
            torch.cuda.synchronize()
            run(L, ws, out, True)
            torch.cuda.synchronize()
            res[name]["full"].append(ev[0].elapsed_time(ev[1]))
            res[name]["total"].append(ev[2].elapsed_time(ev[3]))
    ref = libs[0][3]
    same = {name: bool(torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]))
            for name, _, _, out in libs}
    summ = {}
    for name in res:
        f, t = statistics.median(res[name]["full"]), statistics.median(res[name]["total"])
        summ[name] = {"full_ms": round(f, 4), "total_ms": round(t, 4),
                      "rest_ms": round(t - f, 4), "same_results": same[name],
                      "full_min": round(min(res[name]["full"]), 4)}
    print(json.dumps({"config": f"{N} x {E}, nq {B}, k {K}", "reps": a.reps, "variants": summ},
                     indent=1))


if __name__ == "__main__":
    main()
