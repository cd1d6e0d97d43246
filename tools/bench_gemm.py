"""Microbenchmark of tt_gemm_bf16 / tt_gemm_f32 at the encoder's shapes.

    python tools/bench_gemm.py [--prec bf16] [--M 18340]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

import torch  # noqa: E402

from twotower import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="bf16")
    ap.add_argument("--M", type=int, default=18340)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None, help="N,K,act,res of one shape (e.g. 1152,384,0,0)")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--no-ln", action="store_true")
    a = ap.parse_args()
    L = _lib.lib()
    dt = torch.bfloat16 if a.prec == "bf16" else torch.float32
    fn = L.tt_gemm_bf16 if a.prec == "bf16" else L.tt_gemm_f32
    out = {}
    shapes = [(1152, 384, 0, False), (384, 384, 0, True), (1536, 384, 1, False),
              (384, 1536, 0, True)]
    if a.only:
        n_, k_, act_, res_ = (int(v) for v in a.only.split(","))
        shapes = [(n_, k_, act_, bool(res_))]
    for (N, K, act, res) in shapes:
        A = torch.randn(a.M, K, device="cuda").to(dt)
        W = torch.randn(N, K, device="cuda").to(dt)
        b = torch.randn(N, device="cuda")
        R = torch.randn(a.M, N, device="cuda") if res else None
        # the encoder's outputs: f32 (+residual) for Wo / W2, bf16 only for QKV / W1 (bf16 path)
        C = torch.empty(a.M, N, device="cuda") if (res or a.prec != "bf16") else None
        C16 = torch.empty(a.M, N, device="cuda", dtype=torch.bfloat16) if C is None else None

        def run():
            _lib.check(fn(A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(),
                          R.data_ptr() if res else None, N,
                          C.data_ptr() if C is not None else None, N,
                          C16.data_ptr() if C16 is not None else None, N, a.M, N, K,
                          act, _lib.stream_ptr()), "gemm")
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        # library reference point (hipBLASLt through torch): same shape, bf16/f32 in and out
        bb = b.to(dt)
        if a.no_torch:
            out[f"N{N}_K{K}"] = {"us": round(ms * 1e3, 1),
                                 "tflops": round(2 * a.M * N * K / ms / 1e9, 1)}
            continue
        for _ in range(3):
            torch.nn.functional.linear(A, W, bb)
        e0.record()
        for _ in range(a.iters):
            torch.nn.functional.linear(A, W, bb)
        e1.record()
        torch.cuda.synchronize()
        ms_t = e0.elapsed_time(e1) / a.iters
        out[f"N{N}_K{K}"] = {"us": round(ms * 1e3, 1), "tflops": round(2 * a.M * N * K / ms / 1e9, 1),
                             "torch_tflops": round(2 * a.M * N * K / ms_t / 1e9, 1)}
    if a.prec == "bf16" and not a.no_ln:  # fused GEMM + LayerNorm (Wo / W2 of a layer), in place
        for K in (384, 1536):
            A = torch.randn(a.M, K, device="cuda").to(dt)
            W = (torch.randn(384, K, device="cuda") / K ** 0.5).to(dt)
            b, gm, bt = (torch.randn(384, device="cuda") for _ in range(3))
            X = torch.randn(a.M, 384, device="cuda")
            X16 = torch.empty(a.M, 384, device="cuda", dtype=dt)

            def run_ln():
                _lib.check(L.tt_gemm_ln_bf16(A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(),
                                             gm.data_ptr(), bt.data_ptr(), 1e-12, X.data_ptr(), 384,
                                             X16.data_ptr(), 384, a.M, 384, K, _lib.stream_ptr()),
                           "gemm_ln")
            for _ in range(3):
                run_ln()
            e0.record()
            for _ in range(a.iters):
                run_ln()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            byts = a.M * (2 * K + 384 * 10)
            out[f"LN_N384_K{K}"] = {"us": round(ms * 1e3, 1),
                                    "tflops": round(2 * a.M * 384 * K / ms / 1e9, 1),
                                    "hbm_gbps": round(byts / ms / 1e6, 1)}
    print(json.dumps({"prec": a.prec, "M": a.M, **out}))


if __name__ == "__main__":
    main()
