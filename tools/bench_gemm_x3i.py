"""GEMM microbenchmark at the encoder's QKV / FFN1 shapes, bf16 and x3i (split-bf16 operands
interleaved per 32 k), for A/B between GEMM variants built with tools/exp_build2.sh (run the
variants alternately, several times).

    python tools/bench_gemm_x3i.py [--M 370761,18340] [--iters 20]
Prints one JSON line: per shape us and TFLOP/s (x3i counted as 3 products).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

import torch  # noqa: E402

from twotower import _lib  # noqa: E402
from twotower.item_tower import x3i_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="370761,18340")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L = _lib.lib()
    out = {"lib": os.environ.get("TWOTOWER_HIP_LIB", "in-tree")}
    for M in (int(v) for v in a.M.split(",")):
        for (kind, N, K, act) in (("bf16", 1152, 384, 0), ("bf16", 1536, 384, 1),
                                  ("x3i", 1152, 384, 0), ("x3i", 1536, 384, 1),
                                  ("x3i_ln", 384, 384, 0), ("x3i_ln", 384, 1536, 0)):
            g = torch.Generator(device="cuda").manual_seed(1)
            Af = torch.randn(M, K, device="cuda", generator=g)
            Wf = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
            b = torch.randn(N, device="cuda", generator=g)
            if kind == "bf16":
                A, W = Af.to(torch.bfloat16), Wf.to(torch.bfloat16)
                C16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

                def run():
                    _lib.check(L.tt_gemm_bf16(A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), None,
                                              0, None, N, C16.data_ptr(), N, M, N, K, act,
                                              _lib.stream_ptr()), "gemm")
                fl = 2.0 * M * N * K
            elif kind == "x3i_ln":  # BertSelfOutput / BertOutput: x = LN(A.W^T + b + x)
                A2, W2 = x3i_weights(Af), x3i_weights(Wf)
                X = torch.randn(M, N, device="cuda", generator=g)
                X2 = torch.empty(M, 2 * N, device="cuda", dtype=torch.bfloat16)
                gm = torch.rand(N, device="cuda", generator=g) + 0.5
                bt = torch.randn(N, device="cuda", generator=g)

                def run():
                    _lib.check(L.tt_gemm_ln_x3i(A2.data_ptr(), 2 * K, W2.data_ptr(), 2 * K,
                                                b.data_ptr(), gm.data_ptr(), bt.data_ptr(), 1e-12,
                                                X.data_ptr(), N, X2.data_ptr(), 2 * N, M, N, K,
                                                _lib.stream_ptr()), "x3i_ln")
                fl = 3 * 2.0 * M * N * K
            else:
                A2, W2 = x3i_weights(Af), x3i_weights(Wf)
                C2 = torch.empty(M, 2 * N, device="cuda", dtype=torch.bfloat16)

                def run():
                    _lib.check(L.tt_gemm_x3i(A2.data_ptr(), 2 * K, W2.data_ptr(), 2 * K,
                                             b.data_ptr(), C2.data_ptr(), 2 * N, M, N, K, act,
                                             _lib.stream_ptr()), "x3i")
                fl = 3 * 2.0 * M * N * K
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            out[f"{kind}_M{M}_N{N}_K{K}_act{act}"] = {"us": round(ms * 1e3, 1),
                                                  "tflops": round(fl / (ms * 1e-3) / 1e12, 1)}
            del Af, Wf
            torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
