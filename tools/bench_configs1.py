"""bench.py's configs[1] leg alone (x3 / bf16 / f32 encoders + top-100 per batch of 256).

    python tools/bench_configs1.py [--texts 100000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--texts", type=int, default=100_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = bench.configs1(argparse.Namespace(configs1_texts=a.texts), dev, 0)
    keep = {p: {k: out[p][k] for k in ("texts_per_s", "texts_per_s_one_stream",
                                        "texts_per_s_two_streams", "encode_ms_per_batch",
                                        "ms_per_batch")} for p in ("x3", "bf16", "f32")}
    keep["x3_api_chunks"] = out["x3_api_chunks"]["texts_per_s"]
    print(json.dumps(keep))


if __name__ == "__main__":
    main()
