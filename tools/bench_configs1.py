"""configs[1] leg of bench.py with 2 / 3 / 4 batches in flight (bench.configs1, 25.6k texts
per run): x3 texts/s on one stream and on NS streams."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for rep in range(2):
        for ns in (2, 3, 4):
            a = argparse.Namespace(configs1_texts=25_600, configs1_streams=ns)
            r = bench.configs1(a, dev, 0)
            out.setdefault(str(ns), []).append(
                {"x3_two_streams": round(r["x3"]["texts_per_s_two_streams"]),
                 "x3_one_stream": round(r["x3"]["texts_per_s_one_stream"]),
                 "bf16_ns": round(r["bf16"]["texts_per_s_two_streams"])})
            print(ns, out[str(ns)][-1], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
