"""Print a bench_i8.py JSON result on one line per lib (helper of the GPU scripts)."""
import json
import sys

d = json.load(open(sys.argv[1]))
parts = []
for q, v in d.items():
    if not q.startswith("nq"):
        continue
    s = f"{q} bf16 {v['bf16']['ms_per_search']:.4f} ({v['bf16']['stream_ms']:.4f})"
    if "i8" in v:
        s += (f" i8 {v['i8']['ms_per_search']:.4f} (stream {v['i8']['stream_ms']:.4f}) "
              f"fb {v['i8']['fallbacks_last']} same {v['i8']['same_as_bf16']}")
    parts.append(s)
print(sys.argv[2], " | ".join(parts))
