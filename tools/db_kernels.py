"""Per-kernel durations from a rocprofv3 rocpd SQLite database (the default output format).

    python tools/db_kernels.py gpurun_out/<dir>/run_results.db [name-substring]
"""
import collections
import re
import sqlite3
import sys


def main(path, pat=""):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    d = collections.defaultdict(list)
    for k, s, e in c.execute(f"select {name}, start, end from kernels"):
        k = re.sub(r"^void\s+", "", k).split("(")[0].replace("tt::", "")
        if pat in k:
            d[k].append((e - s) / 1e3)
    tot = sum(sum(v) for v in d.values()) or 1.0
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{k[:60]:60s} calls={len(v):5d} avg_us={sum(v)/len(v):9.2f} "
              f"med={v[len(v)//2]:8.2f} min={v[0]:8.2f} max={v[-1]:8.2f} share={sum(v)/tot:6.1%}")


if __name__ == "__main__":
    main(*sys.argv[1:])
