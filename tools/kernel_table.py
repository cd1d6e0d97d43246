"""Per-kernel average durations from a rocprofv3 kernel-trace CSV (short names, call counts).

    python tools/kernel_table.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def short(k):
    k = re.sub(r"^void\s+", "", k).split("(")[0]
    return k.replace("tt::", "")


def main(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in d.values())
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:60]:60s} calls={len(v):5d} avg_us={sum(v)/len(v):9.1f} "
              f"min={min(v):8.1f} max={max(v):8.1f} share={sum(v)/tot:6.1%}")


if __name__ == "__main__":
    main(sys.argv[1])
