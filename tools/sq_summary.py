"""Summarise tools/exp_sq.sh output: SQ counters of the full-catalog filter launch per variant.

    python tools/sq_summary.py [gpurun_out] [kernel_substring]
"""
import collections
import csv
import glob
import os
import sys


def main(d="gpurun_out", kern="k_filter_ring<384, 1>"):
    res = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "sq_lib_*_*/run_counter_collection.csv"))):
        var = os.path.basename(os.path.dirname(f))[len("sq_lib_"):].rsplit("_", 1)[0]
        best = {}
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            best.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
            best[r["Dispatch_Id"]]["dur_ms"] = dur
        if best:
            last = best[sorted(best, key=int)[-1]]
            res[var].update(last)
    keys = sorted({k for v in res.values() for k in v})
    vars_ = sorted(res)
    print("| counter | " + " | ".join(vars_) + " |")
    print("|---|" + "---|" * len(vars_))
    for k in keys:
        print(f"| {k} | " + " | ".join(f"{res[v].get(k, float('nan')):.4g}" for v in vars_) + " |")


if __name__ == "__main__":
    main(*sys.argv[1:])
