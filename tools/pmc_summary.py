"""Per-kernel summary of a rocprofv3 --pmc counter_collection CSV (one row per dispatch and
counter): for every kernel name, the dispatch count, the mean duration and the mean of each
counter per dispatch.  Replaces the raw per-dispatch dump in profiles/ (the raw
CSVs ran to 56k lines).

    python tools/pmc_summary.py <counter_collection.csv> [out.csv]
"""
import collections
import csv
import sys


def summarize(path):
    disp = collections.defaultdict(dict)  # (kernel, dispatch) -> counters
    dur = {}
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per_kernel = collections.defaultdict(list)
    for (k, d), c in disp.items():
        per_kernel[k].append((dur[(k, d)], c))
    rows = []
    counters = sorted({n for c in disp.values() for n in c})
    for k, lst in per_kernel.items():
        row = {"kernel": k, "dispatches": len(lst),
               "mean_duration_us": sum(x[0] for x in lst) / len(lst)}
        for n in counters:
            vals = [x[1][n] for x in lst if n in x[1]]
            row[n] = sum(vals) / len(vals) if vals else ""
        rows.append(row)
    rows.sort(key=lambda r: -r["mean_duration_us"] * r["dispatches"])
    return rows, ["kernel", "dispatches", "mean_duration_us"] + counters


def main(path, out=None):
    rows, cols = summarize(path)
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.DictWriter(f, fieldnames=cols)
    w.writeheader()
    for r in rows:
        w.writerow(r)


if __name__ == "__main__":
    main(*sys.argv[1:])
