"""Average PMC counter values per kernel (short name) over rocprofv3 counter-collection CSVs.

    python tools/pmc_table.py gpurun_out/pmc*/run_counter_collection.csv
"""
import collections
import csv
import re
import sys


def short(k):
    return re.sub(r"^void\s+", "", k).split("(")[0].replace("tt::", "")


def main(paths):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"]) + f" grid={r.get('Grid_Size', r.get('Grid_Size_X', ''))}"
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in sorted(vals, key=lambda k: -sum(durs[k])):
        if sum(durs[k]) < 50:
            continue
        print(f"== {k[:80]}  dispatches~{len(durs[k])} avg_us={sum(durs[k]) / len(durs[k]):.1f}")
        for c, v in sorted(vals[k].items()):
            print(f"   {c:28s} {sum(v) / len(v):16.4g}")


if __name__ == "__main__":
    main(sys.argv[1:])
