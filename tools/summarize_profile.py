#!/usr/bin/env python
"""Summarise rocprofv3 output (kernel stats + FETCH_SIZE / WRITE_SIZE PMC passes).

    python tools/summarize_profile.py gpurun_out > profiles/rNN_<name>.md

HBM bytes per dispatch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so the
read side is doubled (x2); WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import collections
import csv
import os
import sys


def main(d):
    stats = os.path.join(d, "prof", "run_kernel_stats.csv")
    print(f"# rocprofv3 summary ({d})\n")
    if os.path.exists(stats):
        print("## kernel-trace --stats\n")
        print("| kernel | calls | avg us | min us | max us | % time |")
        print("|---|---|---|---|---|---|")
        for r in list(csv.DictReader(open(stats)))[:15]:
            print(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                  f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | "
                  f"{float(r['Percentage']):.2f} |")
    for pmc, corr in (("pmc_fetch", 2.0), ("pmc_write", 1.0)):
        f = os.path.join(d, pmc, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[(r["Kernel_Name"][:90], r["Counter_Name"])].append((float(r["Counter_Value"]), dur))
        print(f"\n## {pmc} (per dispatch; bytes = KiB x 1024 x {corr:g})\n")
        print("| kernel | counter | dispatches | raw KiB avg | corrected GB / dispatch | GB/s (profiled dur) |")
        print("|---|---|---|---|---|---|")
        for (k, c), v in sorted(agg.items(), key=lambda kv: -max(x for x, _ in kv[1])):
            raw = sum(x for x, _ in v) / len(v)
            gb = raw * 1024 * corr / 1e9
            dur = sum(t for _, t in v) / len(v)
            print(f"| `{k}` | {c} | {len(v)} | {raw:.0f} | {gb:.4f} | {gb / (dur * 1e-6):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
