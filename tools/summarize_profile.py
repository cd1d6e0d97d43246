#!/usr/bin/env python
"""Summarise rocprofv3 output (kernel stats + FETCH_SIZE / WRITE_SIZE PMC passes).

    python tools/summarize_profile.py gpurun_out > profiles/rNN_<name>.md

HBM bytes per dispatch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so the
read side is doubled (x2); WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import collections
import csv
import json
import os
import re
import sys


def short_name(k):
    """'void tt::k_filter_ring<384, 1>(unsigned short const*, ...)' -> 'k_filter_ring<384, 1>'"""
    k = re.sub(r"^void\s+", "", k)
    k = k.split("(")[0]
    return k.replace("tt::", "")


def main(d, traffic_out=None, config=None, source=None):
    traffic = collections.defaultdict(dict)
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
        full = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[(r["Kernel_Name"][:90], r["Counter_Name"])].append((float(r["Counter_Value"]), dur))
            full[short_name(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in full.items():
            traffic[k]["fetch_bytes" if pmc == "pmc_fetch" else "write_bytes"] = (
                sum(v) / len(v) * 1024 * corr)
        print(f"\n## {pmc} (per dispatch; bytes = KiB x 1024 x {corr:g})\n")
        print("| kernel | counter | dispatches | raw KiB avg | corrected GB / dispatch | GB/s (profiled dur) |")
        print("|---|---|---|---|---|---|")
        for (k, c), v in sorted(agg.items(), key=lambda kv: -max(x for x, _ in kv[1])):
            raw = sum(x for x, _ in v) / len(v)
            gb = raw * 1024 * corr / 1e9
            dur = sum(t for _, t in v) / len(v)
            print(f"| `{k}` | {c} | {len(v)} | {raw:.0f} | {gb:.4f} | {gb / (dur * 1e-6):.1f} |")


    if traffic_out:
        kern = {k: dict(v, config=config) for k, v in traffic.items()
                if "fetch_bytes" in v and "write_bytes" in v and k.startswith("k_")}
        json.dump({"source": source, "note": "HBM bytes per dispatch (avg over the profiled "
                   "dispatches): FETCH_SIZE x 1024 x 2 (gfx950 correction) and WRITE_SIZE x 1024",
                   "kernels": kern}, open(traffic_out, "w"), indent=1)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out")
    ap.add_argument("--traffic", help="write per-kernel HBM bytes per dispatch (JSON)")
    ap.add_argument("--config", default="1M x 384 catalog, 10k queries, k=100")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    main(a.dir, a.traffic, a.config, a.source)
