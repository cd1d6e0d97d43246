#!/usr/bin/env python
"""profiles/traffic.json from two rocprofv3 counter passes (tools/final_prof.sh):

    python tools/make_traffic_json.py gpurun_out/pmc_fetch gpurun_out/pmc_write "build label"

HBM bytes per dispatch, averaged over the profiled dispatches of each kernel:
FETCH_SIZE (KiB) x 1024 x 2 -- on gfx950 FETCH_SIZE reports half the bytes of a wide streaming
read (MI355X_MICROARCH.md, HBM / rocprofv3 section) -- and WRITE_SIZE (KiB) x 1024.  Both
count Infinity-Cache (MALL) hits as traffic.  bench.py reads the roofline kernel's entry."""
import collections
import csv
import glob
import json
import os
import re
import sys

CONFIG = "1M x 384 catalog, 10k queries, k=100"


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            k = re.sub(r"^void\s+", "", r["Kernel_Name"]).split("(")[0].replace("tt::", "")
            vals[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main(fetch_dir, write_dir, label):
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    out = {"source": f"{label}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py "
                     "--no-cpu-baseline --no-extra --mode-a-buyers 0 --steps 2 (tools/final_prof.sh)",
           "note": "HBM bytes per dispatch (avg over the profiled dispatches): FETCH_SIZE x 1024 x 2 "
                   "(gfx950 correction) and WRITE_SIZE x 1024",
           "kernels": {}}
    for k in sorted(set(f) & set(w), key=lambda k: -f[k]):
        out["kernels"][k] = {"fetch_bytes": f[k] * 1024 * 2, "write_bytes": w[k] * 1024,
                             "config": CONFIG}
    json.dump(out, open(os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json"),
                        "w"), indent=1)
    for k, v in out["kernels"].items():
        print(f"{k:40s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "final build")
