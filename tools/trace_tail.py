#!/usr/bin/env python
"""Print the last N kernels of a rocprofv3 kernel trace (start offset, duration, grid)."""
import csv
import re
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("tt::", "")[:44]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{name:46s} start {s / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f} us  grid {r['Grid_Size_X']}")
