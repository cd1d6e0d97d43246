#!/usr/bin/env python
"""Instruction mix of a kernel's loops from hipcc -S output (diagnostic).

    python tools/isa_loop_stats.py file.s kernel_substring

Prints, per loop (labels marked "Loop Header" by LLVM), the count of MFMA, VALU, SALU,
LDS, VMEM and waitcnt instructions between the header label and the backward branch.
"""
import re
import sys
from collections import Counter


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, kname):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^\S*{kname}\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end]
    for i, l in enumerate(body):
        if "Loop Header" in l and l.startswith(".LBB"):
            label = l.split(":")[0]
            js = [k for k in range(i + 1, len(body)) if re.search(rf"s_c?branch\S*\s+{re.escape(label)}\b", body[k])]
            j = js[-1] if js else None
            if j is None:
                continue
            c = Counter()
            for x in body[i:j + 1]:
                x = x.strip()
                if not x or x.startswith((";", ".")):
                    continue
                c[classify(x)] += 1
            print(label, dict(c))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
