"""Summarise rocprofv3 --pmc CSV passes (counter_collection.csv) into one JSON
per kernel: counter totals, dispatches, and per-dispatch means.

    python tools/pmc_summary.py OUT.json DIR [DIR ...]

Each DIR is one rocprofv3 -d output directory (one pass, its own counters).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    res = {}
    for k, cs in agg.items():
        res[k] = {c: {"total": v, "dispatches": len(disp[k][c]), "per_dispatch": v / max(1, len(disp[k][c]))}
                  for c, v in sorted(cs.items())}
    json.dump({"sources": dirs, "kernels": res}, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
