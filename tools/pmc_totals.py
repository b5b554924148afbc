"""Per-kernel totals of one rocprofv3 --pmc pass, as one JSON line, then the
pass's database is deleted (GPU-side summaries keep gpurun_out/ small).

    python tools/pmc_totals.py <rocprofv3 -d dir> <label> >> out.jsonl
"""
import glob
import json
import os
import shutil
import sqlite3
import sys


def main():
    d, label = sys.argv[1:3]
    files = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    out = {"label": label, "kernels": {}}
    for f in files:
        db = sqlite3.connect(f)
        for name, cname, total, n in db.execute(
                "select kernel_name, counter_name, sum(value), count(value) from counters_collection "
                "group by kernel_name, counter_name").fetchall():
            if not any(k in name for k in ("k_expand", "k_window_order", "k_owner", "k_store", "k_materialize")):
                continue
            k = out["kernels"].setdefault(name.split("(")[0], {})
            k[cname] = {"total": total, "launches": n}
        db.close()
    print(json.dumps(out))
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
