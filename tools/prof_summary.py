"""Summarise the rocprofv3 databases of tools/gpu/prof.sh into profiles/<round>/:

  kernel_stats_<cfg>.csv     per-kernel calls / total / average (kernel-trace pass)
  pmc_traffic_<cfg>.json     HBM bytes per k_expand launch (FETCH_SIZE and
                             WRITE_SIZE passes, one counter per pass)
  pmc_counters_<cfg>.json    every counter of the other passes present
                             (insts / stall / tcc: tools/gpu/prof_r02.sh) for
                             the same kernel, totals and per launch

    python tools/prof_summary.py gpurun_out/prof r01 MCraftBench
"""
import csv
import glob
import json
import os
import sqlite3
import sys


def one_db(d):
    files = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if len(files) != 1:
        raise SystemExit(f"expected one .db under {d}, found {files}")
    return sqlite3.connect(files[0])


def main():
    src, rnd, stem = sys.argv[1:4]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", rnd)
    os.makedirs(out, exist_ok=True)
    kt = one_db(os.path.join(src, "kt"))
    rows = kt.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    with open(os.path.join(out, f"kernel_stats_{stem}.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow(r)
    expand = [r for r in rows if "k_expand" in r[0]]  # k_expand<...>, k_expand_sort<...>
    name, calls, total_us, avg_us, _pct = max(expand, key=lambda r: r[2])

    def counter(db, cname):
        vals = db.execute("select value from counters_collection where counter_name = ? and kernel_name = ?",
                          (cname, name)).fetchall()
        return [v[0] for v in vals]

    fetch = counter(one_db(os.path.join(src, "fetch")), "FETCH_SIZE")
    write = counter(one_db(os.path.join(src, "write")), "WRITE_SIZE")
    n = len(fetch)
    rec = {
        "command": "tools/gpu/prof.sh: rocprofv3 --kernel-trace --stats | --pmc FETCH_SIZE | --pmc WRITE_SIZE "
                   "(separate passes) -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-probe-ceiling",
        "workload": f"specs/{stem}.cfg, BFS to fixpoint (bench step + the untimed fingerprint-salt re-run)",
        "kernel": name,
        "launches": calls,
        "kernel_total_us": total_us,
        "kernel_avg_us": avg_us,
        "pmc_launches": n,
        "fetch_size_kb_total": sum(fetch),
        "write_size_kb_total": sum(write),
        "hbm_bytes_total": (sum(fetch) + sum(write)) * 1024.0,
        "hbm_bytes_per_launch": (sum(fetch) + sum(write)) * 1024.0 / max(1, n),
        "note": "FETCH_SIZE/WRITE_SIZE in KiB. The accesses are 8-B random probes (one 64-B granule each), "
                "CAS and 40-B state stores, not 16-B/lane streams, so the gfx950 2x FETCH_SIZE correction "
                "for wide streaming reads (MI355X_MICROARCH.md, HBM) is not applied.",
    }
    json.dump(rec, open(os.path.join(out, f"pmc_traffic_{stem}.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))
    extra = {}
    for pas in ("insts", "stall", "tcc", "lds"):
        d = os.path.join(src, pas)
        if not os.path.isdir(d):
            continue
        db = one_db(d)
        for (cname,) in db.execute("select distinct counter_name from counters_collection where kernel_name = ?",
                                   (name,)).fetchall():
            v = counter(db, cname)
            extra[cname] = {"pass": pas, "total": sum(v), "launches": len(v), "per_launch": sum(v) / max(1, len(v))}
    if extra:
        json.dump({"kernel": name, "workload": rec["workload"], "counters": extra,
                   "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md)"},
                  open(os.path.join(out, f"pmc_counters_{stem}.json"), "w"), indent=1)
        for k, v in sorted(extra.items()):
            print(f"{k:24s} {v['per_launch']:.4g} per launch")


if __name__ == "__main__":
    main()
