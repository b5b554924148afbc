"""Summary of one tools/gpu/pmc.sh run (rocprofv3 kernel trace + PMC passes of
`bench.py --steps 1`) into the committed profile files bench.py reads:

  profiles/<round>/pmc_traffic_<cfg>.json   HBM bytes per expansion launch
                                            (FETCH_SIZE + WRITE_SIZE, KiB)
  profiles/<round>/pmc_counters_<cfg>.json  instruction mix, waits, LDS
  profiles/<round>/kernel_stats_<cfg>.csv   rocprofv3 --stats of the kernel trace

    python tools/pmc_summary.py <pmc.sh OUT dir> <profiles/<round>> [cfg stem]
"""
import csv
import glob
import json
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1:3]
    stem = sys.argv[3] if len(sys.argv) > 3 else "MCraftBench"
    os.makedirs(dst, exist_ok=True)
    tot = {}
    for ln in open(os.path.join(src, "totals.jsonl")):
        d = json.loads(ln)
        for k, v in d["kernels"].items():
            for cn, x in v.items():
                tot.setdefault(k, {})[cn] = x
    stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    kavg = {}
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"kernel_stats_{stem}.csv"))
        for row in csv.DictReader(open(stats[0])):
            ns = "AverageNs" in row
            kavg[row["Name"].split("(")[0]] = {
                "calls": int(row["Calls"]),
                "avg_us": float(row["AverageNs"]) / 1e3 if ns else float(row["AverageUs"]),
                "total_ms": float(row["TotalDurationNs"]) / 1e6 if ns else float(row["TotalDurationUs"]) / 1e3,
                "pct": float(row["Percentage"])}
    kname = os.environ.get("PMC_KERNEL", "k_expand_sort")  # k_expand_dist for the sharded path
    exp = [k for k in tot if kname in k and "true, false" not in k.split("<")[-1][:20]]
    if not exp:
        sys.exit("no " + kname + " counters in " + src)
    k = exp[0]
    c = tot[k]
    n = c["FETCH_SIZE"]["launches"]
    hbm = (c["FETCH_SIZE"]["total"] + c["WRITE_SIZE"]["total"]) * 1024.0
    wo = [x for x in tot if "k_window_order" in x]
    wo_b = ((tot[wo[0]]["FETCH_SIZE"]["total"] + tot[wo[0]]["WRITE_SIZE"]["total"]) * 1024.0
            if wo and "FETCH_SIZE" in tot[wo[0]] else None)
    kt = next((v for kk, v in kavg.items() if kname in kk and "<3, 4, 8, true" not in kk), None)
    traffic = {
        "command": "tools/gpu/pmc.sh: rocprofv3 --kernel-trace --stats, then one --pmc pass per counter group "
                   "(FETCH_SIZE | WRITE_SIZE | SQ instruction mix | SQ waits | LDS | TCC atomics) -- python3 bench.py "
                   "--steps 1 --warmup 0 --no-cpu --no-probe-ceiling --v2-config=; per-kernel totals by "
                   "tools/pmc_totals.py",
        "workload": os.environ.get("PMC_WORKLOAD",
                                   f"specs/{stem}.cfg, BFS to fixpoint (bench step + the untimed fingerprint-salt re-run)"),
        "kernel": k,
        "pmc_launches": n,
        "fetch_size_kb_total": c["FETCH_SIZE"]["total"],
        "write_size_kb_total": c["WRITE_SIZE"]["total"],
        "hbm_bytes_total": hbm,
        "hbm_bytes_per_launch": hbm / n,
        "k_window_order_hbm_bytes_per_launch": (wo_b / n) if wo_b is not None else None,
        "kernel_avg_us_rocprofv3": kt["avg_us"] if kt else None,
        "note": "FETCH_SIZE/WRITE_SIZE in KiB. The accesses are 8-B random probes (one 64-B granule each), CAS and "
                "40-B state stores, not 16-B/lane streams, so the gfx950 2x FETCH_SIZE correction for wide streaming "
                "reads (MI355X_MICROARCH.md, HBM) is not applied.",
    }
    json.dump(traffic, open(os.path.join(dst, f"pmc_traffic_{stem}.json"), "w"), indent=1)
    g = lambda name: c[name]["total"] if name in c else None  # noqa: E731
    counters = {"kernel": k, "launches": n, "totals": {cn: x["total"] for cn, x in c.items()}}
    if g("SQ_INSTS_VALU") and g("SQ_INSTS_SALU"):
        counters["salu_per_valu"] = g("SQ_INSTS_SALU") / g("SQ_INSTS_VALU")
    if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
        counters["wait_any_per_wave_cycle"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        counters["lds_bank_conflict_per_idx_active"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    counters["kernel_trace"] = kavg
    counters["all_kernels"] = tot
    json.dump(counters, open(os.path.join(dst, f"pmc_counters_{stem}.json"), "w"), indent=1)
    if g("TCC_EA0_ATOMIC_sum") is not None:  # the atomics pass: per BFS, against the inserts it makes
        nbfs = int(os.environ.get("PMC_BFS", "2"))  # bench.py --steps 1: the step + the salt re-run
        distinct = None
        bj = os.path.join(src, "kt.json")
        if os.path.exists(bj):
            try:
                distinct = json.load(open(bj))["config"]["distinct"]
            except (ValueError, KeyError):
                pass
        ea, l2 = g("TCC_EA0_ATOMIC_sum"), g("TCC_ATOMIC_sum")
        lvl = g("TCC_EA0_ATOMIC_LEVEL_sum")
        ksec = kt["total_ms"] / 1e3 / nbfs if kt else None  # the kernel trace ran the same command
        atom = {"kernel": k, "launches": n, "bfs_per_profile": nbfs,
                "tcc_atomic_per_bfs": l2 / nbfs if l2 is not None else None,
                "tcc_ea0_atomic_per_bfs": ea / nbfs,
                "ea_atomic_avg_latency_cycles": (lvl / ea) if (lvl and ea) else None,
                "distinct_states": distinct,
                "atomics_per_insert": (ea / nbfs / distinct) if distinct else None,
                "kernel_seconds_per_bfs": ksec,
                "ea_atomics_per_s": (ea / nbfs / ksec) if ksec else None,
                "note": "TCC_ATOMIC: atomic requests at the L2 (all types); TCC_EA0_ATOMIC: those that go on "
                        "to memory; every new state is one CAS of its key into the fingerprint set (plus lost CAS "
                        "races, linear-probe CASes and the per-wave counters)"}
        json.dump(atom, open(os.path.join(dst, f"pmc_atomics_{stem}.json"), "w"), indent=1)
    print(json.dumps({"hbm_bytes_per_launch": hbm / n, "launches": n, "kernel_avg_us": kt["avg_us"] if kt else None,
                      "salu_per_valu": counters.get("salu_per_valu"),
                      "wait_any_per_wave_cycle": counters.get("wait_any_per_wave_cycle")}))


if __name__ == "__main__":
    main()
