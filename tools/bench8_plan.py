"""Plan of the 8-GPU bench model specs/MCraftBench8.cfg (MCraftBench with
MaxMsgs 4): its size, the per-rank memory plan and the
cost-model time at N GPUs.  Measurement tool; the model exceeds one GPU, so
its tail is extrapolated from what one GPU can measure:

  prefix_levels.jsonl  tools/level_times.py specs/MCraftBench8.cfg CAP DEPTH on one GPU
                       (per-level frontier, new states, generated, seconds)
  prefix_rounds.txt    RMC_DIST_DEBUG log of the same prefix sharded over N ranks
                       (tools/gpu/dist8.sh CFG=specs/MCraftBench8.cfg DEPTH=...)
  prefix_dist8.json    dist_worker output of that run
  shape_levels.jsonl   per-level counts of a model that reaches its fixpoint on
                       one GPU (MCraftBench): the decline of the per-level growth
                       ratio past the prefix is taken from it, matched at the
                       prefix's last ratio and stretched by 1.0 / 1.15 / 1.3 (the
                       MaxMsgs-4 ratios fall 0.9-0.95x as fast as MaxMsgs 3's)

Per extrapolated level: t1 = f + frontier * tau (tau: seconds per frontier
state over the prefix's last 3 levels), keys to owners = frontier * kappa
(kappa: keys sent per expanded state over the prefix's last 3 levels, from
the rehearsal), rounds = ceil(frontier / N / min(2^25, kcap / rho)) with rho =
kappa / N keys per state to one owner (librmc's round sizing, rmc_dist.cpp).

    python tools/bench8_plan.py prefix_levels.jsonl prefix_rounds.txt prefix_dist8.json shape_levels.jsonl [N]
        [--sizing profiles/r03/sizing_next_bounds.txt] [--k-dist K] [--measured full_levels.jsonl]

--measured: the whole model's per-level times on one GPU (tools/level_times.py of a
model one GPU completes, e.g. specs/MCraftBenchXL.cfg with spill): T1 and the
frontiers past the rehearsed prefix are then measured, not extrapolated — only the
per-rank keys and states of those levels come from the prefix's last 3 levels
(shape_levels is then unused).

--sizing: per-level new-state counts of a longer depth-bounded run of the same
model (tools/sizing.py) extend the measured prefix before the tail is
extrapolated (counts only; the time per state is the prefix's).
"""
import re
import collections
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dist_cost_model as dcm  # noqa: E402

HBM = 288e9          # bytes per MI355X
STATE_B = 40         # rmc_state_bytes(MCraftBench8) (packed: 3 server words + 4 bag slots)
PER_STATE = STATE_B + 8 + 1 + 8 + 1   # state, parent ref, lane, footprint, class (rmc_api.cpp)


def news(path):
    out = {}
    for ln in open(path):
        d = json.loads(ln)
        if "level" in d:
            out[d["level"]] = d
    return out


def extrapolate(prefix_new, shape_new, stretch):
    """prefix_new[i]: new states of level i (0 = Init); the tail follows the
    shape's growth ratios from where they equal the prefix's last ratio."""
    r_shape = [shape_new[i + 1] / shape_new[i] for i in range(len(shape_new) - 1) if shape_new[i]]
    last = prefix_new[-1] / prefix_new[-2]
    start = min(range(len(r_shape) - 1), key=lambda i: abs(r_shape[i] - last) + (1e9 if r_shape[i] > 1.6 else 0))
    x = list(prefix_new)
    k = start + 1.0 / stretch
    while True:
        i = int(k)
        if i + 1 >= len(r_shape):
            break
        f = k - i
        r = r_shape[i] * (1 - f) + r_shape[i + 1] * f
        x.append(x[-1] * r)
        if x[-1] < 1:
            break
        k += 1.0 / stretch
    return [int(v) for v in x]


SPLIT = 4  # rmc_dist.cpp D.split at world > 1 (RMC_DIST_SPLIT)


def slots_for(cap):
    s = 1
    while s < 2 * cap:
        s <<= 1
    return s


def memory_plan(n, distinct):
    """librmc's own sizing (bench.py passes capacity 0 for this model): the
    store gets budget / (PER_STATE + 32) states, budget = 0.8 x free HBM; the
    fingerprint set pow2 >= 2 x capacity slots of 8 B (the 2x growth for send
    markers is skipped when it does not fit); rmc_shard's exchange buffers."""
    budget = 0.8 * (HBM - 2e9)  # ~2 GB taken by the runtime and RCCL before rmc_create
    cap = int(budget / (PER_STATE + 32))
    slots = slots_for(cap)
    store = cap * PER_STATE
    table = slots * 8
    free_after = HBM - 2e9 - store - table
    grown = free_after > table * 2 + 16e9
    kcap = min(1 << 25, max(1 << 20, (1 << 26) // n))
    rb, rbr = STATE_B + 16, STATE_B + 24
    xbuf = (2 * (n * kcap * 16 + 8 * n) + n * kcap * 8 + 2 * n * kcap + 2 * n * kcap * rb +
            max(n * kcap, 1 << 20) * 16 + 2 * (1 << 20) * rbr + (1 << 24) * 2)
    need = distinct / n * 1.07  # the rehearsal's stored-state imbalance (max/mean)
    return {"N": n, "capacity_per_rank": cap, "states_needed_per_rank_max": int(need),
            "fits": need <= cap, "store_GB": store / 1e9, "table_slots": slots, "table_GB": table / 1e9,
            "table_grown_for_markers": grown, "exchange_buffers_GB": xbuf / 1e9,
            "total_GB": (store + table * (2 if grown else 1) + xbuf) / 1e9 + 2.0,
            "table_load_at_fixpoint": need / slots, "kcap": kcap}


def main():
    args = sys.argv[1:]
    sizing = None
    k_dist = 1.0  # the sharded kernel's time per state against the unsharded kernel's
    if "--k-dist" in args:
        k = args.index("--k-dist")
        k_dist = float(args[k + 1])
        del args[k:k + 2]
    if "--sizing" in args:
        k = args.index("--sizing")
        sizing = args[k + 1]
        del args[k:k + 2]
    table_frac = None  # the per-rank fingerprint set's share of the one-GPU set's bytes (level 1's memset)
    if "--table-frac" in args:
        k = args.index("--table-frac")
        table_frac = float(args[k + 1])
        del args[k:k + 2]
    rep_max = 1 << 20  # librmc's RMC_DIST_REP default
    if "--rep-max" in args:
        k = args.index("--rep-max")
        rep_max = int(args[k + 1])
        del args[k:k + 2]
    measured = None
    if "--measured" in args:
        k = args.index("--measured")
        measured = news(args[k + 1])
        del args[k:k + 2]
    lv, rounds_p, pr_p, shape_p = args[:4]
    n = int(args[4]) if len(args) > 4 else 8
    t1, frontier, total1, rounds, keys_in, states, pr = dcm.load(lv, rounds_p, pr_p)
    pl = news(lv)
    depth_p = max(pl)
    prefix_new = [1] + [pl[i]["new"] for i in range(1, depth_p + 1)]
    if sizing:  # "<model> level L distinct D new N" lines (level L's new states = new[L])
        ext = {}
        for ln in open(sizing):
            mm = re.search(r"3:2:2:1:4:1:\S* level (\d+) distinct (\d+) new (\d+)", ln)
            if mm:
                ext[int(mm.group(1))] = int(mm.group(3))
        for L in sorted(ext):
            if L == len(prefix_new):
                prefix_new.append(ext[L])
            elif L < len(prefix_new):
                assert prefix_new[L] == ext[L], (L, prefix_new[L], ext[L])
    sl = news(shape_p)
    shape_new = [1] + [sl[i]["new"] for i in sorted(sl)]
    f = min(t1.values())
    last3 = [L for L in sorted(t1) if L > depth_p - 3]
    tau = sum(t1[L] - f for L in last3) / sum(frontier[L] for L in last3)
    gen_per = sum(pl[L]["generated"] for L in last3) / sum(frontier[L] for L in last3)
    kappa = sum(sum(keys_in[L].values()) for L in last3) / sum(frontier[L] for L in last3)
    share = [sum(states[L][r] for L in last3) / max(1, sum(sum(states[L].values()) for L in last3))
             for r in range(n)]
    kshare = [sum(keys_in[L][r] for L in last3) / max(1, sum(sum(keys_in[L].values()) for L in last3))
              for r in range(n)]
    print(json.dumps({"prefix_depth": depth_p, "counted_levels": len(prefix_new) - 1,
                      "counted_distinct": sum(prefix_new), "f_level_us": f * 1e6,
                      "tau_ns_per_frontier_state": tau * 1e9, "generated_per_frontier_state": gen_per,
                      "keys_per_expanded_state": kappa, "rank_state_share_max": max(share)}))
    kcap = min(1 << 25, max(1 << 20, (1 << 26) // n))
    if measured:  # the whole model's counts (level L's new states) from the one-GPU run
        full_m = [1] + [measured[i]["new"] for i in sorted(measured)]
        full_m = full_m[:max(i for i, v in enumerate(full_m) if v) + 1]
    for stretch in ((None,) if measured else (1.0, 1.15, 1.3)):
        full = full_m if measured else extrapolate(prefix_new, shape_new, stretch)
        distinct = sum(full)
        T1 = dict(t1)
        Fr = dict(frontier)
        Ki = collections.defaultdict(lambda: collections.defaultdict(int))
        St = collections.defaultdict(lambda: collections.defaultdict(int))
        Ro = collections.defaultdict(set)
        for L in t1:
            Ki[L].update(keys_in[L])
            St[L].update(states[L])
            Ro[L] = set(rounds[L])
        for L in range(depth_p + 1, len(full)):
            F = full[L - 1]  # level L expands the states found at level L - 1
            T1[L] = measured[L]["seconds"] if measured else f + F * tau
            Fr[L] = F
            Ki[L].update({r: F * kappa * kshare[r] for r in range(n)})
            St[L].update({r: F * share[r] for r in range(n)})
            rho = kappa / n
            per_round = min(1 << 25, kcap / max(rho, 0.02))
            # librmc: at world > 1 a level of >= 2^21 states in its frontier takes at
            # least D.split rounds (4 since round 6), so each round's exchange
            # overlaps the next round's expansion
            split = SPLIT if (n > 1 and F / n >= (1 << 21)) else 1
            Ro[L] = set(range(max(split, math.ceil(F / n / per_round))))
        if measured:  # the prefix levels too: this model's own one-GPU run (same build as the tail)
            for L in t1:
                if L in measured:
                    T1[L] = measured[L]["seconds"]
        tot1 = sum(T1.values())
        row = {"stretch": stretch, "k_dist": k_dist, "depth": len(full) - 1, "distinct_est": distinct,
               "generated_est": (int(sum(measured[L]["generated"] for L in measured)) + 1 if measured else int(
                   sum(pl[L]["generated"] for L in pl) + sum(full[L - 1] * gen_per for L in range(depth_p + 1, len(full))))),
               "T1_model_s": tot1, "peak_level_new": max(full)}
        row["memory"] = memory_plan(n, distinct)
        for lat in dcm.LATENCIES:
            m = dcm.model(T1, Fr, tot1, Ro, Ki, St, pr, n=n, rep_max=rep_max, lat=lat, k_dist=k_dist,
                          table_frac=table_frac)
            for part in ("expand_ms", "insert_ms", "xgmi_ms", "latency_ms"):
                row.setdefault(part, []).append(round(m.get(part, 0.0), 1))
            mo = dcm.model(T1, Fr, tot1, Ro, Ki, St, pr, n=n, rep_max=rep_max, lat=lat, k_dist=k_dist,
                           table_frac=table_frac, overlap=True)
            row.setdefault("T_N_ms_overlapped", []).append(round(mo["T_N_ms"], 1))
            for part in ("insert_ms", "xgmi_ms", "stall_ms", "latency_ms"):
                row.setdefault("overlapped_" + part, []).append(round(mo.get(part, 0.0), 1))
            row.setdefault("speedup_overlapped", []).append(round(mo["speedup"], 2))
            row.setdefault("T_N_ms", []).append(round(m["T_N_ms"], 1))
            row.setdefault("speedup", []).append(round(m["speedup"], 2))
            row.setdefault("rate_G_per_s", []).append(round(distinct / m["T_N_ms"] / 1e6, 2))
        print(json.dumps(row))


if __name__ == "__main__":
    main()
