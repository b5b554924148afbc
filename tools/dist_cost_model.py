"""Cost model of the sharded BFS at N GPUs, from measurements
made on one GPU:

  levels.jsonl   per-level times of the unsharded BFS (tools/level_times.py)
  rounds.err     RMC_DIST_DEBUG log of the same model sharded over N ranks
                 (gloo, ranks sharing one GPU: tools/gpu/r03d.sh) — rounds per
                 level, keys per round and owner, states received
  per_rank.json  dist_worker output of that run (stored states per rank)

Per level L, every rank r:
  expand   f + (t1[L] - f) * share[L, r] * k_dist  (share: the rank's states of
                                                 the level; f: the fixed cost of a
                                                 level, the smallest t1; k_dist:
                                                 sharded / unsharded kernel time)
  insert   keys_in[L, r] * c_probe              (owner-side random probes)
  rounds   R[L] * (2 * a_sync + 4 * a_coll + 5 * a_launch)
  bytes    (8 + 1) B per key + RB per state, over min(N-1, 7) xGMI links
  level    a_level (all-gather of the counters + read-back)
and T_N = sum_L max_r(expand + insert + bytes) + rounds + level, against
T_1 = sum_L t1[L].  The latencies are parameters (defaults: the assumptions
stated in DESIGN.md); the script prints T_N and the speed-up for a grid of
them.

    python tools/dist_cost_model.py levels.jsonl rounds.err per_rank.json N
"""
import collections
import json
import re
import sys


def main():
    lv_path, log_path, pr_path, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    t1 = {}
    frontier = {}
    total1 = 0.0
    for ln in open(lv_path):
        d = json.loads(ln)
        if "level" in d:
            t1[d["level"]] = d["seconds"]
            frontier[d["level"]] = d["frontier"]
        else:
            total1 = d["seconds"]
    pat = re.compile(r"\[rmc rank (\d+)\] level (\d+) round (\d+) kind (\d) states (\d+): most keys to one owner "
                     r"(\d+) \(cap (\d+)\), parked (\d+)/(\d+), in (\d+), rho")
    rounds = collections.defaultdict(set)
    keys_in = collections.defaultdict(lambda: collections.defaultdict(int))
    states = collections.defaultdict(lambda: collections.defaultdict(int))
    for ln in open(log_path):
        m = pat.search(ln)
        if not m:
            continue
        r, lvl, k, kind, st, mx, cap, pd, pk, tin = (int(x) for x in m.groups())
        rounds[lvl].add(k)
        keys_in[lvl][r] += tin
        states[lvl][r] += st
    pr = json.load(open(pr_path))
    accept = pr["states_sent"] / max(1, pr["keys_sent"])  # phase-2 states per phase-1 key
    stored = [p["stored"] for p in pr["per_rank"]]
    imb = max(stored) / (sum(stored) / len(stored))
    RB = 56
    # fixed per-level cost on one GPU: the smallest level time (a few thousand states)
    f_level = min(t1.values())
    print(json.dumps({"levels": len(t1), "T1_s": total1, "sum_t1": sum(t1.values()), "rounds_total":
                      sum(len(v) for v in rounds.values()), "imbalance_stored": imb,
                      "keys_in_total": sum(sum(v.values()) for v in keys_in.values()),
                      "accepted_per_key": accept, "f_level_us": f_level * 1e6}))
    for k_dist in (1.0, 1.06):
        for a_sync, a_coll, a_launch, a_level in ((10e-6, 15e-6, 5e-6, 40e-6), (20e-6, 30e-6, 8e-6, 80e-6),
                                                  (40e-6, 60e-6, 10e-6, 150e-6)):
            for c_probe in (1 / 30e9,):
                link_bw = 50e9
                tot = 0.0
                parts = collections.Counter()
                for L, t in t1.items():
                    R = max(1, len(rounds.get(L, ())))
                    per_rank = []
                    for r in range(n):
                        # the expansion share of rank r: its states of this level (when logged) else 1/N;
                        # a level's fixed cost (launch + read-back, f_level) does not shrink with N
                        st = states[L][r] if states[L] else None
                        share = (st / max(1, sum(states[L].values()))) if st is not None else 1.0 / n
                        e = f_level + max(0.0, t - f_level) * share * k_dist
                        ins = keys_in[L][r] * c_probe
                        byts = keys_in[L][r] * 9 + accept * keys_in[L][r] * RB
                        x = byts / (link_bw * min(n - 1, 7))
                        per_rank.append((e, ins, x))
                    e, ins, x = max(per_rank, key=lambda v: sum(v))
                    lat = R * (2 * a_sync + 4 * a_coll + 5 * a_launch) + a_level
                    parts["expand"] += e
                    parts["insert"] += ins
                    parts["xgmi"] += x
                    parts["latency"] += lat
                    tot += e + ins + x + lat
                print(json.dumps({"N": n, "k_dist": k_dist, "a_sync_us": a_sync * 1e6, "a_coll_us": a_coll * 1e6,
                                  "a_launch_us": a_launch * 1e6, "a_level_us": a_level * 1e6,
                                  "T_N_ms": tot * 1e3, "speedup": total1 / tot if tot else None,
                                  **{k + "_ms": v * 1e3 for k, v in parts.items()}}))


if __name__ == "__main__":
    main()
