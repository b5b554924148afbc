"""Cost model of the sharded BFS at N GPUs, from measurements
made on one GPU:

  levels.jsonl   per-level times of the unsharded BFS (tools/level_times.py)
  rounds.err     RMC_DIST_DEBUG log of the same model sharded over N ranks
                 (gloo, ranks sharing one GPU, RMC_DIST_REP=0 so every level
                 runs the exchange rounds) — rounds per level, keys per round
                 and owner, states received, states expanded per rank
  per_rank.json  dist_worker output of that run (stored states per rank)

Per level L of global frontier F_L:
  replicated (F_L <= rep_max; librmc's replicated levels): every rank expands
      the whole level, probing only what it owns —
        f + (t1[L] - f) * (a_lane + (1 - a_lane) / N)
      plus the level's record all-gather (F_L * RBR bytes, (N-1)/N of it
      received over min(N-1, 7) xGMI links), one pack launch, the gather and
      the counter all-gather (2 collectives) and one read-back;
  sharded: every rank r —
        expand  f + (t1[L] - f) * share[L, r] * k_dist   (share: the rank's
                states of the level; f: the fixed cost of a level)
        insert  keys_in[L, r] * c_probe                  (owner-side probes)
        bytes   (8 + 1) B per key + RB per accepted state over the links
      plus R[L] rounds of (2 read-backs + 4 collectives + 5 launches) and the
      level end (a_level: counter all-gather + read-back);
T_N = sum over levels of the slowest rank, against T_1 = sum_L t1[L].
Level 1's t1 holds the fingerprint set's clearing (a memset of the whole
table), which shrinks with the per-rank table: it is charged as
t1[1] * table_rank / table_1.

    python tools/dist_cost_model.py levels.jsonl rounds.err per_rank.json N [rep_max ...] [--k-dist K]

k_dist: the sharded expansion kernel's time per state against the unsharded
kernel's (1.0 assumes the same rate; the one-rank bench measures it).
"""
import collections
import json
import re
import sys


def load(lv_path, log_path, pr_path):
    t1, frontier, total1 = {}, {}, 0.0
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
    return t1, frontier, total1, rounds, keys_in, states, pr


def model(t1, frontier, total1, rounds, keys_in, states, pr, n, rep_max, lat, k_dist=1.0, a_lane=0.55,
          link_bw=50e9, c_probe=1 / 30e9, table_frac=None, RB=56, RBR=64, overlap=False):
    """overlap: a level of R >= 2 rounds runs round k's exchange — owner inserts,
    xGMI bytes and its host round trips (count read-back, reply read-back,
    collectives, launches), on the exchange stream while the host waits — under
    round k + 1's expansion, which librmc queues before it waits (two outbox
    sets): the level takes f + e_r + (R - 1) max(e_r, x_r + L_r) + x_r + L_r +
    a_level with e_r, x_r its per-round expansion and exchange and L_r one
    round's latencies, i.e. only the last round's exchange and latency are
    exposed when a round's exchange fits under the next expansion (the "stall"
    part is what does not fit); without overlap (the default) every exchange and
    every round's latency is charged in full, serially."""
    a_sync, a_coll, a_launch, a_level = lat
    accept = pr["states_sent"] / max(1, pr["keys_sent"])  # phase-2 states per phase-1 key
    f_level = min(t1.values())
    links = min(n - 1, 7) if n > 1 else 1
    parts = collections.Counter()
    n_rep = 0
    for L, t in sorted(t1.items()):
        tl = t
        if L == 1 and table_frac is not None:  # the table memset shrinks with the per-rank table
            tl = f_level + (t - f_level) * table_frac
        F = frontier.get(L, 0)
        if F <= rep_max:
            n_rep += 1
            e = f_level + max(0.0, tl - f_level) * (a_lane + (1 - a_lane) / n)
            x = F * RBR * (n - 1) / n / (link_bw * links) if n > 1 else 0.0
            lat_l = a_launch + 2 * a_coll + a_sync
            parts["expand"] += e
            parts["xgmi"] += x
            parts["latency"] += lat_l
            continue
        R = max(1, len(rounds.get(L, ())))
        per_rank = []
        for r in range(n):
            st = states[L][r] if states[L] else None
            share = (st / max(1, sum(states[L].values()))) if st is not None else 1.0 / n
            e = f_level + max(0.0, tl - f_level) * share * k_dist
            ins = keys_in[L][r] * c_probe
            byts = keys_in[L][r] * (KEYB + 1) + accept * keys_in[L][r] * RB  # key record + reply byte
            x = byts / (link_bw * links) if n > 1 else 0.0
            per_rank.append((e, ins, x))
        e, ins, x = max(per_rank, key=lambda v: sum(v))
        l_round = 2 * a_sync + 4 * a_coll + 5 * a_launch
        if overlap and R >= 2:
            er, xr = max(0.0, e - f_level) / R, (ins + x) / R
            parts["expand"] += e
            parts["insert"] += ins / R
            parts["xgmi"] += x / R
            parts["stall"] += (R - 1) * max(0.0, xr + l_round - er)
            parts["latency"] += l_round + a_level
            continue
        parts["expand"] += e
        parts["insert"] += ins
        parts["xgmi"] += x
        parts["latency"] += R * l_round + a_level
    tot = sum(parts.values())
    return {"N": n, "rep_max": rep_max, "replicated_levels": n_rep, "k_dist": k_dist, "a_lane": a_lane,
            "a_sync_us": a_sync * 1e6, "a_coll_us": a_coll * 1e6, "a_launch_us": a_launch * 1e6,
            "a_level_us": a_level * 1e6, "T_N_ms": tot * 1e3, "speedup": total1 / tot if tot else None,
            **{k + "_ms": v * 1e3 for k, v in parts.items()}}


LATENCIES = ((10e-6, 15e-6, 5e-6, 40e-6), (20e-6, 30e-6, 8e-6, 80e-6), (40e-6, 60e-6, 10e-6, 150e-6))
KEYB = 12  # bytes per phase-1 key record: the raw 96-bit fingerprint {k lo, k hi, s32} (rmc_dist.cpp, round 6)


def main():
    args = sys.argv[1:]
    k_dist = 1.0
    if "--k-dist" in args:
        i = args.index("--k-dist")
        k_dist = float(args[i + 1])
        del args[i:i + 2]
    lv_path, log_path, pr_path, n = args[0], args[1], args[2], int(args[3])
    reps = [int(x) for x in args[4:]] or [0, 1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22]
    data = load(lv_path, log_path, pr_path)
    t1, frontier, total1, rounds, keys_in, states, pr = data
    stored = [p["stored"] for p in pr["per_rank"]]
    # per-rank table: pow2 >= 2 x capacity, doubled for send markers; bench.py sizes
    # capacity = 1.5e9 / N * 1.3 (N > 1) against 1.5e9 at N = 1
    def slots(cap):
        s = 1
        while s < 2 * cap:
            s <<= 1
        return s
    table_frac = (2 * slots(1.5e9 / n * 1.3) if n > 1 else slots(1.5e9)) / slots(1.5e9)
    print(json.dumps({"levels": len(t1), "T1_s": total1, "sum_t1": sum(t1.values()),
                      "rounds_total": sum(len(v) for v in rounds.values()),
                      "imbalance_stored": max(stored) / (sum(stored) / len(stored)),
                      "keys_in_total": sum(sum(v.values()) for v in keys_in.values()),
                      "accepted_per_key": pr["states_sent"] / max(1, pr["keys_sent"]),
                      "f_level_us": min(t1.values()) * 1e6, "table_frac_level1": table_frac}))
    for rep in reps:
        for lat in LATENCIES:
            print(json.dumps(model(*data, n=n, rep_max=rep, lat=lat, k_dist=k_dist, table_frac=table_frac)))


if __name__ == "__main__":
    main()
