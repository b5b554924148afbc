"""bench.py — distinct states/sec and time-to-fixpoint of the raft.tla BFS
(BASELINE.json metric) on MI355X, one process per GPU.

A "step" is one complete breadth-first search of the bounded MCraft model to
its fixpoint (time-to-fixpoint); `value` = distinct states / seconds per step,
whole job.  The workload is deterministic: an exhaustive BFS has no input data.
With N > 1 ranks the state space is sharded over the GPUs inside librmc
(rmc_shard: owner-routed successors, fingerprint-first two-phase exchange
over librmc's own RCCL communicator) and the SAME model is searched, so
scaling is strong.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))

import rmc  # noqa: E402

METRIC = "distinct states/sec (whole node) and time-to-fixpoint on MCraft BFS, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=os.path.join(ROOT, "specs", "MCraftBench.cfg"))
    ap.add_argument("--capacity", type=int, default=0,
                    help="state capacity per GPU (0 = 1.5e9 / world * 1.3 for the bench model)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (rehearsal)")
    ap.add_argument("--device", type=int, default=-1, help="-1: LOCAL_RANK (one GPU per rank)")
    ap.add_argument("--keys-per-dest", type=int, default=1 << 25,
                    help="sharded mode: phase-1 keys one chunk may send one owner")
    ap.add_argument("--sent-cache", type=int, default=1 << 30,
                    help="sharded mode: slots of the per-rank cache of fingerprints already sent")
    ap.add_argument("--transport", default="auto", help="sharded mode: rccl | host | auto")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the sharded path even at one rank (measures its overhead)")
    ap.add_argument("--no-probe-ceiling", action="store_true",
                    help="skip the random-probe microbenchmark (roofline ceiling)")
    ap.add_argument("--cpu-levels", type=int, default=22,
                    help="BFS levels of the same model timed on the host CPU oracle")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def cpu_baseline(cfg, levels):
    """C oracle (test infrastructure, kind "port") on a bounded sample of the
    same model: its first `levels` BFS levels, on the host's cores."""
    from tests import oracle_c
    threads = max(1, min(16, os.cpu_count() or 1))
    r, _ln, _lg = oracle_c.bfs(cfg.n_servers, cfg.n_values, cfg.max_term, cfg.max_log_len,
                               cfg.max_msgs, cfg.max_dup, bug=int(bool(cfg.flags & rmc.FLAG_BUG_QUORUM)),
                               inv=cfg.invariants, sym=int(bool(cfg.flags & rmc.FLAG_SYMMETRY)),
                               threads=threads, max_levels=levels, capacity=1 << 27)
    return {"value": r.distinct / r.seconds, "unit": "distinct states/s", "cores": threads,
            "kind": "port",
            "sample": f"C oracle (oracle/rmc_oracle.c, exact state set) BFS levels 1..{r.depth} of the "
                      f"same model: {r.distinct} distinct / {r.generated} generated in {r.seconds:.2f} s"}


def pmc_traffic(config_path):
    """HBM bytes per k_expand launch from the committed rocprofv3 PMC profile
    of this same command (profiles/<round>/pmc_traffic_<cfg>.json): PMC
    counters cannot be read live inside the timed run."""
    stem = os.path.splitext(os.path.basename(config_path))[0]
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    for rnd in sorted(os.listdir(pdir), reverse=True):
        pf = os.path.join(pdir, rnd, f"pmc_traffic_{stem}.json")
        if os.path.exists(pf):
            return json.load(open(pf))["hbm_bytes_per_launch"], os.path.relpath(pf, ROOT)
    return None, None


def main():
    a = parse()
    # The JSON line is the only thing on stdout: libraries that print banners
    # there (RCCL prints its version block at communicator init) are sent to
    # stderr by pointing fd 1 at fd 2 for the rest of the run.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    sharded = world > 1 or a.force_dist
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        import torch
        import torch.distributed as dist
        dev = a.device if a.device >= 0 else local
        torch.cuda.set_device(dev)
        dist.init_process_group(a.dist_backend, init_method="env://")
    # the GPU box has no raft.tla: the bench model checks the compiled-in lemmy/raft.tla
    cfg = rmc.config_from_files(a.config, builtin_raft=True)
    cfg.device = (a.device if a.device >= 0 else local) if sharded else max(a.device, 0)
    cfg.state_capacity = a.capacity or int(1.5e9 / world * (1.3 if sharded else 1.0))
    W = rmc.native().rmc_state_bytes(cfg)
    # roofline ceiling of the fingerprint set: random 8-B probes over 64 GB
    r_max = None
    if not a.no_probe_ceiling and world == 1:
        r_max = rmc.probe_bench(device=cfg.device, table_bytes=64 << 30, accesses=1 << 32, mode=0)

    def barrier():
        if dist is not None:
            dist.barrier()

    last = [None]
    transport_used = [None]  # sharded: "rccl" (librmc's communicator) or "host" (gloo)

    def one_run(ck, first):
        # sharded: rmc_run_bfs is a collective inside librmc (two-phase
        # exchange over its own RCCL communicator); the result is global
        r = ck.run()
        last[0] = r
        return r.distinct, r.generated, r.depth, r.probes, r.expand_kernel_seconds, r.expand_launches

    with rmc.Checker(cfg) as ck:
        if sharded:
            from rmc import dist as rdist
            info = rdist.shard(ck, transport=a.transport, keys_per_dest=a.keys_per_dest,
                               sent_cache_slots=a.sent_cache)
            transport_used[0] = info.transport
        first = True
        for _ in range(a.warmup):
            one_run(ck, first)
            first = False
        barrier()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        kern = 0.0
        launches = 0
        for _ in range(a.steps):
            D, G, depth, NP, ks, nl = one_run(ck, first)
            first = False
            kern += ks
            launches += nl
        barrier()
        dt = time.perf_counter() - t0
        salt_check = None
        if not sharded:  # untimed: same search under another fingerprint salt
            ck.set_seed(0x5A17ED)
            r2 = ck.run()
            ck.set_seed(0)
            salt_check = {"salt": 0x5A17ED, "distinct": r2.distinct, "generated": r2.generated,
                          "depth": r2.depth,
                          "agrees": (r2.distinct, r2.generated, r2.depth) == (D, G, depth)}
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    per_step = dt / a.steps
    # algorithmic bytes per run (DESIGN.md "Roofline"): one random 64-B granule
    # per fingerprint probe + the new state written, read back as frontier,
    # its 8-B parent pointer and 8-B fingerprint
    b_alg = NP * 64 + D * (2 * W + 16)
    ks = kern / a.steps
    nlaunch = max(1, launches // a.steps)
    achieved = b_alg / ks / 1e9 if ks > 0 else 0.0
    traffic, tsrc = pmc_traffic(a.config) if not sharded else (None, None)
    out = {
        "metric": METRIC,
        "value": D / per_step,
        "unit": "distinct states/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": per_step * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (exhaustive BFS of a deterministic bounded model; no input data)",
        "config": {
            "workload": os.path.basename(a.config) + f": raft.tla, {cfg.n_servers} servers, "
                        f"{cfg.n_values} values, CONSTRAINT MaxTerm={cfg.max_term} MaxLogLen="
                        f"{cfg.max_log_len} MaxMsgs={cfg.max_msgs} MaxDup={cfg.max_dup}, BFS to fixpoint",
            "distinct": D, "generated": G, "depth": depth,
            "time_to_fixpoint_s": per_step, "state_bytes": W,
            "parallelism": (f"state-space sharded x{world} (librmc two-phase exchange, "
                            f"{'RCCL' if transport_used[0] == 'rccl' else 'host transport over gloo'})")
                           if sharded else "single GPU",
            "fp_salt_crosscheck": salt_check,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
            "kernel": "k_expand_sort (librmc's default expansion kernel, RMC_EXPAND_VARIANT 6)",
            "kernel_ms_per_step": ks * 1e3,
            "launches_per_step": nlaunch, "alg_bytes_per_launch": b_alg / nlaunch,
            "alg_bytes_per_step": b_alg, "probes_per_step": NP,
            "probe_rate_per_s": NP / ks if ks > 0 else 0.0,
            "probe_ceiling_per_s": r_max,
            "frac_of_probe_ceiling": (NP / ks / r_max) if (ks > 0 and r_max) else None,
        },
    }
    if sharded:
        ld = last[0]
        out["sharded"] = {"in_library": "rmc_shard + rmc_run_bfs (two-phase fingerprint-first exchange)",
                          "transport": transport_used[0], "chunks_rank0": ld.chunks, "keys_sent_rank0": ld.keys_sent,
                          "states_sent_rank0": ld.states_sent, "stored_rank0": ld.stored_here,
                          "exchange_s_rank0": round(ld.exchange_seconds, 6), "keys_per_dest": a.keys_per_dest}
        out["roofline"]["note"] = "per-rank kernel time of rank 0; achieved is rank 0's share"
        out["roofline"]["achieved"] = (b_alg / world) / ks / 1e9 if ks > 0 else 0.0
        out["roofline"]["frac"] = out["roofline"]["achieved"] / HBM_PEAK_GBS
    if rank == 0 and not a.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_levels)
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
