"""bench.py — distinct states/sec and time-to-fixpoint of the raft.tla BFS
(BASELINE.json metric) on MI355X, one process per GPU.

A "step" is one complete breadth-first search of the bounded MCraft model to
its fixpoint (time-to-fixpoint); `value` = distinct states / seconds per step.
The workload is deterministic: no random inputs exist for an exhaustive BFS.
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
    ap.add_argument("--capacity", type=int, default=1_500_000_000,
                    help="state capacity per GPU (0 = auto from free HBM)")
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


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    cfg = rmc.config_from_files(a.config)
    cfg.device = local if world > 1 else 0
    cfg.state_capacity = a.capacity
    W = rmc.native().rmc_state_bytes(cfg)
    # roofline ceiling of the fingerprint set: random 8-B probes over 64 GB
    r_max = None
    if not a.no_probe_ceiling:
        r_max = rmc.probe_bench(device=cfg.device, table_bytes=64 << 30, accesses=1 << 32, mode=0)

    def barrier():
        if dist is not None:
            dist.barrier()

    with rmc.Checker(cfg) as ck:
        for _ in range(a.warmup):
            ck.run()
        barrier()
        t0 = time.perf_counter()
        kern = 0.0
        launches = 0
        for _ in range(a.steps):
            res = ck.run()
            kern += res.expand_kernel_seconds
            launches += res.expand_launches
        barrier()
        dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    per_step = dt / a.steps
    G, D, NP = res.generated, res.distinct, res.probes
    # algorithmic bytes per run (DESIGN.md "Roofline"): one random 64-B granule
    # per fingerprint probe + the new state written, read back as frontier,
    # its 8-B parent pointer and 8-B fingerprint
    b_alg = NP * 64 + D * (2 * W + 16)
    ks = kern / a.steps
    achieved = b_alg / ks / 1e9 if ks > 0 else 0.0
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
            "distinct": D, "generated": G, "depth": res.depth,
            "time_to_fixpoint_s": per_step, "state_bytes": W,
            "parallelism": f"fp-sharded x{world}" if world > 1 else "single GPU",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "kernel": "k_expand", "kernel_ms_per_step": kern / a.steps * 1e3,
            "launches_per_step": launches // a.steps,
            "alg_bytes_per_step": b_alg,
            "probes_per_step": NP,
            "probe_rate_per_s": NP / ks if ks > 0 else 0.0,
            "probe_ceiling_per_s": r_max,
            "frac_of_probe_ceiling": (NP / ks / r_max) if (ks > 0 and r_max) else None,
        },
    }
    if rank == 0 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_levels)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
