"""One rank of a sharded BFS (launched by tests/test_dist.py via torchrun).

Every rank uses GPU `--device` (several ranks may share one GPU with the gloo
backend), runs rmc.dist.run on a golden config and rank 0 writes the global
result as JSON."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))

import torch.distributed as dist  # noqa: E402

import rmc  # noqa: E402
from rmc import dist as rdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--device", type=int, default=-1, help="-1: LOCAL_RANK")
    ap.add_argument("--chunk", type=int, default=1 << 16)
    args = ap.parse_args()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_levels.json")))[args.case]
    p = g["params"]
    dist.init_process_group(args.backend, init_method="env://")
    rank = dist.get_rank()
    dev = args.device if args.device >= 0 else int(os.environ.get("LOCAL_RANK", "0"))
    cfg = rmc.make_config(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                          max_log_len=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                          bug_quorum=bool(p["bug_quorum"]), invariants=p["invariants"],
                          device=dev, state_capacity=max(1 << 20, g["distinct"]))
    with rmc.Checker(cfg) as ck:
        r = rdist.run(ck, chunk_states=args.chunk, cap_per_dest=1 << 20, sent_cache_slots=1 << 20)
        r2 = rdist.run(ck, chunk_states=args.chunk, cap_per_dest=1 << 20, init=False)  # re-run
    if rank == 0:
        json.dump(dict(distinct=r.distinct, generated=r.generated, depth=r.depth,
                       levels=r.levels, violated_inv=r.violated_inv,
                       violation_depth=r.violation_depth, records_sent=r.records_sent,
                       rerun=[r2.distinct, r2.generated, r2.depth]), open(args.out, "w"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
