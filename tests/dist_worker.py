"""One rank of a sharded BFS (launched by tests/test_dist.py or by hand via
torchrun).

Every rank uses GPU `--device` (several ranks may share one GPU with the gloo
backend), runs rmc.dist.run on a golden config (`--case`) or a TLC model
(`--cfg`), and rank 0 writes the global result plus per-rank balance stats as
JSON."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))

import torch.distributed as dist  # noqa: E402

import rmc  # noqa: E402
from rmc import dist as rdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case")
    ap.add_argument("--cfg")
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--device", type=int, default=-1, help="-1: LOCAL_RANK")
    ap.add_argument("--chunk", type=int, default=1 << 16)
    ap.add_argument("--cap-per-dest", type=int, default=1 << 20)
    ap.add_argument("--capacity", type=int, default=0)
    ap.add_argument("--rerun", type=int, default=1)
    args = ap.parse_args()
    dev = args.device if args.device >= 0 else int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "nccl":
        import torch
        torch.cuda.set_device(dev)
    dist.init_process_group(args.backend, init_method="env://")
    rank, world = dist.get_rank(), dist.get_world_size()
    if args.case:
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_levels.json")))[args.case]
        p = g["params"]
        cfg = rmc.make_config(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                              max_log_len=p["max_log_len"], max_msgs=p["max_msgs"],
                              max_dup=p["max_dup"], bug_quorum=bool(p["bug_quorum"]),
                              invariants=p["invariants"], device=dev, symmetry=bool(p["symmetry"]),
                              max_depth=p["max_depth"],
                              state_capacity=args.capacity or max(1 << 20, g["distinct"]))
    else:
        cfg = rmc.config_from_files(args.cfg, builtin_raft=True)
        cfg.device = dev
        cfg.state_capacity = args.capacity or (1 << 26)
    with rmc.Checker(cfg) as ck:
        t0 = time.time()
        r = rdist.run(ck, chunk_states=args.chunk, cap_per_dest=args.cap_per_dest,
                      sent_cache_slots=1 << 24)
        wall = time.time() - t0
        local = ck.result()
        reruns = [rdist.run(ck, chunk_states=args.chunk, cap_per_dest=args.cap_per_dest, init=False)
                  for _ in range(args.rerun)]
        # the trace is identical on every rank (it is broadcast step by step)
        if r.trace:
            mine = [[f, i, bytes(v).hex()] for f, i, v in r.trace]
            allt = [None] * world
            dist.all_gather_object(allt, mine)
            assert all(t == mine for t in allt), "ranks disagree on the trace"

    per_rank = [None] * world
    dist.all_gather_object(per_rank, dict(rank=rank, distinct=local.distinct,
                                          records_sent=r.records_sent))
    if rank == 0:
        json.dump(dict(distinct=r.distinct, generated=r.generated, depth=r.depth,
                       left_on_queue=r.left_on_queue,
                       levels=r.levels, violated_inv=r.violated_inv,
                       violation_depth=r.violation_depth, records_sent=r.records_sent,
                       per_rank=per_rank, wall_s=wall,
                       trace=[[f, i, bytes(v).hex()] for f, i, v in r.trace],
                       owner_mode=os.environ.get("RMC_OWNER", "2"),
                       rerun=[[x.distinct, x.generated, x.depth] for x in reruns]),
                  open(args.out, "w"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
