"""One rank of a sharded BFS (launched by tests/test_dist.py or by hand via
torchrun).

Every rank uses GPU `--device` (several ranks may share one GPU with the gloo
host transport), makes its Checker a shard (rmc_shard through rmc.dist.shard)
of a golden config (`--case`) or a TLC model (`--cfg`), runs the BFS inside
librmc, and rank 0 writes the global result plus per-rank stats as JSON."""
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
    ap.add_argument("--transport", default="auto", help="rccl | host | auto (rccl on nccl)")
    ap.add_argument("--device", type=int, default=-1, help="-1: LOCAL_RANK")
    ap.add_argument("--keys-per-dest", type=int, default=1 << 18)
    ap.add_argument("--capacity", type=int, default=0)
    ap.add_argument("--rerun", type=int, default=1)
    ap.add_argument("--sent-cache", type=int, default=1 << 22, help="sent-cache slots per rank")
    ap.add_argument("--verify", action="store_true", help="full-state verification (RMC_FLAG_VERIFY_STATES)")
    ap.add_argument("--fp-bits", type=int, default=64, help="verification test hook: fingerprint bits kept")
    ap.add_argument("--max-depth", type=int, default=-1, help="override the case's depth bound")
    ap.add_argument("--checkpoint", help="after the run, write each rank's part (rmc_checkpoint)")
    ap.add_argument("--recover", help="before the run, load each rank's part (rmc_recover)")
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
                              state_capacity=args.capacity or max(1 << 20, g["distinct"]),
                              verify_states=args.verify)
    else:
        cfg = rmc.config_from_files(args.cfg, builtin_raft=True)
        cfg.device = dev
        cfg.state_capacity = args.capacity or (1 << 26)
        if args.verify:
            cfg.flags |= rmc.FLAG_VERIFY_STATES
    if args.max_depth >= 0:
        cfg.max_depth = args.max_depth
    with rmc.Checker(cfg) as ck:
        info = rdist.shard(ck, transport=args.transport, keys_per_dest=args.keys_per_dest,
                           sent_cache_slots=args.sent_cache)
        if args.fp_bits < 64:
            ck.set_fp_bits(args.fp_bits)
        if args.recover:
            ck.recover(args.recover)
        t0 = time.time()
        r = ck.run()  # collective: the global result on every rank
        wall = time.time() - t0
        levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
        trace = ck.trace() if (r.violated_inv or r.deadlock) else []
        if trace:  # identical on every rank (gathered step by step)
            mine = [[f, i, bytes(v).hex()] for f, i, v in trace]
            allt = [None] * world
            dist.all_gather_object(allt, mine)
            assert all(t == mine for t in allt), "ranks disagree on the trace"
        if args.checkpoint:
            ck.checkpoint(args.checkpoint)
        reruns = [ck.run() for _ in range(args.rerun)]
        fields = ("distinct", "generated", "depth", "left_on_queue", "violated_inv", "violation_depth",
                  "collisions", "verified")
        summary = {k: getattr(r, k) for k in fields}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, dict(rank=rank, stored=r.stored_here, keys_sent=r.keys_sent,
                                              states_sent=r.states_sent, chunks=r.chunks, parked=r.parked,
                                              summary=summary, exchange_s=r.exchange_seconds,
                                              wait_s=r.exchange_wait_seconds))
    if rank == 0:
        json.dump(dict(summary, levels=levels, keys_sent=sum(p["keys_sent"] for p in per_rank),
                       parked=sum(p["parked"] for p in per_rank),
                       states_sent=sum(p["states_sent"] for p in per_rank), per_rank=per_rank,
                       wall_s=wall, transport=info.transport,
                       trace=[[f, i, bytes(v).hex()] for f, i, v in trace],
                       owner_mode=os.environ.get("RMC_OWNER", "2"),
                       rerun=[[x.distinct, x.generated, x.depth] for x in reruns]),
                  open(args.out, "w"))
    dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # noqa: BLE001 — a failed rank exits at once: a collective
        # still pending in the process group must not keep it alive
        sys.stderr.write(f"dist_worker rank {os.environ.get('RANK')}: {type(e).__name__}: {e}\n")
        sys.stderr.flush()
        os._exit(1)
