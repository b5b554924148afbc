"""Sharded BFS over several GPUs, one process per GPU (rmc_dist_* in rmc.h).

The HIP library expands each rank's share of the frontier and packs the
successors owned by other ranks into a per-destination outbox; this driver
moves them with torch.distributed (backend "nccl" = RCCL over xGMI on
MI355X, or "gloo" through host memory for tests) and hands the received
records back to the library, which inserts them into the local fingerprint
set.  One all-to-all of counts + one of records per frontier chunk, one
all-reduce of level statistics per BFS level.  Replaces TLC's distributed
mode (partitioned FPSet).
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from . import Checker, RmcError


@dataclass
class DistResult:
    generated: int = 0
    distinct: int = 0
    depth: int = 0
    probes: int = 0
    violated_inv: int = 0
    violation_depth: int = 0
    seconds: float = 0.0
    expand_kernel_seconds: float = 0.0
    records_sent: int = 0
    levels: list = field(default_factory=list)


def exchange(outbox: torch.Tensor, send_counts, group=None):
    """All-to-all of the first send_counts[d] records of outbox[d] to rank d
    (all_to_all_single with split sizes: one RCCL alltoallv).  Returns
    (records received, contiguous in source-rank order; per-source counts).
    On a gloo group the tensors travel through host memory."""
    world = dist.get_world_size(group)
    dev = outbox.device
    cpu = dist.get_backend(group) == "gloo"
    send = [int(x) for x in send_counts]
    sc = torch.tensor(send, dtype=torch.int64)
    rc = torch.empty_like(sc)
    if not cpu:
        sc, rc = sc.to(dev), rc.to(dev)
    dist.all_to_all_single(rc, sc, group=group)
    rc = rc.cpu().tolist()
    rw = outbox.shape[-1]
    flat = torch.cat([outbox[d, :send[d]] for d in range(world)])
    out = torch.empty((sum(rc), rw), dtype=outbox.dtype, device="cpu" if cpu else dev)
    if cpu:
        flat = flat.cpu()
    dist.all_to_all_single(out, flat, output_split_sizes=rc, input_split_sizes=send, group=group)
    if cpu and out.device != dev:
        out = out.to(dev)
    return out, rc


def _allreduce(vals, op, dev, cpu, group):
    t = torch.tensor(vals, dtype=torch.int64, device="cpu" if cpu else dev)
    dist.all_reduce(t, op=op, group=group)
    return t.cpu().tolist()


def run(ck: Checker, chunk_states=1 << 22, cap_per_dest=1 << 22, sent_cache_slots=1 << 26,
        group=None, init=True) -> DistResult:
    """Collective: every rank calls it with its own Checker (one GPU each)."""
    lib, ctx = ck.lib, ck.ctx
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    cpu = dist.get_backend(group) == "gloo"
    dev = torch.device("cuda", ck.cfg.device)

    def chk(rc):
        if rc:
            raise RmcError(rc, lib.rmc_last_error(ctx).decode())

    if init:
        chk(lib.rmc_dist_init(ctx, rank, world, sent_cache_slots))
    rw = lib.rmc_dist_record_words(ctx)
    outbox = torch.empty((world, cap_per_dest, rw), dtype=torch.int32, device=dev)
    res = DistResult()
    t0 = time.perf_counter()
    chk(lib.rmc_dist_start(ctx))
    res.generated = 1  # the initial state
    depth = 1
    send = (C.c_uint64 * world)()
    done = C.c_int32()
    out5 = (C.c_uint64 * 5)()
    while True:
        # ---- expand this level's frontier chunk by chunk, exchanging each chunk
        while True:
            chk(lib.rmc_dist_expand(ctx, chunk_states, C.c_void_p(outbox.data_ptr()), cap_per_dest,
                                    send, C.byref(done)))
            res.records_sent += sum(send)
            received, rc = exchange(outbox, list(send), group)
            if received.shape[0]:
                chk(lib.rmc_dist_insert(ctx, C.c_void_p(received.data_ptr()), received.shape[0]))
            more = _allreduce([0 if done.value else 1], dist.ReduceOp.SUM, dev, cpu, group)[0]
            if more == 0:
                break
        chk(lib.rmc_dist_end_level(ctx, out5))
        new, gen, probes = _allreduce([out5[0], out5[1], out5[2]], dist.ReduceOp.SUM, dev, cpu,
                                      group)
        viol = _allreduce([out5[4]], dist.ReduceOp.MAX, dev, cpu, group)[0]
        res.generated += gen
        res.probes += probes
        res.levels.append(new)
        if new:
            depth += 1
        if viol:
            res.violated_inv = viol
            res.violation_depth = depth
            break
        if new == 0:
            break
    res.seconds = time.perf_counter() - t0
    r = ck.result()
    res.expand_kernel_seconds = r.expand_kernel_seconds
    # distinct = states stored over all ranks (each state lives on its owner only)
    res.distinct = _allreduce([r.distinct], dist.ReduceOp.SUM, dev, cpu, group)[0]
    res.depth = depth
    return res
