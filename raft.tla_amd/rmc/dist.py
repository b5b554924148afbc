"""Sharded BFS over several GPUs, one process per GPU (rmc_shard in rmc.h).

The BFS loop, the two-phase fingerprint-first exchange and the level
statistics all run inside librmc (rmc_run_bfs on a sharded ctx).  This module
only sets the ctx up, in one of two ways:
  * RCCL (production, one GPU per rank): rank 0 asks librmc for an RCCL id,
    torch.distributed broadcasts it, every rank calls rmc_shard with it, and
    librmc's own communicator moves the data over xGMI;
  * a host transport (tests, rehearsal): librmc calls back into Python for
    each all-to-all / all-gather, which torch.distributed performs with the
    "gloo" backend on CPU tensors, so several ranks can share one GPU.
Replaces TLC's distributed mode (partitioned FPSet).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from datetime import timedelta

import torch
import torch.distributed as dist

from . import ALLGATHER_FN, ALLTOALLV_FN, Checker, Transport


def dist_timeout_s() -> float:
    """The sharded search's deadline for one collective (RMC_DIST_TIMEOUT_S,
    the same variable librmc reads for its RCCL waits; default 300 s)."""
    try:
        return max(0.1, float(os.environ.get("RMC_DIST_TIMEOUT_S", "300")))
    except ValueError:
        return 300.0


class GlooTransport:
    """rmc_transport over torch.distributed (a backend that moves CPU tensors:
    gloo).  Keep the object alive while the ctx uses it.  Every collective
    waits at most dist_timeout_s(); past it the callback fails, librmc reports
    where (level, round, phase) and the run stops instead of hanging."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.errors = []
        self.timeout = timedelta(seconds=dist_timeout_s())

        def finish(work):
            if not work.wait(self.timeout):
                raise TimeoutError(f"collective not complete within {self.timeout.total_seconds()} s")

        def alltoallv(_user, send, send_bytes, recv, recv_bytes):
            try:
                sb = [int(send_bytes[i]) for i in range(self.world)]
                rb = [int(recv_bytes[i]) for i in range(self.world)]
                src = torch.empty(sum(sb), dtype=torch.uint8)
                if sum(sb):
                    C.memmove(src.data_ptr(), send, sum(sb))
                out = torch.empty(sum(rb), dtype=torch.uint8)
                finish(dist.all_to_all_single(out, src, output_split_sizes=rb, input_split_sizes=sb,
                                              group=self.group, async_op=True))
                if sum(rb):
                    C.memmove(recv, out.data_ptr(), sum(rb))
                return 0
            except Exception as e:  # noqa: BLE001 — reported to librmc as a failed collective
                self.errors.append(repr(e))
                return 1

        def allgather(_user, send, nbytes, recv):
            try:
                n = int(nbytes)
                mine = torch.empty(n, dtype=torch.uint8)
                C.memmove(mine.data_ptr(), send, n)
                parts = [torch.empty(n, dtype=torch.uint8) for _ in range(self.world)]
                finish(dist.all_gather(parts, mine, group=self.group, async_op=True))
                for r, p in enumerate(parts):
                    C.memmove(recv + r * n, p.data_ptr(), n)
                return 0
            except Exception as e:  # noqa: BLE001
                self.errors.append(repr(e))
                return 1

        self._fns = (ALLTOALLV_FN(alltoallv), ALLGATHER_FN(allgather))
        self.struct = Transport(None, self._fns[0], self._fns[1])


@dataclass
class ShardInfo:
    rank: int
    world: int
    transport: str


def shard(ck: Checker, group=None, transport: str = "auto", keys_per_dest: int = 0,
          sent_cache_slots: int = 0) -> ShardInfo:
    """Collective: make every rank's Checker one shard of a world-size BFS;
    then ck.run() / ck.result() / ck.trace() are collectives returning the
    global result.  transport "rccl" (librmc's own RCCL communicator; the
    group only carries the 128-byte id), "host" (GlooTransport) or "auto"
    (rccl when the group's backend is nccl)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    backend = dist.get_backend(group)
    if transport == "auto":
        transport = "rccl" if backend == "nccl" else "host"
    if transport == "rccl":
        from . import rccl_unique_id
        idt = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            idt = torch.frombuffer(bytearray(rccl_unique_id()), dtype=torch.uint8).clone()
        if backend == "nccl":
            idt = idt.cuda(ck.cfg.device)
        dist.broadcast(idt, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        ck.shard(rank, world, rccl_id=bytes(idt.cpu().numpy().tobytes()),
                 keys_per_dest=keys_per_dest, sent_cache_slots=sent_cache_slots)
    else:
        t = GlooTransport(group)
        ck.shard(rank, world, transport=t, keys_per_dest=keys_per_dest, sent_cache_slots=sent_cache_slots)
    return ShardInfo(rank, world, transport)
