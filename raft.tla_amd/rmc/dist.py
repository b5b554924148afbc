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

from . import Checker, RmcError, StateView


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
    left_on_queue: int = 0
    records_sent: int = 0
    max_dest_per_state: float = 0.0  # most records for one destination per expanded state
    chunks: int = 0
    levels: list = field(default_factory=list)
    # counterexample on a violation: [(family, lane, StateView)] from Init to the
    # violating state, gathered across ranks (identical on every rank)
    trace: list = field(default_factory=list)
    # host wall time per phase (s): expand (kernel + count readback), exchange
    # (both all-to-alls), insert (kernel + readback), level (end-of-level stats)
    phase: dict = field(default_factory=lambda: dict(expand=0.0, exchange=0.0, insert=0.0, level=0.0))


def exchange_counts(send, more, dev, cpu, group=None):
    """All-to-all of the per-destination record counts.  Per destination d the
    row is [records for d, my `more` flag, my total records]: `more` (this rank
    still has frontier to expand) rides along so the chunk loop needs no extra
    collective to agree on termination, and the totals tell every rank whether
    ANY rank sends, so all skip the payload collective together (a collective
    skipped by some ranks only deadlocks).  Returns (recv counts, flags, any)."""
    sc = torch.tensor([[c, int(bool(more)), sum(send)] for c in send], dtype=torch.int64)
    rc = torch.empty_like(sc)
    if not cpu:
        sc, rc = sc.to(dev), rc.to(dev)
    dist.all_to_all_single(rc, sc, group=group)
    rcl = rc.cpu().tolist()
    return [x[0] for x in rcl], [x[1] for x in rcl], sum(x[2] for x in rcl) > 0


def payload_start(outbox: torch.Tensor, send, recv, cpu, group=None):
    """Start the all-to-all of the first send[d] records of outbox[d] to rank d
    (all_to_all_single with split sizes: one RCCL alltoallv).  On RCCL the
    collective is asynchronous, so the caller can expand the next chunk into
    the other outbox meanwhile.  Returns a handle for payload_finish."""
    world = outbox.shape[0]
    rw = outbox.shape[-1]
    flat = torch.cat([outbox[d, :send[d]] for d in range(world)])
    out = torch.empty((sum(recv), rw), dtype=outbox.dtype, device="cpu" if cpu else outbox.device)
    if cpu:  # gloo: through host memory, synchronously
        dist.all_to_all_single(out, flat.cpu(), output_split_sizes=recv, input_split_sizes=list(send),
                               group=group)
        return (None, out.to(outbox.device), flat)
    work = dist.all_to_all_single(out, flat, output_split_sizes=recv, input_split_sizes=list(send),
                                  group=group, async_op=True)
    return (work, out, flat)


def payload_finish(handle):
    """Wait for payload_start's collective.  On RCCL the received tensor is
    complete on return: the current stream is synchronised, because librmc
    consumes it on its own stream."""
    work, out, _flat = handle
    if work is not None:
        work.wait()
        torch.cuda.current_stream(out.device).synchronize()
    return out


def exchange(outbox: torch.Tensor, send_counts, group=None, more=None):
    """One synchronous exchange (counts, then records); returns (records
    received, contiguous in source-rank order; per-source counts; per-source
    `more` flags).  The BFS loop uses the split, pipelined form."""
    dev = outbox.device
    cpu = dist.get_backend(group) == "gloo"
    send = [int(x) for x in send_counts]
    recv, flags, anyone = exchange_counts(send, True if more is None else more, dev, cpu, group)
    if not anyone:
        return outbox.new_empty((0, outbox.shape[-1])), recv, flags
    return payload_finish(payload_start(outbox, send, recv, cpu, group)), recv, flags


def _allgather(vals, dev, cpu, group):
    """One collective for a rank's small stats vector: returns [world][len]
    (an all-reduce of a zero matrix holding this rank's row: gloo has no
    all_gather_into_tensor)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    t = torch.zeros((world, len(vals)), dtype=torch.int64)
    t[rank] = torch.tensor(vals, dtype=torch.int64)
    if not cpu:
        t = t.to(dev)
    dist.all_reduce(t, group=group)
    return t.cpu().tolist()


def _allreduce(vals, op, dev, cpu, group):
    t = torch.tensor(vals, dtype=torch.int64, device="cpu" if cpu else dev)
    dist.all_reduce(t, op=op, group=group)
    return t.cpu().tolist()


def trace(ck: Checker, rank0: int, index0: int, group=None) -> list:
    """Collective: the chain of parents from state `index0` on rank `rank0`
    back to an initial state.  Each step, the rank holding the current state
    broadcasts it (decoded view, family, lane, parent's global ref); the
    parent ref names the next rank.  Returns [(family, lane, StateView)] in
    behaviour order, on every rank."""
    lib, ctx = ck.lib, ck.ctx
    rank = dist.get_rank(group)
    cpu = dist.get_backend(group) == "gloo"
    dev = torch.device("cuda", ck.cfg.device)
    nb = C.sizeof(StateView)
    hdr = 3  # family, lane, parent ref (int64 each)
    nwords = hdr + (nb + 7) // 8
    chain = []
    owner, idx = rank0, index0
    for _ in range(1 << 16):
        t = torch.zeros(nwords, dtype=torch.int64)
        if rank == owner:
            sv = StateView()
            fam, inst, pref = C.c_int32(), C.c_int32(), C.c_uint64()
            rc = lib.rmc_dist_state(ctx, idx, C.byref(sv), C.byref(fam), C.byref(inst), C.byref(pref))
            if rc:
                raise RmcError(rc, lib.rmc_last_error(ctx).decode())
            t[0], t[1] = fam.value, inst.value
            t[2] = pref.value - (1 << 64) if pref.value >= 1 << 63 else pref.value
            raw = bytearray(nb + (-nb) % 8)
            C.memmove((C.c_char * nb).from_buffer(raw), C.byref(sv), nb)
            t[hdr:] = torch.frombuffer(raw, dtype=torch.int64)
        if not cpu:
            t = t.to(dev)
        dist.broadcast(t, src=dist.get_global_rank(group, owner) if group is not None else owner, group=group)
        t = t.cpu()
        sv = StateView.from_buffer_copy(t[hdr:].numpy().tobytes()[:nb])
        chain.append((int(t[0]), int(t[1]), sv))
        pref = int(t[2]) & 0xFFFFFFFFFFFFFFFF
        if pref == 0xFFFFFFFFFFFFFFFF:
            break
        owner, idx = pref >> 48, pref & ((1 << 48) - 1)
    chain.reverse()
    return chain


def run(ck: Checker, chunk_states=1 << 22, cap_per_dest=1 << 22, sent_cache_slots=1 << 26,
        group=None, init=True, pipeline_chunks=4, min_chunk=1 << 20) -> DistResult:
    """Collective: every rank calls it with its own Checker (one GPU each).
    A level's local frontier is expanded in about `pipeline_chunks` chunks (of
    at least `min_chunk` states, at most `chunk_states`), so the exchange of
    one chunk overlaps the expansion of the next."""
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
    # two outboxes: chunk k+1 is expanded into one while chunk k's records
    # leave from the other (RCCL all-to-all overlapped with k_expand)
    outboxes = [torch.empty((world, cap_per_dest, rw), dtype=torch.int32, device=dev) for _ in range(2)]
    res = DistResult()
    t0 = time.perf_counter()
    chk(lib.rmc_dist_start(ctx))
    res.generated = 1  # the initial state
    depth = 1
    send = (C.c_uint64 * world)()
    done = C.c_int32()
    out5 = (C.c_uint64 * 5)()
    max_depth = ck.cfg.max_depth
    # adaptive chunk (states per expansion): start where even one record per
    # state for one destination fits, then track the observed ratio
    cap_bound = int(min(chunk_states, cap_per_dest // 2))  # outbox-fill bound on the chunk
    cur_chunk = cap_bound
    # this rank's share of the first level: the initial state lives on its owner
    local_frontier, consumed = int(ck.result().distinct), 0
    ph = res.phase

    def expand(ob):
        """Expand this rank's next chunk into outbox `ob`; returns the send counts."""
        nonlocal consumed, cur_chunk, cap_bound
        t1 = time.perf_counter()
        n_exp = min(cur_chunk, local_frontier - consumed)
        chk(lib.rmc_dist_expand(ctx, cur_chunk, C.c_void_p(outboxes[ob].data_ptr()), cap_per_dest,
                                send, C.byref(done)))
        ph["expand"] += time.perf_counter() - t1
        snd = [int(x) for x in send]
        consumed += max(n_exp, 0)
        res.records_sent += sum(snd)
        res.chunks += 1
        if n_exp > 0:
            # keep the fullest outbox at <= half its capacity (an overflow is an
            # error: dropped records would be lost states)
            rho = max(max(snd), 1) / n_exp
            res.max_dest_per_state = max(res.max_dest_per_state, rho)
            cap_bound = int(min(chunk_states, max(1 << 14, cap_per_dest / (2.0 * rho))))
            cur_chunk = min(cur_chunk, cap_bound)
        return snd

    while True:
        if max_depth > 0 and depth >= max_depth:  # level `depth` stays unexpanded (rmc_run_bfs)
            res.left_on_queue = res.levels[-1] if res.levels else 1
            break
        # ---- expand this level's frontier chunk by chunk; chunk k's records
        # travel while chunk k+1 is expanded; the loop ends when no rank has
        # frontier left (flags ride on the counts all-to-all)
        ob = 0
        # about pipeline_chunks chunks per level (each bounded by the outbox fill)
        cur_chunk = min(cap_bound, max(min_chunk, -(-local_frontier // max(1, pipeline_chunks))))
        snd = expand(ob)
        while True:
            t2 = time.perf_counter()
            recv, flags, anyone = exchange_counts(snd, consumed < local_frontier, dev, cpu, group)
            handle = payload_start(outboxes[ob], snd, recv, cpu, group) if anyone else None
            ph["exchange"] += time.perf_counter() - t2
            more = any(flags)
            if more:  # every rank expands its next chunk (possibly empty) meanwhile
                ob ^= 1
                snd = expand(ob)
            t3 = time.perf_counter()
            if handle is not None:
                received = payload_finish(handle)
                t4 = time.perf_counter()
                ph["exchange"] += t4 - t3
                if received.shape[0]:
                    chk(lib.rmc_dist_insert(ctx, C.c_void_p(received.data_ptr()), received.shape[0]))
                ph["insert"] += time.perf_counter() - t4
            if not more:
                break
        t1 = time.perf_counter()
        chk(lib.rmc_dist_end_level(ctx, out5))
        local_frontier, consumed = int(out5[0]), 0
        stats = _allgather([out5[0], out5[1], out5[2], out5[4], out5[3]], dev, cpu, group)
        ph["level"] += time.perf_counter() - t1
        new, gen, probes = (sum(r[k] for r in stats) for k in range(3))
        viol = max(r[3] for r in stats)
        res.generated += gen
        res.probes += probes
        res.levels.append(new)
        if new:
            depth += 1
        if viol:
            # every violating state of this level has the minimal depth: trace the
            # one of the lowest rank that found one
            vr = min(q for q, r in enumerate(stats) if r[3])
            res.violated_inv = stats[vr][3]
            res.violation_depth = depth
            res.trace = trace(ck, vr, stats[vr][4] - 1, group)
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
