"""bench.py — distinct states/sec and time-to-fixpoint of the raft.tla BFS
(BASELINE.json metric) on MI355X, one process per GPU.

A "step" is one complete breadth-first search of the bounded MCraft model to
its fixpoint (time-to-fixpoint); `value` = distinct states / seconds per step,
whole job.  The workload is deterministic: an exhaustive BFS has no input data.
The default model, specs/MCraftBenchXL.cfg (4.13 G distinct states), is the
largest bounded model sized so far that one GPU completes: on one GPU its
expanded levels leave the device window (RMC_FLAG_SPILL with the trace links
kept in HBM), sharded every rank holds its part resident.
With N > 1 ranks the state space is sharded over the GPUs inside librmc
(rmc_shard: owner-routed successors, fingerprint-first two-phase exchange
over librmc's own RCCL communicator) and the SAME model is searched, so
scaling is strong.

Launch: `python bench.py --gpus N` starts its own N rank processes (before
anything touches a GPU) when no outer launcher set WORLD_SIZE; under
`torch.distributed.run --nproc-per-node N` every process is one rank.  A line
whose rank count differs from --gpus is refused.
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))

METRIC = "distinct states/sec (whole node) and time-to-fixpoint on MCraft BFS, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=os.path.join(ROOT, "specs", "MCraftBenchXL.cfg"))
    ap.add_argument("--capacity", type=int, default=0,
                    help="state capacity per GPU (0: 1.5e9 / world * 1.3 for MCraftBench.cfg, the table size every "
                         "round measured; any other model: librmc's own sizing, 80%% of free HBM)")
    ap.add_argument("--set-bytes", type=int, default=-1,
                    help="fingerprint-set bytes per GPU (rmc_config.set_bytes, TLC -fpmem; 0: librmc's sizing, "
                         "load <= 1/2; -1: the bench default, sparse_set_bytes: 8 slots per state of capacity)")
    ap.add_argument("--spill", default="auto", choices=("auto", "on", "off"),
                    help="RMC_FLAG_SPILL (expanded levels leave the device window; their trace links stay in "
                         "HBM): auto = on for a single GPU unless the model is MCraftBench.cfg")
    ap.add_argument("--device", type=int, default=-1, help="-1: LOCAL_RANK modulo the visible GPUs")
    ap.add_argument("--keys-per-dest", type=int, default=0,
                    help="sharded mode: phase-1 keys one chunk may send one owner (0 = librmc's choice)")
    ap.add_argument("--sent-cache", type=int, default=1 << 30,
                    help="sharded mode: slots of the per-rank cache of fingerprints already sent")
    ap.add_argument("--transport", default="auto",
                    help="sharded mode: rccl | host | auto (rccl when every rank has its own GPU, "
                         "else the host transport over gloo)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the sharded path even at one rank (measures its overhead)")
    ap.add_argument("--no-probe-ceiling", action="store_true",
                    help="skip the random-probe microbenchmark (roofline ceiling)")
    ap.add_argument("--cpu-levels", type=int, default=22,
                    help="BFS levels of the same model timed on the host CPU oracle")
    ap.add_argument("--cpu-fixpoint", default=os.path.join(ROOT, "specs", "MCraftBounded.cfg"),
                    help="model timed to its fixpoint on the host CPU oracle AND on the GPU "
                         "('' to skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--v2-only", default="", help=argparse.SUPPRESS)  # internal: the child of v2_fixpoint_child
    ap.add_argument("--v2-config", default=os.path.join(ROOT, "specs", "MCraftBench.cfg"),
                    help="one GPU: also time this model (the reference's Value = {v1, v2}, MCraft.tla:15-16) "
                         "to its fixpoint after the timed steps, untimed in the line's value ('' to skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch logic only: ranks rendezvous over gloo and report, no GPU, no librmc")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="self-launch: seconds before the rank processes are killed")
    return ap.parse_args(argv)


# ---- self-launch ---------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a, argv):
    """Start N rank processes of this script (torchrun's env contract: RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT) and relay rank 0's JSON line.
    Runs before anything in this process touches a GPU or loads librmc."""
    import tempfile
    n = a.gpus
    port = _free_port()
    procs = []
    out_f = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), RMC_BENCH_LAUNCHER="bench.py --gpus (self-launch)")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=out_f if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))
    # poll every rank: one that fails leaves the others blocked in a collective,
    # so the first failure (or the time limit) ends them all
    t0 = time.time()
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs) or any(rc not in (None, 0) for rc in rcs) \
                or time.time() - t0 > a.launch_timeout:
            break
        time.sleep(0.2)
    if any(rc is None for rc in rcs) or any(rcs):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, 9)
                except ProcessLookupError:
                    pass
            p.wait()
        sys.stderr.write(f"bench.py: rank exit codes {rcs}; no result line\n")
        return 1
    out_f.seek(0)
    out = out_f.read()
    lines = [ln for ln in out.decode().splitlines() if ln.startswith("{")]
    if len(lines) != 1:
        sys.stderr.write("bench.py: rank 0 printed no result line\n")
        return 1
    rec = json.loads(lines[0])
    if rec.get("n_gpus") != n:
        sys.stderr.write(f"bench.py: rank 0 reports {rec.get('n_gpus')} ranks, --gpus {n}: refused\n")
        return 1
    sys.stdout.write(json.dumps(rec) + "\n")
    sys.stdout.flush()
    return 0


# ---- CPU baseline ----------------------------------------------------------------
def host_cpu_info():
    """Cores this process may use (affinity, then the cgroup quota), plus what
    the machine shows: SURVEY.md §8d asks for nproc, physical cores and model."""
    nproc = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = nproc
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    usable = min(allowed, quota) if quota else allowed
    # the job's CPU share when the launcher states one (the GPU pool sets
    # OMP_NUM_THREADS to the box's share of its host cores)
    share = os.environ.get("OMP_NUM_THREADS", "")
    share = int(share) if share.isdigit() and int(share) > 0 else None
    if share:
        usable = min(usable, share)
    model, phys = platform.processor() or "?", set()
    try:
        cur = {}
        for ln in open("/proc/cpuinfo"):
            if ":" in ln:
                k, v = (x.strip() for x in ln.split(":", 1))
                if k == "model name":
                    model = v
                cur[k] = v
            elif cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    return {"nproc": nproc, "affinity_cpus": allowed, "cgroup_quota_cpus": quota, "omp_num_threads": share,
            "usable": usable,
            "physical_cores": len(phys) or None, "model": model}


def cpu_baseline(cfg, levels, fix_cfg, gpu_fix, gpu_levels=None):
    """C oracle (test infrastructure, kind "port") on the host cores this job
    may use: (1) the first `levels` BFS levels of the bench model, (2) a
    complete fixpoint of `fix_cfg` timed next to the GPU on the same model.
    gpu_levels: the bench model's per-level (new states, cumulative generated)
    from one untimed GPU run; `prefix_agree` says whether the oracle's first
    levels equal them."""
    import rmc
    from tests import oracle_c
    info = host_cpu_info()
    threads = info["usable"]

    def run(c, max_levels, capacity):
        return oracle_c.bfs(c.n_servers, c.n_values, c.max_term, c.max_log_len, c.max_msgs, c.max_dup,
                            bug=int(bool(c.flags & rmc.FLAG_BUG_QUORUM)), inv=c.invariants,
                            sym=int(bool(c.flags & rmc.FLAG_SYMMETRY)), threads=threads,
                            max_levels=max_levels, capacity=capacity)

    r, ln, _ = run(cfg, levels, 1 << 27)
    out = {"value": r.distinct / r.seconds, "unit": "distinct states/s", "cores": threads, "kind": "port",
           "host": info,
           "sample": f"C oracle (oracle/rmc_oracle.c, exact state set, {threads} threads) BFS levels 1..{r.depth} "
                     f"of the same model: {r.distinct} distinct / {r.generated} generated in {r.seconds:.2f} s"}
    if gpu_levels is not None:
        new, gen = gpu_levels
        d = len(ln)
        # the GPU's cumulative generated once level d exists (the callback of expanding level d - 1)
        g_at = gen[d - 2] if 2 <= d <= len(gen) + 1 else None
        out["prefix_agree"] = new[:d] == ln and g_at == r.generated
        out["prefix_levels"] = d
    if fix_cfg is not None:
        f = run(fix_cfg, 0, 1 << 27)[0]
        gd, gg, gdep, gt = gpu_fix
        out["fixpoint"] = {
            "model": gpu_fix_name(fix_cfg), "cpu_distinct": f.distinct, "cpu_generated": f.generated,
            "cpu_depth": f.depth, "cpu_seconds": f.seconds, "cpu_rate": f.distinct / f.seconds,
            "gpu_distinct": gd, "gpu_generated": gg, "gpu_depth": gdep, "gpu_seconds": gt,
            "gpu_rate": gd / gt if gt > 0 else None,
            "agree": (f.distinct, f.generated, f.depth) == (gd, gg, gdep),
            "gpu_over_cpu": (f.seconds / gt) if gt > 0 else None}
    return out


def gpu_fix_name(c):
    return (f"S={c.n_servers} V={c.n_values} MaxTerm={c.max_term} MaxLogLen={c.max_log_len} "
            f"MaxMsgs={c.max_msgs} MaxDup={c.max_dup}")


def pmc_traffic(config_path):
    """HBM bytes per expansion launch from the committed rocprofv3 PMC profile
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


def sparse_set_bytes(capacity, per_state=4):
    """The bench's fingerprint-set size (rmc_config.set_bytes, TLC -fpmem): 8-B
    slots for `per_state` times the states the GPU may store, rounded up to a
    power of two (librmc halves it until the store fits beside it) — load <= 1/4
    instead of librmc's default 1/2.  A probe for a new state ends at the first
    empty slot, one dependent load per occupied slot before it: doubling the set
    took XL 731 -> 704 ms and MCraftBench 210 -> 198 ms on one box, its larger
    clear included (profiles/r06/ab/set_size.txt).  The bench takes 8 slots per
    state: with set epochs its runs no longer clear the set, and MCraftBench's
    2^34 slots measured 184.8-186.1 against 188.6-191.2 ms for 2^33
    (profiles/r06/ab/set_size_mcraftbench.txt); XL stays at 2^34, what fits."""
    slots = 1
    while slots < per_state * capacity:
        slots <<= 1
    return slots * 8


def v2_fixpoint_child(path, dev):
    """v2_fixpoint in a child process (a fresh device address space: after the
    XL run's 230 GB were allocated and freed in this one, the same search
    measured 218 vs 205.5 ms)."""
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--v2-only", path, "--device", str(dev)],
                       capture_output=True, text=True, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode or not lines:
        return {"error": f"child exit {r.returncode}: {r.stderr[-400:]}"}
    out = json.loads(lines[-1])
    out["process"] = "child (fresh device address space)"
    return out


def v2_fixpoint(path, dev, runs=3):
    """The bench model of rounds 1-4, MCraftBench.cfg (S=3 with the reference's
    Value = {v1, v2}, MCraft.tla:15-16), searched to its fixpoint on the same GPU
    after the timed steps: one warm run, then the best and mean of `runs`.  Not
    part of the line's value (the XL model, V = 1, is the headline workload)."""
    import rmc
    c = rmc.config_from_files(path, builtin_raft=True)
    c.device = dev
    c.state_capacity = int(1.5e9)  # resident, no spill (the size every round measured)
    c.set_bytes = sparse_set_bytes(c.state_capacity, 8)
    ts = []
    with rmc.Checker(c) as ck:
        ck.run(record_levels=False)
        for _ in range(runs):
            t0 = time.perf_counter()
            r = ck.run(record_levels=False)
            ts.append(time.perf_counter() - t0)
    return {"model": os.path.basename(path) + ": " + gpu_fix_name(c), "distinct": r.distinct,
            "generated": r.generated, "depth": r.depth, "runs": runs, "ms_best": min(ts) * 1e3,
            "ms_mean": sum(ts) / len(ts) * 1e3, "distinct_per_s_best": r.distinct / min(ts)}


# ---- one rank ------------------------------------------------------------------
def dry_run(a, world, rank):
    """Rendezvous + the timing collectives of a real run, without a GPU."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
        ranks = [None] * world
        dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid(),
                                       "local_rank": int(os.environ.get("LOCAL_RANK", "0"))})
        t = torch.tensor([0.001 * (rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        dist.destroy_process_group()
    else:
        ranks, dt = [{"rank": 0, "pid": os.getpid(), "local_rank": 0}], 0.001
    return {"metric": METRIC, "value": 0.0, "unit": "distinct states/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u64", "data": "dry run: launch logic only, nothing measured",
            "config": {"workload": "dry run"}, "dry_run": True, "ranks_seen": ranks,
            "launcher": os.environ.get("RMC_BENCH_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                       else "single process")}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return self_launch(a, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        sys.stderr.write(f"bench.py: {world} ranks but --gpus {a.gpus}: refused (no line printed)\n")
        return 2
    # The JSON line is the only thing on stdout: libraries that print banners
    # there (RCCL prints its version block at communicator init) are sent to
    # stderr by pointing fd 1 at fd 2 for the rest of the run.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if a.v2_only:
        os.write(json_fd, (json.dumps(v2_fixpoint(a.v2_only, max(a.device, 0))) + "\n").encode())
        return 0
    if a.dry_run:
        out = dry_run(a, world, rank)
        if rank == 0:
            os.write(json_fd, (json.dumps(out) + "\n").encode())
        return 0

    import rmc
    dist = None
    sharded = world > 1 or a.force_dist
    ndev = 1
    transport = "none"
    backend = None
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        import torch
        import torch.distributed as dist
        ndev = max(1, torch.cuda.device_count())  # does not initialise the GPU on this image
        shared = ndev < world
        transport = a.transport
        if transport == "auto":
            transport = "host" if shared else "rccl"
        if transport == "rccl" and shared:
            sys.stderr.write(f"bench.py: {world} ranks on {ndev} GPU(s): RCCL needs one GPU per rank "
                             "(use --transport host)\n")
            return 2
        dev = a.device if a.device >= 0 else local % ndev
        backend = "nccl" if transport == "rccl" else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(dev)
        dist.init_process_group(backend, init_method="env://")
    else:
        dev = max(a.device, 0)
    # the GPU box has no raft.tla: the bench model checks the compiled-in lemmy/raft.tla
    cfg = rmc.config_from_files(a.config, builtin_raft=True)
    cfg.device = dev
    ranks_per_gpu = max(1, -(-world // ndev)) if sharded else 1
    small = os.path.basename(a.config) == "MCraftBench.cfg"
    xl = os.path.basename(a.config) == "MCraftBenchXL.cfg"
    if a.capacity:
        cfg.state_capacity = a.capacity
    elif small:
        cfg.state_capacity = int(1.5e9 / world * (1.3 if sharded else 1.0))
    elif xl and sharded:  # 4.13 G states: a rank's share, +20 % for the owner imbalance (the 8-rank
        # rehearsal's fullest rank held 13.4 % of the states, 1.07x its share: profiles/r06/dist8/)
        cfg.state_capacity = int(4.14e9 / world * 1.2)
    elif xl:  # 4,132,397,328 states: the store and the ring window fit beside a 2^34-slot set
        cfg.state_capacity = int(4.14e9)
    else:  # librmc's own sizing (80 % of free HBM)
        cfg.state_capacity = 0
    if a.set_bytes >= 0:
        cfg.set_bytes = a.set_bytes
    elif cfg.state_capacity:  # 8 slots per state (set epochs: a larger set costs no clear per run)
        cfg.set_bytes = sparse_set_bytes(cfg.state_capacity, 8)
    spill = (a.spill == "on" or (a.spill == "auto" and not small)) and not sharded
    if spill:
        cfg.flags |= rmc.FLAG_SPILL
    W = rmc.native().rmc_state_bytes(cfg)
    # roofline ceiling of the fingerprint set: random 8-B probes over 64 GB
    r_max = None
    if not a.no_probe_ceiling and ranks_per_gpu == 1 and rank == 0:
        r_max = rmc.probe_bench(device=cfg.device, table_bytes=(64 << 30) // ranks_per_gpu,
                                accesses=1 << 32, mode=0)

    def barrier():
        if dist is not None:
            dist.barrier()

    last = [None]

    def one_run(ck):
        # sharded: rmc_run_bfs is a collective inside librmc; the result is global
        r = ck.run(record_levels=False)
        last[0] = r
        return r.distinct, r.generated, r.depth, r.probes, r.expand_kernel_seconds, r.expand_launches

    with rmc.Checker(cfg) as ck:
        if sharded:
            from rmc import dist as rdist
            info = rdist.shard(ck, transport=transport, keys_per_dest=a.keys_per_dest,
                               sent_cache_slots=a.sent_cache)
            transport = info.transport
        cold = []  # the ctx's first run clears the whole fingerprint set (librmc's set epochs: DESIGN.md §d)
        for _ in range(a.warmup):
            tw = time.perf_counter()
            one_run(ck)
            cold.append(time.perf_counter() - tw)
        barrier()
        if dist is not None:
            import torch
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        kern = 0.0
        launches = 0
        for _ in range(a.steps):
            D, G, depth, NP, ks, nl = one_run(ck)
            kern += ks
            launches += nl
        if dist is not None:
            import torch
            torch.cuda.synchronize(dev)
        barrier()
        dt = time.perf_counter() - t0
        salt_check = None
        gpu_levels = None
        if not sharded:  # untimed: same search under another fingerprint salt
            ck.set_seed(0x5A17ED)
            r2 = ck.run(record_levels=False)
            ck.set_seed(0)
            salt_check = {"salt": 0x5A17ED, "distinct": r2.distinct, "generated": r2.generated,
                          "depth": r2.depth,
                          "agrees": (r2.distinct, r2.generated, r2.depth) == (D, G, depth)}
            if rank == 0 and not a.no_cpu:  # untimed: per-level counts for the oracle prefix check
                ck.run(record_levels=True)
                gpu_levels = ([1] + [x[3] for x in ck.levels if x[3]], [x[1] for x in ck.levels])
    per_rank = None
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        ld = last[0]
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "device": dev, "stored": ld.stored_here,
                                          "keys_sent": ld.keys_sent, "states_sent": ld.states_sent,
                                          "chunks": ld.chunks, "exchange_s": round(ld.exchange_seconds, 6),
                                          "kernel_s": round(ld.expand_kernel_seconds, 6)})
    per_step = dt / a.steps
    # algorithmic bytes per run, SURVEY.md §8(d)'s per-unit figure:
    # one random 64-B HBM granule per generated successor (the fingerprint-set
    # probe/insert TLC's algorithm makes for it) + for every distinct state the
    # state written, read back as frontier, its 8-B parent ref and 8-B fingerprint
    b_alg = G * 64 + D * (2 * W + 16)
    # what the kernel actually issues: stuttering, out-of-CONSTRAINT and
    # commuting-diamond successors are never probed (NP probes, one 64-B granule each)
    b_issued = NP * 64 + D * (2 * W + 16)
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
            "fingerprint_set": {"slots": last[0].set_slots, "bytes": last[0].set_slots * 8,
                                "epochs": ("tagged: each timed run takes the next set epoch instead of clearing "
                                           "the set; the ctx's first run (the warmup) cleared it, and every 255th "
                                           "run clears it (RMC_SET_EPOCH)")
                                          if os.environ.get("RMC_SET_EPOCH", "1") != "0"
                                          else "cleared before every run",
                                "first_run_ms_with_clear": cold[0] * 1e3 if cold else None,
                                "load": (last[0].distinct / last[0].set_slots) if last[0].set_slots else None,
                                "set_bytes": cfg.set_bytes, "capacity": cfg.state_capacity,
                                "rule": "sparse_set_bytes: 8 slots per state of capacity, halved by librmc until the store fits (TLC -fpmem)"
                                        if a.set_bytes < 0 and cfg.set_bytes else "set_bytes given / librmc's"},
            "spill": ({"flag": "RMC_FLAG_SPILL", "trace_links": "device" if last[0].spill_links_on_device else "host",
                       "window": ("ring (slot reuse, nothing copied)" if last[0].spill_links_on_device
                                  else "shifted (links to host memory)"),
                       "spills_per_step": last[0].spills, "states_out_of_window_per_step": last[0].spilled,
                       "spill_seconds_per_step": last[0].spill_seconds} if spill else None),
            "parallelism": (f"state-space sharded x{world} (librmc two-phase exchange, "
                            f"{'RCCL over xGMI' if transport == 'rccl' else 'host transport over gloo'})")
                           if sharded else "single GPU",
            "fp_salt_crosscheck": salt_check,
        },
        "world": {"ranks": world, "transport": transport, "torch_backend": backend,
                  "gpus_visible": ndev if sharded else 1, "ranks_per_gpu": ranks_per_gpu,
                  "launcher": os.environ.get("RMC_BENCH_LAUNCHER",
                                             "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                             else "single process")},
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
            "kernel": ("k_expand_sort (librmc's default expansion kernel; kernel_ms_per_step brackets each "
                       "expansion launch with HIP events, i.e. k_window_order + k_expand_sort)") if not sharded
                      else "k_expand_dist (librmc's sharded expansion kernel)",
            "kernel_ms_per_step": ks * 1e3,
            "launches_per_step": nlaunch, "alg_bytes_per_launch": b_alg / nlaunch,
            "alg_bytes_per_step": b_alg, "alg_bytes_def": "G*64 + D*(2W+16) (SURVEY.md 8(d))",
            "issued_bytes_per_step": b_issued,
            "issued_frac": (b_issued / ks / 1e9 / HBM_PEAK_GBS) if ks > 0 else 0.0,
            "traffic_frac": (traffic * nlaunch / ks / 1e9 / HBM_PEAK_GBS) if (traffic and ks > 0) else None,
            "probes_per_step": NP,
            "probe_rate_per_s": NP / ks if ks > 0 else 0.0,
            "probe_ceiling_per_s": r_max,
            "frac_of_probe_ceiling": (NP / ks / r_max) if (ks > 0 and r_max) else None,
            # the kernel's whole HBM traffic (probes, CAS write-backs of new keys, frontier
            # reads, state stores: PMC) per second against the random-granule ceiling —
            # the measured random 8-B load rate x the 64-B granule each one moves
            "traffic_frac_of_random_ceiling": (traffic * nlaunch / ks / (r_max * 64.0))
                                              if (traffic and ks > 0 and r_max) else None,
        },
    }
    if sharded:
        ld = last[0]
        out["sharded"] = {"in_library": "rmc_shard + rmc_run_bfs (two-phase fingerprint-first exchange)",
                          "transport": transport, "chunks_rank0": ld.chunks, "keys_sent_rank0": ld.keys_sent,
                          "states_sent_rank0": ld.states_sent, "stored_rank0": ld.stored_here,
                          "exchange_s_rank0": round(ld.exchange_seconds, 6),
                          "host_wait_s_rank0": round(ld.exchange_wait_seconds, 6),
                          "rounds_parked_keys_rank0": ld.parked, "keys_per_dest": a.keys_per_dest,
                          "per_rank": per_rank}
        out["roofline"]["note"] = ("per-rank kernel time of rank 0; achieved = the job's algorithmic bytes / "
                                   "world / rank 0's kernel time")
        out["roofline"]["achieved"] = (b_alg / world) / ks / 1e9 if ks > 0 else 0.0
        out["roofline"]["frac"] = out["roofline"]["achieved"] / HBM_PEAK_GBS
    if rank == 0 and world == 1 and a.v2_config and os.path.abspath(a.v2_config) != os.path.abspath(a.config):
        out["value_set_v2"] = v2_fixpoint_child(a.v2_config, dev)
    if rank == 0 and not a.no_cpu and world == 1:
        fix_cfg, gpu_fix = None, None
        if a.cpu_fixpoint:
            fix_cfg = rmc.config_from_files(a.cpu_fixpoint, builtin_raft=True)
            fix_cfg.device = dev
            with rmc.Checker(fix_cfg) as fk:
                fk.run(record_levels=False)  # warm
                fr = fk.run(record_levels=False)
            gpu_fix = (fr.distinct, fr.generated, fr.depth, fr.seconds)
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_levels, fix_cfg, gpu_fix, gpu_levels)
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
