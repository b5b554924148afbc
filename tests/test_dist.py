"""Sharded multi-rank BFS: N ranks must reproduce the single-GPU / oracle
counts exactly ("run N shards as N ranks on one GPU and
require counts identical to N=1").

The GPU tests run 2 and 4 ranks sharing the box's one GPU over gloo; the
8-GPU RCCL run is the driver's scaling bench.  The CPU test exercises the
host-side exchange protocol (rmc.dist.exchange) with world size 2 on gloo."""
import json
import os
import subprocess
import sys

import pytest

import rmc
from oracle import raft_spec as R
from tests.convert import check_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_levels.json")))


def _torchrun(nproc, args, port, timeout=150, rep="4096"):
    """rep: RMC_DIST_REP, the largest level (states, all ranks) searched as a
    replicated level.  The tests' default, 4096, mixes both kinds in one search:
    the first levels replicated, the larger ones with the key/state exchange."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    env = dict(os.environ, OMP_NUM_THREADS="1", RMC_DIST_REP=rep)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


TRANSPORT_WORKER = r"""
import ctypes as C, os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.path.join(sys.argv[1], 'raft.tla_amd'))
from rmc.dist import GlooTransport
dist.init_process_group('gloo', init_method='env://')
r, w = dist.get_rank(), dist.get_world_size()
t = GlooTransport()
# alltoallv: rank r sends (r + d) % 3 bytes of value 10 * r + d to rank d
sb = [(r + d) % 3 for d in range(w)]
rb = [(s + r) % 3 for s in range(w)]
send = bytes(b for d in range(w) for b in [10 * r + d] * sb[d])
sbuf = C.create_string_buffer(send, max(1, len(send)))
rbuf = C.create_string_buffer(max(1, sum(rb)))
SB, RB = (C.c_uint64 * w)(*sb), (C.c_uint64 * w)(*rb)
assert t.struct.alltoallv(None, C.addressof(sbuf), SB, C.addressof(rbuf), RB) == 0, t.errors
want = bytes(b for s in range(w) for b in [10 * s + r] * rb[s])
assert rbuf.raw[:sum(rb)] == want, (rbuf.raw, want)
# allgather of 8 bytes per rank
mine = C.create_string_buffer(bytes([r] * 8), 8)
out = C.create_string_buffer(8 * w)
assert t.struct.allgather(None, C.addressof(mine), 8, C.addressof(out)) == 0, t.errors
assert out.raw == bytes(b for q in range(w) for b in [q] * 8)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("nproc", [2, 3])
def test_host_transport_gloo(nproc, tmp_path):
    """The host transport librmc's sharded BFS calls back into (rmc_transport):
    all-to-all of byte blocks and all-gather, world 2 and 3 on gloo (CPU)."""
    script = tmp_path / "tw.py"
    script.write_text(TRANSPORT_WORKER)
    r = _torchrun(nproc, [str(script), ROOT], 29611 + nproc)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("case,nproc,backend,rep", [
    ("tiny2_v2", 2, "gloo", "4096"), ("small", 2, "gloo", "4096"), ("small", 4, "gloo", "4096"),
    ("small", 3, "gloo", "0"), ("small", 3, "gloo", "1048576"), ("s5_prefix9", 2, "gloo", "4096"),
    ("small_sym", 2, "gloo", "4096"), ("bounded_sym_prefix16", 3, "gloo", "4096"),
    ("msgs5_dup2_prefix9", 2, "gloo", "4096"), ("s4_prefix10", 3, "gloo", "4096"),
    ("tiny2_log3", 2, "gloo", "4096"), ("s3_log3_prefix14", 2, "gloo", "4096"),
    ("tiny2_log3", 3, "gloo", "1048576"), ("small", 1, "nccl", "4096"), ("small", 1, "nccl", "0")])
def test_sharded_bfs_matches_oracle(case, nproc, backend, rep, tmp_path):
    """The sharded BFS inside librmc (rmc_shard + rmc_run_bfs), through the C
    ABI.  gloo: N ranks share the box's one GPU over the host transport.
    nccl: one rank on librmc's own RCCL communicator, the code path of the
    driver's multi-GPU bench.  SYMMETRY cases route by the canonical
    fingerprint; depth-bounded cases stop with the last level unexpanded, as
    the single-GPU search.  A small key outbox forces several chunks per
    level and several phase-2 rounds.  rep (RMC_DIST_REP): "4096" mixes
    replicated small levels with exchanged large ones in one search, "0"
    exchanges every level, "1048576" replicates every level of these models
    (no key leaves its rank; SYMMETRY never replicates)."""
    g = GOLDEN[case]
    out = tmp_path / "r.json"
    r = _torchrun(nproc, [os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case, "--out",
                          str(out), "--device", "0", "--backend", backend], 29620 + nproc, rep=rep)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert res["distinct"] == g["distinct"]
    assert res["generated"] == g["generated"]
    assert res["depth"] == g["depth"]
    assert res["left_on_queue"] == g["left_on_queue"]
    assert res["levels"] == g["level_new"]
    assert res["rerun"] == [[g["distinct"], g["generated"], g["depth"]]]
    all_rep = rep == "1048576" and not g["params"]["symmetry"]
    if nproc > 1:
        assert (res["keys_sent"] > 0) != all_rep
        assert (res["states_sent"] > 0) != all_rep
    assert sum(p["stored"] for p in res["per_rank"]) == g["distinct"]
    assert all(p["summary"]["distinct"] == g["distinct"] for p in res["per_rank"])  # global on every rank


@pytest.mark.gpu
@pytest.mark.parametrize("case,nproc,backend,ep_max", [("small", 2, "gloo", None), ("s4_prefix10", 3, "gloo", "2"),
                                                      ("tiny2_log3", 3, "gloo", None), ("small", 1, "nccl", None)])
def test_sharded_set_epochs_reruns_equal_the_oracle(case, nproc, backend, ep_max, tmp_path):
    """Set epochs on the sharded send-marker path: after a ctx's first run each
    rank's set is not cleared but takes the next epoch (RMC_SET_EPOCH=2: a full
    clear every second run); four more runs on the same sharded ctxs equal the
    oracle."""
    g = GOLDEN[case]
    out = tmp_path / "r.json"
    env_keep = os.environ.get("RMC_SET_EPOCH")
    if ep_max is not None:
        os.environ["RMC_SET_EPOCH"] = ep_max
    try:
        r = _torchrun(nproc, [os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case, "--out",
                              str(out), "--device", "0", "--backend", backend, "--rerun", "4"], 29660 + nproc)
    finally:
        if ep_max is not None:
            if env_keep is None:
                os.environ.pop("RMC_SET_EPOCH", None)
            else:
                os.environ["RMC_SET_EPOCH"] = env_keep
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert (res["distinct"], res["generated"], res["depth"]) == (g["distinct"], g["generated"], g["depth"])
    assert res["rerun"] == [[g["distinct"], g["generated"], g["depth"]]] * 4


@pytest.mark.gpu
@pytest.mark.parametrize("case,nproc", [("bug_one_leader", 2), ("bug_log_matching", 3), ("bug_both", 2),
                                        ("messages_small", 2), ("bug_cand_term", 3)])
def test_sharded_violation_and_trace(case, nproc, tmp_path):
    """Bug variant (config 5) on N ranks: the violation, its minimal depth and the
    counts at the stopping level equal the oracle's, and the counterexample,
    gathered rank by rank through the global parent refs, is a behaviour of the
    spec ending in a violating state (SURVEY.md §8e "Trace")."""
    g = GOLDEN[case]
    p = g["params"]
    out = tmp_path / "r.json"
    r = _torchrun(nproc, [os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case, "--out",
                          str(out), "--device", "0", "--backend", "gloo"], 29640 + nproc)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert res["violated_inv"] == g["violated_inv"]
    assert res["violation_depth"] == g["violation_depth"]
    assert res["distinct"] == g["distinct"] and res["generated"] == g["generated"]
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                    max_log=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                    bug_quorum=bool(p["bug_quorum"]))
    trace = [(f, i, rmc.StateView.from_buffer_copy(bytes.fromhex(h))) for f, i, h in res["trace"]]
    check_trace(model, trace, res["violated_inv"], res["violation_depth"])


@pytest.mark.gpu
def test_sharded_full_bench_model_equals_single_gpu(tmp_path):
    """The 1.23 G-state bench model (specs/MCraftBench.cfg) is beyond the
    oracles, so the sharded search is pinned against the single-GPU one: 2
    ranks sharing the GPU (host transport), different owner partitions and
    table layouts, must find exactly the single-GPU counts (bench.py's
    fp_salt_crosscheck and the verification mode pin those:
    1,227,465,177 distinct, 21,130,972,267 generated, depth 56)."""
    out = tmp_path / "r.json"
    r = _torchrun(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--cfg",
                      os.path.join(ROOT, "specs", "MCraftBench.cfg"), "--out", str(out), "--device", "0",
                      "--backend", "gloo", "--capacity", "800000000", "--keys-per-dest", str(1 << 24),
                      "--rerun", "0", "--sent-cache", str(1 << 28)], 29660, timeout=220, rep="1048576")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert (res["distinct"], res["generated"], res["depth"]) == (1_227_465_177, 21_130_972_267, 56)
    assert sum(p["stored"] for p in res["per_rank"]) == 1_227_465_177
    assert res["keys_sent"] > 0 and res["states_sent"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case,nproc,overlap", [("small", 2, "1"), ("small_sym", 3, "0"), ("s4_prefix10", 2, "1")])
def test_sharded_outbox_overflow_is_recovered(case, nproc, overlap, tmp_path):
    """an owner's key outbox that fills is not fatal.  With
    4096 keys per owner and round, and rounds sized for 3x that (RMC_DIST_FILL=3),
    the outboxes overflow on every large level; the parked keys go out
    in further rounds of the same level and the counts equal the oracle's.
    overlap "0" runs the rounds without the next expansion queued early
    (RMC_DIST_OVERLAP=0): same counts."""
    g = GOLDEN[case]
    out = tmp_path / "r.json"
    env_over = dict(os.environ, RMC_DIST_OVERLAP=overlap, RMC_DIST_FILL="3", RMC_DIST_REP="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(29680 + nproc),
           os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case, "--out", str(out), "--device", "0",
           "--backend", "gloo", "--keys-per-dest", "4096", "--rerun", "1"]
    env_over["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env_over, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert (res["distinct"], res["generated"], res["depth"]) == (g["distinct"], g["generated"], g["depth"])
    assert res["levels"] == g["level_new"]
    assert res["rerun"] == [[g["distinct"], g["generated"], g["depth"]]]
    assert res["parked"] > 0  # the outboxes did overflow


@pytest.mark.gpu
@pytest.mark.parametrize("case,nproc", [("small", 2), ("small", 4), ("small_sym", 3), ("s3_log3_prefix14", 2)])
def test_sharded_verification(case, nproc, tmp_path):
    """Full-state verification on a sharded search: every
    fingerprint hit, local or at the owner of a remote successor, is compared
    state by state.  Full fingerprints: 0 collisions and the oracle's counts.
    Fingerprints cut to 16 bits: the collisions are found and reported."""
    g = GOLDEN[case]
    out = tmp_path / "r.json"
    base = [os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case, "--device", "0", "--backend", "gloo",
            "--verify", "--rerun", "0"]
    r = _torchrun(nproc, base + ["--out", str(out)], 29700 + nproc)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert (res["distinct"], res["generated"], res["depth"]) == (g["distinct"], g["generated"], g["depth"])
    assert res["collisions"] == 0 and res["verified"] > 0
    assert sum(p["stored"] for p in res["per_rank"]) == g["distinct"]
    out16 = tmp_path / "r16.json"
    r = _torchrun(nproc, base + ["--out", str(out16), "--fp-bits", "16"], 29710 + nproc)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res16 = json.load(open(out16))
    assert res16["collisions"] > 0 and res16["verified"] > 0
    assert res16["distinct"] < g["distinct"]  # the colliding states were (reported as) dropped


@pytest.mark.gpu
def test_sharded_verification_full_bench_model(tmp_path):
    """The 1.23 G-state bench model verified state by state on 2 ranks: the
    single-GPU counts and 0 collisions (SURVEY.md §8d config 3's "full-state
    verification runs at least once", sharded)."""
    out = tmp_path / "r.json"
    r = _torchrun(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--cfg",
                      os.path.join(ROOT, "specs", "MCraftBench.cfg"), "--out", str(out), "--device", "0",
                      "--backend", "gloo", "--capacity", "800000000", "--keys-per-dest", str(1 << 24),
                      "--rerun", "0", "--verify"], 29720, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out))
    assert (res["distinct"], res["generated"], res["depth"]) == (1_227_465_177, 21_130_972_267, 56)
    assert res["collisions"] == 0 and res["verified"] > 1_000_000_000


@pytest.mark.gpu
@pytest.mark.parametrize("case,nproc,stop", [("small", 2, 20), ("small_sym", 3, 25)])
def test_sharded_checkpoint_and_recover(case, nproc, stop, tmp_path):
    """TLC -checkpoint / -recover on a sharded search: N ranks stop at depth
    `stop`, each writes its part (<path>.rank<r>); N new rank processes recover
    their parts (fingerprint sets rebuilt from the states) and finish with the
    oracle's counts."""
    g = GOLDEN[case]
    ck = tmp_path / "ckpt"
    out1, out2 = tmp_path / "r1.json", tmp_path / "r2.json"
    base = [os.path.join(ROOT, "tests", "dist_worker.py"), "--case", case, "--device", "0", "--backend", "gloo",
            "--rerun", "0"]
    r = _torchrun(nproc, base + ["--out", str(out1), "--max-depth", str(stop), "--checkpoint", str(ck)], 29730 + nproc)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    first = json.load(open(out1))
    assert first["depth"] == stop and first["left_on_queue"] > 0
    assert first["levels"] == g["level_new"][:stop]
    assert all(os.path.exists(f"{ck}.rank{k}") for k in range(nproc))
    r = _torchrun(nproc, base + ["--out", str(out2), "--max-depth", "0", "--recover", str(ck)], 29740 + nproc)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.load(open(out2))
    assert (res["distinct"], res["generated"], res["depth"]) == (g["distinct"], g["generated"], g["depth"])
    assert sum(p["stored"] for p in res["per_rank"]) == g["distinct"]


def _launch_ranks(nproc, args, port, env_extra, timeout):
    """Every rank as its own process (no torchrun: it would end the others at the
    first failure, hiding how each rank ends).  Returns [(rc, stderr, seconds)]."""
    import time
    procs = []
    t0 = time.time()
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1", **env_extra)
        procs.append(subprocess.Popen([sys.executable] + args, env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    for p in procs:
        try:
            _, err = p.communicate(timeout=max(1.0, timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            p.kill()
            _, err = p.communicate()
            out.append((None, err, time.time() - t0))
            continue
        out.append((p.returncode, err, time.time() - t0))
    return out


@pytest.mark.gpu
def test_stalled_rank_ends_every_rank_within_the_deadline(tmp_path):
    """a rank that stops answering (RMC_DIST_STALL_RANK=1
    sleeps at level 2) must not hang the others.  With RMC_DIST_TIMEOUT_S=5
    every rank exits non-zero well before an outer limit, and the waiting rank
    names the deadline, the level and the phase it was in."""
    env = {"RMC_DIST_TIMEOUT_S": "5", "RMC_DIST_STALL_RANK": "1", "RMC_DIST_STALL_LEVEL": "2",
           "RMC_DIST_STALL_S": "12"}
    res = _launch_ranks(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "--case", "small", "--out",
                            str(tmp_path / "r.json"), "--device", "0", "--backend", "gloo"], 29790, env, 90)
    for rc, err, secs in res:
        assert rc is not None, "a rank hung past the test's limit:\n" + err[-2000:]
        assert rc != 0, err[-2000:]
        assert secs < 60, (secs, err[-2000:])
    err0 = res[0][1]
    assert "deadline (RMC_DIST_TIMEOUT_S)" in err0 and "level 2" in err0 and "phase" in err0, err0[-2000:]
    assert "RMC_DIST_STALL_RANK" in res[1][1], res[1][1][-2000:]
    assert not (tmp_path / "r.json").exists()


RCCL_INIT_ALONE = r"""
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], 'raft.tla_amd'))
import rmc
cfg = rmc.make_config(n_servers=2, n_values=1, max_term=2, max_log_len=1, max_msgs=2, max_dup=1,
                      device=0, state_capacity=1 << 16)
with rmc.Checker(cfg) as ck:
    try:
        ck.shard(0, 2, rccl_id=rmc.rccl_unique_id())  # rank 1 never comes
    except rmc.RmcError as e:
        print("REFUSED", e, flush=True)
        os._exit(0)
print("JOINED", flush=True)
os._exit(1)
"""


@pytest.mark.gpu
def test_rccl_communicator_init_has_a_deadline(tmp_path):
    """The RCCL path itself (one GPU on the box): a world-2 communicator whose
    second rank never arrives.  The non-blocking init is polled under
    RMC_DIST_TIMEOUT_S and aborted; rmc_shard fails naming the deadline
    instead of blocking forever."""
    script = tmp_path / "alone.py"
    script.write_text(RCCL_INIT_ALONE)
    env = dict(os.environ, RMC_DIST_TIMEOUT_S="4")
    r = subprocess.run([sys.executable, str(script), ROOT], capture_output=True, text=True, timeout=100, env=env,
                       cwd=ROOT)
    assert "REFUSED" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    assert "deadline" in r.stdout and "communicator init" in r.stdout, r.stdout
