"""GPU parity tests: the HIP engine (through the C ABI) against the oracles.

Bit-exact bar (integer work): distinct/generated counts, per-level new-state
counts, depth, violation depth, and per-lane successor sets on fuzzed states
must equal the oracle's."""
import json
import os
import random
import sys
from collections import Counter, defaultdict

import pytest

import rmc
from oracle import raft_spec as R
from tests.convert import check_trace, from_view, random_state, random_state_edge, to_view

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_levels.json")))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cfg_from(p, capacity=1 << 25):
    return rmc.make_config(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                           max_log_len=p["max_log_len"], max_msgs=p["max_msgs"],
                           max_dup=p["max_dup"], symmetry=bool(p["symmetry"]),
                           bug_quorum=bool(p["bug_quorum"]), invariants=p["invariants"],
                           max_depth=p["max_depth"], state_capacity=capacity)


def run(cfg):
    with rmc.Checker(cfg) as ck:
        res = ck.run()
        levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
        trace = ck.trace() if (res.violated_inv or res.deadlock) else None
    return res, levels, trace


def test_kat_first_levels():
    """SURVEY.md §4 KATs: 1/3/18 new states, 6 and 27 generated (levels 1-2)."""
    cfg = rmc.make_config(max_term=14, max_log_len=3, max_msgs=8, max_dup=3, max_depth=3,
                          state_capacity=1 << 16)
    res, levels, _ = run(cfg)
    assert levels == [1, 3, 18]
    assert (res.generated, res.distinct, res.depth, res.left_on_queue) == (34, 22, 3, 18)
    cfg = rmc.make_config(max_term=14, max_log_len=3, max_msgs=8, max_dup=3, max_depth=3,
                          symmetry=True, state_capacity=1 << 16)
    res, levels, _ = run(cfg)
    assert levels == [1, 1, 5]
    assert res.generated == 1 + 6 + 9


BFS_CASES = ["bounded_full", "tiny2", "messages_tiny2", "elections_small", "tiny2_v2", "small", "small_sym", "s3_v1_msgs1", "bounded_prefix14",
             "bounded_sym_prefix16", "msgs5_dup2_prefix9", "s4_prefix10", "s5_prefix9", "isprefix_small",
             "isprefix_s3v1_log2", "s4_sym_prefix16", "s5_sym_prefix16", "tiny2_log3", "s3_log3_prefix14"]


@pytest.mark.parametrize("name", BFS_CASES)
def test_bfs_matches_oracle(name):
    g = GOLDEN[name]
    res, levels, _ = run(cfg_from(g["params"], capacity=max(1 << 25, int(g["distinct"] * 1.25))))
    assert levels == g["level_new"]
    assert res.distinct == g["distinct"]
    assert res.generated == g["generated"]
    assert res.depth == g["depth"]
    assert res.left_on_queue == g["left_on_queue"]
    assert res.violated_inv == 0 and res.deadlock == 0


def test_set_bytes_sizes_the_fingerprint_set():
    """rmc_config.set_bytes (TLC -fpmem) sizes the fingerprint set apart from the
    store: a set just large enough for the run (load <= 0.5) gives the oracle's
    counts, resident and spilling; a set too small for the run stops with a
    capacity error at the level that passes it, not a wrong count; a
    state_capacity the set cannot hold is refused at create."""
    g = GOLDEN["bounded_full"]  # 78.1 M states
    slots = 1 << (2 * g["distinct"] - 1).bit_length()  # 2^28
    for spill in (False, True):
        cfg = cfg_from(g["params"], capacity=0)
        cfg.set_bytes = slots * 8 + 4095  # rounded down to a power of two of slots
        if spill:
            cfg.flags |= rmc.FLAG_SPILL
        res, levels, _ = run(cfg)
        assert levels == g["level_new"] and res.distinct == g["distinct"] and res.generated == g["generated"]
    cfg = cfg_from(g["params"], capacity=0)
    cfg.set_bytes = slots * 4  # holds 67.1 M states
    with pytest.raises(rmc.RmcError) as e:
        run(cfg)
    assert e.value.code == -28
    cfg = cfg_from(g["params"], capacity=slots)
    cfg.set_bytes = slots * 8
    with pytest.raises(rmc.RmcError) as e:
        rmc.Checker(cfg)
    assert e.value.code == -22


SMALL_LAUNCHES = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], 'raft.tla_amd'))
sys.path.insert(0, sys.argv[1])
import rmc
from tests.test_gpu import cfg_from, GOLDEN, run
out = {}
for name in ("small", "bounded_prefix14", "tiny2_v2"):
    g = GOLDEN[name]
    res, levels, _ = run(cfg_from(g["params"], capacity=max(1 << 22, int(g["distinct"] * 1.25))))
    out[name] = [levels == g["level_new"], res.distinct == g["distinct"], res.generated == g["generated"],
                 res.depth == g["depth"], int(res.expand_launches)]
print(json.dumps(out))
"""


def test_many_launches_per_level_keep_every_count(tmp_path):
    """Levels cut into many equal launches (RMC_LAUNCH_LOG2=16: launches of at
    most 65,536 states): every per-level count of three golden models (levels
    of up to 0.09-0.24 M new states) is unchanged."""
    import subprocess
    script = tmp_path / "small_launches.py"
    script.write_text(SMALL_LAUNCHES)
    env = dict(os.environ, RMC_LAUNCH_LOG2="16")
    r = subprocess.run([sys.executable, str(script), ROOT], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    for name, (lv, d, gen, dep, launches) in out.items():
        assert lv and d and gen and dep, name
        # every expanded level in launches of at most 2^16 states (bounded_prefix14's one
        # larger level is its last, never expanded)
        assert launches >= sum(-(-x // 65536) for x in GOLDEN[name]["level_new"][:-1]), (name, launches)
    assert out["small"][4] > GOLDEN["small"]["depth"] and out["tiny2_v2"][4] > GOLDEN["tiny2_v2"]["depth"]


BENCH_MODELS = {  # spec: (final distinct, generated, depth, single-GPU setup)
    "MCraftBench.cfg": ((1_227_465_177, 21_130_972_267, 56), "resident"),
    "MCraftBenchXL.cfg": ((4_132_397_328, 68_825_665_108, 75), "spill"),
}


@pytest.mark.parametrize("spec,prefix", [("MCraftBench.cfg", "bench_prefix22"), ("MCraftBench.cfg", "bench_prefix24"),
                                         ("MCraftBenchXL.cfg", "benchxl_prefix22"),
                                         ("MCraftBenchXL.cfg", "benchxl_prefix24")])
def test_bench_model_prefix_equals_oracle(spec, prefix):
    """The bench workloads themselves (through the front-end, as bench.py loads
    them), searched to their fixpoint: the first levels equal the C oracle's
    level by level (new states per level, and the distinct and generated counts
    once those levels exist), and the whole search ends with the bench line's
    counts (1.23 G and 4.13 G states: beyond the oracle's memory).  The 4.13 G-state
    round-5 bench model runs as bench.py runs it on one GPU: RMC_FLAG_SPILL with
    librmc's own sizing, its trace links in HBM."""
    g = GOLDEN[prefix]
    final, setup = BENCH_MODELS[spec]
    cfg = rmc.config_from_files(os.path.join(ROOT, "specs", spec), builtin_raft=True)
    p = g["params"]
    assert (cfg.n_servers, cfg.n_values, cfg.max_term, cfg.max_log_len, cfg.max_msgs, cfg.max_dup) == \
        (p["n_servers"], p["n_values"], p["max_term"], p["max_log_len"], p["max_msgs"], p["max_dup"])
    if setup == "resident":
        cfg.state_capacity = 1_300_000_000
    else:
        cfg.state_capacity = 0
        cfg.flags |= rmc.FLAG_SPILL
    with rmc.Checker(cfg) as ck:
        res = ck.run()
        lv = list(ck.levels)
    levels = [1] + [x[3] for x in lv if x[3]]
    d = len(g["level_new"])
    assert levels[:d] == g["level_new"]
    at = [x for x in lv if x[2] == g["distinct"]]  # the callback of the level that completed level d
    assert at and at[0][1] == g["generated"]
    assert (res.distinct, res.generated, res.depth) == final
    if setup == "spill":
        assert res.spills > 0 and res.spill_links_on_device == 1


def test_fingerprint_salt_does_not_change_counts():
    """Another member of the fingerprint family (rmc_config.seed) must give the
    same exact counts: evidence against fingerprint collisions at full size."""
    g = GOLDEN["bounded_full"]
    cfg = cfg_from(g["params"], capacity=int(g["distinct"] * 1.25))
    cfg.seed = 0xC0FFEE
    res, levels, _ = run(cfg)
    assert (res.distinct, res.generated, res.depth) == (g["distinct"], g["generated"], g["depth"])
    assert levels == g["level_new"]


@pytest.mark.parametrize("name,spill,ep_max", [("bounded_full", False, None), ("small_sym", False, None),
                                               ("small", False, "2"), ("bounded_full", True, None),
                                               ("small_sym", True, "3"), ("s5_prefix9", False, None)])
def test_set_epochs_repeated_runs_equal_the_oracle(name, spill, ep_max, monkeypatch):
    """Set epochs (raft_packed.h c_set_ep): runs after a ctx's first take the next
    epoch instead of clearing the fingerprint set, and the earlier runs' entries
    read as empty.  Six runs on one ctx, alternating two fingerprint salts (the
    same states land in other slots under other keys), each equal to the oracle
    level by level; RMC_SET_EPOCH=N wraps the epoch (a full clear) every N runs,
    and a run with RMC_SET_EPOCH=0 in between clears the set and leaves it untagged."""
    if ep_max is not None:
        monkeypatch.setenv("RMC_SET_EPOCH", ep_max)
    if spill:
        g, cfg = spill_cfg(name, 1 << 16)
    else:
        g = GOLDEN[name]
        cfg = cfg_from(g["params"], capacity=max(1 << 20, int(g["distinct"] * 1.25)))
    with rmc.Checker(cfg) as ck:
        for i in range(6):
            ck.set_seed(0 if i % 2 == 0 else 0x5A17ED + i)
            if i == 4:
                monkeypatch.setenv("RMC_SET_EPOCH", "0")
            elif i == 5:
                monkeypatch.setenv("RMC_SET_EPOCH", ep_max or "255")
            res = ck.run()
            levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
            assert (res.distinct, res.generated, res.depth, res.left_on_queue) == \
                (g["distinct"], g["generated"], g["depth"], g["left_on_queue"]), i
            assert levels == g["level_new"], i
            assert (res.spills > 0) == spill


def test_set_epochs_checkpoint_of_a_later_run_recovers(tmp_path):
    """A spilled checkpoint dumps the fingerprint set with its entries' epoch
    tag (header pad_); recovering it into a fresh ctx adopts that epoch, so the
    set of a ctx's third run (epoch 3) recovers like a first run's."""
    g, cfg = spill_cfg("tiny2_v2", 4096, max_depth=30)
    with rmc.Checker(cfg) as ck:
        for _ in range(3):
            r1 = ck.run()
        assert r1.depth == 30 and r1.spills > 0
        ck.checkpoint(str(tmp_path / "ck"))
    _, cfg2 = spill_cfg("tiny2_v2", 4096)
    with rmc.Checker(cfg2) as ck:
        ck.recover(str(tmp_path / "ck"))
        r2 = ck.run()
        levels = [lv[3] for lv in ck.levels if lv[3]]
        assert (r2.distinct, r2.generated, r2.depth) == (g["distinct"], g["generated"], g["depth"])
        assert levels == g["level_new"][30:]
        r3 = ck.run()  # a fresh run on the recovered ctx: the next epoch over the recovered set
        assert (r3.distinct, r3.generated, r3.depth) == (g["distinct"], g["generated"], g["depth"])


@pytest.mark.parametrize("name", ["small", "s5_prefix9", "bug_log_matching", "bounded_full", "small_sym",
                                  "s4_sym_prefix16", "sym_bug_one_leader"])
def test_full_state_verification_is_exact(name):
    """RMC_FLAG_VERIFY_STATES: every fingerprint hit is compared with the stored
    state; with 64-bit fingerprints no hit differs, so the counts are certified
    exact (and equal the oracle's exact-state counts)."""
    g = GOLDEN[name]
    cfg = cfg_from(g["params"], capacity=max(1 << 22, int(g["distinct"] * 1.25)))
    cfg.flags |= rmc.FLAG_VERIFY_STATES
    res, levels, _ = run(cfg)
    assert (res.distinct, res.generated, res.depth) == (g["distinct"], g["generated"], g["depth"])
    assert levels == g["level_new"]
    assert res.collisions == 0
    # every probe either inserted a new state or hit an existing one, and
    # every hit was compared (initial state: inserted by the seed kernel)
    assert res.verified == res.probes - (res.distinct - 1)


@pytest.mark.parametrize("bits,name", [(16, "small"), (20, "small"), (14, "small_sym")])
def test_full_state_verification_reports_collisions(bits, name):
    """A fingerprint cut to `bits` bits must collide: the search loses states
    (as TLC would, silently) and the verification reports the colliding hits;
    under SYMMETRY a hit is a collision when no server permutation maps the
    successor onto the stored state."""
    g = GOLDEN[name]
    cfg = cfg_from(g["params"], capacity=1 << 22)
    cfg.flags |= rmc.FLAG_VERIFY_STATES
    with rmc.Checker(cfg) as ck:
        ck.set_fp_bits(bits)
        res = ck.run()
    assert res.distinct <= 1 << bits
    assert res.distinct < g["distinct"]
    assert res.collisions > 0
    assert res.verified == res.probes - (res.distinct - 1)


@pytest.mark.parametrize("name", ["bug_one_leader", "sym_bug_one_leader", "bug_log_matching", "bug_both", "bug_messages",
                                  "messages_small", "bug_leader_votes", "bug_cand_term", "votes_granted_small",
                                  "bug_votes_granted", "bug_quorum_log", "bug_more_up_to_date",
                                  "bug_leader_complete"])
def test_bug_variant_violation_and_trace(name):
    g = GOLDEN[name]
    p = g["params"]
    res, levels, trace = run(cfg_from(p))
    assert res.violated_inv == g["violated_inv"]
    assert res.violation_depth == g["violation_depth"]
    assert res.distinct == g["distinct"] and res.generated == g["generated"]
    # the trace is a behaviour of the spec from Init to a violating state
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                    max_log=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                    bug_quorum=bool(p["bug_quorum"]))
    check_trace(model, trace, res.violated_inv, res.violation_depth)


FUZZ = [
    dict(n_servers=3, n_values=2, max_term=3, max_log=2, max_msgs=4, max_dup=2),
    dict(n_servers=3, n_values=2, max_term=4, max_log=3, max_msgs=7, max_dup=3),
    dict(n_servers=2, n_values=1, max_term=2, max_log=1, max_msgs=2, max_dup=1),
    dict(n_servers=4, n_values=2, max_term=3, max_log=2, max_msgs=4, max_dup=2),
    dict(n_servers=5, n_values=2, max_term=3, max_log=3, max_msgs=6, max_dup=2),
    dict(n_servers=3, n_values=2, max_term=3, max_log=3, max_msgs=4, max_dup=1, bug_quorum=True),
]


@pytest.mark.parametrize("k", range(len(FUZZ)))
def test_expand_matches_oracle_on_fuzzed_states(k):
    """Differential fuzzing in the spirit of SmokeInit:
    every lane of random type-correct states, GPU vs the Python restatement."""
    m = R.Model(**FUZZ[k])
    rng = random.Random(1000 + k)
    compare_expand(m, [random_state(m, rng) for _ in range(600)])


FUZZ_EDGE = [
    dict(n_servers=3, n_values=2, max_term=14, max_log=3, max_msgs=8, max_dup=3),
    dict(n_servers=5, n_values=2, max_term=14, max_log=3, max_msgs=8, max_dup=3),
    dict(n_servers=2, n_values=1, max_term=14, max_log=3, max_msgs=4, max_dup=3, bug_quorum=True),
    dict(n_servers=4, n_values=2, max_term=13, max_log=2, max_msgs=8, max_dup=2),
]


@pytest.mark.parametrize("k", range(len(FUZZ_EDGE)))
def test_expand_matches_oracle_at_capacity_edges(k):
    """The same differential test at the packed capacity's edges (terms 13-15,
    3-entry logs, counts at MaxDup, a full 8-slot bag, mprevLogIndex = -1):
    successors beyond a field's width must leave the CONSTRAINT, never wrap."""
    m = R.Model(**FUZZ_EDGE[k])
    rng = random.Random(2000 + k)
    compare_expand(m, [random_state_edge(m, rng) for _ in range(800)])


def compare_expand(m, states):
    cfg = rmc.make_config(n_servers=m.n_servers, n_values=m.n_values, max_term=m.max_term,
                          max_log_len=m.max_log, max_msgs=m.max_msgs, max_dup=m.max_dup,
                          bug_quorum=m.bug_quorum, state_capacity=1 << 12)
    with rmc.Checker(cfg) as ck:
        out = ck.expand([to_view(m, s) for s in states])
    gpu_gen = defaultdict(Counter)
    gpu_in = defaultdict(Counter)
    fps = {}
    for sv in out:
        fam = rmc.FAMILIES[sv.family]
        gpu_gen[sv.parent][fam] += 1
        if sv.in_constraint:
            t = from_view(sv.state)
            gpu_in[sv.parent][(fam, t)] += 1
            assert fps.setdefault(t, sv.fingerprint) == sv.fingerprint  # fp is a function of the state
    for idx, s in enumerate(states):
        ora_gen = Counter()
        ora_in = Counter()
        for f, _p, t in R.successors(m, s):
            ora_gen[f] += 1
            if R.in_constraint(m, t):
                ora_in[(f, t)] += 1
        assert gpu_gen[idx] == ora_gen, (idx, s)
        assert gpu_in[idx] == ora_in, (idx, s)


CLI = os.path.join(os.path.dirname(os.path.dirname(__file__)), "raft.tla_amd", "bin", "rmc-tlc")
SPECS = os.path.join(os.path.dirname(os.path.dirname(__file__)), "specs")
MODELS = os.path.join(os.path.dirname(__file__), "golden", "models")


def test_cli_bfs_summary_with_verification():
    """rmc-tlc prints TLC's summary lines; -verify adds the collision count."""
    import subprocess
    g = GOLDEN["tiny2"]
    r = subprocess.run([CLI, "-builtin-raft", "-verify", "-config", os.path.join(SPECS, "MCraftTiny2.cfg"),
                        os.path.join(SPECS, "MCraftTiny2.tla")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"{g['generated']} states generated, {g['distinct']} distinct states found, 0 states left on queue." \
        in r.stdout
    assert f"The depth of the complete state graph search is {g['depth']}." in r.stdout
    assert ", 0 collisions." in r.stdout


def test_cli_simulation_mode():
    """rmc-tlc -simulate on a SmokeInit model (k = 3: 3^9 initial states, as
    Smokeraft.tla:17-19 lists); TypeOK holds on every state."""
    import subprocess
    r = subprocess.run([CLI, "-builtin-raft", "-simulate", "num=65536", "-seed", "3", os.path.join(MODELS, "SmokeFixture.tla")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "SmokeInit: 19683 initial states (k = 3)." in r.stdout
    assert "No error has been found in 65536 behaviours." in r.stdout


@pytest.mark.parametrize("name,stop", [("tiny2_v2", 9), ("small_sym", 12), ("bounded_full", 30)])
def test_checkpoint_and_recover(name, stop, tmp_path):
    """TLC -checkpoint / -recover: a search stopped at level `stop`, written,
    loaded into a fresh context (the fingerprint set is rebuilt from the
    states) and continued, ends with the full search's exact counts."""
    g = GOLDEN[name]
    p = dict(g["params"], max_depth=stop)
    cap = max(1 << 22, int(g["distinct"] * 1.25))
    with rmc.Checker(cfg_from(p, capacity=cap)) as ck:
        r1 = ck.run()
        assert r1.depth == stop and r1.left_on_queue > 0
        ck.checkpoint(str(tmp_path / "ck"))
    with rmc.Checker(cfg_from(g["params"], capacity=cap)) as ck:
        ck.recover(str(tmp_path / "ck"))
        r2 = ck.run()
        levels = [lv[3] for lv in ck.levels if lv[3]]
    assert (r2.distinct, r2.generated, r2.depth, r2.left_on_queue) == (g["distinct"], g["generated"], g["depth"], 0)
    assert levels == g["level_new"][stop:]


def test_recover_continues_to_the_violation_and_its_trace(tmp_path):
    g = GOLDEN["bug_one_leader"]
    p = g["params"]
    with rmc.Checker(cfg_from(dict(p, max_depth=6))) as ck:
        ck.run()
        ck.checkpoint(str(tmp_path / "ck"))
    with rmc.Checker(cfg_from(p)) as ck:
        ck.recover(str(tmp_path / "ck"))
        res = ck.run()
        trace = ck.trace()
    assert (res.violated_inv, res.violation_depth) == (g["violated_inv"], g["violation_depth"])
    assert (res.distinct, res.generated) == (g["distinct"], g["generated"])
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                    max_log=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"], bug_quorum=True)
    check_trace(model, trace, res.violated_inv, res.violation_depth)


def test_recover_rejects_another_model(tmp_path):
    g = GOLDEN["tiny2"]
    with rmc.Checker(cfg_from(dict(g["params"], max_depth=5))) as ck:
        ck.run()
        ck.checkpoint(str(tmp_path / "ck"))
    other = dict(g["params"], max_term=g["params"]["max_term"] + 1)
    with rmc.Checker(cfg_from(other)) as ck:
        with pytest.raises(rmc.RmcError, match="another model"):
            ck.recover(str(tmp_path / "ck"))
        with pytest.raises(rmc.RmcError, match="not an rmc checkpoint|cannot open"):
            ck.recover(str(tmp_path / "missing"))
    # a checkpoint of an older format (version 2: a shorter rmc_result in the
    # header) is refused by its version, before its fields are read
    raw = bytearray(open(tmp_path / "ck", "rb").read())
    raw[8:12] = (2).to_bytes(4, "little")
    (tmp_path / "ck2").write_bytes(bytes(raw))
    with rmc.Checker(cfg_from(dict(g["params"], max_depth=5))) as ck:
        with pytest.raises(rmc.RmcError, match="format version 2"):
            ck.recover(str(tmp_path / "ck2"))


FRONT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "front_models.json")))


@pytest.mark.parametrize("model,golden", [("MCraftBug_raft_tla_edited", "bug_both"), ("MCraftTiny2", "tiny2")])
def test_front_end_configs_from_raft_tla_run_to_the_oracle_result(model, golden):
    """Config 5 through the raft.tla file path: the rmc_config the front-end made
    from a raft.tla with line 197 weakened (tests/golden/make_front_fixtures.py,
    CPU side, where raft.tla exists) runs to the oracle's violation, depth and
    counts; likewise an unmodified model verified against raft.tla."""
    f = FRONT[model]
    g = GOLDEN[golden]
    cfg = rmc.make_config(n_servers=f["n_servers"], n_values=f["n_values"], max_term=f["max_term"],
                          max_log_len=f["max_log_len"], max_msgs=f["max_msgs"], max_dup=f["max_dup"],
                          state_capacity=1 << 25)
    cfg.flags, cfg.invariants = f["flags"], f["invariants"]
    p = g["params"]
    assert (cfg.n_servers, cfg.max_term, cfg.max_msgs, bool(cfg.flags & rmc.FLAG_BUG_QUORUM), cfg.invariants) == \
        (p["n_servers"], p["max_term"], p["max_msgs"], bool(p["bug_quorum"]), p["invariants"])
    res, levels, _trace = run(cfg)
    assert (res.distinct, res.generated, res.violated_inv, res.violation_depth) == \
        (g["distinct"], g["generated"], g["violated_inv"], g["violation_depth"])


@pytest.mark.parametrize("cfgname,golden", [("MCraftBug", "bug_both"), ("MCraftMessages", "messages_small")])
def test_cli_counterexample_is_tlc_format_and_replays(cfgname, golden, tmp_path):
    """rmc-tlc's counterexample (config 5 and the MessagesInv model): TLC's
    summary and `State k: <Action line L1, col C1 to line L2, col C2 of module
    M>` headers; tests/tla_transcript.py reads the TLA+ values back and the
    Python restatement re-validates every step, its header (the action and
    its raft.tla or override location) and the violation.  The transcript is
    kept in tmp for the committed-golden check (tests/golden/cli_*.txt)."""
    import subprocess
    from tests import tla_transcript
    g = GOLDEN[golden]
    p = g["params"]
    r = subprocess.run([CLI, "-builtin-raft", "-config", os.path.join(SPECS, cfgname + ".cfg"),
                        os.path.join(SPECS, cfgname + ".tla")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 12, r.stdout[-2000:] + r.stderr
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                    max_log=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                    bug_quorum=bool(p["bug_quorum"]))
    inv, n = tla_transcript.validate(r.stdout, model)
    assert rmc.INV_NAMES[g["violated_inv"]] == inv and n == g["violation_depth"]
    assert f"{g['generated']} states generated, {g['distinct']} distinct states found, 0 states left on queue." \
        in r.stdout
    out = os.path.join(os.path.dirname(os.path.dirname(__file__)), "gpurun_out")
    if os.path.isdir(out):
        open(os.path.join(out, f"cli_{cfgname}.txt"), "w").write(r.stdout)


@pytest.mark.parametrize("prefix,depth,at_least", [("s5_prefix9", 20, 1_348_000_000),
                                                   ("s5_wide_prefix9", 14, 1_194_000_000)])
def test_config3_full_size_is_exact_by_verification_and_salt(prefix, depth, at_least):
    """BASELINE.json config 3 at full size: specs/MCraft5.cfg (5 servers) to BFS
    depth 20, 1.35 G distinct states, and the wider-bound specs/MCraft5Wide.cfg
    (MaxTerm 3, MaxLogLen 2, MaxMsgs 4) to depth 14, 1.19 G -- beyond the
    oracles, so pinned by size-independent properties: (1) the first 9 levels
    equal the oracle fixture level by level; (2) full-state verification
    compares every fingerprint hit with the stored state and finds 0
    collisions, so the count is exact; (3) another fingerprint salt gives the
    same counts."""
    g9 = GOLDEN[prefix]
    p = dict(g9["params"], max_depth=depth)
    cfg = cfg_from(p, capacity=0)
    with rmc.Checker(cfg) as ck:
        r1 = ck.run()
        lv = [1] + [x[3] for x in ck.levels if x[3]]
        ck.set_seed(0xFEED5)
        r2 = ck.run()
    assert r1.distinct > at_least and r1.depth == depth and r1.left_on_queue > 0
    assert lv[:9] == g9["level_new"]
    assert (r2.distinct, r2.generated, r2.depth, r2.left_on_queue) == \
        (r1.distinct, r1.generated, r1.depth, r1.left_on_queue)
    cfg.flags |= rmc.FLAG_VERIFY_STATES
    with rmc.Checker(cfg) as ck:
        r3 = ck.run()
    assert (r3.distinct, r3.generated, r3.depth) == (r1.distinct, r1.generated, r1.depth)
    assert r3.collisions == 0
    assert r3.verified == r3.probes - (r3.distinct - 1)


# ---- frontier spill (RMC_FLAG_SPILL; TLC's states/ directory)

def spill_cfg(name, slack, **kw):
    """A config whose device window holds the largest two consecutive levels
    plus `slack` states — far less than the whole search — so the expanded
    levels must move to host memory for the search to complete."""
    g = GOLDEN[name]
    p = dict(g["params"], **kw)
    L = g["level_new"]
    cfg = cfg_from(p, capacity=max(1 << 20, int(g["distinct"] * 1.25)))
    cfg.flags |= rmc.FLAG_SPILL
    cfg.device_window = max(a + b for a, b in zip(L, L[1:])) + slack
    return g, cfg


@pytest.fixture(params=["device", "host"])
def links(request, monkeypatch):
    """Where a spilled state's trace links live: in HBM (librmc's default when
    they fit) or in host memory (RMC_SPILL_HOST_LINKS=1, the fallback)."""
    if request.param == "host":
        monkeypatch.setenv("RMC_SPILL_HOST_LINKS", "1")
    return request.param


@pytest.mark.parametrize("name,slack", [("bounded_full", 1 << 22), ("small", 1 << 16), ("small_sym", 1 << 14),
                                        ("tiny2_v2", 4096), ("tiny2", 4096)])
def test_spill_completes_with_the_oracle_counts(name, slack, links):
    g, cfg = spill_cfg(name, slack)
    assert cfg.device_window < g["distinct"]
    res, levels, _ = run(cfg)
    assert res.spill_links_on_device == (links == "device")
    assert levels == g["level_new"]
    assert (res.distinct, res.generated, res.depth, res.left_on_queue) == \
        (g["distinct"], g["generated"], g["depth"], g["left_on_queue"])
    assert res.spills > 0
    # resident at the end: at most the window (the ring of device links rounds it up to a power of two)
    assert res.distinct - res.spilled <= (cfg.device_window if links == "host" else 2 * cfg.device_window)


# (with the links in HBM the window is a ring of a power of two states: the cases
# whose ring still wraps before the violation — a violation search usually ends at
# its largest level)
@pytest.mark.parametrize("name,mode", [("bug_one_leader", "host"), ("messages_small", "host"),
                                       ("sym_bug_one_leader", "host"), ("messages_small", "device"),
                                       ("bug_votes_granted", "device"), ("bug_quorum_log", "device")])
def test_spill_trace_equals_the_resident_trace(name, mode, monkeypatch):
    """The counterexample walks parents through spilled states (replayed from
    Init) and the device window; it must be a behaviour of the spec to a
    violating state at the depth the resident run reports (which parent wins a
    race depends on the launch sizes, so the two traces may differ state by state)."""
    if mode == "host":
        monkeypatch.setenv("RMC_SPILL_HOST_LINKS", "1")
    g, cfg = spill_cfg(name, 2048)
    res, _, trace = run(cfg)
    assert res.spills > 0 and res.spill_links_on_device == (mode == "device")
    base, _, trace0 = run(cfg_from(g["params"]))
    assert (res.violated_inv, res.violation_depth, res.distinct, res.generated) == \
        (base.violated_inv, base.violation_depth, base.distinct, base.generated) == \
        (g["violated_inv"], g["violation_depth"], g["distinct"], g["generated"])
    assert len(trace) == len(trace0) == g["violation_depth"]
    p = g["params"]
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                    max_log=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                    bug_quorum=bool(p["bug_quorum"]))
    check_trace(model, trace, res.violated_inv, res.violation_depth)


@pytest.mark.parametrize("name,slack", [("bounded_full", 1 << 22), ("small", 1 << 16), ("small_sym", 1 << 14)])
def test_verification_with_spill_is_exact(name, slack, links):
    """RMC_FLAG_VERIFY_STATES with RMC_FLAG_SPILL: every fingerprint hit is
    compared with the stored state that owns it, also when that state has left
    the device window (its host copy, k_verify_host); the oracle's counts, no
    collision, and every hit compared."""
    g, cfg = spill_cfg(name, slack)
    cfg.flags |= rmc.FLAG_VERIFY_STATES
    res, levels, _ = run(cfg)
    assert res.spills > 0 and res.spill_links_on_device == (links == "device")
    assert levels == g["level_new"]
    assert (res.distinct, res.generated, res.depth) == (g["distinct"], g["generated"], g["depth"])
    assert res.collisions == 0
    assert res.verified == res.probes - (res.distinct - 1)
    assert 0 < res.verified_spilled <= res.verified


@pytest.mark.parametrize("bits,name", [(20, "small"), (20, "small_sym")])
def test_verification_with_spill_reports_collisions(bits, name, links):
    """A weakened fingerprint under spill: the collisions are reported, including
    those whose stored state had left the device window."""
    g, cfg = spill_cfg(name, 1 << 14)
    cfg.flags |= rmc.FLAG_VERIFY_STATES
    with rmc.Checker(cfg) as ck:
        ck.set_fp_bits(bits)
        res = ck.run()
    assert res.spills > 0
    assert res.distinct < g["distinct"]
    assert res.collisions > 0
    assert res.verified == res.probes - (res.distinct - 1)
    assert res.verified_spilled > 0


def test_verification_with_spill_refuses_checkpoints(tmp_path):
    g, cfg = spill_cfg("tiny2_v2", 4096, max_depth=30)
    cfg.flags |= rmc.FLAG_VERIFY_STATES
    with rmc.Checker(cfg) as ck:
        r1 = ck.run()
        assert r1.depth == 30 and r1.spills > 0 and r1.collisions == 0
        with pytest.raises(rmc.RmcError, match="VERIFY_STATES and RMC_FLAG_SPILL"):
            ck.checkpoint(str(tmp_path / "ck"))


@pytest.mark.parametrize("first,second", [("spill", "spill"), ("resident", "spill"), ("spill", "resident")])
def test_spill_checkpoint_and_recover(first, second, tmp_path, links):
    """A spilled search checkpoints its trace links, frontier and fingerprint
    set (the spilled states no longer exist) and recovers into a spilling
    context; a resident checkpoint recovers into a spilling context by
    streaming the old states through the window to rebuild the set; a spilled
    checkpoint cannot become resident."""
    g, scfg = spill_cfg("tiny2_v2", 4096, max_depth=30)
    cfg = scfg if first == "spill" else cfg_from(dict(g["params"], max_depth=30),
                                                 capacity=scfg.state_capacity)
    with rmc.Checker(cfg) as ck:
        r1 = ck.run()
        assert r1.depth == 30 and (r1.spills > 0) == (first == "spill")
        ck.checkpoint(str(tmp_path / "ck"))
    _, cfg2 = spill_cfg("tiny2_v2", 4096)
    if second == "resident":
        cfg2.flags &= ~rmc.FLAG_SPILL
        with rmc.Checker(cfg2) as ck:
            with pytest.raises(rmc.RmcError, match="spilled checkpoint"):
                ck.recover(str(tmp_path / "ck"))
        return
    with rmc.Checker(cfg2) as ck:
        ck.recover(str(tmp_path / "ck"))
        r2 = ck.run()
        levels = [lv[3] for lv in ck.levels if lv[3]]
    assert (r2.distinct, r2.generated, r2.depth, r2.left_on_queue) == (g["distinct"], g["generated"], g["depth"], 0)
    assert levels == g["level_new"][30:]
    assert r2.spills > r1.spills  # the recovered result carries the checkpointed statistics forward


@pytest.mark.parametrize("name,stop,mode", [("bug_one_leader", 9, "host"), ("bug_quorum_log", 15, "device")])
def test_spill_recover_to_the_violation_replays_the_trace(tmp_path, name, stop, mode, monkeypatch):
    if mode == "host":
        monkeypatch.setenv("RMC_SPILL_HOST_LINKS", "1")
    g, cfg = spill_cfg(name, 2048, max_depth=stop)
    with rmc.Checker(cfg) as ck:
        ck.run()
        ck.checkpoint(str(tmp_path / "ck"))
    _, cfg = spill_cfg(name, 2048)
    with rmc.Checker(cfg) as ck:
        ck.recover(str(tmp_path / "ck"))
        res = ck.run()
        trace = ck.trace()
    assert res.spills > 0  # the last levels outgrow the window: the trace replays spilled states
    assert res.spill_links_on_device == (mode == "device")
    assert (res.violated_inv, res.violation_depth, res.distinct, res.generated) == \
        (g["violated_inv"], g["violation_depth"], g["distinct"], g["generated"])
    p = g["params"]
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                    max_log=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                    bug_quorum=bool(p["bug_quorum"]))
    check_trace(model, trace, res.violated_inv, res.violation_depth)


def test_spill_window_too_small_is_a_capacity_error():
    g, cfg = spill_cfg("small", 0)
    cfg.device_window = 4096
    with rmc.Checker(cfg) as ck:
        with pytest.raises(rmc.RmcError, match="device window"):
            ck.run()


def test_cli_spills_by_default_and_reports_it():
    import subprocess
    g = GOLDEN["tiny2"]
    L = g["level_new"]
    win = max(a + b for a, b in zip(L, L[1:])) + 4096
    r = subprocess.run([CLI, "-builtin-raft", "-window", str(win), "-config", os.path.join(SPECS, "MCraftTiny2.cfg"),
                        os.path.join(SPECS, "MCraftTiny2.tla")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"{g['generated']} states generated, {g['distinct']} distinct states found, 0 states left on queue." \
        in r.stdout
    assert "expanded states out of the device window" in r.stdout and "trace links kept in HBM" in r.stdout


@pytest.mark.gpu
def test_diamond_skipping_cuts_probes_not_states(monkeypatch):
    """Commuting-diamond elimination (raft_packed.h) on the GPU: the 78 M-state
    model gives the oracle's exact counts with and without it (RMC_DIAMOND=0),
    and with it the fingerprint set sees >= 20 % fewer probes."""
    g = GOLDEN["bounded_full"]
    p = g["params"]
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("RMC_DIAMOND", flag)
        cfg = rmc.make_config(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                              max_log_len=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                              state_capacity=1 << 27)
        with rmc.Checker(cfg) as ck:
            r = ck.run()
            res[flag] = (r.distinct, r.generated, r.depth, r.probes, [lv[3] for lv in ck.levels if lv[3]])
    for flag in ("0", "1"):
        assert res[flag][:3] == (g["distinct"], g["generated"], g["depth"]), flag
        assert [1] + res[flag][4] == g["level_new"], flag
    assert res["1"][3] <= 0.8 * res["0"][3], (res["1"][3], res["0"][3])


@pytest.mark.gpu
def test_unconstrained_model_under_a_depth_bound():
    """MCraft.cfg as shipped has no CONSTRAINT; under -depth
    it runs level by level.  Fixture in its layout:
    depth 3 gives the survey's KAT (1 + 3 + 18 = 22 distinct, 1 + 6 + 27 = 34
    generated); depths 4-5 equal the C oracle.  Its unbounded fields run on the
    wide layout (depth 6 needed a 4th copy of a message, beyond the packed
    layout: tests/test_wide.py takes it to depth 8); a field that outgrows the
    wide layout is RMC_E_CAPACITY naming it, never a silent filter.  The CLI
    prints TLC's lines for the depth-3 run."""
    import subprocess
    from tests import oracle_c
    cfgp = os.path.join(ROOT, "tests", "golden", "models", "MCunbounded.cfg")
    base, _, _ = rmc.model_from_files(cfgp, builtin_raft=True, depth_bounded=True)
    for depth in (3, 4, 5):
        c = rmc.Config.from_buffer_copy(base)
        c.max_depth = depth
        c.state_capacity = 1 << 22
        with rmc.Checker(c) as ck:
            r = ck.run()
        ref, _, _ = oracle_c.bfs(3, 2, 14, 3, 8, 3, threads=4, max_levels=depth, capacity=1 << 22)
        assert (r.distinct, r.generated, r.depth) == (ref.distinct, ref.generated, ref.depth), depth
        if depth == 3:
            assert (r.distinct, r.generated, r.left_on_queue) == (22, 34, 18)
    exe = os.path.join(ROOT, "raft.tla_amd", "bin", "rmc-tlc")
    out = subprocess.run([exe, "-depth", "3", "-builtin-raft", "-config", cfgp,
                          os.path.join(ROOT, "tests", "golden", "models", "MCunbounded.tla")],
                         capture_output=True, text=True, timeout=120)
    assert "34 states generated, 22 distinct states found, 18 states left on queue." in out.stdout, out.stdout
