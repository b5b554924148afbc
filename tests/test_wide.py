"""The wide layout (raft.tla_amd/csrc/raft_wide.h): models whose fields
outgrow the packed layout — the reference's own MCraft.cfg (no CONSTRAINT)
under a depth bound, Smokeraft's unbounded depth-100 walks, bounds beyond
MaxTerm 14 / MaxLogLen 3 / 8 messages / count 3.

Parity: the same per-level counts as the C oracle (oracle/rmc_oracle.c), the
same successor sets as the Python restatement (oracle/raft_spec.py) on states
far beyond the packed capacity, and replayed walks that are behaviours of
the spec.  RMC_FORCE_WIDE=1 puts packed-size golden models on the wide layout
to compare the two layouts on the same search."""
import json
import os
import random
from collections import Counter

import pytest

import rmc
from oracle import raft_spec as R
from tests import oracle_c
from tests.convert import check_trace, from_view, to_view

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_levels.json")))


@pytest.fixture
def force_wide(monkeypatch):
    monkeypatch.setenv("RMC_FORCE_WIDE", "1")


def cfg_from(p, capacity=1 << 20):
    return rmc.make_config(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"],
                           max_log_len=p["max_log_len"], max_msgs=p["max_msgs"], max_dup=p["max_dup"],
                           bug_quorum=bool(p["bug_quorum"]), invariants=p["invariants"],
                           max_depth=p["max_depth"], state_capacity=capacity)


RECORDS = {"full": ("0", 5080), "compact": ("1", 904), "depth": ("2", 336)}


@pytest.fixture(params=["full", "compact", "depth"])
def wide_record(request, monkeypatch):
    """The BFS store's record: full (5,080 B), compact (904 B, WStateC) or
    depth-sized (336 B, WStateD)."""
    monkeypatch.setenv("RMC_WIDE_COMPACT", RECORDS[request.param][0])
    return RECORDS[request.param][1]


@pytest.mark.parametrize("name", ["tiny2", "tiny2_v2", "small", "s4_prefix10", "msgs5_dup2_prefix9"])
def test_wide_layout_matches_oracle_levels(name, force_wide, wide_record):
    """The wide layout (both records) on packed-size golden models: every
    per-level count, distinct, generated and depth equal the oracle's."""
    g = GOLDEN[name]
    with rmc.Checker(cfg_from(g["params"], capacity=max(1 << 20, int(g["distinct"] * 1.25)))) as ck:
        assert rmc.native().rmc_state_bytes(ck.cfg) == wide_record
        r = ck.run()
        levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
    assert levels == g["level_new"]
    assert (r.distinct, r.generated, r.depth, r.left_on_queue) == (g["distinct"], g["generated"], g["depth"],
                                                                  g["left_on_queue"])


@pytest.mark.parametrize("name", ["bug_one_leader", "bug_log_matching", "messages_small"])
def test_wide_layout_violation_and_trace(name, force_wide, wide_record):
    g = GOLDEN[name]
    p = g["params"]
    with rmc.Checker(cfg_from(p, capacity=int(g["distinct"] * 1.25) + (1 << 16))) as ck:  # 5-KB records
        r = ck.run()
        trace = ck.trace()
    assert r.violated_inv == g["violated_inv"] and r.violation_depth == g["violation_depth"]
    assert (r.distinct, r.generated) == (g["distinct"], g["generated"])
    model = R.Model(n_servers=p["n_servers"], n_values=p["n_values"], max_term=p["max_term"], max_log=p["max_log_len"],
                    max_msgs=p["max_msgs"], max_dup=p["max_dup"], bug_quorum=bool(p["bug_quorum"]))
    check_trace(model, trace, r.violated_inv, r.violation_depth)


def test_reference_mcraft_cfg_under_a_depth_bound():
    """the reference's MCraft.cfg layout (no CONSTRAINT,
    tests/golden/models/MCunbounded) runs past the packed capacity — depth 6
    needed a 4th copy of a message (Duplicate) — to depth 8 on the wide
    layout, level by level equal to the C oracle run with terms and counts
    unbounded and log / bag bounds no state of those depths reaches."""
    cfgp = os.path.join(ROOT, "tests", "golden", "models", "MCunbounded.cfg")
    base, _, _ = rmc.model_from_files(cfgp, builtin_raft=True, depth_bounded=True)
    assert (base.max_term, base.max_log_len, base.max_msgs, base.max_dup) == (255, 32, 64, 255)
    for depth in (6, 7, 8):
        c = rmc.Config.from_buffer_copy(base)
        c.max_depth = depth
        c.state_capacity = 1 << 18  # 56,761 states at depth 8
        assert rmc.native().rmc_state_bytes(c) == 336  # 7 steps: the depth-sized record holds every state
        with rmc.Checker(c) as ck:
            r = ck.run()
            levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
        # terms and counts unbounded (-1); Len(log) <= 3 and 8 messages never bind
        # within 7 steps (a leader needs 5 steps before its first ClientRequest)
        ref, ln, _ = oracle_c.bfs(3, 2, -1, 3, 8, -1, threads=8, max_levels=depth, capacity=1 << 25)
        assert (r.distinct, r.generated, r.depth, r.left_on_queue) == (ref.distinct, ref.generated, ref.depth,
                                                                      ref.left_on_queue), depth
        assert levels == ln, depth


@pytest.mark.parametrize("depth,record", [(12, "depth"), (12, "compact"), (10, "full")])
def test_reference_mcraft_cfg_deeper_on_the_record_sized_from_the_run(depth, record, monkeypatch):
    """MCraft.cfg as shipped (no CONSTRAINT) to depth 12 —
    24.6 M states, beyond the 8 levels the full 5-KB record was tested to — on
    the compact 904-B record the front-end picks for depth <= 17, and on the full
    record at depth 10: every per-level count, distinct, generated and the queue
    equal the C oracle build holding logs of 8 and 12 messages
    (tests/golden/oracle_levels.json mcraft_shipped_d12).  One GPU completes
    depth 13 on the compact record (110.9 M states; profiles/r05/wide5/)."""
    g = GOLDEN["mcraft_shipped_d12"]
    monkeypatch.setenv("RMC_WIDE_COMPACT", RECORDS[record][0])
    cfgp = os.path.join(ROOT, "tests", "golden", "models", "MCunbounded.cfg")
    c, _, _ = rmc.model_from_files(cfgp, builtin_raft=True, depth_bounded=True)
    c.max_depth = depth
    c.state_capacity = int(sum(g["level_new"][:depth]) * 1.1) + 4096
    assert rmc.native().rmc_state_bytes(c) == RECORDS[record][1]
    with rmc.Checker(c) as ck:
        r = ck.run()
        levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
    assert levels == g["level_new"][:depth]
    assert r.distinct == sum(g["level_new"][:depth]) and r.depth == depth
    assert r.left_on_queue == g["level_new"][depth - 1]
    assert r.generated == sum(g["level_generated"][:depth])
    if depth == 12:
        assert (r.distinct, r.generated) == (g["distinct"], g["generated"])


def test_reference_mcraft_cfg_depth_13_and_14_on_one_gpu():
    """MCraft.cfg as shipped on the depth-sized record
    (the front-end's default for depth <= 14): depth 13 gives the counts the
    compact record measured in round 5 (profiles/r05/cli/
    cli_config1_mcraft_as_shipped_depth13.txt), every level to 12 equal to the
    oracle, and depth 14 completes on one GPU."""
    g = GOLDEN["mcraft_shipped_d12"]
    cfgp = os.path.join(ROOT, "tests", "golden", "models", "MCunbounded.cfg")
    c, _, _ = rmc.model_from_files(cfgp, builtin_raft=True, depth_bounded=True)
    for depth in (13, 14):
        c.max_depth = depth
        c.state_capacity = 0
        assert rmc.native().rmc_state_bytes(c) == 336
        with rmc.Checker(c) as ck:
            r = ck.run()
            levels = [1] + [lv[3] for lv in ck.levels if lv[3]]
        assert levels[:12] == g["level_new"] and r.depth == depth
        if depth == 13:
            assert (r.distinct, r.generated) == (110878535, 542251150)
        else:
            assert r.distinct > 110878535 and r.left_on_queue == levels[-1]


def _walk_states(model, n, depth, seed):
    """Random walks from Init of the unconstrained spec (Python restatement)."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        s = R.init_state(model)
        for _ in range(rng.randint(1, depth)):
            succ = R.successors(model, s)
            s = rng.choice(succ)[2]
        out.append(s)
    return out


def _fits_wide(s):
    return (all(t <= 250 for t in s.currentTerm) and all(len(lg) <= 7 for lg in s.log) and len(s.messages) <= 15
            and all(c <= 250 for _, c in s.messages))


def test_wide_successors_equal_the_python_restatement_beyond_the_packed_capacity():
    """Every lane of the wide layout (rmc_expand) on states of long random walks
    — terms, logs, bag sizes and counts far past the packed capacity — gives
    exactly the successor multiset of Next in the Python restatement."""
    model = R.Model()
    states = [s for s in _walk_states(model, 300, 60, 7) if _fits_wide(s)]
    beyond = sum(1 for s in states if max(s.currentTerm) > 15 or max(len(x) for x in s.log) > 3
                 or len(s.messages) > 8 or any(c > 3 for _, c in s.messages))
    assert beyond > 30
    cfg = rmc.make_config(max_term=255, max_log_len=8, max_msgs=16, max_dup=255, max_depth=1, state_capacity=1 << 12)
    with rmc.Checker(cfg) as ck:
        got = ck.expand([to_view(model, s) for s in states])
    by_parent = {}
    for sv in got:
        assert sv.in_constraint
        by_parent.setdefault(sv.parent, []).append((rmc.FAMILIES[sv.family], from_view(sv.state)))
    for k, s in enumerate(states):
        want = Counter((f, t) for f, _p, t in R.successors(model, s))
        have = Counter(by_parent.get(k, []))
        assert have == want, k


def _smoke_cfg(mode_tlc=False):
    cfgp = os.path.join(ROOT, "tests", "golden", "models", "SmokeFixture.cfg")
    c, _, _ = rmc.model_from_files(cfgp, builtin_raft=True, simulate=True)
    c.state_capacity = 1 << 12
    return c


def test_smokeraft_walks_to_depth_100_without_truncation():
    """Smokeraft's walks (no bounds, Smokeraft.cfg:46-48) at
    TLC -simulate's depth 100 on the wide layout, drawn as TLC's simulator draws
    (RMC_SIM_TLC: an enabled action uniformly, then one of its successors): no
    behaviour leaves the layout, and TypeOK holds on every state."""
    c = _smoke_cfg()
    assert (c.max_term, c.max_log_len, c.max_msgs, c.max_dup) == (255, 32, 64, 255)
    with rmc.Checker(c) as ck:
        r = ck.simulate(behaviours=1 << 16, depth=100, smoke_k=2, seed=3, mode=rmc.SIM_TLC)
    assert r.init_states == 512
    assert r.violated_inv == 0
    assert r.truncated == 0, r.truncated
    assert r.steps + 100 * r.deadlocked >= (1 << 16) * 99


def test_smokeraft_uniform_successor_walks_rarely_leave_the_wide_layout():
    """The uniform-successor draw (RMC_SIM_TRUNCATE) weights actions by their
    successor counts, so its walks differ from TLC's; a behaviour whose next
    draw would need more than the wide layout holds ends there and is counted
    (the 568-B layout of 8 log entries and 16 messages lost 6.7 % of them at
    depth 100, and TLC's draw lost 82 %: hence 32 and 64)."""
    c = _smoke_cfg()
    with rmc.Checker(c) as ck:
        r = ck.simulate(behaviours=1 << 16, depth=100, smoke_k=2, seed=3, mode=rmc.SIM_TRUNCATE)
    assert r.violated_inv == 0
    assert r.truncated < (1 << 16) // 100, r.truncated
    assert r.steps + 100 * (r.deadlocked + r.truncated) >= (1 << 16) * 99


def test_smokeraft_wide_replays_are_behaviours_of_the_spec():
    model = R.Model()
    c = _smoke_cfg()
    with rmc.Checker(c) as ck:
        for b, mode in ((0, rmc.SIM_TRUNCATE), (5, rmc.SIM_TLC), (777, rmc.SIM_TLC)):
            views = ck.sim_replay(b, behaviours=1024, depth=100, smoke_k=2, seed=11, mode=mode)
            states = [from_view(v) for v in views]
            assert len(states) == 100
            for a, nxt in zip(states, states[1:]):
                assert nxt in {t for _f, _p, t in R.successors(model, a)}
            assert all(R.type_ok(model, s) for s in states)


def test_wide_capacity_edges_are_never_silently_in_the_model():
    """A lane whose successor outgrows the wide layout — a 33rd log entry, a 65th
    distinct message, a count or a term past 255 — is listed as outside the
    model (the BFS stops with RMC_E_CAPACITY on it when the field has no
    CONSTRAINT, k_wexpand); every other lane of the same state is in it."""
    model = R.Model()
    s = R.init_state(model)
    e = [R.entry(1, 0)] * 32
    s = s._replace(state=(R.LEADER, R.CANDIDATE, R.FOLLOWER), currentTerm=(1, 255, 1),
                   log=(tuple(e), (), ()))
    msgs = {}
    for k in range(64):
        m = R.rec(mtype=R.AEP, mterm=1, msuccess=False, mmatchIndex=k, msource=k % 3, mdest=(k + 1) % 3)
        msgs[m] = 255 if k == 0 else 1
    s = s._replace(messages=frozenset(msgs.items()))
    cfg = rmc.make_config(max_term=255, max_log_len=32, max_msgs=64, max_dup=255, max_depth=1, state_capacity=1 << 12)
    with rmc.Checker(cfg) as ck:
        got = ck.expand([to_view(model, s)])
    out = [(rmc.FAMILIES[sv.family], sv.instance) for sv in got if not sv.in_constraint]
    fams = Counter(f for f, _ in out)
    assert fams["ClientRequest"] == 2          # leader 0: log full (32 entries)
    assert fams["Timeout"] == 1                # candidate 1 at term 255
    assert fams["RequestVote"] == 3            # candidate 1: a 65th message
    assert fams["AppendEntries"] == 2          # leader 0: a 65th message
    assert fams["DuplicateMessage"] == 1       # the message held 255 times
    want = Counter(f for f, _p, t in R.successors(model, s))
    assert sum(want.values()) == len(got)


def _state_with_bag(model, rvq_count):
    """Server 1, a candidate of term 200 whose last log term is 200, has a
    RequestVote request to server 0 in a 64-message bag (63 stale AEP fillers)."""
    s = R.init_state(model)
    s = s._replace(state=(R.FOLLOWER, R.CANDIDATE, R.FOLLOWER), currentTerm=(200, 200, 1),
                   log=((R.entry(150, 0),), (R.entry(200, 1),), ()))
    msgs = {R.rec(mtype=R.RVQ, mterm=200, mlastLogTerm=200, mlastLogIndex=1, msource=1, mdest=0): rvq_count}
    for k in range(63):
        m = R.rec(mtype=R.AEP, mterm=1, msuccess=False, mmatchIndex=k, msource=(k + 1) % 3, mdest=2)
        msgs[m] = 1
    return s._replace(messages=frozenset(msgs.items()))


@pytest.mark.parametrize("rvq_count", [1, 2])
def test_wide_terms_above_127_and_reply_capacity_of_the_net_bag(rvq_count):
    """(1) a RequestVote request's mlastLogTerm is a term, up to 255:
    server 0 (last log term 150) must grant a request whose last log term is 200
    (logOk, raft.tla:249-251) — a signed byte read it as -56; (2) Reply
    (raft.tla:102-103) removes the request as it adds the response, so in a full
    64-message bag a count-1 request's reply is in the model (the request's slot
    is freed) and a count-2 one's is not (a 65th message).  Every in-constraint
    successor equals the Python restatement's."""
    model = R.Model()
    s = _state_with_bag(model, rvq_count)
    assert len(s.messages) == 64
    cfg = rmc.make_config(max_term=255, max_log_len=32, max_msgs=64, max_dup=255, max_depth=1, state_capacity=1 << 12)
    with rmc.Checker(cfg) as ck:
        got = ck.expand([to_view(model, s)])
    have = Counter((rmc.FAMILIES[sv.family], from_view(sv.state)) for sv in got if sv.in_constraint)
    want = Counter((f, t) for f, _p, t in R.successors(model, s) if len(t.messages) <= 64)
    assert have == want
    assert sum(1 for _ in got) == sum(1 for _ in R.successors(model, s))
    granted = [t for f, t in have if f == "Receive" and any(
        R.rget(m, "mtype") == R.RVP and R.rget(m, "mvoteGranted") for m, _c in t.messages)]
    assert len(granted) == (1 if rvq_count == 1 else 0)
    # the request's own sender re-sends: mlastLogTerm 200 decodes as 200
    rv = [t for f, t in have if f == "RequestVote"]
    assert rv and all(R.rget(m, "mlastLogTerm") == 200 for t in rv for m, _c in t.messages
                      if R.rget(m, "mtype") == R.RVQ)


_SIM_PROBE = r"""
import hashlib, json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "raft.tla_amd"))
sys.path.insert(0, sys.argv[1])
import rmc
from tests.convert import from_view
c, _, _ = rmc.model_from_files(os.path.join(sys.argv[1], "tests", "golden", "models", "SmokeFixture.cfg"),
                               builtin_raft=True, simulate=True)
c.state_capacity = 1 << 12
out = {}
with rmc.Checker(c) as ck:
    for mode in (rmc.SIM_WITHIN_CAPACITY, rmc.SIM_TRUNCATE, rmc.SIM_TLC):
        r = ck.simulate(behaviours=4096, depth=100, smoke_k=2, seed=5, mode=mode)
        views = ck.sim_replay(77, behaviours=4096, depth=100, smoke_k=2, seed=5, mode=mode)
        h = hashlib.sha256(repr([from_view(v) for v in views]).encode()).hexdigest()
        out[mode] = [r.steps, r.truncated, r.deadlocked, r.violated_inv, len(views), h]
print(json.dumps(out))
"""


def test_wave_simulator_draws_the_thread_simulators_behaviours():
    """k_wsimulate_w (one wave per behaviour: guards, apply, TypeOK and the
    CONSTRAINT spread over the lanes, the bag moved one message per lane) walks
    exactly the behaviours of k_wsimulate (one thread per behaviour, the serial
    lane code) from the same seeds: equal step, truncation, deadlock and
    violation tallies in every draw mode, and an identical replayed behaviour."""
    import subprocess
    import sys
    res = []
    for wsim in ("0", "1"):
        env = dict(os.environ, RMC_WSIM=wsim, PYTHONHASHSEED="0")  # frozenset reprs in one order
        p = subprocess.run([sys.executable, "-c", _SIM_PROBE, ROOT], env=env, capture_output=True, text=True,
                           timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        res.append(json.loads(p.stdout.strip().splitlines()[-1]))
    assert res[0] == res[1]
    for mode, (steps, _t, _d, viol, nviews, _h) in res[1].items():
        assert steps > 4096 * 50 and viol == 0 and nviews >= 2, (mode, res[1][mode])
