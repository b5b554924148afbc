"""Simulation mode (TLC -simulate on Smokeraft.cfg).

Pinned by: the SmokeInit initial-state counts k^9 (Smokeraft.tla:18: 1, 512,
19683 for k = 1..3), the Smoke domains of every initial state
(Smokeraft.tla:11-15, 24-76), and every step of replayed behaviours being a
successor under the Python restatement of Next.  Which successor TLC's
simulator picks is random, so parity with TLC is distributional only."""
import pytest

import rmc
from oracle import raft_spec as R
from tests.convert import from_view

pytestmark = pytest.mark.gpu


def smoke_cfg(**kw):
    # MaxMsgs 8 selects the 8-slot bag; simulation applies no CONSTRAINT
    return rmc.make_config(n_servers=3, n_values=2, max_term=14, max_log_len=3, max_msgs=8, max_dup=3,
                           state_capacity=1 << 12, **kw)


@pytest.mark.parametrize("k,n", [(1, 1), (2, 512), (3, 19683)])
def test_smokeinit_counts(k, n):
    with rmc.Checker(smoke_cfg()) as ck:
        r = ck.simulate(behaviours=1024, depth=1, smoke_k=k, seed=7)
    assert r.init_states == n
    assert r.steps == 0 and r.violated_inv == 0


def in_smoke_domains(s, nat=2):
    S = range(3)
    ok = all(0 <= t <= nat for t in s.currentTerm) and all(0 <= c <= nat for c in s.commitIndex)
    ok &= all(len(lg) <= 3 and all(0 <= R.rget(e, "term") <= nat for e in lg) for lg in s.log)
    ok &= all(1 <= n <= nat for row in s.nextIndex for n in row)
    ok &= all(0 <= n <= nat for row in s.matchIndex for n in row)
    ok &= all(c == 1 for _m, c in s.messages) and len(s.messages) == 2
    for m, _c in s.messages:
        d = dict(m)
        ok &= 0 <= d["mterm"] <= nat and d["msource"] in S and d["mdest"] in S
        if d["mtype"] == R.AEQ:
            ok &= -1 <= d["mprevLogIndex"] <= 1 and len(d["mentries"]) <= 1
        if d["mtype"] == R.RVP:
            ok &= len(d["mlog"]) <= 1
    return ok


def test_replayed_behaviours_are_behaviours_of_the_spec():
    model = R.Model()  # no CONSTRAINT in simulation
    with rmc.Checker(smoke_cfg()) as ck:
        for b in (0, 1, 2, 777):
            states = [from_view(v) for v in ck.sim_replay(b, behaviours=1024, depth=40, smoke_k=2,
                                                          seed=11)]
            assert len(states) >= 2
            assert in_smoke_domains(states[0])
            for a, nxt in zip(states, states[1:]):
                assert nxt in {t for _f, _p, t in R.successors(model, a)}
            assert all(R.type_ok(model, s) for s in states)


def test_simulation_runs_at_scale():
    """Default mode: draws among the successors within the packed capacity, so
    behaviours run to depth 100 (TLC -simulate's default depth)."""
    with rmc.Checker(smoke_cfg()) as ck:
        r = ck.simulate(behaviours=1 << 18, depth=100, smoke_k=2, seed=3)
    assert r.behaviours == 1 << 18
    assert r.violated_inv == 0  # TypeOK holds (Smokeraft.cfg:38-39)
    assert r.truncated == 0
    assert r.steps + 100 * r.deadlocked >= (1 << 18) * 99


def test_simulation_truncate_mode_counts_capacity_exits():
    """RMC_SIM_TRUNCATE draws among all enabled successors (TLC's distribution
    while the state fits) and ends a behaviour whose draw exceeds the packed
    capacity; such behaviours are counted, never silently dropped."""
    with rmc.Checker(smoke_cfg()) as ck:
        r = ck.simulate(behaviours=1 << 16, depth=100, smoke_k=2, seed=3, mode=1)
    assert r.violated_inv == 0
    assert r.truncated > 0
    assert r.steps < (1 << 16) * 99
    assert r.truncated + r.deadlocked <= 1 << 16


def test_simulation_finds_the_injected_bug():
    """Config 5's bug (BecomeLeader with votesGranted /= {}) is found by random
    simulation from Init too; the reported state index is a real violation."""
    cfg = rmc.make_config(n_servers=3, n_values=2, max_term=14, max_log_len=3, max_msgs=8, max_dup=3,
                          bug_quorum=True, invariants=rmc.INV_ONE_LEADER, state_capacity=1 << 12)
    with rmc.Checker(cfg) as ck:
        r = ck.simulate(behaviours=1 << 20, depth=100, smoke_k=0, seed=5)
        assert r.violated_inv == rmc.INV_ONE_LEADER
        states = [from_view(v) for v in ck.sim_replay(r.violation_behaviour, behaviours=1 << 20,
                                                      depth=100, smoke_k=0, seed=5)]
    model = R.Model(bug_quorum=True)
    assert len(states) == r.violation_depth
    assert states[0] == R.init_state(model)
    assert not R.one_leader_per_term(model, states[-1])
    assert all(R.one_leader_per_term(model, s) for s in states[:-1])
