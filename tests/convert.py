"""Conversions between oracle values (oracle/raft_spec.py) and rmc.StateView,
plus a SmokeInit-style random state generator (Smokeraft.tla:24-76) kept
inside the packed encoding's ranges.  Test infrastructure only."""
import random

import rmc
from oracle import raft_spec as R

ROLE = {R.FOLLOWER: 0, R.CANDIDATE: 1, R.LEADER: 2}
ROLE_INV = {v: k for k, v in ROLE.items()}
MT = {R.RVQ: 0, R.RVP: 1, R.AEQ: 2, R.AEP: 3}
MT_INV = {v: k for k, v in MT.items()}


def msg_to_view(m, count, mv):
    d = dict(m)
    mv.mtype = MT[d["mtype"]]
    mv.mterm = d["mterm"]
    mv.msource = d["msource"]
    mv.mdest = d["mdest"]
    mv.count = count
    if d["mtype"] == R.RVQ:
        mv.mlastLogTerm, mv.mlastLogIndex = d["mlastLogTerm"], d["mlastLogIndex"]
    elif d["mtype"] == R.RVP:
        mv.mvoteGranted = int(d["mvoteGranted"])
        mv.mlog_len = len(d["mlog"])
        for x, e in enumerate(d["mlog"]):
            mv.mlog[x].term, mv.mlog[x].value = R.rget(e, "term"), R.rget(e, "value")
    elif d["mtype"] == R.AEQ:
        mv.mprevLogIndex, mv.mprevLogTerm = d["mprevLogIndex"], d["mprevLogTerm"]
        mv.mentries_len = len(d["mentries"])
        for x, e in enumerate(d["mentries"]):
            mv.mentries[x].term, mv.mentries[x].value = R.rget(e, "term"), R.rget(e, "value")
        mv.mcommitIndex = d["mcommitIndex"]
    else:
        mv.msuccess, mv.mmatchIndex = int(d["msuccess"]), d["mmatchIndex"]


def to_view(model, s):
    v = rmc.StateView()
    S = model.n_servers
    v.n_servers = S
    for i in range(S):
        v.currentTerm[i] = s.currentTerm[i]
        v.state[i] = ROLE[s.state[i]]
        v.votedFor[i] = -1 if s.votedFor[i] == R.NIL else s.votedFor[i]
        v.commitIndex[i] = s.commitIndex[i]
        v.log_len[i] = len(s.log[i])
        for x, e in enumerate(s.log[i]):
            v.log[i][x].term, v.log[i][x].value = R.rget(e, "term"), R.rget(e, "value")
        v.votesResponded[i] = sum(1 << k for k in s.votesResponded[i])
        v.votesGranted[i] = sum(1 << k for k in s.votesGranted[i])
        for j in range(S):
            v.nextIndex[i][j] = s.nextIndex[i][j]
            v.matchIndex[i][j] = s.matchIndex[i][j]
    msgs = sorted(s.messages, key=repr)
    v.n_msgs = len(msgs)
    for q, (m, c) in enumerate(msgs):
        msg_to_view(m, c, v.msgs[q])
    return v


def msg_from_view(mv):
    t = MT_INV[mv.mtype]
    common = dict(mtype=t, mterm=mv.mterm, msource=mv.msource, mdest=mv.mdest)
    if t == R.RVQ:
        return R.rec(mlastLogTerm=mv.mlastLogTerm, mlastLogIndex=mv.mlastLogIndex, **common)
    if t == R.RVP:
        return R.rec(mvoteGranted=bool(mv.mvoteGranted),
                     mlog=tuple(R.entry(mv.mlog[x].term, mv.mlog[x].value)
                                for x in range(mv.mlog_len)), **common)
    if t == R.AEQ:
        return R.rec(mprevLogIndex=mv.mprevLogIndex, mprevLogTerm=mv.mprevLogTerm,
                     mentries=tuple(R.entry(mv.mentries[x].term, mv.mentries[x].value)
                                    for x in range(mv.mentries_len)),
                     mcommitIndex=mv.mcommitIndex, **common)
    return R.rec(msuccess=bool(mv.msuccess), mmatchIndex=mv.mmatchIndex, **common)


def from_view(v):
    S = v.n_servers
    return R.State(
        messages=frozenset((msg_from_view(v.msgs[q]), v.msgs[q].count) for q in range(v.n_msgs)),
        currentTerm=tuple(v.currentTerm[i] for i in range(S)),
        state=tuple(ROLE_INV[v.state[i]] for i in range(S)),
        votedFor=tuple(R.NIL if v.votedFor[i] < 0 else v.votedFor[i] for i in range(S)),
        log=tuple(tuple(R.entry(v.log[i][x].term, v.log[i][x].value) for x in range(v.log_len[i]))
                  for i in range(S)),
        commitIndex=tuple(v.commitIndex[i] for i in range(S)),
        votesResponded=tuple(frozenset(k for k in range(S) if v.votesResponded[i] >> k & 1)
                             for i in range(S)),
        votesGranted=tuple(frozenset(k for k in range(S) if v.votesGranted[i] >> k & 1)
                           for i in range(S)),
        nextIndex=tuple(tuple(v.nextIndex[i][j] for j in range(S)) for i in range(S)),
        matchIndex=tuple(tuple(v.matchIndex[i][j] for j in range(S)) for i in range(S)),
    )


def random_state(model, rng: random.Random):
    """A random type-correct state in the spirit of SmokeInit (Smokeraft.tla:64-76),
    restricted to the model's CONSTRAINT so every field is packable: terms in
    0..MaxTerm (SmokeNat-like, Smokeraft.tla:11-12), logs up to MaxLogLen,
    indexes in their packed ranges, up to MaxMsgs distinct messages."""
    S, V = model.n_servers, model.n_values
    T, L = model.max_term, model.max_log

    def ent():
        return R.entry(rng.randint(0, T), rng.randrange(V))

    def lg():
        return tuple(ent() for _ in range(rng.randint(0, L)))

    def rnd_msg():
        t = rng.choice([R.RVQ, R.RVP, R.AEQ, R.AEP])
        c = dict(mtype=t, mterm=rng.randint(0, T), msource=rng.randrange(S), mdest=rng.randrange(S))
        if t == R.RVQ:
            return R.rec(mlastLogTerm=rng.randint(0, T), mlastLogIndex=rng.randint(0, L), **c)
        if t == R.RVP:
            return R.rec(mvoteGranted=rng.random() < 0.5, mlog=lg(), **c)
        if t == R.AEQ:  # SmokeInt = -1..1 (Smokeraft.tla:14-15, :35): -1 included
            return R.rec(mprevLogIndex=rng.randint(-1, L), mprevLogTerm=rng.randint(0, T),
                         mentries=tuple(ent() for _ in range(rng.randint(0, 1))),
                         mcommitIndex=rng.randint(0, L), **c)
        return R.rec(msuccess=rng.random() < 0.5, mmatchIndex=rng.randint(0, L), **c)

    msgs = {}
    for _ in range(rng.randint(0, model.max_msgs)):
        msgs[rnd_msg()] = rng.randint(1, model.max_dup)
    return R.State(
        messages=frozenset(msgs.items()),
        currentTerm=tuple(rng.randint(0, T) for _ in range(S)),
        state=tuple(rng.choice([R.FOLLOWER, R.CANDIDATE, R.LEADER]) for _ in range(S)),
        votedFor=tuple(rng.choice([R.NIL] + list(range(S))) for _ in range(S)),
        log=tuple(lg() for _ in range(S)),
        commitIndex=tuple(rng.randint(0, L) for _ in range(S)),
        votesResponded=tuple(frozenset(k for k in range(S) if rng.random() < 0.5) for _ in range(S)),
        votesGranted=tuple(frozenset(k for k in range(S) if rng.random() < 0.5) for _ in range(S)),
        nextIndex=tuple(tuple(rng.randint(1, L + 1) for _ in range(S)) for _ in range(S)),
        matchIndex=tuple(tuple(rng.randint(0, L) for _ in range(S)) for _ in range(S)),
    )


def random_state_edge(model, rng: random.Random):
    """random_state pushed to the packed capacity's edges:
    terms at MaxTerm and just below (a Timeout or UpdateTerm there leaves the
    CONSTRAINT, term 15 = MaxTerm + 1 at MaxTerm 14 is the last packable one),
    full 3-entry logs (ClientRequest / NoConflict beyond them), counts at MaxDup
    (Duplicate beyond it), a full bag of MaxMsgs messages, mprevLogIndex = -1."""
    S, V = model.n_servers, model.n_values
    T, L = model.max_term, model.max_log
    term = lambda: rng.choice([0, max(0, T - 1), T, T])
    ent = lambda: R.entry(term(), rng.randrange(V))
    lg = lambda: tuple(ent() for _ in range(rng.choice([0, L, L, L])))

    def rnd_msg():
        t = rng.choice([R.RVQ, R.RVP, R.AEQ, R.AEP])
        c = dict(mtype=t, mterm=term(), msource=rng.randrange(S), mdest=rng.randrange(S))
        if t == R.RVQ:
            return R.rec(mlastLogTerm=term(), mlastLogIndex=rng.choice([0, L]), **c)
        if t == R.RVP:
            return R.rec(mvoteGranted=rng.random() < 0.5, mlog=lg(), **c)
        if t == R.AEQ:
            return R.rec(mprevLogIndex=rng.choice([-1, -1, 0, L - 1, L]), mprevLogTerm=term(),
                         mentries=tuple(ent() for _ in range(rng.randint(0, 1))),
                         mcommitIndex=rng.choice([0, L]), **c)
        return R.rec(msuccess=rng.random() < 0.5, mmatchIndex=rng.choice([0, L]), **c)

    msgs = {}
    target = rng.choice([model.max_msgs, model.max_msgs, rng.randint(0, model.max_msgs)])
    for _ in range(64):
        if len(msgs) >= target:
            break
        msgs[rnd_msg()] = rng.choice([1, model.max_dup, model.max_dup])
    return R.State(
        messages=frozenset(msgs.items()),
        currentTerm=tuple(term() for _ in range(S)),
        state=tuple(rng.choice([R.FOLLOWER, R.CANDIDATE, R.LEADER]) for _ in range(S)),
        votedFor=tuple(rng.choice([R.NIL] + list(range(S))) for _ in range(S)),
        log=tuple(lg() for _ in range(S)),
        commitIndex=tuple(rng.choice([0, L]) for _ in range(S)),
        votesResponded=tuple(frozenset(k for k in range(S) if rng.random() < 0.5) for _ in range(S)),
        votesGranted=tuple(frozenset(k for k in range(S) if rng.random() < 0.5) for _ in range(S)),
        nextIndex=tuple(tuple(rng.choice([1, L, L + 1]) for _ in range(S)) for _ in range(S)),
        matchIndex=tuple(tuple(rng.choice([0, L]) for _ in range(S)) for _ in range(S)),
    )


def check_trace(model, trace, violated_inv, violation_depth):
    """A counterexample [(family, lane, StateView)] must be a behaviour of the
    spec (Python restatement) from Init to a state violating `violated_inv`,
    every earlier state satisfying it, of length `violation_depth`."""
    import rmc
    assert len(trace) == violation_depth
    states = [from_view(v) for _f, _i, v in trace]
    assert states[0] == R.init_state(model) and trace[0][0] == -1
    for a, b, (fam, _inst, _v) in zip(states, states[1:], trace[1:]):
        succ = {(f, t) for f, _p, t in R.successors(model, a)}
        assert (rmc.FAMILIES[fam], b) in succ
        assert R.in_constraint(model, b)
    check = R.INVARIANTS[R.INV_BITS[violated_inv]]
    assert not check(model, states[-1])
    assert all(check(model, s) for s in states[:-1])
