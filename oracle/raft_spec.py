"""CPU restatement of raft.tla (TEST INFRASTRUCTURE ONLY — the oracle).

This module is a slow, deliberately literal Python restatement of the
reference specification `raft.tla:1-505` as TLC evaluates it.  It is the
checker for the MI355X engine (`raft.tla_amd/`); it is never imported by the
product path.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may use anything under `oracle/`.

Values follow TLA+ value semantics (TLC):
  * records are tuples of sorted (field, value) pairs, so record equality is
    structural and records with different field sets differ;
  * sequences are Python tuples (a function on 1..n equals a sequence);
  * sets are frozensets; the bag `messages` is a frozenset of (msg, count)
    pairs with count >= 1 (Bags `(-)` drops keys whose count reaches 0);
  * model values are strings ("Follower", "Nil", ...), servers are 0..S-1,
    values are 0..V-1 (model values r1.. / v1.. of MCraft.tla:5-21).

Every disjunct of `Next` is evaluated separately and each yields its own
successor, which is how TLC enumerates successors.  The
engine-level facts this restatement pins:
  * `AppendEntriesAlreadyDone` (raft.tla:301-317) sets commitIndex' and then
    asserts UNCHANGED logVars; under TLC the second conjunct is an equality
    TEST, so the branch is enabled only when m.mcommitIndex = commitIndex[i]
    and it leaves commitIndex unchanged;
  * `ConflictAppendEntriesRequest` drops exactly the last entry
    (raft.tla:323) and keeps the message;
  * `RequestVote(i, j)` has no i /= j guard (raft.tla:157-166).

Parity status: the reference ships no golden vectors for this path; the
known answers this oracle is pinned by are the hand-derived KATs of
SURVEY.md §4 (levels 1-3: 1/3/18 distinct, 6/27 generated) and the SmokeInit
counts of Smokeraft.tla:18.  TLC itself is absent from this container, so the
distinct-state counts are cross-checked between two independent restatements
(this file and oracle/rmc_oracle.c) — "parity unpinned" against TLC.
"""
from __future__ import annotations

import itertools
from collections import namedtuple
from dataclasses import dataclass

# ---- constants (raft.tla:11-24) -------------------------------------------
FOLLOWER, CANDIDATE, LEADER = "Follower", "Candidate", "Leader"
NIL = "Nil"
RVQ = "RequestVoteRequest"
RVP = "RequestVoteResponse"
AEQ = "AppendEntriesRequest"
AEP = "AppendEntriesResponse"

# ---- state (raft.tla:31-74) ------------------------------------------------
State = namedtuple(
    "State",
    "messages currentTerm state votedFor log commitIndex "
    "votesResponded votesGranted nextIndex matchIndex",
)

# Action families in lane-table order (raft.tla:421-430).
FAMILIES = (
    "Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
    "AdvanceCommitIndex", "AppendEntries", "Receive", "DuplicateMessage",
    "DropMessage",
)


def rec(**fields):
    """A TLA+ record value: a tuple of (field, value) pairs sorted by name."""
    return tuple(sorted(fields.items()))


def rget(r, name):
    for k, v in r:
        if k == name:
            return v
    raise KeyError(name)


def entry(term, value):
    return rec(term=term, value=value)


@dataclass(frozen=True)
class Model:
    """Constants of a bounded MC model (MCraft.tla:15-21 + repo MC modules).

    bug_quorum: the config-5 bug variant, BecomeLeader's guard
    `votesGranted[i] \\in Quorum` (raft.tla:197) weakened to `/= {}`.
    A bound of None means "no constraint on that quantity".
    """

    n_servers: int = 3
    n_values: int = 2
    max_term: int | None = None
    max_log: int | None = None
    max_msgs: int | None = None
    max_dup: int | None = None
    bug_quorum: bool = False

    @property
    def servers(self):
        return range(self.n_servers)

    @property
    def values(self):
        return range(self.n_values)


# ---- helpers (raft.tla:81-108) ----------------------------------------------
def is_quorum(model, s):  # raft.tla:81
    return len(s) * 2 > model.n_servers


def last_term(xlog):  # raft.tla:84
    return 0 if len(xlog) == 0 else rget(xlog[-1], "term")


def bag_add(bag, m):  # WithMessage raft.tla:88, Bags (+)
    d = dict(bag)
    d[m] = d.get(m, 0) + 1
    return frozenset(d.items())


def bag_remove(bag, m):  # WithoutMessage raft.tla:92, Bags (-)
    d = dict(bag)
    if m in d:
        if d[m] <= 1:
            del d[m]
        else:
            d[m] -= 1
    return frozenset(d.items())


def tset(tup, i, v):
    lst = list(tup)
    lst[i] = v
    return tuple(lst)


def init_state(model):  # raft.tla:113-129
    S = model.n_servers
    return State(
        messages=frozenset(),
        currentTerm=(1,) * S,
        state=(FOLLOWER,) * S,
        votedFor=(NIL,) * S,
        log=((),) * S,
        commitIndex=(0,) * S,
        votesResponded=(frozenset(),) * S,
        votesGranted=(frozenset(),) * S,
        nextIndex=((1,) * S,) * S,
        matchIndex=((0,) * S,) * S,
    )


# ---- server-local actions (raft.tla:136-236) ------------------------------
def restart(model, s, i):  # raft.tla:136-143
    S = model.n_servers
    return s._replace(
        state=tset(s.state, i, FOLLOWER),
        votesResponded=tset(s.votesResponded, i, frozenset()),
        votesGranted=tset(s.votesGranted, i, frozenset()),
        nextIndex=tset(s.nextIndex, i, (1,) * S),
        matchIndex=tset(s.matchIndex, i, (0,) * S),
        commitIndex=tset(s.commitIndex, i, 0),
    )


def timeout(model, s, i):  # raft.tla:146-154
    if s.state[i] not in (FOLLOWER, CANDIDATE):
        return None
    return s._replace(
        state=tset(s.state, i, CANDIDATE),
        currentTerm=tset(s.currentTerm, i, s.currentTerm[i] + 1),
        votedFor=tset(s.votedFor, i, NIL),
        votesResponded=tset(s.votesResponded, i, frozenset()),
        votesGranted=tset(s.votesGranted, i, frozenset()),
    )


def request_vote(model, s, i, j):  # raft.tla:157-166
    if s.state[i] != CANDIDATE or j in s.votesResponded[i]:
        return None
    m = rec(mtype=RVQ, mterm=s.currentTerm[i], mlastLogTerm=last_term(s.log[i]),
            mlastLogIndex=len(s.log[i]), msource=i, mdest=j)
    return s._replace(messages=bag_add(s.messages, m))


def append_entries(model, s, i, j):  # raft.tla:171-192
    if i == j or s.state[i] != LEADER:
        return None
    lg = s.log[i]
    ni = s.nextIndex[i][j]
    prev_idx = ni - 1
    prev_term = rget(lg[prev_idx - 1], "term") if 0 < prev_idx <= len(lg) else 0
    last_entry = min(len(lg), ni)
    entries = tuple(lg[ni - 1:last_entry]) if ni <= last_entry else ()  # SubSeq
    m = rec(mtype=AEQ, mterm=s.currentTerm[i], mprevLogIndex=prev_idx,
            mprevLogTerm=prev_term, mentries=entries,
            mcommitIndex=min(s.commitIndex[i], last_entry), msource=i, mdest=j)
    return s._replace(messages=bag_add(s.messages, m))


def become_leader(model, s, i):  # raft.tla:195-203
    if s.state[i] != CANDIDATE:
        return None
    vg = s.votesGranted[i]
    ok = (len(vg) > 0) if model.bug_quorum else is_quorum(model, vg)
    if not ok:
        return None
    S = model.n_servers
    return s._replace(
        state=tset(s.state, i, LEADER),
        nextIndex=tset(s.nextIndex, i, (len(s.log[i]) + 1,) * S),
        matchIndex=tset(s.matchIndex, i, (0,) * S),
    )


def client_request(model, s, i, v):  # raft.tla:206-213
    if s.state[i] != LEADER:
        return None
    return s._replace(log=tset(s.log, i, s.log[i] + (entry(s.currentTerm[i], v),)))


def advance_commit_index(model, s, i):  # raft.tla:219-236
    if s.state[i] != LEADER:
        return None
    lg = s.log[i]

    def agree(index):
        return frozenset({i}) | frozenset(k for k in model.servers
                                          if s.matchIndex[i][k] >= index)

    agree_indexes = [idx for idx in range(1, len(lg) + 1)
                     if is_quorum(model, agree(idx))]
    if agree_indexes and rget(lg[max(agree_indexes) - 1], "term") == s.currentTerm[i]:
        new_ci = max(agree_indexes)
    else:
        new_ci = s.commitIndex[i]
    return s._replace(commitIndex=tset(s.commitIndex, i, new_ci))


# ---- message handlers (raft.tla:244-403) -----------------------------------
def reply(bag, response, request):  # raft.tla:102-103
    return bag_remove(bag_add(bag, response), request)


def handle_rv_request(model, s, i, j, m):  # raft.tla:244-263
    out = []
    lt = last_term(s.log[i])
    log_ok = (rget(m, "mlastLogTerm") > lt or
              (rget(m, "mlastLogTerm") == lt and rget(m, "mlastLogIndex") >= len(s.log[i])))
    grant = (rget(m, "mterm") == s.currentTerm[i] and log_ok
             and s.votedFor[i] in (NIL, j))
    if not rget(m, "mterm") <= s.currentTerm[i]:
        return out
    vf = tset(s.votedFor, i, j) if grant else s.votedFor
    resp = rec(mtype=RVP, mterm=s.currentTerm[i], mvoteGranted=grant,
               mlog=s.log[i], msource=i, mdest=j)
    out.append(s._replace(votedFor=vf, messages=reply(s.messages, resp, m)))
    return out


def handle_rv_response(model, s, i, j, m):  # raft.tla:267-279
    if rget(m, "mterm") != s.currentTerm[i]:
        return []
    vr = tset(s.votesResponded, i, s.votesResponded[i] | {j})
    vg = tset(s.votesGranted, i, s.votesGranted[i] | {j}) if rget(m, "mvoteGranted") \
        else s.votesGranted
    return [s._replace(votesResponded=vr, votesGranted=vg,
                       messages=bag_remove(s.messages, m))]


def handle_ae_request(model, s, i, j, m):  # raft.tla:347-356
    out = []
    lg = s.log[i]
    pidx = rget(m, "mprevLogIndex")
    log_ok = (pidx == 0 or
              (pidx > 0 and pidx <= len(lg) and
               rget(m, "mprevLogTerm") == rget(lg[pidx - 1], "term")))
    mterm, ct = rget(m, "mterm"), s.currentTerm[i]
    if not mterm <= ct:
        return out
    # RejectAppendEntriesRequest  raft.tla:281-293
    if mterm < ct or (mterm == ct and s.state[i] == FOLLOWER and not log_ok):
        resp = rec(mtype=AEP, mterm=ct, msuccess=False, mmatchIndex=0,
                   msource=i, mdest=j)
        out.append(s._replace(messages=reply(s.messages, resp, m)))
    # ReturnToFollowerState  raft.tla:295-299
    if mterm == ct and s.state[i] == CANDIDATE:
        out.append(s._replace(state=tset(s.state, i, FOLLOWER)))
    # AcceptAppendEntriesRequest  raft.tla:333-341
    if mterm == ct and s.state[i] == FOLLOWER and log_ok:
        index = pidx + 1
        ents = rget(m, "mentries")
        # AppendEntriesAlreadyDone raft.tla:301-317.  commitIndex' is bound to
        # [commitIndex EXCEPT ![i] = m.mcommitIndex] and then UNCHANGED logVars
        # tests commitIndex' = commitIndex (TLC semantics).
        if (len(ents) == 0 or
                (len(ents) > 0 and len(lg) >= index and
                 rget(lg[index - 1], "term") == rget(ents[0], "term"))):
            ci_new = tset(s.commitIndex, i, rget(m, "mcommitIndex"))
            if ci_new == s.commitIndex:
                resp = rec(mtype=AEP, mterm=ct, msuccess=True,
                           mmatchIndex=pidx + len(ents), msource=i, mdest=j)
                out.append(s._replace(messages=reply(s.messages, resp, m)))
        # ConflictAppendEntriesRequest raft.tla:319-325 (drops the LAST entry)
        if (len(ents) > 0 and len(lg) >= index and
                rget(lg[index - 1], "term") != rget(ents[0], "term")):
            out.append(s._replace(log=tset(s.log, i, lg[:len(lg) - 1])))
        # NoConflictAppendEntriesRequest raft.tla:327-331
        if len(ents) > 0 and len(lg) == pidx:
            out.append(s._replace(log=tset(s.log, i, lg + (ents[0],))))
    return out


def handle_ae_response(model, s, i, j, m):  # raft.tla:360-370
    if rget(m, "mterm") != s.currentTerm[i]:
        return []
    if rget(m, "msuccess"):
        mm = rget(m, "mmatchIndex")
        ni = tset(s.nextIndex, i, tset(s.nextIndex[i], j, mm + 1))
        mi = tset(s.matchIndex, i, tset(s.matchIndex[i], j, mm))
    else:
        ni = tset(s.nextIndex, i, tset(s.nextIndex[i], j, max(s.nextIndex[i][j] - 1, 1)))
        mi = s.matchIndex
    return [s._replace(nextIndex=ni, matchIndex=mi, messages=bag_remove(s.messages, m))]


def update_term(model, s, i, j, m):  # raft.tla:373-379
    if not rget(m, "mterm") > s.currentTerm[i]:
        return []
    return [s._replace(currentTerm=tset(s.currentTerm, i, rget(m, "mterm")),
                       state=tset(s.state, i, FOLLOWER),
                       votedFor=tset(s.votedFor, i, NIL))]


def drop_stale_response(model, s, i, j, m):  # raft.tla:382-385
    if not rget(m, "mterm") < s.currentTerm[i]:
        return []
    return [s._replace(messages=bag_remove(s.messages, m))]


def receive(model, s, m):  # raft.tla:388-403
    i, j = rget(m, "mdest"), rget(m, "msource")
    t = rget(m, "mtype")
    out = list(update_term(model, s, i, j, m))
    if t == RVQ:
        out += handle_rv_request(model, s, i, j, m)
    elif t == RVP:
        out += drop_stale_response(model, s, i, j, m)
        out += handle_rv_response(model, s, i, j, m)
    elif t == AEQ:
        out += handle_ae_request(model, s, i, j, m)
    elif t == AEP:
        out += drop_stale_response(model, s, i, j, m)
        out += handle_ae_response(model, s, i, j, m)
    return out


def duplicate_message(model, s, m):  # raft.tla:410-412
    return s._replace(messages=bag_add(s.messages, m))


def drop_message(model, s, m):  # raft.tla:415-417
    return s._replace(messages=bag_remove(s.messages, m))


# ---- Next (raft.tla:421-430) -------------------------------------------------
def successors(model, s):
    """All (family, params, successor) triples of Next, one per disjunct."""
    out = []
    S = model.servers
    for i in S:
        out.append(("Restart", (i,), restart(model, s, i)))
    for i in S:
        out.append(("Timeout", (i,), timeout(model, s, i)))
    for i, j in itertools.product(S, S):
        out.append(("RequestVote", (i, j), request_vote(model, s, i, j)))
    for i in S:
        out.append(("BecomeLeader", (i,), become_leader(model, s, i)))
    for i, v in itertools.product(S, model.values):
        out.append(("ClientRequest", (i, v), client_request(model, s, i, v)))
    for i in S:
        out.append(("AdvanceCommitIndex", (i,), advance_commit_index(model, s, i)))
    for i, j in itertools.product(S, S):
        out.append(("AppendEntries", (i, j), append_entries(model, s, i, j)))
    msgs = [m for m, _ in s.messages]
    for m in msgs:
        for t in receive(model, s, m):
            out.append(("Receive", (m,), t))
    for m in msgs:
        out.append(("DuplicateMessage", (m,), duplicate_message(model, s, m)))
    for m in msgs:
        out.append(("DropMessage", (m,), drop_message(model, s, m)))
    return [(f, p, t) for f, p, t in out if t is not None]


# ---- constraint & invariants ------------------------------------------------
def in_constraint(model, s):
    """StateConstraint of specs/MCraftBounded.tla."""
    if model.max_term is not None and any(t > model.max_term for t in s.currentTerm):
        return False
    if model.max_log is not None and any(len(lg) > model.max_log for lg in s.log):
        return False
    if model.max_msgs is not None and len(s.messages) > model.max_msgs:
        return False
    if model.max_dup is not None and any(c > model.max_dup for _, c in s.messages):
        return False
    return True


def _entry_ok(model, e):
    return (isinstance(e, tuple) and [k for k, _ in e] == ["term", "value"]
            and isinstance(rget(e, "term"), int) and rget(e, "term") >= 0
            and rget(e, "value") in model.values)


def _nat(x):
    return isinstance(x, int) and not isinstance(x, bool) and x >= 0


def _msg_ok(model, m):  # raft.tla:443-479
    keys = [k for k, _ in m]
    t = rget(m, "mtype")
    srv = lambda x: x in model.servers and not isinstance(x, bool)
    common = _nat(rget(m, "mterm")) and srv(rget(m, "msource")) and srv(rget(m, "mdest"))
    if t == RVQ:
        return common and keys == sorted(["mtype", "mterm", "mlastLogTerm", "mlastLogIndex",
                                          "msource", "mdest"]) and \
            _nat(rget(m, "mlastLogTerm")) and _nat(rget(m, "mlastLogIndex"))
    if t == AEQ:
        return common and keys == sorted(["mtype", "mterm", "mprevLogIndex", "mprevLogTerm",
                                          "mentries", "mcommitIndex", "msource", "mdest"]) and \
            isinstance(rget(m, "mprevLogIndex"), int) and _nat(rget(m, "mprevLogTerm")) and \
            all(_entry_ok(model, e) for e in rget(m, "mentries")) and \
            _nat(rget(m, "mcommitIndex"))
    if t == RVP:
        return common and keys == sorted(["mtype", "mterm", "mvoteGranted", "mlog",
                                          "msource", "mdest"]) and \
            isinstance(rget(m, "mvoteGranted"), bool) and \
            all(_entry_ok(model, e) for e in rget(m, "mlog"))
    if t == AEP:
        return common and keys == sorted(["mtype", "mterm", "msuccess", "mmatchIndex",
                                          "msource", "mdest"]) and \
            isinstance(rget(m, "msuccess"), bool) and _nat(rget(m, "mmatchIndex"))
    return False


def type_ok(model, s):  # raft.tla:482-492
    S = model.servers
    return (all(c >= 1 for _, c in s.messages)
            and all(_msg_ok(model, m) for m, _ in s.messages)
            and all(_nat(t) for t in s.currentTerm)
            and all(x in (FOLLOWER, CANDIDATE, LEADER) for x in s.state)
            and all(x == NIL or x in S for x in s.votedFor)
            and all(all(_entry_ok(model, e) for e in lg) for lg in s.log)
            and all(_nat(c) for c in s.commitIndex)
            and all(vr <= frozenset(S) for vr in s.votesResponded)
            and all(vg <= frozenset(S) for vg in s.votesGranted)
            and all(all(_nat(n) and n >= 1 for n in row) for row in s.nextIndex)
            and all(all(_nat(n) for n in row) for row in s.matchIndex))


def one_leader_per_term(model, s):
    """Restated ElectionSafety (raft.tla:1124-1129 is ill-defined under TLC,
    SURVEY.md §0.9): at most one leader per term."""
    for i, j in itertools.combinations(model.servers, 2):
        if s.state[i] == LEADER and s.state[j] == LEADER and \
                s.currentTerm[i] == s.currentTerm[j]:
            return False
    return True


def log_matching(model, s):  # raft.tla:1132-1136
    for i, j in itertools.product(model.servers, model.servers):
        li, lj = s.log[i], s.log[j]
        for n in range(1, min(len(li), len(lj)) + 1):
            if rget(li[n - 1], "term") == rget(lj[n - 1], "term") and li[:n] != lj[:n]:
                return False
    return True


def messages_inv(model, s):
    """MessagesInv (raft.tla:941-946) with `m.dest` of :910 read as `m.mdest`.
    `log[src][mprevLogIndex + 1]` outside DOMAIN log[src] is a TLC evaluation
    error; it counts as a violation here."""
    ct, lg = s.currentTerm, s.log
    for m, _c in s.messages:
        t, src, dst, mt = (rget(m, k) for k in ("mtype", "msource", "mdest", "mterm"))
        if mt > ct[src]:  # MessageTermsLtCurrentTerm :934-935
            return False
        if t == RVP and rget(m, "mvoteGranted") and ct[src] == ct[dst] == mt:  # :903-910
            ld, ls = last_term(lg[dst]), last_term(lg[src])
            if not (ld > ls or (ld == ls and len(lg[dst]) >= len(lg[src]))):
                return False
        if t == RVQ and s.state[src] == CANDIDATE and ct[src] == mt:  # :915-920
            if rget(m, "mlastLogIndex") != len(lg[src]) or \
                    rget(m, "mlastLogTerm") != last_term(lg[src]):
                return False
        if t == AEQ and rget(m, "mentries") and mt == ct[src]:  # :924-930
            p = rget(m, "mprevLogIndex")
            if not 1 <= p + 1 <= len(lg[src]):
                return False
            if lg[src][p] != rget(m, "mentries")[0]:
                return False
            if 0 < p <= len(lg[src]) and rget(lg[src][p - 1], "term") != rget(m, "mprevLogTerm"):
                return False
    return True


def leader_votes_quorum(model, s):  # raft.tla:1033-1037
    for i in model.servers:
        if s.state[i] == LEADER:
            q = {j for j in model.servers if s.currentTerm[j] > s.currentTerm[i] or
                 (s.currentTerm[j] == s.currentTerm[i] and s.votedFor[j] == i)}
            if not is_quorum(model, q):
                return False
    return True


def candidate_term_not_in_log(model, s):  # raft.tla:1041-1047
    for i in model.servers:
        if s.state[i] != CANDIDATE:
            continue
        q = {j for j in model.servers if s.currentTerm[j] == s.currentTerm[i] and
             s.votedFor[j] in (i, NIL)}
        if is_quorum(model, q) and any(rget(e, "term") == s.currentTerm[i]
                                       for j in model.servers for e in s.log[j]):
            return False
    return True


def committed(s, i):
    """Committed(i) as restated in specs/MCraftBounded.tla: raft.tla:896's
    SubSeq(log[i], 1, commitIndex[i]) with the commit index clamped to
    Len(log[i]) (this spec lets commitIndex exceed Len, raft.tla:309,323)."""
    return s.log[i][:min(s.commitIndex[i], len(s.log[i]))]


def is_prefix(a, b):  # SequencesExt's IsPrefix (not in raft.tla's EXTENDS)
    return len(a) <= len(b) and b[:len(a)] == a


def votes_granted_inv(model, s):  # raft.tla:1145-1153
    return all(is_prefix(committed(s, j), s.log[i])
               for i in model.servers for j in s.votesGranted[i]
               if s.currentTerm[i] == s.currentTerm[j])


def quorum_log_inv(model, s):  # raft.tla:1157-1161, every quorum enumerated
    quorums = [set(q) for r in range(model.n_servers + 1)
               for q in itertools.combinations(model.servers, r) if is_quorum(model, set(q))]
    return all(any(is_prefix(committed(s, i), s.log[j]) for j in q)
               for i in model.servers for q in quorums)


def more_up_to_date_correct(model, s):  # raft.tla:1167-1172
    for i in model.servers:
        for j in model.servers:
            li, lj = last_term(s.log[i]), last_term(s.log[j])
            if (li > lj or (li == lj and len(s.log[i]) >= len(s.log[j]))) and \
                    not is_prefix(committed(s, j), s.log[i]):
                return False
    return True


def leader_completeness(model, s):  # raft.tla:1176-1180
    return all(is_prefix(committed(s, j), s.log[i])
               for i in model.servers if s.state[i] == LEADER for j in model.servers)


INVARIANTS = {
    "TypeOK": type_ok,
    "OneLeaderPerTerm": one_leader_per_term,
    "LogMatching": log_matching,
    "MessagesInv": messages_inv,
    "LeaderVotesQuorum": leader_votes_quorum,
    "CandidateTermNotInLog": candidate_term_not_in_log,
    "VotesGrantedInv": votes_granted_inv,
    "QuorumLogInv": quorum_log_inv,
    "MoreUpToDateCorrect": more_up_to_date_correct,
    "LeaderCompleteness": leader_completeness,
}


# rmc.h's RMC_INV_* bits
INV_BITS = {1: "TypeOK", 2: "OneLeaderPerTerm", 4: "LogMatching", 8: "MessagesInv",
            16: "LeaderVotesQuorum", 32: "CandidateTermNotInLog", 64: "VotesGrantedInv",
            128: "QuorumLogInv", 256: "MoreUpToDateCorrect", 512: "LeaderCompleteness"}


# ---- symmetry (SYMMETRY Permutations(Server)) -------------------------------
def permute_state(model, s, p):
    """Apply the server permutation p (tuple: old id -> new id) to s."""
    S = model.n_servers
    inv = [0] * S
    for a, b in enumerate(p):
        inv[b] = a

    def pm(m):
        d = dict(m)
        d["msource"] = p[d["msource"]]
        d["mdest"] = p[d["mdest"]]
        return tuple(sorted(d.items()))

    def ps(x):
        return frozenset(p[k] for k in x)

    return State(
        messages=frozenset((pm(m), c) for m, c in s.messages),
        currentTerm=tuple(s.currentTerm[inv[i]] for i in range(S)),
        state=tuple(s.state[inv[i]] for i in range(S)),
        votedFor=tuple(NIL if s.votedFor[inv[i]] == NIL else p[s.votedFor[inv[i]]]
                       for i in range(S)),
        log=tuple(s.log[inv[i]] for i in range(S)),
        commitIndex=tuple(s.commitIndex[inv[i]] for i in range(S)),
        votesResponded=tuple(ps(s.votesResponded[inv[i]]) for i in range(S)),
        votesGranted=tuple(ps(s.votesGranted[inv[i]]) for i in range(S)),
        nextIndex=tuple(tuple(s.nextIndex[inv[i]][inv[j]] for j in range(S))
                        for i in range(S)),
        matchIndex=tuple(tuple(s.matchIndex[inv[i]][inv[j]] for j in range(S))
                         for i in range(S)),
    )


def canonical(model, s):
    """Orbit representative: the least permuted state under a fixed total
    order (repr).  Any orbit-invariant choice gives the same orbit count."""
    best = None
    for p in itertools.permutations(range(model.n_servers)):
        t = permute_state(model, s, p)
        key = repr((sorted(t.messages, key=repr), t[1:]))
        if best is None or key < best[0]:
            best = (key, t)
    return best[1]


# ---- BFS (TLC's breadth-first model checking loop) ---------
@dataclass
class BfsResult:
    generated: int
    distinct: int
    depth: int
    level_new: list
    level_generated: list
    violated: str | None = None
    violation_depth: int | None = None
    trace: list | None = None
    left_on_queue: int = 0


def bfs(model, invariants=("TypeOK",), max_levels=None, init=None, symmetry=False):
    """Level-synchronous BFS with exact state storage.

    `generated` counts the initial states plus every successor of every
    expanded state (including stuttering and out-of-constraint successors);
    out-of-constraint successors are neither stored nor checked (TLC: the
    CONSTRAINT filter sits in front of the seen-set).
    Level 1 is the set of initial states.  `level_generated[d]` is the number
    of successors generated by expanding level d+1 (index 0: init states).
    """
    key = (lambda t: canonical(model, t)) if symmetry else (lambda t: t)
    inits = [init_state(model)] if init is None else list(init)
    seen = {}
    frontier = []
    for s in inits:
        k = key(s)
        if in_constraint(model, s) and k not in seen:
            seen[k] = None
            frontier.append(s)
    generated = len(inits)
    level_new, level_gen = [len(frontier)], [len(inits)]
    for name in invariants:
        for s in frontier:
            if not INVARIANTS[name](model, s):
                return BfsResult(generated, len(seen), 1, level_new, level_gen, name, 1, [s])
    depth = 1 if frontier else 0
    parents = {}
    while frontier and (max_levels is None or depth < max_levels):
        nxt = []
        gen = 0
        for s in frontier:
            for _f, _p, t in successors(model, s):
                gen += 1
                if not in_constraint(model, t):
                    continue
                k = key(t)
                if k in seen:
                    continue
                seen[k] = None
                parents[t] = s
                nxt.append(t)
                for name in invariants:
                    if not INVARIANTS[name](model, t):
                        trace = [t]
                        while trace[-1] in parents:
                            trace.append(parents[trace[-1]])
                        trace.reverse()
                        generated += gen
                        return BfsResult(generated, len(seen), depth + 1,
                                         level_new + [len(nxt)], level_gen + [gen],
                                         name, depth + 1, trace)
        generated += gen
        level_gen.append(gen)
        if nxt:
            level_new.append(len(nxt))
            depth += 1
        frontier = nxt
    return BfsResult(generated, len(seen), depth, level_new, level_gen,
                     left_on_queue=len(frontier))
