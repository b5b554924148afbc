"""Reads a TLC-style counterexample transcript (rmc-tlc's, or TLC's own: the
same `State k: <Action line L1, col C1 to line L2, col C2 of module raft>`
headers and `/\\ var = <TLA+ value>` lines) back into oracle states, and
re-validates it with the Python restatement (oracle/raft_spec.py): every step
is a transition of Next named by the action its header gives, at that
action's raft.tla location; the last state violates the invariant and no
earlier one does.  Test infrastructure only."""
import re

import rmc
from oracle import raft_spec as R

TOK = re.compile(r"\s*(<<|>>|:>|@@|\|->|-?\d+|[A-Za-z_][A-Za-z0-9_]*|[()\[\]{},])")
ROLES = {"Follower": R.FOLLOWER, "Candidate": R.CANDIDATE, "Leader": R.LEADER}
MTYPES = {"RequestVoteRequest": R.RVQ, "RequestVoteResponse": R.RVP, "AppendEntriesRequest": R.AEQ,
          "AppendEntriesResponse": R.AEP}
MT_NAMES = {v: k for k, v in MTYPES.items()}
HEADER = re.compile(r"^State (\d+): <(?:Initial predicate|(\w+) line (\d+), col (\d+) to line (\d+), col (\d+) "
                    r"of module (\w+))>$")


def tokens(s):
    out, i = [], 0
    while i < len(s):
        if s[i].isspace():
            i += 1
            continue
        m = TOK.match(s, i)
        if not m:
            raise ValueError(f"bad token at {s[i:i + 20]!r}")
        out.append(m.group(1))
        i = m.end()
    return out


class Parser:
    """TLA+ values as TLC prints them: integers, model values, TRUE/FALSE,
    <<seq>>, {set}, [record], (k :> v @@ ...) functions."""

    def __init__(self, text):
        self.t = tokens(text)
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def take(self, want=None):
        tok = self.t[self.i]
        if want is not None and tok != want:
            raise ValueError(f"expected {want!r}, got {tok!r}")
        self.i += 1
        return tok

    def value(self):
        tok = self.take()
        if tok == "<<":
            items = []
            while self.peek() != ">>":
                items.append(self.value())
                if self.peek() == ",":
                    self.take()
            self.take(">>")
            return ("seq", tuple(items))
        if tok == "{":
            items = []
            while self.peek() != "}":
                items.append(self.value())
                if self.peek() == ",":
                    self.take()
            self.take("}")
            return ("set", frozenset(items))
        if tok == "[":
            rec = {}
            while self.peek() != "]":
                k = self.take()
                self.take("|->")
                rec[k] = self.value()
                if self.peek() == ",":
                    self.take()
            self.take("]")
            return ("rec", tuple(sorted(rec.items())))
        if tok == "(":
            fn = {}
            while True:
                k = self.value()
                self.take(":>")
                fn[k] = self.value()
                if self.peek() == "@@":
                    self.take()
                    continue
                break
            self.take(")")
            return ("fn", fn)
        if re.fullmatch(r"-?\d+", tok):
            return int(tok)
        if tok in ("TRUE", "FALSE"):
            return tok == "TRUE"
        return ("mv", tok)


def parse_value(text):
    p = Parser(text)
    v = p.value()
    if p.peek() is not None:
        raise ValueError(f"trailing tokens {p.t[p.i:p.i + 5]}")
    return v


def _server(v):
    assert v[0] == "mv" and re.fullmatch(r"r\d+", v[1]), v
    return int(v[1][1:]) - 1


def _value(v):
    assert v[0] == "mv" and re.fullmatch(r"v\d+", v[1]), v
    return int(v[1][1:]) - 1


def _entries(v):
    if v == ("fn", {}):
        return ()
    assert v[0] == "seq", v
    out = []
    for e in v[1]:
        d = dict(e[1])
        out.append(R.entry(d["term"], _value(d["value"])))
    return tuple(out)


def _per_server(v, S, conv):
    assert v[0] == "fn" and len(v[1]) == S, v
    return tuple(conv(v[1][("mv", f"r{i + 1}")]) for i in range(S))


def _message(v):
    d = dict(v[1])
    t = MTYPES[d["mtype"][1]]
    common = dict(mtype=t, mterm=d["mterm"], msource=_server(d["msource"]), mdest=_server(d["mdest"]))
    if t == R.RVQ:
        return R.rec(mlastLogTerm=d["mlastLogTerm"], mlastLogIndex=d["mlastLogIndex"], **common)
    if t == R.RVP:
        return R.rec(mvoteGranted=d["mvoteGranted"], mlog=_entries(d["mlog"]), **common)
    if t == R.AEQ:
        return R.rec(mprevLogIndex=d["mprevLogIndex"], mprevLogTerm=d["mprevLogTerm"],
                     mentries=_entries(d["mentries"]), mcommitIndex=d["mcommitIndex"], **common)
    return R.rec(msuccess=d["msuccess"], mmatchIndex=d["mmatchIndex"], **common)


def to_state(vars_, S):
    msgs = vars_["messages"]
    bag = frozenset() if msgs in (("seq", ()), ("fn", {})) else \
        frozenset((_message(k), c) for k, c in msgs[1].items())
    vf = lambda x: R.NIL if x == ("mv", "Nil") else _server(x)
    return R.State(
        messages=bag,
        currentTerm=_per_server(vars_["currentTerm"], S, int),
        state=_per_server(vars_["state"], S, lambda x: ROLES[x[1]]),
        votedFor=_per_server(vars_["votedFor"], S, vf),
        log=_per_server(vars_["log"], S, _entries),
        commitIndex=_per_server(vars_["commitIndex"], S, int),
        votesResponded=_per_server(vars_["votesResponded"], S, lambda x: frozenset(_server(y) for y in x[1])),
        votesGranted=_per_server(vars_["votesGranted"], S, lambda x: frozenset(_server(y) for y in x[1])),
        nextIndex=_per_server(vars_["nextIndex"], S, lambda x: _per_server(x, S, int)),
        matchIndex=_per_server(vars_["matchIndex"], S, lambda x: _per_server(x, S, int)),
    )


def parse_transcript(text, n_servers):
    """[(header match, State)] of the counterexample in `text`, plus the
    violated invariant's name."""
    inv = re.search(r"^Error: Invariant (\w+) is violated\.$", text, re.M)
    steps, cur, raw, last = [], None, {}, None
    for line in text.splitlines() + ["<end>"]:
        h = HEADER.match(line)
        if h or line == "<end>" or (cur is not None and not line.strip()):
            if cur is not None and raw:
                steps.append((cur, to_state({k: parse_value(v) for k, v in raw.items()}, n_servers)))
                cur, raw, last = None, {}, None
            if h:
                cur = h
            continue
        if cur is None:
            continue
        m = re.match(r"^/\\ (\w+) = (.*)$", line)
        if m:
            last = m.group(1)
            raw[last] = m.group(2)
        elif last:  # a value wrapped over several lines
            raw[last] += " " + line.strip()
    return (inv.group(1) if inv else None), steps


def expected_header(model, a, fam, param, overrides=None):
    """TLC's header for the step a --fam(param)--> (oracle family names);
    overrides: {family: (name, l1, c1, l2, c2, module)} for actions replaced
    in the cfg (`BecomeLeader <- BugBecomeLeader`)."""
    if overrides and fam in overrides:
        return overrides[fam]
    action = fam
    shown = fam
    if fam == "Receive":
        m = param[0]
        if R.rget(m, "mterm") > a.currentTerm[R.rget(m, "mdest")]:
            action = shown = "UpdateTerm"
        else:
            action = "Receive:" + MT_NAMES[R.rget(m, "mtype")]
    return (shown,) + rmc.action_location(action) + ("raft",)


def overrides_of(text):
    """Action locations of cfg overrides, from rmc-tlc's front-end notes."""
    m = re.search(r"^BecomeLeader <- \w+ .*; action <(\w+) line (\d+), col (\d+) to line (\d+), col (\d+) "
                  r"of module (\w+)>$", text, re.M)
    if not m:
        return {}
    return {"BecomeLeader": (m.group(1),) + tuple(int(m.group(k)) for k in range(2, 6)) + (m.group(6),)}


def validate(text, model, overrides=None):
    """Re-validate a transcript; returns (invariant, number of states)."""
    if overrides is None:
        overrides = overrides_of(text)
    inv, steps = parse_transcript(text, model.n_servers)
    assert inv is not None, "no 'Error: Invariant X is violated.' line"
    assert steps, "no states"
    h0, s0 = steps[0]
    assert h0.group(1) == "1" and h0.group(2) is None and s0 == R.init_state(model)
    for k, ((_ha, a), (hb, b)) in enumerate(zip(steps, steps[1:]), start=2):
        assert int(hb.group(1)) == k
        got = (hb.group(2),) + tuple(int(hb.group(x)) for x in range(3, 7)) + (hb.group(7),)
        want = {expected_header(model, a, f, p, overrides) for f, p, t in R.successors(model, a) if t == b}
        assert want, f"State {k} is not a successor of State {k - 1}"
        assert got in want, (k, got, want)
        assert R.in_constraint(model, b)
    check = R.INVARIANTS[inv]
    assert not check(model, steps[-1][1])
    assert all(check(model, s) for _h, s in steps[:-1])
    return inv, len(steps)
