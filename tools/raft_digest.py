"""Generates raft.tla_amd/csrc/model_digests.inc — what the front-end compares a
model against (DESIGN.md "Front-end").

The engine compiles ONE specification, lemmy/raft.tla's module body
(raft.tla:1-505), plus a few repo-local definitions (the restated invariants
and the config-5 BecomeLeader variant in specs/MCraftBounded.tla, SmokeInit for
simulation).  The front-end refuses a model whose raft.tla, invariants or
overrides differ from those.  It does so by digest: every top-level unit of a
module (definition, declaration, ASSUME) is normalised and hashed, and the
table below holds the digests of the compiled-in text.  This script is run
once, here, where /root/reference exists; its output (digests and line/column
spans, no source text) is committed.

Normalisation (rmc_front.cpp implements the same, byte for byte):
  * comments become spaces (\\* to end of line, nested (* *)), strings kept;
  * the module body runs from the `---- MODULE name ----` line to the first
    line that starts with `====`;
  * a unit starts at a column-1 line that opens a definition
    (`[LOCAL] Name[(params)] ==`) or a declaration keyword; a `----` line ends
    a unit; other lines continue the current unit;
  * each non-blank line of a unit becomes `<indent>|<tokens>` (leading spaces
    counted, inner whitespace runs collapsed to one space); a definition's name
    is dropped from its first line; lines are joined by newlines;
  * digest = FNV-1a 64 of that text; a definition's deep digest also covers the
    model-module definitions it uses, recursively.

    python tools/raft_digest.py [/root/reference]
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(ROOT, "raft.tla_amd", "csrc", "model_digests.inc")

FNV_OFF, FNV_PRIME = 0xCBF29CE484222325, 0x100000001B3

STATE_VARS = ("messages", "currentTerm", "state", "votedFor", "log", "commitIndex",
              "votesResponded", "votesGranted", "nextIndex", "matchIndex")


def fnv(s: str) -> int:
    h = FNV_OFF
    for b in s.encode():
        h = ((h ^ b) * FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h


def strip_comments(text: str) -> str:
    out, i, n, depth, in_str = [], 0, len(text), 0, False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 2
                continue
            if c == '"':
                in_str = False
            i += 1
            continue
        if depth == 0 and c == '"':
            in_str = True
            out.append(c)
            i += 1
            continue
        if text.startswith("(*", i):
            depth += 1
            out.append("  ")
            i += 2
            continue
        if depth and text.startswith("*)", i):
            depth -= 1
            out.append("  ")
            i += 2
            continue
        if depth:
            out.append("\n" if c == "\n" else " ")
            i += 1
            continue
        if text.startswith("\\*", i):
            while i < n and text[i] != "\n":
                out.append(" ")
                i += 1
            continue
        out.append(c)
        i += 1
    return "".join(out)


DEF_RE = re.compile(r"^(LOCAL\s+)?([A-Za-z_][A-Za-z0-9_]*)\s*(\([^)]*\))?\s*==")
KW_RE = re.compile(r"^(VARIABLES?|CONSTANTS?|ASSUME|AXIOM|EXTENDS|INSTANCE|THEOREM|LEMMA|RECURSIVE|USE|HIDE)\b")
HDR_RE = re.compile(r"^\s*-{4,}\s*MODULE\s+([A-Za-z_][A-Za-z0-9_]*)\s*-{4,}\s*$")


class Unit:
    def __init__(self, line, name):
        self.line = line          # 1-based line of the unit's first line
        self.name = name          # definition name, or "" for declarations
        self.lines = []           # (lineno, stripped text)

    def norm(self):
        out = []
        first = True
        for _ln, s in self.lines:
            if not s.strip():
                continue
            s = s.replace("\t", " ")
            ind = len(s) - len(s.lstrip(" "))
            content = " ".join(s.split())
            if first and self.name:
                m = DEF_RE.match(content)
                content = content[m.start(2) + len(self.name):].strip() if m else content
            first = False
            out.append(f"{ind}|{content}")
        return "\n".join(out)

    def digest(self):
        return fnv(self.norm())

    def text(self):
        return "\n".join(s for _ln, s in self.lines)


def parse_module(path):
    raw = open(path).read()
    lines = strip_comments(raw).split("\n")
    start = None
    for k, s in enumerate(lines):
        m = HDR_RE.match(s)
        if m:
            start, name = k + 1, m.group(1)
            break
    assert start is not None, path
    units, cur = [], None
    for k in range(start, len(lines)):
        s = lines[k]
        if re.match(r"^\s*={4,}", s):
            break
        if re.match(r"^\s*-{4,}\s*$", s):
            cur = None
            continue
        if s[:1] not in ("", " ", "\t") and (DEF_RE.match(s) or KW_RE.match(s)):
            m = DEF_RE.match(s)
            cur = Unit(k + 1, m.group(2) if m and not KW_RE.match(s) else "")
            units.append(cur)
        if cur is None:
            if s.strip():
                raise SystemExit(f"{path}:{k + 1}: text outside any unit")
            continue
        cur.lines.append((k + 1, s))
    return name, units


def idents(text):
    text = re.sub(r'"(\\.|[^"\\])*"', '""', text)
    return set(re.findall(r"(?<![A-Za-z0-9_\\])[A-Za-z_][A-Za-z0-9_]*", text))


def deep_digest(name, defs, exclude=()):
    u = defs[name]
    refs = sorted(r for r in idents(u.text()) if r in defs and r != name and r not in exclude)
    s = f"{u.digest():016x}" + "".join(f";{r}={deep_digest(r, defs, exclude):016x}" for r in refs)
    return fnv(s)


def mc_defs(paths):
    d = {}
    for p in paths:
        for u in parse_module(p)[1]:
            if u.name:
                d[u.name] = u
    return d


def body_span(u):
    """(line, col) of the first character after `==` to the last non-blank
    character of the unit (1-based, inclusive): TLC's location of the action."""
    ln0, s0 = u.lines[0]
    p = s0.index("==") + 2
    l1, c1 = None, None
    for ln, s in u.lines:
        seg = s[p:] if ln == ln0 else s
        off = p if ln == ln0 else 0
        if seg.strip():
            l1, c1 = ln, off + len(seg) - len(seg.lstrip()) + 1
            break
    last = [(ln, s) for ln, s in u.lines if s.strip()][-1]
    return l1, c1, last[0], len(last[1].rstrip())


def receive_spans(u):
    """Spans of Receive's top-level disjuncts (raft.tla:393-403), each from the
    token after `\\/` to its last character."""
    rows = [(ln, s) for ln, s in u.lines if s.strip()]
    col = None
    starts = []
    for k, (ln, s) in enumerate(rows):
        t = s.lstrip()
        c = len(s) - len(t)
        if t.startswith("\\/") and (col is None or c == col):
            col = c
            rest = t[2:]
            starts.append((k, ln, c + 2 + len(rest) - len(rest.lstrip()) + 1))
    spans = []
    for q, (k, ln, c) in enumerate(starts):
        endk = starts[q + 1][0] - 1 if q + 1 < len(starts) else len(rows) - 1
        spans.append((ln, c, rows[endk][0], len(rows[endk][1].rstrip())))
    return spans


def main():
    raft_path = os.path.join(REF, "raft.tla")
    name, units = parse_module(raft_path)
    assert name == "raft"
    defs = {u.name: u for u in units if u.name}
    # config 5: raft.tla:197 weakened (votesGranted[i] \in Quorum -> /= {})
    bl = defs["BecomeLeader"]
    bug = Unit(bl.line, "BecomeLeader")
    bug.lines = [(ln, s.replace("votesGranted[i] \\in Quorum", "votesGranted[i] /= {}")) for ln, s in bl.lines]
    assert bug.digest() != bl.digest()

    specs = os.path.join(ROOT, "specs")
    mcb = mc_defs([os.path.join(specs, "MCraftBounded.tla")])
    known = []  # (role, deep digest, source)
    for inv in ("OneLeaderPerTerm", "LogMatching", "MessagesInv", "LeaderVotesQuorum",
                "CandidateTermNotInLog", "VotesGrantedInv", "QuorumLogInv", "MoreUpToDateCorrect",
                "LeaderCompleteness"):
        if inv in mcb:
            known.append((inv, deep_digest(inv, mcb), "specs/MCraftBounded.tla"))
    known.append(("BecomeLeader", deep_digest("BugBecomeLeader", mcb), "specs/MCraftBounded.tla"))
    # SmokeInit (Smokeraft.tla:64-76); k and SmokeNat are the sampler's parameters
    ex = ("k", "SmokeNat")
    smk = mc_defs([os.path.join(REF, "MCraft.tla"), os.path.join(REF, "Smokeraft.tla")])
    known.append(("SmokeInit", deep_digest("SmokeInit", smk, ex), "Smokeraft.tla"))
    # this repo's restatement (specs/MCraftSmoke.tla; the test fixture carries the same text)
    own = mc_defs([os.path.join(specs, "MCraftBounded.tla"), os.path.join(specs, "MCraftSmoke.tla")])
    fix = mc_defs([os.path.join(ROOT, "tests", "golden", "models", "MCtoolbox.tla"),
                   os.path.join(ROOT, "tests", "golden", "models", "SmokeFixture.tla")])
    assert deep_digest("SmokeInit", own, ex) == deep_digest("SmokeInit", fix, ex)
    known.append(("SmokeInit", deep_digest("SmokeInit", own, ex), "specs/MCraftSmoke.tla"))

    spans = []
    for a in ("Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
              "AdvanceCommitIndex", "AppendEntries", "DuplicateMessage", "DropMessage",
              "UpdateTerm"):
        spans.append((a, *body_span(defs[a])))
    rs = receive_spans(defs["Receive"])
    assert len(rs) == 5, rs
    for tag, sp in zip(("UpdateTerm@Receive", "Receive:RequestVoteRequest", "Receive:RequestVoteResponse",
                        "Receive:AppendEntriesRequest", "Receive:AppendEntriesResponse"), rs):
        if tag.startswith("Receive:"):
            spans.append((tag, *sp))

    with open(OUT, "w") as f:
        f.write("// Generated by tools/raft_digest.py from lemmy/raft.tla (module body, raft.tla:1-505),\n"
                "// Smokeraft.tla's SmokeInit and specs/MCraftBounded.tla.  Digests and spans only.\n"
                "// Do not edit: re-run the script.\n")
        f.write(f"static const int kRaftUnitCount = {len(units)};\n")
        f.write("static const RaftUnit kRaftUnits[] = {\n")
        for u in units:
            f.write(f'    {{"{u.name}", {u.line}, 0x{u.digest():016x}ull}},\n')
        f.write("};\n")
        f.write(f"static const uint64_t kBugBecomeLeaderDigest = 0x{bug.digest():016x}ull;  // raft.tla:197 weakened\n")
        f.write("static const KnownDef kKnownDefs[] = {\n")
        for role, d, src in known:
            f.write(f'    {{"{role}", 0x{d:016x}ull, "{src}"}},\n')
        f.write("};\n")
        f.write("// TLC's location of each action of Next: the body of its definition\n")
        f.write("static const ActionSpan kActionSpans[] = {\n")
        for a, l1, c1, l2, c2 in spans:
            f.write(f'    {{"{a}", {l1}, {c1}, {l2}, {c2}}},\n')
        f.write("};\n")
    print(f"wrote {OUT}: {len(units)} raft units, {len(known)} known definitions, {len(spans)} spans")


if __name__ == "__main__":
    main()
