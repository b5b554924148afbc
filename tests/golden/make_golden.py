"""Generates tests/golden/oracle_levels.json from the C oracle (oracle/rmc_oracle.c).

The reference ships no golden vectors for this path, and TLC
is absent from this container, so these fixtures are produced by the repo's
own CPU restatements.  Tiny configs are cross-checked against the Python
restatement (oracle/raft_spec.py) in tests/test_oracle.py; the hand-derived
KATs of SURVEY.md §4 are asserted there too.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests import oracle_c  # noqa: E402

# name: (S, V, MaxTerm, MaxLog, MaxMsgs, MaxDup, bug, inv_mask, sym, max_levels)
CONFIGS = {
    "tiny2": (2, 1, 2, 1, 2, 1, 0, 1, 0, 0),
    "tiny2_v2": (2, 2, 3, 2, 2, 1, 0, 1, 0, 0),
    "small": (3, 2, 2, 1, 1, 1, 0, 1, 0, 0),
    "small_sym": (3, 2, 2, 1, 1, 1, 0, 1, 1, 0),
    "s3_v1_msgs1": (3, 1, 2, 1, 1, 1, 0, 1, 0, 0),
    "bounded_prefix14": (3, 2, 2, 1, 2, 1, 0, 1, 0, 14),
    "bounded_sym_prefix16": (3, 2, 2, 1, 2, 1, 0, 1, 1, 16),
    "msgs5_dup2_prefix9": (3, 2, 3, 2, 5, 2, 0, 1, 0, 9),
    "s4_prefix10": (4, 1, 2, 1, 2, 1, 0, 1, 0, 10),
    "s5_prefix9": (5, 2, 2, 1, 2, 1, 0, 1, 0, 9),
    "bug_one_leader": (3, 2, 3, 1, 3, 1, 1, 2, 0, 0),
    "bug_log_matching": (3, 2, 3, 1, 3, 1, 1, 4, 0, 0),
    "bug_both": (3, 2, 3, 1, 3, 1, 1, 6, 0, 0),
    # MessagesInv (raft.tla:941-946, inv bit 8): holds for 2 servers, violated by the
    # unmodified spec for 3 (a candidate whose own RequestVote is still in flight
    # grants its vote to another candidate of the same term, raft.tla:250-252)
    "messages_tiny2": (2, 1, 2, 1, 2, 1, 0, 9, 0, 0),
    "messages_small": (3, 2, 2, 1, 1, 1, 0, 9, 0, 0),
    "bug_messages": (3, 2, 3, 1, 3, 1, 1, 8, 0, 0),
    # ElectionsCorrect (raft.tla:1049): LeaderVotesQuorum (bit 16) and
    # CandidateTermNotInLog (bit 32) hold for the spec, fail for the bug variant
    "elections_tiny2": (2, 1, 2, 1, 2, 1, 0, 49, 0, 0),
    "elections_small": (3, 2, 2, 1, 1, 1, 0, 49, 0, 0),
    "bug_leader_votes": (3, 2, 2, 1, 1, 1, 1, 16, 0, 0),
    "bug_cand_term": (3, 2, 2, 1, 1, 1, 1, 32, 0, 0),
    # The IsPrefix invariants (raft.tla:1143-1180, restated in specs/MCraftBounded.tla
    # with Committed(i) clamped to Len(log[i])): VotesGrantedInv (64) fails on the
    # unmodified spec; QuorumLogInv (128), MoreUpToDateCorrect (256) and
    # LeaderCompleteness (512) hold, also with 2-entry logs; the bug variant breaks all.
    "votes_granted_small": (3, 2, 2, 1, 1, 1, 0, 64, 0, 0),
    "isprefix_small": (3, 2, 2, 1, 1, 1, 0, 897, 0, 0),
    "isprefix_s3v1_log2": (3, 1, 2, 2, 1, 1, 0, 897, 0, 0),
    "bug_votes_granted": (3, 2, 2, 1, 1, 1, 1, 64, 0, 0),
    "bug_quorum_log": (3, 2, 2, 1, 1, 1, 1, 128, 0, 0),
    "bug_more_up_to_date": (3, 2, 2, 1, 1, 1, 1, 256, 0, 0),
    "bug_leader_complete": (3, 2, 2, 1, 1, 1, 1, 512, 0, 0),
    # SYMMETRY Permutations(Server) with 4 and 5 servers (signature-sorted canonical keys)
    "s4_sym_prefix16": (4, 1, 2, 1, 2, 1, 0, 1, 1, 16),
    "s5_sym_prefix16": (5, 2, 2, 1, 2, 1, 0, 1, 1, 16),
    "sym_bug_one_leader": (3, 2, 3, 1, 3, 1, 1, 2, 1, 0),
    # config 3, wider bounds (specs/MCraft5Wide.cfg): the first 9 levels
    "s5_wide_prefix9": (5, 2, 3, 2, 4, 1, 0, 1, 0, 9),
    # 3-entry logs with 2 values: an RVP's mlog then fills the message's top bit
    # (bit 29), which a sharded record once shared with its "seen" flag
    "tiny2_log3": (2, 2, 3, 3, 2, 1, 0, 1, 0, 0),
    "s3_log3_prefix14": (3, 2, 3, 3, 2, 1, 0, 1, 0, 14),
    # the bench model (specs/MCraftBench.cfg) itself: its first 22 and 24 levels (31 M, 76 M
    # states; the whole 1.23 G-state model exceeds the oracle's memory)
    "bench_prefix22": (3, 2, 2, 1, 3, 1, 0, 1, 0, 22),
    "bench_prefix24": (3, 2, 2, 1, 3, 1, 0, 1, 0, 24),
    # the round-5 bench model (specs/MCraftBenchXL.cfg: V = 1, MaxLogLen 2; 4.13 G states):
    # its first 22 and 24 levels (43 M, 87 M states)
    "benchxl_prefix22": (3, 1, 2, 2, 3, 1, 0, 1, 0, 22),
    "benchxl_prefix24": (3, 1, 2, 2, 3, 1, 0, 1, 0, 24),
    # MCraftBounded.cfg at full size (78 M states, ~2 min on 8 threads, ~10 GB)
    "bounded_full": (3, 2, 2, 1, 2, 1, 0, 1, 0, 0),
}
# The reference's own MCraft.cfg (no CONSTRAINT: tests/golden/models/MCunbounded.cfg)
# under a depth bound, on the oracle build holding logs of 8 entries and 12
# messages (liboracle_wide.so): terms and counts unbounded (-1); Len(log) <= 8 and
# 12 messages never bind within 11 steps (each step adds at most one entry and
# one distinct message), so these are the unconstrained spec's levels.
WIDE_CONFIGS = {
    "mcraft_shipped_d12": (3, 2, -1, 8, 12, -1, 0, 1, 0, 12),
}


def main(only=None):
    """`only`: names to (re)generate, merged into the existing file; without
    names every entry is regenerated (bounded_full included)."""
    path = os.path.join(ROOT, "tests", "golden", "oracle_levels.json")
    out = json.load(open(path)) if only else {}
    todo = [(n, c, False) for n, c in CONFIGS.items()] + [(n, c, True) for n, c in WIDE_CONFIGS.items()]
    for name, (S, V, mt, ml, mm, md, bug, inv, sym, lv), wide in todo:
        if only and name not in only:
            continue
        r, ln, lg = oracle_c.bfs(S, V, mt, ml, mm, md, bug=bug, inv=inv, sym=sym, threads=8,
                                 max_levels=lv, capacity=1 << (26 if wide else 27), wide=wide)
        out[name] = dict(params=dict(n_servers=S, n_values=V, max_term=mt, max_log_len=ml,
                                     max_msgs=mm, max_dup=md, bug_quorum=bug, invariants=inv,
                                     symmetry=sym, max_depth=lv),
                         generated=r.generated, distinct=r.distinct, depth=r.depth,
                         left_on_queue=r.left_on_queue, violated_inv=r.violated_inv,
                         violation_depth=r.violation_depth, level_new=ln,
                         level_generated=lg[:r.depth])
        print(name, r.distinct, r.generated, r.depth, r.violated_inv, r.violation_depth,
              f"{r.seconds:.2f}s", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
