---- MODULE SmokeFixture ----
\* Parse fixture for simulation models: `Init <- SmokeInit` with the sampler's
\* parameters k and SmokeNat, and a run-budget constraint that bounds no
\* variable.  SmokeInit restates Smokeraft.tla:64-76 (same domains, this
\* repo's own layout); the engine samples it itself (rmc_simulate), and the
\* front-end accepts only this definition or Smokeraft's.
EXTENDS MCtoolbox, TLC, Randomization

SmokeNat ==
    0..3

k ==
   3

UpTo(S, n) == UNION {[1..len -> S] : len \in 0..n}

Entry == [term : SmokeNat, value : Value]

RVQ == [mtype : {RequestVoteRequest}, mterm : SmokeNat, mlastLogTerm : SmokeNat,
        mlastLogIndex : SmokeNat, msource : Server, mdest : Server]
AEQ == [mtype : {AppendEntriesRequest}, mterm : SmokeNat, mprevLogIndex : -1..1,
        mprevLogTerm : SmokeNat, mentries : UpTo(Entry, 1), mcommitIndex : SmokeNat,
        msource : Server, mdest : Server]
RVP == [mtype : {RequestVoteResponse}, mterm : SmokeNat, mvoteGranted : BOOLEAN,
        mlog : UpTo(Entry, 1), msource : Server, mdest : Server]
AEP == [mtype : {AppendEntriesResponse}, mterm : SmokeNat, msuccess : BOOLEAN,
        mmatchIndex : SmokeNat, msource : Server, mdest : Server]

SmokeInit ==
    /\ currentTerm \in RandomSubset(k, [Server -> SmokeNat])
    /\ state \in RandomSubset(k, [Server -> {Follower, Candidate, Leader}])
    /\ votedFor \in RandomSubset(k, [Server -> Server \cup {Nil}])
    /\ log \in RandomSubset(k, [Server -> UpTo(Entry, 3)])
    /\ commitIndex \in RandomSubset(k, [Server -> SmokeNat])
    /\ votesResponded \in RandomSubset(k, [Server -> SUBSET Server])
    /\ votesGranted \in RandomSubset(k, [Server -> SUBSET Server])
    /\ nextIndex \in RandomSubset(k, [Server -> [Server -> {n \in SmokeNat : n >= 1}]])
    /\ matchIndex \in RandomSubset(k, [Server -> [Server -> SmokeNat]])
    /\ messages \in [RandomSubset(k, RandomSubset(k, RVQ) \cup RandomSubset(k, AEQ)
                                     \cup RandomSubset(k, RVP) \cup RandomSubset(k, AEP)) -> {1}]

Budget == TLCGet("duration") < 10
====
