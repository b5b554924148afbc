---- MODULE MCraftSmoke ----
\* Simulation model of config 4 (BASELINE.json configs[3]): the parameters of
\* Smokeraft.tla's SmokeInit sampler (k = 2 -> 512 initial states, SmokeNat =
\* 0..2, Smokeraft.tla:10-19) over MCraft's 3 servers and 2 values.  rmc-tlc
\* -simulate samples SmokeInit itself (RandomSubset(k, .) per variable,
\* Smokeraft.tla:64-76).  SmokeInit below restates Smokeraft's sampler (same
\* domains, this repo's layout), so TLC runs the same model.
EXTENDS MCraftBounded, TLC, Randomization

SmokeNat ==
    0..2

k ==
    2

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

Budget == TLCGet("duration") < 1
====
