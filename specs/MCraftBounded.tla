---------------------------- MODULE MCraftBounded ----------------------------
\* Repo-local bounded model of raft.tla (SURVEY.md §7 step 0).  MCraft.cfg as
\* shipped has no CONSTRAINT, so its state space is infinite (SURVEY.md §0.2);
\* this module adds the state constraint that TLC and rmc-tlc both apply
\* before the seen-set.  Model values as in MCraft.tla:5-21.
EXTENDS raft, FiniteSets, TLC

CONSTANTS r1, r2, r3, r4, r5, v1, v2
CONSTANTS MaxTerm, MaxLogLen, MaxMsgs, MaxDup

Servers2 == {r1, r2}
Servers3 == {r1, r2, r3}
Servers4 == {r1, r2, r3, r4}
Servers5 == {r1, r2, r3, r4, r5}
Values1 == {v1}
Values2 == {v1, v2}

StateConstraint ==
    /\ \A i \in Server : currentTerm[i] <= MaxTerm /\ Len(log[i]) <= MaxLogLen
    /\ Cardinality(DOMAIN messages) <= MaxMsgs
    /\ \A m \in DOMAIN messages : messages[m] <= MaxDup

\* ElectionSafety (raft.tla:1124-1129) takes Max of a possibly empty set and
\* cannot be evaluated by TLC (SURVEY.md §0.9); this is the standard form.
OneLeaderPerTerm ==
    \A i, j \in Server :
        (state[i] = Leader /\ state[j] = Leader /\ currentTerm[i] = currentTerm[j]) => i = j

\* raft.tla:1132-1136 (restated: past the module end of raft.tla).
LogMatching ==
    \A i, j \in Server :
        \A n \in (1..Len(log[i])) \cap (1..Len(log[j])) :
            log[i][n].term = log[j][n].term =>
            SubSeq(log[i],1,n) = SubSeq(log[j],1,n)

\* ---- Proof invariants of raft.tla, restated -------------------------------
\* raft.tla defines these past its module end (raft.tla:892-1180), where SANY
\* and TLC never read them, so a model that checks them must define them
\* itself.  The restatements below are what rmc-tlc compiles (the front-end
\* refuses any other definition under these names).

\* MessagesInv (raft.tla:941-946) and its four parts (:903-935).  `m.dest` at
\* :910 is read as `m.mdest`; `log[src][mprevLogIndex + 1]` outside the log's
\* domain is a violation here, where raft.tla's text would be an evaluation
\* error.
RVResponseInv(m) ==
    (/\ m.mtype = RequestVoteResponse
     /\ m.mvoteGranted
     /\ currentTerm[m.msource] = currentTerm[m.mdest]
     /\ currentTerm[m.msource] = m.mterm)
    => \/ LastTerm(log[m.mdest]) > LastTerm(log[m.msource])
       \/ /\ LastTerm(log[m.mdest]) = LastTerm(log[m.msource])
          /\ Len(log[m.mdest]) >= Len(log[m.msource])

RVRequestInv(m) ==
    (/\ m.mtype = RequestVoteRequest
     /\ state[m.msource] = Candidate
     /\ currentTerm[m.msource] = m.mterm)
    => /\ m.mlastLogIndex = Len(log[m.msource])
       /\ m.mlastLogTerm = LastTerm(log[m.msource])

AERequestInv(m) ==
    (/\ m.mtype = AppendEntriesRequest
     /\ m.mentries /= << >>
     /\ m.mterm = currentTerm[m.msource])
    => /\ m.mprevLogIndex + 1 \in DOMAIN log[m.msource]
       /\ log[m.msource][m.mprevLogIndex + 1] = m.mentries[1]
       /\ m.mprevLogIndex > 0 => log[m.msource][m.mprevLogIndex].term = m.mprevLogTerm

MessagesInv ==
    \A m \in DOMAIN messages :
        /\ RVResponseInv(m)
        /\ RVRequestInv(m)
        /\ AERequestInv(m)
        /\ m.mterm <= currentTerm[m.msource]

\* LeaderVotesQuorum (raft.tla:1033-1037): a leader's term is backed by a
\* quorum that voted for it or has moved on to a higher term.
LeaderVotesQuorum ==
    \A i \in Server : state[i] = Leader =>
        {j \in Server : \/ currentTerm[j] > currentTerm[i]
                        \/ currentTerm[j] = currentTerm[i] /\ votedFor[j] = i} \in Quorum

\* CandidateTermNotInLog (raft.tla:1041-1047): a candidate that can still win
\* has no entry of its term in any log.
CandidateTermNotInLog ==
    \A i \in Server :
        (/\ state[i] = Candidate
         /\ {j \in Server : currentTerm[j] = currentTerm[i] /\ votedFor[j] \in {i, Nil}} \in Quorum)
        => \A j \in Server : \A n \in DOMAIN log[j] : log[j][n].term /= currentTerm[i]

\* The IsPrefix invariants (raft.tla:1143-1180).  raft.tla's Committed(i) is
\* SubSeq(log[i], 1, commitIndex[i]), out of range whenever commitIndex[i]
\* exceeds Len(log[i]) -- which this spec allows (AppendEntriesAlreadyDone
\* adopts m.mcommitIndex, :309; ConflictAppendEntriesRequest shortens the log,
\* :319-325).  The rule chosen here: the committed prefix is the part of the
\* log the commit index covers, min(commitIndex[i], Len(log[i])) entries.
\* IsPrefix is not defined by raft.tla's EXTENDS; this is SequencesExt's.
IsPrefix(s, t) == Len(s) <= Len(t) /\ SubSeq(t, 1, Len(s)) = s

Committed(i) ==
    SubSeq(log[i], 1, IF commitIndex[i] <= Len(log[i]) THEN commitIndex[i] ELSE Len(log[i]))

VotesGrantedInv ==
    \A i \in Server : \A j \in votesGranted[i] :
        currentTerm[i] = currentTerm[j] => IsPrefix(Committed(j), log[i])

QuorumLogInv ==
    \A i \in Server : \A Q \in Quorum : \E j \in Q : IsPrefix(Committed(i), log[j])

MoreUpToDateCorrect ==
    \A i, j \in Server :
        (\/ LastTerm(log[i]) > LastTerm(log[j])
         \/ LastTerm(log[i]) = LastTerm(log[j]) /\ Len(log[i]) >= Len(log[j]))
        => IsPrefix(Committed(j), log[i])

LeaderCompleteness ==
    \A i \in Server : state[i] = Leader => \A j \in Server : IsPrefix(Committed(j), log[i])

ServerSymmetry == Permutations(Server)

\* Config-5 bug variant: BecomeLeader with the quorum guard (raft.tla:197)
\* weakened.  Selected in a cfg with `BecomeLeader <- BugBecomeLeader`.
BugBecomeLeader(i) ==
    /\ state[i] = Candidate
    /\ votesGranted[i] /= {}
    /\ state'      = [state EXCEPT ![i] = Leader]
    /\ nextIndex'  = [nextIndex EXCEPT ![i] =
                         [j \in Server |-> Len(log[i]) + 1]]
    /\ matchIndex' = [matchIndex EXCEPT ![i] =
                         [j \in Server |-> 0]]
    /\ UNCHANGED <<messages, currentTerm, votedFor, candidateVars, logVars>>
=============================================================================
