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
