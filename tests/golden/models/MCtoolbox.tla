---- MODULE MCtoolbox ----
\* Parse fixture: a model module in the layout the TLA+ Toolbox generates
\* (model values declared as CONSTANTS, set-valued definitions named
\* const_<id>, sections closed by separator lines), plus a state bound.
EXTENDS raft, FiniteSets

CONSTANTS
s1, s2, s3
----

CONSTANTS
w1, w2
----

const_100 ==
{s1, s2, s3}
----

const_200 ==
{w1, w2}
----

Bound ==
    /\ \A i \in Server : currentTerm[i] <= 2 /\ Len(log[i]) <= 1
    /\ Cardinality(DOMAIN messages) <= 2
    /\ \A m \in DOMAIN messages : messages[m] <= 1
====
