---- MODULE MCunbounded ----
\* Fixture: a model module in the layout the TLA+ Toolbox generates, with NO
\* state constraint — the shape of the reference's MCraft.cfg as shipped
\* (model values for servers and values, Server/Value bound by `<-`, TypeOK).
\* Its state space is infinite; it runs only under a depth bound (-depth N).
EXTENDS raft

CONSTANTS
s1, s2, s3
----

CONSTANTS
w1, w2
----

const_300 ==
{w1, w2}
----

const_400 ==
{s1, s2, s3}
----
====
