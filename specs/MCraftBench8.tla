---- MODULE MCraftBench8 ----
\* Root module for MCraftBench8.cfg (the 8-GPU bench workload, MaxMsgs 4): the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
