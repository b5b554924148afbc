---- MODULE MCraftBench ----
\* Root module for MCraftBench.cfg (the bench workload): the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
