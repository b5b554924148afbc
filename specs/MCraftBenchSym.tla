---- MODULE MCraftBenchSym ----
\* Root module for MCraftBenchSym.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
