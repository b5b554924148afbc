---- MODULE MCraftBoundedSym ----
\* Root module for MCraftBoundedSym.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
