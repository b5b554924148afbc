---- MODULE MCraftSmall ----
\* Root module for MCraftSmall.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
