---- MODULE MCraftBug ----
\* Root module for MCraftBug.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
