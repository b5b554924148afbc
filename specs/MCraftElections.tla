---- MODULE MCraftElections ----
\* Root module for MCraftElections.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
