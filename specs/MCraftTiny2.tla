---- MODULE MCraftTiny2 ----
\* Root module for MCraftTiny2.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
