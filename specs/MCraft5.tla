---- MODULE MCraft5 ----
\* Root module for MCraft5.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
