---- MODULE MCraft5Wide ----
\* Root module for MCraft5Wide.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
