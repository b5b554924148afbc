---- MODULE MCraftMessages ----
\* Root module for MCraftMessages.cfg: the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
