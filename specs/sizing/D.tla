---- MODULE D ----
EXTENDS MCraftBounded
====
