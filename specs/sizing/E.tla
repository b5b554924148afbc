---- MODULE E ----
EXTENDS MCraftBounded
====
