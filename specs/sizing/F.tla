---- MODULE F ----
EXTENDS MCraftBounded
====
