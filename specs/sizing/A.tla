---- MODULE A ----
EXTENDS MCraftBounded
====
