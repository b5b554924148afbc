---- MODULE B ----
EXTENDS MCraftBounded
====
