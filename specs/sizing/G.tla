---- MODULE G ----
EXTENDS MCraftBounded
====
