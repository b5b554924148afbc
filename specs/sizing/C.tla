---- MODULE C ----
EXTENDS MCraftBounded
====
