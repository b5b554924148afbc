---- MODULE MCraftBenchXL ----
\* Root module for MCraftBenchXL.cfg (the bench workload of round 5: the largest bounded
\* model found that one GPU completes): the model lives in MCraftBounded.tla.
EXTENDS MCraftBounded
====
