---- MODULE SmokeFixture ----
\* Parse fixture for simulation models: `Init <- SmokeInit` with the sampler's
\* parameters k and SmokeNat, and a run-budget constraint that bounds no
\* variable.  The engine samples SmokeInit itself (rmc_simulate); the body
\* below only has to exist.
EXTENDS MCtoolbox, TLC

SmokeNat ==
    0..3

k ==
   3

SmokeInit == Init

Budget == TLCGet("duration") < 10
====
