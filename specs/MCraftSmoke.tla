---- MODULE MCraftSmoke ----
\* Simulation model of config 4 (BASELINE.json configs[3]): the parameters of
\* Smokeraft.tla's SmokeInit sampler (k = 2 -> 512 initial states, SmokeNat =
\* 0..2, Smokeraft.tla:10-19) over MCraft's 3 servers and 2 values.  rmc-tlc
\* -simulate samples SmokeInit itself (RandomSubset(k, .) per variable,
\* Smokeraft.tla:64-76); run the reference's own Smokeraft.tla/.cfg with TLC.
EXTENDS MCraftBounded, TLC

SmokeNat ==
    0..2

k ==
    2

SmokeInit == Init

Budget == TLCGet("duration") < 1
====
