"""Per-level times of one BFS on one GPU (the sharded cost model's input):
one JSON line per level — level, frontier expanded, new states, generated,
seconds since the start — for a TLC model file.  Measurement tool.

    python tools/level_times.py specs/MCraftBench.cfg [capacity [max_depth [spill [set_bytes]]]] > levels.jsonl

capacity 0: librmc's own sizing; max_depth 0: to the fixpoint; `spill`:
RMC_FLAG_SPILL (how bench.py runs specs/MCraftBenchXL.cfg on one GPU);
set_bytes: rmc_config.set_bytes (bench.py's sparse set: 137438953472 for XL).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

cfg = rmc.config_from_files(sys.argv[1], builtin_raft=True)
cfg.state_capacity = int(sys.argv[2]) if len(sys.argv) > 2 else 1_500_000_000
if len(sys.argv) > 3:
    cfg.max_depth = int(sys.argv[3])  # a prefix of a model larger than one GPU
if len(sys.argv) > 4 and sys.argv[4] == "spill":
    cfg.flags |= rmc.FLAG_SPILL
if len(sys.argv) > 5:
    cfg.set_bytes = int(sys.argv[5])
with rmc.Checker(cfg) as ck:
    ck.run()  # warm
    r = ck.run()
    prev_t, prev_new, prev_gen = 0.0, 1, 1
    for (level, gen, distinct, new, sec) in ck.levels:
        print(json.dumps({"level": level, "frontier": prev_new, "new": new, "generated": gen - prev_gen,
                          "seconds": sec - prev_t, "t": sec}))
        prev_t, prev_new, prev_gen = sec, new, gen
    print(json.dumps({"distinct": r.distinct, "generated": r.generated, "depth": r.depth, "seconds": r.seconds,
                      "kernel_s": r.expand_kernel_seconds}))
