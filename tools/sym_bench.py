"""SYMMETRY expansion timing (config 2 kernel) for one librmc.so build: the
MCraftBench bounds (MaxMsgs 3) under SYMMETRY Permutations(Server) and the
MCraftBoundedSym bounds (MaxMsgs 2), 3 runs each.  Measurement tool.

    python tools/sym_bench.py [abtest/librmc_<name>.so] [state_capacity]

state_capacity sizes the fingerprint set (0 = auto: most of HBM, whose
memset then costs ~14 ms per run).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] != "default":
    rmc.LIB_PATH = os.path.join(ROOT, sys.argv[1])
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for msgs in (3, 2):
    for rep in range(3):
        cfg = rmc.make_config(max_msgs=msgs, symmetry=True, state_capacity=cap)
        with rmc.Checker(cfg) as ck:
            r = ck.run()
        print(json.dumps(dict(lib=sys.argv[1] if len(sys.argv) > 1 else "default", capacity=cap, max_msgs=msgs, rep=rep,
                              distinct=r.distinct, generated=r.generated, depth=r.depth,
                              seconds=r.seconds, kernel_s=r.expand_kernel_seconds,
                              orbits_per_s=r.distinct / r.seconds)), flush=True)
