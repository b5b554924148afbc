"""SYMMETRY expansion timing (config 2 kernel) for one librmc.so build: the
MCraftBench bounds (MaxMsgs 3) under SYMMETRY Permutations(Server) and the
MCraftBoundedSym bounds (MaxMsgs 2), 3 runs each.  Measurement tool.

    python tools/sym_bench.py [abtest/librmc_<name>.so]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

if len(sys.argv) > 1:
    rmc.LIB_PATH = os.path.join(ROOT, sys.argv[1])
for msgs in (3, 2):
    for rep in range(3):
        cfg = rmc.make_config(max_msgs=msgs, symmetry=True)
        with rmc.Checker(cfg) as ck:
            r = ck.run()
        print(json.dumps(dict(lib=sys.argv[1] if len(sys.argv) > 1 else "default", max_msgs=msgs, rep=rep,
                              distinct=r.distinct, generated=r.generated, depth=r.depth,
                              seconds=r.seconds, kernel_s=r.expand_kernel_seconds,
                              orbits_per_s=r.distinct / r.seconds)), flush=True)
