"""The bench model (specs/MCraftBenchXL.cfg) to its fixpoint under several
fingerprint salts, as bench.py runs it on one GPU (spill, librmc's sizing):
distinct / generated / depth per salt.  Equal counts under independent members
of the fingerprint family are the size-independent evidence that no
fingerprint collision dropped a state (measurement tool).

    python tools/xl_salts.py [config] [salt ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

args = sys.argv[1:]
cfgp = args.pop(0) if args and args[0].endswith(".cfg") else os.path.join(ROOT, "specs", "MCraftBenchXL.cfg")
salts = [int(x, 0) for x in args] or [0, 0x5A17ED, 0xC0FFEE]
cfg = rmc.config_from_files(cfgp, builtin_raft=True)
cfg.flags |= rmc.FLAG_SPILL
with rmc.Checker(cfg) as ck:
    for s in salts:
        ck.set_seed(s)
        r = ck.run(record_levels=False)
        print(json.dumps({"config": os.path.basename(cfgp), "salt": s, "distinct": r.distinct,
                          "generated": r.generated, "depth": r.depth, "seconds": r.seconds,
                          "collision_estimate": r.collision_probability}), flush=True)
