"""The reference's own MCraft.cfg layout (tests/golden/models/MCunbounded.cfg: no
CONSTRAINT, terms / logs / bags / counts unbounded) under a BFS depth bound on
the wide layout: per level the new states, generated,
cumulative seconds and rate; the deepest bound one GPU completes; the record
size the front-end picked (336-B depth-sized up to depth 14, 904-B compact up to
depth 17).  Measurement tool.

    python tools/mcraft_shipped.py MAX_DEPTH [record: auto|full|compact|depth] > levels.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
depth = int(sys.argv[1])
rec = sys.argv[2] if len(sys.argv) > 2 else "auto"
if rec != "auto":
    os.environ["RMC_WIDE_COMPACT"] = {"full": "0", "compact": "1", "depth": "2"}[rec]
import rmc  # noqa: E402

base, _, _ = rmc.model_from_files(os.path.join(ROOT, "tests", "golden", "models", "MCunbounded.cfg"),
                                  builtin_raft=True, depth_bounded=True)
c = rmc.Config.from_buffer_copy(base)
c.max_depth = depth
c.state_capacity = 0  # librmc's own sizing: 80 % of free HBM
nbytes = rmc.native().rmc_state_bytes(c)


def progress(s):
    print(json.dumps({"level": s.level, "new": s.new_states, "distinct": s.distinct, "generated": s.generated,
                      "seconds": s.seconds}), flush=True)
    return 0


with rmc.Checker(c) as ck:
    try:
        r = ck.run(progress=progress)
        print(json.dumps({"max_depth": depth, "record_bytes": nbytes, "complete": True, "distinct": r.distinct,
                          "generated": r.generated, "depth": r.depth, "left_on_queue": r.left_on_queue,
                          "seconds": r.seconds, "distinct_per_s": r.distinct / r.seconds if r.seconds else None,
                          "capacity": ck.capacity if hasattr(ck, "capacity") else None}), flush=True)
    except rmc.RmcError as e:
        print(json.dumps({"max_depth": depth, "record_bytes": nbytes, "complete": False, "error": str(e)}), flush=True)
