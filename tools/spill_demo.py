"""Frontier spill at scale: the MCraftBench bounds searched with every state
resident, then again with a device window of about the two largest levels —
well under half the search — so the expanded levels move to pinned host
memory.  Counts must agree; prints one JSON line per run.  Measurement tool.

    python tools/spill_demo.py [window_states]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402


def run(cfg, tag):
    with rmc.Checker(cfg) as ck:
        r = ck.run()
        levels = [lv[3] for lv in ck.levels if lv[3]]
    out = dict(run=tag, distinct=r.distinct, generated=r.generated, depth=r.depth, seconds=r.seconds,
               kernel_s=r.expand_kernel_seconds, launches=r.expand_launches, spilled=r.spilled, spills=r.spills,
               spill_s=r.spill_seconds, window=cfg.device_window, capacity=cfg.state_capacity)
    print(json.dumps(out), flush=True)
    return r, [1] + levels


r0, L = run(rmc.make_config(max_msgs=3), "resident")
pair = max(a + b for a, b in zip(L, L[1:]))
win = int(sys.argv[1]) if len(sys.argv) > 1 else int(pair * 1.05) + (1 << 26)
cfg = rmc.make_config(max_msgs=3, spill=True, device_window=win, state_capacity=int(r0.distinct * 1.3))
r1, L1 = run(cfg, "spill")
assert (r1.distinct, r1.generated, r1.depth) == (r0.distinct, r0.generated, r0.depth) and L1 == L
print(json.dumps(dict(check="counts and levels agree", largest_pair=pair, window=win,
                      resident_fraction=win / r0.distinct)), flush=True)
