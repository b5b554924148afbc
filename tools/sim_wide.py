"""Smokeraft's walks: specs/MCraftSmoke.cfg (no bounds
but its 1-s Budget, so the front-end puts it on the wide layout) in each draw
mode, and the same model held to the packed capacity (MaxTerm 14, MaxLogLen 3,
8 messages, count 3: what rounds 1-3 ran), with the fraction of behaviours that
left the layout (truncated) and the steps/s.  Measurement tool.

    python tools/sim_wide.py [behaviours] > sim_wide.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
UNB = rmc.FLAG_UNBOUNDED_TERM | rmc.FLAG_UNBOUNDED_LOG | rmc.FLAG_UNBOUNDED_MSGS | rmc.FLAG_UNBOUNDED_DUP
for wide in (True, False):
    cfg, _, _ = rmc.model_from_files(os.path.join(ROOT, "specs", "MCraftSmoke.cfg"), builtin_raft=True, simulate=True)
    cfg.state_capacity = 1 << 12
    label = "MCraftSmoke.cfg, wide layout (unbounded)"
    if not wide:
        cfg.max_term, cfg.max_log_len, cfg.max_msgs, cfg.max_dup = 14, 3, 8, 3
        cfg.flags &= ~UNB
        label = "MCraftSmoke.cfg held to the packed capacity"
    modes = (rmc.SIM_WITHIN_CAPACITY, rmc.SIM_TRUNCATE) + ((rmc.SIM_TLC,) if wide else ())
    with rmc.Checker(cfg) as ck:
        for mode in modes:
            ck.simulate(behaviours=1 << 16, depth=100, smoke_k=2, seed=1, mode=mode)  # warm
            r = ck.simulate(behaviours=n, depth=100, smoke_k=2, seed=7, mode=mode)
            print(json.dumps({"model": label, "state_bytes": rmc.native().rmc_state_bytes(cfg), "mode": mode,
                              "behaviours": r.behaviours, "steps": r.steps, "truncated": r.truncated,
                              "truncated_frac": r.truncated / max(1, r.behaviours), "deadlocked": r.deadlocked,
                              "violated_inv": r.violated_inv, "seconds": r.seconds,
                              "steps_per_s": r.steps / r.seconds if r.seconds else None,
                              "bounds": [cfg.max_term, cfg.max_log_len, cfg.max_msgs, cfg.max_dup]}), flush=True)
