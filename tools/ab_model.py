"""A/B timing of one TLC model on alternative librmc.so builds (measurement
tool): python tools/ab_model.py abtest/librmc_<name>.so specs/X.cfg [depth] [sim]
prints one JSON line (best of 3 runs) — BFS, or with `sim` the config-4
simulation (16 M behaviours of depth 100, SmokeInit k = 2)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

rmc.LIB_PATH = os.path.join(ROOT, sys.argv[1])
cfg_path = sys.argv[2]
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 0
sim = len(sys.argv) > 4 and sys.argv[4] == "sim"
if sim:
    cfg, sc, _ = rmc.model_from_files(cfg_path, builtin_raft=True, simulate=True)
else:
    cfg = rmc.config_from_files(cfg_path, builtin_raft=True)
cfg.max_depth = depth
cfg.state_capacity = 1_500_000_000
best = None
with rmc.Checker(cfg) as ck:
    for _ in range(3):
        if sim:
            r = ck.simulate(1 << 24, 100, sc.smoke_k, sc.smoke_nat, seed=1)
            t, rec = r.seconds, {"steps": r.steps}
        else:
            r = ck.run(record_levels=False)
            t, rec = r.seconds, {"distinct": r.distinct, "generated": r.generated, "depth": r.depth,
                                 "kernel_s": r.expand_kernel_seconds}
        if best is None or t < best[0]:
            best = (t, rec)
print(json.dumps({"lib": sys.argv[1], "cfg": cfg_path, "depth": depth, "sim": sim, "seconds": best[0], **best[1]}))
