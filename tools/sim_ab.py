"""A/B of the wide simulator's knobs on Smokeraft's walks (MCraftSmoke.cfg,
depth 100): one process per setting (the knobs are read once per process),
settings alternated over rounds.  Measurement tool.

    python tools/sim_ab.py BEHAVIOURS MODE ROUNDS ENV=V[,ENV=V] ENV=V[,...] ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "raft.tla_amd"))
import rmc
c, _, _ = rmc.model_from_files(os.path.join(sys.argv[1], "specs", "MCraftSmoke.cfg"), builtin_raft=True, simulate=True)
c.state_capacity = 1 << 12
n, mode = int(sys.argv[2]), int(sys.argv[3])
with rmc.Checker(c) as ck:
    ck.simulate(behaviours=1 << 16, depth=100, smoke_k=2, seed=1, mode=mode)
    r = ck.simulate(behaviours=n, depth=100, smoke_k=2, seed=7, mode=mode)
print(json.dumps({"steps": r.steps, "truncated": r.truncated, "seconds": r.seconds,
                  "steps_per_s": r.steps / r.seconds}))
"""
n, mode, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
for rnd in range(rounds):
    for setting in sys.argv[4:]:
        env = dict(os.environ)
        for kv in setting.split(","):
            k, v = kv.split("=")
            env[k] = v
        p = subprocess.run([sys.executable, "-c", PROBE, ROOT, str(n), str(mode)], env=env, capture_output=True,
                           text=True, timeout=300)
        if p.returncode:
            sys.exit(p.stderr[-2000:])
        d = json.loads(p.stdout.strip().splitlines()[-1])
        print(json.dumps({"round": rnd, "setting": setting, "mode": mode, **d}), flush=True)
