import json, os, subprocess, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
probe = r'''
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "raft.tla_amd")); sys.path.insert(0, sys.argv[1])
import rmc
from tests.convert import from_view
c, _, _ = rmc.model_from_files(os.path.join(sys.argv[1], "tests", "golden", "models", "SmokeFixture.cfg"), builtin_raft=True, simulate=True)
c.state_capacity = 1 << 12
with rmc.Checker(c) as ck:
    views = ck.sim_replay(77, behaviours=4096, depth=100, smoke_k=2, seed=5, mode=rmc.SIM_TRUNCATE)
    print(json.dumps([repr(from_view(v)) for v in views]))
'''
outs = []
for w in ("0", "1"):
    p = subprocess.run([sys.executable, "-c", probe, ROOT], env=dict(os.environ, RMC_WSIM=w, PYTHONHASHSEED="0"), capture_output=True, text=True, timeout=200)
    if p.returncode: print(p.stderr[-3000:]); sys.exit(1)
    outs.append(json.loads(p.stdout.strip().splitlines()[-1]))
a, b = outs
for i, (x, y) in enumerate(zip(a, b)):
    if x != y:
        print("first difference at step", i)
        print("prev :", a[i-1])
        print("thread:", x)
        print("wave  :", y)
        break
else:
    print("identical", len(a), len(b))
