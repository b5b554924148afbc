"""A/B bench of alternative librmc.so builds on one GPU box (measurement tool,
not shipped).  Copy the builds to abtest/librmc_<name>.so (git-ignored .so),
then `bash tools/ab_bench.sh` under gpurun runs bench.py against each in turn.

    python tools/ab_bench.py librmc_old.so
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

rmc.LIB_PATH = os.path.join(ROOT, "abtest", sys.argv[1])
sys.argv = ["bench.py", "--no-cpu", "--no-probe-ceiling", "--steps", "5", "--warmup", "1"]
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
