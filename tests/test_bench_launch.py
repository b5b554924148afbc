"""bench.py's launch contract: `--gpus N` runs N ranks by
itself when no outer launcher set WORLD_SIZE, a torchrun launch of N
processes is one rank each, and a line whose rank count differs from --gpus
is refused.  The CPU tests use --dry-run (rendezvous and timing collectives
over gloo, no GPU, no librmc); the GPU test runs the real sharded search on
the box's one GPU with the ranks sharing it over the host transport."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_levels.json")))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_starts_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], capture_output=True, text=True,
                       timeout=180, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["n_gpus"] == n and rec["dry_run"]
    assert sorted(x["rank"] for x in rec["ranks_seen"]) == list(range(n))
    assert len({x["pid"] for x in rec["ranks_seen"]}) == n  # one process per rank
    assert rec["launcher"].startswith("bench.py --gpus")


def test_torchrun_launch_is_one_rank_per_process():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29701", BENCH, "--gpus", "2", "--dry-run"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["launcher"] == "torchrun"
    assert sorted(x["rank"] for x in rec["ranks_seen"]) == [0, 1]


def test_rank_count_mismatch_is_refused():
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "refused" in r.stderr


@pytest.mark.gpu
def test_self_launch_two_ranks_on_the_gpu_matches_oracle():
    """`bench.py --gpus 2` on a one-GPU box: two rank processes share the GPU
    over the host transport and report the oracle's counts for MCraftSmall."""
    g = GOLDEN["small"]
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--transport", "host", "--config",
                        os.path.join(ROOT, "specs", "MCraftSmall.cfg"), "--steps", "1", "--warmup", "0",
                        "--no-cpu", "--capacity", str(1 << 22), "--keys-per-dest", str(1 << 16)],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["world"]["ranks"] == 2 and rec["world"]["transport"] == "host"
    c = rec["config"]
    assert (c["distinct"], c["generated"], c["depth"]) == (g["distinct"], g["generated"], g["depth"])
    assert sum(p["stored"] for p in rec["sharded"]["per_rank"]) == g["distinct"]
