"""Host-side checks of the packed successor code (raft.tla_amd/csrc/raft_packed.h,
compiled for the host with g++; no GPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_incremental_symmetry_keys_equal_whole_successor_keys(tmp_path):
    """canon_delta_inc (the single-GPU SYMMETRY kernel's keys, from the parent's
    frame) must equal canon_delta (every relabelled component hashed) on every
    in-model lane of random walks from Init, for S = 2..5 and K = 4/8: same tie
    flag, and the same 64-bit key when untied, so orbit counts cannot differ."""
    exe = tmp_path / "sym_inc_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I",
                    os.path.join(ROOT, "raft.tla_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "sym_inc_check.cpp"), "-o", str(exe)], check=True)
    for walks, depth, seed in ((1500, 40, 1), (300, 100, 7)):
        r = subprocess.run([str(exe), str(walks), str(depth), str(seed)], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.startswith("ok "), r.stdout


def test_lane_superset_covers_every_enabled_lane(tmp_path):
    """k_expand_sort / k_expand_sym / k_expand_dist walk only the lanes in the
    OR over a wave of lane_superset (role and slot occupancy): every lane that
    lane_delta enables must be in it, or successors would be silently dropped.
    Random walks from Init, every shape with <= 64 lanes, |Value| = 1 and 2."""
    exe = tmp_path / "lane_mask_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I",
                    os.path.join(ROOT, "raft.tla_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "lane_mask_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "1500", "60", "3"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
