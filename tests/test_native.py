"""Host-side checks of the packed successor code (raft.tla_amd/csrc/raft_packed.h,
compiled for the host with g++; no GPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lane_superset_covers_every_enabled_lane(tmp_path):
    """k_expand_sort / k_expand_sym / k_expand_dist walk only the lanes in the
    OR over a wave of lane_superset (role and slot occupancy): every lane that
    lane_delta enables must be in it, or successors would be silently dropped.
    Random walks from Init, every shape (S = 2..5, K = 4 and 8), |Value| = 1 and 2."""
    exe = tmp_path / "lane_mask_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I",
                    os.path.join(ROOT, "raft.tla_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "lane_mask_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "1500", "60", "3"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout


def test_diamond_skipping_keeps_every_level_count(tmp_path):
    """Commuting-diamond probe elimination (raft_packed.h diamond_of /
    diamond_skip, used by k_expand_sort and k_expand_dist): a host BFS on the
    kernels' own lane code, run with and without skipping, must find the same
    per-level new-state counts, generated count and depth, and the kernels'
    rule must agree with the model's independent restatement on every probed
    lane.  The counts are the oracle's (tests/golden/oracle_levels.json)."""
    import json
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_levels.json")))
    exe = tmp_path / "diamond_model"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I",
                    os.path.join(ROOT, "raft.tla_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "diamond_model.cpp"), "-o", str(exe)], check=True)
    for case in ("tiny2", "tiny2_v2", "s4_prefix10", "s5_prefix9", "msgs5_dup2_prefix9", "bounded_prefix14"):
        g = golden[case]
        p = g["params"]
        r = subprocess.run([str(exe)] + [str(p[k]) for k in ("n_servers", "n_values", "max_term", "max_log_len",
                                                              "max_msgs", "max_dup", "max_depth")],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout + r.stderr
        rec = json.loads(r.stdout)
        assert rec["same_levels"] and rec["kernel_rule_mismatches"] == 0, rec
        assert (rec["with_skip"]["distinct"], rec["with_skip"]["generated"]) == (g["distinct"], g["generated"]), case
        assert rec["skippable_frac"] > 0.15, rec  # worth a kernel change


def test_tlc_draw_follows_the_random_start_prime_stride_rule(tmp_path):
    """RMC_SIM_TLC (raft_wide.h tlc_draw, both wide simulators): for random sets
    of enabled lanes, every lane is drawn with the exact probability of TLC's
    simulator rule — random start among Next's actions, random prime stride,
    the first action with a successor, a uniform successor of it — within 6
    standard deviations over 200,000 draws per set; the rule is measurably not
    "uniform over the enabled actions" (VERDICT r04 missing item 4)."""
    exe = tmp_path / "tlc_draw_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I",
                    os.path.join(ROOT, "raft.tla_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "tlc_draw_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "30", "200000", "5"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
    assert float(r.stdout.split("max |P(action) - 1/(enabled actions)| ")[1]) > 0.01
