"""The measurement tools behind DESIGN.md §e's numbers, run on the committed
inputs: the 8-GPU plan of the XL bench workload (profiles/r06/dist8/), the cost
model of the old bench model (profiles/r04/dist8/) and the plan of
specs/MCraftBench8.cfg reproduce the figures DESIGN quotes, and the sharded
kernel's measured rate (--k-dist) enters the expansion term.  CPU only."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D8 = os.path.join(ROOT, "profiles", "r04", "dist8")
X8 = os.path.join(ROOT, "profiles", "r06", "dist8")


def _run(args):
    out = subprocess.run([sys.executable] + args, cwd=ROOT, check=True, capture_output=True, text=True).stdout
    return [json.loads(ln) for ln in out.splitlines() if ln.strip()]


def _cost_model(*extra):
    return _run(["tools/dist_cost_model.py", os.path.join(D8, "levels_MCraftBench.jsonl"),
                 os.path.join(D8, "rounds_MCraftBench_rep.txt"), os.path.join(D8, "dist8_MCraftBench_rep.json"),
                 "8", str(1 << 20), *extra])


def test_cost_model_reproduces_the_design_table():
    head, fast, mid, slow = _cost_model()
    assert head["levels"] == 56 and head["rounds_total"] == 54
    assert head["T1_s"] == pytest.approx(0.2380, abs=1e-3)
    assert mid["replicated_levels"] == 23
    # the serial model at the three latency rows with 12-B key records (round 6;
    # DESIGN.md §e quoted 55.8 / 63.2 / 76.6 ms for round 5's 16-B records)
    for row, t8 in ((fast, 54.6), (mid, 62.0), (slow, 75.4)):
        assert row["T_N_ms"] == pytest.approx(t8, abs=0.1)
        assert row["expand_ms"] == pytest.approx(35.7, abs=0.1)


def test_xl_plan_reproduces_the_design_table():
    rows = _run(["tools/bench8_plan.py", os.path.join(X8, "levels_MCraftBenchXL_depth36.jsonl"),
                 os.path.join(X8, "rounds_MCraftBenchXL_depth36.txt"),
                 os.path.join(X8, "dist8_MCraftBenchXL_depth36.json"), os.path.join(D8, "levels_MCraftBench.jsonl"),
                 "8", "--k-dist", "1.072", "--table-frac", "0.5", "--measured",
                 os.path.join(X8, "levels_MCraftBenchXL.jsonl")])
    head, plan = rows[0], rows[-1]
    assert head["prefix_depth"] == 35 and head["counted_distinct"] == 1_223_708_472
    assert plan["distinct_est"] == 4_132_397_328 and plan["T1_model_s"] == pytest.approx(0.7398, abs=1e-3)
    # DESIGN.md §e (round 6): serial 178.0 / 194.7 / 224.7 ms, overlapped 133.7 / 142.9 / 162.1 ms
    assert plan["T_N_ms"] == pytest.approx([178.0, 194.7, 224.7], abs=0.11)
    assert plan["T_N_ms_overlapped"] == pytest.approx([133.7, 142.9, 162.1], abs=0.11)
    assert plan["expand_ms"][0] == pytest.approx(112.7, abs=0.11)
    # the pipelined rounds expose the last round's exchange and latency only
    assert plan["overlapped_latency_ms"][1] < plan["latency_ms"][1]


def test_cost_model_prices_the_sharded_kernel_rate():
    base = _cost_model()[2]
    slow = _cost_model("--k-dist", "1.2")[2]
    assert slow["k_dist"] == 1.2
    assert slow["expand_ms"] > base["expand_ms"]
    # only the exchanged levels' per-state share scales; everything else is unchanged
    assert slow["latency_ms"] == base["latency_ms"] and slow["xgmi_ms"] == base["xgmi_ms"]
    assert slow["T_N_ms"] - base["T_N_ms"] == pytest.approx(slow["expand_ms"] - base["expand_ms"], rel=1e-9)


def test_bench8_plan_sizes_the_8_gpu_model():
    rows = _run(["tools/bench8_plan.py", os.path.join(D8, "levels_MCraftBench8_depth28.jsonl"),
                 os.path.join(D8, "rounds_MCraftBench8_depth28.txt"),
                 os.path.join(D8, "dist8_MCraftBench8_depth28.json"), os.path.join(D8, "levels_MCraftBench.jsonl"),
                 "8", "--sizing", os.path.join(ROOT, "profiles", "r03", "sizing_next_bounds.txt")])
    head, plans = rows[0], rows[1:]
    assert head["prefix_depth"] == 27  # the depth-28 run expands 27 levels
    assert [p["stretch"] for p in plans] == [1.0, 1.15, 1.3]
    est = [p["distinct_est"] for p in plans]
    assert est == sorted(est) and 13.0e9 < est[0] and est[-1] < 15.7e9
    for p in plans:
        m = p["memory"]
        assert m["fits"] and m["total_GB"] < 288
        assert len(p["T_N_ms"]) == 3 and all(s > 4 for s in p["speedup"])
