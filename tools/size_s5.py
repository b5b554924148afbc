"""Per-level sizes of 5-server models on one GPU (config 3 sizing): BFS with a
progress callback that stops before the device store fills.  Measurement tool.

    python tools/size_s5.py MaxTerm MaxLogLen MaxMsgs MaxDup [stop_at]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

mt, ml, mm, md = (int(x) for x in sys.argv[1:5])
stop = float(sys.argv[5]) if len(sys.argv) > 5 else 2.0e9
cfg = rmc.make_config(n_servers=5, n_values=2, max_term=mt, max_log_len=ml, max_msgs=mm, max_dup=md,
                      state_capacity=0)
rows = []


def prog(s):
    rows.append(dict(level=s.level + 1, distinct=s.distinct, new=s.new_states, generated=s.generated,
                     seconds=round(s.seconds, 3)))
    print(json.dumps(rows[-1]), flush=True)
    return int(s.distinct + 1.8 * s.new_states > stop)


with rmc.Checker(cfg) as ck:
    r = ck.run(progress=prog)
print(json.dumps(dict(bounds=[mt, ml, mm, md], distinct=r.distinct, depth=r.depth, left=r.left_on_queue,
                      kernel_s=r.expand_kernel_seconds)), flush=True)
