"""Model sizing on one GPU: run a list of bounded raft models (BFS to fixpoint or
until a time budget) and print one JSON line per model with distinct/generated/
depth/time.  Used to calibrate config 3 (5 servers, >= 1e9 distinct states,
BASELINE.json configs[2]).

    python tools/sizing.py S:V:MaxTerm:MaxLogLen:MaxMsgs:MaxDup[:verify][:spill][:dDEPTH][:cCAPACITY] ... [--budget SECONDS]

`spill`: expanded levels move to host memory when the device store fills
(RMC_FLAG_SPILL), so a model larger than HBM still runs to its fixpoint while
its fingerprints fit.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))

import rmc  # noqa: E402


def main():
    budget = 90.0
    specs = []
    args = sys.argv[1:]
    while args:
        a = args.pop(0)
        if a == "--budget":
            budget = float(args.pop(0))
        else:
            specs.append(a)
    for sp in specs:
        f = sp.split(":")
        s, v, t, l, mm, dd = (int(x) for x in f[:6])
        verify = "verify" in f[6:]
        spill = "spill" in f[6:]
        depth = max([int(x[1:]) for x in f[6:] if x.startswith("d")] or [0])
        cap = max([int(x[1:]) for x in f[6:] if x.startswith("c")] or [0])  # cN: state capacity (0: librmc's)
        cfg = rmc.make_config(n_servers=s, n_values=v, max_term=t, max_log_len=l, max_msgs=mm, max_dup=dd,
                              check_deadlock=False, verify_states=verify, max_depth=depth,
                              spill=spill, state_capacity=cap)
        t0 = time.time()
        rec = {"model": sp}
        try:
            with rmc.Checker(cfg) as ck:
                def prog(st):
                    print(f"  {sp} level {st.level} distinct {st.distinct} new {st.new_states} "
                          f"t {st.seconds:.2f}s", file=sys.stderr, flush=True)
                    return st.seconds > budget
                r = ck.run(prog)
                rec.update(distinct=r.distinct, generated=r.generated, depth=r.depth,
                           left_on_queue=r.left_on_queue, seconds=r.seconds,
                           kernel_seconds=r.expand_kernel_seconds, probes=r.probes,
                           complete=r.left_on_queue == 0,
                           verified=r.verified, collisions=r.collisions,
                           spilled=getattr(r, "spilled", 0), spills=getattr(r, "spills", 0),
                           rate=r.distinct / r.seconds if r.seconds else None)
        except rmc.RmcError as e:
            rec["error"] = str(e)
        rec["wall"] = time.time() - t0
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
