"""Generates tests/golden/front_models.json: the rmc_config the front-end
(rmc_model_from_files) produces for models read WITH a raft.tla on disk.

The GPU box has no raft.tla (it is the reference's source, which does not
travel), so the GPU tests cannot run the front-end on a real raft.tla
themselves.  This script runs it here, where /root/reference/raft.tla exists,
on (a) every shipped model in specs/ next to an unmodified raft.tla and (b)
BASELINE.json config 5 as it is worded, "bug-injected raft.tla": MCraftBug.cfg
without its BecomeLeader override, next to a raft.tla whose line 197 is
weakened.  tests/test_gpu.py runs the recorded configs and compares them with
the oracle fixtures; tests/test_front.py re-derives this file on CPU.

    python tests/golden/make_front_fixtures.py
"""
import json
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "raft.tla_amd"))
import rmc  # noqa: E402

REF_RAFT = "/root/reference/raft.tla"
FIELDS = ("n_servers", "n_values", "max_term", "max_log_len", "max_msgs", "max_dup", "flags", "invariants")


def build():
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for f in os.listdir(os.path.join(ROOT, "specs")):
            if f.endswith((".tla", ".cfg")):
                shutil.copy(os.path.join(ROOT, "specs", f), d)
        shutil.copy(REF_RAFT, d)
        for f in sorted(os.listdir(d)):
            if f.endswith(".cfg"):
                sim = "Smoke" in f
                cfg, _sc, info = rmc.model_from_files(os.path.join(d, f), simulate=sim)
                out[f[:-4]] = dict({k: getattr(cfg, k) for k in FIELDS}, notes=info.replace(d, "<dir>"))
        # config 5 as BASELINE.json words it: the bug injected into raft.tla itself
        text = open(REF_RAFT).read()
        weak = text.replace("/\\ votesGranted[i] \\in Quorum", "/\\ votesGranted[i] /= {}")
        assert weak != text
        with open(os.path.join(d, "raft.tla"), "w") as f:
            f.write(weak)
        bug = open(os.path.join(d, "MCraftBug.cfg")).read().replace("CONSTANT BecomeLeader <- BugBecomeLeader", "")
        with open(os.path.join(d, "MCraftBugRaft.cfg"), "w") as f:
            f.write(bug)
        shutil.copy(os.path.join(d, "MCraftBug.tla"), os.path.join(d, "MCraftBugRaft.tla"))
        with open(os.path.join(d, "MCraftBugRaft.tla")) as f:
            t = f.read().replace("MODULE MCraftBug ", "MODULE MCraftBugRaft ")
        with open(os.path.join(d, "MCraftBugRaft.tla"), "w") as f:
            f.write(t)
        cfg, _sc, info = rmc.model_from_files(os.path.join(d, "MCraftBugRaft.cfg"))
        out["MCraftBug_raft_tla_edited"] = dict({k: getattr(cfg, k) for k in FIELDS}, notes=info.replace(d, "<dir>"))
    return out


def main():
    path = os.path.join(ROOT, "tests", "golden", "front_models.json")
    with open(path, "w") as f:
        json.dump(build(), f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
