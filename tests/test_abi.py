"""CPU tests of the C-ABI boundary (include/rmc.h) and the TLC front-end.
No compute calls: the GPU paths are in test_gpu.py."""
import ctypes as C
import os
import re
import subprocess

import pytest

import rmc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = os.path.join(ROOT, "specs")


def header_functions():
    text = open(os.path.join(ROOT, "include", "rmc.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rmc_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = rmc.native()
    declared = header_functions()
    assert set(declared) == set(rmc.EXPORTS), declared
    for name in declared:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", rmc.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in declared:
        assert re.search(rf"\bT {name}\b", out), name


def header_struct_fields(name):
    text = open(os.path.join(ROOT, "include", "rmc.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), text, flags=re.S).group(1)
    names = []
    for _, decl in re.findall(r"\b(u?int\d+_t|double|float)\s+([\w\s,\[\]]+);", body):
        names += [re.sub(r"\[.*", "", d).strip() for d in decl.split(",")]
    return names


@pytest.mark.parametrize("cname,pyname", [("rmc_config", "Config"), ("rmc_result", "Result"),
                                          ("rmc_sim_config", "SimConfig"), ("rmc_sim_result", "SimResult")])
def test_ctypes_structs_mirror_the_header(cname, pyname):
    """The Python binding's structs list the header's fields in order (a field
    added to one and not the other shifts every later field)."""
    want = header_struct_fields(cname)
    got = [f[0] for f in getattr(rmc, pyname)._fields_]
    assert got == want, (cname, got, want)


def test_library_is_gfx950_code():
    blob = open(rmc.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_version_and_state_bytes():
    lib = rmc.native()
    assert b"gfx950" in lib.rmc_version()
    cfg = rmc.make_config(n_servers=3, max_msgs=4)
    assert lib.rmc_state_bytes(C.byref(cfg)) == (2 * 3 + 4) * 4
    cfg = rmc.make_config(n_servers=5, max_msgs=6)
    assert lib.rmc_state_bytes(C.byref(cfg)) == (2 * 5 + 8) * 4


def test_wide_bfs_record_is_sized_from_the_run(monkeypatch):
    """the wide BFS stores compact 904-B records (16 log
    entries, 16 messages) when no state of the run can need more — a CONSTRAINT
    within them, or at most 16 steps of an unbounded field (one step adds at
    most one log entry and one distinct message) — else the full 5,080 B."""
    lib = rmc.native()
    unb = rmc.FLAG_UNBOUNDED_TERM | rmc.FLAG_UNBOUNDED_LOG | rmc.FLAG_UNBOUNDED_MSGS | rmc.FLAG_UNBOUNDED_DUP

    def nbytes(**kw):
        flags = kw.pop("flags", 0)
        cfg = rmc.make_config(**kw)
        cfg.flags |= flags
        return lib.rmc_state_bytes(C.byref(cfg))
    shipped = dict(max_term=255, max_log_len=32, max_msgs=64, max_dup=255, flags=unb)  # MCraft.cfg as shipped
    assert nbytes(max_depth=17, **shipped) == 904
    assert nbytes(max_depth=18, **shipped) == 5080
    assert nbytes(max_depth=0, **shipped) == 5080
    assert nbytes(max_log_len=16, max_msgs=16) == 904     # bounded within the compact record
    assert nbytes(max_log_len=16, max_msgs=17) == 5080
    assert nbytes(max_log_len=17, max_msgs=9, max_depth=17) == 904  # bounded beyond it, but 16 steps
    monkeypatch.setenv("RMC_WIDE_COMPACT", "0")
    assert nbytes(max_depth=8, **shipped) == 5080


def test_create_validates_config():
    lib = rmc.native()
    ctx = C.c_void_p()
    bad = rmc.make_config(max_log_len=33)  # beyond the wide layout's 32 entries too
    assert lib.rmc_create(C.byref(bad), C.byref(ctx)) == -22
    bad = rmc.make_config(max_log_len=4, symmetry=True)  # the wide layout has no SYMMETRY
    assert lib.rmc_create(C.byref(bad), C.byref(ctx)) == -22
    bad = rmc.make_config(max_term=256)
    assert lib.rmc_create(C.byref(bad), C.byref(ctx)) == -22
    bad = rmc.make_config(n_servers=6, symmetry=True)
    assert lib.rmc_create(C.byref(bad), C.byref(ctx)) == -22
    bad = rmc.make_config(invariants=1 << 10)
    assert lib.rmc_create(C.byref(bad), C.byref(ctx)) == -22


def test_create_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(rmc.RmcError) as e:
        rmc.Checker(rmc.make_config())
    assert e.value.code == -19


def test_cli_reports_model_and_fails_without_gpu():
    exe = os.path.join(ROOT, "raft.tla_amd", "bin", "rmc-tlc")
    r = subprocess.run([exe, "-builtin-raft", "-config", os.path.join(SPECS, "MCraftBug.cfg"),
                        os.path.join(SPECS, "MCraftBug.tla")], capture_output=True, text=True)
    assert "quorum guard weakened" in r.stdout
    try:
        import torch
        gpu = torch.cuda.is_available()
    except ImportError:
        gpu = False
    if not gpu:
        assert r.returncode != 0
