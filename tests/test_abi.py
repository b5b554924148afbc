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


@pytest.mark.parametrize("name,expect", [
    ("MCraftBounded", (3, 2, 2, 1, 2, 1, rmc.FLAG_CHECK_DEADLOCK, rmc.INV_TYPEOK)),
    ("MCraftBoundedSym", (3, 2, 2, 1, 2, 1, rmc.FLAG_CHECK_DEADLOCK | rmc.FLAG_SYMMETRY,
                          rmc.INV_TYPEOK)),
    ("MCraftTiny2", (2, 1, 2, 1, 2, 1, rmc.FLAG_CHECK_DEADLOCK, rmc.INV_TYPEOK)),
    ("MCraft5", (5, 2, 2, 1, 2, 1, rmc.FLAG_CHECK_DEADLOCK, rmc.INV_TYPEOK)),
    ("MCraftBug", (3, 2, 3, 1, 3, 1, rmc.FLAG_CHECK_DEADLOCK | rmc.FLAG_BUG_QUORUM,
                   rmc.INV_ONE_LEADER | rmc.INV_LOG_MATCHING)),
    ("MCraftMessages", (3, 2, 2, 1, 1, 1, rmc.FLAG_CHECK_DEADLOCK, rmc.INV_TYPEOK | rmc.INV_MESSAGES)),
    ("MCraftElections", (3, 2, 2, 1, 1, 1, rmc.FLAG_CHECK_DEADLOCK,
                         rmc.INV_TYPEOK | rmc.INV_LEADER_VOTES | rmc.INV_CAND_TERM)),
])
def test_front_end_reads_tlc_models(name, expect):
    c = rmc.config_from_files(os.path.join(SPECS, name + ".cfg"))
    got = (c.n_servers, c.n_values, c.max_term, c.max_log_len, c.max_msgs, c.max_dup, c.flags,
           c.invariants)
    assert got == expect


def test_front_end_rejects_unbounded_and_unknown(tmp_path):
    for f in os.listdir(SPECS):
        if f.endswith(".tla"):
            (tmp_path / f).write_text(open(os.path.join(SPECS, f)).read())
    base = open(os.path.join(SPECS, "MCraftBounded.cfg")).read()
    # no CONSTRAINT: MCraft.cfg as shipped is infinite
    (tmp_path / "MCraftBounded.cfg").write_text(base.replace("CONSTRAINT StateConstraint", ""))
    with pytest.raises(rmc.RmcError, match="infinite"):
        rmc.config_from_files(str(tmp_path / "MCraftBounded.cfg"))
    (tmp_path / "MCraftBounded.cfg").write_text(base.replace("INVARIANT TypeOK",
                                                             "INVARIANT LeaderCompleteness"))
    with pytest.raises(rmc.RmcError, match="LeaderCompleteness"):
        rmc.config_from_files(str(tmp_path / "MCraftBounded.cfg"))
    (tmp_path / "MCraftBounded.cfg").write_text(base + "\nPROPERTY Liveness\n")
    with pytest.raises(rmc.RmcError, match="liveness"):
        rmc.config_from_files(str(tmp_path / "MCraftBounded.cfg"))


MODELS = os.path.join(os.path.dirname(__file__), "golden", "models")


def test_front_end_reads_toolbox_layout():
    """Toolbox-generated model modules close each definition with a separator
    line (the layout of the reference's MCraft.tla)."""
    c = rmc.config_from_files(os.path.join(MODELS, "MCtoolbox.cfg"))
    assert (c.n_servers, c.n_values, c.max_term, c.max_log_len, c.max_msgs, c.max_dup) == (3, 2, 2, 1, 2, 1)
    assert c.invariants == rmc.INV_TYPEOK and c.flags == rmc.FLAG_CHECK_DEADLOCK


def test_front_end_reads_simulation_models():
    """Init <- SmokeInit (Smokeraft.cfg:43-48): BFS refuses it, simulation
    takes k, SmokeNat, CHECK_DEADLOCK FALSE and the packed capacity bounds."""
    path = os.path.join(MODELS, "SmokeFixture.cfg")
    with pytest.raises(rmc.RmcError, match="simulation"):
        rmc.config_from_files(path)
    c, sc = rmc.sim_config_from_files(path)
    assert (c.n_servers, c.n_values) == (3, 2)
    assert c.flags == 0 and c.invariants == rmc.INV_TYPEOK
    assert (sc.smoke_k, sc.smoke_nat, sc.depth, sc.behaviours) == (3, 3, 100, 1 << 20)
    # an Init-based model simulates from Init
    c2, sc2 = rmc.sim_config_from_files(os.path.join(MODELS, "MCtoolbox.cfg"))
    assert sc2.smoke_k == 0 and c2.max_term == 2


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference checkout absent")
def test_front_end_reads_the_reference_models():
    """The reference's own model files, read in place (CPU only; the GPU box
    has no /root/reference): MCraft.cfg as shipped is infinite, Smokeraft.cfg
    is a simulation model with k = 2 (Smokeraft.tla:17-19)."""
    with pytest.raises(rmc.RmcError, match="infinite"):
        rmc.config_from_files("/root/reference/MCraft.cfg")
    c, sc = rmc.sim_config_from_files("/root/reference/Smokeraft.cfg")
    assert (c.n_servers, c.n_values, sc.smoke_k, sc.smoke_nat) == (3, 2, 2, 2)
    assert c.flags == 0 and c.invariants == rmc.INV_TYPEOK


def test_create_validates_config():
    lib = rmc.native()
    ctx = C.c_void_p()
    bad = rmc.make_config(max_log_len=4)
    assert lib.rmc_create(C.byref(bad), C.byref(ctx)) == -22
    bad = rmc.make_config(n_servers=5, symmetry=True)
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
    r = subprocess.run([exe, "-config", os.path.join(SPECS, "MCraftBug.cfg"),
                        os.path.join(SPECS, "MCraftBug.tla")], capture_output=True, text=True)
    assert "quorum guard weakened" in r.stdout
    try:
        import torch
        gpu = torch.cuda.is_available()
    except ImportError:
        gpu = False
    if not gpu:
        assert r.returncode != 0
