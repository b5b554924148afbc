"""ctypes binding of the C oracle (oracle/rmc_oracle.c) — test infrastructure."""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


class OrcResult(C.Structure):
    _fields_ = [("generated", C.c_uint64), ("distinct", C.c_uint64), ("left_on_queue", C.c_uint64),
                ("depth", C.c_int32), ("violated_inv", C.c_int32), ("violation_depth", C.c_int32),
                ("overflow", C.c_int32), ("violation_index", C.c_uint64), ("seconds", C.c_double)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           capture_output=True)
        lib = C.CDLL(LIB)
        lib.orc_bfs.argtypes = [C.c_int] * 11 + [C.c_uint64, C.POINTER(OrcResult),
                                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                                 C.c_int]
        lib.orc_bfs.restype = C.c_int
        _lib = lib
    return _lib


def bfs(S, V, max_term, max_log, max_msgs, max_dup, bug=0, inv=1, sym=0, threads=8,
        max_levels=0, capacity=1 << 24):
    """Run the C oracle; returns (OrcResult, level_new list, level_gen list)."""
    lib = load()
    r = OrcResult()
    ln = (C.c_uint64 * 512)()
    lg = (C.c_uint64 * 512)()
    rc = lib.orc_bfs(S, V, max_term, max_log, max_msgs, max_dup, bug, inv, sym, threads,
                     max_levels, capacity, C.byref(r), ln, lg, 512)
    assert rc == 0, rc
    assert not r.overflow, "oracle capacity overflow"
    return r, [ln[d] for d in range(r.depth)], [lg[d] for d in range(r.depth + 1)]
