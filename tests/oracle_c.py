"""ctypes binding of the C oracle (oracle/rmc_oracle.c) — test infrastructure."""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
LIB_WIDE = os.path.join(ROOT, "oracle", "_build", "liboracle_wide.so")  # logs of 8, 12 messages


class OrcResult(C.Structure):
    _fields_ = [("generated", C.c_uint64), ("distinct", C.c_uint64), ("left_on_queue", C.c_uint64),
                ("depth", C.c_int32), ("violated_inv", C.c_int32), ("violation_depth", C.c_int32),
                ("overflow", C.c_int32), ("violation_index", C.c_uint64), ("seconds", C.c_double)]


_libs = {}


def load(wide=False):
    path = LIB_WIDE if wide else LIB
    if path not in _libs:
        if not os.path.exists(path):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           capture_output=True)
        lib = C.CDLL(path)
        lib.orc_bfs.argtypes = [C.c_int] * 11 + [C.c_uint64, C.POINTER(OrcResult),
                                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                                 C.c_int]
        lib.orc_bfs.restype = C.c_int
        _libs[path] = lib
    return _libs[path]


def bfs(S, V, max_term, max_log, max_msgs, max_dup, bug=0, inv=1, sym=0, threads=8,
        max_levels=0, capacity=1 << 24, wide=False):
    """Run the C oracle; returns (OrcResult, level_new list, level_gen list).
    wide: the build holding logs of 8 entries and 12 messages."""
    lib = load(wide)
    r = OrcResult()
    ln = (C.c_uint64 * 512)()
    lg = (C.c_uint64 * 512)()
    rc = lib.orc_bfs(S, V, max_term, max_log, max_msgs, max_dup, bug, inv, sym, threads,
                     max_levels, capacity, C.byref(r), ln, lg, 512)
    assert rc == 0, rc
    assert not r.overflow, "oracle capacity overflow"
    return r, [ln[d] for d in range(r.depth)], [lg[d] for d in range(r.depth + 1)]
