"""Python binding of librmc.so (include/rmc.h) — used by tests and bench.py.

The product is the HIP library; this module is a thin ctypes layer with the
same names and meanings as the C ABI.  It never falls back to a CPU path:
if `lib/librmc.so` is missing, importing `rmc.native()` raises.

TLC correspondence: `Config` = the .cfg bounds,
`Checker.run()` = `tlc2.TLC` BFS to fixpoint, `Result` = TLC's summary
("N states generated, M distinct states found, Q left on queue", depth).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "librmc.so")
if os.environ.get("RMC_LIB"):  # another in-tree build of librmc (same-box A/B of two builds)
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", os.environ["RMC_LIB"])

MAX_SERVERS, MAX_LOG, MAX_MSGS = 5, 3, 8  # the packed layout's capacity
WIDE_MAX_TERM, WIDE_MAX_LOG, WIDE_MAX_MSGS, WIDE_MAX_DUP = 255, 32, 64, 255  # the wide layout's
VIEW_LOG, VIEW_MSGS = 32, 64  # rmc_state_view sizes (RMC_VIEW_LOG, RMC_VIEW_MSGS)
SIM_WITHIN_CAPACITY, SIM_TRUNCATE, SIM_TLC = 0, 1, 2
FLAG_SYMMETRY, FLAG_CHECK_DEADLOCK, FLAG_BUG_QUORUM, FLAG_VERIFY_STATES, FLAG_SPILL = 1, 2, 4, 8, 16
INV_TYPEOK, INV_ONE_LEADER, INV_LOG_MATCHING, INV_MESSAGES = 1, 2, 4, 8
INV_LEADER_VOTES, INV_CAND_TERM = 16, 32
INV_VOTES_GRANTED, INV_QUORUM_LOG, INV_MORE_UP_TO_DATE, INV_LEADER_COMPLETE = 64, 128, 256, 512
INV_NAMES = {INV_TYPEOK: "TypeOK", INV_ONE_LEADER: "OneLeaderPerTerm",
             INV_LOG_MATCHING: "LogMatching", INV_MESSAGES: "MessagesInv",
             INV_LEADER_VOTES: "LeaderVotesQuorum", INV_CAND_TERM: "CandidateTermNotInLog",
             INV_VOTES_GRANTED: "VotesGrantedInv", INV_QUORUM_LOG: "QuorumLogInv",
             INV_MORE_UP_TO_DATE: "MoreUpToDateCorrect", INV_LEADER_COMPLETE: "LeaderCompleteness"}
FRONT_BUILTIN_RAFT, FRONT_SIMULATE, FRONT_DEPTH_BOUNDED = 1, 2, 4
FLAG_UNBOUNDED_TERM, FLAG_UNBOUNDED_LOG, FLAG_UNBOUNDED_MSGS, FLAG_UNBOUNDED_DUP = 32, 64, 128, 256
FAMILIES = ("Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
            "AdvanceCommitIndex", "AppendEntries", "Receive", "DuplicateMessage",
            "DropMessage")
ERRORS = {-22: "EINVAL", -12: "ENOMEM", -5: "HIP", -28: "CAPACITY", -19: "NOGPU",
          -74: "PARSE", -71: "STATE", -61: "IO"}


class Config(C.Structure):
    _fields_ = [("n_servers", C.c_int32), ("n_values", C.c_int32), ("max_term", C.c_int32),
                ("max_log_len", C.c_int32), ("max_msgs", C.c_int32), ("max_dup", C.c_int32),
                ("flags", C.c_uint32), ("invariants", C.c_uint32), ("device", C.c_int32),
                ("max_depth", C.c_int32), ("state_capacity", C.c_uint64), ("seed", C.c_uint64),
                ("device_window", C.c_uint64), ("set_bytes", C.c_uint64)]


class Result(C.Structure):
    _fields_ = [("generated", C.c_uint64), ("distinct", C.c_uint64), ("left_on_queue", C.c_uint64),
                ("depth", C.c_int32), ("violated_inv", C.c_int32), ("violation_depth", C.c_int32),
                ("deadlock", C.c_int32), ("collision_probability", C.c_double),
                ("seconds", C.c_double), ("expand_kernel_seconds", C.c_double),
                ("expand_launches", C.c_uint64), ("probes", C.c_uint64),
                ("collisions", C.c_uint64), ("verified", C.c_uint64),
                ("keys_sent", C.c_uint64), ("states_sent", C.c_uint64), ("chunks", C.c_uint64),
                ("exchange_seconds", C.c_double), ("stored_here", C.c_uint64),
                ("spilled", C.c_uint64), ("spills", C.c_uint64), ("spill_seconds", C.c_double),
                ("parked", C.c_uint64), ("exchange_wait_seconds", C.c_double),
                ("spill_links_on_device", C.c_int32), ("pad2", C.c_int32),
                ("verified_spilled", C.c_uint64), ("set_slots", C.c_uint64)]


class LevelStats(C.Structure):
    _fields_ = [("level", C.c_int32), ("pad", C.c_int32), ("generated", C.c_uint64),
                ("distinct", C.c_uint64), ("new_states", C.c_uint64), ("seconds", C.c_double)]


class Entry(C.Structure):
    _fields_ = [("term", C.c_int32), ("value", C.c_int32)]


class MsgView(C.Structure):
    _fields_ = [("mtype", C.c_int32), ("mterm", C.c_int32), ("msource", C.c_int32),
                ("mdest", C.c_int32), ("mlastLogTerm", C.c_int32), ("mlastLogIndex", C.c_int32),
                ("mvoteGranted", C.c_int32), ("mlog_len", C.c_int32), ("mlog", Entry * VIEW_LOG),
                ("mprevLogIndex", C.c_int32), ("mprevLogTerm", C.c_int32),
                ("mentries_len", C.c_int32), ("mentries", Entry * 1), ("mcommitIndex", C.c_int32),
                ("msuccess", C.c_int32), ("mmatchIndex", C.c_int32), ("count", C.c_int32)]


class StateView(C.Structure):
    _fields_ = [("n_servers", C.c_int32), ("n_msgs", C.c_int32),
                ("currentTerm", C.c_int32 * MAX_SERVERS), ("state", C.c_int32 * MAX_SERVERS),
                ("votedFor", C.c_int32 * MAX_SERVERS), ("commitIndex", C.c_int32 * MAX_SERVERS),
                ("log_len", C.c_int32 * MAX_SERVERS),
                ("log", (Entry * VIEW_LOG) * MAX_SERVERS),
                ("votesResponded", C.c_uint32 * MAX_SERVERS),
                ("votesGranted", C.c_uint32 * MAX_SERVERS),
                ("nextIndex", (C.c_int32 * MAX_SERVERS) * MAX_SERVERS),
                ("matchIndex", (C.c_int32 * MAX_SERVERS) * MAX_SERVERS),
                ("msgs", MsgView * VIEW_MSGS)]


class SuccView(C.Structure):
    _fields_ = [("parent", C.c_uint64), ("family", C.c_int32), ("instance", C.c_int32),
                ("in_constraint", C.c_int32), ("pad", C.c_int32), ("fingerprint", C.c_uint64),
                ("state", StateView)]


class SimConfig(C.Structure):
    _fields_ = [("behaviours", C.c_uint64), ("depth", C.c_int32), ("smoke_k", C.c_int32),
                ("smoke_nat", C.c_int32), ("mode", C.c_int32), ("seed", C.c_uint64)]


class SimResult(C.Structure):
    _fields_ = [("behaviours", C.c_uint64), ("steps", C.c_uint64), ("init_states", C.c_uint64),
                ("truncated", C.c_uint64), ("deadlocked", C.c_uint64), ("violated_inv", C.c_int32),
                ("violation_depth", C.c_int32), ("violation_behaviour", C.c_uint64),
                ("seconds", C.c_double), ("kernel_seconds", C.c_double)]


PROGRESS_FN = C.CFUNCTYPE(C.c_int, C.POINTER(LevelStats), C.c_void_p)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p,
                           C.POINTER(C.c_uint64))
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)


class Transport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("alltoallv", ALLTOALLV_FN), ("allgather", ALLGATHER_FN)]

# Every symbol include/rmc.h declares (checked by tests/test_abi.py).
EXPORTS = ("rmc_create", "rmc_destroy", "rmc_last_error", "rmc_version", "rmc_run_bfs",
           "rmc_get_result", "rmc_trace", "rmc_state_bytes", "rmc_expand",
           "rmc_config_from_files", "rmc_probe_bench", "rmc_rccl_unique_id", "rmc_shard",
           "rmc_set_seed", "rmc_simulate", "rmc_sim_replay", "rmc_set_fp_bits",
           "rmc_sim_config_from_files", "rmc_checkpoint", "rmc_recover", "rmc_model_from_files",
           "rmc_action_location", "rmc_smoke_init")

_lib = None


def native():
    """Load lib/librmc.so (built by `make -C raft.tla_amd`); raise if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"librmc.so not built: {LIB_PATH} (run __graft_entry__.build())")
        lib = C.CDLL(LIB_PATH)
        lib.rmc_create.argtypes = [C.POINTER(Config), C.POINTER(C.c_void_p)]
        lib.rmc_create.restype = C.c_int
        lib.rmc_destroy.argtypes = [C.c_void_p]
        lib.rmc_destroy.restype = None
        lib.rmc_last_error.argtypes = [C.c_void_p]
        lib.rmc_last_error.restype = C.c_char_p
        lib.rmc_version.argtypes = []
        lib.rmc_version.restype = C.c_char_p
        lib.rmc_run_bfs.argtypes = [C.c_void_p, PROGRESS_FN, C.c_void_p]
        lib.rmc_run_bfs.restype = C.c_int
        lib.rmc_get_result.argtypes = [C.c_void_p, C.POINTER(Result)]
        lib.rmc_get_result.restype = C.c_int
        lib.rmc_trace.argtypes = [C.c_void_p, C.POINTER(StateView), C.POINTER(C.c_int32),
                                  C.POINTER(C.c_int32), C.c_size_t, C.POINTER(C.c_size_t)]
        lib.rmc_trace.restype = C.c_int
        lib.rmc_state_bytes.argtypes = [C.POINTER(Config)]
        lib.rmc_state_bytes.restype = C.c_size_t
        lib.rmc_expand.argtypes = [C.c_void_p, C.POINTER(StateView), C.c_size_t,
                                   C.POINTER(SuccView), C.c_size_t, C.POINTER(C.c_size_t)]
        lib.rmc_expand.restype = C.c_int
        lib.rmc_config_from_files.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(Config),
                                              C.c_char_p, C.c_size_t]
        lib.rmc_config_from_files.restype = C.c_int
        lib.rmc_sim_config_from_files.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(Config),
                                                  C.POINTER(SimConfig), C.c_char_p, C.c_size_t]
        lib.rmc_sim_config_from_files.restype = C.c_int
        lib.rmc_model_from_files.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_uint32,
                                             C.POINTER(Config), C.POINTER(SimConfig), C.c_char_p,
                                             C.c_size_t]
        lib.rmc_model_from_files.restype = C.c_int
        lib.rmc_action_location.argtypes = [C.c_char_p, C.POINTER(C.c_int32)]
        lib.rmc_action_location.restype = C.c_int
        lib.rmc_smoke_init.argtypes = [C.POINTER(Config), C.POINTER(SimConfig), C.POINTER(StateView),
                                       C.c_size_t, C.POINTER(C.c_size_t)]
        lib.rmc_smoke_init.restype = C.c_int
        lib.rmc_checkpoint.argtypes = [C.c_void_p, C.c_char_p]
        lib.rmc_checkpoint.restype = C.c_int
        lib.rmc_recover.argtypes = [C.c_void_p, C.c_char_p]
        lib.rmc_recover.restype = C.c_int
        lib.rmc_probe_bench.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int,
                                        C.POINTER(C.c_double)]
        lib.rmc_probe_bench.restype = C.c_int
        lib.rmc_rccl_unique_id.argtypes = [C.c_char_p]
        lib.rmc_rccl_unique_id.restype = C.c_int
        lib.rmc_shard.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p, C.POINTER(Transport),
                                  C.c_uint64, C.c_uint64]
        lib.rmc_shard.restype = C.c_int
        lib.rmc_set_seed.argtypes = [C.c_void_p, C.c_uint64]
        lib.rmc_set_seed.restype = C.c_int
        lib.rmc_set_fp_bits.argtypes = [C.c_void_p, C.c_int32]
        lib.rmc_set_fp_bits.restype = C.c_int
        lib.rmc_simulate.argtypes = [C.c_void_p, C.POINTER(SimConfig), C.POINTER(SimResult)]
        lib.rmc_simulate.restype = C.c_int
        lib.rmc_sim_replay.argtypes = [C.c_void_p, C.POINTER(SimConfig), C.c_uint64,
                                       C.POINTER(StateView), C.c_size_t, C.POINTER(C.c_size_t)]
        lib.rmc_sim_replay.restype = C.c_int
        _lib = lib
    return _lib


class RmcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rmc error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


def make_config(n_servers=3, n_values=2, max_term=2, max_log_len=1, max_msgs=2, max_dup=1,
                symmetry=False, bug_quorum=False, invariants=INV_TYPEOK, check_deadlock=True,
                device=0, max_depth=0, state_capacity=0, verify_states=False, spill=False, device_window=0,
                set_bytes=0):
    flags = (FLAG_SYMMETRY if symmetry else 0) | (FLAG_BUG_QUORUM if bug_quorum else 0) | \
        (FLAG_CHECK_DEADLOCK if check_deadlock else 0) | (FLAG_VERIFY_STATES if verify_states else 0) | \
        (FLAG_SPILL if spill else 0)
    return Config(n_servers, n_values, max_term, max_log_len, max_msgs, max_dup, flags,
                  invariants, device, max_depth, state_capacity, 0, device_window, set_bytes)


def model_from_files(cfg_path, tla_path=None, raft_path=None, builtin_raft=False, simulate=False,
                     depth_bounded=False):
    """rmc_model_from_files: (Config, SimConfig or None, provenance notes).
    Raises RmcError naming the construct when the model is not the compiled-in
    raft.tla (with its recognised bug variant, bounds and invariants).
    depth_bounded: the caller sets max_depth (TLC -depth), so fields without a
    CONSTRAINT are accepted at the packed capacity (RMC_FLAG_UNBOUNDED_*)."""
    lib = native()
    cfg, sc = Config(), SimConfig()
    info = C.create_string_buffer(4096)
    opts = (FRONT_BUILTIN_RAFT if builtin_raft else 0) | (FRONT_SIMULATE if simulate else 0) | \
        (FRONT_DEPTH_BOUNDED if depth_bounded else 0)
    rc = lib.rmc_model_from_files(cfg_path.encode(), tla_path.encode() if tla_path else None,
                                  raft_path.encode() if raft_path else None, opts, C.byref(cfg),
                                  C.byref(sc) if simulate else None, info, 4096)
    if rc:
        raise RmcError(rc, info.value.decode())
    return cfg, (sc if simulate else None), info.value.decode()


def config_from_files(cfg_path, tla_path=None, raft_path=None, builtin_raft=False):
    return model_from_files(cfg_path, tla_path, raft_path, builtin_raft)[0]


def sim_config_from_files(cfg_path, tla_path=None, raft_path=None, builtin_raft=False):
    """(Config, SimConfig) of a simulation model (Smokeraft.cfg: Init <- SmokeInit)."""
    cfg, sc, _ = model_from_files(cfg_path, tla_path, raft_path, builtin_raft, simulate=True)
    return cfg, sc


def smoke_init(cfg, smoke_k, smoke_nat=2, seed=0):
    """The SmokeInit initial states rmc_simulate would draw (host only)."""
    sc = SimConfig(1, 100, smoke_k, smoke_nat, 0, seed)
    n = C.c_size_t()
    rc = native().rmc_smoke_init(C.byref(cfg), C.byref(sc), None, 0, C.byref(n))
    if rc:
        raise RmcError(rc, "rmc_smoke_init failed")
    st = (StateView * n.value)()
    rc = native().rmc_smoke_init(C.byref(cfg), C.byref(sc), st, n.value, C.byref(n))
    if rc:
        raise RmcError(rc, "rmc_smoke_init failed")
    return list(st)


def rccl_unique_id() -> bytes:
    """rmc_rccl_unique_id: the 128-byte id rank 0 hands to every rank's rmc_shard."""
    buf = C.create_string_buffer(128)
    rc = native().rmc_rccl_unique_id(buf)
    if rc:
        raise RmcError(rc, "rmc_rccl_unique_id failed")
    return buf.raw


def action_location(action):
    """(line, col, line, col) of an action of Next in raft.tla (TLC's trace headers)."""
    out = (C.c_int32 * 4)()
    rc = native().rmc_action_location(action.encode(), out)
    if rc:
        raise RmcError(rc, f"no action {action!r}")
    return tuple(out)


def probe_bench(device=0, table_bytes=64 << 30, accesses=1 << 31, mode=0):
    """Random 8-byte probe (mode 0) / CAS (mode 1) rate over a table of
    table_bytes: the roofline ceiling R_max of the fingerprint set."""
    rate = C.c_double()
    rc = native().rmc_probe_bench(device, table_bytes, accesses, mode, C.byref(rate))
    if rc:
        raise RmcError(rc, "rmc_probe_bench failed")
    return rate.value


class Checker:
    """One model-checking context on one GPU (rmc_ctx)."""

    def __init__(self, cfg: Config):
        self.lib = native()
        self.cfg = cfg
        self.ctx = C.c_void_p()
        rc = self.lib.rmc_create(C.byref(cfg), C.byref(self.ctx))
        if rc:
            raise RmcError(rc, "rmc_create failed (see stderr)")

    def close(self):
        if self.ctx:
            self.lib.rmc_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        if rc:
            raise RmcError(rc, self.lib.rmc_last_error(self.ctx).decode())

    def run(self, progress=None, record_levels=True) -> Result:
        """rmc_run_bfs.  record_levels=False (and no progress callback) passes
        no callback at all, as a Java caller without a progress listener
        would: a sharded search then skips the per-level stop vote."""
        levels = []

        def cb(p, _u):
            s = p.contents
            levels.append((s.level, s.generated, s.distinct, s.new_states, s.seconds))
            return int(bool(progress and progress(s)))

        fn = PROGRESS_FN(cb) if (record_levels or progress) else PROGRESS_FN()
        self._check(self.lib.rmc_run_bfs(self.ctx, fn, None))
        res = Result()
        self._check(self.lib.rmc_get_result(self.ctx, C.byref(res)))
        self.levels = levels
        return res

    def simulate(self, behaviours=1 << 20, depth=100, smoke_k=2, smoke_nat=2, seed=0, mode=0) -> SimResult:
        """TLC -simulate over Smokeraft-style initial states (rmc_simulate);
        mode 0 = RMC_SIM_WITHIN_CAPACITY, 1 = RMC_SIM_TRUNCATE, 2 = RMC_SIM_TLC (TLC's
        draw: an action, then a successor; the wide layout only)."""
        sc = SimConfig(behaviours, depth, smoke_k, smoke_nat, mode, seed)
        out = SimResult()
        self._check(self.lib.rmc_simulate(self.ctx, C.byref(sc), C.byref(out)))
        return out

    def sim_replay(self, behaviour, behaviours=1 << 20, depth=100, smoke_k=2, smoke_nat=2, seed=0, mode=0):
        """States of one behaviour of the same simulation (rmc_sim_replay)."""
        sc = SimConfig(behaviours, depth, smoke_k, smoke_nat, mode, seed)
        st = (StateView * depth)()
        n = C.c_size_t()
        self._check(self.lib.rmc_sim_replay(self.ctx, C.byref(sc), behaviour, st, depth, C.byref(n)))
        return [st[k] for k in range(min(n.value, depth))]

    def shard(self, rank: int, world: int, rccl_id: bytes | None = None, transport=None,
              keys_per_dest: int = 0, sent_cache_slots: int = 0):
        """rmc_shard: make this ctx rank `rank` of `world`.  RCCL when rccl_id
        (from rccl_unique_id() on rank 0) is given, else `transport` (a
        Transport, e.g. rmc.dist.GlooTransport().struct)."""
        self._shard_keep = transport  # the callbacks must outlive the ctx
        st = getattr(transport, "struct", transport)
        self._check(self.lib.rmc_shard(self.ctx, rank, world, rccl_id,
                                       C.byref(st) if st is not None else None,
                                       keys_per_dest, sent_cache_slots))

    def checkpoint(self, path: str):
        """Write the stopped search to `path` (rmc_checkpoint; TLC -checkpoint)."""
        self._check(self.lib.rmc_checkpoint(self.ctx, path.encode()))

    def recover(self, path: str):
        """Load a checkpoint; the next run() continues it (rmc_recover; TLC -recover)."""
        self._check(self.lib.rmc_recover(self.ctx, path.encode()))

    def set_fp_bits(self, bits: int):
        """Verification-mode test hook: keep only `bits` fingerprint bits (rmc_set_fp_bits)."""
        self._check(self.lib.rmc_set_fp_bits(self.ctx, bits))

    def set_seed(self, seed: int):
        """Fingerprint salt for the next run (rmc_set_seed)."""
        self._check(self.lib.rmc_set_seed(self.ctx, seed))

    def result(self) -> Result:
        res = Result()
        self._check(self.lib.rmc_get_result(self.ctx, C.byref(res)))
        return res

    def trace(self):
        n = C.c_size_t()
        self._check(self.lib.rmc_trace(self.ctx, None, None, None, 0, C.byref(n)))
        st = (StateView * n.value)()
        fam = (C.c_int32 * n.value)()
        inst = (C.c_int32 * n.value)()
        self._check(self.lib.rmc_trace(self.ctx, st, fam, inst, n.value, C.byref(n)))
        return [(fam[k], inst[k], st[k]) for k in range(n.value)]

    def expand(self, views):
        arr = (StateView * len(views))(*views)
        lanes_max = 5 + 5 + 25 + 5 + 10 + 5 + 25 + 3 * VIEW_MSGS
        cap = max(1, len(views) * lanes_max)
        out = (SuccView * cap)()
        n = C.c_size_t()
        self._check(self.lib.rmc_expand(self.ctx, arr, len(views), out, cap, C.byref(n)))
        return [out[k] for k in range(min(n.value, cap))]
