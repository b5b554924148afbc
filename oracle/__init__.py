"""Test-infrastructure oracle for the raft.tla BFS hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this package.  The product (`raft.tla_amd/`) never does.
"""
