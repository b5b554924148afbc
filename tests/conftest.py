import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "raft.tla_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle_lib():
    """The C oracle (test infrastructure), built by __graft_entry__.build()."""
    from tests.oracle_c import load
    return load()
