import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as entry  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 device (run with -m gpu on the MI355X box)")


@pytest.fixture(scope="session")
def lcrc():
    """The product package (leveldb-rust_amd) with its native library built and loaded."""
    m = entry.load()
    if not os.path.exists(m.LIB_PATH):
        entry.build()
    m.lib()
    return m


@pytest.fixture(scope="session")
def orc():
    """The CPU oracle (test infrastructure only)."""
    return entry.load_oracle()


@pytest.fixture(scope="session")
def synth(lcrc):
    import importlib
    return importlib.import_module("leveldb_rust_amd.synth")


@pytest.fixture(scope="session")
def engines(lcrc):
    """One Engine per mode on device 0 (GPU tests only; fails loudly without a device)."""
    e = {lcrc.MODE_REF: lcrc.Engine(0, lcrc.MODE_REF), lcrc.MODE_C: lcrc.Engine(0, lcrc.MODE_C)}
    yield e
    for v in e.values():
        v.close()
