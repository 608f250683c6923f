import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "quantumoptimalcontrol.jl_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libqoc_mi355x.so)")


@pytest.fixture(scope="session")
def built_lib():
    import __graft_entry__ as g
    g.build_lib()
    from qoc_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def golden_dir():
    import pathlib
    return pathlib.Path(ROOT) / "tests" / "golden"
