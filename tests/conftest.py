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
def built_lib(request):
    import __graft_entry__ as g
    g.build_lib()
    # GPU sessions: let torch bring up its HIP runtime before libqoc_mi355x.so touches the device, so
    # that the device-pointer tests (torch tensors handed to the C ABI) work in any test order.
    if request.node.get_closest_marker("gpu") is not None or any(
            it.get_closest_marker("gpu") for it in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
                torch.empty(1, device="cuda")
        except Exception:
            pass
    from qoc_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def golden_dir():
    import pathlib
    return pathlib.Path(ROOT) / "tests" / "golden"
