import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libedet.so on cuda:0)")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(params=["partials", "atomics"])
def workspace_mode(request):
    """Weight-gradient kernels with the registered split-reduction workspace (fixed-order
    partial sums) and without it (atomics fallback)."""
    from tf2mv_amd import _lib as L
    from tf2mv_amd.runtime import ensure_workspace
    if request.param == "atomics":
        L.call("edet_set_workspace", None, 0)
    else:
        ensure_workspace("cuda")
    yield request.param
    ensure_workspace("cuda")
