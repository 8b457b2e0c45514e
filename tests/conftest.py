import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP kernel library")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_ok():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_ok():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    """The native kernel module; builds the library first if needed (GPU tests only)."""
    from rag_llm_k8s_amd import _build

    _build.build_hip()
    from rag_llm_k8s_amd.ops import native as n

    n._lib.lib()
    return n
