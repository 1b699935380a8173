import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "probabilistic-multiplanar-unet_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libpmunet_hip.so")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _debug_build_bounds_check(request):
    """PMU_LIB=debug (the bounds-checked debug library, csrc `make DEBUG=1`): after every GPU test,
    fail it if any kernel recorded an index-bound violation (pmu_debug_read)."""
    yield
    if os.environ.get("PMU_LIB") == "debug" and request.node.get_closest_marker("gpu") is not None:
        from pmu_hip import _lib as L
        if L._LIB is not None:
            L.debug_check()
