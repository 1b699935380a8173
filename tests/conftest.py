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


_EXP = {}


@pytest.fixture
def exp_lib(dev):
    """The experiments library (csrc `make EXPERIMENTS=1`, include/pmunet_hip_experiments.h) in place of
    the shipped one for this test: the kernels the default dispatch does not reach are tested against
    it (the shipped library does not export them).  Skips when it is not built."""
    from pmu_hip import _lib as L
    if not os.path.exists(L.EXP_LIB_PATH):
        pytest.skip("experiments library not built (make -C csrc EXPERIMENTS=1)")
    prev = L.lib()
    if "lib" not in _EXP:
        _EXP["lib"] = L.load_library(L.EXP_LIB_PATH)
    L._LIB = _EXP["lib"]
    try:
        yield _EXP["lib"]
    finally:
        L._LIB = prev
