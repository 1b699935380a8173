"""pmu_hip — MI355X (gfx950) HIP hot path of the Probabilistic Multi-Planar U-Net.

``libpmunet_hip.so`` (built from ../csrc) exposes the C ABI of include/pmunet_hip.h;
``_lib`` binds it with ctypes, ``engine`` sequences the kernels, ``functions`` wraps them as
autograd Functions used by the drop-in ``model`` package.
"""
from ._lib import LIB_PATH, load_library, lib  # noqa: F401
