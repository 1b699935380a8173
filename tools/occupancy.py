import ctypes, sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "probabilistic-multiplanar-unet_amd"))
import torch
from pmu_hip import _lib as L
torch.zeros(1, device="cuda")
for n in ("pmu_occupancy_conv3x3_raw", "pmu_occupancy_wgrad3x3_bf16", "pmu_occupancy_conv3x3_pipe"):
    v = ctypes.c_int(0)
    rc = getattr(L.lib(), n)(ctypes.byref(v))
    print(n, rc, v.value)
print(torch.cuda.get_device_properties(0))
