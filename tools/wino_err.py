#!/usr/bin/env python3
"""fp32 error of the Winograd conv kernels vs fp64 on ReLU-like (non-negative, DC-heavy) operands:
F(2x2,3x3) (pmu_conv3x3_fwd_wino_raw) and F(4x4,3x3) (pmu_conv3x3_fwd_wino4)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))
import torch  # noqa: E402
import torch.nn.functional as TF  # noqa: E402
from pmu_hip import _lib as L  # noqa: E402
from pmu_hip.engine import pack_weights_wino, pack_weights_wino4  # noqa: E402

dev = torch.device("cuda")
for (N, H, Cin, Cout, dc) in [(2, 64, 64, 64, 0.0), (2, 64, 64, 64, 1.0), (2, 32, 512, 512, 1.0), (2, 64, 256, 256, 3.0)]:
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(N, H, H, Cin, generator=g) + dc).clamp_min(0).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (9 * Cin)) ** 0.5).to(dev)
    b = torch.zeros(Cout, device=dev)
    ref = TF.conv2d(x.permute(0, 3, 1, 2).double().cpu(), w.double().cpu(), None, padding=1).permute(0, 2, 3, 1)
    out = {}
    for name, fn, pk, tiles in [("F2", "pmu_conv3x3_fwd_wino_raw", pack_weights_wino, "pmu_conv3x3_tiles_wino"),
                                ("F4", "pmu_conv3x3_fwd_wino4", pack_weights_wino4, "pmu_conv3x3_tiles_wino4")]:
        z = torch.empty(N, H, H, Cout, device=dev)
        part = torch.empty(getattr(L.lib(), tiles)(N, H, H), 2 * Cout, device=dev)
        wp = pk(w, False)
        L.call(fn, x.data_ptr(), Cin, N, H, H, wp.data_ptr(), b.data_ptr(), Cout, z.data_ptr(), part.data_ptr(), L.stream())
        torch.cuda.synchronize()
        d = (z.double().cpu() - ref)
        out[name] = (float(d.abs().max() / ref.abs().max()), float(d.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()))
    # direct fp32 (torch CPU) for scale
    r32 = TF.conv2d(x.permute(0, 3, 1, 2).cpu(), w.cpu(), None, padding=1).permute(0, 2, 3, 1).double()
    d = r32 - ref
    print(f"N={N} H={H} Cin={Cin} Cout={Cout} dc={dc}: direct32 max {float(d.abs().max()/ref.abs().max()):.2e} "
          f"rms {float(d.pow(2).mean().sqrt()/ref.pow(2).mean().sqrt()):.2e} | " +
          " | ".join(f"{k} max {v[0]:.2e} rms {v[1]:.2e}" for k, v in out.items()), flush=True)
