"""GPU parity of the fp32 Winograd F(2x2,3x3) kernels in 1024-thread workgroups (pmu_conv3x3_fwd_wino2h /
_dgrad_wino2h: four waves per SIMD, component-split waves), the forward of nn.Conv2d at
PMU/model/unet/unet_parts.py:15,18 and its input gradient.

Reference: the same materialised operand convolved in fp64 on the CPU; F(2x2)'s transforms have
coefficients 0, +-1, +-1/2, so the tolerance is the F(2x2) kernels' max|d| / max|ref| <= 2e-5.
"""
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu

TOL4 = 2e-5


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 32, 32, 64, 64), (1, 37, 45, 16, 40), (1, 70, 33, 48, 32),
                                            (2, 64, 64, 128, 96), (1, 33, 40, 8, 24), (1, 256, 64, 64, 64),
                                            (4, 100, 90, 64, 96)])  # last: more work items than workgroups
def test_conv3x3_fwd_wino2h(dev, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from pmu_hip.engine import pack_weights_wino2h
    g = torch.Generator().manual_seed(43 + H + Cin)
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    z = torch.full((N, H, W, Cout), float("nan"), device=dev)
    part = torch.full((L.lib().pmu_conv3x3_tiles_wino2h(N, H, W), 2 * Cout), float("nan"), device=dev)
    wp = pack_weights_wino2h(w, False)
    L.call("pmu_conv3x3_fwd_wino2h", x.data_ptr(), Cin, N, H, W, wp.data_ptr(), b.data_ptr(), Cout, z.data_ptr(),
           part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref = TF.conv2d(x.permute(0, 3, 1, 2).double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    err = _rel(z, ref)
    assert err <= TOL4, err
    tot = part.double().sum(0).cpu()
    assert float(((tot[:Cout] - ref.sum((0, 1, 2))).abs() / ref.abs().sum((0, 1, 2))).max()) <= 1e-5
    assert float(((tot[Cout:] - (ref * ref).sum((0, 1, 2))).abs() / (ref * ref).sum((0, 1, 2))).max()) <= 1e-5


@pytest.mark.parametrize("N,H,W,Cin,Cout,split", [(2, 40, 36, 64, 64, 64), (2, 33, 64, 128, 64, 64),
                                                  (1, 32, 48, 96, 128, 32), (1, 45, 37, 24, 16, 8),
                                                  (4, 100, 90, 96, 64, 64)])  # last: items > workgroups
def test_conv3x3_dgrad_wino2h(dev, N, H, W, Cin, Cout, split):
    from pmu_hip import _lib as L
    from pmu_hip.engine import pack_weights_wino2h
    g = torch.Generator().manual_seed(9 + H + Cout)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    wp = pack_weights_wino2h(w, True)
    dx0 = torch.full((N, H, W, split), float("nan"), device=dev)
    dx1 = torch.full((N, H, W, Cin - split), float("nan"), device=dev) if split < Cin else None
    L.call("pmu_conv3x3_dgrad_wino2h", dz.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, split, dx0.data_ptr(),
           L.ptr(dx1), L.stream())
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, W), w.double().cpu(), dz.permute(0, 3, 1, 2).double().cpu(),
                                     padding=1).permute(0, 2, 3, 1)
    got = dx0 if dx1 is None else torch.cat([dx0, dx1], dim=3)
    err = _rel(got, ref)
    assert err <= TOL4, err


def test_wino2h_rejects_bad_args(dev):
    from pmu_hip import _lib as L
    lb = L.lib()
    x = torch.zeros(1, 32, 32, 12, device=dev)
    # Cin % 8 != 0 is rejected on the host, before any launch
    assert lb.pmu_conv3x3_fwd_wino2h(x.data_ptr(), 12, 1, 32, 32, x.data_ptr(), None, 8, x.data_ptr(), None,
                                    None) == L.PMU_ERR_ARG


_MULTIPASS4 = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from pmu_hip import _lib as L
from pmu_hip.engine import pack_weights_wino2h
N, H, W, Cin, Cout, split = 2, 40, 36, 160, 64, 96
g = torch.Generator().manual_seed(19)
dz = torch.randn(N, H, W, Cout, generator=g).cuda()
w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).cuda()
wp = pack_weights_wino2h(w, True)
dx0 = torch.empty(N, H, W, split, device="cuda")
dx1 = torch.empty(N, H, W, Cin - split, device="cuda")
L.call("pmu_conv3x3_dgrad_wino2h", dz.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, split, dx0.data_ptr(),
       dx1.data_ptr(), L.stream())
torch.cuda.synchronize()
ref = torch.nn.grad.conv2d_input((N, Cin, H, W), w.double().cpu(), dz.permute(0, 3, 1, 2).double().cpu(),
                                 padding=1).permute(0, 2, 3, 1)
got = torch.cat([dx0, dx1], dim=3).double().cpu()
err = float((got - ref).abs().max() / ref.abs().max())
Cin, Cout = 64, 160
x = torch.randn(N, H, W, Cin, generator=g).cuda()
w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).cuda()
b = torch.randn(Cout, generator=g).cuda()
z = torch.empty(N, H, W, Cout, device="cuda")
part = torch.empty(L.lib().pmu_conv3x3_tiles_wino2h(N, H, W), 2 * Cout, device="cuda")
wp = pack_weights_wino2h(w, False)
L.call("pmu_conv3x3_fwd_wino2h", x.data_ptr(), Cin, N, H, W, wp.data_ptr(), b.data_ptr(), Cout, z.data_ptr(),
       part.data_ptr(), L.stream())
torch.cuda.synchronize()
ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double().cpu(), w.double().cpu(), b.double().cpu(),
                                 padding=1).permute(0, 2, 3, 1)
err = max(err, float((z.double().cpu() - ref).abs().max() / ref.abs().max()))
tot = part.double().sum(0).cpu()
err = max(err, float(((tot[:Cout] - ref.sum((0, 1, 2))).abs() / ref.abs().sum((0, 1, 2))).max()))
print(err)
"""


@pytest.mark.parametrize("cpb", [2, 3, 5])
def test_wino2h_multipass(cpb):
    """Output-channel passes of the 1024-thread F(2x2) kernels (a workgroup walking cpb co-blocks of one spatial
    block, the next pass's first chunk fetched under this pass's MFMAs), forced through PMU_WINO2H_CPB:
    input gradient with Cin = 160 (5 co-blocks, concat split inside a pass) and forward with
    Cout = 160 (bias and BN partial sums per pass)."""
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "probabilistic-multiplanar-unet_amd")
    env = dict(os.environ, PMU_WINO2H_CPB=str(cpb))
    out = subprocess.run([sys.executable, "-c", _MULTIPASS4, pkg], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    assert float(out.stdout.strip().splitlines()[-1]) <= TOL4
