"""Weight gradient of the 3x3 convolution by Winograd F(4x4,3x3) (pmu_conv3x3_wgrad_wino4; the autograd
of nn.Conv2d w.r.t. its weight, PMU/model/unet/unet_parts.py:15,18) against the fp64 direct sum, and
against the F(2x2) kernel: fp32 rounding only (~1.3e-6 of rms |dw|, tools/wgrad_err.py), edge tiles,
odd map sizes and split-K over many K-tiles included."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 32, 32, 64, 32), (1, 37, 45, 64, 64), (2, 16, 16, 128, 64),
                                            (2, 64, 48, 64, 96), (3, 9, 13, 64, 32), (1, 8, 8, 256, 128)])
def test_wgrad_wino4_vs_fp64(dev, exp_lib, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(11 + H + Cin)
    x = torch.relu(torch.randn(N, H, W, Cin, generator=g))
    dz = torch.randn(N, H, W, Cout, generator=g) * 1e-2
    ref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (Cout, Cin, 3, 3),
                                      dz.double().permute(0, 3, 1, 2), padding=1)
    xd, dzd = x.to(dev), dz.to(dev)
    wsb = L.lib().pmu_conv3x3_wgrad_ws_wino4(N, H, W, Cin, Cout)
    assert wsb > 0
    ws = torch.full(((wsb + 3) // 4,), float("nan"), device=dev)
    dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=dev)
    L.call("pmu_conv3x3_wgrad_wino4", dzd.data_ptr(), xd.data_ptr(), N, H, W, Cout, Cin, dw.data_ptr(),
           ws.data_ptr(), wsb, L.stream())
    wsb2 = L.lib().pmu_conv3x3_wgrad_ws_wino(N, H, W, Cin, Cout)
    ws2 = torch.empty((wsb2 + 3) // 4, device=dev)
    dw2 = torch.empty_like(dw)
    L.call("pmu_conv3x3_wgrad_wino", dzd.data_ptr(), xd.data_ptr(), N, H, W, Cout, Cin, dw2.data_ptr(),
           ws2.data_ptr(), wsb2, L.stream())
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    err4 = float((dw.double().cpu() - ref).abs().max()) / scale
    err2 = float((dw2.double().cpu() - ref).abs().max()) / scale
    assert err4 <= 2e-5, (err4, err2)
    # rms error well inside the model-level 1e-3 gradient contract
    rms = float(((dw.double().cpu() - ref) ** 2).mean().sqrt() / (ref ** 2).mean().sqrt())
    assert rms <= 1e-5, rms


def test_wgrad_wino4_ws_size_rules(dev, exp_lib):
    from pmu_hip import _lib as L
    assert L.lib().pmu_conv3x3_wgrad_ws_wino4(2, 16, 16, 64, 48) == 0    # Cout % 32
    assert L.lib().pmu_conv3x3_wgrad_ws_wino4(2, 16, 16, 96, 32) == 0    # Cin % 64
    x = torch.zeros(1, device=dev)
    rc = L.lib().pmu_conv3x3_wgrad_wino4(x.data_ptr(), x.data_ptr(), 2, 16, 16, 32, 64, x.data_ptr(), x.data_ptr(), 4,
                                         L.stream())
    assert rc == L.PMU_ERR_ARG   # workspace too small: refused on the host, nothing launched
