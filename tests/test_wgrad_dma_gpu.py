"""The bf16 weight gradient with both operands staged by LDS-DMA (pmu_conv3x3_wgrad_bf16_dma,
csrc/wgrad3x3_bf16_dma.hip): nn.Conv2d's weight gradient (PMU/model/unet/unet_parts.py:15,18
backward) under torch.autocast(bfloat16) — bf16 operands, fp32 sums — against the fp64 sum of the same
bf16 operands, and against the register-staged kernel it replaces.  Shapes cover every workgroup
layout (64/64: two strip lanes; 64 out / >64 in; >64 out), ragged channels (units past Cin / Cout and
the last 32-channel fragment masked), maps not a multiple of the 16-pixel strip, segments cut inside a
strip (few strips, many splits), segment tails past the image, and the c5 shapes at reduced batch."""
import pytest
import torch

from test_bf16_gpu import TOL, _bf16_values, _nchw, _rb, _rel, _to_bf16

pytestmark = pytest.mark.gpu


def _run(entry, ws_entry, dzt, xt, N, H, W, Cout, Cin, dev):
    from pmu_hip import _lib as L
    wsb = getattr(L.lib(), ws_entry)(N, H, W, Cin, Cout)
    ws = torch.full((wsb // 4 + 1,), float("nan"), device=dev)
    dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=dev)
    L.call(entry, dzt.data_ptr(), xt.data_ptr(), N, H, W, Cout, Cin, dw.data_ptr(), ws.data_ptr(), wsb, L.stream())
    torch.cuda.synchronize()
    return dw


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 32, 32, 64, 64), (2, 24, 40, 64, 128), (3, 19, 21, 32, 64),
                                            (2, 16, 16, 128, 192), (1, 11, 17, 12, 20), (4, 64, 48, 128, 64),
                                            (1, 70, 33, 256, 512), (2, 20, 36, 1024, 96), (1, 7, 16, 40, 1032),
                                            (16, 32, 32, 64, 64), (32, 16, 16, 64, 128)])
def test_wgrad_bf16_dma_vs_fp64(dev, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src
    assert L.lib().pmu_conv3x3_wgrad_dma_ok(N, H, W, Cin, Cout)
    g = torch.Generator().manual_seed(7 + H + W + Cout)
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    xt = _to_bf16([Src(x)], N, H, W, Cin)
    dzt = _to_bf16([Src(dz)], N, H, W, Cout)
    dw = _run("pmu_conv3x3_wgrad_bf16_dma", "pmu_conv3x3_wgrad_ws_bf16_dma", dzt, xt, N, H, W, Cout, Cin, dev)
    ref = torch.nn.grad.conv2d_weight(_nchw(_rb(x)).double().cpu(), (Cout, Cin, 3, 3),
                                      _nchw(_rb(dz)).double().cpu(), padding=1)
    assert not torch.isnan(dw).any()
    assert _rel(dw, ref) <= TOL, _rel(dw, ref)
    old = _run("pmu_conv3x3_wgrad_bf16", "pmu_conv3x3_wgrad_ws_bf16", dzt, xt, N, H, W, Cout, Cin, dev)
    assert _rel(dw, old.double().cpu()) <= TOL


@pytest.mark.parametrize("H,Cin,Cout", [(512, 64, 64), (256, 128, 128), (128, 256, 256), (64, 512, 512),
                                        (32, 1024, 1024), (64, 1024, 512), (512, 128, 64)])
def test_wgrad_bf16_dma_c5_shapes(dev, H, Cin, Cout):
    """c5's layer shapes (512^2 input) at batch 2 vs the register-staged kernel (both fp32 sums of the
    same bf16 products; relative difference within the fp32 summation-order noise)."""
    from pmu_hip.engine import Src
    N = 2
    g = torch.Generator().manual_seed(H + Cin)
    x = torch.randn(N, H, H, Cin, generator=g).to(dev)
    dz = torch.randn(N, H, H, Cout, generator=g).to(dev)
    xt = _to_bf16([Src(x)], N, H, H, Cin)
    dzt = _to_bf16([Src(dz)], N, H, H, Cout)
    dw = _run("pmu_conv3x3_wgrad_bf16_dma", "pmu_conv3x3_wgrad_ws_bf16_dma", dzt, xt, N, H, H, Cout, Cin, dev)
    old = _run("pmu_conv3x3_wgrad_bf16", "pmu_conv3x3_wgrad_ws_bf16", dzt, xt, N, H, H, Cout, Cin, dev)
    assert float((dw - old).abs().max()) <= 1e-4 * float(old.abs().max())


def test_wgrad_dma_refuses_narrow_maps(dev):
    from pmu_hip import _lib as L
    assert not L.lib().pmu_conv3x3_wgrad_dma_ok(2, 16, 15, 64, 64)
    assert L.lib().pmu_conv3x3_wgrad_dma_ok(2, 1, 16, 64, 64)
