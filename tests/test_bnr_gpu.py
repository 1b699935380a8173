"""The input-gradient kernels fused with the BatchNorm+ReLU backward reduction of the producer layer
(pmu_conv3x3_dgrad_{wino4,wino2h,dma}_bnr): dx equals the plain input gradient bit for bit, and the
per-tile partial sums (sum g, sum g*xhat; g = dx * relu'(bn(z)), xhat = (z - mean) * invstd) add up to
what pmu_bn_bwd_reduce computes from (dx, z) — the reduction of PMU/model/unet/unet_parts.py:16-17's
BatchNorm2d + ReLU backward, formed in the epilogue instead of a second pass over dx and z."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bn_inputs(N, H, W, C, g, dev):
    z = torch.randn(N, H, W, C, generator=g).to(dev)
    coef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3]).to(dev)
    mean = (torch.randn(C, generator=g) * 0.2).to(dev)
    invstd = (torch.rand(C, generator=g) + 0.5).to(dev)
    return z, coef, mean, invstd


def _ref_sums(dx, z, coef, mean, invstd):
    """fp64 (sum g, sum g*xhat) per channel."""
    C = z.shape[3]
    d, zz = dx.double().cpu().reshape(-1, C), z.double().cpu().reshape(-1, C)
    sc, sh = coef[:C].double().cpu(), coef[C:].double().cpu()
    m = ((zz * sc + sh) > 0).double()   # exact in fp64: the sign of the kernels' fp32 fmaf
    gg = d * m
    return gg.sum(0), (gg * (zz - mean.double().cpu()) * invstd.double().cpu()).sum(0)


def _check(dx, part, z, coef, mean, invstd, dev):
    from pmu_hip import _lib as L
    C = z.shape[3]
    s1, s2 = _ref_sums(dx, z, coef, mean, invstd)
    got = part.double().view(-1, 2, C).sum(0).cpu()
    scale1, scale2 = s1.abs().max().item() + 1e-30, s2.abs().max().item() + 1e-30
    assert float((got[0] - s1).abs().max()) <= 1e-5 * max(scale1, dx.abs().sum().item() / C)
    assert float((got[1] - s2).abs().max()) <= 1e-5 * max(scale2, dx.abs().sum().item() / C)
    # the separate reduction pass over the same (dx, z) agrees with the fused one
    P = z.numel() // C
    R = L.lib().pmu_bn_bwd_tiles(P, C)
    ref_part = torch.empty(R, 2 * C, device=dev)
    L.call("pmu_bn_bwd_reduce", dx.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), P, C,
           ref_part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    rp = ref_part.double().view(-1, 2, C).sum(0).cpu()
    assert float((got - rp).abs().max()) <= 1e-5 * max(scale1, scale2, dx.abs().sum().item() / C)


@pytest.mark.parametrize("kind,N,H,W,Cin,Cout", [("wino4", 2, 64, 64, 64, 64), ("wino4", 1, 45, 37, 48, 40),
                                                 ("wino2h", 2, 16, 16, 256, 128), ("wino2h", 1, 20, 13, 64, 32)])
def test_dgrad_bnr_fp32(dev, kind, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from pmu_hip.engine import pack_weights_wino2h, pack_weights_wino4
    g = torch.Generator().manual_seed(5 + H + Cin)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    z, coef, mean, invstd = _bn_inputs(N, H, W, Cin, g, dev)
    wp = (pack_weights_wino4 if kind == "wino4" else pack_weights_wino2h)(w, True)
    R = getattr(L.lib(), f"pmu_conv3x3_tiles_{kind}")(N, H, W)
    dx = torch.empty(N, H, W, Cin, device=dev)
    part = torch.full((R, 2 * Cin), float("nan"), device=dev)
    L.call(f"pmu_conv3x3_dgrad_{kind}_bnr", dz.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, dx.data_ptr(),
           z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), L.stream())
    plain = torch.empty_like(dx)
    L.call(f"pmu_conv3x3_dgrad_{kind}", dz.data_ptr(), Cout, N, H, W, wp.data_ptr(), Cin, Cin, plain.data_ptr(), None,
           L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, plain)
    _check(dx, part, z, coef, mean, invstd, dev)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 40, 64, 64, 64), (1, 33, 45, 128, 96), (2, 32, 32, 256, 128)])
def test_dgrad_bnr_dma(dev, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, pack_weights_dma
    g = torch.Generator().manual_seed(17 + H + Cin)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    z, coef, mean, invstd = _bn_inputs(N, H, W, Cin, g, dev)
    dzt = frame_to_bf16([Src(dz)], N, H, W)
    wp = pack_weights_dma(w, True)
    R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3])
    dx = torch.empty(N, H, W, Cin, device=dev)
    part = torch.full((R, 2 * Cin), float("nan"), device=dev)
    L.call("pmu_conv3x3_dgrad_dma_bnr", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, dx.data_ptr(),
           z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), L.stream())
    plain = torch.empty_like(dx)
    L.call("pmu_conv3x3_dgrad_dma", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cin, plain.data_ptr(),
           None, L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, plain)
    _check(dx, part, z, coef, mean, invstd, dev)
