"""The pooled layer's activation gradient left unstored (engine.PoolSumDa, CFG.pool_fuse; config c5's
skip levels): da = skip + routed dpool (MaxPool2d(2) backward, PMU/model/unet/unet_parts.py:33, plus the
skip path, unet_parts.py:66) is formed twice in registers instead of written in fp32 and re-read (bf16
parts with a bf16 dz, or — config c2 — fp32 parts with an fp32 dz) —
  * pmu_maxpool2_bwd_bnr_stats_dxb: the BN-backward partial sums alone, bit-equal to those of
    pmu_maxpool2_bwd_bnr_dxb;
  * pmu_maxpool2_bwd_bnbwd_dxb: the layer's bf16 dz, bit-equal to pmu_frame_to_bf16 of the BN-backward
    frame over the stored da;
so the whole UNet backward is bit-identical with and without it."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.to(torch.bfloat16).view(torch.int16)


@pytest.mark.parametrize("N,H,W,C", [(2, 64, 64, 64), (1, 33, 45, 32), (2, 16, 16, 512), (1, 7, 9, 1024),
                                     (1, 8, 6, 2048), (16, 128, 128, 128)])
def test_stats_and_dz_match_stored_da(dev, N, H, W, C):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16
    from test_bnr_gpu import _bn_inputs
    g = torch.Generator().manual_seed(67 + H + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    dpb = _bits(torch.randn(N, H // 2, W // 2, C, generator=g)).to(dev)
    skb = _bits(torch.randn(N, H, W, C, generator=g)).to(dev)
    bcoef = torch.cat([coef[:C].cpu(), coef[C:].cpu(), torch.randn(C, generator=g) * 0.2,
                       torch.randn(C, generator=g), torch.randn(C, generator=g)]).to(dev)
    R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, H, W, C)
    da = torch.full((N, H, W, C), float("nan"), device=dev)
    part = torch.full((R, 2 * C), float("nan"), device=dev)
    L.call("pmu_maxpool2_bwd_bnr_dxb", dpb.data_ptr(), skb.data_ptr(), z.data_ptr(), coef.data_ptr(),
           mean.data_ptr(), invstd.data_ptr(), N, H, W, C, da.data_ptr(), part.data_ptr(), L.stream())
    ps = torch.full((R, 2 * C), float("nan"), device=dev)
    L.call("pmu_maxpool2_bwd_bnr_stats_dxb", dpb.data_ptr(), skb.data_ptr(), z.data_ptr(), coef.data_ptr(),
           mean.data_ptr(), invstd.data_ptr(), N, H, W, C, ps.data_ptr(), L.stream())
    want = frame_to_bf16([Src(da, L.SRC_BNBWD, bcoef, z=z)], N, H, W)
    got = torch.full((N, H, W, C), -1, dtype=torch.int16, device=dev)
    L.call("pmu_maxpool2_bwd_bnbwd_dxb", dpb.data_ptr(), skb.data_ptr(), z.data_ptr(), coef.data_ptr(),
           bcoef.data_ptr(), N, H, W, C, C, got.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert not torch.isnan(da).any()
    assert torch.equal(ps, part)
    assert torch.equal(got, want)


@pytest.mark.parametrize("N,H,W,C", [(2, 64, 64, 64), (1, 33, 45, 32), (2, 16, 16, 512), (32, 64, 64, 128)])
def test_fp32_stats_and_dz_match_stored_da(dev, N, H, W, C):
    """fp32 parts (config c2): the partials bit-equal to pmu_maxpool2_bwd_bnr accumulating into the skip
    gradient, dz bit-equal to pmu_frame_to_f32 of the BN-backward frame over that stored da."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_f32
    from test_bnr_gpu import _bn_inputs
    g = torch.Generator().manual_seed(73 + H + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    dp = torch.randn(N, H // 2, W // 2, C, generator=g).to(dev)
    sk = torch.randn(N, H, W, C, generator=g).to(dev)
    bcoef = torch.cat([coef[:C].cpu(), coef[C:].cpu(), torch.randn(C, generator=g) * 0.2,
                       torch.randn(C, generator=g), torch.randn(C, generator=g)]).to(dev)
    R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, H, W, C)
    da = sk.clone()
    part = torch.full((R, 2 * C), float("nan"), device=dev)
    L.call("pmu_maxpool2_bwd_bnr", dp.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
           N, H, W, C, da.data_ptr(), 1, part.data_ptr(), L.stream())
    ps = torch.full((R, 2 * C), float("nan"), device=dev)
    L.call("pmu_maxpool2_bwd_bnr_stats", dp.data_ptr(), sk.data_ptr(), z.data_ptr(), coef.data_ptr(),
           mean.data_ptr(), invstd.data_ptr(), N, H, W, C, ps.data_ptr(), L.stream())
    want = frame_to_f32([Src(da, L.SRC_BNBWD, bcoef, z=z)], N, H, W)
    got = torch.full((N, H, W, C), float("nan"), device=dev)
    L.call("pmu_maxpool2_bwd_bnbwd", dp.data_ptr(), sk.data_ptr(), z.data_ptr(), coef.data_ptr(), bcoef.data_ptr(),
           N, H, W, C, C, got.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(ps, part)
    assert torch.equal(got, want)


def test_bnbwd_refuses_unsupported_channels(dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import pool_fuse_ok
    assert not pool_fuse_ok(96) and not pool_fuse_ok(1040) and pool_fuse_ok(64) and pool_fuse_ok(2048)
    t = torch.empty(4 * 8 * 8 * 96, device=dev)
    rc = L.lib().pmu_maxpool2_bwd_bnbwd_dxb(t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(),
                                           1, 8, 8, 96, 96, t.data_ptr(), L.stream())
    assert rc == L.PMU_ERR_ARG


@pytest.mark.parametrize("bf16,channels,classes,filters,N,H", [(True, 3, 3, [16, 32, 64, 128], 2, 128),
                                                               (True, 3, 3, [64, 128, 256, 512, 1024], 2, 64),
                                                               (False, 1, 1, [16, 32, 64, 128], 2, 64),
                                                               (False, 1, 1, [64, 128, 256, 512, 1024], 4, 64)])
def test_unet_backward_bit_identical(dev, bf16, channels, classes, filters, N, H):
    """model.UNet (under autocast: bf16 parts; fp32: c2's path): every gradient bit-identical with
    CFG.pool_fuse on and off."""
    from model import UNet
    from pmu_hip import engine
    torch.manual_seed(0)
    net = UNet(channels, classes, filters).to(dev).train()
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(8)
    x = torch.rand(N, channels, H, H, generator=g).to(dev)
    r = torch.randn(N, classes, H, H, generator=g).to(dev)
    grads = []
    old = engine.CFG.pool_fuse
    try:
        for fuse in (True, False):
            engine.CFG.pool_fuse = fuse
            net.load_state_dict(sd)
            net.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x)
            (out.float() * r).sum().backward()
            torch.cuda.synchronize()
            grads.append({k: p.grad.clone() for k, p in net.named_parameters()})
    finally:
        engine.CFG.pool_fuse = old
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k
