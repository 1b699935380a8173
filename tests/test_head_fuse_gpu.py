"""The last layer's activation gradient left unstored (engine.HeadDa, CFG.head_fuse): OutConv's input
gradient (PMU/model/unet/unet_parts.py:70-76 backward) is only ever consumed by the last DoubleConv's
BN+ReLU backward (unet_parts.py:19), so
  * pmu_head1x1_bwd_bnr with da NULL forms the BN-backward partials and the head's weight gradient
    bit-equal to the da-storing pass;
  * pmu_head1x1_bwd_dz writes that layer's dz (bf16 or fp32) straight from dy, bit-equal to
    pmu_frame_to_bf16 / _f32 of the BN-backward frame over the stored da;
and the whole UNet backward is bit-identical with and without it (fp32 and bf16 autocast)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,C,sig", [(1, 64, True), (3, 64, False), (2, 32, False), (1, 16, True)])
@pytest.mark.parametrize("bf16", [True, False])
def test_head_dz_matches_stored_da(dev, K, C, sig, bf16):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, frame_to_f32
    from test_bnr_gpu import _bn_inputs
    if bf16 and C % 8:
        pytest.skip("bf16 dz takes C % 8 == 0")
    N, H, W = 3, 40, 56
    g = torch.Generator().manual_seed(71 + K + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    dy = torch.randn(N, K, H, W, generator=g).to(dev)
    y = torch.rand(N, K, H, W, generator=g).to(dev)
    w = (torch.randn(K, C, generator=g) * 0.3).to(dev)
    bcoef = torch.cat([coef[:C].cpu(), coef[C:].cpu(), torch.randn(C, generator=g) * 0.2,
                       torch.randn(C, generator=g), torch.randn(C, generator=g)]).to(dev)
    R = L.lib().pmu_head1x1_bwd_tiles(N, H, W)
    wsb = L.lib().pmu_wgrad1x1_ws(N * H * W, K, C)
    outs = []
    for store in (True, False):
        da = torch.full((N, H, W, C), float("nan"), device=dev) if store else None
        part = torch.full((R, 2 * C), float("nan"), device=dev)
        dw = torch.full((K, C), float("nan"), device=dev)
        db = torch.full((K,), float("nan"), device=dev)
        ws = torch.empty((wsb + 3) // 4, device=dev)
        L.call("pmu_head1x1_bwd_bnr", dy.data_ptr(), y.data_ptr(), int(sig), w.data_ptr(), K, C, N, H, W, None,
               L.ptr(da), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(),
               dw.data_ptr(), db.data_ptr(), ws.data_ptr(), wsb, L.stream())
        outs.append((da, part, dw, db))
    torch.cuda.synchronize()
    da = outs[0][0]
    for a, b in zip(outs[0][1:], outs[1][1:]):
        assert torch.equal(a, b)
    src = Src(da, L.SRC_BNBWD, bcoef, z=z)
    want = frame_to_bf16([src], N, H, W) if bf16 else frame_to_f32([src], N, H, W)
    got = torch.empty(N, H, W, C, dtype=torch.int16 if bf16 else torch.float32, device=dev)
    L.call("pmu_head1x1_bwd_dz", dy.data_ptr(), y.data_ptr(), int(sig), w.data_ptr(), K, C, N, H, W, z.data_ptr(),
           bcoef.data_ptr(), int(bf16), got.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("bf16,channels,classes,filters,N,H", [(False, 1, 1, [16, 32, 64, 128], 2, 64),
                                                               (True, 3, 3, [32, 64, 128, 256], 2, 128)])
def test_unet_backward_bit_identical(dev, bf16, channels, classes, filters, N, H):
    """model.UNet: every gradient bit-identical with CFG.head_fuse on and off (fp32: c2's one-class
    sigmoid head; bf16 autocast: c5's three-class head)."""
    from model import UNet
    from pmu_hip import engine
    torch.manual_seed(0)
    net = UNet(channels, classes, filters).to(dev).train()
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(9)
    x = torch.rand(N, channels, H, H, generator=g).to(dev)
    r = torch.randn(N, classes, H, H, generator=g).to(dev)
    grads = []
    old = engine.CFG.head_fuse
    try:
        for fuse in (True, False):
            engine.CFG.head_fuse = fuse
            net.load_state_dict(sd)
            net.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(x)
            (out.float() * r).sum().backward()
            torch.cuda.synchronize()
            grads.append({k: p.grad.clone() for k, p in net.named_parameters()})
    finally:
        engine.CFG.head_fuse = old
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


@pytest.mark.parametrize("K,C,sig", [(1, 8, True), (3, 16, False), (3, 64, False), (1, 64, True), (2, 128, False),
                                     (4, 256, True)])
@pytest.mark.parametrize("xbf", [False, True])
def test_head_fwd_fast_vs_fp64(dev, K, C, sig, xbf):
    """pmu_head1x1_fwd's channel-quad fast path (OutConv on the last layer's BN+ReLU, unet_parts.py:70-76):
    the per-class sum over a pixel's C/4 quad lanes by DPP row moves (pmu_group_sum, plus xor shuffles
    across rows for C/4 = 32, 64) against the fp64 sum of the same products; the source's x in fp32 or
    bf16 (autocast's activations)."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    N, H, W = 2, 37, 45
    g = torch.Generator().manual_seed(13 + K + C)
    z = torch.randn(N, H, W, C, generator=g)
    if xbf:
        z = z.to(torch.bfloat16).float()
    coef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3])
    w = torch.randn(K, C, generator=g) * 0.3
    b = torch.randn(K, generator=g)
    a = torch.relu(z.double() * coef[:C].double() + coef[C:].double())
    ref = torch.einsum("nhwc,kc->nkhw", a, w.double()) + b.double().view(1, K, 1, 1)
    if sig:
        ref = torch.sigmoid(ref)
    zx = z.to(torch.bfloat16).view(torch.int16).to(dev) if xbf else z.to(dev)
    src = Src(zx, L.SRC_BNRELU, coef.to(dev))
    f = frame_of([src], N, H, W)
    y = torch.full((N, K, H, W), float("nan"), device=dev)
    wd, bd = w.to(dev), b.to(dev)
    L.call("pmu_head1x1_fwd", f, wd.data_ptr(), bd.data_ptr(), K, int(sig), y.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert not torch.isnan(y).any()
    assert (y.double().cpu() - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())
