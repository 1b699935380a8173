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


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 40, 64, 64, 64), (1, 33, 45, 128, 96), (2, 32, 32, 256, 128),
                                            (32, 90, 70, 64, 64)])  # last: more tiles than resident workgroups
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


@pytest.mark.parametrize("N,H,W,Cskip,Cup,Cout", [(2, 64, 64, 64, 64, 64), (1, 33, 45, 128, 64, 96)])
def test_dgrad_dma_split_bf16_copy(dev, N, H, W, Cskip, Cup, Cout):
    """pmu_conv3x3_dgrad_dma_x1b: dx0 / dx1 bit-equal to pmu_conv3x3_dgrad_dma with the same split, and
    dx1b the bf16 (RNE) rounding of dx1 — what pmu_frame_to_bf16 makes of it (unet_parts.py:52,66)."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, pack_weights_dma
    g = torch.Generator().manual_seed(23 + H + Cskip)
    Cin = Cskip + Cup
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    dzt = frame_to_bf16([Src(dz)], N, H, W)
    wp = pack_weights_dma(w, True)
    dx0, dx1 = torch.empty(N, H, W, Cskip, device=dev), torch.empty(N, H, W, Cup, device=dev)
    dx1b = torch.empty(N, H, W, Cup, dtype=torch.int16, device=dev)
    L.call("pmu_conv3x3_dgrad_dma_x1b", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip,
           dx0.data_ptr(), dx1.data_ptr(), dx1b.data_ptr(), L.stream())
    r0, r1 = torch.empty_like(dx0), torch.empty_like(dx1)
    L.call("pmu_conv3x3_dgrad_dma", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip, r0.data_ptr(),
           r1.data_ptr(), L.stream())
    ref_b = frame_to_bf16([Src(r1)], N, H, W)
    torch.cuda.synchronize()
    assert torch.equal(dx0, r0) and torch.equal(dx1, r1)
    assert torch.equal(dx1b, ref_b)


@pytest.mark.parametrize("N,H,W,Cskip,Cup,Cout", [(2, 64, 64, 64, 64, 64), (1, 33, 45, 128, 64, 96)])
def test_dgrad_dma_split_bf16_colsum(dev, N, H, W, Cskip, Cup, Cout):
    """pmu_conv3x3_dgrad_dma_x1b_sum: dx0 / dx1b bit-equal to pmu_conv3x3_dgrad_dma_x1b, no fp32 dx1, and
    pmu_convT2x2_dbias_rows over its per-tile column sums = the transposed conv's bias gradient, the
    sum of dx1 over all pixels (unet_parts.py:52 backward), to fp32 summation rounding."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, pack_weights_dma
    g = torch.Generator().manual_seed(29 + H + Cskip)
    Cin = Cskip + Cup
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    dzt = frame_to_bf16([Src(dz)], N, H, W)
    wp = pack_weights_dma(w, True)
    dx0, dx1b = torch.empty(N, H, W, Cskip, device=dev), torch.empty(N, H, W, Cup, dtype=torch.int16, device=dev)
    R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3])
    part = torch.full((R, 2 * Cin), float("nan"), device=dev)
    L.call("pmu_conv3x3_dgrad_dma_x1b_sum", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip,
           dx0.data_ptr(), dx1b.data_ptr(), part.data_ptr(), L.stream())
    db = torch.empty(Cup, device=dev)
    wsd = torch.empty(L.lib().pmu_convT2x2_dbias_rows_ws(Cup) // 4, device=dev)
    L.call("pmu_convT2x2_dbias_rows", part.data_ptr() + 4 * Cskip, R, 2 * Cin, Cup, db.data_ptr(), wsd.data_ptr(),
           L.stream())
    r0, r1 = torch.empty_like(dx0), torch.empty(N, H, W, Cup, device=dev)
    rb = torch.empty_like(dx1b)
    L.call("pmu_conv3x3_dgrad_dma_x1b", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip,
           r0.data_ptr(), r1.data_ptr(), rb.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx0, r0) and torch.equal(dx1b, rb)
    ref = r1.double().sum(dim=(0, 1, 2))
    assert ((db.double() - ref).abs() <= 1e-5 * (r1.double().abs().sum(dim=(0, 1, 2)) + 1)).all()
    assert (part[:, Cin:] == 0).all()


@pytest.mark.parametrize("N,H,W,C", [(2, 64, 64, 64), (1, 33, 45, 32), (2, 16, 16, 512), (1, 7, 9, 1040), (2, 9, 11, 192),
                                     (1, 6, 8, 2064)])
def test_maxpool2_bwd_bnr(dev, N, H, W, C):
    """pmu_maxpool2_bwd_bnr: dx bit-equal to pmu_maxpool2_bwd accumulated onto the same skip gradient
    (odd maps: the last row / column gets the skip gradient only), and the partials of the result."""
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(31 + H + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    z[:, ::3, ::2, :5] = -coef[C:C + 5].cpu().to(dev) / coef[:5]   # a few exact ties of the activation at 0
    dpool = torch.randn(N, H // 2, W // 2, C, generator=g).to(dev)
    skip = torch.randn(N, H, W, C, generator=g).to(dev)
    dx = skip.clone()
    R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, H, W, C)
    part = torch.full((R, 2 * C), float("nan"), device=dev)
    L.call("pmu_maxpool2_bwd_bnr", dpool.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(),
           invstd.data_ptr(), N, H, W, C, dx.data_ptr(), 1, part.data_ptr(), L.stream())
    ref = skip.clone()
    L.call("pmu_maxpool2_bwd", dpool.data_ptr(), z.data_ptr(), coef.data_ptr(), N, H, W, C, ref.data_ptr(), 1,
           L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx, ref)
    # against torch's max_pool2d backward on the activation (first max of each window)
    act = torch.relu(z.double().cpu() * coef[:C].double().cpu() + coef[C:].double().cpu()).permute(0, 3, 1, 2)
    act.requires_grad_(True)
    torch.nn.functional.max_pool2d(act, 2).backward(dpool.double().cpu().permute(0, 3, 1, 2))
    want = skip.double().cpu() + act.grad.permute(0, 2, 3, 1)
    assert float((dx.double().cpu() - want).abs().max()) <= 1e-6 * float(want.abs().max())
    _check(dx, part, z, coef, mean, invstd, dev)


@pytest.mark.parametrize("N,H,W,C,K,sig", [(2, 64, 64, 64, 1, 1), (3, 37, 45, 32, 3, 0), (1, 16, 16, 256, 2, 0)])
@pytest.mark.parametrize("fused_wgrad", [False, True])
def test_head1x1_bwd_bnr(dev, N, H, W, C, K, sig, fused_wgrad):
    """pmu_head1x1_bwd_bnr: da (and dl) bit-equal to pmu_head1x1_bwd, the BN-backward partials of da,
    and (fused_wgrad) the head's dw / db bit-equal to pmu_wgrad1x1 on the BN+ReLU activation of z."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    g = torch.Generator().manual_seed(41 + H + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    dy = torch.randn(N, K, H, W, generator=g).to(dev)
    y = torch.rand(N, K, H, W, generator=g).to(dev)
    w = (torch.randn(K, C, generator=g) * 0.1).to(dev)
    lb = L.lib()
    assert lb.pmu_head1x1_bwd_bnr_ok(N, H, W, C)
    R = lb.pmu_head1x1_bwd_tiles(N, H, W)
    part = torch.full((R, 2 * C), float("nan"), device=dev)
    dl, da = torch.empty(N, K, H, W, device=dev), torch.empty(N, H, W, C, device=dev)
    wsb = lb.pmu_wgrad1x1_ws(N * H * W, K, C)
    ws = torch.empty(wsb // 4 + 1, device=dev)
    dw, db = torch.full((K, C), float("nan"), device=dev), torch.full((K,), float("nan"), device=dev)
    L.call("pmu_head1x1_bwd_bnr", dy.data_ptr(), y.data_ptr(), sig, w.data_ptr(), K, C, N, H, W,
           None if fused_wgrad else dl.data_ptr(), da.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(),
           invstd.data_ptr(), part.data_ptr(), dw.data_ptr() if fused_wgrad else None,
           db.data_ptr() if fused_wgrad else None, ws.data_ptr(), wsb, L.stream())
    dl2, da2 = torch.empty_like(dl), torch.empty_like(da)
    L.call("pmu_head1x1_bwd", dy.data_ptr(), y.data_ptr(), sig, w.data_ptr(), K, C, N, H, W, dl2.data_ptr(),
           da2.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(da, da2)
    if fused_wgrad:
        dw2, db2 = torch.empty_like(dw), torch.empty_like(db)
        ws2 = torch.empty_like(ws)
        L.call("pmu_wgrad1x1", dl2.data_ptr(), frame_of([Src(z, L.SRC_BNRELU, coef)], N, H, W), K, dw2.data_ptr(),
               db2.data_ptr(), ws2.data_ptr(), wsb, L.stream())
        torch.cuda.synchronize()
        assert torch.equal(dw, dw2) and torch.equal(db, db2)
    else:
        assert torch.equal(dl, dl2)
    _check(da, part, z, coef, mean, invstd, dev)


@pytest.mark.parametrize("N,H,W,C", [(2, 64, 64, 64), (3, 33, 45, 128), (2, 16, 16, 1040), (1, 7, 9, 192)])
@pytest.mark.parametrize("kind", ["avgpool", "mean"])
def test_encoder_bwd_bnr(dev, N, H, W, C, kind):
    """The Probabilistic U-Net encoder's passes that complete a layer's da (probabilistic_unet.py:36
    AvgPool2d(2, ceil_mode) backward, :39 spatial-mean backward) fused with that layer's BN+ReLU backward
    partials: da bit-equal to pmu_avgpool2_bwd / pmu_spatial_mean_bwd, the partials equal to
    pmu_bn_bwd_reduce's on the same (da, z) bit for bit (same blocks, same pixel order) and to fp64."""
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(41 + H + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    if kind == "avgpool":
        src = torch.randn(N, (H + 1) // 2, (W + 1) // 2, C, generator=g).to(dev)
        ref = torch.empty(N, H, W, C, device=dev)
        L.call("pmu_avgpool2_bwd", src.data_ptr(), N, H, W, C, ref.data_ptr(), L.stream())
        name = "pmu_avgpool2_bwd_bnr"
    else:
        src = torch.randn(N, C, generator=g).to(dev)
        ref = torch.empty(N, H, W, C, device=dev)
        L.call("pmu_spatial_mean_bwd", src.data_ptr(), N, H, W, C, ref.data_ptr(), L.stream())
        name = "pmu_spatial_mean_bwd_bnr"
    P = N * H * W
    R = L.lib().pmu_bn_bwd_tiles(P, C)
    da = torch.full((N, H, W, C), float("nan"), device=dev)
    part = torch.full((R, 2 * C), float("nan"), device=dev)
    L.call(name, src.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), N, H, W, C,
           da.data_ptr(), part.data_ptr(), L.stream())
    ref_part = torch.empty(R, 2 * C, device=dev)
    L.call("pmu_bn_bwd_reduce", ref.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), P, C,
           ref_part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(da, ref)
    assert torch.equal(part, ref_part)
    _check(da, part, z, coef, mean, invstd, dev)
