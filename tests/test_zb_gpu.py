"""bf16 storage of the pre-BN conv output z (config c5's torch.autocast dtype for a conv output,
PMU/model/unet/unet_parts.py:15,18 under autocast), centred on the BN running mean: the LDS-DMA forward
writes bf16(z - rm) (RNE) with the BN partial sums of stored + rm, and every consumer reads the stored
bf16 exactly — bit-for-bit what the fp32 kernels compute on the same values held in fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    """bf16 (RNE) of an fp32 tensor as int16 bit patterns, and those values back in fp32."""
    b = t.to(torch.bfloat16)
    return b.view(torch.int16).contiguous(), b.float().contiguous()


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 40, 64, 64, 64), (1, 33, 45, 128, 96), (2, 32, 32, 256, 128)])
def test_fwd_dma_zb_is_rounded_fp32(dev, exp_lib, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, pack_weights_dma
    g = torch.Generator().manual_seed(3 + H + Cin)
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    xt = frame_to_bf16([Src(x)], N, H, W)
    wp = pack_weights_dma(w, False)
    R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cout, xt.shape[3])
    z32 = torch.empty(N, H, W, Cout, device=dev)
    p32 = torch.empty(R, 2 * Cout, device=dev)
    L.call("pmu_conv3x3_fwd_dma", xt.data_ptr(), xt.shape[3], N, H, W, wp.data_ptr(), b.data_ptr(), Cout,
           z32.data_ptr(), p32.data_ptr(), L.stream())
    z16 = torch.empty(N, H, W, Cout, dtype=torch.int16, device=dev)
    p16 = torch.full((R, 2 * Cout), float("nan"), device=dev)
    off = (torch.randn(Cout, generator=g) * 3).to(dev)
    L.call("pmu_conv3x3_fwd_dma_zb", xt.data_ptr(), xt.shape[3], N, H, W, wp.data_ptr(), b.data_ptr(), Cout,
           z16.data_ptr(), off.data_ptr(), p16.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref_bits, ref_vals = _bits(z32 - off)
    assert torch.equal(z16, ref_bits)   # the same fp32 value, centred, rounded once (RNE)
    # BN partial sums: of the stored values + the offset
    zz = (ref_vals + off).double().reshape(-1, Cout)
    s1, s2 = zz.sum(0).cpu(), (zz * zz).sum(0).cpu()
    got = p16.double().view(-1, 2, Cout).sum(0).cpu()
    assert float((got[0] - s1).abs().max()) <= 1e-5 * float(zz.abs().sum(0).max())
    assert float((got[1] - s2).abs().max()) <= 1e-5 * float(s2.abs().max())


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 40, 64, 64, 64), (1, 33, 45, 128, 96)])
def test_dgrad_dma_bnr_zb(dev, exp_lib, N, H, W, Cin, Cout):
    """The *_bnr_zb partials equal the fp32-z kernel's on z rounded to bf16 bit for bit (same arithmetic
    on the same values), and dx is unchanged."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, pack_weights_dma
    g = torch.Generator().manual_seed(29 + H + Cin)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    z16, z = _bits(torch.randn(N, H, W, Cin, generator=g).to(dev))
    coef = torch.cat([torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.3]).to(dev)
    mean, invstd = (torch.randn(Cin, generator=g) * 0.2).to(dev), (torch.rand(Cin, generator=g) + 0.5).to(dev)
    dzt = frame_to_bf16([Src(dz)], N, H, W)
    wp = pack_weights_dma(w, True)
    R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3])
    outs = []
    for name, zp in (("pmu_conv3x3_dgrad_dma_bnr", z), ("pmu_conv3x3_dgrad_dma_bnr_zb", z16)):
        dx = torch.empty(N, H, W, Cin, device=dev)
        part = torch.full((R, 2 * Cin), float("nan"), device=dev)
        L.call(name, dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, dx.data_ptr(), zp.data_ptr(),
               coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), L.stream())
        outs.append((dx, part))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_bn_bwd_reduce_and_maxpool_bwd_zb(dev, exp_lib):
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(41)
    N, H, W, C = 2, 34, 50, 64
    P = N * H * W
    da = torch.randn(N, H, W, C, generator=g).to(dev)
    z16, z = _bits(torch.randn(N, H, W, C, generator=g).to(dev))
    coef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3]).to(dev)
    mean, invstd = (torch.randn(C, generator=g) * 0.2).to(dev), (torch.rand(C, generator=g) + 0.5).to(dev)
    R = L.lib().pmu_bn_bwd_tiles(P, C)
    parts = []
    for name, zp in (("pmu_bn_bwd_reduce", z), ("pmu_bn_bwd_reduce_zb", z16)):
        part = torch.full((R, 2 * C), float("nan"), device=dev)
        L.call(name, da.data_ptr(), zp.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), P, C,
               part.data_ptr(), L.stream())
        parts.append(part)
    dpool = torch.randn(N, H // 2, W // 2, C, generator=g).to(dev)
    dxs = []
    for name, zp in (("pmu_maxpool2_bwd", z), ("pmu_maxpool2_bwd_zb", z16)):
        dx = torch.randn(N, H, W, C, generator=torch.Generator().manual_seed(7)).to(dev)   # accumulate=1
        L.call(name, dpool.data_ptr(), zp.data_ptr(), coef.data_ptr(), N, H, W, C, dx.data_ptr(), 1, L.stream())
        dxs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(parts[0], parts[1])
    assert torch.equal(dxs[0], dxs[1])


@pytest.mark.parametrize("mode", ["bnrelu", "bnrelu_pool", "concat", "bnbwd"])
def test_frames_with_bf16_sources(dev, exp_lib, mode):
    """pmu_frame_to_bf16 / _f32 over bf16-stored sources = over the same values stored in fp32."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of, frame_to_bf16, frame_to_f32
    g = torch.Generator().manual_seed(53)
    N, H, W, C = 2, 18, 22, 64
    z16, z = _bits(torch.randn(N, H, W, C, generator=g).to(dev))
    coef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3]).to(dev)
    if mode == "bnrelu":
        a16, a32, fh, fw = [Src(z16, L.SRC_BNRELU, coef)], [Src(z, L.SRC_BNRELU, coef)], H, W
    elif mode == "bnrelu_pool":
        a16, a32 = [Src(z16, L.SRC_BNRELU, coef, pool=L.POOL_MAX2)], [Src(z, L.SRC_BNRELU, coef, pool=L.POOL_MAX2)]
        fh, fw = H // 2, W // 2
    elif mode == "concat":
        u = torch.randn(N, H - 2, W - 4, 32, generator=g).to(dev)
        a16 = [Src(z16, L.SRC_BNRELU, coef), Src(u, L.SRC_RAW, off=(1, 2))]
        a32 = [Src(z, L.SRC_BNRELU, coef), Src(u, L.SRC_RAW, off=(1, 2))]
        fh, fw = H, W
    else:
        da = torch.randn(N, H, W, C, generator=g).to(dev)
        bco = torch.cat([coef, (torch.randn(C, generator=g) * 0.1).to(dev), (torch.randn(3 * C, generator=g) * 0.1
                                                                             ).to(dev)[:2 * C]])
        a16, a32, fh, fw = [Src(da, L.SRC_BNBWD, bco, z=z16)], [Src(da, L.SRC_BNBWD, bco, z=z)], H, W
    r16, r32 = frame_to_bf16(a16, N, fh, fw), frame_to_bf16(a32, N, fh, fw)
    f16, f32 = frame_to_f32(a16, N, fh, fw), frame_to_f32(a32, N, fh, fw)
    torch.cuda.synchronize()
    assert torch.equal(r16, r32)
    assert torch.equal(f16, f32)
    # a fused-staging kernel refuses bf16-stored sources instead of misreading them
    if mode == "bnrelu":
        w = torch.randn(C, C, 3, 3, device=dev)
        out = torch.empty(N, H, W, C, device=dev)
        rc = L.lib().pmu_conv3x3_fwd(frame_of(a16, N, H, W), w.data_ptr(), None, None, C, out.data_ptr(), None, None,
                                     L.stream())
        assert rc == L.PMU_ERR_ARG


def test_head_with_bf16_source(dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    g = torch.Generator().manual_seed(61)
    N, H, W, C, K = 2, 16, 24, 64, 3
    z16, z = _bits(torch.randn(N, H, W, C, generator=g).to(dev))
    coef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3]).to(dev)
    w = torch.randn(K, C, generator=g).to(dev)
    b = torch.randn(K, generator=g).to(dev)
    ys = []
    for zz in (z16, z):
        y = torch.empty(N, K, H, W, device=dev)
        L.call("pmu_head1x1_fwd", frame_of([Src(zz, L.SRC_BNRELU, coef)], N, H, W), w.data_ptr(), b.data_ptr(), K, 0,
               y.data_ptr(), L.stream())
        ys.append(y)
    dl = torch.randn(N, K, H, W, generator=g).to(dev)
    dws = []
    for zz in (z16, z):
        dw, db = torch.empty(K, C, device=dev), torch.empty(K, device=dev)
        wsb = L.lib().pmu_wgrad1x1_ws(N * H * W, K, C)
        ws = torch.empty(max(1, (wsb + 3) // 4), device=dev)
        L.call("pmu_wgrad1x1", dl.data_ptr(), frame_of([Src(zz, L.SRC_BNRELU, coef)], N, H, W), K, dw.data_ptr(),
               db.data_ptr(), ws.data_ptr(), wsb, L.stream())
        dws.append((dw, db))
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])
    assert torch.equal(dws[0][0], dws[1][0]) and torch.equal(dws[0][1], dws[1][1])


@pytest.mark.parametrize("bf16_z", [True, False])
def test_unet_bf16_z_modes_vs_oracle(dev, exp_lib, monkeypatch, bf16_z):
    """Model level, both z modes against the oracle's autocast arithmetic with the same z rounding
    (oracle.unet_ref.BF16_Z): one training step of UNet(3, 3, [64, 128, 256]) at 64 x 64 (DMA convs
    with bf16-stored z at 64 and 32 wide, raw convs with rounded fp32 z at 16 wide).  Tolerance as
    test_bf16_gpu.py::test_unet_autocast_bf16: max(2e-3, 2 x the oracle's own fp32-vs-fp64 error)."""
    import oracle.unet_ref as U
    from helpers import grad_err
    from model import UNet
    from pmu_hip import engine
    monkeypatch.setattr(engine.CFG, "bf16_z", bf16_z)
    monkeypatch.setattr(U, "BF16_Z", bf16_z)
    torch.manual_seed(0)
    net = UNet(3, 3, [64, 128, 256])
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(4)
    x = torch.rand(2, 3, 64, 64, generator=g)
    tgt = torch.randint(0, 3, (2, 1, 64, 64), generator=g)
    keys = U.unet_param_keys(sd)

    def oracle(dt):
        sdd = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        params = {k: sdd[k].clone().requires_grad_(True) for k in keys}
        work = dict(sdd)
        work.update(params)
        o = U.unet_forward(work, x.to(dt), 3, 3, bf16=True)
        lo = U.unet_loss(o, tgt, 3)
        lo.backward()
        return o.detach(), float(lo), {k: params[k].grad for k in keys}

    ref, lref, gref = oracle(torch.float64)
    o32, l32, g32 = oracle(torch.float32)
    rel = lambda a, b: float((a.double().cpu() - b.double()).abs().max()) / float(b.abs().max())  # noqa: E731
    tol_out = max(2e-3, 2 * rel(o32, ref))
    tol_g = max(2e-3, 2 * grad_err(g32, gref)[0])
    net = net.to(dev).train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x.to(dev))
    loss = U.unet_loss(out, tgt.to(dev), 3)
    loss.backward()
    torch.cuda.synchronize()
    assert rel(out, ref) <= tol_out, (rel(out, ref), tol_out)
    assert abs(float(loss) - lref) <= max(2e-3, 2 * abs(l32 - lref) / abs(lref)) * abs(lref)
    named = dict(net.named_parameters())
    err, worst = grad_err({k: named[k].grad for k in keys}, gref)
    assert err <= tol_g, (err, worst, tol_g)


def test_bn_center(dev, exp_lib):
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(71)
    C = 96
    coef = torch.randn(2 * C, generator=g).to(dev)
    mean = torch.randn(C, generator=g).to(dev)
    off = torch.randn(C, generator=g).to(dev)
    c2, m2 = coef.clone(), mean.clone()
    L.call("pmu_bn_center", c2.data_ptr(), m2.data_ptr(), off.data_ptr(), C, c2.data_ptr(), m2.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(c2[:C], coef[:C])
    assert torch.allclose(c2[C:], coef[C:] + off * coef[:C], rtol=0, atol=1e-6)
    assert torch.equal(m2, mean - off)
