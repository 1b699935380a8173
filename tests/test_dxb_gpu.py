"""bf16 activation gradients (config c5; the *_dxb entries of include/pmunet_hip.h).

torch.autocast(bfloat16) returns a conv's input gradient in bf16 (PMU/model/unet/unet_parts.py:15,18
backward).  The LDS-DMA input gradient stores it so and its consumers read it so:
  * pmu_conv3x3_dgrad_dma{,_bnr,_x1b,_x1b_sum}_dxb: dx / dx0 = the bf16 (RNE) rounding of what the fp32
    entry computes, bit for bit (same kernel, same accumulation order); dx1, dx1b, column sums and the
    producer's BN-backward partials formed from the rounded values;
  * the BN-backward dz frame (pmu_frame_to_bf16 / _f32, streaming and generic kernels), pmu_bn_bwd_reduce_dxb,
    pmu_maxpool2_bwd_bnr_dxb and pmu_conv_first_wgrad on a bf16 da: bit-equal to the fp32 entries on an
    fp32 copy of the same values;
  * the UNet under autocast with and without bf16 dx (engine CFG.dx_bf16 / oracle BF16_DX) against the
    oracle modelling the same storage."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    """fp32 -> bf16 (RNE) bit patterns as int16, the kernels' storage."""
    return t.to(torch.bfloat16).view(torch.int16)


def _val(b):
    return b.view(torch.bfloat16).float()


def _setup(N, H, W, Cin, Cout, seed, dev):
    from pmu_hip.engine import Src, frame_to_bf16, pack_weights_dma
    g = torch.Generator().manual_seed(seed)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    return g, frame_to_bf16([Src(dz)], N, H, W), pack_weights_dma(w, True)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 40, 64, 64, 64), (1, 33, 45, 128, 96), (4, 32, 32, 256, 512)])
def test_dgrad_dma_dxb_and_bnr(dev, N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from test_bnr_gpu import _bn_inputs, _check
    g, dzt, wp = _setup(N, H, W, Cin, Cout, 41 + H + Cin, dev)
    ref = torch.empty(N, H, W, Cin, device=dev)
    L.call("pmu_conv3x3_dgrad_dma", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cin, ref.data_ptr(),
           None, L.stream())
    dxb = torch.full((N, H, W, Cin), -1, dtype=torch.int16, device=dev)
    L.call("pmu_conv3x3_dgrad_dma_dxb", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cin, dxb.data_ptr(),
           None, L.stream())
    z, coef, mean, invstd = _bn_inputs(N, H, W, Cin, g, dev)
    R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3])
    part = torch.full((R, 2 * Cin), float("nan"), device=dev)
    dxr = torch.full((N, H, W, Cin), -1, dtype=torch.int16, device=dev)
    L.call("pmu_conv3x3_dgrad_dma_bnr_dxb", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, dxr.data_ptr(),
           z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dxb, _bits(ref))
    assert torch.equal(dxr, dxb)
    _check(_val(dxr).contiguous(), part, z, coef, mean, invstd, dev)   # partials of the rounded dx


@pytest.mark.parametrize("N,H,W,Cskip,Cup,Cout", [(2, 64, 64, 64, 64, 64), (1, 33, 45, 128, 64, 96)])
def test_dgrad_dma_split_dxb(dev, N, H, W, Cskip, Cup, Cout):
    """the concat split: dx0 bf16; dx1 (fp32 storage) the rounded values, dx1b their bits; the column-sum
    variant's transposed-conv bias gradient = the sum of the rounded dx1."""
    from pmu_hip import _lib as L
    _, dzt, wp = _setup(N, H, W, Cskip + Cup, Cout, 43 + H + Cskip, dev)
    Cin = Cskip + Cup
    r0, r1 = torch.empty(N, H, W, Cskip, device=dev), torch.empty(N, H, W, Cup, device=dev)
    L.call("pmu_conv3x3_dgrad_dma", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip, r0.data_ptr(),
           r1.data_ptr(), L.stream())
    d0 = torch.empty(N, H, W, Cskip, dtype=torch.int16, device=dev)
    d1 = torch.empty(N, H, W, Cup, device=dev)
    d1b = torch.empty(N, H, W, Cup, dtype=torch.int16, device=dev)
    L.call("pmu_conv3x3_dgrad_dma_dxb", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip, d0.data_ptr(),
           d1.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(d0, _bits(r0)) and torch.equal(d1, _val(_bits(r1)))
    e0, e1 = torch.empty_like(d0), torch.empty_like(d1)
    L.call("pmu_conv3x3_dgrad_dma_x1b_dxb", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip,
           e0.data_ptr(), e1.data_ptr(), d1b.data_ptr(), L.stream())
    R = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, dzt.shape[3])
    part = torch.full((R, 2 * Cin), float("nan"), device=dev)
    f0, f1b = torch.empty_like(d0), torch.empty_like(d1b)
    L.call("pmu_conv3x3_dgrad_dma_x1b_sum_dxb", dzt.data_ptr(), dzt.shape[3], N, H, W, wp.data_ptr(), Cin, Cskip,
           f0.data_ptr(), f1b.data_ptr(), part.data_ptr(), L.stream())
    db = torch.empty(Cup, device=dev)
    wsd = torch.empty(L.lib().pmu_convT2x2_dbias_rows_ws(Cup) // 4, device=dev)
    L.call("pmu_convT2x2_dbias_rows", part.data_ptr() + 4 * Cskip, R, 2 * Cin, Cup, db.data_ptr(), wsd.data_ptr(),
           L.stream())
    torch.cuda.synchronize()
    assert torch.equal(e0, d0) and torch.equal(e1, d1) and torch.equal(d1b, _bits(r1))
    assert torch.equal(f0, d0) and torch.equal(f1b, d1b)
    rr = _val(d1b).double()
    ref = rr.sum(dim=(0, 1, 2))
    assert ((db.double() - ref).abs() <= 1e-5 * (rr.abs().sum(dim=(0, 1, 2)) + 1)).all()


def test_dxb_rejects_odd_channels(dev):
    from pmu_hip import _lib as L
    _, dzt, wp = _setup(1, 32, 32, 36, 32, 3, dev)
    d = torch.empty(1, 32, 32, 36, dtype=torch.int16, device=dev)
    rc = L.lib().pmu_conv3x3_dgrad_dma_dxb(dzt.data_ptr(), dzt.shape[3], 1, 32, 32, wp.data_ptr(), 36, 36, d.data_ptr(),
                                           None, L.stream())
    assert rc == L.PMU_ERR_ARG


@pytest.mark.parametrize("stream", ["1", "0"])
@pytest.mark.parametrize("N,H,W,C", [(2, 64, 64, 64), (3, 17, 23, 128), (1, 8, 8, 1024)])
def test_bnbwd_frame_bf16_da(dev, stream, N, H, W, C):
    """The BN-backward dz frame over a bf16-stored da: bf16 and fp32 operands bit-equal to the same frame
    over an fp32 copy of da (streaming kernel and, PMU_FRAME_STREAM=0, the generic one)."""
    from pmu_hip.engine import Src, frame_to_bf16, frame_to_f32
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(47 + H + C)
    dab = _bits(torch.randn(N, H, W, C, generator=g)).to(dev)
    z = torch.randn(N, H, W, C, generator=g).to(dev)
    bcoef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3,
                       torch.randn(C, generator=g) * 0.2, torch.randn(C, generator=g), torch.randn(C, generator=g)]).to(dev)
    daf = _val(dab).contiguous()
    old = os.environ.get("PMU_FRAME_STREAM")
    os.environ["PMU_FRAME_STREAM"] = stream
    try:
        got_b = frame_to_bf16([Src(dab, L.SRC_BNBWD, bcoef, z=z)], N, H, W)
        want_b = frame_to_bf16([Src(daf, L.SRC_BNBWD, bcoef, z=z)], N, H, W)
        got_f = frame_to_f32([Src(dab, L.SRC_BNBWD, bcoef, z=z)], N, H, W)
        want_f = frame_to_f32([Src(daf, L.SRC_BNBWD, bcoef, z=z)], N, H, W)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("PMU_FRAME_STREAM")
        else:
            os.environ["PMU_FRAME_STREAM"] = old
    assert torch.equal(got_b, want_b) and torch.equal(got_f, want_f)


@pytest.mark.parametrize("N,H,W,C", [(2, 64, 64, 64), (1, 33, 45, 32), (2, 16, 16, 512), (1, 7, 9, 1040)])
def test_maxpool2_bwd_bnr_dxb(dev, N, H, W, C):
    """bf16 pooled and skip gradients: dx = skip + routed dpool and the partials bit-equal to
    pmu_maxpool2_bwd_bnr accumulating onto an fp32 copy of the skip gradient; without a skip, to the
    non-accumulating form."""
    from pmu_hip import _lib as L
    from test_bnr_gpu import _bn_inputs
    g = torch.Generator().manual_seed(53 + H + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    dpb = _bits(torch.randn(N, H // 2, W // 2, C, generator=g)).to(dev)
    skb = _bits(torch.randn(N, H, W, C, generator=g)).to(dev)
    R = L.lib().pmu_maxpool2_bwd_bnr_tiles(N, H, W, C)
    for acc in (1, 0):
        dx = torch.full((N, H, W, C), float("nan"), device=dev)
        part = torch.full((R, 2 * C), float("nan"), device=dev)
        L.call("pmu_maxpool2_bwd_bnr_dxb", dpb.data_ptr(), skb.data_ptr() if acc else None, z.data_ptr(),
               coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), N, H, W, C, dx.data_ptr(), part.data_ptr(),
               L.stream())
        ref = _val(skb).contiguous() if acc else torch.full((N, H, W, C), float("nan"), device=dev)
        rpart = torch.full((R, 2 * C), float("nan"), device=dev)
        L.call("pmu_maxpool2_bwd_bnr", _val(dpb).contiguous().data_ptr(), z.data_ptr(), coef.data_ptr(),
               mean.data_ptr(), invstd.data_ptr(), N, H, W, C, ref.data_ptr(), acc, rpart.data_ptr(), L.stream())
        torch.cuda.synchronize()
        if acc:
            assert torch.equal(dx, ref) and torch.equal(part, rpart)
        else:   # (the fp32 form leaves positions outside full windows as they were; compare where written)
            m = ~torch.isnan(ref)
            assert torch.equal(dx[m], ref[m]) and torch.equal(part, rpart)


@pytest.mark.parametrize("P,C", [(40000, 64), (1234, 128), (5000, 1024)])
def test_bn_bwd_reduce_dxb(dev, P, C):
    from pmu_hip import _lib as L
    from test_bnr_gpu import _bn_inputs
    g = torch.Generator().manual_seed(59 + C)
    z, coef, mean, invstd = _bn_inputs(1, 1, P, C, g, dev)
    dab = _bits(torch.randn(1, 1, P, C, generator=g)).to(dev)
    R = L.lib().pmu_bn_bwd_tiles(P, C)
    a, b = torch.empty(R, 2 * C, device=dev), torch.empty(R, 2 * C, device=dev)
    L.call("pmu_bn_bwd_reduce_dxb", dab.data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
           P, C, a.data_ptr(), L.stream())
    L.call("pmu_bn_bwd_reduce", _val(dab).contiguous().data_ptr(), z.data_ptr(), coef.data_ptr(), mean.data_ptr(),
           invstd.data_ptr(), P, C, b.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("Cin,Cout", [(3, 64), (1, 32)])
def test_conv_first_wgrad_bf16_da(dev, Cin, Cout):
    """The first layer's weight gradient over a BN-backward frame whose da is bf16 (the second conv's
    *_dxb input gradient) equals the fp32-da result on the same values."""
    import ctypes
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    N, H, W = 2, 48, 64
    g = torch.Generator().manual_seed(61 + Cin)
    dab = _bits(torch.randn(N, H, W, Cout, generator=g)).to(dev)
    z = torch.randn(N, H, W, Cout, generator=g).to(dev)
    bcoef = torch.cat([torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g) * 0.3,
                       torch.randn(Cout, generator=g) * 0.2, torch.randn(Cout, generator=g),
                       torch.randn(Cout, generator=g)]).to(dev)
    planes = [torch.randn(N, H, W, generator=g).to(dev) for _ in range(Cin)]
    arr = (ctypes.c_void_p * Cin)(*[p.data_ptr() for p in planes])
    wsb = L.lib().pmu_conv_first_wgrad_ws(N, H, W, Cin, Cout)
    out = []
    for da in (dab, _val(dab).contiguous()):
        dw = torch.empty(Cout, Cin, 3, 3, device=dev)
        ws = torch.empty((wsb + 3) // 4, device=dev)
        L.call("pmu_conv_first_wgrad", frame_of([Src(da, L.SRC_BNBWD, bcoef, z=z)], N, H, W), arr, Cin, Cout,
               dw.data_ptr(), ws.data_ptr(), wsb, L.stream())
        out.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("dxb", [True, False])
@pytest.mark.parametrize("filters,n_cls,N,H,W,C", [([16, 32, 64], 3, 2, 64, 64, 1),
                                                   ([32, 64, 128, 256], 3, 2, 80, 72, 3)])
def test_unet_autocast_dx_storage(dev, dxb, filters, n_cls, N, H, W, C):
    """model.UNet under autocast with bf16 (CFG.dx_bf16, the default) and fp32 activation gradients, each
    against the oracle modelling the same storage (oracle.unet_ref.BF16_DX) in fp64, at the tolerance of
    test_bf16_gpu.py::test_unet_autocast_bf16 (max(2e-3, 2 x the oracle's own fp32-vs-fp64 error))."""
    import oracle.unet_ref as ur
    from helpers import grad_err
    from model import UNet
    from pmu_hip import engine
    from test_bf16_gpu import _rel
    torch.manual_seed(0)
    net = UNet(C, n_cls, filters)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(4)
    x = torch.rand(N, C, H, W, generator=g)
    tgt = torch.randint(0, n_cls, (N, 1, H, W), generator=g)
    keys = ur.unet_param_keys(sd)
    old_o, old_e = ur.BF16_DX, engine.CFG.dx_bf16
    ur.BF16_DX, engine.CFG.dx_bf16 = dxb, dxb
    try:
        def oracle(dt):
            sdd = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
            params = {k: sdd[k].clone().requires_grad_(True) for k in keys}
            work = dict(sdd)
            work.update(params)
            o = ur.unet_forward(work, x.to(dt), len(filters), n_cls, bf16=True)
            lo = ur.unet_loss(o, tgt, n_cls)
            lo.backward()
            return o.detach(), float(lo), {k: params[k].grad for k in keys}
        ref, lref, gref = oracle(torch.float64)
        o32, l32, g32 = oracle(torch.float32)
        tol_g = max(2e-3, 2 * grad_err(g32, gref)[0])
        net = net.to(dev).train()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = net(x.to(dev))
        loss = ur.unet_loss(out, tgt.to(dev), n_cls)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        ur.BF16_DX, engine.CFG.dx_bf16 = old_o, old_e
    assert _rel(out, ref) <= max(2e-3, 2 * _rel(o32, ref))
    assert abs(float(loss) - lref) <= max(2e-3, 2 * abs(l32 - lref) / abs(lref)) * abs(lref)
    named = dict(net.named_parameters())
    err, worst = grad_err({k: named[k].grad for k in keys}, gref)
    assert err <= tol_g, (err, worst, tol_g)


@pytest.mark.parametrize("N,H,W,Cin,Cout,off", [(2, 32, 32, 128, 64, (0, 0)), (1, 16, 24, 256, 128, (1, 0)),
                                                (2, 8, 8, 1024, 512, (0, 1))])
def test_convT_dgrad_dma_dxb(dev, N, H, W, Cin, Cout, off):
    """pmu_convT2x2_dgrad_dma_dxb: the bf16 (RNE) bits of pmu_convT2x2_dgrad_dma's dx (same kernel, same
    sums), including an F.pad offset into du."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_to_bf16, pack_convT_weights_dma
    g = torch.Generator().manual_seed(67 + H + Cin)
    Hd, Wd = 2 * H + off[0] + 1, 2 * W + off[1]
    du = torch.randn(N, Hd, Wd, Cout, generator=g).to(dev)
    w = (torch.randn(Cin, Cout, 2, 2, generator=g) * 0.05).to(dev)
    dut = frame_to_bf16([Src(du)], N, Hd, Wd)
    wp = pack_convT_weights_dma(w, True)
    ref = torch.empty(N, H, W, Cin, device=dev)
    L.call("pmu_convT2x2_dgrad_dma", dut.data_ptr(), dut.shape[3], Hd, Wd, off[0], off[1], wp.data_ptr(), N, H, W, Cin,
           Cout, ref.data_ptr(), L.stream())
    got = torch.full((N, H, W, Cin), -1, dtype=torch.int16, device=dev)
    L.call("pmu_convT2x2_dgrad_dma_dxb", dut.data_ptr(), dut.shape[3], Hd, Wd, off[0], off[1], wp.data_ptr(), N, H, W,
           Cin, Cout, got.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(got, _bits(ref))
