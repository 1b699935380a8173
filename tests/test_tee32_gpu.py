"""GPU parity of the fp32 operand tee (pmu_conv3x3_fwd / _dgrad ``tee``) and of the weight gradient
on the teed RAW operands.

The conv kernels copy the operand they staged (BN+ReLU, max-pool, F.pad+cat, or the BN+ReLU backward
of dz) to the tee tensor; it must equal the frame materialised by pmu_frame_to_f32 bit for bit, and
the weight gradient over the two RAW frames must equal the one that re-derives them (same staged
values, same MFMA order: equal up to FMA contraction, rel 1e-6).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _to_f32(srcs, N, H, W):
    from pmu_hip import _lib as L
    from pmu_hip.engine import frame_of
    C = sum(sr.C for sr in srcs)
    out = torch.empty(N, H, W, C, device=srcs[0].x.device)
    L.call("pmu_frame_to_f32", frame_of(srcs, N, H, W), out.data_ptr(), L.stream())
    return out


def _coef(C, g, dev):
    return torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.2]).to(dev)


def _bcoef(C, g, dev):
    return torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1,
                      torch.randn(C, generator=g) * 0.1, torch.randn(C, generator=g) * 0.01,
                      torch.randn(C, generator=g) * 0.01]).to(dev)


def _frames(kind, N, H, W, g, dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src
    if kind == "bnrelu":
        z = torch.randn(N, H, W, 64, generator=g).to(dev)
        return [Src(z, L.SRC_BNRELU, _coef(64, g, dev))]
    if kind == "maxpool":
        z = torch.randn(N, 2 * H, 2 * W, 64, generator=g).to(dev)
        return [Src(z, L.SRC_BNRELU, _coef(64, g, dev), pool=L.POOL_MAX2)]
    if kind == "concat":
        z = torch.randn(N, H, W, 64, generator=g).to(dev)
        u = torch.randn(N, H - 1, W - 2, 64, generator=g).to(dev)
        return [Src(z, L.SRC_BNRELU, _coef(64, g, dev)), Src(u, off=(0, 1))]
    if kind == "narrow":  # reduction channels not a multiple of 16: the synchronous kernel
        z = torch.randn(N, H, W, 20, generator=g).to(dev)
        return [Src(z, L.SRC_BNRELU, _coef(20, g, dev))]
    raise ValueError(kind)


@pytest.mark.parametrize("kind,N,H,W", [("bnrelu", 2, 40, 36), ("maxpool", 2, 24, 20), ("concat", 2, 33, 17),
                                        ("narrow", 1, 16, 16), ("bnrelu", 1, 7, 9)])
def test_conv3x3_fwd_tee32(dev, exp_lib, kind, N, H, W):
    from pmu_hip import _lib as L
    from pmu_hip.engine import frame_of, pack_weights
    g = torch.Generator().manual_seed(5 + H)
    srcs = _frames(kind, N, H, W, g, dev)
    Cin, Cout = sum(s.C for s in srcs), 128
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    z0, z1 = torch.empty(N, H, W, Cout, device=dev), torch.empty(N, H, W, Cout, device=dev)
    R = L.lib().pmu_conv3x3_tiles(N, H, W)
    p0, p1 = torch.empty(R, 2 * Cout, device=dev), torch.empty(R, 2 * Cout, device=dev)
    tee = torch.full((N, H, W, Cin), float("nan"), device=dev)
    wp = pack_weights(w, False)
    L.call("pmu_conv3x3_fwd", frame_of(srcs, N, H, W), w.data_ptr(), wp.data_ptr(), b.data_ptr(), Cout,
           z0.data_ptr(), p0.data_ptr(), None, L.stream())
    L.call("pmu_conv3x3_fwd", frame_of(srcs, N, H, W), w.data_ptr(), wp.data_ptr(), b.data_ptr(), Cout,
           z1.data_ptr(), p1.data_ptr(), tee.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(tee, _to_f32(srcs, N, H, W))
    assert torch.equal(z0, z1) and torch.equal(p0, p1)  # the tee does not perturb the product


@pytest.mark.parametrize("N,H,W,Cin,Cout,split", [(2, 40, 36, 128, 64, 64), (2, 17, 33, 64, 128, 64),
                                                  (1, 8, 8, 64, 64, 64)])
def test_conv3x3_dgrad_tee32_and_raw_wgrad(dev, exp_lib, N, H, W, Cin, Cout, split):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of, pack_weights
    g = torch.Generator().manual_seed(17 + W)
    da = torch.randn(N, H, W, Cout, generator=g).to(dev)
    z = torch.randn(N, H, W, Cout, generator=g).to(dev)
    dsrc = [Src(da, L.SRC_BNBWD, _bcoef(Cout, g, dev), z=z)]
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    xsrc = [Src(x, L.SRC_BNRELU, _coef(Cin, g, dev))]
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    wp = pack_weights(w, True)
    dx0 = torch.empty(N, H, W, split, device=dev)
    dx1 = torch.empty(N, H, W, Cin - split, device=dev) if split < Cin else None
    dzt = torch.full((N, H, W, Cout), float("nan"), device=dev)
    L.call("pmu_conv3x3_dgrad", frame_of(dsrc, N, H, W), w.data_ptr(), wp.data_ptr(), Cin, split, dx0.data_ptr(),
           L.ptr(dx1), dzt.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dzt, _to_f32(dsrc, N, H, W))
    xt = _to_f32(xsrc, N, H, W)
    wsb = L.lib().pmu_conv3x3_wgrad_ws(N, H, W, Cin, Cout)
    ws = torch.empty(wsb // 4 + 1, device=dev)
    dw_fused, dw_raw = torch.empty_like(w), torch.empty_like(w)
    L.call("pmu_conv3x3_wgrad", frame_of(dsrc, N, H, W), frame_of(xsrc, N, H, W), Cout, dw_fused.data_ptr(),
           ws.data_ptr(), wsb, L.stream())
    L.call("pmu_conv3x3_wgrad", frame_of([Src(dzt)], N, H, W), frame_of([Src(xt)], N, H, W), Cout,
           dw_raw.data_ptr(), ws.data_ptr(), wsb, L.stream())
    torch.cuda.synchronize()
    rel = float((dw_raw - dw_fused).abs().max() / dw_fused.abs().max())
    assert rel <= 1e-6, rel
