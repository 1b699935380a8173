"""ConvTranspose2d(k2, s2) of Up (PMU/model/unet/unet_parts.py:41-67) on the pipelined fp32 kernels,
against a float64 CPU reference: the forward with the producer's BN+ReLU applied while staging
(pmu_convT2x2_fwd), and the input gradient (pmu_convT2x2_dgrad) and the weight/bias gradient (pmu_convT2x2_wgrad).  Power-of-two maps take the
shift/mask epilogue, the odd ones the division epilogue; M = N*H*W is not a multiple of the
128-row tile in the odd cases."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))

TOL = 2e-5   # fp32 MFMA sums vs float64, relative to the output's max magnitude


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 16, 16, 128, 64), (3, 13, 10, 128, 64), (1, 8, 32, 256, 128),
                                            (2, 7, 9, 64, 32)])
def test_convT_fwd_dgrad_match_float64(N, H, W, Cin, Cout):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of, pack_convT_weights
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + W)
    z = torch.randn(N, H, W, Cin, generator=g)
    sc, sh = torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.2
    w = torch.randn(Cin, Cout, 2, 2, generator=g) * 0.05
    b = torch.randn(Cout, generator=g) * 0.1
    du = torch.randn(N, 2 * H, 2 * W, Cout, generator=g)
    # float64 reference
    act = torch.relu(z.double() * sc.double() + sh.double()).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv_transpose2d(act, w.double(), b.double(), stride=2).permute(0, 2, 3, 1)
    a = act.clone().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    torch.nn.functional.conv_transpose2d(a, wr, br, stride=2).backward(du.double().permute(0, 3, 1, 2))
    ref_dx = a.grad.permute(0, 2, 3, 1)
    # HIP
    zd, wd, bd, dud = z.to(dev), w.to(dev), b.to(dev), du.to(dev)
    coef = torch.cat([sc, sh]).to(dev)
    u = torch.empty(N, 2 * H, 2 * W, Cout, device=dev)
    dx = torch.empty(N, H, W, Cin, device=dev)
    s = L.stream()
    L.call("pmu_convT2x2_fwd", frame_of([Src(zd, L.SRC_BNRELU, coef)], N, H, W), wd.data_ptr(),
           pack_convT_weights(wd, False).data_ptr(), bd.data_ptr(), Cout, u.data_ptr(), s)
    L.call("pmu_convT2x2_dgrad", dud.data_ptr(), 2 * H, 2 * W, 0, 0, wd.data_ptr(),
           pack_convT_weights(wd, True).data_ptr(), N, H, W, Cin, Cout, dx.data_ptr(), s)
    dw = torch.empty_like(wd)
    db = torch.empty(Cout, device=dev)
    wsb = L.lib().pmu_convT2x2_wgrad_ws(N, H, W, Cin, Cout)
    ws = torch.empty(max(1, (wsb + 3) // 4), device=dev)
    L.call("pmu_convT2x2_wgrad", dud.data_ptr(), 2 * H, 2 * W, 0, 0, frame_of([Src(zd, L.SRC_BNRELU, coef)], N, H, W),
           Cout, dw.data_ptr(), db.data_ptr(), ws.data_ptr(), wsb, s)
    torch.cuda.synchronize()
    e_w = ((dw.cpu().double() - wr.grad).abs().max() / wr.grad.abs().max()).item()
    e_b = ((db.cpu().double() - br.grad).abs().max() / br.grad.abs().max()).item()
    assert e_w <= TOL and e_b <= TOL, (e_w, e_b)
    e_u = ((u.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    e_dx = ((dx.cpu().double() - ref_dx).abs().max() / ref_dx.abs().max()).item()
    assert e_u <= TOL and e_dx <= TOL, (e_u, e_dx)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,Cin,Cup,Cskip", [(2, 16, 16, 128, 64, 64), (1, 8, 32, 256, 128, 128),
                                                  (1, 7, 9, 128, 64, 64)])  # odd pixel count (pair stores)
def test_concat_operand_built_in_place(N, H, W, Cin, Cup, Cskip):
    """The Up block's concat operand written in place (unet_parts.py:52,66): pmu_convT2x2_fwd_ld /
    pmu_convT2x2_fwd_dma_ldb fill channels [Cskip, Cskip + Cup) and pmu_frame_to_f32_ld /
    pmu_frame_to_bf16_ld channels [0, Cskip) of one tensor — bit-equal to materialising the two-source
    frame (skip activation, convT output) with pmu_frame_to_f32 / pmu_frame_to_bf16."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import (BF16S, Src, frame_of, frame_to_bf16, frame_to_f32, pack_convT_weights,
                                pack_convT_weights_dma)
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(H * 7 + Cin)
    z = torch.randn(N, H, W, Cin, generator=g).to(dev)
    coef = torch.cat([torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.2]).to(dev)
    zs = torch.randn(N, 2 * H, 2 * W, Cskip, generator=g).to(dev)
    cs = torch.cat([torch.rand(Cskip, generator=g) + 0.5, torch.randn(Cskip, generator=g) * 0.2]).to(dev)
    w = (torch.randn(Cin, Cup, 2, 2, generator=g) * 0.05).to(dev)
    b = (torch.randn(Cup, generator=g) * 0.1).to(dev)
    Ho, Wo, Cc = 2 * H, 2 * W, Cskip + Cup
    act, skip = Src(z, L.SRC_BNRELU, coef), Src(zs, L.SRC_BNRELU, cs)
    s = L.stream()
    # fp32
    fin = frame_of([act], N, H, W)
    assert L.lib().pmu_convT2x2_fwd_ld_ok(fin, Cup)
    wp = pack_convT_weights(w, dgrad=False)
    u = torch.empty(N, Ho, Wo, Cup, device=dev)
    L.call("pmu_convT2x2_fwd", fin, w.data_ptr(), wp.data_ptr(), b.data_ptr(), Cup, u.data_ptr(), s)
    ref = frame_to_f32([skip, Src(u)], N, Ho, Wo)
    xcat = torch.full((N, Ho, Wo, Cc), float("nan"), device=dev)
    L.call("pmu_convT2x2_fwd_ld", fin, w.data_ptr(), wp.data_ptr(), b.data_ptr(), Cup, xcat.data_ptr() + 4 * Cskip,
           Cc, s)
    L.call("pmu_frame_to_f32_ld", frame_of([skip], N, Ho, Wo), xcat.data_ptr(), Cc, s)
    # bf16
    xt = frame_to_bf16([act], N, H, W)
    wpd = pack_convT_weights_dma(w, dgrad=False)
    ub = torch.empty(N, Ho, Wo, Cup, device=dev)
    L.call("pmu_convT2x2_fwd_dma", xt.data_ptr(), xt.shape[3], N, H, W, wpd.data_ptr(), b.data_ptr(), Cin, Cup,
           ub.data_ptr(), s)
    refb = frame_to_bf16([skip, Src(ub)], N, Ho, Wo)
    xcatb = torch.full((N, Ho, Wo, Cc), -1, dtype=BF16S, device=dev)
    L.call("pmu_convT2x2_fwd_dma_ldb", xt.data_ptr(), xt.shape[3], N, H, W, wpd.data_ptr(), b.data_ptr(), Cin, Cup,
           xcatb.data_ptr() + 2 * Cskip, Cc, s)
    L.call("pmu_frame_to_bf16_ld", frame_of([skip], N, Ho, Wo), Cskip, xcatb.data_ptr(), Cc, s)
    torch.cuda.synchronize()
    assert torch.equal(xcat, ref)
    assert torch.equal(xcatb, refb)
