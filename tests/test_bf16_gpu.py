"""GPU parity of the bf16-MFMA kernels (config c5) against a PyTorch reference of the same arithmetic.

The kernels round each operand to bf16 (RNE) after the fp32 BN/ReLU/pool/concat transform and sum
the exact bf16 x bf16 products in fp32.  The reference therefore rounds the same operands to bf16
and convolves them in fp64: the only differences left are the fp32 summation order and rare
operands whose fp32 transform lands on the other side of a bf16 rounding boundary.
Tolerance: max|d| / max|ref| <= 1e-3 (observed ~1e-6).
"""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu

TOL = 1e-3


def _rb(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _pack(w, dgrad):
    from pmu_hip import _lib as L
    n = L.lib().pmu_conv3x3_packed_size_bf16(w.shape[0], w.shape[1], int(dgrad)) // 2
    wp = torch.empty(n, dtype=torch.int16, device=w.device)
    L.call("pmu_conv3x3_pack_bf16", w.data_ptr(), w.shape[0], w.shape[1], int(dgrad), wp.data_ptr(), L.stream())
    return wp


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _bnrelu(z, coef):
    C = z.shape[-1]
    return torch.relu(z * coef[:C] + coef[C:])


def _fwd(srcs, N, H, W, w, bias, dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import frame_of
    Cout = w.shape[0]
    z = torch.empty(N, H, W, Cout, device=dev)
    R = L.lib().pmu_conv3x3_tiles(N, H, W)
    part = torch.empty(R, 2 * Cout, device=dev)
    wp = _pack(w, False)
    L.call("pmu_conv3x3_fwd_bf16", frame_of(srcs, N, H, W), wp.data_ptr(), L.ptr(bias), Cout, z.data_ptr(),
           part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    return z, part


def _ref_conv(op_nhwc, w, bias):
    y = TF.conv2d(_nchw(_rb(op_nhwc)).double().cpu(), _rb(w).double().cpu(),
                  None if bias is None else bias.double().cpu(), padding=1)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 40, 40, 32, 96), (1, 64, 64, 64, 64), (3, 12, 20, 16, 128),
                                            (2, 9, 7, 6, 10)])
def test_conv3x3_fwd_bf16_raw(dev, N, H, W, Cin, Cout):
    from pmu_hip.engine import Src
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + H)
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    z, part = _fwd([Src(x)], N, H, W, w, b, dev)
    ref = _ref_conv(x, w, b)
    assert _rel(z, ref) <= TOL
    # BN partials: the per-tile (sum, sum of squares) add up to the column sums of z
    s = part.view(-1, 2, Cout).double().sum(0).cpu()
    zz = z.double().cpu().reshape(-1, Cout)
    assert _rel(s[0], zz.sum(0)) <= 1e-4
    assert _rel(s[1], (zz * zz).sum(0)) <= 1e-4


def test_conv3x3_fwd_bf16_bnrelu_maxpool(dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src
    N, H, W, Cin, Cout = 2, 34, 30, 64, 64
    g = torch.Generator().manual_seed(5)
    z0 = torch.randn(N, 2 * H + 1, 2 * W, Cin, generator=g).to(dev)   # odd height: floor pooling
    coef = torch.cat([torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.2]).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05).to(dev)
    z, _ = _fwd([Src(z0, L.SRC_BNRELU, coef, pool=L.POOL_MAX2)], N, H, W, w, None, dev)
    a = _bnrelu(z0, coef)
    op = TF.max_pool2d(_nchw(a), 2).permute(0, 2, 3, 1)
    assert _rel(z, _ref_conv(op, w, None)) <= TOL


def test_conv3x3_fwd_bf16_concat_pad(dev):
    """cat([skip, F.pad(up)], 1) with the up source offset inside the frame (unet_parts.py:58-66)."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src
    N, H, W, C0, C1, Cout = 2, 21, 19, 32, 32, 64
    g = torch.Generator().manual_seed(7)
    zs = torch.randn(N, H, W, C0, generator=g).to(dev)
    coef = torch.cat([torch.rand(C0, generator=g) + 0.5, torch.randn(C0, generator=g) * 0.2]).to(dev)
    u = torch.randn(N, H - 1, W - 1, C1, generator=g).to(dev)
    w = (torch.randn(Cout, C0 + C1, 3, 3, generator=g) * 0.05).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    z, _ = _fwd([Src(zs, L.SRC_BNRELU, coef), Src(u, off=(0, 0))], N, H, W, w, b, dev)
    up = torch.zeros(N, H, W, C1, device=dev)
    up[:, :H - 1, :W - 1] = u
    op = torch.cat([_bnrelu(zs, coef), up], dim=3)
    assert _rel(z, _ref_conv(op, w, b)) <= TOL


@pytest.mark.parametrize("N,H,W,Cin,Cout,split", [(2, 40, 36, 64, 32, 64), (2, 17, 33, 128, 64, 64),
                                                  (1, 8, 8, 96, 128, 32)])
def test_conv3x3_dgrad_bf16(dev, N, H, W, Cin, Cout, split):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    g = torch.Generator().manual_seed(11 + H)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1).to(dev)
    wp = _pack(w, True)
    dx0 = torch.empty(N, H, W, split, device=dev)
    dx1 = torch.empty(N, H, W, Cin - split, device=dev) if split < Cin else None
    L.call("pmu_conv3x3_dgrad_bf16", frame_of([Src(dz)], N, H, W), wp.data_ptr(), Cin, split, dx0.data_ptr(),
           L.ptr(dx1), L.stream())
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, W), _rb(w).double().cpu(), _nchw(_rb(dz)).double().cpu(),
                                     padding=1).permute(0, 2, 3, 1)
    got = dx0 if dx1 is None else torch.cat([dx0, dx1], dim=3)
    assert _rel(got, ref) <= TOL
