"""Streaming operand materialisation (wgrad3x3_bf16.hip frame_stream_kernel): pmu_frame_to_bf16 /
_f32 / _ld on single-source frames must equal the generic kernels (PMU_FRAME_STREAM=0) bit for bit,
and the operand the reference computes — BN+ReLU (unet_parts.py:24-27), MaxPool2d(2) of it
(unet_parts.py:38-39), the BN+ReLU backward — within fp32 rounding.  Ragged pixel counts, odd pooled
sources (floor mode), every power-of-two unit count up to 256, strided (_ld) outputs."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda")


def _frame(kind, N, H, W, C, dev, odd=False):
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src
    g = torch.Generator().manual_seed(H * 31 + C)
    SH, SW = (2 * H + int(odd), 2 * W + int(odd)) if kind == "pool" else (H, W)
    x = torch.randn(N, SH, SW, C, generator=g)
    sc, sh = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.3
    if kind == "bwd":
        z = torch.randn(N, SH, SW, C, generator=g)
        mu, kx, kc = torch.randn(C, generator=g) * 0.1, torch.randn(C, generator=g) * 0.1, torch.randn(C, generator=g) * 0.1
        coef = torch.cat([sc, sh, mu, kx, kc])
        xd = x.double()
        zd = z.double()
        ref = sc.double() * torch.where(zd * sc.double() + sh.double() > 0, xd, 0) + (kx.double() * (zd - mu.double()) + kc.double())
        return Src(x.to(dev), L.SRC_BNBWD, coef.to(dev), z=z.to(dev)), ref
    coef = torch.cat([sc, sh])
    a = torch.relu(x.double() * sc.double() + sh.double())
    if kind == "pool":
        a = torch.nn.functional.max_pool2d(a.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
        return Src(x.to(dev), L.SRC_BNRELU, coef.to(dev), pool=L.POOL_MAX2), a
    if kind == "raw":
        return Src(x.to(dev)), x.double()
    return Src(x.to(dev), L.SRC_BNRELU, coef.to(dev)), a


def _run(src, N, H, W, C, bf, ldo, generic):
    from pmu_hip import _lib as L
    from pmu_hip.engine import frame_of
    dt = torch.int16 if bf else torch.float32
    out = torch.full((N, H, W, ldo), -7, dtype=dt, device=src.x.device)
    f = frame_of([src], N, H, W)
    if generic:
        os.environ["PMU_FRAME_STREAM"] = "0"
    try:
        if ldo != C:
            name = "pmu_frame_to_bf16_ld" if bf else "pmu_frame_to_f32_ld"
            args = (f, C, out.data_ptr(), ldo) if bf else (f, out.data_ptr(), ldo)
        else:
            name = "pmu_frame_to_bf16" if bf else "pmu_frame_to_f32"
            args = (f, C, out.data_ptr()) if bf else (f, out.data_ptr())
        L.call(name, *args, L.stream())
        torch.cuda.synchronize()
    finally:
        os.environ.pop("PMU_FRAME_STREAM", None)
    return out


CASES = [("fwd", 3, 7, 9, 64), ("fwd", 2, 33, 17, 8), ("fwd", 1, 5, 5, 2048), ("raw", 2, 9, 11, 128),
         ("pool", 2, 8, 8, 64), ("pool", 3, 5, 7, 128), ("pool", 1, 4, 4, 1024), ("bwd", 2, 13, 11, 64),
         ("bwd", 1, 6, 6, 512), ("bwd", 5, 3, 3, 16), ("fwd", 2, 6, 6, 24)]


@pytest.mark.parametrize("bf", [True, False])
@pytest.mark.parametrize("kind,N,H,W,C", CASES)
def test_frame_stream_equals_generic(dev, bf, kind, N, H, W, C):
    src, ref = _frame(kind, N, H, W, C, dev, odd=(H % 2 == 1))
    got = _run(src, N, H, W, C, bf, C, generic=False)
    gen = _run(src, N, H, W, C, bf, C, generic=True)
    assert torch.equal(got, gen)
    val = got.view(torch.bfloat16).double().cpu() if bf else got.double().cpu()
    tol = 2 ** -8 if bf else 1e-6
    assert ((val - ref).abs() <= tol * (1 + ref.abs())).all()


@pytest.mark.parametrize("bf", [True, False])
@pytest.mark.parametrize("kind,C,ldo", [("fwd", 64, 128), ("fwd", 256, 512), ("pool", 128, 256)])
def test_frame_stream_ld(dev, bf, kind, C, ldo):
    """Strided output (the skip half of the Up block's concat operand): channels [C, ldo) untouched."""
    N, H, W = 2, 10, 6
    src, _ = _frame(kind, N, H, W, C, dev)
    got = _run(src, N, H, W, C, bf, ldo, generic=False)
    gen = _run(src, N, H, W, C, bf, ldo, generic=True)
    assert torch.equal(got, gen)
    assert (got[..., C:] == -7).all()


@pytest.mark.parametrize("bf", [True, False])
@pytest.mark.parametrize("N,H,W,C,Ccat", [(2, 8, 8, 64, 128), (3, 5, 7, 128, 192), (1, 16, 4, 8, 16)])
def test_frame_pool_skip(dev, bf, N, H, W, C, Ccat):
    """pmu_frame_to_*_pool_skip: the max-pooled operand and the unpooled skip half of the concat operand
    from one pass, bit-equal to pmu_frame_to_* of the pooled frame + pmu_frame_to_*_ld of the unpooled
    one (unet_parts.py:33 and :66); the concat's other channels untouched."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    src, _ = _frame("pool", N, H, W, C, dev)
    dt = torch.int16 if bf else torch.float32
    f = frame_of([src], N, H, W)
    assert L.lib().pmu_frame_pool_skip_ok(f)
    pooled = torch.full((N, H, W, C), -3, dtype=dt, device=dev)
    xcat = torch.full((N, 2 * H, 2 * W, Ccat), -7, dtype=dt, device=dev)
    L.call("pmu_frame_to_bf16_pool_skip" if bf else "pmu_frame_to_f32_pool_skip", f, pooled.data_ptr(),
           xcat.data_ptr(), Ccat, L.stream())
    torch.cuda.synchronize()
    ref_pool = _run(src, N, H, W, C, bf, C, generic=True)
    unpooled = Src(src.x, src.mode, src.coef)
    ref_skip = _run(unpooled, N, 2 * H, 2 * W, C, bf, Ccat, generic=True)
    assert torch.equal(pooled, ref_pool)
    assert torch.equal(xcat[..., :C], ref_skip[..., :C])
    assert (xcat[..., C:] == -7).all()


def test_frame_pool_skip_refuses_odd_sources(dev):
    """Floor-mode pooling of an odd map leaves a row / column outside every window: not this path."""
    from pmu_hip import _lib as L
    from pmu_hip.engine import frame_of
    src, _ = _frame("pool", 1, 5, 5, 64, dev, odd=True)
    assert not L.lib().pmu_frame_pool_skip_ok(frame_of([src], 1, 5, 5))
