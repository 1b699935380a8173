"""Persistent tile schedule of the LDS-DMA bf16 convs (conv3x3_bf16_dma.hip, PERS): one resident
workgroup per slot walks a run of tiles, fetching the next tile's first chunk under the current one's
last.  Each tile's arithmetic is the one-tile-per-workgroup kernel's, so the two schedules must agree
bit for bit, on every output: z / dx / the bf16 copies / the BN and column-sum partials.  The schedule
is an experiments-build variant (measured slower): these tests run on that library
(exp_lib), PMU_DMA_PERS=1 against unset.  Shapes: both workgroup shapes, ragged tiles and channel
blocks, 1-4 channel blocks per tile, the concat split, the bf16-dx and BN-backward epilogues."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _pack(w, dgrad):
    from pmu_hip import _lib as L
    n = L.lib().pmu_conv3x3_packed_size_dma(w.shape[0], w.shape[1], int(dgrad)) // 2
    wp = torch.empty(n, dtype=torch.int16, device=w.device)
    L.call("pmu_conv3x3_pack_dma", w.data_ptr(), w.shape[0], w.shape[1], int(dgrad), wp.data_ptr(), L.stream())
    return wp


def _both(monkeypatch, run):
    """run() under the persistent and the one-tile schedule; returns both output tuples"""
    outs = []
    for v in ("1", None):
        if v is None:
            monkeypatch.delenv("PMU_DMA_PERS")
        else:
            monkeypatch.setenv("PMU_DMA_PERS", v)
        outs.append(run())
        torch.cuda.synchronize()
    monkeypatch.setenv("PMU_DMA_PERS", "1")
    return outs


def _same(a, b):
    for x, y in zip(a, b):
        if x is None:
            continue
        assert torch.equal(x.view(torch.int16) if x.dtype == torch.bfloat16 else x,
                           y.view(torch.int16) if y.dtype == torch.bfloat16 else y)


@pytest.mark.parametrize("N,H,W,Cp,Cout", [(10, 256, 256, 64, 64), (9, 250, 200, 64, 96),
                                           (6, 130, 130, 256, 256), (4, 128, 160, 256, 512)])
def test_fwd_persistent_matches_one_tile(dev, exp_lib, monkeypatch, N, H, W, Cp, Cout):
    from pmu_hip import _lib as L
    monkeypatch.setenv("PMU_DMA_PERS", "1")
    assert exp_lib.pmu_conv3x3_dma_persistent(N, H, W, Cout, Cp) == 1
    g = torch.Generator().manual_seed(5 + H + Cout)
    xt = torch.randn(N, H, W, Cp, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, Cp, 3, 3, generator=g) * 0.05).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    wp = _pack(w, False)
    tiles = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cout, Cp)

    def run():
        z = torch.full((N, H, W, Cout), float("nan"), device=dev)
        part = torch.full((tiles, 2 * Cout), float("nan"), device=dev)
        L.call("pmu_conv3x3_fwd_dma", xt.data_ptr(), Cp, N, H, W, wp.data_ptr(), b.data_ptr(), Cout, z.data_ptr(),
               part.data_ptr(), L.stream())
        return z, part

    p, o = _both(monkeypatch, run)
    assert not torch.isnan(p[0]).any() and not torch.isnan(p[1]).any()
    _same(p, o)
    # and against the math on two images (fp32 conv of the bf16 operand)
    ref = torch.nn.functional.conv2d(xt[:2].float().permute(0, 3, 1, 2), w.float(), b, padding=1).permute(0, 2, 3, 1)
    err = ((p[0][:2] - ref).norm() / ref.norm()).item()
    assert err < 2e-3


@pytest.mark.parametrize("kind", ["plain", "dxb", "x1b_sum_dxb", "bnr", "bnr_dxb"])
@pytest.mark.parametrize("N,H,W,Cp,Cin,split", [(10, 256, 256, 64, 128, 64), (6, 130, 130, 256, 256, 128)])
def test_dgrad_persistent_matches_one_tile(dev, exp_lib, monkeypatch, kind, N, H, W, Cp, Cin, split):
    from pmu_hip import _lib as L
    if kind.startswith("bnr"):
        split = Cin
    monkeypatch.setenv("PMU_DMA_PERS", "1")
    assert exp_lib.pmu_conv3x3_dma_persistent(N, H, W, Cin, Cp) == 1
    g = torch.Generator().manual_seed(17 + H + Cin)
    dzt = torch.randn(N, H, W, Cp, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cp, Cin, 3, 3, generator=g) * 0.05).to(dev)
    wp = _pack(w, True)
    tiles = L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, Cp)
    z = torch.randn(N, H, W, Cin, generator=g).to(dev)
    coef = torch.cat([torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.2]).to(dev)
    mean = (torch.randn(Cin, generator=g) * 0.1).to(dev)
    invstd = (torch.rand(Cin, generator=g) + 0.5).to(dev)
    bf = torch.bfloat16

    def run():
        nan = float("nan")
        if kind == "plain":
            dx0 = torch.full((N, H, W, split), nan, device=dev)
            dx1 = torch.full((N, H, W, Cin - split), nan, device=dev)
            L.call("pmu_conv3x3_dgrad_dma", dzt.data_ptr(), Cp, N, H, W, wp.data_ptr(), Cin, split, dx0.data_ptr(),
                   dx1.data_ptr(), L.stream())
            return dx0, dx1
        if kind == "dxb":
            dx0 = torch.full((N, H, W, split), nan, device=dev, dtype=bf)
            dx1 = torch.full((N, H, W, Cin - split), nan, device=dev)
            L.call("pmu_conv3x3_dgrad_dma_dxb", dzt.data_ptr(), Cp, N, H, W, wp.data_ptr(), Cin, split,
                   dx0.data_ptr(), dx1.data_ptr(), L.stream())
            return dx0, dx1
        if kind == "x1b_sum_dxb":
            dx0 = torch.full((N, H, W, split), nan, device=dev, dtype=bf)
            dx1b = torch.full((N, H, W, Cin - split), nan, device=dev, dtype=bf)
            part = torch.full((tiles, 2 * Cin), nan, device=dev)
            L.call("pmu_conv3x3_dgrad_dma_x1b_sum_dxb", dzt.data_ptr(), Cp, N, H, W, wp.data_ptr(), Cin, split,
                   dx0.data_ptr(), dx1b.data_ptr(), part.data_ptr(), L.stream())
            return dx0, dx1b, part
        dtype = bf if kind == "bnr_dxb" else torch.float32
        dx = torch.full((N, H, W, Cin), nan, device=dev, dtype=dtype)
        part = torch.full((tiles, 2 * Cin), nan, device=dev)
        L.call("pmu_conv3x3_dgrad_dma_" + kind, dzt.data_ptr(), Cp, N, H, W, wp.data_ptr(), Cin, dx.data_ptr(),
               z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), L.stream())
        return dx, part

    p, o = _both(monkeypatch, run)
    for t in p:
        assert not torch.isnan(t.float()).any()
    _same(p, o)


def test_persistent_shape_rules(dev, exp_lib, monkeypatch):
    """odd chunk counts and grids under two workgroups per slot keep one tile per workgroup"""
    monkeypatch.setenv("PMU_DMA_PERS", "1")
    lib = exp_lib
    assert lib.pmu_conv3x3_dma_persistent(10, 256, 256, 64, 48) == 0   # 3 chunks
    assert lib.pmu_conv3x3_dma_persistent(1, 64, 64, 64, 64) == 0      # 8 tiles
    assert lib.pmu_conv3x3_dma_persistent(16, 512, 512, 64, 64) == 1   # c5's widest layer
