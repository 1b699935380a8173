"""First 3x3 layer (Cin <= 4 input planes; unet_parts.py:15 on the image, probabilistic_unet.py:38,88):
pmu_conv_first_fwd and pmu_conv_first_wgrad (its tiled BN-backward fast path) against fp64 torch on
ragged maps (tiles cut by the image edge), vs the same products summed in fp64."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda")


def _planes(N, Cin, H, W, g, dev):
    x = torch.randn(N, Cin, H, W, generator=g)
    return x, [x[:, c].contiguous().to(dev) for c in range(Cin)]


@pytest.mark.parametrize("xb", [False, True])
@pytest.mark.parametrize("N,Cin,H,W,Cout", [(2, 3, 37, 45, 64), (1, 1, 16, 64, 32), (3, 4, 9, 70, 16)])
def test_conv_first_wgrad_bnbwd(dev, N, Cin, H, W, Cout, xb):
    """xb: da stored as bf16 (the c5 path: the second conv's *_dxb input gradient), the reference on the
    same bf16-rounded values."""
    import ctypes
    from pmu_hip import _lib as L
    from pmu_hip.engine import Src, frame_of
    g = torch.Generator().manual_seed(H * 7 + Cin)
    x, planes = _planes(N, Cin, H, W, g, dev)
    da = torch.randn(N, H, W, Cout, generator=g)
    if xb:
        da = da.to(torch.bfloat16).float()
    z = torch.randn(N, H, W, Cout, generator=g)
    coef = torch.cat([torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g) * 0.3,
                      torch.randn(Cout, generator=g) * 0.1, torch.randn(Cout, generator=g) * 0.1,
                      torch.randn(Cout, generator=g) * 0.1])
    sc, sh, mu, kx, kc = [t.double() for t in coef.view(5, Cout)]
    dz = sc * torch.where(z.double() * sc + sh > 0, da.double(), 0) + (kx * (z.double() - mu) + kc)
    ref = torch.nn.grad.conv2d_weight(x.double(), (Cout, Cin, 3, 3), dz.permute(0, 3, 1, 2), padding=1)
    wsb = L.lib().pmu_conv_first_wgrad_ws(N, H, W, Cin, Cout)
    ws = torch.empty(wsb // 4 + 1, device=dev)
    dw = torch.empty(Cout, Cin, 3, 3, device=dev)
    arr = (ctypes.c_void_p * Cin)(*[p.data_ptr() for p in planes])
    dax = da.to(torch.bfloat16).view(torch.int16).to(dev) if xb else da.to(dev)
    src = Src(dax, L.SRC_BNBWD, coef.to(dev), z=z.to(dev))   # (kept alive over the call)
    f = frame_of([src], N, H, W)
    L.call("pmu_conv_first_wgrad", f, arr, Cin, Cout, dw.data_ptr(), ws.data_ptr(), wsb, L.stream())
    torch.cuda.synchronize()
    err = (dw.double().cpu() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("N,Cin,H,W,Cout", [(2, 3, 37, 45, 64), (1, 1, 16, 64, 32), (3, 4, 9, 70, 16),
                                             (2, 4, 40, 33, 64), (1, 2, 24, 40, 64)])
def test_conv_first_fwd(dev, N, Cin, H, W, Cout):
    import ctypes
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(H * 5 + Cin)
    x, planes = _planes(N, Cin, H, W, g, dev)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.2
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    z = torch.empty(N, H, W, Cout, device=dev)
    R = L.lib().pmu_conv_first_tiles(N, H, W)
    part = torch.empty(R, 2 * Cout, device=dev)
    arr = (ctypes.c_void_p * Cin)(*[p.data_ptr() for p in planes])
    wd, bd = w.to(dev), b.to(dev)
    L.call("pmu_conv_first_fwd", arr, Cin, N, H, W, wd.data_ptr(), bd.data_ptr(), Cout, z.data_ptr(),
           part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert (z.double().cpu() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    s = part.double().cpu().view(R, 2, Cout).sum(0)
    zz = ref.reshape(-1, Cout)
    assert (s[0] - zz.sum(0)).abs().max().item() <= 1e-5 * zz.abs().sum(0).max().item()
    assert (s[1] - (zz * zz).sum(0)).abs().max().item() <= 1e-5 * (zz * zz).sum(0).max().item()
