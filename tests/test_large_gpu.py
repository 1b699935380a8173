"""Operands of 4 GiB and more: the LDS-DMA Winograd kernels address their operand with 32-bit byte
offsets, so their launchers split such a launch over images (pmu_image_chunks in pmu_common.h)
instead of failing.  A 4.4 GB launch must equal the same kernels launched on two halves of the
batch (each below 4 GiB) bit for bit — outputs and BatchNorm partials."""
import pytest
import torch

pytestmark = pytest.mark.gpu

N, H, W, C = 520, 64, 64, 512          # N*H*W*C*4 = 4.36 GB >= 4 GiB
HALF = 256


@pytest.mark.timeout(300)
def test_wino2h_forward_over_4gib_splits_over_images(dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import pack_weights_wino2h
    assert N * H * W * C * 4 >= 1 << 32 and HALF * H * W * C * 4 < 1 << 32
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.rand(N, H, W, C, device=dev, generator=g)
    w = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.02
    b = torch.randn(C, device=dev, generator=g)
    wp = pack_weights_wino2h(w, dgrad=False)
    lb = L.lib()
    tiles = lb.pmu_conv3x3_tiles_wino2h(1, H, W)

    def run(xs):
        n = xs.shape[0]
        z = torch.empty(n, H, W, C, device=dev)
        part = torch.empty(n * tiles, 2 * C, device=dev)
        L.call("pmu_conv3x3_fwd_wino2h", xs.data_ptr(), C, n, H, W, wp.data_ptr(), b.data_ptr(), C, z.data_ptr(),
               part.data_ptr(), L.stream())
        return z, part
    z, part = run(x)
    z0, p0 = run(x[:HALF])
    torch.cuda.synchronize()
    assert torch.equal(z[:HALF], z0) and torch.equal(part[:HALF * tiles], p0)
    del z0, p0
    z1, p1 = run(x[HALF:])
    torch.cuda.synchronize()
    assert torch.equal(z[HALF:], z1) and torch.equal(part[HALF * tiles:], p1)


@pytest.mark.timeout(300)
def test_wino4_input_gradient_over_4gib_splits_over_images(dev):
    from pmu_hip import _lib as L
    from pmu_hip.engine import pack_weights_wino4
    g = torch.Generator(device=dev).manual_seed(4)
    dz = torch.randn(N, H, W, C, device=dev, generator=g)
    w = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.02
    wp = pack_weights_wino4(w, dgrad=True)
    sp = 320                                 # a concat split: two outputs

    def run(d):
        n = d.shape[0]
        dx0 = torch.empty(n, H, W, sp, device=dev)
        dx1 = torch.empty(n, H, W, C - sp, device=dev)
        L.call("pmu_conv3x3_dgrad_wino4", d.data_ptr(), C, n, H, W, wp.data_ptr(), C, sp, dx0.data_ptr(),
               dx1.data_ptr(), L.stream())
        return dx0, dx1
    a0, a1 = run(dz)
    b0, b1 = run(dz[:HALF])
    torch.cuda.synchronize()
    assert torch.equal(a0[:HALF], b0) and torch.equal(a1[:HALF], b1)
    del b0, b1
    c0, c1 = run(dz[HALF:])
    torch.cuda.synchronize()
    assert torch.equal(a0[HALF:], c0) and torch.equal(a1[HALF:], c1)
