"""GPU parity of the drop-in blocks called on their own (reference module tree: DoubleConv, Down,
Up, OutConv — PMU/model/unet/unet_parts.py:9-76; Encoder — probabilistic_unet.py:11-53), the
reference's block-by-block UNet.forward composed from them, the AxisAlignedConvGaussian debug
attributes, and the batched latent-grid sampling (sample_at over a z grid, visualize_sampling.py).

Each block is compared with a torch-CPU restatement (the oracle's functional layers) on the same
inputs: outputs |d| <= 1e-3, input and parameter gradients max|dg|/max|g| <= 1e-3, BN running
statistics |d| <= 1e-3.
"""
import pytest
import torch
import torch.nn.functional as F

from helpers import ACT_TOL, GRAD_TOL, grad_err, max_abs

pytestmark = pytest.mark.gpu


def _ref_params(module):
    sd = {k: v.detach().cpu().clone() for k, v in module.state_dict().items()}
    names = [k for k, _ in module.named_parameters()]
    for k in names:
        sd[k] = sd[k].requires_grad_(True)
    return sd, names


def _compare(module, sd, names, out, ref, inputs, ref_inputs):
    assert out.shape == ref.shape
    assert max_abs(out, ref) <= ACT_TOL
    w = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3))
    (ref * w).sum().backward()
    (out * w.to(out.device)).sum().backward()
    named = dict(module.named_parameters())
    err, key = grad_err({k: named[k].grad for k in names}, {k: sd[k].grad for k in names})
    assert err <= GRAD_TOL, (err, key)
    for x, xr in zip(inputs, ref_inputs):
        if xr.grad is not None:
            err, _ = grad_err({"x": x.grad}, {"x": xr.grad})
            assert err <= GRAD_TOL, ("input grad", err)
    bufs = dict(module.named_buffers())
    for k, v in bufs.items():
        if "running" in k:
            assert max_abs(v, sd[k]) <= ACT_TOL, k


def _inputs(shape, seed, dev, grad=True):
    x = torch.randn(shape, generator=torch.Generator().manual_seed(seed))
    xr = x.clone().requires_grad_(grad)
    xd = x.to(dev).requires_grad_(grad)
    return xd, xr


@pytest.mark.parametrize("cin,cout,H,W,grad", [(3, 16, 20, 18, True), (16, 32, 17, 23, True), (1, 8, 16, 16, False)])
def test_double_conv_block(dev, cin, cout, H, W, grad):
    from model.unet.unet_parts import DoubleConv
    from oracle.unet_ref import double_conv
    torch.manual_seed(1)
    m = DoubleConv(cin, cout)
    sd, names = _ref_params(m)
    xd, xr = _inputs((2, cin, H, W), 2, dev, grad)
    ref = double_conv(xr, sd, "", True)
    m = m.to(dev).train()
    out = m(xd)
    _compare(m, sd, names, out, ref, [xd], [xr])


@pytest.mark.parametrize("H,W", [(20, 18), (21, 17)])
def test_down_block(dev, H, W):
    """MaxPool2d(2) on an arbitrary (signed) input, floor sizes, gradient to the first max."""
    from model.unet.unet_parts import Down
    from oracle.unet_ref import double_conv
    torch.manual_seed(1)
    m = Down(8, 16)
    sd, names = _ref_params(m)
    xd, xr = _inputs((2, 8, H, W), 4, dev)
    ref = double_conv(F.max_pool2d(xr, 2), sd, "maxpool_conv.1.", True)
    m = m.to(dev).train()
    out = m(xd)
    _compare(m, sd, names, out, ref, [xd], [xr])


@pytest.mark.parametrize("h,w,hs,ws", [(8, 6, 16, 12), (5, 7, 11, 15)])
def test_up_block(dev, h, w, hs, ws):
    """ConvTranspose2d -> F.pad to the skip (odd skip sizes: the pad branch) -> cat -> DoubleConv."""
    from model.unet.unet_parts import Up
    from oracle.unet_ref import double_conv
    torch.manual_seed(1)
    m = Up(32, 16, bilinear=False)
    sd, names = _ref_params(m)
    x1d, x1r = _inputs((2, 32, h, w), 5, dev)
    x2d, x2r = _inputs((2, 16, hs, ws), 6, dev)
    u = F.conv_transpose2d(x1r, sd["up.weight"], sd["up.bias"], stride=2)
    dY, dX = hs - u.shape[2], ws - u.shape[3]
    u = F.pad(u, [dX // 2, dX - dX // 2, dY // 2, dY - dY // 2])
    ref = double_conv(torch.cat([x2r, u], dim=1), sd, "conv.", True)
    m = m.to(dev).train()
    out = m(x1d, x2d)
    _compare(m, sd, names, out, ref, [x1d, x2d], [x1r, x2r])


def test_outconv_block(dev):
    from model.unet.unet_parts import OutConv
    torch.manual_seed(1)
    m = OutConv(16, 3)
    sd, names = _ref_params(m)
    xd, xr = _inputs((2, 16, 13, 11), 7, dev)
    ref = F.conv2d(xr, sd["conv.weight"], sd["conv.bias"])
    m = m.to(dev).train()
    out = m(xd)
    _compare(m, sd, names, out, ref, [xd], [xr])


def test_encoder_block(dev):
    """Encoder.forward of the posterior (2 input channels), odd sizes: AvgPool2d(2, ceil) windows."""
    from model.probabilistic_unet.probabilistic_unet import Encoder
    from oracle.probunet_ref import encoder_forward
    torch.manual_seed(1)
    m = Encoder(1, [8, 16, 32], 2, {"w": "he_normal", "b": "normal"}, posterior=True)
    sd, names = _ref_params(m)
    xd, xr = _inputs((2, 2, 21, 19), 8, dev)
    ref = encoder_forward(sd, "", xr, 3, True, 2)
    m = m.to(dev).train()
    out = m(xd)
    _compare(m, sd, names, out, ref, [xd], [xr])


def test_unet_composed_from_blocks_matches_fused_forward(dev):
    """The reference's UNet.forward written block by block (unet_model.py:31-54) on the drop-in
    blocks equals the fused one-node forward: outputs and every parameter gradient."""
    from model import UNet
    torch.manual_seed(0)
    net = UNet(1, 3, [8, 16, 32]).to(dev).train()
    x = torch.rand(2, 1, 36, 30, generator=torch.Generator().manual_seed(9)).to(dev)
    t = torch.randint(0, 3, (2, 36, 30), generator=torch.Generator().manual_seed(10)).to(dev)
    fused = net(x)
    F.cross_entropy(fused, t).backward()
    g_fused = {k: p.grad.clone() for k, p in net.named_parameters()}
    for p in net.parameters():
        p.grad = None
    xs = [net.inc(x)]
    for i in range(len(net.down_blocks)):
        xs.append(net.down_blocks[i](xs[i]))
    for i in range(len(net.up_blocks)):
        xs.append(net.up_blocks[i](xs[-1], xs[-(2 + i * 2)]))
    out = net.outc(xs[-1])
    assert max_abs(out, fused) <= ACT_TOL
    F.cross_entropy(out, t).backward()
    err, key = grad_err({k: p.grad for k, p in net.named_parameters()}, g_fused)
    assert err <= GRAD_TOL, (err, key)


def _probnet(dev):
    from model import ProbabilisticUnet
    torch.manual_seed(0)
    return ProbabilisticUnet(1, 3, [4, 8, 16], latent_dim=6, no_convs_fcomb=4, beta=10.0).to(dev)


def test_gaussian_debug_attributes(dev):
    """show_img / show_seg / show_concat / sum_input / show_enc of the posterior (:85-93)."""
    from oracle.probunet_ref import encoder_forward
    net = _probnet(dev).train()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(2, 1, 20, 20, generator=g)
    segm = torch.randint(0, 3, (2, 1, 20, 20), generator=g).float()
    sd = {k: v.detach().cpu() for k, v in net.posterior.state_dict().items()}
    enc_ref = encoder_forward(sd, "encoder.", torch.cat([x, segm], 1), 3, True)
    net.forward(x.to(dev), segm.to(dev), training=True)
    post = net.posterior
    assert torch.equal(post.show_concat.cpu(), torch.cat([x, segm], 1))
    assert abs(float(post.sum_input) - float(torch.cat([x, segm], 1).sum())) <= 1e-3
    assert max_abs(post.show_enc, enc_ref) <= ACT_TOL
    assert net.prior.show_concat == 0 and net.prior.sum_input == 0   # the prior never sees a mask


def test_sample_at_latent_grid(dev):
    """sample_at over a latent grid in one fused pass == the reference's per-point sample_at(z)
    loop (visualize_sampling.py:21-27) and the oracle's Fcomb at every grid point."""
    from model import ProbabilisticUnet
    from oracle.probunet_ref import fcomb_forward
    net = _probnet(dev).train()
    g = torch.Generator().manual_seed(4)
    x = torch.rand(1, 1, 24, 20, generator=g).to(dev)
    segm = torch.randint(0, 3, (1, 1, 24, 20), generator=g).float().to(dev)
    with torch.no_grad():
        net.forward(x, segm, training=False)
        mu = net.prior_latent_space.base_dist.loc.squeeze()
        sigma = net.prior_latent_space.base_dist.scale.squeeze() * 40.0
        z = ProbabilisticUnet.latent_grid(3, mu, sigma)
        assert z.shape == (9, 6)
        grid = net.sample_at(z)                                   # (9, 1, 3, H, W)
        loop = torch.stack([net.sample_at(z[i]) for i in range(9)])
    assert max_abs(grid, loop) <= 1e-5
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    feat = net.unet_features.detach().cpu()
    for i in range(9):
        ref = fcomb_forward(sd, feat, z[i:i + 1].cpu(), 4)
        assert max_abs(grid[i], ref) <= ACT_TOL
    # the grid order is the reference's: z_0 outer, z_1 inner, k in range(-(n//2), n//2 + 1)
    ks = [-1, 0, 1]
    for a in range(3):
        for b in range(3):
            want = mu.clone()
            want[0] = ks[a] * sigma[0] + mu[0]
            want[1] = ks[b] * sigma[1] + mu[1]
            assert torch.allclose(z[3 * a + b], want)
