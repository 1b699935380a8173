"""GPU parity: the HIP U-Net (model.UNet on cuda) vs the CPU oracle on the same seeded inputs.

Tolerances: outputs |d| <= 1e-3, loss rel <= 1e-3, gradients max|dg|/max|g| <= 1e-3,
BN running stats |d| <= 1e-3.
"""
import pytest
import torch

from helpers import ACT_TOL, GRAD_TOL, LOSS_RTOL, grad_err, max_abs

pytestmark = pytest.mark.gpu

# the one ill-conditioned geometry: full depth at 37x45 with N=2, BatchNorm over 8 values at the
# deepest level; accepted at 2x the fp32 reference's own error vs fp64
ILL_CONDITIONED = ([64, 128, 256, 512, 1024], 3, 2, 37, 45)
CASES = [
    # (num_filters, n_classes, N, H, W)
    ([16, 32], 1, 4, 64, 64),            # c1 geometry
    ([4, 8, 16, 32, 64], 3, 2, 64, 64),  # G2 geometry
    ([4, 8, 16, 32, 64], 3, 1, 170, 170),  # odd sizes: F.pad branch fires (170->85->42->21->10)
    ([64, 128, 256], 1, 2, 64, 64),      # vector fast paths
    ([64, 128, 256, 512, 1024], 1, 2, 64, 48),  # full c2 architecture, small batch, non-square
    ([64, 128, 256, 512, 1024], 3, 2, 37, 45),  # full depth, odd sizes, CE
    ([6, 12, 24], 3, 2, 40, 36),         # 6 channels (not a multiple of 4): scalar/generic paths
]


def _run(num_filters, n_classes, N, H, W, dev):
    from model import UNet
    from oracle.unet_ref import unet_forward, unet_loss, unet_param_keys

    torch.manual_seed(0)
    net = UNet(1, n_classes, num_filters)
    sd_cpu = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    x = torch.rand(N, 1, H, W, generator=g)
    if n_classes == 1:
        target = (torch.rand(N, 1, H, W, generator=g) > 0.5).float()
    else:
        target = torch.randint(0, n_classes, (N, 1, H, W), generator=g)

    # oracle (fp32 like the reference, plus fp64 to measure the reference's own noise floor)
    keys = unet_param_keys(sd_cpu)

    def oracle(dt):
        sd = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in sd_cpu.items()}
        params = {k: sd[k].clone().requires_grad_(True) for k in keys}
        work = dict(sd)
        work.update(params)
        o = unet_forward(work, x.to(dt), len(num_filters), n_classes)
        l_ = unet_loss(o, target.to(dt) if n_classes == 1 else target, n_classes)
        l_.backward()
        return o.detach(), l_.detach(), {k: params[k].grad for k in keys}, work

    out_ref, loss_ref, gref, work = oracle(torch.float32)
    _, _, g64, _ = oracle(torch.float64)
    global _NOISE
    _NOISE = (g64, grad_err(gref, g64)[0])

    # HIP
    net = net.to(dev).train()
    xd = x.to(dev)
    out = net(xd)
    tgt = target.to(dev).float() if n_classes == 1 else target.to(dev)
    loss = unet_loss(out, tgt, n_classes)
    loss.backward()
    torch.cuda.synchronize()
    named = dict(net.named_parameters())
    ggot = {k: named[k].grad for k in keys}
    sd_after = net.state_dict()
    return out, out_ref, loss, loss_ref, ggot, gref, sd_after, work


@pytest.mark.parametrize("num_filters,n_classes,N,H,W", CASES)
def test_unet_train_step_parity(num_filters, n_classes, N, H, W, dev):
    out, out_ref, loss, loss_ref, ggot, gref, sd_after, work = _run(num_filters, n_classes, N, H, W, dev)
    assert out.shape == out_ref.shape
    assert max_abs(out, out_ref) <= ACT_TOL
    assert abs(float(loss) - float(loss_ref)) <= LOSS_RTOL * abs(float(loss_ref))
    missing = [k for k, v in ggot.items() if v is None]
    assert not missing, f"no grad for {missing[:4]}"
    err, key = grad_err(ggot, gref)
    if err > GRAD_TOL and (num_filters, n_classes, N, H, W) == ILL_CONDITIONED:
        # accept if we are as close to the fp64 truth as the fp32 reference itself is (within 2x)
        g64, ref_noise = _NOISE
        err64, key64 = grad_err(ggot, g64)
        assert err64 <= max(GRAD_TOL, 2.0 * ref_noise), \
            f"grad error {err:.3e} at {key}; vs fp64 {err64:.3e} at {key64} (reference fp32 noise {ref_noise:.3e})"
    else:
        assert err <= GRAD_TOL, f"grad error {err:.3e} at {key}"
    for k, v in sd_after.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert max_abs(v, work[k]) <= ACT_TOL, k
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(work[k]), k


def test_unet_eval_mode_parity(dev):
    from model import UNet
    from oracle.unet_ref import unet_forward

    torch.manual_seed(0)
    net = UNet(1, 3, [8, 16, 32])
    # non-trivial running stats
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    x = torch.rand(3, 1, 40, 40, generator=torch.Generator().manual_seed(3))
    ref = unet_forward(sd, x, 3, 3, training=False)
    net = net.to(dev).eval()
    with torch.no_grad():
        out = net(x.to(dev))
    assert max_abs(out, ref) <= ACT_TOL
    assert torch.equal(out.argmax(1).cpu(), ref.argmax(1))


def test_unet_features_mode(dev):
    """apply_last_layer=False returns the last DoubleConv activation (unet_model.py:51-54)."""
    from model import UNet
    from oracle.unet_ref import unet_forward, unet_param_keys

    torch.manual_seed(0)
    net = UNet(1, 3, [8, 16], apply_last_layer=False)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    x = torch.rand(2, 1, 32, 32, generator=torch.Generator().manual_seed(5))
    keys = unet_param_keys(sd)
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    ref = unet_forward(work, x, 2, 3, apply_last_layer=False)
    wgt = torch.rand_like(ref)
    (ref * wgt).sum().backward()
    net = net.to(dev).train()
    out = net(x.to(dev))
    assert out.shape == ref.shape
    assert max_abs(out, ref) <= ACT_TOL
    (out * wgt.to(dev)).sum().backward()
    named = dict(net.named_parameters())
    gref = {k: params[k].grad for k in keys if params[k].grad is not None}
    ggot = {k: named[k].grad for k in gref}
    err, key = grad_err(ggot, gref)
    assert err <= GRAD_TOL, f"{err} {key}"
    assert named["outc.conv.weight"].grad is None


def test_unet_applied_twice_in_one_graph(dev):
    """loss(net(x1)) + loss(net(x2)): both HIP nodes' gradients must add (g1 + g2), as the reference's
    per-op autograd graph does — the flat-buffer views must not alias across the two nodes."""
    from model import UNet
    from oracle.unet_ref import unet_forward, unet_loss, unet_param_keys
    torch.manual_seed(0)
    net = UNet(1, 3, [8, 16, 32])
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(9)
    x1, x2 = torch.rand(2, 1, 32, 32, generator=g), torch.rand(3, 1, 32, 32, generator=g)
    t1, t2 = torch.randint(0, 3, (2, 1, 32, 32), generator=g), torch.randint(0, 3, (3, 1, 32, 32), generator=g)
    keys = unet_param_keys(sd)
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    (unet_loss(unet_forward(work, x1, 3, 3), t1, 3) + 0.5 * unet_loss(unet_forward(work, x2, 3, 3), t2, 3)).backward()
    net = net.to(dev).train()
    loss = unet_loss(net(x1.to(dev)), t1.to(dev), 3) + 0.5 * unet_loss(net(x2.to(dev)), t2.to(dev), 3)
    loss.backward()
    named = dict(net.named_parameters())
    err, key = grad_err({k: named[k].grad for k in keys}, {k: params[k].grad for k in keys})
    assert err <= GRAD_TOL, (err, key)
    # a following single application goes back to the flat gradient buffer
    for p in net.parameters():
        p.grad = None
    unet_loss(net(x1.to(dev)), t1.to(dev), 3).backward()
    buf = net.__dict__["_pmu_grad_flat"]
    lo, hi = buf.data_ptr(), buf.data_ptr() + 4 * buf.numel()
    assert all(lo <= p.grad.data_ptr() < hi for p in net.parameters())


def test_bn_cumulative_average_momentum_none(dev):
    """nn.BatchNorm2d(momentum=None) keeps a cumulative average of the batch statistics: two training
    forwards of the same batch leave running_mean / running_var at that batch's statistics — what
    momentum=1.0 gives after one — and num_batches_tracked at 2 (the engine's host-side path; the
    default momentum's counter is advanced by the finalize kernel, test_unet_train_step_parity)."""
    from model import UNet
    torch.manual_seed(0)
    x = torch.rand(2, 1, 48, 40, generator=torch.Generator().manual_seed(5)).to(dev)
    stats = []
    for mom, passes in ((None, 2), (1.0, 1)):
        torch.manual_seed(0)
        net = UNet(1, 1, [8, 16, 32]).to(dev).train()
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.momentum = mom
        with torch.no_grad():
            for _ in range(passes):
                net(x)
        torch.cuda.synchronize()
        stats.append({k: v.detach().clone() for k, v in net.state_dict().items()})
    cum, one = stats
    n = 0
    for k, v in cum.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert max_abs(v, one[k]) <= 1e-5 * max(1.0, float(one[k].abs().max())), k
            n += 1
        if k.endswith("num_batches_tracked"):
            assert int(v) == 2 and int(one[k]) == 1, k
    assert n >= 8
