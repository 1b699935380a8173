"""GPU parity of the probabilistic path (rows a9-a12): the HIP ProbabilisticUnet vs the reference's
own G3 golden vectors (tests/golden/g3_probunet.npz, produced by importing the reference) and vs
the CPU oracle on larger seeded cases.

Tolerances: outputs |d| <= 1e-3, losses rel <= 1e-3, gradients max|dg|/max|g| <= 1e-3,
BN running stats |d| <= 1e-3.  Latent noise is injected (mu + sigma * eps), which is exactly what
Normal.rsample computes, so the comparison is deterministic.
"""
import os

import numpy as np
import pytest
import torch

from helpers import ACT_TOL, GRAD_TOL, LOSS_RTOL, grad_err, max_abs

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _g3():
    return np.load(os.path.join(GOLD, "g3_probunet.npz"), allow_pickle=False)


def _sd(z, prefix):
    pre = prefix + "/"
    return {k[len(pre):]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith(pre)}


def _inject(dist, eps, method):
    def draw(sample_shape=torch.Size()):
        v = dist.base_dist.loc + dist.base_dist.scale * eps
        return v if method == "rsample" else v.detach()
    setattr(dist, method, draw)


def _net(dev, num_filters=(4, 8, 16, 32, 64), n_classes=3, seed=0, init=None):
    """The G3 network.  With ``init`` the reference's initial weights are loaded: the orthogonal
    Fcomb init goes through LAPACK QR, whose last bits depend on the host CPU (bit-equality of the
    seeded init is checked in the build container, tests/test_probunet_cpu.py)."""
    from model import ProbabilisticUnet
    torch.manual_seed(seed)
    net = ProbabilisticUnet(input_channels=1, num_classes=n_classes, num_filters=list(num_filters), latent_dim=6,
                            no_convs_fcomb=4, beta=10.0)
    if init is not None:
        net.load_state_dict(_sd(init, "init"))
    return net.to(dev)


@pytest.mark.parametrize("tag", ["s64", "s45"])
def test_probunet_train_step_matches_reference_g3(tag, dev):
    z = _g3()
    net = _net(dev, init=z).train()
    x = torch.from_numpy(z[f"{tag}/x"]).to(dev)
    segm = torch.from_numpy(z[f"{tag}/segm"]).to(dev)
    eps = torch.from_numpy(z[f"{tag}/eps_post"]).to(dev)
    net.forward(x, segm, training=True)
    _inject(net.posterior_latent_space, eps, "rsample")
    elbo = net.elbo(segm)
    (-elbo).backward()
    torch.cuda.synchronize()
    for name, d in (("post", net.posterior_latent_space), ("prior", net.prior_latent_space)):
        assert max_abs(d.base_dist.loc, torch.from_numpy(z[f"{tag}/{name}_mu"])) <= ACT_TOL, name
        assert max_abs(d.base_dist.scale, torch.from_numpy(z[f"{tag}/{name}_sigma"])) <= ACT_TOL, name
    assert max_abs(net.unet_features, torch.from_numpy(z[f"{tag}/feat"])) <= ACT_TOL
    assert max_abs(net.reconstruction, torch.from_numpy(z[f"{tag}/rec"])) <= ACT_TOL
    for q, ref in (("kl", net.kl), ("ce", net.reconstruction_loss), ("elbo", elbo)):
        r = float(z[f"{tag}/{q}"])
        assert abs(float(ref) - r) <= LOSS_RTOL * max(1.0, abs(r)), (q, float(ref), r)
    named = dict(net.named_parameters())
    gref = _sd(z, f"{tag}/grad")
    missing = [k for k in gref if named[k].grad is None]
    assert not missing, missing[:4]
    err, key = grad_err({k: named[k].grad for k in gref}, gref)
    assert err <= GRAD_TOL, (err, key)
    # the discarded unet.outc gets no gradient, as in the reference
    assert set(gref) == {k for k, p in named.items() if p.grad is not None}
    bufs = dict(net.named_buffers())
    for k, v in _sd(z, f"{tag}/after").items():
        assert max_abs(bufs[k].float(), v.float()) <= ACT_TOL, k


@pytest.mark.parametrize("tag", ["s64", "s45"])
def test_probunet_samples_and_eval_match_reference_g3(tag, dev):
    z = _g3()
    net = _net(dev, init=z).train()
    x = torch.from_numpy(z[f"{tag}/x"]).to(dev)
    segm = torch.from_numpy(z[f"{tag}/segm"]).to(dev)
    net.forward(x, segm, training=True)
    eps_prior = torch.from_numpy(z[f"{tag}/eps_prior"]).to(dev)
    ref = torch.from_numpy(z[f"{tag}/samples"])
    with torch.no_grad():
        d = net.prior_latent_space
        zs = d.base_dist.loc + d.base_dist.scale * eps_prior           # (S, N, L)
        one = torch.stack([net.fcomb.forward(net.unet_features, zs[s]) for s in range(zs.shape[0])])
        many = net.fcomb.forward_samples(net.unet_features, zs)      # fused S-sample pass
    assert max_abs(one, ref) <= ACT_TOL
    assert max_abs(many, ref) <= ACT_TOL
    # eval mode: BN running statistics, sample(testing=True)
    with torch.no_grad():
        net.eval()
        net.forward(x, segm, training=False)
        _inject(net.prior_latent_space, torch.from_numpy(z[f"{tag}/eps_eval"]).to(dev), "sample")
        y = net.sample(testing=True)
    assert max_abs(net.prior_latent_space.base_dist.loc, torch.from_numpy(z[f"{tag}/eval_prior_mu"])) <= ACT_TOL
    assert max_abs(y, torch.from_numpy(z[f"{tag}/eval_sample"])) <= ACT_TOL


@pytest.mark.parametrize("N,H,W,F,K,NH,quant", [(2, 64, 64, 64, 3, 3, 0), (3, 45, 37, 64, 3, 3, 0),
                                                (1, 20, 13, 32, 1, 2, 0), (2, 16, 16, 8, 5, 1, 0),
                                                (2, 24, 20, 30, 2, 2, 0), (6, 5, 3, 16, 2, 1, 0),
                                                (8, 128, 100, 64, 3, 3, 1)])
def test_fcomb_fwd_bwd_vs_fp64_oracle(N, H, W, F, K, NH, quant, dev):
    """Fcomb alone at trainer width (F=64, 3 hidden layers) and at other legal shapes, including
    pixel counts that are not tile multiples, images smaller than one 32-pixel group (6x5x3) and a
    batch where each wave of the backward walks several groups across image boundaries (8x128x100);
    forward and every gradient vs float64 torch.

    At 10^5 pixels x 192 hidden units a few pre-activations land within fp32 rounding of zero, where
    fp32 and fp64 legitimately disagree on the ReLU mask; the large case therefore quantises weights,
    biases, features and z to short dyadic grids (steps 1/8, 1/16, 1/4) on which the whole hidden
    chain is exact in fp32, so the masks are identical and the comparison stays tight."""
    from model.probabilistic_unet.probabilistic_unet import Fcomb
    torch.manual_seed(5)
    fc = Fcomb([F], 6, 1, K, NH + 1, {"w": "orthogonal", "b": "normal"}).to(dev)
    with torch.no_grad():
        for p in fc.parameters():
            if p.dim() == 1:
                p.normal_(0, 0.1)
            if quant:
                p.copy_((p * 8).round().clamp(-2, 2) / 8 if p.dim() > 1 else (p * 16).round() / 16)
    g = torch.Generator().manual_seed(6)
    feat = torch.relu(torch.randn(N, F, H, W, generator=g))
    zl = torch.randn(N, 6, generator=g)
    if quant:
        feat = (feat * 4).round().clamp(0, 4) / 4
        zl = (zl * 4).round().clamp(-8, 8) / 4
    feat = feat.to(dev).contiguous(memory_format=torch.channels_last)
    zl = zl.to(dev)
    feat.requires_grad_(True)
    zl.requires_grad_(True)
    y = fc.forward(feat, zl)
    dy = torch.randn(y.shape, generator=g).to(dev)
    (y * dy).sum().backward()
    torch.cuda.synchronize()
    # float64 reference on the CPU with autograd
    from oracle.probunet_ref import fcomb_forward
    sd = {"fcomb." + k: v.detach().cpu().double().requires_grad_(True) for k, v in fc.state_dict().items()}
    f64 = feat.detach().cpu().double().requires_grad_(True)
    z64 = zl.detach().cpu().double().requires_grad_(True)
    yr = fcomb_forward(sd, f64, z64, NH + 1)
    (yr * dy.cpu().double()).sum().backward()
    assert max_abs(y, yr) <= 1e-4 * max(1.0, float(yr.abs().max()))
    assert max_abs(feat.grad, f64.grad) <= 1e-4 * max(1.0, float(f64.grad.abs().max()))
    assert max_abs(zl.grad, z64.grad) <= 1e-4 * max(1.0, float(z64.grad.abs().max()))
    got = {k: p.grad for k, p in fc.named_parameters()}
    ref = {k[6:]: v.grad for k, v in sd.items()}
    err, key = grad_err(got, ref)
    assert err <= 1e-4, (err, key)


def test_probunet_full_width_vs_oracle(dev):
    """ProbUNetTrainer architecture ([64..1024], 3 classes, no_convs_fcomb=4, beta=10) at 64x48, N=2:
    loss and all 68.78M gradients vs the fp32 CPU oracle."""
    from oracle.probunet_ref import probunet_param_keys, probunet_train_step
    torch.manual_seed(0)
    net = _net(dev, num_filters=(64, 128, 256, 512, 1024)).train()
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(7)
    N, H, W = 2, 64, 48
    x = torch.rand(N, 1, H, W, generator=g)
    segm = torch.randint(0, 3, (N, 1, H, W), generator=g).float()
    eps = torch.randn(N, 6, generator=g)
    res, gref = probunet_train_step(sd, x, segm, eps, 5, 6, 3, 4, 10.0)
    net.forward(x.to(dev), segm.to(dev), training=True)
    _inject(net.posterior_latent_space, eps.to(dev), "rsample")
    elbo = net.elbo(segm.to(dev))
    (-elbo).backward()
    torch.cuda.synchronize()
    assert abs(float(-elbo) - float(res["loss"])) <= LOSS_RTOL * abs(float(res["loss"]))
    assert max_abs(net.reconstruction, res["rec"]) <= ACT_TOL     # measured 2.5e-6 (tools/parity_diag.py)
    named = dict(net.named_parameters())
    keys = [k for k in probunet_param_keys(sd) if not k.startswith("unet.outc")]
    err, key = grad_err({k: named[k].grad for k in keys}, {k: gref[k] for k in keys})
    assert err <= GRAD_TOL, (err, key)                            # measured 1.5e-4


@pytest.mark.timeout(900)
def test_probunet_c4_geometry_vs_oracle(dev):
    """Config c4 exactly as bench.py --workload probunet runs it (ProbUNetTrainer architecture,
    256x256, 3 classes, batch 32): the train step's loss, reconstruction and every gradient vs the
    fp32 CPU oracle, then the evaluation sweep — 16 prior samples through the fused Fcomb pass
    (sample_many) and the per-class Dice counts of each (PU/probabilistic_unet.py:225-240,281-308,
    PMU/dice_loss.py:5-12) — vs the oracle's Fcomb and Dice.  The grid sizes, split-K slab counts
    and Fcomb group ranges of the benchmarked shapes, at the parity contract's tolerances (measured
    by tools/parity_diag.py: reconstruction 3.1e-6, gradients 2.4e-5, samples 5.0e-6, Dice 1.6e-6)."""
    from oracle.probunet_ref import fcomb_forward, probunet_param_keys, probunet_train_step
    from oracle.unet_ref import trainer_dice
    from pmu_hip.metrics import dice_counts, dice_from_counts
    torch.manual_seed(0)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    net = _net(dev, num_filters=(64, 128, 256, 512, 1024)).train()
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(11)
    N, H, W, S = 32, 256, 256, 16
    x = torch.rand(N, 1, H, W, generator=g)
    segm = torch.randint(0, 3, (N, 1, H, W), generator=g).float()
    eps = torch.randn(N, 6, generator=g)
    eps_prior = torch.randn(S, N, 6, generator=g)
    res, gref = probunet_train_step(sd, x, segm, eps, 5, 6, 3, 4, 10.0)
    net.forward(x.to(dev), segm.to(dev), training=True)
    _inject(net.posterior_latent_space, eps.to(dev), "rsample")
    elbo = net.elbo(segm.to(dev))
    (-elbo).backward()
    torch.cuda.synchronize()
    assert abs(float(-elbo) - float(res["loss"])) <= LOSS_RTOL * abs(float(res["loss"]))
    assert max_abs(net.reconstruction, res["rec"]) <= ACT_TOL
    named = dict(net.named_parameters())
    keys = [k for k in probunet_param_keys(sd) if not k.startswith("unet.outc")]
    err, key = grad_err({k: named[k].grad for k in keys}, {k: gref[k] for k in keys})
    assert err <= GRAD_TOL, (err, key)
    # the evaluation sweep of the c4 step
    d = net.prior_latent_space
    assert max_abs(d.base_dist.loc, res["mu_p"]) <= ACT_TOL
    ep = eps_prior.to(dev)
    d.sample = lambda shape=torch.Size(): d.base_dist.loc + d.base_dist.scale * ep
    with torch.no_grad():
        ys = net.sample_many(S)                                       # (S, N, 3, H, W)
    assert tuple(ys.shape) == (S, N, 3, H, W)
    zs = res["mu_p"][None] + torch.exp(res["ls_p"])[None] * eps_prior
    fsd = {k: v for k, v in sd.items() if k.startswith("fcomb.")}
    for s in range(S):
        yr = fcomb_forward(fsd, res["feat"], zs[s], 4)
        assert max_abs(ys[s], yr) <= ACT_TOL, s
        # argmax label map bit-exact away from fp32 ties: flips only where the oracle's top-2 margin < 1e-5
        top = yr.topk(2, dim=1).values
        flip = ys[s].argmax(1).cpu() != yr.argmax(1)
        assert not bool((flip & ((top[:, 0] - top[:, 1]) >= 1e-5)).any()), (s, int(flip.sum()))
        got = dice_from_counts(dice_counts(ys[s], segm.to(dev), 3)).cpu()[1:].tolist()
        want = trainer_dice(yr, segm, 3)
        assert max(abs(a - b) for a, b in zip(got, want)) <= 1e-3, (s, got, want)


def test_probunet_flat_grad_buffer(dev):
    """All gradients of one backward land in the model's single flat buffer (one all-reduce)."""
    from pmu_hip.functions import flat_grad_buffer
    net = _net(dev).train()
    x = torch.rand(2, 1, 32, 32, device=dev)
    segm = torch.randint(0, 3, (2, 1, 32, 32), device=dev).float()
    net.forward(x, segm, training=True)
    # the trainer's step: a prior sample (masks_pred, with grad) stays alive while -elbo backpropagates,
    # so a second Fcomb node is pending but never reached: Fcomb still gets the flat-buffer views
    masks_pred = net.sample(testing=False)
    loss = -net.elbo(segm)
    assert net.fcomb.__dict__["_pmu_live"] == 2
    loss.backward()
    buf = flat_grad_buffer(net)
    lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * 4
    seen = 0
    for k, p in net.named_parameters():
        if p.grad is not None:
            assert lo <= p.grad.data_ptr() < hi, k
            seen += k.startswith("fcomb.")
    assert seen == len(list(net.fcomb.parameters()))
    del masks_pred


def test_probunet_odd_filters_vs_oracle(dev):
    """num_filters not multiples of 4 (any count is legal in the reference): every generic/scalar
    path of the encoders, U-Net and Fcomb at once, vs the fp32 CPU oracle."""
    from oracle.probunet_ref import probunet_train_step
    from model import ProbabilisticUnet
    torch.manual_seed(0)
    net = ProbabilisticUnet(1, 3, [6, 12, 24], latent_dim=5, no_convs_fcomb=3, beta=10.0).to(dev).train()
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(9)
    N, H, W = 2, 33, 29
    x = torch.rand(N, 1, H, W, generator=g)
    segm = torch.randint(0, 3, (N, 1, H, W), generator=g).float()
    eps = torch.randn(N, 5, generator=g)
    res, gref = probunet_train_step(sd, x, segm, eps, 3, 5, 3, 3, 10.0)
    net.forward(x.to(dev), segm.to(dev), training=True)
    _inject(net.posterior_latent_space, eps.to(dev), "rsample")
    elbo = net.elbo(segm.to(dev))
    (-elbo).backward()
    torch.cuda.synchronize()
    assert abs(float(-elbo) - float(res["loss"])) <= LOSS_RTOL * abs(float(res["loss"]))
    assert max_abs(net.reconstruction, res["rec"]) <= ACT_TOL
    named = dict(net.named_parameters())
    keys = [k for k in gref if not k.startswith("unet.outc")]
    err, key = grad_err({k: named[k].grad for k in keys}, {k: gref[k] for k in keys})
    assert err <= GRAD_TOL, (err, key)


def test_fcomb_applied_twice_in_one_graph(dev):
    """Fcomb on two latent samples in one loss (sample() + reconstruct() both with grad): the
    parameter gradients add, as in the reference (probabilistic_unet.py:167-181)."""
    from oracle.probunet_ref import fcomb_forward
    net = _net(dev).train()
    fc = net.fcomb
    g = torch.Generator().manual_seed(4)
    feat = torch.randn(2, 4, 12, 10, generator=g)
    z1, z2 = torch.randn(2, 6, generator=g), torch.randn(2, 6, generator=g)
    w = torch.randn(2, 3, 12, 10, generator=g)
    sd = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in fc.state_dict().items()}
    ref_sd = {"fcomb." + k: v for k, v in sd.items()}
    (((fcomb_forward(ref_sd, feat, z1, 4) * w).sum()) + 2.0 * (fcomb_forward(ref_sd, feat, z2, 4) * w).sum()).backward()
    fd = feat.to(dev)
    wd = w.to(dev)
    ((fc(fd, z1.to(dev)) * wd).sum() + 2.0 * (fc(fd, z2.to(dev)) * wd).sum()).backward()
    named = dict(fc.named_parameters())
    err, key = grad_err({k: named[k].grad for k in sd}, {k: sd[k].grad for k in sd})
    assert err <= GRAD_TOL, (err, key)


def test_probunet_concurrent_streams_bit_identical(dev):
    """ProbabilisticUnet.forward runs the UNet, prior and posterior on three HIP streams (engine CFG
    .prob_streams, functions.run_concurrent), their backwards on the same streams: 3 training steps
    (forward, injected posterior sample, -elbo, backward, clip+SGD, then the 16-sample sweep) at the c4
    filters, 256x256, batch 8, give bit-identical losses, parameters, BN statistics and samples with the
    streams on and off — the parts are independent and every kernel's summation order is fixed."""
    from pmu_hip import engine
    from pmu_hip.optim import FusedSGD
    g = torch.Generator().manual_seed(3)
    N, S = 8, 256
    x = torch.rand(N, 1, S, S, generator=g).to(dev)
    segm = torch.randint(0, 3, (N, 1, S, S), generator=g).float().to(dev)
    eps = [torch.randn(N, 6, generator=g).to(dev) for _ in range(3)]
    eps_prior = torch.randn(16, N, 6, generator=g).to(dev)
    runs = []
    prev = engine.CFG.prob_streams
    try:
        for on in (False, True):
            engine.CFG.prob_streams = on
            net = _net(dev, num_filters=(64, 128, 256, 512, 1024)).train()
            opt = FusedSGD(net.parameters(), lr=1e-3, momentum=0.9, clip=0.1)
            losses = []
            for k in range(3):
                opt.zero_grad()
                net.forward(x, segm, training=True)
                _inject(net.posterior_latent_space, eps[k], "rsample")
                loss = -net.elbo(segm)
                loss.backward()
                opt.step()
                losses.append(float(loss))
            d = net.prior_latent_space
            d.sample = lambda shape=torch.Size(): d.base_dist.loc + d.base_dist.scale * eps_prior
            with torch.no_grad():
                ys = net.sample_many(16)
            torch.cuda.synchronize()
            runs.append((losses, {k: v.detach().clone() for k, v in net.state_dict().items()}, ys.clone()))
    finally:
        engine.CFG.prob_streams = prev
    (l0, sd0, y0), (l1, sd1, y1) = runs
    assert l0 == l1, (l0, l1)
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k
    assert torch.equal(y0, y1)
