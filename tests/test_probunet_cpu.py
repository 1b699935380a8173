"""CPU checks of the probabilistic path: oracle vs the reference's G3 golden vectors, the drop-in
module surface (state_dict keys/values, RNG order) and CPU refusal.  No GPU compute."""
import os

import numpy as np
import pytest
import torch

from helpers import grad_err, max_abs

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CFG = dict(n_levels=5, latent_dim=6, n_classes=3, n_convs_fcomb=4, beta=10.0)


def _g3():
    return np.load(os.path.join(GOLD, "g3_probunet.npz"), allow_pickle=False)


def _sd(z, prefix):
    pre = prefix + "/"
    return {k[len(pre):]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith(pre)}


@pytest.mark.parametrize("tag", ["s64", "s45"])
def test_oracle_matches_reference_g3_train(tag):
    """Posterior/prior mu and sigma, KL, CE-sum, ELBO, reconstruction logits, every gradient and
    the BN running statistics of one ProbabilisticUnet training step (probabilistic_unet.py:215-308)."""
    from oracle.probunet_ref import probunet_train_step
    z = _g3()
    sd = _sd(z, "init")
    x, segm = torch.from_numpy(z[f"{tag}/x"]), torch.from_numpy(z[f"{tag}/segm"])
    res, grads = probunet_train_step(sd, x, segm, torch.from_numpy(z[f"{tag}/eps_post"]), **CFG)
    for name, key in (("post_mu", "mu_q"), ("prior_mu", "mu_p")):
        assert max_abs(res[key], torch.from_numpy(z[f"{tag}/{name}"])) <= 1e-5, name
    for name, key in (("post_sigma", "ls_q"), ("prior_sigma", "ls_p")):
        assert max_abs(torch.exp(res[key]), torch.from_numpy(z[f"{tag}/{name}"])) <= 1e-5, name
    assert abs(float(res["kl"]) - float(z[f"{tag}/kl"])) <= 1e-4 * max(1.0, abs(float(z[f"{tag}/kl"])))
    assert abs(float(res["ce"]) - float(z[f"{tag}/ce"])) <= 1e-5 * abs(float(z[f"{tag}/ce"]))
    assert abs(float(res["elbo"]) - float(z[f"{tag}/elbo"])) <= 1e-5 * abs(float(z[f"{tag}/elbo"]))
    assert max_abs(res["rec"], torch.from_numpy(z[f"{tag}/rec"])) <= 1e-5
    assert max_abs(res["feat"], torch.from_numpy(z[f"{tag}/feat"])) <= 1e-5
    err, key = grad_err(grads, _sd(z, f"{tag}/grad"))
    assert err <= 1e-5, (err, key)
    for k, v in _sd(z, f"{tag}/after").items():
        assert max_abs(sd[k].float(), v.float()) <= 1e-5, k


@pytest.mark.parametrize("tag", ["s64", "s45"])
def test_oracle_matches_reference_g3_samples_and_eval(tag):
    """Fcomb on prior samples (sample(), :225-240) and the eval-mode pass (BN running stats,
    sample(testing=True))."""
    from oracle.probunet_ref import fcomb_forward, gaussian_forward, probunet_train_step
    from oracle.unet_ref import unet_forward
    z = _g3()
    sd = _sd(z, "init")
    x, segm = torch.from_numpy(z[f"{tag}/x"]), torch.from_numpy(z[f"{tag}/segm"])
    res, _ = probunet_train_step(sd, x, segm, torch.from_numpy(z[f"{tag}/eps_post"]), **CFG)
    eps_prior = torch.from_numpy(z[f"{tag}/eps_prior"])
    with torch.no_grad():
        sig_p = torch.exp(res["ls_p"])
        samples = torch.stack([fcomb_forward(sd, res["feat"], res["mu_p"] + sig_p * e, 4) for e in eps_prior])
        assert max_abs(samples, torch.from_numpy(z[f"{tag}/samples"])) <= 1e-5
        mu_p, ls_p = gaussian_forward(sd, "prior.", x, 5, 6, training=False)
        assert max_abs(mu_p, torch.from_numpy(z[f"{tag}/eval_prior_mu"])) <= 1e-5
        usd = {k[5:]: v for k, v in sd.items() if k.startswith("unet.")}
        feat = unet_forward(usd, x, 5, 3, apply_last_layer=False, training=False)
        y = fcomb_forward(sd, feat, mu_p + torch.exp(ls_p) * torch.from_numpy(z[f"{tag}/eps_eval"]), 4)
        assert max_abs(y, torch.from_numpy(z[f"{tag}/eval_sample"])) <= 1e-4


def test_probunet_state_dict_matches_reference():
    """Same module tree, key order and RNG consumption as the reference ctor: with the same seed
    the drop-in's initial state_dict equals the reference's (G3 'init')."""
    from model import ProbabilisticUnet
    z = _g3()
    ref = _sd(z, "init")
    torch.manual_seed(0)
    net = ProbabilisticUnet(input_channels=1, num_classes=3, num_filters=[4, 8, 16, 32, 64], latent_dim=6,
                            no_convs_fcomb=4, beta=10.0)
    sd = net.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k in sd:
        assert sd[k].shape == ref[k].shape, k
        assert torch.equal(sd[k].cpu(), ref[k]), k


def test_probunet_trainer_config_param_count():
    """ProbUNetTrainer's network (probunet_trainer.py:16): counts taken from the reference itself
    (68,780,702 total = unet 31,042,499 + prior 18,862,284 + posterior 18,862,860 + fcomb 13,059)."""
    from model import ProbabilisticUnet
    net = ProbabilisticUnet(input_channels=1, num_classes=3, num_filters=[64, 128, 256, 512, 1024], latent_dim=6,
                            no_convs_fcomb=4, beta=10)
    count = lambda m: sum(p.numel() for p in m.parameters())  # noqa: E731
    assert [count(m) for m in (net.unet, net.prior, net.posterior, net.fcomb)] == [31042499, 18862284, 18862860, 13059]
    assert count(net) == 68780702


def test_probunet_forward_refuses_cpu():
    from model import ProbabilisticUnet
    net = ProbabilisticUnet(1, 3, [4, 8], latent_dim=2, no_convs_fcomb=3)
    x = torch.rand(1, 1, 16, 16)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        net.forward(x, x, training=True)
