"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

Runs only in the build container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box).  The reference is imported unmodified
with in-process shims for the pieces that do not import on this image:
  - builtins torch/nn/np (probabilistic_unet.py:4-9 uses them without importing),
  - stub modules utils.dataset (absent file), nibabel (not installed; serves in-memory
    arrays), torch.utils.tensorboard (not installed).
Outputs are data only (.npz): inputs, weights, and the reference's outputs/gradients.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import builtins
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference/Probabilistic-Multiplanar-Unet"
OUT = os.path.dirname(os.path.abspath(__file__))


def install_shims():
    builtins.torch, builtins.nn, builtins.np = torch, nn, np
    ud = types.ModuleType("utils.dataset")
    ud.BasicDataset = object
    sys.modules["utils.dataset"] = ud
    nib = types.ModuleType("nibabel")
    nib.store = {}

    class _Img:
        def __init__(self, a):
            self.a = a

        def get_fdata(self):
            return self.a

    nib.load = lambda p: _Img(nib.store[os.path.basename(p)])
    sys.modules["nibabel"] = nib
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, n):
            return lambda *a, **k: None

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    sys.path.insert(0, REF)
    return nib


def sd_np(prefix, sd):
    return {f"{prefix}/{k}": v.detach().cpu().numpy().copy() for k, v in sd.items()}


def grads_np(prefix, module):
    return {f"{prefix}/{k}": p.grad.detach().cpu().numpy().copy() for k, p in module.named_parameters()
            if p.grad is not None}


def g1_unet_c1():
    """Config c1: UNet(1,1,[16,32]), 64x64, batch 4, BCE; one step + 10 SGD steps (train.py:85-110)."""
    from model import UNet
    torch.manual_seed(0)
    net = UNet(1, 1, [16, 32])
    out = sd_np("init", net.state_dict())
    g = torch.Generator().manual_seed(1)
    xs = [torch.rand(4, 1, 64, 64, generator=g) for _ in range(10)]
    ts = [(torch.rand(4, 1, 64, 64, generator=g) > 0.5).float() for _ in range(10)]
    for i in range(10):
        out[f"x{i}"] = xs[i].numpy()
        out[f"t{i}"] = ts[i].numpy()
    net.train()
    crit = nn.BCELoss()
    opt = torch.optim.SGD(net.parameters(), lr=1e-3, momentum=0.9)
    losses = []
    for i in range(10):
        opt.zero_grad()
        y = net(xs[i])
        loss = crit(y, ts[i])
        loss.backward()
        if i == 0:
            out["y0"] = y.detach().numpy()
            out["loss0"] = np.array(loss.item(), dtype=np.float32)
            out.update(grads_np("grad0", net))
            out.update(sd_np("after0", net.state_dict()))
        nn.utils.clip_grad_value_(net.parameters(), 0.1)
        opt.step()
        losses.append(loss.item())
    out["losses"] = np.array(losses, dtype=np.float32)
    out.update(sd_np("final", net.state_dict()))
    np.savez_compressed(os.path.join(OUT, "g1_unet_c1.npz"), **out)


def g2_unet_multiclass():
    """All 5 levels at small width: UNet(1,3,[4,8,16,32,64]) at 64x64 (N=2) and 170x170 (N=1,
    F.pad branch at 21 and 85), CrossEntropyLoss (unet_trainer.py:23,30-37)."""
    from model import UNet
    out = {}
    for tag, (N, H) in {"s64": (2, 64), "s170": (1, 170)}.items():
        torch.manual_seed(0)
        net = UNet(1, 3, [4, 8, 16, 32, 64])
        out.update(sd_np(f"{tag}/init", net.state_dict()))
        g = torch.Generator().manual_seed(2)
        x = torch.rand(N, 1, H, H, generator=g)
        t = torch.randint(0, 3, (N, 1, H, H), generator=g)
        net.train()
        y = net(x)
        loss = nn.CrossEntropyLoss()(y, t.squeeze(1))
        loss.backward()
        out[f"{tag}/x"] = x.numpy()
        out[f"{tag}/t"] = t.numpy().astype(np.int64)
        out[f"{tag}/y"] = y.detach().numpy()
        out[f"{tag}/argmax"] = torch.argmax(torch.softmax(y.detach(), 1), 1).numpy().astype(np.int64)
        out[f"{tag}/loss"] = np.array(loss.item(), dtype=np.float32)
        out.update(grads_np(f"{tag}/grad", net))
        out.update(sd_np(f"{tag}/after", net.state_dict()))
    np.savez_compressed(os.path.join(OUT, "g2_unet_multiclass.npz"), **out)


def _inject(dist, eps, method):
    """Make a torch Independent(Normal) return loc + scale * eps from rsample()/sample() — what
    Normal.rsample computes for that eps, so gradients still flow through loc and scale."""
    def draw(sample_shape=torch.Size()):
        v = dist.base_dist.loc + dist.base_dist.scale * eps
        return v if method == "rsample" else v.detach()
    setattr(dist, method, draw)


def g3_probunet():
    """ProbabilisticUnet(1,3,[4,8,16,32,64],latent_dim=6,no_convs_fcomb=4,beta=10) — the
    ProbUNetTrainer configuration (probunet_trainer.py:16) at small width — with injected latent
    noise: one training forward + elbo + backward (probabilistic_unet.py:215-308), 8 prior
    samples through Fcomb, and an eval-mode pass (training=False, sample(testing=True))."""
    from model import ProbabilisticUnet
    out = {}
    for tag, (N, H, W, S) in {"s64": (2, 64, 64, 8), "s45": (3, 45, 37, 2)}.items():
        torch.manual_seed(0)
        net = ProbabilisticUnet(input_channels=1, num_classes=3, num_filters=[4, 8, 16, 32, 64], latent_dim=6,
                                no_convs_fcomb=4, beta=10.0)
        if tag == "s64":  # same seed and architecture for both cases: one copy of the initial weights
            out.update(sd_np("init", net.state_dict()))
        g = torch.Generator().manual_seed(3)
        x = torch.rand(N, 1, H, W, generator=g)
        segm = torch.randint(0, 3, (N, 1, H, W), generator=g).float()
        eps_post = torch.randn(N, 6, generator=g)
        eps_prior = torch.randn(S, N, 6, generator=g)
        eps_eval = torch.randn(N, 6, generator=g)
        out[f"{tag}/x"], out[f"{tag}/segm"] = x.numpy(), segm.numpy()
        out[f"{tag}/eps_post"], out[f"{tag}/eps_prior"], out[f"{tag}/eps_eval"] = (
            eps_post.numpy(), eps_prior.numpy(), eps_eval.numpy())
        net.train()
        net.forward(x, segm, training=True)
        _inject(net.posterior_latent_space, eps_post, "rsample")
        elbo = net.elbo(segm)
        loss = -elbo
        loss.backward()
        for name, d in (("post", net.posterior_latent_space), ("prior", net.prior_latent_space)):
            out[f"{tag}/{name}_mu"] = d.base_dist.loc.detach().numpy().copy()
            out[f"{tag}/{name}_sigma"] = d.base_dist.scale.detach().numpy().copy()
        out[f"{tag}/feat"] = net.unet_features.detach().numpy().copy()
        out[f"{tag}/kl"] = np.array(net.kl.item(), dtype=np.float32)
        out[f"{tag}/ce"] = np.array(net.reconstruction_loss.item(), dtype=np.float32)
        out[f"{tag}/elbo"] = np.array(elbo.item(), dtype=np.float32)
        out[f"{tag}/rec"] = net.reconstruction.detach().numpy().copy()
        out.update(grads_np(f"{tag}/grad", net))
        out.update(sd_np(f"{tag}/after", dict(net.named_buffers())))   # BN running statistics
        with torch.no_grad():
            mu_p, sd_p = net.prior_latent_space.base_dist.loc, net.prior_latent_space.base_dist.scale
            out[f"{tag}/samples"] = torch.stack(
                [net.fcomb.forward(net.unet_features, mu_p + sd_p * eps_prior[s]) for s in range(S)]).numpy()
            net.eval()
            net.forward(x, segm, training=False)
            _inject(net.prior_latent_space, eps_eval, "sample")
            out[f"{tag}/eval_sample"] = net.sample(testing=True).numpy().copy()
            out[f"{tag}/eval_prior_mu"] = net.prior_latent_space.base_dist.loc.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "g3_probunet.npz"), **out)


def g4_dice():
    """dice_coeff known answers (dice_loss.py:5-12) and trainer-style per-class Dice
    (unet_trainer.py:39-58) from the reference trainer's eval()."""
    import dice_loss
    from trainer import UNetTrainer
    out = {}
    g = torch.Generator().manual_seed(4)
    cases = {
        "rand": ((torch.rand(3, 20, 20, generator=g) > 0.5).float(), (torch.rand(3, 20, 20, generator=g) > 0.3).float()),
        "empty": (torch.zeros(2, 8, 8), torch.zeros(2, 8, 8)),
        "ones": (torch.ones(2, 8, 8), torch.ones(2, 8, 8)),
        "disjoint": (torch.cat([torch.ones(1, 8, 8), torch.zeros(1, 8, 8)]), torch.cat([torch.zeros(1, 8, 8), torch.ones(1, 8, 8)])),
    }
    for k, (p, t) in cases.items():
        out[f"{k}/pred"], out[f"{k}/target"] = p.numpy(), t.numpy()
        out[f"{k}/dice"] = np.array(dice_loss.dice_coeff(p, t).item(), dtype=np.float32)
    # trainer eval, multi-class and binary (constructed on CPU; eval() only uses self.device for one_hot)
    tr = UNetTrainer.__new__(UNetTrainer)
    tr.device = torch.device("cpu")
    tr.net = types.SimpleNamespace(n_classes=3)
    y = torch.randn(2, 3, 24, 24, generator=g)
    m = torch.randint(0, 3, (2, 1, 24, 24), generator=g)
    out["mc/y"], out["mc/mask"] = y.numpy(), m.numpy().astype(np.int64)
    out["mc/dice"] = tr.eval(None, m, y).astype(np.float64)
    tr.net = types.SimpleNamespace(n_classes=1)
    yb = torch.rand(2, 1, 24, 24, generator=g)
    mb = (torch.rand(2, 1, 24, 24, generator=g) > 0.5).float()
    out["bin/y"], out["bin/mask"] = yb.numpy(), mb.numpy()
    out["bin/dice"] = tr.eval(None, mb, yb).astype(np.float64)
    np.savez_compressed(os.path.join(OUT, "g4_dice.npz"), **out)


def g5_slicer(nib):
    """MRI_Dataset (utils/mri_dataset.py:11-143) on tiny in-memory volumes: non-cube shapes
    padded at the end of the argmin axis, 3-view slicing, per-slice max-norm, fg filter."""
    import utils.mri_dataset as md
    g = np.random.default_rng(5)
    vols = {"a.nii": (6, 8, 8), "b.nii": (8, 5, 8), "c.nii": (8, 8, 7)}
    out = {}
    for name, shp in vols.items():
        img = g.random(shp) * 100.0
        img[0] = 0.0  # an all-zero slice (max-norm skipped)
        lab = np.zeros(shp)
        lab[1:4, 2:5, 1:6] = 1.0
        lab[2:3, 3:4, 2:4] = 2.0
        nib.store["img_" + name] = img
        nib.store["lab_" + name] = lab
        out[f"vol/{name}/img"] = img
        out[f"vol/{name}/lab"] = lab
    imgs = sorted(vols)
    md.listdir = lambda d: list(imgs)
    # the dataset joins dir + file name; route both dirs to the in-memory store by prefix
    orig_load = nib.load
    nib.load = lambda p: orig_load(("img_" if "imgs" in p else "lab_") + os.path.basename(p))
    for filt in (True, False):
        ds = md.MRI_Dataset("/imgs", "/labs", 3, filter=filt)
        key = "filt" if filt else "all"
        out[f"{key}/index_map"] = np.array(ds.index_map, dtype=np.int64)
        out[f"{key}/image_dims"] = np.array(ds.image_dims, dtype=np.int64)
        ims = [ds[i]["image"].numpy() for i in range(len(ds))]
        mks = [ds[i]["mask"].numpy() for i in range(len(ds))]
        out[f"{key}/images"] = np.stack(ims)
        out[f"{key}/masks"] = np.stack(mks)
    nib.load = orig_load
    np.savez_compressed(os.path.join(OUT, "g5_slicer.npz"), **out)


def g6_fusion():
    """3-view fusion (eval.py:157-203).  eval.py does not parse (:137-138); the fixture comes from
    the build's own restatement of its flow (oracle/data_ref.py: per-slice softmax :157, per-view
    volumes with the :182/:188 permutes, 3-view average :193, per-class Dice of the argmax one-hot
    :42-49), with the Dice itself computed by the reference's importable dice_loss.dice_coeff.
    Parity of this row is therefore pinned by the restatement, not by running eval.py."""
    import dice_loss
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from oracle.data_ref import fuse
    out = {}
    g = torch.Generator().manual_seed(6)
    for tag, (D0, D1, D2) in {"cube": (16, 16, 16), "box": (10, 12, 9)}.items():
        C = 3
        truth = torch.randint(0, C, (D0, D1, D2), generator=g).float()
        logits = [torch.randn(n, C, a, b, generator=g) * 2.0 for n, a, b in ((D0, D1, D2), (D1, D0, D2), (D2, D0, D1))]
        probs = [torch.softmax(lg, dim=1) for lg in logits]          # per-slice softmax over C
        vols = fuse(*probs)
        out[f"{tag}/truth"] = truth.numpy()
        for v in range(3):
            out[f"{tag}/logits{v}"] = logits[v].numpy()
            out[f"{tag}/probs{v}"] = probs[v].numpy()
        out[f"{tag}/avg"] = vols[3].numpy()
        out[f"{tag}/label"] = torch.argmax(vols[3], 1).numpy().astype(np.int32)

        def class_dice(vol, k):
            idx = torch.argmax(vol, 1, keepdim=True)
            one_hot = torch.zeros(vol.shape).scatter_(1, idx, 1)   # contiguous, as eval.py:44-46
            return dice_loss.dice_coeff(one_hot[:, k], (truth == k).float()).item()
        out[f"{tag}/dice"] = np.array([[class_dice(vol, k) for k in (1, 2)] for vol in vols])
    np.savez_compressed(os.path.join(OUT, "g6_fusion.npz"), **out)


def g7_dp_accumulation():
    """Gradient accumulation of train.py:85-110 on config c1: UNet(1,1,[16,32]), 8 micro-batches
    of 4 slices at 64x64, loss / 8 per micro-batch, summed into one gradient — what data-parallel
    ranks must reproduce with a SUM all-reduce."""
    from model import UNet
    torch.manual_seed(0)
    net = UNet(1, 1, [16, 32])
    out = sd_np("init", net.state_dict())
    g = torch.Generator().manual_seed(7)
    x = torch.rand(32, 1, 64, 64, generator=g)
    t = (torch.rand(32, 1, 64, 64, generator=g) > 0.5).float()
    out["x"], out["t"] = x.numpy(), t.numpy()
    net.train()
    crit = nn.BCELoss()
    acc = 8
    for i in range(acc):
        loss = crit(net(x[4 * i:4 * i + 4]), t[4 * i:4 * i + 4]) / acc
        loss.backward()
    out.update(grads_np("grad", net))
    np.savez_compressed(os.path.join(OUT, "g7_dp.npz"), **out)


def g8_train_net(nib):
    """The reference's own train_net (train.py:27-196) end to end on a tiny in-memory multi-planar
    dataset: two 24x24x20 scans (cube-padded to 24^3, 3 views, background slices filtered) with
    binary ellipsoid labels, a UNet(1,1,[16,32]) in place of the trainer's default-width net,
    batch 8 (4 accumulated micro-batches of 2), 2 epochs, validation 10%, ReduceLROnPlateau.

    Recorded: the initial weights, the seed set right before train_net, the volumes, every
    SummaryWriter scalar (tag, value, global_step) and image (tag, step, tensor), the dataset item
    order, and the final state_dict.  Shims beyond the import ones: the DataLoader runs with
    num_workers=0 (the worker processes change neither the RNG draws nor the batches), the
    SummaryWriter records instead of writing, checkpoints go to a temporary directory."""
    import tempfile
    import utils.mri_dataset as md
    md.mri_collate = None   # imported by train.py:19, never defined (SURVEY.md §8c shim 4)
    import train as ref_train
    from model import UNet
    from torch.utils.data import DataLoader
    from trainer import UNetTrainer
    g = np.random.default_rng(8)
    out = {}
    names = ["s0.nii", "s1.nii"]
    ax = np.arange(24) - 11.5
    for i, name in enumerate(names):
        ii, jj, kk = np.meshgrid(ax, ax, ax[:20] + 2, indexing="ij")
        r2 = (ii / (7.0 + i)) ** 2 + (jj / 6.0) ** 2 + (kk / 5.0) ** 2
        lab = (r2 < 1.0).astype(np.float64)
        img = g.random((24, 24, 20)) * 80.0 + lab * 120.0
        nib.store["img_" + name], nib.store["lab_" + name] = img, lab
        out[f"vol/{name}/img"], out[f"vol/{name}/lab"] = img, lab
    md.listdir = lambda d: list(names)
    orig_load = nib.load
    nib.load = lambda p: orig_load(("img_" if "imgs" in p else "lab_") + os.path.basename(p))
    order = []

    class LoggedDataset(md.MRI_Dataset):
        def __getitem__(self, i):
            order.append(int(i))
            return super().__getitem__(i)
    ref_train.MRI_Dataset = LoggedDataset
    ref_train.DataLoader = lambda *a, **k: DataLoader(*a, **{**k, "num_workers": 0, "pin_memory": False})
    scalars, images = [], []

    class RecordingWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, tag, v, step):
            scalars.append((tag, float(v), int(step)))

        def add_images(self, tag, t, step):
            images.append((tag, int(step), t.detach().cpu().float().numpy().copy()))

        def close(self):
            pass
    ref_train.SummaryWriter = RecordingWriter
    tmp = tempfile.mkdtemp()
    ref_train.dir_img, ref_train.dir_mask, ref_train.dir_checkpoint = "/imgs/", "/labs/", tmp + "/"
    tr = UNetTrainer(torch.device("cpu"), 1, 1)
    torch.manual_seed(0)
    tr.net = UNet(1, 1, [16, 32])
    out.update(sd_np("init", tr.net.state_dict()))
    torch.manual_seed(123)
    ref_train.train_net(tr, torch.device("cpu"), epochs=2, batch_size=8, lr=0.01, lrf=0.5, lrp=0, om=0.9,
                        val_percent=0.1)
    out.update(sd_np("final", tr.net.state_dict()))
    out["seed"] = np.array(123)
    out["order"] = np.array(order, dtype=np.int64)
    out["scalar_tags"] = np.array([t for t, _, _ in scalars])
    out["scalar_values"] = np.array([v for _, v, _ in scalars], dtype=np.float64)
    out["scalar_steps"] = np.array([s for _, _, s in scalars], dtype=np.int64)
    for i, (tag, step, t) in enumerate(images):
        out[f"image{i}/tag"], out[f"image{i}/step"], out[f"image{i}/data"] = np.array(tag), np.array(step), t
    nib.load = orig_load
    np.savez_compressed(os.path.join(OUT, "g8_train_net.npz"), **out)


def main():
    if not os.path.isdir(REF):
        raise SystemExit(f"reference not found at {REF}: fixtures are generated in the build container only")
    nib = install_shims()
    which = set(sys.argv[1:]) or {"g1", "g2", "g3", "g4", "g5", "g6", "g7", "g8"}
    if "g1" in which:
        g1_unet_c1()
    if "g2" in which:
        g2_unet_multiclass()
    if "g3" in which:
        g3_probunet()
    if "g4" in which:
        g4_dice()
    if "g5" in which:
        g5_slicer(nib)
    if "g6" in which:
        g6_fusion()
    if "g7" in which:
        g7_dp_accumulation()
    if "g8" in which:
        g8_train_net(nib)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
