"""CPU checks of the training driver's host logic: the oracle's train_net restatement against the
reference's own end-to-end run (G8), and train.py's micro-batch dealing / RNG consumption."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def g8():
    return np.load(os.path.join(GOLD, "g8_train_net.npz"), allow_pickle=False)


def g8_scans(z):
    names = sorted({k.split("/")[1] for k in z.files if k.startswith("vol/")})
    return names, [(np.array(z[f"vol/{n}/img"]), np.array(z[f"vol/{n}/lab"])) for n in names]


def g8_sd(z, prefix):
    pre = prefix + "/"
    return {k[len(pre):]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith(pre)}


G8_ARGS = dict(epochs=2, batch_size=8, lr=0.01, lrf=0.5, lrp=0, om=0.9, val_percent=0.1)


def test_oracle_train_net_matches_reference_g8():
    """oracle/train_ref.py reproduces the reference's train_net: sample order, every TensorBoard
    scalar and image, and the final weights + BN buffers (PMU/train.py:27-196)."""
    from oracle.data_ref import build_dataset
    from oracle.train_ref import train_net_ref
    z = g8()
    _, scans = g8_scans(z)
    _, _, items = build_dataset(scans, filt=True)
    torch.set_num_threads(4)
    sd, scalars, images, order = train_net_ref(g8_sd(z, "init"), items, 2, 1, seed=int(z["seed"]), **G8_ARGS)
    assert order == z["order"].tolist()
    assert [t for t, _, _ in scalars] == z["scalar_tags"].tolist()
    assert [s for _, _, s in scalars] == z["scalar_steps"].tolist()
    assert np.allclose([v for _, v, _ in scalars], z["scalar_values"], rtol=1e-5, atol=1e-6)
    for i, (tag, step, t) in enumerate(images):
        assert tag == str(z[f"image{i}/tag"]) and step == int(z[f"image{i}/step"])
        assert np.allclose(t.numpy(), z[f"image{i}/data"], atol=1e-6), tag
    final = g8_sd(z, "final")
    for k, v in final.items():
        assert float((sd[k].double() - v.double()).abs().max()) <= 1e-5, k


def test_train_dp_micro_batches_exact_for_any_world():
    """Every optimizer step holds exactly the reference's acc_steps micro-batches, dealt k % world;
    world > acc_steps leaves ranks idle instead of growing the batch."""
    import train
    order = list(range(70))
    for acc in (1, 4, 8):
        ref_mbs = [order[i:i + 2] for i in range(0, 69, 2)]
        nsteps = len(ref_mbs) // acc
        for world in (1, 2, 3, 4, 8, 12):
            per = [train.dp_micro_batches(order, 2, acc, world, r) for r in range(world)]
            for s in range(nsteps):
                got = sorted(mb for r in range(world) for mb in per[r][0][s])
                assert got == sorted(ref_mbs[s * acc:(s + 1) * acc]), (acc, world, s)
                for r in range(world):
                    assert per[r][0][s] == ref_mbs[s * acc + r:(s + 1) * acc:world]
            left = sorted(mb for r in range(world) for mb in per[r][1])
            assert left == sorted(ref_mbs[nsteps * acc:])


def test_train_loader_order_consumes_rng_like_the_reference():
    """train.loader_order draws the DataLoader's base seed, then the RandomSampler's seed."""
    import train
    from torch.utils.data import DataLoader
    torch.manual_seed(5)
    ref = [int(i) for b in DataLoader(list(range(23)), batch_size=1, shuffle=True) for i in b]
    after_ref = torch.rand(1)
    torch.manual_seed(5)
    got = train.loader_order(23, True, 1)
    assert got == ref
    assert torch.equal(torch.rand(1), after_ref)
    torch.manual_seed(5)
    list(DataLoader(list(range(5)), batch_size=1, shuffle=False))
    after_ref = torch.rand(1)
    torch.manual_seed(5)
    assert train.loader_order(5, False, 1) == list(range(5))
    assert torch.equal(torch.rand(1), after_ref)


def test_leftover_micro_batches_run_predict_and_loss_with_grad(tmp_path):
    """Trailing micro-batches that fill no optimizer step run exactly as the reference runs them
    (PMU/train.py:77-98): predict with grad enabled (for ProbUNetTrainer: the posterior encoder and
    its BatchNorm statistics) and the loss (the posterior sample); no optimizer step follows."""
    import train as T
    events = []

    class Net(torch.nn.Module):
        n_classes = 1

        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(1))

    net = Net()

    class DS:
        def __len__(self):
            return 32

        def get_batch(self, idx):
            return {"image": torch.rand(len(idx), 1, 4, 4), "mask": torch.zeros(len(idx), 1, 4, 4)}

    class Tr:
        name, mask_type, device = "probe", torch.float32, torch.device("cpu")

        def __init__(self):
            self.net = net

        def predict(self, imgs, masks):
            events.append(("predict", torch.is_grad_enabled(), net.training))
            return imgs.mean() * net.w

        def loss(self, imgs, masks, pred):
            events.append(("loss", torch.is_grad_enabled(), net.training))
            return pred * 1.0

        def eval(self, imgs, masks, pred):
            return np.array([1.0])

    steps = []

    class SGDProbe(torch.optim.SGD):
        def step(self, closure=None):
            steps.append(1)
            return super().step(closure)

    T.dir_checkpoint = str(tmp_path) + "/"
    # batch 12 -> acc_steps 4 (reference rule), micro-batch 3: 10 micro-batches = 2 steps + 2 leftover
    T.train_net(Tr(), torch.device("cpu"), epochs=1, batch_size=12, lr=0.1, val_percent=0.0, dataset=DS(),
                optimizer_factory=lambda ps: SGDProbe(ps, lr=0.1))
    train_events = [e for e in events if e[2]]
    assert len(steps) == 2
    assert train_events == [("predict", True, True), ("loss", True, True)] * 10


def test_acc_steps_flag_splits_the_global_batch():
    """--acc-steps / train_net(acc_steps=): the global batch stays batch_size, dealt as acc_steps
    micro-batches; absent, the reference's rule (4 if batch_size > 4 else 1, PMU/train.py:45)."""
    import train as T
    assert T.reference_acc_steps(32) == 4 and T.reference_acc_steps(4) == 1
    a = T.get_args(["-b", "256", "--acc-steps", "8", "--dtype", "bf16", "--filters", "16,32", "--bench"])
    assert (a.batchsize, a.acc_steps, a.dtype, a.filters, a.bench) == (256, 8, "bf16", "16,32", True)
    assert T.get_args([]).acc_steps is None and T.get_args([]).dtype == "fp32"
    steps, left = T.dp_micro_batches(list(range(256)), 32, 8, 8, 3)
    assert steps == [[list(range(96, 128))]] and left == []
