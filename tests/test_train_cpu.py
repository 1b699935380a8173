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
