"""GPU parity of the data-side rows and the drop-in loops.

  * slicer (a13): MRI_Dataset on resident scans vs the reference's G5 items — bit-exact;
    at 256^3 vs the oracle restatement on the same volume — bit-exact;
  * Dice (a8): dice_coeff and the trainers' eval vs the reference's G4 — bit-exact;
  * fusion (a14): pmu_fuse3view vs G6 (probabilities in: average, label map and Dice bit-exact;
    logits in: softmax inside the kernel, labels equal up to fp32 ties) and at 128^3 vs the
    restatement;
  * train_net / predict_volume run end to end on a synthetic scan set.
"""
import os
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _g5_dataset(filt, dev):
    from utils.mri_dataset import MRI_Dataset
    z = _load("g5_slicer.npz")
    names = sorted({k.split("/")[1] for k in z.files if k.startswith("vol/")})
    store = {n: (z[f"vol/{n}/img"], z[f"vol/{n}/lab"]) for n in names}

    def loader(p):
        return store[os.path.basename(p)][0 if "imgs" in p else 1]
    return z, MRI_Dataset("/imgs", "/labs", 3, filter=filt, loader=loader, files=names, device=dev)


@pytest.mark.parametrize("filt", [True, False])
def test_slicer_matches_reference_g5(filt, dev):
    z, ds = _g5_dataset(filt, dev)
    key = "filt" if filt else "all"
    assert tuple(ds.image_dims) == tuple(z[f"{key}/image_dims"])
    assert np.array_equal(np.array(ds.index_map), z[f"{key}/index_map"])
    assert len(ds) == len(z[f"{key}/images"])
    imgs = np.stack([ds[i]["image"].cpu().numpy() for i in range(len(ds))])
    masks = np.stack([ds[i]["mask"].cpu().numpy() for i in range(len(ds))])
    assert np.array_equal(imgs, z[f"{key}/images"])      # bit-exact, incl. the f64 max normalisation
    assert np.array_equal(masks, z[f"{key}/masks"])
    # a batched gather equals the items
    b = ds.get_batch(list(range(min(5, len(ds)))))
    assert np.array_equal(b["image"].cpu().numpy(), imgs[:5])


def test_slicer_full_size_vs_oracle(dev):
    """A 256x256x200 scan (padded along axis 2) with a spherical mask: every 7th slice of every
    view, gathered in batches, vs the numpy restatement — bit-exact."""
    from oracle.data_ref import build_dataset
    from utils.mri_dataset import MRI_Dataset
    g = np.random.default_rng(11)
    img = g.random((256, 256, 200)) * 1000.0
    ii, jj, kk = np.meshgrid(np.arange(256), np.arange(256), np.arange(200), indexing="ij")
    lab = ((ii - 128) ** 2 + (jj - 120) ** 2 + (kk - 90) ** 2 < 60 ** 2).astype(np.float64)
    lab[(ii - 128) ** 2 + (jj - 120) ** 2 + (kk - 90) ** 2 < 25 ** 2] = 2.0
    ds = MRI_Dataset("/imgs", "/labs", 3, filter=True, loader=lambda p: img if "imgs" in p else lab, files=["s"],
                     device=dev)
    dims, imap, items = build_dataset([(img, lab)], True)
    assert ds.index_map == [tuple(t) for t in imap] and tuple(ds.image_dims) == tuple(dims)
    sel = list(range(0, len(ds), 7))
    for s0 in range(0, len(sel), 16):
        chunk = sel[s0:s0 + 16]
        b = ds.get_batch(chunk)
        want_i = np.stack([items[i][0] for i in chunk])
        want_m = np.stack([items[i][1] for i in chunk])
        assert np.array_equal(b["image"].cpu().numpy(), want_i)
        assert np.array_equal(b["mask"].cpu().numpy(), want_m)


def test_dice_matches_reference_g4(dev):
    from dice_loss import dice_coeff
    from trainer import UNetTrainer
    z = _load("g4_dice.npz")
    for k in ("rand", "empty", "ones", "disjoint"):
        d = dice_coeff(torch.from_numpy(z[f"{k}/pred"]).to(dev), torch.from_numpy(z[f"{k}/target"]).to(dev))
        assert np.float32(d.item()) == np.float32(z[f"{k}/dice"]), k
    tr = UNetTrainer.__new__(UNetTrainer)
    tr.device = dev
    tr.net = types.SimpleNamespace(n_classes=3)
    got = tr.eval(None, torch.from_numpy(z["mc/mask"]).to(dev), torch.from_numpy(z["mc/y"]).to(dev))
    assert np.array_equal(got.astype(np.float32), z["mc/dice"].astype(np.float32))
    tr.net = types.SimpleNamespace(n_classes=1)
    got = tr.eval(None, torch.from_numpy(z["bin/mask"]).to(dev), torch.from_numpy(z["bin/y"]).to(dev))
    assert np.array_equal(got.astype(np.float32), z["bin/dice"].astype(np.float32))


@pytest.mark.parametrize("tag", ["cube", "box"])
def test_fusion_matches_g6(tag, dev):
    from pmu_hip.fusion import fuse_views
    z = _load("g6_fusion.npz")
    truth = torch.from_numpy(z[f"{tag}/truth"]).to(dev)
    probs = [torch.from_numpy(z[f"{tag}/probs{v}"]).to(dev) for v in range(3)]
    r = fuse_views(*probs, truth)
    assert np.array_equal(r["avg"].cpu().numpy(), z[f"{tag}/avg"])              # bit-exact average
    assert np.array_equal(r["label"].cpu().numpy(), z[f"{tag}/label"])          # bit-exact label map
    assert np.array_equal(r["dice"][:, 1:3].cpu().numpy(), z[f"{tag}/dice"].astype(np.float32))
    logits = [torch.from_numpy(z[f"{tag}/logits{v}"]).to(dev) for v in range(3)]
    r2 = fuse_views(*logits, truth, logits=True)
    assert float((r2["avg"] - r["avg"]).abs().max()) <= 1e-6
    mism = int((r2["label"] != r["label"]).sum())
    assert mism <= 1, mism      # softmax inside the kernel: identical up to fp32 near-ties


def test_fusion_large_vs_restatement(dev):
    """128 x 120 x 100 volume, 3 classes, probabilities in: vs the torch restatement on the CPU (the
    reference's arithmetic: torch's GPU `/ 3.0` multiplies by the reciprocal instead of dividing)."""
    from oracle.data_ref import fuse
    from pmu_hip.fusion import fuse_views
    g = torch.Generator(device="cpu").manual_seed(12)
    D0, D1, D2, C = 128, 120, 100, 3
    st = [torch.softmax(torch.randn(n, C, a, b, generator=g), 1).to(dev)
          for n, a, b in ((D0, D1, D2), (D1, D0, D2), (D2, D0, D1))]
    truth = torch.randint(0, C, (D0, D1, D2), generator=g).float().to(dev)
    r = fuse_views(*st, truth)
    vols = [v.to(dev) for v in fuse(*[t.cpu() for t in st])]
    assert torch.equal(r["avg"], vols[3])
    lab = torch.argmax(vols[3], 1).int()
    assert torch.equal(r["label"], lab)
    for v in range(4):
        am = torch.argmax(vols[v], 1)
        for c in range(C):
            inter = float(((am == c) & (truth == c)).sum())
            assert float(r["counts"][v, c, 0]) == inter
            assert float(r["counts"][v, c, 1]) == float((am == c).sum())
            assert float(r["counts"][v, c, 2]) == float((truth == c).sum())


@pytest.mark.parametrize("D0,D1,D2", [(512, 64, 48), (40, 512, 56)])
def test_fusion_512_edge_vs_restatement(dev, D0, D1, D2):
    """Config c5's eval volume has 512-voxel edges (PMU/eval.py:157-203 on a 512^3 scan; the bench runs
    512^3 on random-init weights only): a 512-edge volume along the view-0 slice axis and along a
    transposed axis, 3 classes, vs the restatement.  Probabilities in: average, label map and counts
    exact.  Logits in (the predictor's path, softmax inside the kernel): average within 1e-6 and labels
    equal but at fp32 near-ties of the top two classes."""
    from oracle.data_ref import fuse
    from pmu_hip.fusion import fuse_views
    g = torch.Generator(device="cpu").manual_seed(D0 + 3 * D1 + 7 * D2)
    C = 3
    logits = [torch.randn(n, C, a, b, generator=g) * 3.0 for n, a, b in ((D0, D1, D2), (D1, D0, D2), (D2, D0, D1))]
    st = [torch.softmax(t, 1) for t in logits]
    truth = torch.randint(0, C, (D0, D1, D2), generator=g).float()
    vols = fuse(*st)
    r = fuse_views(*[t.to(dev) for t in st], truth.to(dev))
    assert torch.equal(r["avg"].cpu(), vols[3])
    lab = torch.argmax(vols[3], 1).int()
    assert torch.equal(r["label"].cpu(), lab)
    for v in range(4):
        am = torch.argmax(vols[v], 1)
        for c in range(C):
            assert float(r["counts"][v, c, 0]) == float(((am == c) & (truth == c)).sum())
            assert float(r["counts"][v, c, 1]) == float((am == c).sum())
            assert float(r["counts"][v, c, 2]) == float((truth == c).sum())
    r2 = fuse_views(*[t.to(dev) for t in logits], truth.to(dev), logits=True)
    assert float((r2["avg"].cpu() - vols[3]).abs().max()) <= 1e-6
    top = torch.topk(vols[3], 2, dim=1).values
    flips = r2["label"].cpu() != lab
    assert bool(((top[:, 0] - top[:, 1])[flips] < 1e-5).all()), int(flips.sum())


def _argmax_dim1(x):
    """torch.argmax(x, 1) (first index of the maximum) as C-1 elementwise passes: torch's CPU
    reduction over a short middle axis takes ~30 s per 512^3 x 3 volume, this ~1.5 s (no NaN here)."""
    best = x[:, 0].clone()
    idx = torch.zeros(best.shape, dtype=torch.long)
    for c in range(1, x.shape[1]):
        m = x[:, c] > best
        idx[m] = c
        best = torch.where(m, x[:, c], best)
    return idx


def test_fusion_512_cubed_vs_restatement(dev):
    """Config c5's eval at full size (PMU/eval.py:157-203 on a 512^3 scan, 3 classes):
    one pmu_fuse3view launch over three 512^3 x 3-class view stacks vs the restatement
    (oracle/data_ref.fuse + eval.py:42-49's argmax Dice) on the CPU.  Predictions correlate with a nested-ellipsoid truth, so the Dice values are far from 0
    and 1.  Probabilities in: average and label volume bit-exact, Dice counts exact, per-class Dice of
    all four volumes within 1e-6 of eval.py's formula on the restated counts (contract: 1e-3).
    Logits in (the predictor's path, softmax in the kernel): average within 1e-6, labels equal except
    at fp32 near-ties of the top two classes."""
    from oracle.data_ref import fuse
    from pmu_hip.fusion import fuse_views
    D, C = 512, 3
    g = torch.Generator(device="cpu").manual_seed(512)
    ax = torch.arange(D, dtype=torch.float32) - D / 2
    r2 = ((ax[:, None, None] / (0.40 * D)) ** 2 + (ax[None, :, None] / (0.33 * D)) ** 2 +
          (ax[None, None, :] / (0.28 * D)) ** 2)
    truth = (r2 < 1.0).float() + (r2 < 0.35).float()
    del r2
    # per-view stacks in their own frames (the inverse of eval.py:176-188's permutes): evidence + noise
    logits = []
    for perm in ((0, 1, 2), (1, 0, 2), (2, 0, 1)):
        t = truth.permute(*perm).unsqueeze(1)
        lg = torch.randn(D, C, D, D, generator=g) * 1.5
        lg += 2.0 * (t == torch.arange(C, dtype=torch.float32)[None, :, None, None]).float()
        logits.append(lg)
        del t
    st = [torch.softmax(t, 1) for t in logits]
    vols = fuse(*st)
    truth_d = truth.to(dev)
    r = fuse_views(*[t.to(dev) for t in st], truth_d)
    r_avg, r_lab, r_cnt, r_dice = r["avg"].cpu(), r["label"].cpu(), r["counts"].cpu(), r["dice"].cpu()
    del r
    torch.cuda.empty_cache()
    r2 = fuse_views(*[t.to(dev) for t in logits], truth_d, logits=True)
    l_avg, l_lab = r2["avg"].cpu(), r2["label"].cpu()
    del r2, truth_d
    torch.cuda.empty_cache()
    avg = vols[3]
    lab = _argmax_dim1(avg).int()
    assert torch.equal(lab[200:204], torch.argmax(avg[200:204], 1).int())   # the helper is torch.argmax
    assert torch.equal(r_avg, avg)
    assert torch.equal(r_lab, lab)
    assert float((l_avg - avg).abs().max()) <= 1e-6
    f = (l_lab != lab).nonzero(as_tuple=True)
    top = torch.topk(avg[f[0], :, f[1], f[2]], 2, dim=1).values if f[0].numel() else torch.zeros(0, 2)
    flips, near_tie_flips = int(f[0].numel()), int(((top[:, 0] - top[:, 1]) < 1e-5).sum())
    # eval.py:42-49's argmax of each volume; views 1 and 2 argmax'ed in their own frame and the label
    # volume permuted (the same per-voxel argmax, first index on ties, as argmax of the permuted view)
    ams = [_argmax_dim1(st[0]), _argmax_dim1(st[1]).permute(1, 0, 2),
           _argmax_dim1(st[2]).permute(1, 2, 0), lab.long()]
    tl = truth.long()
    counts = torch.zeros(4, C, 3, dtype=torch.float64)
    for v in range(4):
        conf = torch.bincount((ams[v] * C + tl).reshape(-1), minlength=C * C).reshape(C, C).double()
        counts[v, :, 0] = conf.diagonal()
        counts[v, :, 1] = conf.sum(1)
        counts[v, :, 2] = conf.sum(0)
    assert flips == near_tie_flips, (flips, near_tie_flips)
    assert torch.equal(r_cnt, counts)
    for v in range(4):   # eval.py:42-49's Dice (dice_coeff's 1e-6 smoothing) on the restated counts
        for c in range(C):
            ref = (2.0 * counts[v, c, 0] + 1e-6) / (counts[v, c, 1] + counts[v, c, 2] + 1e-6)
            assert abs(float(r_dice[v, c]) - float(ref)) <= 1e-6, (v, c, float(r_dice[v, c]), float(ref))
    assert 0.05 < float(r_dice[3, 1]) < 0.999 and 0.05 < float(r_dice[3, 2]) < 0.999, r_dice


def _synthetic_scans(n, shape, seed):
    g = np.random.default_rng(seed)
    out = {}
    for s in range(n):
        img = g.random(shape) * 100.0
        ii, jj, kk = np.meshgrid(*[np.arange(d) for d in shape], indexing="ij")
        r2 = (ii - shape[0] / 2) ** 2 + (jj - shape[1] / 2) ** 2 + (kk - shape[2] / 2) ** 2
        lab = np.zeros(shape)
        lab[r2 < (min(shape) / 3) ** 2] = 1.0
        lab[r2 < (min(shape) / 6) ** 2] = 2.0
        out[f"scan{s}.nii"] = (img, lab)
    return out


def test_train_net_and_predict_volume_end_to_end(dev, tmp_path):
    """train.py's train_net (1 epoch, batch 8 -> 4 micro-batches of 2, clip+SGD, validation Dice,
    checkpoints) and predict_volume + fusion on a synthetic 16^3 scan set."""
    import train as train_mod
    from predict import predict_volume
    from trainer import UNetTrainer
    from utils.mri_dataset import MRI_Dataset
    scans = _synthetic_scans(2, (16, 16, 16), 3)
    ds = MRI_Dataset("/imgs", "/labs", 3, filter=True, files=sorted(scans),
                     loader=lambda p: scans[os.path.basename(p)][0 if "imgs" in p else 1], device=dev)
    torch.manual_seed(0)
    tr = UNetTrainer(dev, n_channels=1, n_classes=3)
    train_mod.dir_checkpoint = str(tmp_path) + "/"
    before = {k: v.clone() for k, v in tr.net.state_dict().items()}
    train_mod.train_net(tr, dev, epochs=1, batch_size=8, lr=1e-3, val_percent=0.2, dataset=ds)
    after = tr.net.state_dict()
    assert any(not torch.equal(before[k], after[k]) for k in before)
    assert all(torch.isfinite(v.float()).all() for v in after.values())
    assert os.path.exists(os.path.join(str(tmp_path), "unet_checkpoint0.pt"))
    res = predict_volume(tr.net, ds, 0, batch_size=8)
    from oracle.data_ref import fuse
    probs = [torch.softmax(s, 1).cpu() for s in res["stacks"]]
    vols = fuse(*probs)
    truth = res["truth"].cpu()
    for v in range(4):
        for k in (1, 2):
            lo, hi, n_tie = _dice_bounds(vols[v], truth, k)
            got = float(res["dice"][v, k])
            assert lo - 1e-3 <= got <= hi + 1e-3, (v, k, got, lo, hi, n_tie)


def _dice_bounds(vol, truth, k, tie=1e-5):
    """eval.py's dice(volume, truth, k) (:42-49) as an interval over the fp32 near-ties: voxels whose
    top-two probabilities are within ``tie`` (softmax / averaging rounding can order them either
    way) may take either of those two labels.  Without near-ties lo == hi == the reference's Dice."""
    s = 1e-6
    top = torch.topk(vol, 2, dim=1)
    amb = (top.values[:, 0] - top.values[:, 1]) < tie
    lab = top.indices[:, 0]
    t = truth.reshape(lab.shape) == k
    sure = (lab == k) & ~amb
    cand = amb & ((top.indices[:, 0] == k) | (top.indices[:, 1] == k))
    i0, p0, tt = float((sure & t).sum()), float(sure.sum()), float(t.sum())
    a, b = float((cand & t).sum()), float((cand & ~t).sum())
    return (2 * i0 + s) / (p0 + b + tt + s), (2 * (i0 + a) + s) / (p0 + a + tt + s), int(amb.sum())


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 3])
def test_dice_counts_multiblock_exact(K):
    """pmu_dice_counts over a grid-strided multi-block launch: the per-class counts equal a float64
    CPU count (softmax -> argmax for K > 1, pred > 0.5 for K == 1) exactly."""
    from pmu_hip.metrics import dice_counts
    g = torch.Generator().manual_seed(5 + K)
    N, H, W = 8, 128, 160
    y = torch.randn(N, K, H, W, generator=g) if K > 1 else torch.rand(N, 1, H, W, generator=g)
    mask = torch.randint(0, max(K, 2), (N, 1, H, W), generator=g).float()
    got = dice_counts(y.cuda(), mask.cuda(), K).cpu()
    if K == 1:
        pr = (y[:, 0] > 0.5).double()
        t = mask[:, 0].double()
        want = torch.tensor([[(pr * t).sum(), pr.sum(), t.sum()]], dtype=torch.float64)
    else:
        am = torch.softmax(y, 1).argmax(1)
        t = mask[:, 0].long()
        want = torch.tensor([[((am == k) & (t == k)).sum(), (am == k).sum(), (t == k).sum()] for k in range(K)],
                            dtype=torch.float64)
    assert torch.equal(got, want), (got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("K,S", [(1, 3), (3, 16), (4, 5)])
def test_dice_counts_many_equals_per_sample(K, S):
    """pmu_dice_counts_many (the c4 eval's 16 prior samples in one launch): every sample's counts equal
    its own pmu_dice_counts call exactly."""
    from pmu_hip.metrics import dice_counts, dice_counts_many
    g = torch.Generator().manual_seed(11 + K + S)
    N, H, W = 4, 96, 80
    ys = torch.randn(S, N, K, H, W, generator=g) if K > 1 else torch.rand(S, N, 1, H, W, generator=g)
    mask = torch.randint(0, max(K, 2), (N, 1, H, W), generator=g).float().cuda()
    ys = ys.cuda()
    got = dice_counts_many(ys, mask, K).cpu()
    assert got.shape == (S, K, 3)
    for s in range(S):
        assert torch.equal(got[s], dice_counts(ys[s], mask, K).cpu()), s
