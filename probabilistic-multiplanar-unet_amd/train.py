"""Training loop — drop-in for PMU/train.py:27-250 (train_net, get_args, __main__).

Same signature and loop semantics as the reference's train_net:
  * random_split of the slice dataset into train/validation (val_percent), per-epoch shuffled
    train order (RandomSampler), drop_last batches of batch_size // acc_steps slices,
    acc_steps = 4 if batch_size > 4 else 1 gradient-accumulation micro-batches per step (:39-48);
  * loss / acc_steps, backward, and every acc_steps micro-batches clip_grad_value_(0.1) +
    SGD(lr, momentum=om) + zero_grad (:93-110) — here one fused kernel (pmu_hip.optim.FusedSGD);
  * validation: trainer.eval Dice and loss, ReduceLROnPlateau(factor=lrf, patience=lrp) on the
    Dice (1 class) or the validation loss (:121-176), checkpoints per epoch (:180-185).

MI355X-first differences: batches are assembled on the GPU from resident scans
(MRI_Dataset.get_batch) instead of a 6-worker DataLoader re-reading volumes from disk, and the loop
is data-parallel when launched with torch.distributed (one process per GPU, RCCL):

  every optimizer step consumes the reference's acc_steps consecutive micro-batches; micro-batch k
  of a step goes to rank k % world, every rank scales its loss by 1 / acc_steps, and one SUM
  all-reduce of the flat gradient buffer yields exactly the reference's accumulated gradient, for
  any world size (ranks beyond acc_steps are idle for the step; the global batch never changes).
  ``dp_micro_batches`` / ``allreduce_grads``; checked against the reference's own accumulation in
  tests/test_dp_gloo.py.  BatchNorm statistics stay per micro-batch, as in the reference; before
  validation and checkpoints the replicas' running statistics are averaged (``BNSync``) so every
  rank validates, schedules the learning rate and saves the same model.  The all-reduce is
  bucketed and issued during the last micro-batch's backward (pmu_hip.dp; PMU_DP_OVERLAP=0 selects
  the one-shot all-reduce after the backward).

The default RNG stream is consumed as the reference's (random_split, then per loader iterator a
base-seed draw and the RandomSampler's seed), so a seeded single-GPU run visits the slices in the
reference's order (tests/test_train_gpu.py checks a whole run against golden vectors G8).
"""
from __future__ import annotations

import argparse
import gc
import logging
import os

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import RandomSampler, random_split

from trainer import ProbUNetTrainer, UNetTrainer

# Image locations (module globals, as in the reference :22-25; -d/--dir overrides them)
dir_img = "data/imgs/"
dir_mask = "data/masks/"
dir_checkpoint = "checkpoints/"


class _NullWriter:
    """Stand-in for torch.utils.tensorboard.SummaryWriter when tensorboard is not installed."""

    def __getattr__(self, name):
        return lambda *a, **k: None


def _writer(comment):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(comment=comment)
    except Exception:  # tensorboard is optional (out of scope for the hot path)
        return _NullWriter()


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shared_generator():
    """A generator seeded identically on every rank (rank 0 draws the seed from the default RNG and
    broadcasts it), so all ranks agree on the split and the per-epoch order."""
    seed = torch.empty((), dtype=torch.int64).random_().item()
    world, _ = world_info()
    if world > 1:
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([seed], dtype=torch.int64, device=dev)
        dist.broadcast(t, 0)
        seed = int(t.item())
    return torch.Generator().manual_seed(int(seed))


def loader_order(n, shuffle, world):
    """Sample order of one pass of the reference's DataLoader (:47-48), with its RNG draws: creating
    the loader iterator draws a base seed from the default generator (workers' seeds), then a
    RandomSampler (shuffle) draws its own seed and permutes.  Reproducing both draws keeps the
    default RNG stream — and so the split and every epoch's order — identical to the reference's.
    world > 1: rank 0's draws, broadcast, so all ranks agree."""
    seed = torch.empty((), dtype=torch.int64).random_().item()   # _BaseDataLoaderIter._base_seed
    del seed
    if not shuffle:
        return list(range(n))
    if world == 1:
        return list(RandomSampler(range(n)))
    return torch.randperm(n, generator=shared_generator()).tolist()


def epoch_order(n, world):
    """Shuffled sample order of one training epoch (see loader_order)."""
    return loader_order(n, True, world)


def dp_micro_batches(order, micro, acc_steps, world, rank):
    """Deal one epoch's drop_last micro-batches (sample ``order``, ``micro`` slices each) to ranks,
    exactly as the reference accumulates them (:45-49, :77-110).

    Every optimizer step consumes the reference's ``acc_steps`` consecutive micro-batches; micro-
    batch k of a step goes to rank k % world.  Each rank scales its loss by 1 / acc_steps (the
    reference's loss / acc_steps) and a SUM all-reduce then gives exactly the reference's
    accumulated gradient — for any world size: with world > acc_steps the extra ranks are idle for
    the step (they contribute zeros), so the global batch never changes.

    Returns (steps, leftover): ``steps[s]`` = this rank's micro-batches of optimizer step s (lists
    of dataset indices; empty = idle), ``leftover`` = this rank's share of the trailing micro-
    batches that fill no step (the reference runs them and never steps: only their BatchNorm
    running-statistics updates survive)."""
    mbs = [list(order[i:i + micro]) for i in range(0, len(order) - micro + 1, micro)]
    nsteps = len(mbs) // acc_steps
    steps = [[mbs[s * acc_steps + k] for k in range(rank, acc_steps, world)] for s in range(nsteps)]
    rest = mbs[nsteps * acc_steps:]
    return steps, [rest[k] for k in range(rank, len(rest), world)]


def allreduce_grads(net, plist=None, idle=False):
    """SUM all-reduce of every gradient: one collective over the flat gradient buffer when all
    grads are its views (the HIP autograd nodes arrange that), else one flattened bucket.
    ``idle``: this rank ran no micro-batch this step; it contributes zeros and adopts the sums
    (every parameter gets a gradient; ones no rank computed stay zero)."""
    world, _ = world_info()
    if world == 1:
        return
    from pmu_hip.functions import _offsets, flat_grad_buffer
    plist = plist if plist is not None else [p for p in net.parameters()]
    if idle:
        buf = flat_grad_buffer(net, plist)
        buf.zero_()
        dist.all_reduce(buf)
        offs = _offsets(net, plist)
        for p in plist:
            p.grad = buf[offs[id(p)]:offs[id(p)] + p.numel()].view_as(p)
        return
    with_grad = [p for p in plist if p.grad is not None]
    buf = net.__dict__.get("_pmu_grad_flat")
    if buf is not None:
        lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * buf.element_size()
        if all(lo <= p.grad.data_ptr() < hi for p in with_grad):
            # params without a grad keep zeros in their slots on every rank: the sum stays exact
            dist.all_reduce(flat_grad_buffer(net, plist))
            return
    if with_grad:
        flat = torch.cat([p.grad.reshape(-1) for p in with_grad])
        dist.all_reduce(flat)
        off = 0
        for p in with_grad:
            n = p.grad.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n


class BNSync:
    """Keeps the replicas' BatchNorm buffers identical for validation and checkpoints (world > 1):
    running_mean / running_var are averaged over the ranks (each rank's EMA saw only its own
    micro-batches) and num_batches_tracked becomes the count over all ranks, which equals the
    reference's single-process count."""

    def __init__(self, net):
        self.bns = [m for m in net.modules() if isinstance(m, torch.nn.BatchNorm2d) and m.track_running_stats]
        self.base = [int(m.num_batches_tracked) for m in self.bns]

    def __call__(self):
        world, _ = world_info()
        if world == 1 or not self.bns:
            return
        dev = self.bns[0].running_mean.device if dist.get_backend() == "nccl" else torch.device("cpu")
        stats = torch.cat([torch.cat([m.running_mean, m.running_var]) for m in self.bns]).to(dev)
        dist.all_reduce(stats)
        stats = (stats / world).to(self.bns[0].running_mean.device)
        cnt = torch.tensor([int(m.num_batches_tracked) - b for m, b in zip(self.bns, self.base)],
                           dtype=torch.int64, device=dev)
        dist.all_reduce(cnt)
        o = 0
        for i, m in enumerate(self.bns):
            c = m.running_mean.numel()
            m.running_mean.copy_(stats[o:o + c])
            m.running_var.copy_(stats[o + c:o + 2 * c])
            o += 2 * c
            m.num_batches_tracked.fill_(self.base[i] + int(cnt[i]))
            self.base[i] = int(m.num_batches_tracked)


def _sync(device):
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _from_rank(value, src, dev):
    """A float held by rank ``src`` on every rank (the reference logs the last micro-batch's loss)."""
    world, rank = world_info()
    if world == 1:
        return value
    t = torch.tensor([value if rank == src else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(t)


def reference_acc_steps(batch_size):
    """The reference's gradient-accumulation rule (:44-45)."""
    return 4 if batch_size > 4 else 1


def train_net(trainer, device, epochs=5, batch_size=1, lr=0.001, lrf=0.1, lrp=2, om=0.9, val_percent=0.1,
              save_cp=False, dataset=None, writer=None, acc_steps=None, dtype="fp32", stats=None,
              optimizer_factory=None):
    """train.py:27-196.  ``dataset`` (an MRI_Dataset; default: built from dir_img/dir_mask) and
    ``writer`` (a SummaryWriter-like sink; default: TensorBoard when installed) are injectable.

    Build-side options (all default to the reference's behaviour):
      acc_steps: micro-batches per optimizer step (None: the reference's 4 if batch_size > 4 else 1).
        The global batch stays ``batch_size`` = acc_steps micro-batches of batch_size // acc_steps,
        with loss / acc_steps.  Config c3 — 8 ranks x 32 slices — is ``batch_size=256, acc_steps=8``
        on 8 ranks: one micro-batch of 32 per rank per step, the reference's accumulation of 8
        micro-batches (:95-110).
      dtype: "bf16" runs the predictions under torch.autocast("cuda", bfloat16) (config c5's
        arithmetic on the bf16-MFMA kernels); "fp32" is the reference's.
      stats: a list that receives one dict per epoch with the train phase's throughput.
      optimizer_factory: params -> optimizer (default: FusedSGD(lr, momentum=om, clip=0.1), the
        reference's clip_grad_value_(0.1) + SGD(lr, momentum=om) in one kernel)."""
    import time
    from contextlib import nullcontext
    from utils.mri_dataset import MRI_Dataset

    world, rank = world_info()
    if dataset is None:
        dataset = MRI_Dataset(dir_img, dir_mask, trainer.net.n_classes)
    n_val = int(len(dataset) * val_percent)
    n_train = len(dataset) - n_val
    if world == 1:
        train, val = random_split(dataset, [n_train, n_val])
    else:
        train, val = random_split(dataset, [n_train, n_val], generator=shared_generator())
    if acc_steps is None:
        acc_steps = reference_acc_steps(batch_size)
    if acc_steps < 1 or batch_size // acc_steps < 1:
        raise ValueError(f"batch size {batch_size} cannot be split into {acc_steps} micro-batches")
    micro = batch_size // acc_steps
    if dtype not in ("fp32", "bf16"):
        raise ValueError(f"dtype must be fp32 or bf16, not {dtype!r}")

    def precision():
        return torch.autocast("cuda", dtype=torch.bfloat16) if dtype == "bf16" else nullcontext()
    if writer is None:
        writer = _writer(f"LRF_{lrf}_LRP_{lrp}_EP_{epochs}_LR_{lr}_BS_{batch_size}") if rank == 0 else _NullWriter()
    elif rank != 0:
        writer = _NullWriter()
    global_step = 0
    logging.info(f"Starting training: epochs {epochs}, batch size {batch_size}, lr {lr}, training size {n_train}, "
                 f"validation size {n_val}, checkpoints {save_cp}, device {device}, ranks {world}")
    if world > acc_steps:
        logging.warning(f"{world} ranks > {acc_steps} accumulation micro-batches per step: {world - acc_steps} "
                        f"rank(s) idle each step (the global batch stays {batch_size}, as in the reference)")
    net = trainer.net
    if optimizer_factory is None:
        from pmu_hip.optim import FusedSGD
        optimizer = FusedSGD(net.parameters(), lr=lr, momentum=om, clip=0.1)
    else:
        optimizer = optimizer_factory(net.parameters())
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "min" if net.n_classes > 1 else "max",
                                                           factor=lrf, patience=lrp)
    plist = list(net.parameters())
    sync = None
    if world > 1 and os.environ.get("PMU_DP_OVERLAP", "1") != "0":
        from pmu_hip.dp import BucketAllReduce
        sync = BucketAllReduce(net)
    bn_sync = BNSync(net)
    n_train_mb = n_train // micro if micro else 0
    for epoch in range(epochs):
        net.train()
        # ---- train phase
        order = [train.indices[i] for i in epoch_order(n_train, world)]
        steps, leftover = dp_micro_batches(order, micro, acc_steps, world, rank)
        scale = 1.0 / acc_steps
        optimizer.zero_grad()
        if stats is not None:
            _sync(device)
            t0 = time.perf_counter()
        for s, step_mbs in enumerate(steps):
            last = None
            for i, mb in enumerate(step_mbs):
                b = dataset.get_batch(mb)
                imgs = b["image"]
                true_masks = b["mask"].to(dtype=trainer.mask_type)
                with precision():
                    masks_pred = trainer.predict(imgs, true_masks)
                loss = trainer.loss(imgs, true_masks, masks_pred) * scale
                # the prediction's own graph is not the loss's for ProbUNetTrainer (the loss
                # reconstructs from the posterior sample): drop it before the backward so its pending
                # Fcomb node does not turn the reconstruction's gradients into non-flat tensors
                del masks_pred
                if sync is not None and i == len(step_mbs) - 1:
                    sync.begin()      # the last micro-batch's backward issues the bucket all-reduces
                loss.backward()
                last = loss
            idle = not step_mbs
            if sync is not None:
                if idle:
                    sync.begin()
                sync.finish(idle=idle)
            else:
                allreduce_grads(net, plist, idle=idle and world > 1)
            # the reference logs the step's last micro-batch (k = acc_steps - 1) at its global step
            owner = (acc_steps - 1) % world
            out_loss = _from_rank(float(last.item()) if (last is not None and rank == owner) else 0.0, owner, device)
            writer.add_scalar("Loss/train", out_loss, global_step + s * acc_steps + acc_steps - 1)
            optimizer.step()
            optimizer.zero_grad()
        if stats is not None:
            _sync(device)
            if world > 1:
                dist.barrier()
            dt = time.perf_counter() - t0
            stats.append({"epoch": epoch, "optimizer_steps": len(steps), "slices": len(steps) * micro * acc_steps,
                          "seconds": dt, "slices_per_s": len(steps) * micro * acc_steps / dt if dt > 0 else 0.0,
                          "ranks": world, "acc_steps": acc_steps, "micro_batch": micro, "dtype": dtype})
        # Trailing micro-batches that fill no step: the reference runs predict, loss and backward on
        # them (:77-98) and its validation zero_grad drops the gradient (:122).  Predict and loss run
        # here exactly as in a step (grad enabled: the posterior encoder runs and updates its BatchNorm
        # statistics, the posterior sample is drawn); the backward, whose result is discarded, is not.
        for mb in leftover:
            b = dataset.get_batch(mb)
            imgs, true_masks = b["image"], b["mask"].to(dtype=trainer.mask_type)
            with precision():
                masks_pred = trainer.predict(imgs, true_masks)
            trainer.loss(imgs, true_masks, masks_pred)
            del masks_pred
        global_step += n_train_mb
        # ---- validation phase (replicas agree on BN statistics; every rank evaluates the split)
        bn_sync()
        net.eval()
        loader_order(n_val, False, world)     # the validation loader's iterator draw (:49)
        val_batches = [list(val.indices[i:i + micro]) for i in range(0, n_val - micro + 1, micro)] if micro else []
        val_count = len(val_batches)
        dices, dice_sums, loss_sum = 0, np.zeros(max(0, net.n_classes - 1)), 0.0
        for mb in val_batches:
            b = dataset.get_batch(mb)
            imgs, true_masks = b["image"], b["mask"].to(dtype=trainer.mask_type)
            with torch.no_grad():
                with precision():
                    masks_pred = trainer.predict(imgs, true_masks)
                dice = trainer.eval(imgs, true_masks, masks_pred)
                loss_sum += trainer.loss(imgs, true_masks, masks_pred).item()
            if net.n_classes > 1:
                dice_sums += dice
            else:
                dices += dice
            if global_step % val_count == 0:   # one example per validation round (:155-160)
                writer.add_images("images", imgs, global_step)
                writer.add_images("masks/true", trainer.mask_to_image(true_masks), global_step)
                writer.add_images("masks/pred", trainer.mask_to_image(masks_pred, prediction=True), global_step)
            global_step += 1
        val_count = max(1, val_count)
        avg_loss = loss_sum / val_count
        writer.add_scalar("Loss/validation", avg_loss, global_step)
        writer.add_scalar("learning_rate", optimizer.param_groups[0]["lr"], global_step)
        for c in range(net.n_classes - 1):
            writer.add_scalar(f"dice/class_{c + 1}", dice_sums[c] / val_count, global_step)
        if net.n_classes == 1:
            val_score = float((dices / val_count)[0]) if val_batches else 0.0
            logging.info(f"Validation Dice Coeff: {val_score}")
            writer.add_scalar("metrics/dice", val_score, global_step)
        else:
            val_score = avg_loss
        val_score = _from_rank(val_score, 0, device)   # one learning-rate schedule for all replicas
        scheduler.step(val_score)
        if rank == 0:
            os.makedirs(dir_checkpoint, exist_ok=True)
            torch.save(net.state_dict(), os.path.join(dir_checkpoint, trainer.name + f"_checkpoint{epoch}.pt"))
            logging.info(f"Saved model {trainer.name}_checkpoint{epoch}.pt")
        gc.collect()
    if rank == 0:
        os.makedirs(dir_checkpoint, exist_ok=True)
        torch.save(net.state_dict(), os.path.join(dir_checkpoint, trainer.name + "_model.pt"))
        logging.info(f"Saved model {trainer.name}_model.pt")
    writer.close()


def get_args(argv=None):
    parser = argparse.ArgumentParser(description="Train the UNet on images and target masks",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-e", "--epochs", metavar="E", type=int, default=5, help="Number of epochs", dest="epochs")
    parser.add_argument("-b", "--batch-size", metavar="B", type=int, nargs="?", default=2, help="Batch size",
                        dest="batchsize")
    parser.add_argument("-l", "--learning-rate", metavar="LR", type=float, nargs="?", default=0.001,
                        help="Learning rate", dest="lr")
    parser.add_argument("-r", "--schedule-factor", metavar="LRF", type=float, nargs="?", default=0.1,
                        help="Learning rate scheduler factor", dest="lrf")
    parser.add_argument("-p", "--schedule-patience", metavar="LRP", type=int, nargs="?", default=5,
                        help="Learning rate scheduler patience", dest="lrp")
    parser.add_argument("-o", "--optimizer-momentum", metavar="OM", type=float, nargs="?", default=0.9,
                        help="Optimizer momentum", dest="om")
    parser.add_argument("-f", "--load", dest="load", type=str, default=None, help="Load model from a .pth file")
    parser.add_argument("-s", "--scale", dest="scale", type=float, default=1, help="Downscaling factor of the images")
    parser.add_argument("-v", "--validation", dest="val", type=float, default=10.0,
                        help="Percent of the data that is used as validation (0-100)")
    parser.add_argument("-m", "--model", dest="net", type=str, default="unet", help="what model to use: unet or probunet")
    parser.add_argument("-d", "--dir", dest="dir", type=str, default=None, help="image and label superdirs.")
    # build-side flags; every default is the reference's behaviour
    parser.add_argument("--acc-steps", dest="acc_steps", type=int, default=None,
                        help="micro-batches per optimizer step (default: the reference's 4 if batch size > 4 else 1); "
                             "c3 = 8 ranks x 32: -b 256 --acc-steps 8 on 8 ranks")
    parser.add_argument("--dtype", dest="dtype", choices=["fp32", "bf16"], default="fp32",
                        help="bf16: predictions under torch.autocast(bfloat16) on the bf16-MFMA kernels (config c5)")
    parser.add_argument("--filters", dest="filters", type=str, default=None,
                        help="comma-separated num_filters of the U-Net (default 64,128,256,512,1024)")
    parser.add_argument("--classes", dest="classes", type=int, default=None,
                        help="number of classes (default: 1 for unet, 3 for probunet, as the reference's __main__)")
    parser.add_argument("--channels", dest="channels", type=int, default=1, help="input channels per slice")
    parser.add_argument("--nproc", dest="nproc", type=int, default=1,
                        help="launch this many ranks on this node, one per GPU (torch.distributed.run, RCCL); "
                             "ignored when already launched by torchrun")
    parser.add_argument("--bench", dest="bench", action="store_true",
                        help="train on a seeded synthetic ellipsoid phantom resident on the GPU (no data "
                             "directory) and print the train phase's throughput per epoch as JSON")
    parser.add_argument("--bench-size", dest="bench_size", type=int, default=256, help="--bench phantom edge D (D^3)")
    parser.add_argument("--bench-scans", dest="bench_scans", type=int, default=2, help="--bench phantom count")
    return parser.parse_args(argv)


def _relaunch(nproc, argv):
    """--nproc N outside torchrun: run this script under torch.distributed.run with N ranks as a child
    process (nothing here has touched the GPU yet) and return its exit code."""
    import socket
    import subprocess
    import sys
    args, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == "--nproc":
            skip = True
            continue
        if a.startswith("--nproc="):
            continue
        args.append(a)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + args
    return subprocess.call(cmd)


def bench_dataset(n_classes, size, scans, device, seed=11):
    """--bench data: ``scans`` seeded size^3 volumes — two nested ellipsoid shells (labels 1, 2 as the
    knee labels of PMU/Utils/nii.py:83-90; 1 class: the union) under a noisy contrast — resident on
    the GPU as an MRI_Dataset (filtered 3-view index map, as the reference's)."""
    from utils.mri_dataset import MRI_Dataset
    rng = np.random.default_rng(seed)
    vols = {}
    ax = np.arange(size) - size / 2
    ii, jj, kk = np.meshgrid(ax, ax, ax, indexing="ij", sparse=True)
    for s in range(scans):
        a, b, c = 0.30 + 0.1 * rng.random(3)
        r2 = (ii / (a * size)) ** 2 + (jj / (b * size)) ** 2 + (kk / (c * size)) ** 2
        lab = np.where(r2 < 1.0, 1.0, 0.0)
        if n_classes > 2:
            lab = lab + np.where(r2 < 0.35, 1.0, 0.0)
        img = rng.random((size, size, size)) * 200.0 + lab * 300.0
        vols[f"scan{s}"] = (img, lab)
    return MRI_Dataset("/bench/images", "/bench/labels", n_classes, filter=True, files=sorted(vols),
                       loader=lambda p: vols[os.path.basename(p)][0 if "images" in p else 1], device=device)


def main(argv=None):
    global dir_img, dir_mask
    import json
    import sys
    logging.basicConfig(level=logging.INFO, format="%(levelname)s: %(message)s")
    argv = sys.argv[1:] if argv is None else argv
    args = get_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.nproc > 1 and "WORLD_SIZE" not in os.environ:
        return _relaunch(args.nproc, argv)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    logging.info(f"Using device {device} with properties= {torch.cuda.get_device_properties(device)}")
    filters = [int(f) for f in args.filters.split(",")] if args.filters else None
    if args.net == "unet":
        trainer = UNetTrainer(device, n_channels=args.channels, n_classes=args.classes or 1, load_model=args.load,
                              num_filters=filters)
    elif args.net == "probunet":
        trainer = ProbUNetTrainer(device, n_channels=args.channels, n_classes=args.classes or 3, load_model=args.load,
                                  latent_dim=6, beta=10, num_filters=filters)
    else:
        raise SystemExit(f"Error! {args.net} is not a valid model")
    if world > 1:  # identical replicas
        for t in list(trainer.net.parameters()) + list(trainer.net.buffers()):
            dist.broadcast(t.data, 0)
        from pmu_hip.engine import invalidate_packs
        invalidate_packs()   # written through .data: invisible to the packed-weight cache
    if args.dir is not None:
        dir_img = os.path.join(args.dir, "images")
        dir_mask = os.path.join(args.dir, "labels")
    dataset = bench_dataset(trainer.net.n_classes, args.bench_size, args.bench_scans, device) if args.bench else None
    stats = [] if args.bench else None
    try:
        train_net(trainer=trainer, epochs=args.epochs, batch_size=args.batchsize, lr=args.lr, lrf=args.lrf,
                  lrp=args.lrp, om=args.om, device=device, val_percent=args.val / 100, dataset=dataset,
                  acc_steps=args.acc_steps, dtype=args.dtype, stats=stats)
    except KeyboardInterrupt:
        torch.save(trainer.net.state_dict(), "INTERRUPTED.pth")
        logging.info("Saved interrupt")
    if stats is not None and int(os.environ.get("RANK", "0")) == 0:
        for st in stats:
            print("TRAIN_BENCH " + json.dumps({"model": args.net, "batch_size": args.batchsize, **st}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
