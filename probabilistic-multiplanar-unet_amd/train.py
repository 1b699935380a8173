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

  the acc micro-batches of an optimizer step are dealt round-robin over the ranks (each rank takes
  max(1, acc_steps // world)), every rank scales its loss by 1 / (micro-batches per step), and one
  SUM all-reduce of the flat gradient buffer yields exactly the reference's accumulated gradient
  (``dp_micro_batches`` / ``allreduce_grads``; checked against the reference's own accumulation in
  tests/test_dp_gloo.py).  BatchNorm statistics stay per micro-batch, as in the reference.  The
  all-reduce is bucketed and issued during the last micro-batch's backward (pmu_hip.dp;
  PMU_DP_OVERLAP=0 selects the one-shot all-reduce after the backward).
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


def epoch_order(n, world):
    """Shuffled sample order of one epoch: the reference DataLoader's RandomSampler (:47) on one
    rank, a broadcast-seeded permutation shared by all ranks otherwise."""
    if world == 1:
        return list(RandomSampler(range(n)))
    return torch.randperm(n, generator=shared_generator()).tolist()


def dp_micro_batches(order, micro, acc_steps, world, rank):
    """Deal the drop_last micro-batches of one epoch's sample ``order`` to ranks.

    Returns (steps, per_rank_acc): ``steps`` is a list of optimizer steps, each a list of this
    rank's micro-batches (lists of dataset indices).  Every optimizer step consumes
    per_rank_acc * world micro-batches, dealt round-robin (micro-batch k of a step -> rank k % world)."""
    per_rank = max(1, acc_steps // world)
    per_step = per_rank * world
    mbs = [list(order[i:i + micro]) for i in range(0, len(order) - micro + 1, micro)]
    nsteps = len(mbs) // per_step
    steps = []
    for s in range(nsteps):
        group = mbs[s * per_step:(s + 1) * per_step]
        steps.append([group[k] for k in range(rank, per_step, world)])
    return steps, per_rank


def allreduce_grads(net, plist=None):
    """SUM all-reduce of every gradient: one collective over the flat gradient buffer when all
    grads are its views (the HIP autograd nodes arrange that), else one flattened bucket."""
    world, _ = world_info()
    if world == 1:
        return
    from pmu_hip.functions import flat_grad_buffer
    plist = plist if plist is not None else [p for p in net.parameters()]
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


def train_net(trainer, device, epochs=5, batch_size=1, lr=0.001, lrf=0.1, lrp=2, om=0.9, val_percent=0.1,
              save_cp=False, dataset=None):
    from pmu_hip.optim import FusedSGD
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
    acc_steps = 4 if batch_size > 4 else 1
    micro = batch_size // acc_steps
    writer = _writer(f"LRF_{lrf}_LRP_{lrp}_EP_{epochs}_LR_{lr}_BS_{batch_size}") if rank == 0 else _NullWriter()
    global_step = 0
    logging.info(f"Starting training: epochs {epochs}, batch size {batch_size}, lr {lr}, training size {n_train}, "
                 f"validation size {n_val}, checkpoints {save_cp}, device {device}, ranks {world}")
    net = trainer.net
    optimizer = FusedSGD(net.parameters(), lr=lr, momentum=om, clip=0.1)
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "min" if net.n_classes > 1 else "max",
                                                           factor=lrf, patience=lrp)
    plist = list(net.parameters())
    sync = None
    if world > 1 and os.environ.get("PMU_DP_OVERLAP", "1") != "0":
        from pmu_hip.dp import BucketAllReduce
        sync = BucketAllReduce(net)
    for epoch in range(epochs):
        net.train()
        # ---- train phase
        order = [train.indices[i] for i in epoch_order(n_train, world)]
        steps, per_rank = dp_micro_batches(order, micro, acc_steps, world, rank)
        scale = 1.0 / (per_rank * world)
        optimizer.zero_grad()
        for step_mbs in steps:
            for i, mb in enumerate(step_mbs):
                b = dataset.get_batch(mb)
                imgs = b["image"]
                true_masks = b["mask"].to(dtype=trainer.mask_type)
                masks_pred = trainer.predict(imgs, true_masks)
                loss = trainer.loss(imgs, true_masks, masks_pred) * scale
                if sync is not None and i == len(step_mbs) - 1:
                    sync.begin()      # the last micro-batch's backward issues the bucket all-reduces
                loss.backward()
            if sync is not None:
                sync.finish()
            else:
                allreduce_grads(net, plist)
            optimizer.step()
            optimizer.zero_grad()
            writer.add_scalar("Loss/train", loss.item(), global_step)
            global_step += 1
        # ---- validation phase (every rank evaluates the full validation split)
        net.eval()
        val_batches = [list(val.indices[i:i + micro]) for i in range(0, n_val - micro + 1, micro)] if micro else []
        dices, dice_sums, loss_sum = 0, np.zeros(max(0, net.n_classes - 1)), 0.0
        for mb in val_batches:
            b = dataset.get_batch(mb)
            imgs, true_masks = b["image"], b["mask"].to(dtype=trainer.mask_type)
            with torch.no_grad():
                masks_pred = trainer.predict(imgs, true_masks)
                dice = trainer.eval(imgs, true_masks, masks_pred)
                loss_sum += trainer.loss(imgs, true_masks, masks_pred).item()
            if net.n_classes > 1:
                dice_sums += dice
            else:
                dices += dice
        val_count = max(1, len(val_batches))
        avg_loss = loss_sum / val_count
        writer.add_scalar("Loss/validation", avg_loss, global_step)
        for c in range(net.n_classes - 1):
            writer.add_scalar(f"dice/class_{c + 1}", dice_sums[c] / val_count, global_step)
        val_score = (dices / val_count)[0] if net.n_classes == 1 and val_batches else avg_loss
        scheduler.step(val_score)
        if rank == 0:
            os.makedirs(dir_checkpoint, exist_ok=True)
            torch.save(net.state_dict(), os.path.join(dir_checkpoint, trainer.name + f"_checkpoint{epoch}.pt"))
            logging.info(f"Saved model {trainer.name}_checkpoint{epoch}.pt")
        gc.collect()
    if rank == 0:
        torch.save(net.state_dict(), os.path.join(dir_checkpoint, trainer.name + "_model.pt"))
        logging.info(f"Saved model {trainer.name}_model.pt")
    writer.close()


def get_args():
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
    return parser.parse_args()


def main():
    global dir_img, dir_mask
    logging.basicConfig(level=logging.INFO, format="%(levelname)s: %(message)s")
    args = get_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    logging.info(f"Using device {device} with properties= {torch.cuda.get_device_properties(device)}")
    if args.net == "unet":
        trainer = UNetTrainer(device, n_channels=1, n_classes=1, load_model=args.load)
    elif args.net == "probunet":
        trainer = ProbUNetTrainer(device, n_channels=1, n_classes=3, load_model=args.load, latent_dim=6, beta=10)
    else:
        raise SystemExit(f"Error! {args.net} is not a valid model")
    if world > 1:  # identical replicas
        for t in list(trainer.net.parameters()) + list(trainer.net.buffers()):
            dist.broadcast(t.data, 0)
    if args.dir is not None:
        dir_img = os.path.join(args.dir, "images")
        dir_mask = os.path.join(args.dir, "labels")
    try:
        train_net(trainer=trainer, epochs=args.epochs, batch_size=args.batchsize, lr=args.lr, lrf=args.lrf,
                  lrp=args.lrp, om=args.om, device=device, val_percent=args.val / 100)
    except KeyboardInterrupt:
        torch.save(trainer.net.state_dict(), "INTERRUPTED.pth")
        logging.info("Saved interrupt")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
