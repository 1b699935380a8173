"""Rehearsal of the overlapped data-parallel step on ONE GPU (row e): N ranks share cuda:0 over gloo.

Each rank runs the HIP forward/backward of a small UNet on its own batch twice: once alone (its
local gradient) and once with pmu_hip.dp.BucketAllReduce issuing the bucket all-reduces from
inside the backward.  The synchronised gradient must equal the sum of all ranks' local gradients
(all-gathered), on every rank.  Launch:

  PMU_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 tools/dp_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # gloo: N ranks sharing cuda:0; nccl (RCCL): one rank per device, so on a 1-GPU box world 1 — the
    # real RCCL communicator and collectives under the overlapped buckets
    backend = os.environ.get("PMU_DIST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    cdev = dev if backend == "nccl" else torch.device("cpu")   # RCCL collectives take device tensors
    from model import UNet
    from pmu_hip.dp import BucketAllReduce
    torch.manual_seed(0)
    net = UNet(1, 2, [16, 32, 64]).to(dev).train()
    plist = list(net.parameters())
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.rand(4, 1, 64, 64, generator=g).to(dev)
    t = torch.randint(0, 2, (4, 64, 64), generator=g).to(dev)
    crit = torch.nn.CrossEntropyLoss()

    def backward():
        for p in plist:
            p.grad = None
        crit(net(x), t).backward()

    # local gradient (BN running stats move; the weights do not, so both passes see the same net)
    backward()
    local = torch.cat([p.grad.reshape(-1) for p in plist]).to(cdev)
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    want = allg[0].clone()
    for a in allg[1:]:
        want += a
    want = want.cpu()
    from pmu_hip.engine import unet_report_order
    sync = BucketAllReduce(net, bucket_bytes=64 << 10)
    # the backward's real report order, seen through the reducer's flush callback
    reports = []
    orig = net.__dict__["_pmu_grad_ready"]
    net.__dict__["_pmu_grad_ready"] = lambda ps, flat=True: (reports.append([id(p) for p in ps]), orig(ps, flat))
    ok = True
    for it in range(3):
        for p in plist:
            p.grad = None
        reports.clear()
        sync.begin()
        crit(net(x), t).backward()
        issued, first, flushes = sync.issued_in_backward, (sync.issued_at or [None])[0], sync.flushes
        sync.finish()
        torch.cuda.synchronize()
        got = torch.cat([p.grad.reshape(-1) for p in plist]).cpu()
        err = (got - want).abs().max().item()
        buf = net.__dict__["_pmu_grad_flat"]
        adopted = all(buf.data_ptr() <= p.grad.data_ptr() < buf.data_ptr() + 4 * buf.numel() for p in plist)
        order_ok = reports == [[id(p) for p in grp] for grp in unet_report_order(net)]
        nb = len(sync.buckets)
        print(f"rank {rank} iter {it}: buckets {nb} issued in backward {issued} (bucket 0 at flush {first} of "
              f"{flushes}) max|sync - sum(local)| {err:.3e} adopted {adopted} report order {order_ok}", flush=True)
        ok = ok and err == 0.0 and adopted and order_ok
        if it > 0:   # the learned layout: every bucket from inside the backward, bucket 0 early
            ok = ok and issued == nb and nb > 2 and first is not None and first < flushes // 2
    flag = torch.tensor([1 if ok else 0], device=cdev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        print("DP_CHECK", backend, "world", world, "OK" if flag.item() == 1 else "FAIL", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if flag.item() == 1 else 1)


if __name__ == "__main__":
    main()
