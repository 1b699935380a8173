"""Data-parallel host logic on CPU with the gloo backend, world size 2 (row e).

Each rank computes its round-robin share of the 8 micro-batches of G7 (c1, 4 slices each) with
loss / (micro-batches per step), as train.py's loop does, and train.allreduce_grads sums them.
The result must equal the reference's single-process accumulation (tests/golden/g7_dp.npz).
Both all-reduce paths are exercised: the flat gradient buffer (grads are views of it, as the HIP
autograd nodes produce them) and the flattened-bucket fallback.  The per-rank gradients here come
from the CPU oracle: the HIP forward/backward needs a GPU, the all-reduce logic under test does not.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, flat, q):
    import sys
    for p in (os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"), ROOT, os.path.dirname(__file__)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        from model import UNet
        from oracle.unet_ref import unet_forward, unet_loss
        from pmu_hip.functions import grad_sink_for
        from train import allreduce_grads, dp_micro_batches, shared_generator
        z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
        net = UNet(1, 1, [16, 32])
        sd = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("init/")}
        net.load_state_dict(sd)
        x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["t"])
        # the 32 samples in order; train.py deals micro-batches of 4 round-robin, 4 per rank per step
        steps, per_rank = dp_micro_batches(list(range(32)), 4, 8, world, rank)
        assert len(steps) == 1 and per_rank == 4
        named = dict(net.named_parameters())
        plist = list(net.parameters())
        keys = list(named)
        params = {k: named[k].detach().clone().requires_grad_(True) for k in keys}
        work = dict(sd)
        work.update(params)
        for mb in steps[0]:
            idx = torch.tensor(mb)
            (unet_loss(unet_forward(work, x[idx], 2, 1), t[idx], 1) / (per_rank * world)).backward()
        if flat:
            sink = grad_sink_for(net, plist)      # views of the flat buffer, as the HIP nodes write them
            for k, p in named.items():
                g = sink.new(p)
                g.copy_(params[k].grad)
                p.grad = g
        else:
            for k, p in named.items():
                p.grad = params[k].grad.clone()
        allreduce_grads(net, plist)
        # every rank must agree on the generator the loop shuffles with
        seed = shared_generator().initial_seed()
        out = {k: p.grad.detach().numpy().copy() for k, p in named.items()}
        q.put((rank, out, seed, [i for st in steps for mb in st for i in mb]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("flat", [True, False])
def test_dp_allreduce_matches_reference_accumulation(flat):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, flat, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
    ref = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("grad/")}
    from helpers import grad_err
    for rank, out, _, _ in res:
        err, key = grad_err({k: torch.from_numpy(out[k]) for k in ref}, ref)
        assert err <= 1e-5, (rank, err, key)
    assert res[0][2] == res[1][2]                          # shared shuffle seed
    assert sorted(res[0][3] + res[1][3]) == list(range(32)) and not set(res[0][3]) & set(res[1][3])


def _bucket_worker(rank, world, port, mode, q):
    """Rank body of the bucketed, backward-overlapped all-reduce (pmu_hip.dp.BucketAllReduce)."""
    import sys
    for p in (os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"), ROOT, os.path.dirname(__file__)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        from model import UNet
        from oracle.unet_ref import unet_forward, unet_loss
        from pmu_hip.dp import BucketAllReduce
        from pmu_hip.functions import grad_sink_for
        from train import dp_micro_batches
        z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
        net = UNet(1, 1, [16, 32])
        sd = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("init/")}
        net.load_state_dict(sd)
        x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["t"])
        steps, per_rank = dp_micro_batches(list(range(32)), 4, 8, world, rank)
        named = dict(net.named_parameters())
        plist = list(net.parameters())
        params = {k: named[k].detach().clone().requires_grad_(True) for k in named}
        work = dict(sd)
        work.update(params)
        for mb in steps[0]:
            idx = torch.tensor(mb)
            (unet_loss(unet_forward(work, x[idx], 2, 1), t[idx], 1) / (per_rank * world)).backward()
        sync = BucketAllReduce(net, bucket_bytes=16 << 10)   # several buckets on this small net
        nb = len(sync.buckets)
        # 2 rounds: the buffer and the bucket state are reused from step to step
        for _ in range(2):
            for p in plist:
                p.grad = None
            sync.begin()
            order = list(named.items())
            if mode != "forward_order":
                order = order[::-1]                     # the order the HIP backward reports layers
            if mode == "foreign":
                for k, p in order:
                    p.grad = params[k].grad.clone()      # accumulated outside the flat buffer
            else:
                sink = grad_sink_for(net, plist)
                for k, p in order:
                    g = sink.new(p)
                    g.copy_(params[k].grad)
                    p.grad = g
                    sink.flush()                          # one layer's gradient kernels enqueued
            issued = sync.issued_in_backward
            sync.finish()
        out = {k: p.grad.detach().numpy().copy() for k, p in named.items()}
        q.put((rank, out, nb, issued))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["backward_order", "forward_order", "foreign"])
def test_dp_bucketed_overlap_matches_reference_accumulation(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
    ref = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("grad/")}
    from helpers import grad_err
    for rank, out, nb, issued in res:
        err, key = grad_err({k: torch.from_numpy(out[k]) for k in ref}, ref)
        assert err <= 1e-5, (mode, rank, err, key)
        assert nb > 2
        if mode == "backward_order":
            assert issued == nb          # every bucket was issued from inside the "backward"
        elif mode == "forward_order":
            assert issued == nb          # the last report completes bucket 0, then all issue in order
        else:
            assert issued == 0           # no flat-buffer sink: nothing issued before finish()
