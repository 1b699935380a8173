"""Data-parallel host logic on CPU with the gloo backend, world sizes 2, 4 and 8 (row e).

Each rank computes its share of the micro-batches of one optimizer step as train.py deals them
(micro-batch k -> rank k % world, loss / acc_steps), and the all-reduce sums them.  The result must
equal the reference's single-process accumulation: G7 (tests/golden/g7_dp.npz: 8 micro-batches of
4 slices, loss / 8, produced by the reference itself), and for world > acc_steps (idle ranks) the
oracle's accumulation of 2 micro-batches (the oracle is pinned to G1/G7).  Paths exercised: the
one-shot flat-buffer all-reduce, the flattened fallback, and the bucketed all-reduce overlapped
with the backward (pmu_hip.dp.BucketAllReduce) replaying the HIP backward's report order
(engine.unet_report_order).  The per-rank gradients come from the CPU oracle: the HIP backward
needs a GPU, the exchange logic under test does not.
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


def _setup(rank, world, port):
    import sys
    for p in (os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"), ROOT, os.path.dirname(__file__)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def _local_grads(net, sd, x, t, mbs, acc):
    """This rank's summed gradients of its micro-batches, loss / acc each (oracle fwd/bwd)."""
    from oracle.unet_ref import unet_forward, unet_loss
    named = dict(net.named_parameters())
    params = {k: named[k].detach().clone().requires_grad_(True) for k in named}
    work = dict(sd)
    work.update(params)
    for mb in mbs:
        idx = torch.tensor(mb)
        (unet_loss(unet_forward(work, x[idx], 2, 1), t[idx], 1) / acc).backward()
    return {k: (params[k].grad if params[k].grad is not None else None) for k in named}


def _g7_net():
    from model import UNet
    z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
    net = UNet(1, 1, [16, 32])
    sd = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("init/")}
    net.load_state_dict(sd)
    return net, sd, torch.from_numpy(z["x"]), torch.from_numpy(z["t"])


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def _reference(acc):
    """G7's gradients (acc = 8), or the oracle's accumulation of G7's first `acc` micro-batches."""
    z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
    if acc == 8:
        return {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("grad/")}
    net, sd, x, t = _g7_net()
    g = _local_grads(net, sd, x, t, [list(range(4 * i, 4 * i + 4)) for i in range(acc)], acc)
    return g


# ------------------------------------------------------------------------ one-shot all-reduce
def _flat_worker(rank, world, port, q, flat, acc):
    _setup(rank, world, port)
    try:
        from pmu_hip.functions import grad_sink_for
        from train import allreduce_grads, dp_micro_batches, shared_generator
        net, sd, x, t = _g7_net()
        steps, leftover = dp_micro_batches(list(range(4 * acc)), 4, acc, world, rank)
        assert len(steps) == 1 and not leftover
        mbs = steps[0]
        assert len(mbs) == len(range(rank, acc, world))
        named = dict(net.named_parameters())
        plist = list(net.parameters())
        idle = not mbs
        if not idle:
            g = _local_grads(net, sd, x, t, mbs, acc)
            if flat:
                sink = grad_sink_for(net, plist)      # views of the flat buffer, as the HIP nodes write them
                for k, p in named.items():
                    v = sink.new(p)
                    v.copy_(g[k])
                    p.grad = v
            else:
                for k, p in named.items():
                    p.grad = g[k].clone()
        allreduce_grads(net, plist, idle=idle)
        seed = shared_generator().initial_seed()   # every rank must agree on the shuffle generator
        out = {k: p.grad.detach().numpy().copy() for k, p in named.items()}
        q.put((rank, out, seed, [i for mb in mbs for i in mb]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,acc,flat", [(2, 8, True), (2, 8, False), (4, 8, True), (8, 8, True),
                                            (3, 8, True), (4, 2, True)])
def test_dp_allreduce_matches_reference_accumulation(world, acc, flat):
    res = _run(_flat_worker, world, flat, acc)
    ref = _reference(acc)
    from helpers import grad_err
    for rank, out, _, _ in res:
        err, key = grad_err({k: torch.from_numpy(out[k]) for k in ref}, ref)
        assert err <= 1e-5, (rank, err, key)
    assert len({r[2] for r in res}) == 1                       # shared shuffle seed
    seen = [i for r in res for i in r[3]]
    assert sorted(seen) == list(range(4 * acc)) and len(set(seen)) == len(seen)


# ------------------------------------------------------------------------ bucketed, overlapped
def _bucket_worker(rank, world, port, q, mode, acc):
    _setup(rank, world, port)
    try:
        from pmu_hip.dp import BucketAllReduce
        from pmu_hip.engine import unet_report_order
        from pmu_hip.functions import grad_sink_for
        from train import dp_micro_batches
        net, sd, x, t = _g7_net()
        steps, _ = dp_micro_batches(list(range(4 * acc)), 4, acc, world, rank)
        mbs = steps[0]
        named = dict(net.named_parameters())
        plist = list(net.parameters())
        g = _local_grads(net, sd, x, t, mbs, acc) if mbs else None
        name_of = {id(p): k for k, p in named.items()}
        groups = unet_report_order(net)
        if mode == "forward_order":
            groups = groups[::-1]
        sync = BucketAllReduce(net, bucket_bytes=16 << 10)   # several buckets on this small net
        log = []
        # 3 rounds: round 0 learns the layout, later rounds reuse buffer and bucket state
        for rnd in range(3):
            for p in plist:
                if mode == "kept" and p.grad is not None:
                    p.grad.zero_()       # zero_grad(set_to_none=False): round 0's old-layout views survive
                else:
                    p.grad = None
            sync.begin()
            if g is not None:
                if mode == "kept" and rnd > 0:
                    sink = grad_sink_for(net, plist)
                    assert not sink.flat                     # .grad exists: autograd accumulates into it
                    for grp in groups:
                        for p in grp:
                            v = sink.new(p)
                            v.copy_(g[name_of[id(p)]])
                            p.grad.add_(v)
                        sink.flush()
                elif mode == "foreign":
                    for p in plist:
                        p.grad = g[name_of[id(p)]].clone()   # accumulated outside the flat buffer
                elif mode == "accumulated":
                    # several micro-batches per rank: the earlier backward left flat-buffer .grad views
                    # (here zeros), so the last one's sink hands out plain tensors that autograd adds in
                    first = grad_sink_for(net, plist)
                    for p in plist:
                        p.grad = first.new(p).zero_()
                    sink = grad_sink_for(net, plist)
                    assert not sink.flat
                    for grp in groups:
                        for p in grp:
                            v = sink.new(p)
                            v.copy_(g[name_of[id(p)]])
                            p.grad.add_(v)
                        sink.flush()                         # reports the order, issues nothing
                else:
                    sink = grad_sink_for(net, plist)
                    for grp in groups:
                        for p in grp:
                            v = sink.new(p)
                            v.copy_(g[name_of[id(p)]])
                            p.grad = v
                        sink.flush()                         # one layer's gradient kernels enqueued
            log.append((sync.issued_in_backward, sync.issued_at[0] if sync.issued_at else None, sync.flushes,
                        len(sync.buckets or [])))
            sync.finish(idle=g is None)
            out = {k: p.grad.detach().numpy().copy() for k, p in named.items()}
        # after the relayout the buffer's pads (and slots without a gradient) hold zeros, not the
        # first layout's stale values
        from pmu_hip.functions import _offsets, _slot, flat_grad_buffer
        buf, offs = flat_grad_buffer(net, plist), _offsets(net, plist)
        pad = sum(float(buf[offs[id(p)] + p.numel():offs[id(p)] + _slot(p.numel())].abs().sum()) for p in plist)
        q.put((rank, out, log + [pad]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,world,acc", [("backward_order", 2, 8), ("forward_order", 2, 8), ("foreign", 2, 8),
                                            ("accumulated", 2, 8), ("kept", 2, 8),
                                            ("backward_order", 4, 8), ("backward_order", 8, 8),
                                            ("backward_order", 4, 2)])
def test_dp_bucketed_overlap_matches_reference_accumulation(mode, world, acc):
    res = _run(_bucket_worker, world, mode, acc)
    ref = _reference(acc)
    from helpers import grad_err
    for rank, out, log in res:
        err, key = grad_err({k: torch.from_numpy(out[k]) for k in ref}, ref)
        assert err <= 1e-5, (mode, rank, err, key)
        log, pad = log[:-1], log[-1]
        assert pad == 0.0, (mode, rank, pad)
        issued0, _, _, nb0 = log[0]
        assert issued0 == 0 and nb0 == 0            # round 0 records the report order
        for issued, first, flushes, nb in log[1:]:
            if mode == "foreign":                     # no flat-buffer reports: nothing to learn
                assert issued == 0 and nb == 0
                continue
            assert nb > 2
            busy = rank < acc
            if mode == "backward_order" and busy:
                assert issued == nb                   # every bucket issued from inside the "backward"
                assert first is not None and first < flushes // 2   # bucket 0 long before the end
            elif mode == "forward_order" and busy:
                assert issued == nb                   # the layout follows the learned (reversed) order too
            elif mode in ("accumulated", "kept"):
                assert issued == 0                    # learned from plain-sink reports; exchanged at finish()
            else:
                assert issued == 0                    # foreign grads / idle rank: all at finish()


# ------------------------------------------------------------------------ train_net itself (config c3)
def _train_net_worker(rank, world, port, q, acc, overlap, ckpt_dir):
    os.environ["PMU_DP_OVERLAP"] = overlap
    _setup(rank, world, port)
    try:
        import train as T
        from torch.utils.data import Subset
        from oracle.unet_ref import trainer_dice, unet_forward, unet_loss
        net, sd, x, t = _g7_net()
        seen = []

        class G7Slices:
            """G7's 32 slices behind MRI_Dataset's batch interface (get_batch)."""
            def __len__(self):
                return x.shape[0]

            def get_batch(self, idx):
                seen.append([int(i) for i in idx])
                i = torch.tensor([int(v) for v in idx])
                return {"image": x[i], "mask": t[i]}

        class OracleTrainer:
            """UNetTrainer's interface on the CPU oracle over the module's own parameters and buffers
            (the HIP forward needs a GPU; the data-parallel logic under test does not)."""
            name, mask_type, device = "unet", torch.float32, torch.device("cpu")

            def __init__(self):
                self.net = net

            def predict(self, imgs, masks):
                return unet_forward(dict(net.state_dict(keep_vars=True)), imgs, 2, 1, training=net.training)

            def loss(self, imgs, masks, pred):
                return unet_loss(pred, masks, 1)

            def eval(self, imgs, masks, pred):
                return np.array(trainer_dice(pred, masks, 1))

        class ClipSGD(torch.optim.SGD):
            """clip_grad_value_(0.1) + SGD(momentum) (PMU/train.py:65,108-110) on CPU tensors."""
            def step(self, closure=None):
                torch.nn.utils.clip_grad_value_([p for g in self.param_groups for p in g["params"]], 0.1)
                return super().step(closure)

        # G7's micro-batch grouping: the split and the epoch order are identities here (the seeded
        # shuffles are tested elsewhere), so micro-batch k is slices 4k..4k+3, as G7 accumulates them
        T.random_split = lambda ds, lengths, generator=None: [Subset(ds, list(range(lengths[0]))),
                                                              Subset(ds, list(range(lengths[0], sum(lengths))))]
        T.epoch_order = lambda n, world: list(range(n))
        T.dir_checkpoint = ckpt_dir + "/"
        stats = []
        T.train_net(OracleTrainer(), torch.device("cpu"), epochs=1, batch_size=4 * acc, lr=0.1, val_percent=0.0,
                    dataset=G7Slices(), acc_steps=acc, stats=stats,
                    optimizer_factory=lambda ps: ClipSGD(ps, lr=0.1, momentum=0.9))
        out = {k: p.detach().numpy().copy() for k, p in net.named_parameters()}
        q.put((rank, out, seen, stats))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,overlap", [(8, "1"), (8, "0"), (4, "1")])
def test_train_net_dp_matches_reference_step(world, overlap, tmp_path):
    """train.py's train_net on `world` gloo ranks with acc_steps=8, batch 32 (config c3's shape, 8
    micro-batches of 4): every rank trains (at world 8 exactly one micro-batch per rank, no idle
    rank) and the replicas end the step on the parameters of the reference's single-process step —
    G7's accumulated gradient (8 micro-batches, loss / 8), clip_grad_value_(0.1), SGD(0.1, 0.9)."""
    acc = 8
    res = _run(_train_net_worker, world, acc, overlap, str(tmp_path))
    z = np.load(os.path.join(GOLD, "g7_dp.npz"), allow_pickle=False)
    init = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("init/")}
    grads = {k[5:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("grad/")}
    from oracle.unet_ref import sgd_clip_step
    params = {k: init[k].clone() for k in grads}
    sgd_clip_step(params, grads, {k: torch.zeros_like(v) for k, v in params.items()}, 0.1)
    for rank, out, seen, stats in res:
        assert len(seen) == acc // world, (rank, seen)          # no idle rank, an equal share each
        assert [sorted(mb) for mb in seen] == [list(range(4 * k, 4 * k + 4)) for k in range(rank, acc, world)]
        for k, want in params.items():
            d = float((torch.from_numpy(out[k]) - want).abs().max())
            assert d <= 1e-6, (rank, k, d)
        assert stats and stats[0]["slices"] == 32 and stats[0]["optimizer_steps"] == 1
