#!/usr/bin/env python3
"""Throughput benchmark of the reference's headline metric on MI355X.

metric : "2D slices/sec fwd+bwd, 256x256x1 batch32 U-Net; Dice vs ref"  (BASELINE.json)
step   : one training step of PMU/train.py:85-110 on one batch of synthetic 256x256x1 slices:
         UNet(1,1,[64,128,256,512,1024]) forward -> BCELoss -> backward -> (all-reduce) ->
         clip_grad_value_(0.1) + SGD(momentum 0.9), all on the HIP path (model.UNet + FusedSGD).
N GPUs : one process per GPU (torch.distributed.run; `--gpus N` outside torchrun starts the N ranks
         itself as a child process), 32 slices per GPU (weak scaling), one
         RCCL all-reduce of the flat gradient buffer per step.

Prints ONE JSON line on rank 0.  `roofline` is the dominant MFMA kernel family timed with HIP
events on the launch stream during one instrumented step after the timed region;
`cpu_baseline` times the CPU oracle (oracle/unet_ref.py, a torch-CPU restatement of the
reference) per BASELINE.md's protocol (c2: batch 32, 1 warm-up, median of 3 steps, all permitted
host cores; with and without the SGD update), rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "probabilistic-multiplanar-unet_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from pmu_hip._lib import MFMA_ENTRY_POINTS  # noqa: E402  (the table only; the library loads lazily)

METRIC = "2D slices/sec fwd+bwd, 256×256×1 batch32 U-Net; Dice vs ref"
METRIC_C5 = "2D slices/sec fwd+bwd, 512×512×3 batch16 U-Net bf16 (BASELINE.json configs[4])"
METRIC_C4 = ("2D slices/sec ProbabilisticUnet train step (prior+posterior, latent 6, KL+CE) + 16 fcomb samples, "
             "256×256×1 batch32 (BASELINE.json configs[3])")
FP32_MFMA_PEAK_TF = 157.3
BF16_MFMA_PEAK_TF = 2516.0   # dense bf16 MFMA (MI355X_MICROARCH.md; 2.5 PF, no sparsity)
FILTERS = [64, 128, 256, 512, 1024]


def conv_flops_per_slice(H, W, filters, n_ch=1, n_cls=1):
    """Algorithmic FLOPs per slice: 2 x MACs x (fwd + dgrad + wgrad) over every conv, convT and
    the 1x1 head, without the first layer's dgrad."""
    fl = 0.0
    h, w = H, W
    levels = []
    for i, f in enumerate(filters):
        cin = n_ch if i == 0 else filters[i - 1]
        first = 9 * h * w * cin * f * 2          # conv1 fwd
        fl += first * (2 if i == 0 else 3)
        fl += 9 * h * w * f * f * 2 * 3           # conv2
        levels.append((h, w))
        h, w = h // 2, w // 2
    for i in reversed(range(len(filters) - 1)):
        hi, wi = levels[i + 1]
        cin = filters[i + 1]
        fl += hi * wi * cin * (cin // 2) * 4 * 2 * 3          # convT 2x2
        hs, ws = levels[i]
        fl += 9 * hs * ws * (cin) * filters[i] * 2 * 3        # up conv1 (concat input = cin channels)
        fl += 9 * hs * ws * filters[i] * filters[i] * 2 * 3   # up conv2
    fl += H * W * filters[0] * n_cls * 2 * 3                  # outc
    return fl


class KernelTimer:
    """HIP-event timing of every launch, with algorithmic FLOPs for the MFMA kernels."""

    MFMA = MFMA_ENTRY_POINTS   # pmu_hip._lib: every C-ABI entry whose kernels issue MFMAs

    @staticmethod
    def _base(name):
        """The call family of a fused variant: the BN-backward epilogue (_bnr), bf16-z (_zb), concat-split
        bf16 copy / column-sum (_x1b, _x1b_sum) and in-place concat (_ld, _ldb) forms take the same
        leading arguments and do the same MFMA work as the plain call."""
        if name.endswith("_dxb"):   # bf16-dx storage of the same GEMM
            name = name[:-4]
        for suf in ("_bnr_zb", "_x1b_sum", "_x1b", "_bnr", "_zb", "_ldb", "_ld"):
            if name.endswith(suf):
                return name[: -len(suf)]
        return name

    def __init__(self):
        self.rec = []

    @staticmethod
    def _flops(name, args):
        name = KernelTimer._base(name)
        if name == "pmu_conv3x3_wgrad_wino4":
            N, H, W, cout, cin = args[2], args[3], args[4], args[5], args[6]
            return 2.0 * 36 * N * ((H + 3) // 4) * ((W + 3) // 4) * cin * cout
        if name in ("pmu_conv3x3_fwd_dma", "pmu_conv3x3_dgrad_dma"):
            cp, N, H, W, nout = args[1], args[2], args[3], args[4], args[7] if name.endswith("fwd_dma") else args[6]
            return 2.0 * N * H * W * cp * nout * 9
        if name == "pmu_convT2x2_fwd_dma":
            N, H, W, cin, cout = args[2], args[3], args[4], args[7], args[8]
            return 2.0 * N * H * W * cin * cout * 4
        if name == "pmu_convT2x2_dgrad_dma":
            N, H, W, cin, cout = args[7], args[8], args[9], args[10], args[11]
            return 2.0 * N * H * W * cin * cout * 4
        if name in ("pmu_conv3x3_fwd_wino4", "pmu_conv3x3_dgrad_wino4"):
            # Winograd F(4x4,3x3): 36 products per 4x4 output tile per channel pair
            cin, N, H, W = args[1], args[2], args[3], args[4]
            nout = args[7] if name.startswith("pmu_conv3x3_fwd") else args[6]
            return 2.0 * 36 * N * ((H + 3) // 4) * ((W + 3) // 4) * cin * nout
        if name in ("pmu_conv3x3_fwd_wino_raw", "pmu_conv3x3_dgrad_wino_raw", "pmu_conv3x3_fwd_wino2h",
                    "pmu_conv3x3_dgrad_wino2h"):
            cin, N, H, W = args[1], args[2], args[3], args[4]
            nout = args[7] if name.startswith("pmu_conv3x3_fwd") else args[6]
            return 2.0 * 16 * N * ((H + 1) // 2) * ((W + 1) // 2) * cin * nout
        if name == "pmu_conv3x3_wgrad_wino":
            N, H, W, cout, cin = args[2], args[3], args[4], args[5], args[6]
            return 2.0 * 16 * N * ((H + 1) // 2) * ((W + 1) // 2) * cin * cout
        if name in ("pmu_conv3x3_fwd_wino", "pmu_conv3x3_dgrad_wino"):
            # Winograd F(2x2,3x3): 16 products per 2x2 output tile per channel pair (the MFMA work of
            # the algorithm; the direct sum it replaces is 36)
            f = args[0]._obj
            cframe = sum(f.src[i].C for i in range(f.nsrc))
            nout = args[3] if name.endswith("fwd_wino") else args[2]
            return 2.0 * 16 * f.N * ((f.H + 1) // 2) * ((f.W + 1) // 2) * cframe * nout
        if name == "pmu_conv3x3_fwd_bf16":
            f = args[0]._obj
            return 2.0 * f.N * f.H * f.W * sum(f.src[i].C for i in range(f.nsrc)) * args[3] * 9
        if name == "pmu_conv3x3_dgrad_bf16":
            f = args[0]._obj
            return 2.0 * f.N * f.H * f.W * f.src[0].C * args[2] * 9
        if name in ("pmu_conv3x3_wgrad_bf16", "pmu_conv3x3_wgrad_bf16_dma"):
            N, H, W, cout, cin = args[2], args[3], args[4], args[5], args[6]
            return 2.0 * N * H * W * cin * cout * 9
        if name in ("pmu_conv3x3_fwd_raw", "pmu_conv3x3_dgrad_raw"):
            cp, N, H, W, nout = args[1], args[2], args[3], args[4], args[7] if name.endswith("fwd_raw") else args[6]
            return 2.0 * N * H * W * cp * nout * 9
        if name == "pmu_convT2x2_wgrad_bf16":
            N, H, W, cin, cout = args[3], args[4], args[5], args[10], args[11]
            return 2.0 * N * H * W * cin * cout * 4
        if name == "pmu_convT2x2_fwd_bf16":
            f = args[0]._obj
            return 2.0 * f.N * f.H * f.W * f.src[0].C * args[3] * 4
        if name == "pmu_convT2x2_dgrad_bf16":
            N, H, W, cin, cout = args[6], args[7], args[8], args[9], args[10]
            return 2.0 * N * H * W * cin * cout * 4
        if name in ("pmu_conv3x3_fwd", "pmu_conv3x3_dgrad", "pmu_conv3x3_wgrad"):
            f = args[0]._obj
            cframe = sum(f.src[i].C for i in range(f.nsrc))
            if name == "pmu_conv3x3_fwd":
                cin, cout = cframe, args[4]
            elif name == "pmu_conv3x3_dgrad":
                cout, cin = cframe, args[3]
            else:
                a = args[1]._obj
                cin, cout = sum(a.src[i].C for i in range(a.nsrc)), args[2]
            return 2.0 * f.N * f.H * f.W * cin * cout * 9
        if name == "pmu_convT2x2_fwd":
            f = args[0]._obj
            cin = sum(f.src[i].C for i in range(f.nsrc))
            return 2.0 * f.N * f.H * f.W * cin * args[4] * 4
        if name == "pmu_convT2x2_dgrad":
            N, H, W, cin, cout = args[7], args[8], args[9], args[10], args[11]
            return 2.0 * N * H * W * cin * cout * 4
        if name == "pmu_convT2x2_wgrad":
            a = args[5]._obj
            cin = sum(a.src[i].C for i in range(a.nsrc))
            return 2.0 * a.N * a.H * a.W * cin * args[6] * 4
        return fcomb_flops(name, args)

    @staticmethod
    def _direct(name, args, fl):
        """The direct-sum FLOPs of a launch: a Winograd F(2x2,3x3) launch executes 16
        products per 2x2 output tile and channel pair where the direct sum takes 9 per pixel."""
        name = KernelTimer._base(name)
        if "_wino" not in name or not fl:
            return fl
        if name.endswith("_wino4"):
            H, W = args[3], args[4]
            return fl * (9.0 * H * W) / (36.0 * ((H + 3) // 4) * ((W + 3) // 4))
        if name in ("pmu_conv3x3_fwd_wino_raw", "pmu_conv3x3_dgrad_wino_raw", "pmu_conv3x3_fwd_wino2h",
                    "pmu_conv3x3_dgrad_wino2h"):
            H, W = args[3], args[4]
        elif name == "pmu_conv3x3_wgrad_wino":
            H, W = args[3], args[4]
        else:
            f = args[0]._obj
            H, W = f.H, f.W
        return fl * (9.0 * H * W) / (16.0 * ((H + 1) // 2) * ((W + 1) // 2))

    def __call__(self, name, args, e0, e1):
        fl = self._flops(name, args)
        self.rec.append((name, fl, self._direct(name, args, fl), e0, e1))

    def summary(self):
        """{name: [launches, executed MFMA FLOPs, seconds, direct-sum FLOPs]}"""
        torch.cuda.synchronize()
        per = {}
        for name, fl, dfl, e0, e1 in self.rec:
            t = e0.elapsed_time(e1) * 1e-3
            d = per.setdefault(name, [0, 0.0, 0.0, 0.0])
            d[0] += 1
            d[1] += fl
            d[2] += t
            d[3] += dfl
        return per


def host_cpu():
    """(threads to use, description) of the host cores this process may run on: the affinity set,
    capped by a cgroup CPU quota when one is set (a GPU box grants a share of a bigger machine)."""
    total = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = total
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    threads = min(avail, quota) if quota else avail
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"cpu_model": model, "os_cpu_count": total, "affinity_cpus": avail, "cgroup_cpu_quota": quota}


def cpu_baseline(workload="unet", size=256, channels=1, classes=1, batch=32, steps=3):
    """CPU oracle (torch-CPU restatement of the reference) timed per BASELINE.md's protocol: the bench
    geometry at ``batch`` (c2: 32, the GPU batch), seeded weights (0) and input (1), 1 warm-up step,
    then the median of ``steps`` steps, on every host core this process may use; the UNet step is
    reported with and without its clip+SGD update.  The reference's CPU path is fp32 only, so the c5
    (bf16) sample is fp32."""
    from oracle.unet_ref import sgd_clip_step, unet_param_keys, unet_train_step
    from oracle.probunet_ref import probunet_train_step
    threads, host = host_cpu()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(1)
    B = batch
    x = torch.rand(B, channels, size, size, generator=g)
    if workload == "unet":
        from model import UNet
        sd = {k: v.clone() for k, v in UNet(channels, classes, FILTERS).state_dict().items()}
        if classes == 1:
            t = (torch.rand(B, 1, size, size, generator=g) > 0.5).float()
        else:
            t = torch.randint(0, classes, (B, 1, size, size), generator=g)
        keys = unet_param_keys(sd)
        bufs = {k: torch.zeros_like(sd[k]) for k in keys}

        def one():
            t0 = time.perf_counter()
            _, _, grads = unet_train_step(sd, x, t, 5, classes)
            t1 = time.perf_counter()
            cur = {k: sd[k].detach() for k in keys}
            sgd_clip_step(cur, grads, bufs, 1e-3)
            sd.update(cur)
            return t1 - t0, time.perf_counter() - t0
        what = "UNet fwd+loss+bwd+clip+SGD steps"
    else:
        from model import ProbabilisticUnet
        net = ProbabilisticUnet(channels, classes, FILTERS, latent_dim=6, no_convs_fcomb=4, beta=10.0)
        sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
        del net
        segm = torch.randint(0, classes, (B, 1, size, size), generator=g).float()
        eps = torch.randn(B, 6, generator=g)

        def one():
            t0 = time.perf_counter()
            probunet_train_step(sd, x, segm, eps, 5, 6, classes, 4, 10.0)
            dt = time.perf_counter() - t0
            return dt, dt
        what = "ProbabilisticUnet fwd+elbo+bwd steps (no optimizer, no eval samples)"
    one()  # warm-up
    times = sorted(one() for _ in range(steps))
    fb = sorted(t[0] for t in times)[len(times) // 2]
    full = sorted(t[1] for t in times)[len(times) // 2]
    res = {"value": round(B / full, 4), "unit": "slices/s", "cores": threads, "kind": "port",
           "sample": f"oracle/{'unet' if workload == 'unet' else 'probunet'}_ref.py torch-CPU fp32, "
                     f"{size}x{size}x{channels}, {classes} class(es), filters {FILTERS}, batch {B}, median of "
                     f"{steps} {what} after 1 warm-up, {threads} threads",
           "ms_per_step": round(full * 1e3, 1)}
    if workload == "unet":
        res["value_without_sgd"] = round(B / fb, 4)
    res.update(host)
    return res


def cpu_leg(args, step):
    """The bench's CPU-oracle leg (rank 0, N=1, after the timed region): the oracle as the checker
    of the bench batch (``dice_vs_ref``) and the timed CPU baseline.  The only place bench.py
    touches oracle/."""
    dvr = None
    if args.workload != "probunet":
        xb, tb = step.batch()
        dvr = dice_vs_ref(step.net, xb, tb, args.classes, args.precision)
    else:
        dvr = dice_vs_ref_probunet(step.net, *step.batch())
    # c2: BASELINE.md's protocol (batch 32, median of 3); c4 / c5 at a bounded batch (a batch-32 c4 or
    # batch-16 c5 step takes 30-40 s on the box's 16 host threads)
    cpu_batch = {"unet": 32, "probunet": 32, "c5": 2}[args.workload] if args.batch >= 8 else args.batch
    cpu = cpu_baseline(workload="probunet" if args.workload == "probunet" else "unet", size=args.size,
                       channels=args.channels, classes=3 if args.workload == "probunet" else args.classes,
                       batch=cpu_batch)
    return cpu, dvr


def dice_vs_ref_probunet(net, x, segm, n=8):
    """c4's "Dice vs ref": the HIP ProbabilisticUnet's reconstruction (forward(training=True) + elbo
    with the posterior sample mu + sigma * eps, eps seeded and injected on both sides, as
    tests/test_probunet_gpu.py does) on the first ``n`` slices of the bench batch vs the fp32 CPU
    oracle's (oracle/probunet_ref.py) for the same weights: argmax label maps per class, label
    agreement, Dice of each side against segm, loss and reconstruction deltas."""
    from oracle.probunet_ref import probunet_forward_loss
    from oracle.unet_ref import dice_coeff
    threads, _ = host_cpu()
    torch.set_num_threads(threads)
    x, segm = x[:n], segm[:n]
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    eps = torch.randn(x.shape[0], 6, generator=torch.Generator().manual_seed(7))
    with torch.no_grad():
        net.forward(x, segm, training=True)
        d = net.posterior_latent_space
        d.rsample = lambda sample_shape=torch.Size(): d.base_dist.loc + d.base_dist.scale * eps.to(x.device)
        loss = float(-net.elbo(segm))
        y = net.reconstruction.float().cpu()
        res = probunet_forward_loss(sd, x.cpu(), segm.cpu(), eps, len(FILTERS), 6, 3, 4, 10.0)
    yr = res["rec"].float()
    lab, labr, tgt = y.argmax(1), yr.argmax(1), segm.cpu()[:, 0].long()
    ks = [1, 2]
    def dc(a, b):
        return float(dice_coeff(a.float(), b.float()))
    to_t = [dc(lab == k, tgt == k) for k in ks]
    to_tr = [dc(labr == k, tgt == k) for k in ks]
    return {"classes": ks, "dice_hip_vs_oracle_labels": [round(dc(lab == k, labr == k), 6) for k in ks],
            "label_agreement": round(float((lab == labr).float().mean()), 7),
            "dice_to_target_hip": [round(v, 6) for v in to_t], "dice_to_target_oracle": [round(v, 6) for v in to_tr],
            "max_abs_dice_delta": float(max(abs(a - b) for a, b in zip(to_t, to_tr))),
            "max_abs_output_delta": float((y - yr).abs().max()),
            "loss_rel_delta": abs(loss - float(res["loss"])) / abs(float(res["loss"])),
            "precision": "fp32", "oracle": "oracle/probunet_ref.py torch-CPU fp32",
            "sample": f"the first {x.shape[0]} slices of the bench batch after the timed steps, train mode, "
                      "posterior noise injected (seeded)"}


def dice_vs_ref(net, x, t, classes, precision):
    """The "Dice vs ref" half of the headline metric (BASELINE.json): the HIP network's prediction on
    the bench batch vs the fp32 CPU oracle's (oracle/unet_ref.py) for the same weights and input,
    both in train mode (BatchNorm batch statistics) as in the timed step.  Label maps: (p > 0.5) for
    one class (the trainer's eval, unet_trainer.py:39-58), softmax argmax otherwise.  Reported: per
    class the Dice of the HIP labels against the oracle's labels, the label agreement, each side's
    Dice against the target (trainer eval) and their difference."""
    from oracle.unet_ref import dice_coeff, unet_forward
    threads, _ = host_cpu()
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    with torch.no_grad():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=precision == "bf16"):
            y = net(x).float().cpu()
        yr = unet_forward(sd, x.cpu(), len(FILTERS), classes)
    tc = t.cpu()
    if classes == 1:
        lab, labr, tgt, ks = (y > 0.5).long()[:, 0], (yr > 0.5).long()[:, 0], tc[:, 0].long(), [1]
    else:
        lab, labr = y.argmax(1), yr.argmax(1)
        tgt, ks = tc.reshape(lab.shape).long(), list(range(1, classes))
    def d(a, b):
        return float(dice_coeff(a.float(), b.float()))
    per = [d(lab == k, labr == k) for k in ks]
    to_t = [d(lab == k, tgt == k) for k in ks]
    to_tr = [d(labr == k, tgt == k) for k in ks]
    # label flips, and how many of them sit at an fp32 tie (the oracle's decision margin below 1e-5:
    # |p - 0.5| for one class, the top-two logit gap otherwise), where either evaluation order may win
    flip = lab != labr
    if classes == 1:
        margin = (yr[:, 0] - 0.5).abs()
    else:
        top = torch.topk(yr, 2, dim=1).values
        margin = top[:, 0] - top[:, 1]
    return {"classes": ks, "dice_hip_vs_oracle_labels": [round(v, 6) for v in per],
            "label_agreement": round(float((lab == labr).float().mean()), 7),
            "label_flips": int(flip.sum()), "label_flips_at_fp32_ties": int((flip & (margin < 1e-5)).sum()),
            "dice_to_target_hip": [round(v, 6) for v in to_t], "dice_to_target_oracle": [round(v, 6) for v in to_tr],
            "max_abs_dice_delta": float(max(abs(a - b) for a, b in zip(to_t, to_tr))),
            "max_abs_output_delta": float((y - yr).abs().max()),
            "precision": precision, "oracle": "oracle/unet_ref.py torch-CPU fp32",
            "sample": f"the bench batch ({x.shape[0]} slices) after the timed steps, train mode"}


# C-ABI entry -> regex over the device kernels it launches (rocprof kernel names), for the PMC traffic lookup
KERNEL_FAMILY = {
    "pmu_conv3x3_fwd": r"conv3x3_(pipe_)?kernel<false", "pmu_conv3x3_dgrad": r"conv3x3_(pipe_)?kernel<true",
    "pmu_conv3x3_wgrad": r"wgrad3x3_kernel<",
    "pmu_conv3x3_fwd_wino": r"conv3x3_wino_(pipe_)?kernel<false", "pmu_conv3x3_dgrad_wino": r"conv3x3_wino_(pipe_)?kernel<true",
    "pmu_conv3x3_wgrad_wino": (r"wgrad3x3_wino(32)?_kernel", r"wgrad_wino_reduce_kernel"),
    "pmu_conv3x3_fwd_wino4": r"conv3x3_wino4_kernel<false", "pmu_conv3x3_dgrad_wino4": r"conv3x3_wino4_kernel<true",
    "pmu_conv3x3_fwd_wino2h": r"conv3x3_wino2h_kernel<false", "pmu_conv3x3_dgrad_wino2h": r"conv3x3_wino2h_kernel<true",
    "pmu_conv3x3_fwd_wino_raw": r"conv3x3_wino_raw_kernel<false", "pmu_conv3x3_dgrad_wino_raw": r"conv3x3_wino_raw_kernel<true", "pmu_convT2x2_fwd": r"convT_pipe_kernel<false>|ActRowA",
    "pmu_convT2x2_dgrad": r"convT_pipe_kernel<true>|DuGatherA",
    "pmu_convT2x2_wgrad": r"convT_wgrad_(pipe_)?kernel", "pmu_fcomb_fwd": r"fcomb_fwd_kernel",
    "pmu_fcomb_bwd": r"fcomb_bwd_kernel",
    "pmu_conv3x3_fwd_bf16": r"conv3x3_bf16_pipe_kernel<false|conv3x3_bf16_kernel<\d, \d+, false>",
    "pmu_conv3x3_dgrad_bf16": r"conv3x3_bf16_pipe_kernel<true|conv3x3_bf16_kernel<\d, \d+, true>",
    "pmu_conv3x3_wgrad_bf16": r"wgrad3x3_bf16_kernel<", "pmu_conv3x3_wgrad_bf16_dma": r"wgrad3x3_bf16_dma_kernel<", "pmu_conv3x3_fwd_raw": r"conv3x3_raw_kernel<false",
    "pmu_conv3x3_dgrad_raw": r"conv3x3_raw_kernel<true", "pmu_convT2x2_fwd_bf16": r"convT_bf16_kernel<false>",
    "pmu_convT2x2_dgrad_bf16": r"convT_bf16_kernel<true>", "pmu_convT2x2_wgrad_bf16": r"convT_wgrad_bf16_kernel",
    "pmu_conv3x3_dgrad_wino4_bnr": r"conv3x3_wino4_kernel<true", "pmu_conv3x3_dgrad_wino2h_bnr": r"conv3x3_wino2h_kernel<true",
    "pmu_conv3x3_wgrad_wino4": (r"wgrad3x3_wino4_kernel", r"wgrad_wino4_reduce_kernel"),
    "pmu_conv3x3_fwd_dma": r"conv3x3_dma_kernel<false", "pmu_conv3x3_fwd_dma_zb": r"conv3x3_dma_kernel<false",
    "pmu_conv3x3_dgrad_dma": r"conv3x3_dma_kernel<true", "pmu_conv3x3_dgrad_dma_bnr": r"conv3x3_dma_kernel<true",
    "pmu_conv3x3_dgrad_dma_bnr_zb": r"conv3x3_dma_kernel<true",
    "pmu_convT2x2_fwd_dma": r"convT_dma_kernel<false", "pmu_convT2x2_dgrad_dma": r"convT_dma_kernel<true",
    "pmu_conv3x3_dgrad_dma_x1b": r"conv3x3_dma_kernel<true", "pmu_conv3x3_dgrad_dma_x1b_sum": r"conv3x3_dma_kernel<true",
    "pmu_conv3x3_dgrad_dma_dxb": r"conv3x3_dma_kernel<true", "pmu_conv3x3_dgrad_dma_bnr_dxb": r"conv3x3_dma_kernel<true",
    "pmu_conv3x3_dgrad_dma_x1b_dxb": r"conv3x3_dma_kernel<true",
    "pmu_conv3x3_dgrad_dma_x1b_sum_dxb": r"conv3x3_dma_kernel<true",
    "pmu_convT2x2_dgrad_dma_dxb": r"convT_dma_kernel<true",
    "pmu_convT2x2_fwd_ld": r"convT_pipe_kernel<false", "pmu_convT2x2_fwd_dma_ldb": r"convT_dma_kernel<false",
}


def pmc_traffic(workload, api):
    """HBM bytes per C-ABI call of ``api`` from the newest committed PMC summary
    (profiles/r*/pmc_traffic_<workload>.json, written by tools/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this bench command): the bytes of its main kernel family (a
    regex) plus those of an auxiliary kernel the call also launches (e.g. the weight gradient's
    slab reduce), divided by the main kernel's dispatch count.  None when absent."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_traffic_{workload}.json")),
                   key=lambda f: int(re.search(r"r(\d+)", os.path.relpath(f, ROOT)).group(1)))
    fam = KERNEL_FAMILY.get(api)
    if not files or fam is None:
        return None, None
    main, aux = fam if isinstance(fam, tuple) else (fam, None)
    data = json.load(open(files[-1]))["kernels"]
    tot, n = 0.0, 0
    for k, v in data.items():
        d = v["dispatches_fetch_pass"]
        if re.search(main, k):
            tot += v["hbm_bytes_per_dispatch"] * d
            n += d
        elif aux and re.search(aux, k):
            tot += v["hbm_bytes_per_dispatch"] * d
    if n == 0:
        return None, None
    return tot / n, os.path.relpath(files[-1], ROOT)


def fcomb_flops(name, args):
    """MACs the fused Fcomb kernels execute (z folded into a bias, so layer 1 is F x F per pixel)."""
    if name == "pmu_fcomb_fwd":
        F_, K, NH, S, N, H, W = args[6], args[8], args[9], args[10], args[11], args[12], args[13]
        return 2.0 * N * H * W * (F_ * F_ + S * ((NH - 1) * F_ * F_ + F_ * K))
    if name == "pmu_fcomb_bwd":
        F_, K, NH, N, H, W = args[8], args[10], args[11], args[12], args[13], args[14]
        return 2.0 * N * H * W * (3 * NH * F_ * F_ + 2 * F_ * K)
    return 0.0


def dp_sync(net, world):
    """N > 1: bucketed gradient all-reduce overlapped with the backward (pmu_hip.dp); the
    one-shot all-reduce after the backward with PMU_DP_OVERLAP=0."""
    if world == 1 or os.environ.get("PMU_DP_OVERLAP", "1") == "0":
        return None
    from pmu_hip.dp import BucketAllReduce
    return BucketAllReduce(net)


def build_unet(args, dev, world, rank):
    """c2: UNet fwd + loss + bwd + (all-reduce) + fused clip/SGD on one batch of slices."""
    from model import UNet
    from pmu_hip.functions import flat_grad_buffer
    from pmu_hip.optim import FusedSGD
    import torch.distributed as dist
    torch.manual_seed(0)
    net = UNet(args.channels, args.classes, FILTERS).to(dev).train()
    if world > 1:  # identical replicas: broadcast rank 0's weights
        for t in list(net.parameters()) + list(net.buffers()):
            dist.broadcast(t.data, 0)
        from pmu_hip.engine import invalidate_packs
        invalidate_packs()   # written through .data: invisible to the packed-weight cache
    opt = FusedSGD(net.parameters(), lr=1e-3, momentum=0.9, clip=0.1)
    sync = dp_sync(net, world)
    g = torch.Generator(device="cpu").manual_seed(1 + rank)
    B, S = args.batch, args.size
    from pmu_hip.loss import BCELoss, CrossEntropyLoss   # the trainer's criteria (row a6) on HIP kernels
    crit = BCELoss() if args.classes == 1 else CrossEntropyLoss()
    batches = None
    if args.data == "phantom":
        batches, gather_rate = phantom_batches(S, B, rank, world, dev)
    else:
        x = torch.rand(B, args.channels, S, S, generator=g).to(dev)
        if args.classes == 1:
            tgt = (torch.rand(B, 1, S, S, generator=g) > 0.5).float().to(dev)
        else:
            tgt = torch.randint(0, args.classes, (B, S, S), generator=g).to(dev)
    plist = list(net.parameters())

    def step():
        nonlocal x, tgt
        if batches is not None:  # multi-planar batch gathered on the GPU (one launch per tensor)
            b = next(batches)
            x = b["image"]
            tgt = (b["mask"] > 0).float() if args.classes == 1 else b["mask"][:, 0].long()
        for p in plist:
            p.grad = None
        # bf16: the reference's model code under torch.autocast(bfloat16), the PyTorch idiom for
        # config c5; the engine runs every 3x3 conv (fwd, dgrad, wgrad) on bf16 MFMA
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.precision == "bf16"):
            out = net(x)
        loss = crit(out, tgt)
        if sync is not None:
            sync.begin()
        loss.backward()
        if sync is not None:
            sync.finish()
        elif world > 1:
            dist.all_reduce(flat_grad_buffer(net, plist))
        opt.step(grad_scale=1.0 / world)
        return loss

    step.net = net
    step.batch = lambda: (x, tgt)
    step.gather_rate = gather_rate if args.data == "phantom" else None
    flops = conv_flops_per_slice(S, S, FILTERS, args.channels, args.classes) * B
    lossn = "BCE" if args.classes == 1 else "CE"
    tag = "c5" if args.workload == "c5" else "c2"
    config = {"workload": "%s: UNet(n_channels=%d, n_classes=%d, num_filters=%s), %dx%dx%d slices, "
                          "fwd+%s+bwd+clip(0.1)+SGD(0.9) per step, %s" % (tag, args.channels, args.classes, FILTERS,
                                                                         S, S, args.channels, lossn,
                                                                         args.precision),
              "global_batch": B * world, "per_gpu_batch": B, "image": [S, S], "parallelism": f"dp{world}"}
    data = "synthetic (x~U[0,1), random %s masks, seeded)" % ("binary" if args.classes == 1 else
                                                              "%d-class" % args.classes)
    if args.data == "phantom":
        config["workload"] = ("c3: " + config["workload"][4:] + "; batches of axial/coronal/sagittal slices "
                              "gathered on the GPU from a resident %d^3 phantom (MRI_Dataset)" % S)
        data = "synthetic seeded %d^3 ellipsoid phantom (nested-shell classes), 3-view slices, rank-sharded" % S
    return step, flops, config, data


def phantom_batches(S, B, rank, world, dev):
    """Endless per-rank batches of multi-planar slices (config c3): a seeded S^3 phantom with two
    nested ellipsoid shells (classes 1, 2) resident on the GPU through MRI_Dataset; the shuffled
    3-view index map is dealt round-robin over the ranks."""
    import numpy as np
    from utils.mri_dataset import MRI_Dataset
    rng = np.random.default_rng(11)
    ax = np.arange(S) - S / 2
    ii, jj, kk = np.meshgrid(ax, ax, ax, indexing="ij", sparse=True)
    r2 = (ii / (0.40 * S)) ** 2 + (jj / (0.35 * S)) ** 2 + (kk / (0.30 * S)) ** 2
    lab = np.where(r2 < 1.0, 1.0, 0.0) + np.where(r2 < 0.35, 1.0, 0.0)
    img = (rng.random((S, S, S)) * 200.0 + lab * 300.0).astype(np.float64)
    ds = MRI_Dataset("/imgs", "/labs", 3, filter=True, loader=lambda p: img if "imgs" in p else lab,
                     files=["phantom"], device=dev)
    del img
    order = np.random.default_rng(7).permutation(len(ds))[rank::world]

    def gen():
        i = 0
        while True:
            if i + B > len(order):
                i = 0
            yield ds.get_batch(order[i:i + B])
            i += B

    def gather_rate(nb=50):
        """The slicer's own rate (row a13 / f1): nb batches of B slices gathered back to back with no
        training step, timed with HIP events on the launch stream (host index upload included)."""
        it = gen()
        next(it)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(nb):
            next(it)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / nb
        return {"slices_per_s": round(B / (ms * 1e-3), 1), "ms_per_batch": round(ms, 4), "batches": nb,
                "batch": B, "note": "MRI_Dataset.get_batch alone: two pmu_gather_slices launches (image, mask)"}
    return gen(), gather_rate


def roofline_peak(kernel):
    """Dense MFMA peak (TFLOP/s) for a C-ABI kernel family: bf16 for the *_bf16 family, the LDS-DMA
    bf16 GEMMs (*_dma*) and the bf16 raw GEMMs (pmu_conv3x3_{fwd,dgrad}_raw), fp32 otherwise (the
    Winograd raw kernels are *_wino_raw)."""
    bf16 = (kernel.endswith("_bf16") or "_dma" in kernel or (kernel.endswith("_raw") and "_wino" not in kernel))
    return BF16_MFMA_PEAK_TF if bf16 else FP32_MFMA_PEAK_TF


@torch.no_grad()   # inference: no autograd graph, no saved activations per batch
def c5_eval(net, dev, D, batch, precision):
    """Config c5's evaluation (PMU/eval.py:131-203 via predict.predict_volume's batching): predict all
    3 x D slices (D x D x 3 channels) of a seeded D^3 phantom along the axial/coronal/sagittal views
    with the network in eval mode, then fuse the three views with pmu_fuse3view (softmax, average,
    argmax label map, per-class Dice of every volume).  Returns timings and the fused Dice."""
    from pmu_hip.fusion import fuse_views
    C = net.n_classes
    g = torch.Generator(device=dev).manual_seed(5)
    ax = torch.arange(D, dtype=torch.float32, device=dev) - D / 2
    r2 = ((ax[:, None, None] / (0.40 * D)) ** 2 + (ax[None, :, None] / (0.35 * D)) ** 2 +
          (ax[None, None, :] / (0.30 * D)) ** 2)
    lab = (r2 < 1.0).float() + (r2 < 0.35).float()
    del r2
    vol = torch.empty(3, D, D, D, device=dev)
    for c in range(3):  # three "modalities": the label-driven contrast under different seeded noise
        vol[c] = 0.6 * torch.rand(D, D, D, generator=g, device=dev) + 0.2 * (c + 1) * lab
    net.eval()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stacks = []
    for v in range(3):
        out = torch.empty(D, C, D, D, device=dev)
        for s0 in range(0, D, batch):
            s1 = min(D, s0 + batch)
            if v == 0:
                xb = vol[:, s0:s1].permute(1, 0, 2, 3)
            elif v == 1:
                xb = vol[:, :, s0:s1].permute(2, 0, 1, 3)
            else:
                xb = vol[:, :, :, s0:s1].permute(3, 0, 1, 2)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=precision == "bf16"):
                out[s0:s1] = net(xb.contiguous())
        stacks.append(out)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = fuse_views(stacks[0], stacks[1], stacks[2], lab, logits=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    net.train()
    dice = res["dice"].tolist()
    return {"volume": [D, D, D], "channels": 3, "slices": 3 * D, "batch": batch, "predict_s": round(t1 - t0, 4),
            "predict_slices_per_s": round(3 * D / (t1 - t0), 2), "fuse_ms": round((t2 - t1) * 1e3, 3),
            "dice_average_volume": [round(x, 4) for x in dice[3]],
            "note": "random-init weights: the Dice values only show the pipeline runs end to end"}


def build_probunet(args, dev, world, rank):
    """c4: one ProbUNetTrainer training step (probunet_trainer.py:27-39 + train.py:85-110):
    forward(training=True) -> sample() (the trainer's predict) -> -elbo (CE-sum + beta*KL) ->
    backward -> (all-reduce) -> clip+SGD, then the evaluation sweep: 16 prior samples through
    Fcomb in one fused pass + per-class Dice counts of every sample."""
    from model import ProbabilisticUnet
    from pmu_hip.functions import flat_grad_buffer
    from pmu_hip.metrics import dice_counts_many
    from pmu_hip.optim import FusedSGD
    import torch.distributed as dist
    torch.manual_seed(0)
    n_cls = 3
    net = ProbabilisticUnet(input_channels=1, num_classes=n_cls, num_filters=FILTERS, latent_dim=6,
                            no_convs_fcomb=4, beta=10.0).to(dev).train()
    if world > 1:
        for t in list(net.parameters()) + list(net.buffers()):
            dist.broadcast(t.data, 0)
        from pmu_hip.engine import invalidate_packs
        invalidate_packs()   # written through .data: invisible to the packed-weight cache
    opt = FusedSGD(net.parameters(), lr=1e-3, momentum=0.9, clip=0.1)
    sync = dp_sync(net, world)
    g = torch.Generator(device="cpu").manual_seed(1 + rank)
    B, S = args.batch, args.size
    x = torch.rand(B, 1, S, S, generator=g).to(dev)
    segm = torch.randint(0, n_cls, (B, 1, S, S), generator=g).float().to(dev)
    plist = list(net.parameters())
    n_samples = 16

    def step():
        for p in plist:
            p.grad = None
        net.forward(x, segm, training=True)
        net.sample(testing=False)
        loss = -net.elbo(segm)
        if sync is not None:
            sync.begin()
        loss.backward()
        if sync is not None:
            sync.finish()
        elif world > 1:
            dist.all_reduce(flat_grad_buffer(net, plist))
        opt.step(grad_scale=1.0 / world)
        with torch.no_grad():
            ys = net.sample_many(n_samples)                  # (16, B, 3, S, S)
            dice_counts_many(ys, segm, n_cls)                # every sample's counts, one launch
        return loss

    config = {"workload": "c4: ProbabilisticUnet(1, 3, %s, latent_dim=6, no_convs_fcomb=4, beta=10), %dx%dx1 "
                          "slices; train step (fwd, prior sample, -elbo, bwd, clip+SGD) + 16 fcomb samples + Dice"
                          % (FILTERS, S, S),
              "global_batch": B * world, "per_gpu_batch": B, "image": [S, S], "parallelism": f"dp{world}"}
    data = "synthetic (x~U[0,1), random 3-class masks, seeded)"
    step.net = net
    step.batch = lambda: (x, segm)
    return step, None, config, data


def mfma_families(per):
    """Group the instrumented step's MFMA C-ABI entries into kernel families (KernelTimer._base: a fused
    variant — BN-backward epilogue _bnr, bf16 dx _dxb, concat copies _x1b(_sum), in-place concat _ld(b) —
    is the same GEMM as its plain entry) and rank them by their summed launch time.  Returns
    [(family, [launches, executed FLOPs, seconds, direct-sum FLOPs], [member entries])], longest first:
    c5's input gradient, split over _bnr_dxb / _x1b_sum_dxb / _dxb entries, is one family."""
    fam = {}
    for k, v in per.items():
        if k not in KernelTimer.MFMA:
            continue
        b = KernelTimer._base(k)
        d, members = fam.setdefault(b, ([0, 0.0, 0.0, 0.0], []))
        for i in range(4):
            d[i] += v[i]
        members.append(k)
    return sorted(((b, d, sorted(m)) for b, (d, m) in fam.items()), key=lambda e: -e[1][2])


def roofline_entry(workload, family, d, members):
    """The roofline object of one MFMA kernel family: executed FLOPs / its HIP-event time vs the dtype
    peak, PMC traffic per launch from the newest committed summary."""
    n, fl, t, dfl = d
    ach = fl / t / 1e12
    traffic, tsrc = pmc_traffic(workload, family)
    peak = roofline_peak(family)
    roof = {"kernel": family, "members": members, "bound": "mfma", "achieved": round(ach, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(ach / peak, 4),
            "traffic": round(traffic) if traffic is not None else None, "traffic_unit": "bytes/launch (HBM)",
            "traffic_source": tsrc, "launches": n, "avg_launch_ms": round(t / n * 1e3, 4),
            "family_ms": round(t * 1e3, 3), "flops_per_launch": fl / n,
            "flops_basis": "MFMA products the kernel executes"}
    if "_wino" in family:  # Winograd executes 16 of the direct sum's 36 products per 2x2 tile
        roof["flops_basis"] = ("executed Winograd F(2x2,3x3) MFMA products (16 per 2x2 output tile per "
                               "channel pair); frac is MFMA utilisation")
        if family.endswith("_wino4"):
            roof["flops_basis"] = ("executed Winograd F(4x4,3x3) MFMA products (36 per 4x4 output tile per "
                                   "channel pair); frac is MFMA utilisation")
        roof["direct_sum_flops_per_launch"] = dfl / n
        roof["direct_sum_equiv_tflops"] = round(dfl / t / 1e12, 2)
        roof["direct_sum_equiv_frac"] = round(dfl / t / 1e12 / peak, 4)
        roof["direct_sum_note"] = ("SURVEY.md §8(d) basis (9 MACs per pixel per channel pair): >1 is possible "
                                   "because Winograd executes 16/36 (F(2x2)) or 36/144 (F(4x4)) of those "
                                   "products; not a utilisation")
    return roof


def check_layout(backend, world, ndev):
    """Refuse a rank layout that would not time ``world`` distinct GPUs (pure host logic): under RCCL
    (backend nccl) every rank needs its own device, so world > the visible device count is an error;
    gloo may rehearse N ranks on fewer GPUs.  Returns an error message or None."""
    if world > 1 and backend == "nccl" and world > ndev:
        return (f"{world} RCCL ranks but {ndev} visible GPU(s): each rank needs its own device "
                f"(PMU_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
    return None


def check_devices(backend, devices):
    """Refuse an RCCL run whose ranks report the same GPU (devices: one PCI identity per rank, gathered
    to every rank).  Returns an error message or None."""
    if backend == "nccl" and len(set(devices)) != len(devices):
        return f"RCCL ranks share a GPU: {devices}"
    return None


def device_identity(dev):
    """PCI domain:bus:device of a GPU (and its uuid): one string per physical device."""
    p = torch.cuda.get_device_properties(dev)
    return "%04x:%02x:%02x.0 %s" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                    getattr(p, "pci_device_id", 0), str(getattr(p, "uuid", "")))


def launch_plan(gpus, argv, env):
    """How to run ``bench.py --gpus N`` (pure host logic, no GPU call).

    Returns None when this process is the rank to run (N == 1 outside torchrun, or any N under
    torchrun with WORLD_SIZE == N), or the command list of a ``torch.distributed.run`` child that
    starts N ranks of this script on this node (N > 1 outside torchrun) — the driver's own N-GPU
    launch, one process per GPU, so ``--gpus N`` always measures N GPUs.  Raises ValueError when
    ``--gpus`` disagrees with a torchrun world size: a run that would time a different number of GPUs
    than it reports.  The child gets the same argv (``--gpus`` kept, so each rank re-checks it)."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise ValueError(f"--gpus {gpus} but WORLD_SIZE={world}: launch with --nproc-per-node {gpus} "
                             f"or drop --gpus")
        return None
    if gpus == 1:
        return None
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--classes", type=int, default=1)
    ap.add_argument("--workload", choices=["unet", "probunet", "c5"], default="unet",
                    help="unet: c2 (default); probunet: c4; c5: UNet(3,3) on 512x512x3 slices, batch 16, bf16")
    ap.add_argument("--channels", type=int, default=None)
    ap.add_argument("--precision", choices=["fp32", "bf16"], default=None,
                    help="bf16: 3x3 convs on bf16 MFMA (torch.autocast(bfloat16) arithmetic)")
    ap.add_argument("--data", choices=["synthetic", "phantom"], default="synthetic",
                    help="phantom: multi-planar slices gathered on the GPU from a resident phantom (c3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-eval", action="store_true", help="c5: skip the 3-view volume-fusion evaluation")
    ap.add_argument("--eval-size", type=int, default=512, help="c5 evaluation volume edge (D^3 voxels)")
    args = ap.parse_args()
    try:
        cmd = launch_plan(args.gpus, sys.argv[1:], os.environ)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        return 2
    if cmd is not None:
        # N ranks outside torchrun: start them as a child process (nothing here has touched the GPU;
        # an exec from a GPU-initialised process is not allowed) and pass its exit code on; rank 0's
        # JSON line reaches stdout through the inherited descriptor.
        import subprocess
        return subprocess.call(cmd)
    c5 = args.workload == "c5"
    if args.channels is None:
        args.channels = 3 if c5 else 1
    if args.precision is None:
        args.precision = "bf16" if c5 else "fp32"
    if c5:
        if "--batch" not in sys.argv:
            args.batch = 16
        if "--size" not in sys.argv:
            args.size = 512
        if "--classes" not in sys.argv:
            args.classes = 3

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; rank -> device modulo the visible count so a multi-rank run can be
    # rehearsed on fewer GPUs (PMU_DIST_BACKEND=gloo: RCCL needs distinct devices per rank)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(1, ndev))
    backend = os.environ.get("PMU_DIST_BACKEND", "nccl") if world > 1 else None
    err = check_layout(backend, world, ndev)
    if err:
        print(f"bench.py: {err}", file=sys.stderr)
        return 2
    dist_info = {"backend": backend, "world": world, "visible_devices": ndev}
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        devices = [None] * world
        dist.all_gather_object(devices, device_identity(dev))
        dist_info["devices"] = devices
        err = check_devices(backend, devices)
        if err:
            print(f"bench.py: {err}", file=sys.stderr)
            dist.destroy_process_group()
            return 2
    else:
        dist_info["devices"] = [device_identity(dev)]

    from pmu_hip import _lib as L

    build = build_probunet if args.workload == "probunet" else build_unet
    step, flops_step, config, data = build(args, dev, world, rank)
    B = args.batch

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt)
    ms = dt / args.steps * 1e3
    value = world * B * args.steps / dt

    roof = roof_next = kernels = mfma_busy = None
    if not args.no_kernel_timing:
        timer = KernelTimer()
        # the instrumented step runs on one stream: events bracketing a launch on a stream that other
        # streams' kernels overlap would time their work too (c4's concurrent parts, engine CFG.prob_streams)
        from pmu_hip.engine import CFG
        prev_streams, CFG.prob_streams = CFG.prob_streams, False
        L.set_call_observer(timer)
        step()
        L.set_call_observer(None)
        CFG.prob_streams = prev_streams
        per = timer.summary()
        mf = {k: v for k, v in per.items() if k in KernelTimer.MFMA}
        fams = mfma_families(per)
        # the dominant MFMA kernel family (summed over its fused entry variants) and the runner-up
        roof = roofline_entry(args.workload, *fams[0])
        roof_next = roofline_entry(args.workload, *fams[1]) if len(fams) > 1 else None
        kernels = {k: {"launches": v[0], "ms": round(v[2] * 1e3, 3),
                       "tflops": (round(v[1] / v[2] / 1e12, 2) if v[1] else None)} for k, v in sorted(per.items())}
        # executed MFMA work of the step at each kernel's own peak, over the step time: the MFMA-busy
        # equivalent of the whole step (BN, pooling, optimizer and launch gaps count as idle)
        mfma_busy = sum(v[1] / (roofline_peak(k) * 1e12) for k, v in mf.items()) / (ms * 1e-3)
        if flops_step is None:   # direct-sum FLOPs of the step = those of the MFMA kernels it launches
            flops_step = sum(v[3] for v in per.values())
    evalres = None
    if args.workload == "c5" and not args.no_eval and rank == 0:
        evalres = c5_eval(step.net, dev, args.eval_size, B, args.precision)
    cpu = dvr = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, dvr = cpu_leg(args, step)
    if rank == 0:
        res = {
            "metric": METRIC_C5 if args.workload == "c5" else METRIC_C4 if args.workload == "probunet" else METRIC,
            "value": round(value, 3), "unit": "slices/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.precision if args.workload != "probunet" else "fp32",
            "data": data, "config": config,
            "step_tflops": round(flops_step / (ms * 1e-3) / 1e12, 2) if flops_step else None,
            "step_tflops_basis": "direct-sum algorithmic FLOPs per step (SURVEY.md §8d) / step time",
            "step_mfma_busy_frac": round(mfma_busy, 4) if mfma_busy is not None else None,
            "step_mfma_busy_basis": ("sum over MFMA kernels of executed FLOPs / that kernel's dtype peak, over the "
                                     "step time (HIP events of one instrumented step)"),
            "roofline": roof, "roofline_next": roof_next, "dist": dist_info, "cpu_baseline": cpu, "dice_vs_ref": dvr, "kernels": kernels,
            "loss": float(loss.detach()),
        }
        if evalres is not None:
            res["c5_volume_fusion_eval"] = evalres
        if getattr(step, "gather_rate", None) is not None:
            res["gather"] = step.gather_rate()
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
