#!/usr/bin/env python3
"""Seed spread and floors of the c5 Dice contract (tests/test_bf16_gpu.py::test_c5_bf16_dice_gap_vs_fp32_oracle):
config c5's UNet(3, 3, [64..1024]) trained 12 identical steps (CE + clip + SGD, lr 0.05) on the seeded
3-channel phantom batch, per weight-init seed, by

  ref      the fp32 oracle on the CPU (oracle/unet_ref.py: the reference's arithmetic) — every gap below is
           the per-class Dice-to-target gap of an argmax map against this one's;
  o32gpu   the same oracle code in fp32 on the GPU (torch's im2col + rocBLAS; another summation order);
  o64      the oracle in fp64 on the GPU (the fp32 rounding floor);
  oac      the oracle under torch.autocast(bfloat16)'s own semantics (oracle.unet_ref.AUTOCAST_ALL: every
           conv's operands, weights, dy and dx rounded to bf16), fp32 sums on the GPU — what autocast does to
           the reference itself;
  oacf     oac with the forward rounding only (operands and weights), oacb with the backward's only;
  tac      the oracle's fp32 code under torch.autocast(bfloat16) itself, on the GPU (PyTorch's bf16
           convolutions: bf16 conv outputs, BN in fp32), the reference as autocast would run it;
  hip32    the HIP path in fp32;
  hip16    the HIP path under torch.autocast(bfloat16) (the shipped c5 arithmetic);
  hip16dx  the same with fp32 activation gradients (engine CFG.dx_bf16 off, oracle BF16_DX off).

For each, the eval-mode (BN running statistics) and train-mode (batch statistics) gaps, and for the eval
maps the number of pixels whose label differs from ref's and how many of those lie where ref's top-2 logit
margin is below 1e-3 / 1e-2 (near-ties), plus ref's own near-tie counts.

usage: python tools/dice_gap_seeds.py [--seeds 0,1,2,3,4,5,6,7] [--out file.json] [--cols ...]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))

FILTERS = [64, 128, 256, 512, 1024]
D, N, STEPS, LR = 128, 8, 12, 0.05
MODES = ("eval", "train")


def margin(out):
    """top-1 minus top-2 logit per pixel (N, H, W)."""
    v = out.float().topk(2, dim=1).values
    return v[:, 0] - v[:, 1]


def oracle_run(sd0, x, t, device, dtype, autocast=False, parts=("fwd", "bwd"), torch_autocast=False):
    """12 oracle steps from sd0, then the eval / train outputs.  autocast: the oracle's restatement of
    torch.autocast(bfloat16) (AUTOCAST_ALL; ``parts`` picks the forward and / or backward rounding);
    torch_autocast: the oracle's fp32 code run under torch.autocast itself on the GPU (PyTorch's own bf16
    convolutions, cudnn off: im2col + rocBLAS)."""
    import oracle.unet_ref as U
    # (a copy: the oracle's BatchNorm updates the running statistics in place)
    sd = {k: (v.to(device, dtype) if v.is_floating_point() else v.to(device)).clone() for k, v in sd0.items()}
    bufs = {k: torch.zeros_like(sd[k]) for k in U.unet_param_keys(sd)}
    xo, to = x.to(device, dtype), t.to(device)
    prev = U.AUTOCAST_ALL, U.ROUND_PARTS
    U.AUTOCAST_ALL, U.ROUND_PARTS = autocast, tuple(parts)
    try:
        with torch.backends.cudnn.flags(enabled=False), \
                torch.autocast("cuda", dtype=torch.bfloat16, enabled=torch_autocast):
            for _ in range(STEPS):
                U.unet_train_step(sd, xo, to, len(FILTERS), 3, lr=LR, bufs=bufs, bf16=autocast)
            outs = {}
            with torch.no_grad():
                for m in MODES:
                    outs[m] = U.unet_forward({k: v.clone() for k, v in sd.items()}, xo, len(FILTERS), 3,
                                             training=m == "train", bf16=autocast).float().cpu()
    finally:
        U.AUTOCAST_ALL, U.ROUND_PARTS = prev
    return outs


def hip_run(sd0, x, y, dev, bf16, dx_bf16=True):
    from model import UNet
    from pmu_hip import engine
    from pmu_hip.optim import FusedSGD
    prev = engine.CFG.dx_bf16
    engine.CFG.dx_bf16 = dx_bf16
    try:
        net = UNet(3, 3, FILTERS)
        net.load_state_dict(sd0)
        net = net.to(dev).train()
        opt = FusedSGD(net.parameters(), lr=LR, momentum=0.9, clip=0.1)
        xd, td = x.to(dev), y.to(dev)
        for _ in range(STEPS):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                out = net(xd)
            torch.nn.functional.cross_entropy(out, td).backward()
            opt.step()
        outs = {}
        for m in MODES:
            net.train(m == "train")
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                outs[m] = net(xd).float().cpu()
        return outs
    finally:
        engine.CFG.dx_bf16 = prev


def compare(outs, ref, ref_dice, t):
    from oracle.unet_ref import trainer_dice
    r = {}
    for m in MODES:
        d = trainer_dice(outs[m], t, 3)
        r[f"gap_{m}"] = max(abs(a - b) for a, b in zip(d, ref_dice[m]))
    lab, rlab = outs["eval"].argmax(1), ref["eval"].argmax(1)
    flip = lab != rlab
    mg = margin(ref["eval"])
    r["flips_eval"] = int(flip.sum())
    r["flips_eval_margin_lt_1e-3"] = int((flip & (mg < 1e-3)).sum())
    r["flips_eval_margin_lt_1e-2"] = int((flip & (mg < 1e-2)).sum())
    r["max_ref_margin_at_flip_eval"] = float(mg[flip].max()) if bool(flip.any()) else 0.0
    r["max_abs_dlogit_eval"] = float((outs["eval"] - ref["eval"]).abs().max())
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--cols", default="o32gpu,o64,oac,hip32,hip16,hip16dx")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from model import UNet
    from oracle.unet_ref import trainer_dice
    from test_bf16_gpu import _phantom_slices
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    dev = torch.device("cuda", 0)
    cols = args.cols.split(",")
    x, y = _phantom_slices(D, N)
    t = y[:, None]
    rows = []
    for seed in [int(s) for s in args.seeds.split(",")]:
        t0 = time.time()
        torch.manual_seed(seed)
        net0 = UNet(3, 3, FILTERS)
        sd0 = {k: v.clone() for k, v in net0.state_dict().items()}
        ref = oracle_run(sd0, x, t, "cpu", torch.float32)
        ref_dice = {m: trainer_dice(ref[m], t, 3) for m in MODES}
        mg = margin(ref["eval"])
        row = {"seed": seed, "ref_dice_eval": ref_dice["eval"], "ref_dice_train": ref_dice["train"],
               "ref_eval_pixels_margin_lt_1e-3": int((mg < 1e-3).sum()),
               "ref_eval_pixels_margin_lt_1e-2": int((mg < 1e-2).sum()),
               "ref_eval_pixels_margin_lt_1e-1": int((mg < 1e-1).sum()), "pixels": int(mg.numel())}
        runs = {"o32gpu": lambda: oracle_run(sd0, x, t, dev, torch.float32),
                "o64": lambda: oracle_run(sd0, x, t, dev, torch.float64),
                "oac": lambda: oracle_run(sd0, x, t, dev, torch.float32, autocast=True),
                "oacf": lambda: oracle_run(sd0, x, t, dev, torch.float32, autocast=True, parts=("fwd",)),
                "oacb": lambda: oracle_run(sd0, x, t, dev, torch.float32, autocast=True, parts=("bwd",)),
                "tac": lambda: oracle_run(sd0, x, t, dev, torch.float32, torch_autocast=True),
                "hip32": lambda: hip_run(sd0, x, y, dev, False),
                "hip16": lambda: hip_run(sd0, x, y, dev, True),
                "hip16dx": lambda: hip_run(sd0, x, y, dev, True, dx_bf16=False)}
        for c in cols:
            row[c] = compare(runs[c](), ref, ref_dice, t)
        row["seconds"] = round(time.time() - t0, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    summary = {"lib": os.environ.get("PMU_LIB", "") or "release", "geometry": f"UNet(3,3,{FILTERS}) {N}x3x{D}x{D}",
               "steps": STEPS, "rows": rows}
    for c in cols:
        for m in MODES:
            v = [r[c][f"gap_{m}"] for r in rows]
            summary[f"{c}_max_gap_{m}"] = max(v)
            summary[f"{c}_mean_gap_{m}"] = sum(v) / len(v)
    print("SUMMARY " + json.dumps({k: v for k, v in summary.items() if k != "rows"}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
