#!/usr/bin/env python3
"""Seed spread of tests/test_bf16_gpu.py::test_c5_bf16_dice_gap_vs_fp32_oracle's statistic: config c5's
UNet(3, 3, [64..1024]) trained 12 identical steps on the seeded phantom batch by the fp32 oracle
(oracle/unet_ref.py, here on the GPU's torch ops) and by the HIP bf16 path (torch.autocast), then the
per-class Dice-to-target gap of the eval / train argmax maps — for several weight-init seeds, so a
kernel change's effect on the gap can be told from the bf16 trajectory's own seed-to-seed spread.

usage: python tools/dice_gap_seeds.py [--seeds 0,1,2,3,4] [--out file.json]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "probabilistic-multiplanar-unet_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2,3,4")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from model import UNet
    from oracle.unet_ref import trainer_dice, unet_forward, unet_param_keys, unet_train_step
    from pmu_hip.optim import FusedSGD
    from test_bf16_gpu import _phantom_slices
    dev = torch.device("cuda", 0)
    D, N, steps, lr = 128, 8, 12, 0.05
    x, y = _phantom_slices(D, N)
    t = y[:, None]
    rows = []
    for seed in [int(s) for s in args.seeds.split(",")]:
        torch.manual_seed(seed)
        net0 = UNet(3, 3, [64, 128, 256, 512, 1024])
        sd0 = {k: v.clone() for k, v in net0.state_dict().items()}
        sd = {k: v.clone().to(dev) for k, v in sd0.items()}
        bufs = {k: torch.zeros_like(sd[k]) for k in unet_param_keys(sd)}
        xo, to = x.to(dev), t.to(dev)
        for _ in range(steps):
            unet_train_step(sd, xo, to, 5, 3, lr=lr, bufs=bufs)
        row = {"seed": seed}
        ref = {}
        with torch.no_grad():
            for m in ("eval", "train"):
                o = unet_forward({k: v.clone() for k, v in sd.items()}, xo, 5, 3, training=m == "train").cpu()
                ref[m] = trainer_dice(o, t, 3)
        net = UNet(3, 3, [64, 128, 256, 512, 1024])
        net.load_state_dict(sd0)
        net = net.to(dev).train()
        opt = FusedSGD(net.parameters(), lr=lr, momentum=0.9, clip=0.1)
        xd, td = x.to(dev), y.to(dev)
        for _ in range(steps):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = net(xd)
            torch.nn.functional.cross_entropy(out, td).backward()
            opt.step()
        for m in ("eval", "train"):
            net.train(m == "train")
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                out = net(xd).float().cpu()
            d = trainer_dice(out, t, 3)
            row[f"gap_{m}"] = max(abs(a - b) for a, b in zip(d, ref[m]))
        rows.append(row)
        print(json.dumps(row), flush=True)
    summary = {"lib": os.environ.get("PMU_LIB", "") or "release", "rows": rows,
               "max_gap_eval": max(r["gap_eval"] for r in rows), "max_gap_train": max(r["gap_train"] for r in rows),
               "mean_gap_eval": sum(r["gap_eval"] for r in rows) / len(rows),
               "mean_gap_train": sum(r["gap_train"] for r in rows) / len(rows)}
    print("SUMMARY " + json.dumps(summary))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
