#!/usr/bin/env python3
"""Per-call breakdown of one c2 training step: every C-ABI launch with its operand description
(frame sources, pooling, channels, spatial size) and HIP-event time, grouped by layer signature.

    python tools/step_profile.py [--batch 32] [--size 256] [--workload unet|probunet]
"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402

POOL = {0: "", 1: "max", 2: "avg"}
MODE = {0: "raw", 1: "bnrelu", 2: "bnbwd"}


def describe(name, args):
    try:
        if name in ("pmu_conv3x3_fwd_wino_raw", "pmu_conv3x3_dgrad_wino_raw"):
            return f"{args[3]}x{args[4]} C{args[1]} -> {args[7] if 'fwd' in name else args[6]}"
        if name == "pmu_conv3x3_wgrad_wino":
            return f"{args[3]}x{args[4]} {args[5]}x{args[6]}"
        if name in ("pmu_conv3x3_fwd_raw", "pmu_conv3x3_dgrad_raw"):
            return f"{args[3]}x{args[4]} Cp{args[1]} -> {args[7] if name.endswith('fwd_raw') else args[6]}"
        if name == "pmu_conv3x3_wgrad_bf16":
            return f"{args[3]}x{args[4]} {args[5]}x{args[6]}"
        if name in ("pmu_conv3x3_fwd", "pmu_conv3x3_dgrad", "pmu_conv3x3_wgrad", "pmu_convT2x2_fwd"):
            f = args[0]._obj
            srcs = "+".join(f"{MODE[f.src[i].mode]}{POOL[f.src[i].pool]}{f.src[i].C}" for i in range(f.nsrc))
            extra = ""
            if name == "pmu_conv3x3_wgrad":
                a = args[1]._obj
                extra = " act=" + "+".join(f"{MODE[a.src[i].mode]}{POOL[a.src[i].pool]}{a.src[i].C}"
                                          for i in range(a.nsrc))
            return f"{f.H}x{f.W} {srcs}{extra}"
    except Exception:
        pass
    return ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--workload", default="unet", help="unet (c2), c5 or probunet")
    ap.add_argument("--precision", default=None)
    args = ap.parse_args()
    import bench
    from pmu_hip import _lib as L
    c5 = args.workload == "c5"
    ns = argparse.Namespace(batch=16 if c5 else args.batch, size=512 if c5 else args.size, classes=3 if c5 else 1,
                            workload=args.workload, data="synthetic", channels=3 if c5 else 1,
                            precision=args.precision or ("bf16" if c5 else "fp32"))
    build = bench.build_probunet if args.workload == "probunet" else bench.build_unet
    step, _, _, _ = build(ns, torch.device("cuda", 0), 1, 0)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    rec = []
    L.set_call_observer(lambda name, a, e0, e1: rec.append((name, describe(name, a), e0, e1)))
    step()
    L.set_call_observer(None)
    torch.cuda.synchronize()
    groups = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for name, d, e0, e1 in rec:
        t = e0.elapsed_time(e1)
        groups[(name, d)][0] += 1
        groups[(name, d)][1] += t
        total += t
    for (name, d), (n, t) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        print(f"{t:8.3f} ms  x{n:2d}  {name:24s} {d}")
    print(f"{total:8.3f} ms  total of instrumented calls")


if __name__ == "__main__":
    main()
