#!/usr/bin/env python3
"""Per-shape timing of the operand materialisation passes (pmu_frame_to_bf16 / _f32) on the c2 / c5
UNet shapes: the streaming kernels against the generic ones (PMU_FRAME_STREAM=0), with a bitwise
comparison of the outputs.

    python tools/kbench_frame.py [--c5] [--iters 20]

GB/s = algorithmic bytes (fp32 source reads, z for the BN backward, output writes) / time."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from pmu_hip import _lib as L  # noqa: E402
from pmu_hip.engine import Src, frame_of  # noqa: E402


def run(kind, bf, N, H, W, C, dev):
    g = torch.Generator(device=dev).manual_seed(H + C)
    pool = kind == "pool"
    SH, SW = (2 * H, 2 * W) if pool else (H, W)
    x = torch.randn(N, SH, SW, C, device=dev, generator=g)
    if kind == "bwd":
        z = torch.randn(N, SH, SW, C, device=dev, generator=g)
        coef = torch.randn(5 * C, device=dev, generator=g)
        src = Src(x, L.SRC_BNBWD, coef, z=z)
    else:
        coef = torch.cat([torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g)])
        src = Src(x, L.SRC_BNRELU, coef, pool=L.POOL_MAX2 if pool else L.POOL_NONE)
    f = frame_of([src], N, H, W)
    out = torch.empty(N, H, W, C, dtype=torch.int16 if bf else torch.float32, device=dev)
    s = L.stream()
    fn = ((lambda: L.call("pmu_frame_to_bf16", f, C, out.data_ptr(), s)) if bf else
          (lambda: L.call("pmu_frame_to_f32", f, out.data_ptr(), s)))
    res = {}
    outs = {}
    for mode in MODES:
        os.environ["PMU_FRAME_STREAM"] = "0" if mode == "g" else "1"
        res[mode] = timeit(fn, ITERS)
        fn()
        torch.cuda.synchronize()
        outs[mode] = out.clone()
    os.environ.pop("PMU_FRAME_STREAM")
    rd = x.numel() * 4 * (2 if kind == "bwd" else 1)
    wr = out.numel() * out.element_size()
    gbs = {m: (rd + wr) / (ms * 1e-3) / 1e9 for m, ms in res.items()}
    same = all(torch.equal(outs[m], outs["g"]) for m in outs)
    cols = "  ".join(f"{'stream' if m == 's' else 'generic'} {res[m]:6.3f} ms {gbs[m]:5.0f} GB/s" for m in res)
    print(f"{kind:4s} {'bf16' if bf else 'f32 '} N={N} {H}x{W}x{C:5d}  {cols}  same={same}", flush=True)
    return res, same


ITERS = 20
# stream (the library's policy; with PMU_LIB=exp, PMU_FRAME_NT=0 / 3 forces plain / nontemporal) and generic
MODES = ("s", "g")


def main():
    global ITERS
    ap = argparse.ArgumentParser()
    ap.add_argument("--c5", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    ITERS = args.iters
    dev = torch.device("cuda")
    if args.c5:
        N, R, bf = 16, 512, True
    else:
        N, R, bf = 32, 256, False
    tot = {m: 0.0 for m in MODES}
    ok = True
    for lev, C in enumerate([64, 128, 256, 512, 1024]):
        H = R >> lev
        for kind in ("fwd", "pool", "bwd"):
            if kind == "pool" and lev == 0:
                continue
            Hk = H
            res, same = run(kind, bf, N, Hk, Hk, C if kind != "pool" else C // 2, dev)
            ok = ok and same
            for m in tot:
                tot[m] += res[m]
    print("TOTAL " + "  ".join(f"{m} {v:.3f} ms" for m, v in tot.items()) + f"  all_same={ok}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
