#!/usr/bin/env python3
"""Per-shape HBM traffic of one kernel family from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
of `tools/kbench.py --ops OP --iters I` (every shape launches 2 warm-up + I timed dispatches, in
kbench's SHAPES order), next to the op's algorithmic bytes:
  dgrad_w4b   F(4x4) BN-backward input gradient: dz + dx (fp32) + the producer's z + the packed U (36/9)
  dgrad_dmabx c5 LDS-DMA BN-backward input gradient: dz (bf16) + dx (bf16) + the producer's z (fp32) + w
  dgrad_dmax  c5 LDS-DMA input gradient: dz (bf16) + dx (bf16) + w
  fwd_dma     c5 LDS-DMA forward: x (bf16) + z (fp32) + w
  mat_bnrelu  BN+ReLU bf16 operand: z (fp32) in, x (bf16) out
  mat_bnbwd_xb BN-backward bf16 dz from the bf16 dx: dx (bf16) + z (fp32) in, dz (bf16) out
  mat_pool_skip max-pooled BN+ReLU operand + unpooled skip half: z (fp32) in, pooled + skip (bf16) out
  mat32       BN+ReLU fp32 operand (config c2): z in, x out, fp32
  mat32_bnbwd BN-backward fp32 dz (config c2): da + z in, dz out, fp32
  mp_stats_xb max-pool backward, BN-backward partials only: pooled + skip gradients (bf16) + z (fp32) in
  mp_bnbwd_xb max-pool backward to the layer's bf16 dz: the same in, dz (bf16) out

    python tools/pmc_shapes.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR ITERS [--N 32] [--op dgrad_w4b] [--c5]

Bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 correction, tools/pmc_traffic.py)."""
import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kbench import SHAPES  # noqa: E402


def per_dispatch(d, counter, sub):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and sub in r["Kernel_Name"]:
                k = int(r["Dispatch_Id"])
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("kernel")
    ap.add_argument("iters", type=int)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--op", default="dgrad_w4b")
    ap.add_argument("--c5", action="store_true", help="kbench --c5 shapes (512x512 input)")
    a = ap.parse_args()
    shapes = [(2 * h, ci, co) for (h, ci, co) in SHAPES] if a.c5 else SHAPES
    fe, wr = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel), per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    # kbench's own setup streams the dz and x operands of every shape: two frame_stream dispatches first
    lead = 2 if a.op.startswith("mat") else 0
    per = lead + 2 + a.iters
    assert len(fe) == len(wr) == per * len(shapes), (len(fe), len(wr), per * len(shapes))
    print(f"op {a.op} N {a.N}; bytes per dispatch = (2 FETCH_SIZE + WRITE_SIZE) x 1024")
    print(f"{'H':>4} {'Cin':>5} {'Cout':>5} {'PMC MB':>9} {'alg MB':>9} {'ratio':>6}")
    tp = ta = 0.0
    for s, (H, Cin, Cout) in enumerate(shapes):
        idx = range(s * per + lead + 2, (s + 1) * per)
        hbm = sum((2 * fe[i] + wr[i]) * 1024 for i in idx) / a.iters
        px = a.N * H * H
        cpi, cpo = (Cin + 7) // 8 * 8, (Cout + 7) // 8 * 8
        alg = {"dgrad_w4b": px * Cout * 4 + px * Cin * 4 + px * Cin * 4 + Cin * Cout * 36 * 4,
               "dgrad_dmabx": px * cpo * 2 + px * Cin * 2 + px * Cin * 4 + Cin * Cout * 9 * 2,
               "dgrad_dmax": px * cpo * 2 + px * Cin * 2 + Cin * Cout * 9 * 2,
               "fwd_dma": px * cpi * 2 + px * Cout * 4 + Cin * Cout * 9 * 2,
               "mat_bnrelu": px * Cin * 4 + px * cpi * 2,
               "mat_bnbwd_xb": px * Cout * (2 + 4) + px * cpo * 2,
               "mat_pool_skip": px * Cin * 4 + px // 4 * Cin * 2 + px * Cin * 2,
               "mat32": px * Cin * 4 * 2,
               "mat32_bnbwd": px * Cout * 4 * 3,
               "mp_stats_xb": px // 4 * Cout * 2 + px * Cout * (2 + 4),
               "mp_bnbwd_xb": px // 4 * Cout * 2 + px * Cout * (2 + 4) + px * Cout * 2}[a.op]
        tp += hbm
        ta += alg
        print(f"{H:4d} {Cin:5d} {Cout:5d} {hbm / 1e6:9.1f} {alg / 1e6:9.1f} {hbm / alg:6.2f}")
    print(f"{'all':>16} {tp / 1e6:9.1f} {ta / 1e6:9.1f} {tp / ta:6.2f}")


if __name__ == "__main__":
    main()
