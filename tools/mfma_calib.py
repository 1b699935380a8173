#!/usr/bin/env python3
"""Summarise scripts/gpu_mfma_calib.sh: per kernel dispatch the MFMA counters next to the executed
MFMA work the launch implies, to validate SQ_VALU_MFMA_BUSY_CYCLES (MI355X_MICROARCH.md: cycles,
32 per v_mfma_f32_32x32x16_bf16, 32 per v_mfma_f32_16x16x4_f32) and SQ_INSTS_VALU_MFMA_MOPS_* (FLOPs / 512)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True)):
        run = os.path.relpath(f, d).split(os.sep)[0]
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (did, k), c in per.items():
            rows.append((run, int(did), k, c))
    rows.sort(key=lambda r: (r[0], r[1]))
    for run, did, k, c in rows:
        name = k.replace("(anonymous namespace)::", "")
        name = name[:60]
        mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        ninst = c.get("SQ_INSTS_VALU_MFMA_F32", 0.0) + c.get("SQ_INSTS_VALU_MFMA_BF16", 0.0)
        grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
        util = busy / (grbm * 1024) if grbm else float("nan")     # MfmaUtil (counter_defs.yaml), SIMD_NUM = 1024
        print(f"{run:16s} {did:5d} {name:60s} flops(MOPS*512)={mops * 512:.4e} mfma_insts={ninst:.4e} "
              f"busy={busy:.4e} busy/inst={busy / ninst if ninst else float('nan'):.2f} grbm={grbm:.4e} "
              f"MfmaUtil={util:.4f}")


if __name__ == "__main__":
    main(sys.argv[1])
