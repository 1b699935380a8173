#!/usr/bin/env python3
"""Summarise scripts/gpu_mfma_calib.sh: per kernel dispatch the MFMA counters next to the executed
MFMA work the launch implies, to validate SQ_VALU_MFMA_BUSY_CYCLES (MI355X_MICROARCH.md: cycles,
32 per v_mfma_f32_32x32x16_bf16, 32 per v_mfma_f32_16x16x4_f32) and SQ_INSTS_VALU_MFMA_MOPS_* (FLOPs / 512).

Normalisation.  GRBM_GUI_ACTIVE is reported as the sum over the 8 XCDs (MI355X_MICROARCH.md, 'DVFS
give-back'), so the dispatch's cycles are GRBM / 8 and its effective clock GRBM / 8 / wall time (wall
time from the same run's kernel trace).  The counter MFMA-busy fraction is then
    busy / (1024 SIMDs x GRBM / 8)
-- the share of SIMD-cycles the matrix cores were busy at the clock the chip actually held -- and the
fraction of the 2.4 GHz dense peak is  flops / wall / peak.  The two differ by the clock ratio
(f_eff / 2.4 GHz).  counter_defs.yaml's MfmaUtil (busy / (GRBM x SIMD_NUM)) omits the /8 and reads 8x low
on gfx950.

Rows whose effective clock reads above 2.4 GHz (the chip's peak clock) are marked `excluded`: the
counter window of such a dispatch is longer than the dispatch itself (GRBM / 8 > 2.4 GHz x wall), so
neither f_eff nor the busy fraction derived from it is physical.  Short dispatches (batch 1, < 0.3 ms)
fall under the same rule; one long dispatch does too (the first 512-channel bf16 weight-gradient
launch of round 4, 0.40 ms at a read 2.88 GHz, its two repeats at 2.02-2.03 GHz)."""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 1024
F_MAX_GHZ = 2.4        # gfx950 peak engine clock: a higher f_eff means the counter window overran
PEAK = {"bf16": 2.5166e15, "f32": 157.3e12}     # dense MFMA peaks at 2.4 GHz (MI355X_MICROARCH.md)


def _durations(run_dir):
    dur = {}
    for f in glob.glob(os.path.join(run_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return dur


def main(d):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True)):
        run = os.path.relpath(f, d).split(os.sep)[0]
        dur = _durations(os.path.join(d, run))
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (int(r.get("Dispatch_Id") or r.get("Correlation_Id")), r["Kernel_Name"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (did, k), c in per.items():
            rows.append((run, did, k, c, dur.get(did)))
    rows.sort(key=lambda r: (r[0], r[1]))
    print(f"{'run':16s} {'kernel':44s} {'flops=MOPS*512':>14s} {'busy/inst':>9s} {'ms':>7s} {'f_eff GHz':>9s} "
          f"{'busy_frac':>9s} {'peak_frac':>9s} use")
    for run, did, k, c, t in rows:
        mops_b = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        mops_f = c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        if busy == 0.0:
            continue                                 # torch fill / copy kernels of the harness
        ninst = c.get("SQ_INSTS_VALU_MFMA_F32", 0.0) + c.get("SQ_INSTS_VALU_MFMA_BF16", 0.0)
        grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
        cyc = grbm / 8.0
        flops = (mops_b + mops_f) * 512
        peak = PEAK["bf16"] if mops_b >= mops_f else PEAK["f32"]
        name = k.replace("(anonymous namespace)::", "").replace("void ", "")[:44]
        feff = cyc / t / 1e9 if t else float("nan")
        pf = flops / t / peak if t else float("nan")
        print(f"{run:16s} {name:44s} {flops:14.4e} {busy / ninst if ninst else float('nan'):9.2f} "
              f"{(t or float('nan')) * 1e3:7.3f} {feff:9.2f} {busy / (SIMDS * cyc) if cyc else float('nan'):9.3f} "
              f"{pf:9.3f} {'yes' if feff <= F_MAX_GHZ else 'excluded'}")


if __name__ == "__main__":
    main(sys.argv[1])
