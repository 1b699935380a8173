#!/usr/bin/env python3
"""Print tools/dice_gap_seeds.py's JSON as a per-seed table (eval / train gaps per column, flips, near-ties).

usage: python tools/dice_gap_table.py dice_gap_seeds.json"""
import json
import sys

COLS = ["o32gpu", "o64", "oac", "oacf", "oacb", "tac", "hip32", "hip16", "hip16dx"]


def main(path):
    d = json.load(open(path))
    cols = [c for c in COLS if c in d["rows"][0]]
    print(d.get("geometry", ""), "steps", d.get("steps"), "| gaps = max per-class |Dice - Dice(ref fp32 CPU oracle)|")
    print(f"{'seed':>4} {'mode':>5} " + " ".join(f"{c:>9}" for c in cols) + "   ref near-ties (<1e-3 / <1e-2 px)")
    for r in d["rows"]:
        for m in ("eval", "train"):
            tail = (f"   {r['ref_eval_pixels_margin_lt_1e-3']} / {r['ref_eval_pixels_margin_lt_1e-2']}"
                    if m == "eval" else "")
            print(f"{r['seed']:>4} {m:>5} " + " ".join(f"{r[c]['gap_' + m]:9.2e}" for c in cols) + tail)
        print(f"{'':>4} {'flips':>5} " + " ".join(f"{r[c]['flips_eval']:>9d}" for c in cols))
    for m in ("eval", "train"):
        print(f"{'max':>4} {m:>5} " + " ".join(f"{max(r[c]['gap_' + m] for r in d['rows']):9.2e}" for c in cols))
        print(f"{'mean':>4} {m:>5} " + " ".join(
            f"{sum(r[c]['gap_' + m] for r in d['rows']) / len(d['rows']):9.2e}" for c in cols))


if __name__ == "__main__":
    main(sys.argv[1])
