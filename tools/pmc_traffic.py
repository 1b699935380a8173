#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of one command.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [--steps S]

gfx950 correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE counts half
the bytes of wide (16 B/lane) coalesced reads, and both counters are in KiB, so

    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024        per dispatch.

Every kernel we launch reads with 16-B lanes on its streaming operands, so the doubling applies;
narrower accesses (scalar bias/coefficient reads) are a negligible share.  Output: for each kernel
name, dispatch count and mean fetch / write / HBM bytes per dispatch.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        yield from csv.DictReader(open(f))


def collect(d, counter):
    per = defaultdict(list)
    for r in _rows(d):
        if r["Counter_Name"] != counter:
            continue
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch = collect(fdir, "FETCH_SIZE")
    write = collect(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fm = sum(f) / len(f) if f else 0.0
        wm = sum(w) / len(w) if w else 0.0
        res[k] = {"dispatches_fetch_pass": len(f), "dispatches_write_pass": len(w),
                  "fetch_kib_mean": fm, "write_kib_mean": wm,
                  "hbm_bytes_per_dispatch": (2.0 * fm + wm) * 1024.0}
    meta = {"formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch (gfx950 FETCH_SIZE counts half "
                       "of 16B/lane reads; counters in KiB)",
            "fetch_dir": fdir, "write_dir": wdir}
    steps = 0
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
    if steps > 0:
        # every dispatch of the profiled command (timed + warm-up steps, plus the one-time setup launches:
        # weight init, the first packs) divided by the steps it ran: an upper bound on the per-step bytes
        tot = sum(v["hbm_bytes_per_dispatch"] * max(v["dispatches_fetch_pass"], 1) for v in res.values())
        meta["steps_profiled"] = steps
        meta["hbm_gb_per_step"] = tot / steps / 1e9
        print(f"HBM per step: {tot / steps / 1e9:.2f} GB ({steps} steps profiled, setup launches included)")
    json.dump({"meta": meta, "kernels": res}, open(out, "w"), indent=1)
    top = sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_dispatch"] * max(1, kv[1]["dispatches_fetch_pass"]))
    for k, v in top[:12]:
        print(f"{v['hbm_bytes_per_dispatch'] / 1e6:12.2f} MB/disp  x{v['dispatches_fetch_pass']:4d}  {k[:90]}")


if __name__ == "__main__":
    main()
