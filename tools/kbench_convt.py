#!/usr/bin/env python3
"""Per-shape timing of the ConvTranspose2d(k2, s2) kernels on the c2 decoder shapes (batch 32).

    python tools/kbench_convt.py [--ops fwd,dgrad,wgrad] [--iters 20]

TFLOP/s against the f32 MFMA peak 157.3 (2 * M * Cin * 4 * Cout FLOP per pass)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402
from pmu_hip import _lib as L  # noqa: E402
from pmu_hip.engine import Src, frame_of, pack_convT_weights  # noqa: E402

# (H_in, Cin, Cout) of the 4 Up blocks' ConvTranspose2d
SHAPES = [(16, 1024, 512), (32, 512, 256), (64, 256, 128), (128, 128, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--c5", action="store_true", help="config c5's decoder shapes (512x512 input), batch 16")
    args = ap.parse_args()
    global SHAPES
    if args.c5:
        SHAPES = [(2 * h, ci, co) for (h, ci, co) in SHAPES]
        if "--N" not in sys.argv:
            args.N = 16
    dev = torch.device("cuda")
    N, s = args.N, L.stream()
    tot = {}
    for (H, Cin, Cout) in SHAPES:
        W, Hd, Wd = H, 2 * H, 2 * H
        z = torch.randn(N, H, W, Cin, device=dev)
        coef = torch.cat([torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1])
        w = torch.randn(Cin, Cout, 2, 2, device=dev) * 0.05
        b = torch.zeros(Cout, device=dev)
        u = torch.empty(N, Hd, Wd, Cout, device=dev)
        du = torch.randn(N, Hd, Wd, Cout, device=dev)
        dx = torch.empty(N, H, W, Cin, device=dev)
        dw = torch.empty_like(w)
        db = torch.empty(Cout, device=dev)
        fin = frame_of([Src(z, L.SRC_BNRELU, coef)], N, H, W)
        wpf, wpd = pack_convT_weights(w, False), pack_convT_weights(w, True)
        wsb = L.lib().pmu_convT2x2_wgrad_ws(N, H, W, Cin, Cout)
        ws = torch.empty(max(1, (wsb + 3) // 4), device=dev)
        flops = 2.0 * N * H * W * Cin * Cout * 4
        from pmu_hip.engine import frame_to_bf16, pack_convT_weights_bf16, pack_convT_weights_dma
        xt = frame_to_bf16([Src(z, L.SRC_BNRELU, coef)], N, H, W)
        dut = frame_to_bf16([Src(du)], N, Hd, Wd)
        exp = hasattr(L.lib(), "pmu_convT2x2_pack_bf16")   # register-staged bf16 ConvT: experiments library
        wbf, wbd = (pack_convT_weights_bf16(w, False), pack_convT_weights_bf16(w, True)) if exp else (None, None)
        wdf, wdd = pack_convT_weights_dma(w, False), pack_convT_weights_dma(w, True)
        wsbb = L.lib().pmu_convT2x2_wgrad_ws_bf16(N, H, W, Cin, Cout)
        wsb16 = torch.empty(max(1, (wsbb + 3) // 4), device=dev)
        ucat = torch.empty(N, Hd, Wd, 2 * Cout, dtype=torch.int16, device=dev)   # c5: bf16 into the concat operand
        ops = {
            "fwd_bf16": lambda: L.call("pmu_convT2x2_fwd_bf16", fin, wbf.data_ptr(), b.data_ptr(), Cout, u.data_ptr(), s),
            "fwd_dma": lambda: L.call("pmu_convT2x2_fwd_dma", xt.data_ptr(), xt.shape[3], N, H, W, wdf.data_ptr(),
                                      b.data_ptr(), Cin, Cout, u.data_ptr(), s),
            "dgrad_bf16": lambda: L.call("pmu_convT2x2_dgrad_bf16", du.data_ptr(), Hd, Wd, 0, 0, wbd.data_ptr(), N, H, W,
                                         Cin, Cout, dx.data_ptr(), s),
            "fwd_ldb": lambda: L.call("pmu_convT2x2_fwd_dma_ldb", xt.data_ptr(), xt.shape[3], N, H, W, wdf.data_ptr(),
                                      b.data_ptr(), Cin, Cout, ucat.data_ptr(), 2 * Cout, s),
            "dgrad_dma": lambda: L.call("pmu_convT2x2_dgrad_dma", dut.data_ptr(), dut.shape[3], Hd, Wd, 0, 0,
                                        wdd.data_ptr(), N, H, W, Cin, Cout, dx.data_ptr(), s),
            "wgrad_bf16": lambda: L.call("pmu_convT2x2_wgrad_bf16", xt.data_ptr(), dut.data_ptr(), du.data_ptr(), N, H, W,
                                         Hd, Wd, 0, 0, Cin, Cout, dw.data_ptr(), db.data_ptr(), wsb16.data_ptr(), wsbb, s),
            "fwd": lambda: L.call("pmu_convT2x2_fwd", fin, w.data_ptr(), wpf.data_ptr(), b.data_ptr(), Cout,
                                  u.data_ptr(), s),
            "dgrad": lambda: L.call("pmu_convT2x2_dgrad", du.data_ptr(), Hd, Wd, 0, 0, w.data_ptr(), wpd.data_ptr(),
                                    N, H, W, Cin, Cout, dx.data_ptr(), s),
            "wgrad": lambda: L.call("pmu_convT2x2_wgrad", du.data_ptr(), Hd, Wd, 0, 0, fin, Cout, dw.data_ptr(),
                                    db.data_ptr(), ws.data_ptr(), wsb, s),
        }
        # algorithmic HBM bytes of the LDS-DMA / bf16 kernels as kbench calls them (fp32 u / dx here; c5's
        # *_ldb / *_dxb forms store bf16): the pass is bound by these, not by its MFMAs (2 FLOP per 4-6 B)
        pin = N * H * W
        hbm = {"fwd_dma": pin * Cin * 2 + 4 * pin * Cout * 4 + Cin * Cout * 4 * 2,
               "fwd_ldb": pin * Cin * 2 + 4 * pin * Cout * 2 + Cin * Cout * 4 * 2,
               "dgrad_dma": 4 * pin * Cout * 2 + pin * Cin * 4 + Cin * Cout * 4 * 2,
               "wgrad_bf16": pin * Cin * 2 + 4 * pin * Cout * (2 + 4) + Cin * Cout * 4 * 4}
        for op in args.ops.split(","):
            if op not in ops:
                continue
            ms = timeit(ops[op], args.iters)
            if op in hbm:
                print(f"{op:6s} H={H:4d} Cin={Cin:5d} Cout={Cout:5d}  {hbm[op] / 1e6:8.1f} MB algorithmic  "
                      f"{hbm[op] / (ms * 1e-3) / 1e9:7.1f} GB/s", flush=True)
            tf = flops / (ms * 1e-3) / 1e12
            tot.setdefault(op, [0.0, 0.0])
            tot[op][0] += ms
            tot[op][1] += flops
            peak = 2516.0 if ("bf16" in op or "dma" in op) else 157.3
            print(f"{op:6s} H={H:4d} Cin={Cin:5d} Cout={Cout:5d}  {ms:8.3f} ms  {tf:7.2f} TF  ({tf / peak * 100:5.1f}%)",
                  flush=True)
    for op, (ms, fl) in tot.items():
        print(f"TOTAL {op:6s} {ms:8.3f} ms  {fl / (ms * 1e-3) / 1e12:7.2f} TF")


if __name__ == "__main__":
    main()
