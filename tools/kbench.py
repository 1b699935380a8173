#!/usr/bin/env python3
"""Per-shape timing of the conv kernels on the c2 layer shapes (batch 32, 256x256 input).

    python tools/kbench.py [--ops fwd,dgrad,wgrad,convT] [--iters 20]

Prints one line per (op, layer shape) with ms and TFLOP/s (% of the f32 MFMA peak 157.3, or of the
bf16 peak 2516 for the *_bf16 ops)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))
import torch  # noqa: E402

from pmu_hip import _lib as L  # noqa: E402
from pmu_hip.engine import Src, frame_of  # noqa: E402

# (H, Cin, Cout) of every 3x3 conv of the c2 U-Net (encoder, then decoder)
SHAPES = [(256, 64, 64), (128, 64, 128), (128, 128, 128), (64, 128, 256), (64, 256, 256), (32, 256, 512),
          (32, 512, 512), (16, 512, 1024), (16, 1024, 1024),
          (32, 1024, 512), (64, 512, 256), (128, 256, 128), (256, 128, 64)]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--only", default=None, help="H,Cin,Cout of a single shape")
    ap.add_argument("--unpacked", action="store_true", help="stage weights from the PyTorch layout")
    ap.add_argument("--c5", action="store_true", help="config c5's layer shapes (512x512 input) at batch 16")
    args = ap.parse_args()
    if args.c5:
        global SHAPES
        SHAPES = [(2 * h, ci, co) for (h, ci, co) in SHAPES]
        if "--N" not in sys.argv:
            args.N = 16
    dev = torch.device("cuda")
    N = args.N
    s = L.stream()
    tot = {}
    shapes = SHAPES if args.only is None else [tuple(int(v) for v in args.only.split(","))]
    for (H, Cin, Cout) in shapes:
        W = H
        z = torch.randn(N, H, W, Cin, device=dev)
        coef = torch.cat([torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1])
        w = torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05
        b = torch.zeros(Cout, device=dev)
        out = torch.empty(N, H, W, Cout, device=dev)
        flops = 2.0 * N * H * W * Cin * Cout * 9
        R = L.lib().pmu_conv3x3_tiles(N, H, W)
        part = torch.empty(R, 2 * Cout, device=dev)
        fin = frame_of([Src(z, L.SRC_BNRELU, coef)], N, H, W)
        da = torch.randn(N, H, W, Cout, device=dev)
        zz = torch.randn(N, H, W, Cout, device=dev)
        bco = torch.cat([torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev) * 0.1,
                         torch.randn(Cout, device=dev) * 0.1, torch.randn(Cout, device=dev) * 0.01,
                         torch.randn(Cout, device=dev) * 0.01])
        fdz = frame_of([Src(da, L.SRC_BNBWD, bco, z=zz)], N, H, W)
        dx = torch.empty(N, H, W, Cin, device=dev)
        dw = torch.empty_like(w)
        wsb = L.lib().pmu_conv3x3_wgrad_ws(N, H, W, Cin, Cout)
        ws = torch.empty(wsb // 4 + 1, device=dev)
        from pmu_hip.engine import pack_weights
        exp = hasattr(L.lib(), "pmu_conv3x3_fwd")   # the direct-sum conv: experiments library (PMU_LIB=exp)
        wpf = pack_weights(w, False) if exp and not args.unpacked else None
        wpd = pack_weights(w, True) if exp and not args.unpacked else None
        def packb(wt, dg):
            n = L.lib().pmu_conv3x3_packed_size_bf16(wt.shape[0], wt.shape[1], int(dg)) // 2
            t = torch.empty(n, dtype=torch.int16, device=dev)
            L.call("pmu_conv3x3_pack_bf16", wt.data_ptr(), wt.shape[0], wt.shape[1], int(dg), t.data_ptr(), s)
            return t
        wbf = packb(w, False)
        wbd = packb(w, True)
        cpo, cpi = (Cout + 7) // 8 * 8, (Cin + 7) // 8 * 8
        dzt = torch.empty(N, H, W, cpo, dtype=torch.int16, device=dev)
        xt = torch.empty(N, H, W, cpi, dtype=torch.int16, device=dev)
        L.call("pmu_frame_to_bf16", fdz, cpo, dzt.data_ptr(), s)
        L.call("pmu_frame_to_bf16", fin, cpi, xt.data_ptr(), s)
        wsbb = L.lib().pmu_conv3x3_wgrad_ws_bf16(N, H, W, Cin, Cout)
        wsb16 = torch.empty(wsbb // 4 + 1, device=dev)
        wsbd = L.lib().pmu_conv3x3_wgrad_ws_bf16_dma(N, H, W, Cin, Cout)
        wsd16 = torch.empty(wsbd // 4 + 1, device=dev)
        def packr(wt, dg):
            n = L.lib().pmu_conv3x3_packed_size_raw(wt.shape[0], wt.shape[1], int(dg)) // 2
            t = torch.empty(n, dtype=torch.int16, device=dev)
            L.call("pmu_conv3x3_pack_raw", wt.data_ptr(), wt.shape[0], wt.shape[1], int(dg), t.data_ptr(), s)
            return t
        wrf = packr(w, False)
        partr = torch.empty(L.lib().pmu_conv3x3_tiles_raw(N, H, W, Cout), 2 * Cout, device=dev)
        wrd = packr(w, True)
        xt32 = torch.randn(N, H, W, Cin, device=dev)
        dzt32 = torch.randn(N, H, W, Cout, device=dev)
        wsbw = L.lib().pmu_conv3x3_wgrad_ws_wino(N, H, W, Cin, Cout)
        wsw = torch.empty(max(wsbw, 4) // 4, device=dev)
        wsb4 = L.lib().pmu_conv3x3_wgrad_ws_wino4(N, H, W, Cin, Cout) if exp else 0
        ws4 = torch.empty(max(wsb4, 4) // 4, device=dev)
        from pmu_hip.engine import pack_weights_wino
        wwf, wwd = pack_weights_wino(w, False), pack_weights_wino(w, True)
        partw = torch.empty(L.lib().pmu_conv3x3_tiles_wino(N, H, W), 2 * Cout, device=dev)
        from pmu_hip.engine import pack_weights_wino4
        w4f, w4d = pack_weights_wino4(w, False), pack_weights_wino4(w, True)
        part4 = torch.empty(L.lib().pmu_conv3x3_tiles_wino4(N, H, W), 2 * Cout, device=dev)
        from pmu_hip.engine import pack_weights_wino2h
        w2f, w2d = pack_weights_wino2h(w, False), pack_weights_wino2h(w, True)
        def packd(wt, dg):
            n = L.lib().pmu_conv3x3_packed_size_dma(wt.shape[0], wt.shape[1], int(dg)) // 2
            t = torch.empty(n, dtype=torch.int16, device=dev)
            L.call("pmu_conv3x3_pack_dma", wt.data_ptr(), wt.shape[0], wt.shape[1], int(dg), t.data_ptr(), s)
            return t
        wdf, wdd = packd(w, False), packd(w, True)
        partd = torch.empty(L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cout, cpi), 2 * Cout, device=dev)
        # a producer of the Cin channels for the *_bnr input gradients (BN-backward partials in the epilogue)
        zp = torch.randn(N, H, W, Cin, device=dev)
        cp = torch.cat([torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1])
        mp, ip = torch.randn(Cin, device=dev) * 0.1, torch.rand(Cin, device=dev) + 0.5
        def bnr(tiles):
            pp = torch.empty(tiles, 2 * Cin, device=dev)
            return (dx.data_ptr(), zp.data_ptr(), cp.data_ptr(), mp.data_ptr(), ip.data_ptr(), pp.data_ptr(), s)
        bnr4 = bnr(L.lib().pmu_conv3x3_tiles_wino4(N, H, W))
        bnr2 = bnr(L.lib().pmu_conv3x3_tiles_wino2h(N, H, W))
        bnrd = bnr(L.lib().pmu_conv3x3_tiles_dma(N, H, W, Cin, cpo))
        dxb = torch.empty(N, H, W, Cin, dtype=torch.int16, device=dev)
        # the c5 operand streams (frame_stream_kernel): BN-backward dz from a bf16 activation gradient (the
        # *_dxb dx), and the max-pooled BN+ReLU operand with its unpooled skip half written in the same pass
        dab = torch.randn(N, H, W, Cout, device=dev).to(torch.bfloat16).view(torch.int16)
        fdzb = frame_of([Src(dab, L.SRC_BNBWD, bco, z=zz)], N, H, W)
        fpool = frame_of([Src(z, L.SRC_BNRELU, coef, pool=L.POOL_MAX2)], N, H // 2, W // 2)
        pool_ok = bool(L.lib().pmu_frame_pool_skip_ok(fpool)) and H % 2 == 0
        pooled = torch.empty(N, H // 2, W // 2, Cin, dtype=torch.int16, device=dev) if pool_ok else None
        xcat = torch.empty(N, H, W, 2 * Cin, dtype=torch.int16, device=dev) if pool_ok else None
        # the max-pool backward of a skip level (c5, bf16 parts): C = Cout channels at H x W, the pooled
        # gradient at H/2 x W/2 — the stats-only pass (BN-backward partials) and the dz pass
        dpb = torch.randn(N, H // 2, W // 2, Cout, device=dev).to(torch.bfloat16).view(torch.int16)
        dskb = torch.randn(N, H, W, Cout, device=dev).to(torch.bfloat16).view(torch.int16)
        mpm, mpi = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
        mpc = bco[:2 * Cout].contiguous()
        mpart = torch.empty(L.lib().pmu_maxpool2_bwd_bnr_tiles(N, H, W, Cout), 2 * Cout, device=dev)
        mdz = torch.empty(N, H, W, Cout, dtype=torch.int16, device=dev)
        px = N * H * W
        hbm = {"mat32": px * Cin * 4 * 2,
               "mat32_bnbwd": px * Cout * 4 * 3,
               "mp_stats_xb": px // 4 * Cout * 2 + px * Cout * (2 + 4),
               "mp_bnbwd_xb": px // 4 * Cout * 2 + px * Cout * (2 + 4) + px * Cout * 2,"mat_bnrelu": px * Cin * 4 + px * cpi * 2,
               "mat_bnbwd_xb": px * Cout * (2 + 4) + px * cpo * 2,
               "mat_pool_skip": px * Cin * 4 + px // 4 * Cin * 2 + px * Cin * 2}
        ops = {
            "dgrad_w4b": lambda: L.call("pmu_conv3x3_dgrad_wino4_bnr", dzt32.data_ptr(), Cout, N, H, W, w4d.data_ptr(),
                                        Cin, *bnr4),
            "dgrad_w2hb": lambda: L.call("pmu_conv3x3_dgrad_wino2h_bnr", dzt32.data_ptr(), Cout, N, H, W,
                                         w2d.data_ptr(), Cin, *bnr2),
            "dgrad_dmab": lambda: L.call("pmu_conv3x3_dgrad_dma_bnr", dzt.data_ptr(), cpo, N, H, W, wdd.data_ptr(), Cin,
                                         *bnrd),
            # c5's shipped forms: bf16 dx (the *_dxb entries), with and without the producer's BN partials
            "dgrad_dmabx": lambda: L.call("pmu_conv3x3_dgrad_dma_bnr_dxb", dzt.data_ptr(), cpo, N, H, W, wdd.data_ptr(),
                                          Cin, dxb.data_ptr(), *bnrd[1:]),
            "dgrad_dmax": lambda: L.call("pmu_conv3x3_dgrad_dma_dxb", dzt.data_ptr(), cpo, N, H, W, wdd.data_ptr(), Cin,
                                         Cin, dxb.data_ptr(), None, s),
            "fwd_dma": lambda: L.call("pmu_conv3x3_fwd_dma", xt.data_ptr(), cpi, N, H, W, wdf.data_ptr(), b.data_ptr(),
                                      Cout, out.data_ptr(), partd.data_ptr(), s),
            "dgrad_dma": lambda: L.call("pmu_conv3x3_dgrad_dma", dzt.data_ptr(), cpo, N, H, W, wdd.data_ptr(), Cin, Cin,
                                        dx.data_ptr(), None, s),
            "fwd_raw": lambda: L.call("pmu_conv3x3_fwd_raw", xt.data_ptr(), cpi, N, H, W, wrf.data_ptr(), b.data_ptr(),
                                      Cout, out.data_ptr(), partr.data_ptr(), s),
            "dgrad_raw": lambda: L.call("pmu_conv3x3_dgrad_raw", dzt.data_ptr(), cpo, N, H, W, wrd.data_ptr(), Cin, Cin,
                                        dx.data_ptr(), None, s),
            "wgrad_bf16": lambda: L.call("pmu_conv3x3_wgrad_bf16", dzt.data_ptr(), xt.data_ptr(), N, H, W, Cout, Cin,
                                         dw.data_ptr(), wsb16.data_ptr(), wsbb, s),
            "wgrad_bf16d": lambda: L.call("pmu_conv3x3_wgrad_bf16_dma", dzt.data_ptr(), xt.data_ptr(), N, H, W, Cout,
                                          Cin, dw.data_ptr(), wsd16.data_ptr(), wsbd, s),
            "mat_bnrelu": lambda: L.call("pmu_frame_to_bf16", fin, cpi, xt.data_ptr(), s),
            "mat_bnbwd_xb": lambda: L.call("pmu_frame_to_bf16", fdzb, cpo, dzt.data_ptr(), s),
            "mat_pool_skip": (lambda: L.call("pmu_frame_to_bf16_pool_skip", fpool, pooled.data_ptr(), xcat.data_ptr(),
                                             2 * Cin, s)) if pool_ok else None,
            "mp_stats_xb": lambda: L.call("pmu_maxpool2_bwd_bnr_stats_dxb", dpb.data_ptr(), dskb.data_ptr(), zz.data_ptr(),
                                          mpc.data_ptr(), mpm.data_ptr(), mpi.data_ptr(), N, H, W, Cout,
                                          mpart.data_ptr(), s),
            "mp_bnbwd_xb": lambda: L.call("pmu_maxpool2_bwd_bnbwd_dxb", dpb.data_ptr(), dskb.data_ptr(), zz.data_ptr(),
                                          mpc.data_ptr(), bco.data_ptr(), N, H, W, Cout, Cout, mdz.data_ptr(), s),
            "mat_bf16": lambda: (L.call("pmu_frame_to_bf16", fdz, cpo, dzt.data_ptr(), s),
                                 L.call("pmu_frame_to_bf16", fin, cpi, xt.data_ptr(), s)),
            "fwd_bf16": lambda: L.call("pmu_conv3x3_fwd_bf16", fin, wbf.data_ptr(), b.data_ptr(), Cout,
                                       out.data_ptr(), part.data_ptr(), xt.data_ptr(), s),
            "dgrad_bf16": lambda: L.call("pmu_conv3x3_dgrad_bf16", fdz, wbd.data_ptr(), Cin, Cin, dx.data_ptr(),
                                         None, dzt.data_ptr(), s),
            "fwd": lambda: L.call("pmu_conv3x3_fwd", fin, w.data_ptr(), L.ptr(wpf), b.data_ptr(), Cout,
                                  out.data_ptr(), part.data_ptr(), None, s),
            "dgrad": lambda: L.call("pmu_conv3x3_dgrad", fdz, w.data_ptr(), L.ptr(wpd), Cin, Cin, dx.data_ptr(),
                                    None, None, s),
            "fwd_tee": lambda: L.call("pmu_conv3x3_fwd", fin, w.data_ptr(), L.ptr(wpf), b.data_ptr(), Cout,
                                      out.data_ptr(), part.data_ptr(), xt32.data_ptr(), s),
            "dgrad_tee": lambda: L.call("pmu_conv3x3_dgrad", fdz, w.data_ptr(), L.ptr(wpd), Cin, Cin, dx.data_ptr(),
                                        None, dzt32.data_ptr(), s),
            "wgrad_t32": lambda: L.call("pmu_conv3x3_wgrad", frame_of([Src(dzt32)], N, H, W),
                                        frame_of([Src(xt32)], N, H, W), Cout, dw.data_ptr(), ws.data_ptr(), wsb, s),
            "fwd_wr": lambda: L.call("pmu_conv3x3_fwd_wino_raw", xt32.data_ptr(), Cin, N, H, W, wwf.data_ptr(),
                                       b.data_ptr(), Cout, out.data_ptr(), partw.data_ptr(), s),
            "dgrad_wr": lambda: L.call("pmu_conv3x3_dgrad_wino_raw", dzt32.data_ptr(), Cout, N, H, W, wwd.data_ptr(),
                                         Cin, Cin, dx.data_ptr(), None, s),
            "fwd_w4": lambda: L.call("pmu_conv3x3_fwd_wino4", xt32.data_ptr(), Cin, N, H, W, w4f.data_ptr(),
                                     b.data_ptr(), Cout, out.data_ptr(), part4.data_ptr(), s),
            "dgrad_w4": lambda: L.call("pmu_conv3x3_dgrad_wino4", dzt32.data_ptr(), Cout, N, H, W, w4d.data_ptr(),
                                       Cin, Cin, dx.data_ptr(), None, s),
            "fwd_w2h": lambda: L.call("pmu_conv3x3_fwd_wino2h", xt32.data_ptr(), Cin, N, H, W, w2f.data_ptr(),
                                      b.data_ptr(), Cout, out.data_ptr(), partw.data_ptr(), s),
            "dgrad_w2h": lambda: L.call("pmu_conv3x3_dgrad_wino2h", dzt32.data_ptr(), Cout, N, H, W, w2d.data_ptr(),
                                        Cin, Cin, dx.data_ptr(), None, s),
            "mat32": lambda: L.call("pmu_frame_to_f32", fin, xt32.data_ptr(), s),
            "mat32_bnbwd": lambda: L.call("pmu_frame_to_f32", fdz, dzt32.data_ptr(), s),
            "fwd_wino": lambda: L.call("pmu_conv3x3_fwd_wino", fin, wwf.data_ptr(), b.data_ptr(), Cout,
                                       out.data_ptr(), partw.data_ptr(), None, s),
            "dgrad_wino": lambda: L.call("pmu_conv3x3_dgrad_wino", fdz, wwd.data_ptr(), Cin, Cin, dx.data_ptr(),
                                         None, None, s),
            "wgrad_w4": lambda: L.call("pmu_conv3x3_wgrad_wino4", dzt32.data_ptr(), xt32.data_ptr(), N, H, W, Cout,
                                       Cin, dw.data_ptr(), ws4.data_ptr(), wsb4, s),
            "wgrad_wino": lambda: L.call("pmu_conv3x3_wgrad_wino", dzt32.data_ptr(), xt32.data_ptr(), N, H, W, Cout,
                                         Cin, dw.data_ptr(), wsw.data_ptr(), wsbw, s),
            "pack": lambda: pack_weights(w, False),
            "wgrad": lambda: L.call("pmu_conv3x3_wgrad", fdz, fin, Cout, dw.data_ptr(), ws.data_ptr(), wsb, s),
        }
        for op in args.ops.split(","):
            if ops.get(op) is None:
                continue
            ms = timeit(ops[op], args.iters)
            if op in hbm:
                tot.setdefault(op, [0.0, 0.0])
                tot[op][0] += ms
                tot[op][1] += hbm[op]
                print(f"{op:6s} H={H:4d} Cin={Cin:5d} Cout={Cout:5d}  {ms:8.3f} ms  "
                      f"{hbm[op] / (ms * 1e-3) / 1e9:7.1f} GB/s  ({hbm[op] / 1e6:8.1f} MB algorithmic)", flush=True)
                continue
            tf = flops / (ms * 1e-3) / 1e12
            tot.setdefault(op, [0.0, 0.0])
            tot[op][0] += ms
            tot[op][1] += flops
            peak = 2516.0 if (op.endswith("bf16") or op.endswith("bf16d") or op.endswith("raw") or "dma" in op) else 157.3
            print(f"{op:6s} H={H:4d} Cin={Cin:5d} Cout={Cout:5d}  {ms:8.3f} ms  {tf:7.2f} TF  ({tf / peak * 100:5.1f}%)",
                  flush=True)
    for op, (ms, fl) in tot.items():
        if op in hbm:
            print(f"TOTAL {op:6s} {ms:8.3f} ms  {fl / (ms * 1e-3) / 1e9:7.1f} GB/s")
        else:
            print(f"TOTAL {op:6s} {ms:8.3f} ms  {fl / (ms * 1e-3) / 1e12:7.2f} TF")


if __name__ == "__main__":
    main()
