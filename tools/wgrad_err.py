#!/usr/bin/env python3
"""fp32 rounding of the 3x3 weight gradient computed by Winograd F(2x2,3x3) vs F(4x4,3x3), emulated in
numpy against the fp64 direct sum (the autograd of nn.Conv2d w.r.t. its weight, PMU/model/unet/
unet_parts.py:15,18).  Per-tile products are accumulated sequentially in fp32 within a split of
`--tiles-per-split` tiles (as the MFMA K loop does), splits summed in fp32, output transform in fp64.

    python tools/wgrad_err.py [--H 64] [--C 32] [--N 2]
"""
import argparse

import numpy as np

BT4 = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], dtype=np.float64)
G4 = np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
               [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], dtype=np.float64)
AT4 = np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]], dtype=np.float64)
BT2 = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=np.float64)
G2 = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=np.float64)
AT2 = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=np.float64)


def direct(x, dy):
    """fp64 dw[co][ci][a][b] = sum_{n,h,w} dy[n,h,w,co] * xpad[n,h+a,w+b,ci]."""
    N, H, W, Ci = x.shape
    xp = np.zeros((N, H + 2, W + 2, Ci))
    xp[:, 1:-1, 1:-1] = x
    dw = np.zeros((dy.shape[3], Ci, 3, 3))
    for a in range(3):
        for b in range(3):
            dw[:, :, a, b] = np.einsum("nhwo,nhwi->oi", dy, xp[:, a:a + H, b:b + W])
    return dw


def winograd(x, dy, m, tps):
    """fp32 emulation of the Winograd weight gradient with output tiles m x m."""
    BT, G, AT = (BT4, G4, AT4) if m == 4 else (BT2, G2, AT2)
    a = m + 2
    N, H, W, Ci = x.shape
    Co = dy.shape[3]
    th, tw = -(-H // m), -(-W // m)
    xp = np.zeros((N, th * m + 2, tw * m + 2, Ci), np.float32)
    xp[:, 1:H + 1, 1:W + 1] = x
    dp = np.zeros((N, th * m, tw * m, Co), np.float32)
    dp[:, :H, :W] = dy
    BT32, A32 = BT.astype(np.float32), AT.T.astype(np.float32)
    # per tile: Z = A dY A^T (a x a x Co), V = B^T X B (a x a x Ci), in fp32
    Zs, Vs = [], []
    for n in range(N):
        for ty in range(th):
            for tx in range(tw):
                X = xp[n, ty * m:ty * m + a, tx * m:tx * m + a]          # a x a x Ci
                D = dp[n, ty * m:ty * m + m, tx * m:tx * m + m]          # m x m x Co
                V = np.einsum("ir,rsc,js->ijc", BT32, X, BT32).astype(np.float32)
                Z = np.einsum("ir,rsc,js->ijc", A32, D, A32).astype(np.float32)
                Zs.append(Z)
                Vs.append(V)
    T = len(Zs)
    Mtot = np.zeros((a, a, Co, Ci), np.float32)
    for s0 in range(0, T, tps):
        Ms = np.zeros((a, a, Co, Ci), np.float32)
        for t in range(s0, min(T, s0 + tps)):
            Ms += np.einsum("ijo,ijc->ijoc", Zs[t], Vs[t]).astype(np.float32)
        Mtot += Ms
    M = Mtot.astype(np.float64)
    return np.einsum("ai,ijoc,jb->ocab", G.T, M, G)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=2)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--C", type=int, default=16)
    ap.add_argument("--tiles-per-split", type=int, default=64)
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    x = np.maximum(rng.standard_normal((args.N, args.H, args.H, args.C)), 0).astype(np.float32)   # ReLU-like
    dy = (rng.standard_normal((args.N, args.H, args.H, args.C)) * 1e-3).astype(np.float32)
    ref = direct(x.astype(np.float64), dy.astype(np.float64))
    scale = np.abs(ref).max()
    # the fp32 direct sum (sequential per split, as a direct-sum GEMM would)
    for m in (2, 4):
        got = winograd(x, dy, m, args.tiles_per_split)
        err = got - ref
        print(f"F({m}x{m}) wgrad: max |err| / max|dw| = {np.abs(err).max() / scale:.3e}, "
              f"rms / rms = {np.sqrt((err ** 2).mean() / (ref ** 2).mean()):.3e}")


if __name__ == "__main__":
    main()
