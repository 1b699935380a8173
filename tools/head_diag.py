"""Diagnostic: determinism of pmu_head1x1_bwd_bnr (with / without the da store) across repeated calls."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "probabilistic-multiplanar-unet_amd"))
from pmu_hip import _lib as L
from test_bnr_gpu import _bn_inputs
dev = torch.device("cuda", 0)
for (K, C, sig) in [(1, 16, True), (1, 32, True), (1, 64, True), (3, 16, False)]:
    N, H, W = 3, 40, 56
    g = torch.Generator().manual_seed(71 + K + C)
    z, coef, mean, invstd = _bn_inputs(N, H, W, C, g, dev)
    dy = torch.randn(N, K, H, W, generator=g).to(dev)
    y = torch.rand(N, K, H, W, generator=g).to(dev)
    w = (torch.randn(K, C, generator=g) * 0.3).to(dev)
    R = L.lib().pmu_head1x1_bwd_tiles(N, H, W)
    wsb = L.lib().pmu_wgrad1x1_ws(N * H * W, K, C)
    outs = []
    for store in (True, True, False, False):
        da = torch.full((N, H, W, C), float("nan"), device=dev) if store else None
        part = torch.full((R, 2 * C), float("nan"), device=dev)
        dw = torch.full((K, C), float("nan"), device=dev)
        db = torch.full((K,), float("nan"), device=dev)
        ws = torch.full(((wsb + 3) // 4,), float("nan"), device=dev)
        L.call("pmu_head1x1_bwd_bnr", dy.data_ptr(), y.data_ptr(), int(sig), w.data_ptr(), K, C, N, H, W, None,
               L.ptr(da), z.data_ptr(), coef.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(),
               dw.data_ptr(), db.data_ptr(), ws.data_ptr(), wsb, L.stream())
        torch.cuda.synchronize()
        outs.append((part.clone(), dw.clone(), db.clone(), ws[: R * K * (C + 1)].clone()))
    names = ("part", "dw", "db", "ws")
    for i, j in ((0, 1), (2, 3), (0, 2)):
        diffs = {n: float((outs[i][q] - outs[j][q]).abs().max()) for q, n in enumerate(names)}
        nans = {n: int(torch.isnan(outs[i][q]).sum()) for q, n in enumerate(names)}
        print(K, C, sig, (i, j), diffs, "nans", nans, flush=True)
