#!/usr/bin/env python3
"""Gradient error of the HIP UNet vs the fp32 and fp64 oracles for one test geometry (tests/test_unet_gpu.py
CASES), for the current PMU_* settings:  python tools/unet_err.py '[64,128,256,512,1024]' 1 2 64 48"""
import ast
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import test_unet_gpu as T  # noqa: E402
from helpers import grad_err, max_abs  # noqa: E402

nf, nc, N, H, W = ast.literal_eval(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
out, out_ref, loss, loss_ref, ggot, gref, sd_after, work = T._run(nf, nc, N, H, W, torch.device("cuda"))
g64, noise = T._NOISE
print(os.environ.get("PMU_WINO4", "1"), "out", max_abs(out, out_ref), "grad vs fp32", grad_err(ggot, gref),
      "vs fp64", grad_err(ggot, g64), "fp32 ref noise", noise, flush=True)
