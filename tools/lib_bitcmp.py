"""Bit-for-bit comparison of two builds of the HIP library on model steps: the release library
(libpmunet_hip.so) against another one selected by PMU_LIB (default "prev": a previous revision's
release build, e.g. built from `git worktree` of HEAD into pmu_hip/libpmunet_hip_prev.so).  Each build
runs in its own child process on the same seeded model and inputs: UNet forward + backward under
autocast (config c5's bf16 path) and in fp32 (config c2's Winograd path), at geometries whose levels
take the LDS-DMA / F(2x2) / F(4x4) kernels.  Prints one line per case and exits 1 on any difference.
A kernel change meant to move no bits (scheduling, addressing, layouts) is checked with this before it
is measured.

usage: python tools/lib_bitcmp.py [--other prev]"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch
sys.path[:0] = [sys.argv[2], sys.argv[2] + "/probabilistic-multiplanar-unet_amd"]
from model import UNet
dev = torch.device("cuda")
out = {}
cases = [("c5_bf16", True, 3, 3, [64, 128, 256, 512, 1024], 4, 128),
         ("c2_fp32", False, 1, 1, [64, 128, 256, 512, 1024], 4, 128)]
for name, bf16, ch, cl, filters, N, H in cases:
    torch.manual_seed(0)
    net = UNet(ch, cl, filters).to(dev).train()
    g = torch.Generator().manual_seed(8)
    x = torch.rand(N, ch, H, H, generator=g).to(dev)
    r = torch.randn(N, cl, H, H, generator=g).to(dev)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        y = net(x)
    (y.float() * r).sum().backward()
    torch.cuda.synchronize()
    out[name + "/out"] = y.float().cpu()
    for k, p in net.named_parameters():
        out[name + "/grad/" + k] = p.grad.cpu()
    for k, b in net.named_buffers():
        out[name + "/buf/" + k] = b.cpu()
torch.save(out, sys.argv[1])
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--other", default="prev")
    args = ap.parse_args()
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for lib in ("", args.other):
            path = os.path.join(td, f"out_{lib or 'release'}.pt")
            env = dict(os.environ, PMU_LIB=lib)
            r = subprocess.run([sys.executable, "-c", CHILD, path, ROOT], env=env, capture_output=True, text=True,
                               timeout=600)
            if r.returncode != 0:
                print(r.stderr[-3000:])
                return 2
            import torch
            res[lib] = torch.load(path, weights_only=True)
    import torch
    a, b = res[""], res[args.other]
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    cases = sorted({k.split("/")[0] for k in a})
    for c in cases:
        n = sum(1 for k in a if k.startswith(c + "/"))
        nb = sum(1 for k in bad if k.startswith(c + "/"))
        print(f"{c}: {n} tensors, {nb} differ" + (f" (first: {[k for k in bad if k.startswith(c + '/')][:3]})" if nb else ""))
    print("BITCMP", "OK" if not bad else "DIFFER")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
