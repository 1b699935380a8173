"""Round 6's conflict-free Winograd patch reads (DESIGN.md §3a'): the F(2x2) and F(4x4) kernels read a
lane's patch as ds_read_b64 channel pairs and only the rows its component half uses; the round-5 form
(one ds_read_b32 per channel and element) stays selectable in the experiments library
(PMU_WINO2H_B32=1 / PMU_WINO4_B32=1, read once per process).  The two forms do the same arithmetic in
the same order, so their outputs — z, dx, and the BN partial sums of the fused epilogues — must be equal
bit for bit.  Each form runs in its own child process on the same seeded inputs."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch
sys.path[:0] = [sys.argv[2], sys.argv[2] + "/probabilistic-multiplanar-unet_amd"]
from pmu_hip import _lib as L
from pmu_hip.engine import pack_weights_wino2h, pack_weights_wino4
dev = torch.device("cuda")
out = {}
for (N, H, W, Cin, Cout) in [(2, 32, 48, 64, 64), (1, 45, 37, 128, 64), (4, 16, 16, 256, 128), (1, 64, 70, 32, 96)]:
    g = torch.Generator().manual_seed(H * 131 + Cin)
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    dz = torch.randn(N, H, W, Cout, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    zp = torch.randn(N, H, W, Cin, generator=g).to(dev)
    cp = torch.cat([torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.1]).to(dev)
    mp, ip = (torch.randn(Cin, generator=g) * 0.1).to(dev), (torch.rand(Cin, generator=g) + 0.5).to(dev)
    s = L.stream()
    key = f"{N}x{H}x{W}x{Cin}x{Cout}"
    z = torch.empty(N, H, W, Cout, device=dev)
    part = torch.empty(L.lib().pmu_conv3x3_tiles_wino2h(N, H, W), 2 * Cout, device=dev)
    L.call("pmu_conv3x3_fwd_wino2h", x.data_ptr(), Cin, N, H, W, pack_weights_wino2h(w, False).data_ptr(),
           b.data_ptr(), Cout, z.data_ptr(), part.data_ptr(), s)
    out[key + "/fwd2/z"], out[key + "/fwd2/part"] = z, part
    dx = torch.empty(N, H, W, Cin, device=dev)
    L.call("pmu_conv3x3_dgrad_wino2h", dz.data_ptr(), Cout, N, H, W, pack_weights_wino2h(w, True).data_ptr(), Cin,
           Cin, dx.data_ptr(), None, s)
    out[key + "/dgrad2/dx"] = dx
    if H >= 32 and W >= 32:
        w4 = pack_weights_wino4(w, True)
        dx4 = torch.empty(N, H, W, Cin, device=dev)
        L.call("pmu_conv3x3_dgrad_wino4", dz.data_ptr(), Cout, N, H, W, w4.data_ptr(), Cin, Cin, dx4.data_ptr(),
               None, s)
        out[key + "/dgrad4/dx"] = dx4
        dx4b = torch.empty(N, H, W, Cin, device=dev)
        p4 = torch.empty(L.lib().pmu_conv3x3_tiles_wino4(N, H, W), 2 * Cin, device=dev)
        L.call("pmu_conv3x3_dgrad_wino4_bnr", dz.data_ptr(), Cout, N, H, W, w4.data_ptr(), Cin, dx4b.data_ptr(),
               zp.data_ptr(), cp.data_ptr(), mp.data_ptr(), ip.data_ptr(), p4.data_ptr(), s)
        out[key + "/dgrad4b/dx"], out[key + "/dgrad4b/part"] = dx4b, p4
torch.cuda.synchronize()
torch.save({k: v.cpu() for k, v in out.items()}, sys.argv[1])
'''


def test_b64_patch_reads_bit_equal_to_b32(tmp_path):
    from pmu_hip import _lib as L
    if not os.path.exists(L.EXP_LIB_PATH):
        pytest.skip("experiments library not built (make -C csrc EXPERIMENTS=1)")
    res = {}
    for b32 in ("0", "1"):
        path = str(tmp_path / f"b32_{b32}.pt")
        env = dict(os.environ, PMU_LIB="exp", PMU_WINO2H_B32=b32, PMU_WINO4_B32=b32)
        r = subprocess.run([sys.executable, "-c", CHILD, path, ROOT], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        res[b32] = torch.load(path, weights_only=True)
    assert res["0"].keys() == res["1"].keys() and len(res["0"]) >= 16
    for k in res["0"]:
        assert torch.equal(res["0"][k], res["1"][k]), k
