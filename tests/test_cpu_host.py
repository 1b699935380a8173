"""CPU-only checks: oracle vs the reference's golden vectors, drop-in surface, C ABI exports.

No GPU compute here: the library is loaded and its symbols resolved, nothing is launched.
"""
import os
import re

import numpy as np
import pytest
import torch

from helpers import ACT_TOL, GRAD_TOL, LOSS_RTOL, grad_err, max_abs

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _sd(z, prefix):
    pre = prefix + "/"
    return {k[len(pre):]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith(pre)}


# ----------------------------------------------------------------------------- oracle pinning
def test_oracle_matches_reference_g1_step():
    """G1 (config c1): one train step of UNet(1,1,[16,32]) — outputs, loss, grads, BN stats."""
    from oracle.unet_ref import unet_forward, unet_loss, unet_param_keys
    z = _load("g1_unet_c1.npz")
    sd = _sd(z, "init")
    x, t = torch.from_numpy(z["x0"]), torch.from_numpy(z["t0"])
    keys = unet_param_keys(sd)
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    y = unet_forward(work, x, 2, 1)
    loss = unet_loss(y, t, 1)
    loss.backward()
    assert max_abs(y, torch.from_numpy(z["y0"])) <= 1e-6
    assert abs(float(loss) - float(z["loss0"])) <= 1e-6
    gref = _sd(z, "grad0")
    err, key = grad_err({k: params[k].grad for k in keys}, gref)
    assert err <= 1e-5, (err, key)
    after = _sd(z, "after0")
    for k in after:
        if "running" in k:
            assert max_abs(work[k], after[k]) <= 1e-6, k


def test_oracle_matches_reference_g1_ten_steps():
    """G1: params after 10 clip(0.1)+SGD(lr 1e-3, momentum 0.9) steps (train.py:85-110)."""
    from oracle.unet_ref import unet_param_keys, unet_train_step
    z = _load("g1_unet_c1.npz")
    sd = _sd(z, "init")
    bufs = {k: torch.zeros_like(sd[k]) for k in unet_param_keys(sd)}
    losses = []
    for i in range(10):
        _, loss, _ = unet_train_step(sd, torch.from_numpy(z[f"x{i}"]), torch.from_numpy(z[f"t{i}"]), 2, 1,
                                     lr=1e-3, bufs=bufs)
        losses.append(float(loss))
    assert np.allclose(losses, z["losses"], rtol=1e-5, atol=1e-6)
    final = _sd(z, "final")
    for k, v in final.items():
        assert max_abs(sd[k], v) <= 1e-5, k


@pytest.mark.parametrize("tag", ["s64", "s170"])
def test_oracle_matches_reference_g2(tag):
    """G2: all 5 levels at small width, CE loss; 170x170 exercises the F.pad branch."""
    from oracle.unet_ref import unet_forward, unet_loss, unet_param_keys
    z = _load("g2_unet_multiclass.npz")
    sd = _sd(z, f"{tag}/init")
    x, t = torch.from_numpy(z[f"{tag}/x"]), torch.from_numpy(z[f"{tag}/t"])
    keys = unet_param_keys(sd)
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    work = dict(sd)
    work.update(params)
    y = unet_forward(work, x, 5, 3)
    loss = unet_loss(y, t, 3)
    loss.backward()
    assert max_abs(y, torch.from_numpy(z[f"{tag}/y"])) <= 1e-5
    assert torch.equal(torch.argmax(torch.softmax(y.detach(), 1), 1), torch.from_numpy(z[f"{tag}/argmax"]))
    assert abs(float(loss) - float(z[f"{tag}/loss"])) <= 1e-5 * abs(float(z[f"{tag}/loss"]))
    err, key = grad_err({k: params[k].grad for k in keys}, _sd(z, f"{tag}/grad"))
    assert err <= 1e-4, (err, key)


def test_oracle_dice_matches_reference_g4():
    from oracle.unet_ref import dice_coeff, trainer_dice
    z = _load("g4_dice.npz")
    for case in ("rand", "empty", "ones", "disjoint"):
        d = dice_coeff(torch.from_numpy(z[f"{case}/pred"]), torch.from_numpy(z[f"{case}/target"]))
        assert float(d) == pytest.approx(float(z[f"{case}/dice"]), abs=1e-7), case
    mc = trainer_dice(torch.from_numpy(z["mc/y"]), torch.from_numpy(z["mc/mask"]), 3)
    assert np.allclose(mc, z["mc/dice"], atol=1e-7)
    b = trainer_dice(torch.from_numpy(z["bin/y"]), torch.from_numpy(z["bin/mask"]), 1)
    assert np.allclose(b, z["bin/dice"], atol=1e-7)


# ----------------------------------------------------------------------------- drop-in surface
def test_unet_state_dict_matches_reference_g1():
    """Same construction order => torch.manual_seed(0) reproduces the reference's weights/keys."""
    from model import UNet
    z = _load("g1_unet_c1.npz")
    ref = _sd(z, "init")
    torch.manual_seed(0)
    sd = UNet(1, 1, [16, 32]).state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k in ref:
        assert torch.equal(sd[k], ref[k]), k


def test_unet_state_dict_matches_reference_g2():
    from model import UNet
    z = _load("g2_unet_multiclass.npz")
    ref = _sd(z, "s64/init")
    torch.manual_seed(0)
    sd = UNet(1, 3, [4, 8, 16, 32, 64]).state_dict()
    assert list(sd.keys()) == list(ref.keys())
    assert all(torch.equal(sd[k], ref[k]) for k in ref)


def test_unet_default_is_c2_architecture():
    from model import UNet
    net = UNet(1, 1)
    assert net.num_filters == [64, 128, 256, 512, 1024]
    assert sum(p.numel() for p in net.parameters()) == 31042369
    assert len(net.state_dict()) == 136


def test_unet_forward_refuses_cpu():
    """No CPU fallback: the product path must fail loudly without the GPU."""
    from model import UNet
    net = UNet(1, 1, [4, 8])
    with pytest.raises(RuntimeError):
        net(torch.rand(1, 1, 8, 8))


def test_bilinear_up_rejected_like_reference():
    from model import UNet
    with pytest.raises(TypeError):
        UNet(1, 1, [4, 8], bilinear=True)


# ----------------------------------------------------------------------------- C ABI
def _header_functions(path=None):
    from pmu_hip._lib import HEADER_PATH
    src = open(path or HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pmu_[A-Za-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    """The shipped library exports exactly include/pmunet_hip.h (every declaration resolves, the ctypes
    table mirrors it, and none of include/pmunet_hip_experiments.h is exported); the experiments library
    exports both headers."""
    from pmu_hip._lib import EXP_HEADER_PATH, EXP_LIB_PATH, EXP_SIGNATURES, LIB_PATH, SIGNATURES, load_library
    if not os.path.exists(LIB_PATH):
        pytest.skip("libpmunet_hip.so not built (run __graft_entry__.build())")
    cdll = load_library()
    names = _header_functions()
    exp_names = _header_functions(EXP_HEADER_PATH)
    assert len(names) >= 25 and len(exp_names) >= 10
    assert not set(names) & set(exp_names)
    for n in names:
        assert hasattr(cdll, n), f"{n} declared in include/pmunet_hip.h but not exported"
    assert set(SIGNATURES) == set(names), "ctypes SIGNATURES out of sync with the header"
    assert set(EXP_SIGNATURES) == set(exp_names), "ctypes EXP_SIGNATURES out of sync with the experiments header"
    shipped_exp = [n for n in exp_names if hasattr(cdll, n)]
    assert not shipped_exp, f"experiments entries exported by the shipped library: {shipped_exp}"
    if os.path.exists(EXP_LIB_PATH):
        exp = load_library(EXP_LIB_PATH)
        for n in names + exp_names:
            assert hasattr(exp, n), f"{n} not exported by the experiments library"


def test_library_rejects_bad_arguments_without_gpu():
    """Host-side validation returns PMU_ERR_ARG before any launch (safe without a GPU)."""
    import ctypes
    from pmu_hip._lib import LIB_PATH, PMU_ERR_ARG, load_library
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    cdll = load_library()
    assert cdll.pmu_conv3x3_fwd_wino(None, None, None, 0, None, None, None, None) == PMU_ERR_ARG
    assert cdll.pmu_conv3x3_fwd_dma(None, 16, 1, 32, 32, None, None, 64, None, None, None) == PMU_ERR_ARG
    assert cdll.pmu_sgd_clip(None, 0, None, ctypes.c_float(1), ctypes.c_float(1), ctypes.c_float(0.9),
                             ctypes.c_float(0.1), None) == PMU_ERR_ARG
    assert cdll.pmu_conv3x3_tiles(32, 256, 256) == 32 * 32 * 8


def test_wgrad_dma_shape_rule_without_gpu():
    """The bf16 weight gradient's buffer descriptors need each operand below 2^31 bytes (their
    out-of-range marker is voffset 0x80000000) and 16-wide maps: pmu_conv3x3_wgrad_dma_ok, a host
    function, admits c5's largest shapes and refuses what would overflow (the engine then takes the
    register-staged kernel)."""
    from pmu_hip._lib import LIB_PATH, load_library
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    cdll = load_library()
    ok = cdll.pmu_conv3x3_wgrad_dma_ok
    assert ok(16, 512, 512, 128, 64) and ok(16, 512, 512, 64, 64)       # c5's 512^2 layers: 1.07 GB operands
    assert not ok(32, 512, 512, 128, 64)                                  # x at 2.1 GB
    assert not ok(64, 512, 512, 64, 128)                                  # dz at 4.3 GB
    assert not ok(2, 64, 15, 64, 64)                                      # narrower than a strip


def test_bench_roofline_peak_by_kernel_family():
    """bench.py prices the dominant kernel against the MFMA peak of the dtype it computes in."""
    import bench
    for k in ("pmu_conv3x3_wgrad_bf16", "pmu_conv3x3_fwd_raw", "pmu_conv3x3_dgrad_raw", "pmu_convT2x2_fwd_bf16"):
        assert bench.roofline_peak(k) == bench.BF16_MFMA_PEAK_TF, k
    for k in ("pmu_conv3x3_fwd_wino_raw", "pmu_conv3x3_dgrad_wino_raw", "pmu_conv3x3_wgrad_wino",
              "pmu_convT2x2_wgrad", "pmu_fcomb_bwd"):
        assert bench.roofline_peak(k) == bench.FP32_MFMA_PEAK_TF, k


def _fake_args(name):
    """Arguments of the ctypes signature of ``name`` as bench.KernelTimer sees them: every int 64, every
    frame a 2-image 64x64 frame of one 64-channel source, pointers None."""
    import ctypes
    from pmu_hip import _lib
    res, types = {**_lib.SIGNATURES, **_lib.EXP_SIGNATURES}[name]
    args = []
    for t in types:
        if t is ctypes.c_int or t is ctypes.c_longlong or t is ctypes.c_size_t:
            args.append(64)
        elif t is _lib._FP:
            f = _lib.PmuFrame()
            f.nsrc, f.N, f.H, f.W = 1, 2, 64, 64
            f.src[0].C, f.src[0].H, f.src[0].W = 64, 64, 64
            args.append(ctypes.byref(f))
        else:
            args.append(None)
    return args


def test_bench_counts_every_mfma_entry_point():
    """Every C-ABI entry whose kernels issue MFMAs (pmu_hip._lib.MFMA_ENTRY_POINTS, next to the ctypes
    table) is declared in the table, counted by bench.KernelTimer and has a non-zero FLOP formula — no
    MFMA kernel prints "tflops": null and step_mfma_busy_frac sees all of them."""
    import bench
    from pmu_hip import _lib
    assert bench.KernelTimer.MFMA is _lib.MFMA_ENTRY_POINTS
    for name in _lib.MFMA_ENTRY_POINTS:
        assert name in _lib.SIGNATURES or name in _lib.EXP_SIGNATURES, name
        fl = bench.KernelTimer._flops(name, _fake_args(name))
        assert fl > 0, name
        # the direct-sum basis of a Winograd launch is larger than its executed products, never zero
        assert bench.KernelTimer._direct(name, _fake_args(name), fl) >= fl, name
    # the fused variants count as their base call (same shapes, same MFMA work)
    for v, base in (("pmu_conv3x3_dgrad_dma_x1b_sum", "pmu_conv3x3_dgrad_dma"),
                    ("pmu_conv3x3_dgrad_dma_x1b", "pmu_conv3x3_dgrad_dma"),
                    ("pmu_convT2x2_fwd_dma_ldb", "pmu_convT2x2_fwd_dma"), ("pmu_convT2x2_fwd_ld", "pmu_convT2x2_fwd")):
        assert bench.KernelTimer._flops(v, _fake_args(v)) == bench.KernelTimer._flops(base, _fake_args(base)), v
    # and each has a kernel family for the PMC traffic lookup
    for name in _lib.MFMA_ENTRY_POINTS:
        assert name in bench.KERNEL_FAMILY, name


def test_debug_build_exports_and_identifies_itself():
    """The bounds-checked debug library (csrc `make DEBUG=1`, selected by PMU_LIB=debug) exports the
    same C ABI and reports its build flags; the shipped library is neither a debug nor an experiments
    build (kernel-variant A/B switches ignored)."""
    import ctypes
    from pmu_hip import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    rel = _lib.load_library(os.path.join(os.path.dirname(_lib.LIB_PATH), "libpmunet_hip.so"))
    assert rel.pmu_build_flags() == 0
    out = (ctypes.c_int * 5)(*([7] * 5))
    assert rel.pmu_debug_read(out, None) == 0 and list(out) == [0] * 5
    dbg_path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libpmunet_hip_debug.so")
    if not os.path.exists(dbg_path):
        pytest.skip("debug library not built (make -C csrc DEBUG=1)")
    dbg = _lib.load_library(dbg_path)   # every SIGNATURES export must resolve
    assert dbg.pmu_build_flags() == _lib.BUILD_DEBUG


def test_bench_gpus_launch_plan():
    """bench.py --gpus N: outside torchrun N > 1 becomes a torch.distributed.run child
    with N ranks on this node and the same argv; under torchrun --gpus must equal WORLD_SIZE."""
    import bench
    assert bench.launch_plan(1, [], {}) is None
    cmd = bench.launch_plan(4, ["--gpus", "4", "--steps", "3"], {})
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert bench.launch_plan(2, [], {"WORLD_SIZE": "2"}) is None
    assert bench.launch_plan(1, [], {"WORLD_SIZE": "1"}) is None
    for gpus, world in ((1, "8"), (8, "1"), (2, "4")):
        with pytest.raises(ValueError):
            bench.launch_plan(gpus, [], {"WORLD_SIZE": world})
    with pytest.raises(ValueError):
        bench.launch_plan(0, [], {})


def test_bench_refuses_gpus_world_mismatch():
    """The mismatch check runs before anything touches torch.cuda: rc 2 and a message, no JSON line."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=2" in r.stderr and r.stdout.strip() == ""


def test_bench_roofline_by_kernel_family():
    """bench.py groups the MFMA entries into kernel families before picking the dominant one (VERDICT r5
    #3): c5's input gradient runs as three entries (_bnr_dxb, _x1b_sum_dxb, _dxb) whose summed time beats
    the forward's, so the line names the input gradient, with the forward as the runner-up."""
    import bench
    per = {  # name: [launches, executed FLOPs, seconds, direct-sum FLOPs] (c5-like proportions)
        "pmu_conv3x3_dgrad_dma_bnr_dxb": [9, 2.7e12, 3.4e-3, 2.7e12],
        "pmu_conv3x3_dgrad_dma_x1b_sum_dxb": [4, 1.6e12, 2.1e-3, 1.6e12],
        "pmu_conv3x3_dgrad_dma_dxb": [3, 0.8e12, 1.0e-3, 0.8e12],
        "pmu_conv3x3_fwd_dma": [17, 5.9e12, 5.4e-3, 5.9e12],
        "pmu_conv3x3_wgrad_bf16_dma": [17, 5.5e12, 4.7e-3, 5.5e12],
        "pmu_frame_to_bf16": [30, 0.0, 2.8e-3, 0.0],   # not an MFMA entry: never a family
    }
    fams = bench.mfma_families(per)
    assert [f[0] for f in fams] == ["pmu_conv3x3_dgrad_dma", "pmu_conv3x3_fwd_dma", "pmu_conv3x3_wgrad_bf16_dma"]
    fam, d, members = fams[0]
    assert members == sorted(["pmu_conv3x3_dgrad_dma_bnr_dxb", "pmu_conv3x3_dgrad_dma_x1b_sum_dxb",
                              "pmu_conv3x3_dgrad_dma_dxb"])
    assert d[0] == 16 and abs(d[2] - 6.5e-3) < 1e-12
    roof = bench.roofline_entry("c5", *fams[0])
    assert roof["kernel"] == "pmu_conv3x3_dgrad_dma" and roof["launches"] == 16
    assert roof["peak"] == bench.BF16_MFMA_PEAK_TF
    assert abs(roof["frac"] - 5.1e12 / 6.5e-3 / 1e12 / bench.BF16_MFMA_PEAK_TF) < 1e-4
    # a Winograd family carries its direct-sum figure beside the executed-product utilisation
    w = bench.roofline_entry("unet", "pmu_conv3x3_dgrad_wino4", [15, 1.0e12, 9.8e-3, 2.25e12],
                             ["pmu_conv3x3_dgrad_wino4", "pmu_conv3x3_dgrad_wino4_bnr"])
    assert w["peak"] == bench.FP32_MFMA_PEAK_TF and w["direct_sum_equiv_frac"] > w["frac"]


def test_bench_refuses_bad_rank_layouts():
    """Under RCCL every rank needs its own GPU: world > visible devices, or two ranks reporting the same
    PCI identity, is refused (exit 2); gloo may rehearse N ranks on one device."""
    import bench
    assert bench.check_layout("nccl", 8, 8) is None
    assert bench.check_layout(None, 1, 1) is None and bench.check_layout(None, 1, 0) is None
    assert bench.check_layout("gloo", 2, 1) is None
    assert "2 RCCL ranks but 1" in bench.check_layout("nccl", 2, 1)
    assert bench.check_layout("nccl", 4, 0)
    assert bench.check_devices("nccl", ["0000:05:00.0 a", "0000:15:00.0 b"]) is None
    assert bench.check_devices("gloo", ["0000:05:00.0 a", "0000:05:00.0 a"]) is None
    assert "share a GPU" in bench.check_devices("nccl", ["0000:05:00.0 a", "0000:05:00.0 a"])


def test_bench_refuses_rccl_ranks_beyond_devices():
    """End to end: a rank of a 2-rank RCCL run on a host with fewer GPUs exits 2 with the reason before
    any process group is formed (here: no GPU at all), and prints no JSON line."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29599", PMU_DIST_BACKEND="nccl")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "RCCL ranks but" in r.stderr and r.stdout.strip() == ""


def test_oracle_bf16_dx_rule_matches_engine(monkeypatch):
    """oracle/unet_ref.py models the HIP path's bf16 activation gradients (BF16_DX) by the same rule the
    engine uses to pick the *_dxb input gradients (engine.dxb_ok, through the library's
    pmu_conv3x3_dma_ok; the transposed conv: pmu_convT2x2_dma_ok) — checked here over a grid of shapes so
    the parity tests compare like with like."""
    import oracle.unet_ref as ur
    from pmu_hip import _lib as L
    from pmu_hip.engine import dxb_ok
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("library not built")
    lb = L.load_library()   # host-side shape predicates only (no GPU call)
    monkeypatch.setattr(L, "_LIB", lb)
    assert ur.BF16_DX
    x = torch.empty(1, 1, 1, 1)
    for W in (16, 31, 32, 45, 64):
        xx = x.expand(1, 1, 1, W)
        for cin in (3, 8, 12, 32, 40, 64, 96, 128, 1024):
            for cout in (8, 12, 16, 20, 32, 64, 1024):
                for split in (None, 8, 16, 32, 64):
                    if split is not None and split >= cin:
                        continue
                    want = dxb_ok(7, W, cout, cin, cin if split is None else split)
                    assert ur._dma_dxb(xx, cin, cout, split) == want, (W, cin, cout, split)
    for cin in (32, 64, 96, 128, 256, 1024):
        for cout in (16, 32, 64, 512):
            assert bool(lb.pmu_convT2x2_dma_ok(cin, cout, 1)) == (cin % 128 == 0 and cout % 32 == 0), (cin, cout)
