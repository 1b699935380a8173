"""Row e on the GPU: the backward-overlapped bucket all-reduce (pmu_hip.dp) around the real HIP
backward, rehearsed with 2 ranks sharing cuda:0 over gloo (tools/dp_check.py; RCCL needs one
device per rank, the driver's multi-GPU bench runs it over RCCL).  Launched as a child process."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_bucketed_allreduce_overlapped_with_hip_backward():
    env = dict(os.environ, PMU_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "dp_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "DP_CHECK gloo world 2 OK" in out, out[-4000:]


@pytest.mark.gpu
def test_bucketed_allreduce_over_rccl_one_rank():
    """The same check over RCCL (backend nccl) with the one rank this box's single GPU allows: the RCCL
    communicator, the bucket all-reduces issued from inside the HIP backward on RCCL's stream behind the
    compute stream's events, and the learned bucket layout; the synchronised gradient equals the local one
    bit for bit."""
    env = dict(os.environ, PMU_DIST_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "dp_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "DP_CHECK nccl world 1 OK" in out, out[-4000:]


@pytest.mark.gpu
def test_bench_gpus_2_launches_two_ranks():
    """bench.py --gpus 2 outside torchrun starts 2 ranks itself and the line reports the
    whole job: n_gpus 2, global batch 64, dp2.  Rehearsed on the 1-GPU box over gloo (both ranks on
    cuda:0); the driver's N-GPU node runs the same path over RCCL."""
    import json
    env = dict(os.environ, PMU_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-kernel-timing"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 64 and res["config"]["parallelism"] == "dp2"
    assert res["value"] > 0 and res["steps"] == 2
    # the line records its topology: gloo, 2 ranks, each rank's GPU identity (both cuda:0 on this box)
    d = res["dist"]
    assert d["backend"] == "gloo" and d["world"] == 2 and len(d["devices"]) == 2, d


@pytest.mark.gpu
def test_bench_refuses_two_rccl_ranks_on_one_gpu():
    """The same launch over RCCL on a box with one GPU: each rank exits 2 before forming a process group
    (two RCCL ranks on one device would time one GPU as two), and no JSON line is printed."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    env = dict(os.environ, PMU_DIST_BACKEND="nccl")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--no-kernel-timing"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, (r.stdout + r.stderr)[-4000:]
    assert "RCCL ranks but 1 visible GPU" in r.stderr, r.stderr[-4000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
