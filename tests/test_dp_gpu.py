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
    assert r.returncode == 0 and "DP_CHECK OK" in out, out[-4000:]
