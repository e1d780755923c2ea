"""The N > 1 bench path end to end (the driver's 8-GPU scaling run uses it): bench.py under
torch.distributed.run with two ranks sharing ONE GPU over gloo (RCCL cannot put two ranks
on one device), both decompositions.  Checks the JSON line's contract: n_gpus, the real
backend label, the output check, a roofline fraction <= 1 from the timed steps, and the
row bounds covering the image."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(extra):
    env = dict(os.environ, ASP_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--particles", "2000000", "--grid", "1024", "--steps", "3", "--warmup", "1",
           "--cpu-baseline", "off", "--quiet"] + extra
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints ONE line
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("decomp", ["rows", "zslab"])
def test_bench_two_ranks_one_gpu(gpu, decomp):
    d = _run(["--decomp", decomp])
    assert d["n_gpus"] == 2 and d["output_ok"] is True
    assert d["config"]["backend"].startswith("gloo")
    assert d["config"]["decomp"] == decomp
    assert 0.0 < d["roofline"]["frac"] <= 1.0
    assert d["value"] > 0 and d["ms_per_step"] > 0
    if decomp == "rows":
        R = d["config"]["row_bounds"]
        assert R[0] == 0 and R[-1] == 1024 and all(a < b for a, b in zip(R, R[1:]))
