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
@pytest.mark.parametrize("decomp", ["default", "rows", "rows-dst"])
def test_bench_two_ranks_one_gpu(gpu, decomp):
    extra = {"default": [], "rows": ["--decomp", "rows"],
             "rows-dst": ["--decomp", "rows", "--rows-gather", "dst", "--steps", "2"]}[decomp]
    d = _run(extra)
    assert d["n_gpus"] == 2 and d["output_ok"] is True
    assert d["config"]["backend"].startswith("gloo")
    # north_star / BASELINE configs[3]: Z-slabs + one grid collective are the N > 1 default
    want = "zslab" if decomp == "default" else "rows"
    assert d["config"]["decomp"] == want
    assert d["config"]["parallelism"] == ("zslab2" if want == "zslab" else "rows2")
    assert 0.0 < d["roofline"]["frac"] <= 1.0
    assert d["value"] > 0 and d["ms_per_step"] > 0
    if want == "zslab":
        assert "Z-slab x2" in d["config"]["workload"] and d["config"]["collective"] == "reduce"
        assert "partition_ms" not in d
    else:
        R = d["config"]["row_bounds"]
        assert R[0] == 0 and R[-1] == 1024 and all(a < b for a, b in zip(R, R[1:]))
        assert "image row slabs x2" in d["config"]["workload"]
        assert d["partition_ms"] > 0  # the timed all-to-all from the reader's split
        assert d["config"]["collective"] == ("p2p_gather" if decomp == "rows-dst" else "all_gather")
