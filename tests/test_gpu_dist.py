"""Multi-rank bench path on one GPU: two ranks (gloo backend, both on cuda:0)
run the row-block partition, the per-rank HIP pipeline and the gather of C
row blocks to rank 0; the gathered C must equal the single-rank C.  (The nccl
= RCCL variant differs only in the backend; one GPU cannot host two RCCL ranks.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(nproc, mtx, aat, scaling="strong"):
    args = ["bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--check", "--mtx", mtx,
            "--aat", str(aat), "--gpus", str(nproc), "--scaling", scaling]
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + ["--backend", "gloo"]
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("name,aat", [("x_powerlaw_400", 0), ("x_rect_50x130", 1)])
def test_two_ranks_gather_equals_single_rank(name, aat):
    mtx = os.path.join(REPO, "tests", "golden", "fixtures", name + ".mtx")
    one = _bench(1, mtx, aat)
    two = _bench(2, mtx, aat)
    assert two["n_gpus"] == 2 and two["config"]["parallelism"].startswith("row-block2")
    assert two["scaling"] == "strong"
    assert two["check"] == one["check"]
    assert two["config"]["nnzC"] == one["config"]["nnzC"]


@pytest.mark.parametrize("name,aat", [("x_powerlaw_400", 1)])
def test_two_ranks_weak_stacked_product(name, aat):
    """Weak scaling (the bench default): each rank owns one A-sized row block of
    [A; A] * B, no collective on the data path; every block equals the 1-rank C
    (bench asserts this across ranks) and the job counts twice the work."""
    mtx = os.path.join(REPO, "tests", "golden", "fixtures", name + ".mtx")
    one = _bench(1, mtx, aat, "weak")
    two = _bench(2, mtx, aat, "weak")
    assert two["scaling"] == "weak" and two["config"]["parallelism"].startswith("stacked-row-block2")
    assert two["check"] == one["check"]
    assert two["config"]["nnzC"] == 2 * one["config"]["nnzC"]
    assert two["config"]["nnzCub"] == 2 * one["config"]["nnzCub"]
    assert two["gather_ms"] is None
