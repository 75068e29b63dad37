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


def _bench(nproc, mtx, aat, scaling=None, extra=()):
    args = ["bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--check", "--tiled", "0",
            "--gpus", str(nproc)]
    if mtx:
        args += ["--mtx", mtx, "--aat", str(aat)]
    if scaling:  # default invocation (no flag) = strong: north_star's partition + gather of C
        args += ["--scaling", scaling]
    args += list(extra)
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + ["--backend", "gloo"]
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("name,aat", [("x_powerlaw_400", 0), ("x_rect_50x130", 1)])
def test_two_ranks_gather_equals_single_rank(name, aat):
    """The DEFAULT multi-rank invocation (no --scaling flag) is north_star's
    exchange step: strong scaling, the fixed product, work-balanced row pieces,
    B replicated, the gather of C to rank 0 inside the timed region with its
    exposed time reported as gather_ms."""
    mtx = os.path.join(REPO, "tests", "golden", "fixtures", name + ".mtx")
    one = _bench(1, mtx, aat)
    assert one["scaling"] == "single" and one["config"]["parallelism"] == "single"
    two = _bench(2, mtx, aat)
    assert two["n_gpus"] == 2 and two["config"]["parallelism"].startswith("row-pieces2")
    assert two["scaling"] == "strong"
    assert two["gather_ms"] is not None and two["gather_ms"] >= 0.0
    assert two["check"] == one["check"]
    assert two["config"]["nnzC"] == one["config"]["nnzC"]
    assert two["work_share"]["max_over_mean"] >= 1.0
    # the line reads itself against the link bound: per-rank compute,
    # the largest peer's bytes over one xGMI link, the single-GPU time of the
    # same product and the ceiling they give
    sm = two["scale_model"]
    assert len(sm["compute_ms"]) == 2 and all(x > 0 for x in sm["compute_ms"])
    assert sm["gather_floor_ms"] > 0 and sm["max_peer_bytes"] > 0
    assert sm["rank0_received_bytes"] == sm["max_peer_bytes"]
    assert sum(sm["nnzC"]) == one["config"]["nnzC"]
    assert sm["t1_ms"] > 0 and sm["ceiling_speedup"] > 0 and sm["measured_speedup"] > 0
    assert one["scale_model"] is None


@pytest.mark.parametrize("name,aat", [("x_powerlaw_400", 1)])
def test_two_ranks_weak_stacked_product(name, aat):
    """Weak scaling (--scaling weak, NOT the north-star metric): each rank owns
    one A-sized row block of [A; A] * B, no collective on the data path; every
    block equals the 1-rank C (bench asserts this across ranks) and the job
    counts twice the work."""
    mtx = os.path.join(REPO, "tests", "golden", "fixtures", name + ".mtx")
    one = _bench(1, mtx, aat)
    two = _bench(2, mtx, aat, "weak")
    assert two["scaling"] == "weak" and two["config"]["parallelism"].startswith("stacked-row-block2")
    assert two["check"] == one["check"]
    assert two["config"]["nnzC"] == 2 * one["config"]["nnzC"]
    assert two["config"]["nnzCub"] == 2 * one["config"]["nnzCub"]
    assert two["gather_ms"] is None


def _mawi_rows(scale, products):
    from spgemm_amd import synth
    import numpy as np
    m, n, rp, ci, vv = synth.mawi(scale=scale)
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    rows = int(np.searchsorted(cum, products, side="right") - 1) // 16 * 16
    return (m, n, rp, ci, vv), rows


def test_mawi_eight_ranks_gather_vs_oracle(tmp_path):
    """BASELINE config 5 rehearsed on one GPU: the mawi stand-in at 1e-2 scale
    (2.26 M nodes, hub degree 1e5), a row prefix of ~2e8 intermediate products
    (the full A^2 is ~1e10 products, past int32 nnz(C)), partitioned 8 ways by
    work, each rank's block through the HIP pipeline, the C blocks gathered to
    rank 0 (gloo here; RCCL on an 8-GPU node).  The gathered C -- row pointers,
    columns and values, array by array (bench.py --dump) -- must equal the
    oracle's product of the same rows, and the line reports each rank's share
    of the work."""
    import numpy as np
    import _oracle as O
    (m, n, rp, ci, vv), rows = _mawi_rows(0.01, 2e8)
    dump = str(tmp_path / "c8.npz")
    eight = _bench(8, None, 0, "strong", extra=("--matrix", "mawi", "--scale", "0.01", "--rows", str(rows), "--dump", dump,
                                      "--gather-sub", "3"))
    assert eight["n_gpus"] == 8 and eight["scaling"] == "strong"
    assert eight["config"]["gather_rounds"] == 3  # the overlapped gather: rounds received in place on rank 0
    assert eight["config"]["parallelism"] == "row-pieces8x3 + RCCL gather"
    ws = eight["work_share"]
    assert len(ws["products"]) == 8 and sum(ws["products"]) == eight["config"]["nnzCub"]
    assert ws["max_over_mean"] >= 1.0
    oA = O.OMat.from_csr(rows, n, rp[:rows + 1].copy(), ci[:rp[rows]].copy(), vv[:rp[rows]].copy())
    oB = O.OMat.from_csr(m, n, rp, ci, vv)
    _, _, erp, eci, evv = O.gustavson(oA, oB).csr()
    got = np.load(dump)
    np.testing.assert_array_equal(got["rowptr"], erp)
    np.testing.assert_array_equal(got["col"], eci)
    np.testing.assert_allclose(got["val"], evv, rtol=1e-10, atol=0)
    want = {"nnz": int(len(eci)), "rowptr_sum": int(erp.astype(np.int64).sum()),
            "col_sum": int(eci.astype(np.int64).sum()), "val_sum": float(evv.sum())}
    assert eight["check"] == want
    assert eight["config"]["nnzC"] == want["nnz"]


def test_blocked_rows_equal_single_block():
    """Sequential row blocks (the mode for products past int32 nnz(C), e.g. the
    full LiveJournal stand-in): forcing tiny blocks gives the same C checksum
    as one block, and the job still counts the whole product."""
    mtx = os.path.join(REPO, "tests", "golden", "fixtures", "x_powerlaw_400.mtx")
    one = _bench(1, mtx, 0)
    blk = _bench(1, mtx, 0, extra=("--block-products", "300"))
    assert blk["config"]["row_blocks"] > 3
    assert blk["check"] == one["check"]
    assert blk["config"]["nnzCub"] == one["config"]["nnzCub"]
    two = _bench(2, mtx, 0, "strong", extra=("--block-products", "300"))
    assert "sequential blocks" in two["config"]["parallelism"]
    assert two["check"] == one["check"]


@pytest.mark.parametrize("nsub", [1, 3])
def test_two_ranks_streaming_gather_arrays(tmp_path, nsub):
    """The overlapped gather (--gather-sub, dist.RoundGather): rows in 2 x nsub
    pieces, each round received straight into rank 0's final C while the next
    one computes; the gathered C equals the single-rank C array by array
    (--dump)."""
    import numpy as np
    mtx = os.path.join(REPO, "tests", "golden", "fixtures", "x_powerlaw_400.mtx")
    d1, d2 = str(tmp_path / "one.npz"), str(tmp_path / "two.npz")
    one = _bench(1, mtx, 0, extra=("--dump", d1))
    two = _bench(2, mtx, 0, "strong", extra=("--dump", d2, "--gather-sub", str(nsub)))
    assert two["config"]["gather_rounds"] == nsub and two["gather_ms"] is not None
    a, b = np.load(d1), np.load(d2)
    for k in ("rowptr", "col", "val"):
        np.testing.assert_array_equal(a[k], b[k])
    assert two["check"] == one["check"]
