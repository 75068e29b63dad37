"""Multi-rank path on CPU (gloo, world_size 2 and 3): work partition of A's tile
rows, row slicing, per-rank block products and the gather of C row blocks to
rank 0 (spgemm_amd/dist.py).  On the GPU the per-rank block
product is the HIP pipeline and the backend is nccl (= RCCL); here each rank's
block is computed by the oracle so the partition/gather logic is checked
against the oracle's full product without a GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle as O
from spgemm_amd import dist as tdist
from spgemm_amd import synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _matrix(kind):
    if kind == "powerlaw":
        return synth.random_csr(700, 700, density=0.004, seed=5)
    if kind == "aat":
        return synth.random_csr(300, 520, density=0.01, seed=9)
    return synth.random_csr(2, 2, density=0.0, seed=1)  # all-empty


def _worker(rank, world, port, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, n, rp, ci, vv = _matrix(kind)
        if kind == "aat":
            oB = O.transpose(O.OMat.from_csr(m, n, rp, ci, vv))
        else:
            oB = O.OMat.from_csr(m, n, rp, ci, vv)
        mb, nb, rpb, cib, vvb = oB.csr()
        work = tdist.tile_row_work(rp, ci, rpb, m, 16)
        parts = tdist.partition_tile_rows(work, world)
        t0, t1 = parts[rank]
        mblk, rpk, cik, vvk = tdist.slice_rows(m, rp, ci, vv, t0 * 16, t1 * 16)
        Ck = O.gustavson(O.OMat.from_csr(mblk, n, rpk, cik, vvk), oB)
        _, _, crp, cci, cvv = Ck.csr()
        out = tdist.gather_csr_blocks(torch.from_numpy(crp.copy()), torch.from_numpy(cci.copy()),
                                      torch.from_numpy(cvv.copy()), rank, world)
        if rank == 0:
            q.put(("ok", parts, [x.numpy() for x in out]))
        else:
            assert out is None
    except Exception as e:  # surface worker failures to the parent
        q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["powerlaw", "aat", "empty"])
def test_row_block_partition_and_gather_matches_full_product(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, parts, got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert status == "ok", parts
    m, n, rp, ci, vv = _matrix(kind)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    oB = O.transpose(oA) if kind == "aat" else O.OMat.alias(oA)
    _, _, erp, eci, evv = O.gustavson(oA, oB).csr()
    # the ranges tile [0, tilem) contiguously
    tilem = (m + 15) // 16
    assert parts[0][0] == 0 and parts[-1][1] == tilem
    assert all(parts[r][1] == parts[r + 1][0] for r in range(world - 1))
    np.testing.assert_array_equal(got[0], erp)
    np.testing.assert_array_equal(got[1], eci)
    np.testing.assert_array_equal(got[2], evv)


def test_partition_balances_work():
    work = np.array([100, 1, 1, 1, 1, 100, 1, 1, 1, 1] * 10, dtype=np.int64)
    parts = tdist.partition_tile_rows(work, 4)
    loads = [work[a:b].sum() for a, b in parts]
    assert max(loads) <= 1.3 * (work.sum() / 4)
    # more ranks than tile rows: trailing ranks get empty ranges, still contiguous
    parts = tdist.partition_tile_rows(np.array([5, 5]), 4)
    assert parts[0][0] == 0 and parts[-1][1] == 2
    assert all(a <= b for a, b in parts)


def test_tile_row_work_is_nnzcub_per_tile_row():
    m, n, rp, ci, vv = synth.random_csr(100, 100, density=0.05, seed=2)
    w = tdist.tile_row_work(rp, ci, rp, m, 16)
    blen = np.diff(rp)
    ref = [sum(int(blen[ci[p]]) for p in range(rp[r0], rp[min(r0 + 16, m)])) for r0 in range(0, m, 16)]
    np.testing.assert_array_equal(w, ref)


@pytest.mark.parametrize("cap", [1, 50, 1000, 10 ** 9])
def test_product_blocks_cover_rows_within_cap(cap):
    """Sequential row blocks (products past int32 nnz(C)): contiguous,
    tile-row aligned, each within `cap` products unless one tile row alone
    exceeds it."""
    m, n, rp, ci, vv = synth.random_csr(1000, 1000, density=0.01, seed=3)
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    for r_lo, r_hi in [(0, m), (160, 800)]:
        b = tdist.product_blocks(cum, r_lo, r_hi, cap, 16)
        assert b[0][0] == r_lo and b[-1][1] == r_hi
        assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
        for b0, b1 in b:
            assert b1 > b0 and (b0 % 16 == 0)
            work = cum[b1] - cum[b0]
            assert work <= cap or b1 - b0 <= 16


def _worker_rounds(rank, world, port, kind, nsub, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, n, rp, ci, vv = _matrix(kind)
        oB = O.transpose(O.OMat.from_csr(m, n, rp, ci, vv)) if kind == "aat" else O.OMat.from_csr(m, n, rp, ci, vv)
        mb, nb, rpb, cib, vvb = oB.csr()
        blen = np.diff(rpb.astype(np.int64))
        cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
        pieces = tdist.row_pieces(cum, m, world, nsub)
        meta = dist.new_group(backend="gloo")  # the counts' host group (bench.py: beside RCCL)
        # capacity 1: rank 0's arrays grow from the gathered counts (round by round)
        g = tdist.RoundGather(rank, world, pieces, 1, meta_group=meta)
        caps = []
        for step in range(2):  # the second step reuses the arrays sized by the first
            g.reset()
            for s in range(nsub):  # each round's piece "computed" (oracle) then pushed
                b0, b1 = pieces[s][rank]
                mk, rpk, cik, vvk = tdist.slice_rows(m, rp, ci, vv, b0, b1)
                _, _, crp, cci, cvv = O.gustavson(O.OMat.from_csr(mk, n, rpk, cik, vvk), oB).csr()
                # padded arrays + the host count: only the first nnz entries travel
                pc = np.concatenate([cci.astype(np.int32), np.full(3, -7, np.int32)])
                pv = np.concatenate([cvv, np.full(3, np.nan)])
                g.push(s, torch.from_numpy(crp.astype(np.int32)), torch.from_numpy(pc), torch.from_numpy(pv),
                       nnz=len(cci))
            out = g.finish()
            caps.append(g.cap)
        if rank == 0:
            # sized by the gathered nnz (not the products bound), allocated once
            assert caps[0] == caps[1] == max(1, len(out[1])), (caps, len(out[1]))
            q.put(("ok", pieces, [x.numpy().copy() for x in out]))
        else:
            assert out is None
    except Exception as e:  # surface worker failures to the parent
        q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def _run(world, target, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,nsub", [(2, 3), (3, 4), (2, 1), (8, 2)])
@pytest.mark.parametrize("kind", ["powerlaw", "aat", "empty"])
def test_round_gather_of_row_pieces_matches_full_product(world, nsub, kind):
    """The overlapped gather (dist.RoundGather): rows cut into world x nsub
    pieces of equal products at row granularity, rank r computing piece (s, r)
    in round s; rank 0 receives every round straight into the final C at its
    exact offsets (no concatenation), the counts exchanged on a host group with
    no device read-back, its arrays sized by the gathered nnz and reused by the
    next step.  The gathered row pointers, columns and values equal the full
    product array by array, and the pieces tile the rows in round-major order."""
    status, pieces, got = _run(world, _worker_rounds, (kind, nsub))
    assert status == "ok", pieces
    m, n, rp, ci, vv = _matrix(kind)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    oB = O.transpose(oA) if kind == "aat" else O.OMat.alias(oA)
    _, _, erp, eci, evv = O.gustavson(oA, oB).csr()
    flat = [b for rnd in pieces for b in rnd]
    assert flat[0][0] == 0 and flat[-1][1] == m and all(flat[i][1] == flat[i + 1][0] for i in range(len(flat) - 1))
    assert len(pieces) == nsub and all(len(rnd) == world for rnd in pieces)
    np.testing.assert_array_equal(got[0], erp)
    np.testing.assert_array_equal(got[1], eci)
    np.testing.assert_array_equal(got[2], evv)


def test_row_pieces_balance_and_split_hub_tile_rows():
    """Pieces of ~equal products; a heavy tile row's rows go to different ranks
    (row granularity), so no rank carries a hub tile row whole."""
    rng = np.random.default_rng(4)
    m = 4000
    per_row = rng.integers(0, 20, size=m).astype(np.int64)
    per_row[1600:1616] = 20000  # one hub tile row: 16 rows of 20 K products
    cum = np.concatenate([[0], np.cumsum(per_row)])
    for world, nsub in [(2, 1), (8, 1), (8, 4)]:
        pieces = tdist.row_pieces(cum, m, world, nsub)
        loads = [sum(cum[b] - cum[a] for a, b in [pieces[s][r] for s in range(nsub)]) for r in range(world)]
        assert max(loads) <= 1.15 * cum[-1] / world + 20000, (world, nsub, loads)
        owners = {r for s in range(nsub) for r in range(world) if pieces[s][r][0] < 1616 and pieces[s][r][1] > 1600}
        assert len(owners) > 1 or world == 1
