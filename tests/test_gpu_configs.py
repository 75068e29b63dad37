"""BASELINE configs that the full-size tests cannot hold in one int32 C.

com-LiveJournal (config 4): the R-MAT stand-in's A^2 has 1.3e11 intermediate
products -- past the reference's `int nnzC` (src/tilespgemm-cuda.h:2327) -- so
the product runs as sequential tile-row blocks (spgemm_amd.dist.product_blocks,
what `bench.py --matrix lj` times).  Here: the block with the most work (the
hub rows, the load-imbalanced case) and strided blocks, each C against the
numeric Gustavson oracle at 1e8-product blocks (host-checkable sizes).
(Here: the heaviest block and twenty strided ones.)  And the whole product,
every one of the 90 row blocks bench.py times, through size-independent
properties: C x = A_b (B x) for random x, rows strictly column-sorted.

mawi_201512020330 (config 5) at FULL scale (226 M rows, hub degree 10^7): the
row prefix of ~2e8 products that `bench.py --matrix mawi` times a larger
version of, through the default route (its hub-neighbour rows take the
dominant-run kernels), against scipy's SpGEMM of the same rows (the oracle's
dense row accumulator would need 226 M doubles per thread); and the benched
prefix itself (1.49e9 nonzeros of C) whole, through the oracle's SPA pattern
and per-row value sums by linearity, plus every value of every 48th row
against scipy.
"""
import numpy as np
import pytest

import _oracle as O
from spgemm_amd import dist as tdist
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lj():
    m, n, rp, ci, vv = synth.rmat()
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    return m, n, rp, ci, vv, cum


def test_lj_heaviest_and_strided_row_blocks_vs_oracle(lj):
    m, n, rp, ci, vv, cum = lj
    blocks = tdist.product_blocks(cum, 0, m, 1e8, 16)
    assert len(blocks) > 1000  # 1.3e11 products
    work = np.array([cum[b1] - cum[b0] for b0, b1 in blocks], dtype=np.float64)
    rows = np.array([b1 - b0 for b0, b1 in blocks])
    dens = work / rows
    # the heaviest block and twenty strided ones
    pick = [int(np.argmax(dens))] + [k * len(blocks) // 21 for k in range(1, 21)]
    B = T.Matrix.from_csr(m, n, rp, ci, vv)
    oB = O.OMat.from_csr(m, n, rp, ci, vv)
    for k in pick:
        b0, b1 = blocks[k]
        mb, rpb, cib, vvb = tdist.slice_rows(m, rp, ci, vv, b0, b1)
        A = T.Matrix.from_csr(mb, n, rpb, cib, vvb)
        Cm, st = T.spgemm(A, B)
        got = Cm.csr()
        ref = O.gustavson(O.OMat.from_csr(mb, n, rpb, cib, vvb), oB).csr()
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(got[3], ref[3])
        np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=0)
        assert st["nnzCub"] == 0 or st["nnzCub"] == cum[b1] - cum[b0]
        del Cm, A


def _spmv(rowptr, col, val, x):
    """y = M x for a device CSR (torch; a checker, not the product path)"""
    import torch
    return torch.segment_reduce(val * x[col.long()], "sum", offsets=rowptr.long())


def test_lj_every_row_block_by_random_vectors(lj):
    """The WHOLE LiveJournal stand-in (every row block bench.py times, 1.3e11
    products; the oracle cannot hold them): per block, C x = A_b (B x) for two
    random x, and every C row strictly column-sorted within [0, n).  The values
    are positive, so no sum cancels: a missing, extra, doubled or misplaced
    column moves C x far past the tolerance (1e-10 relative, fp64 sums in other
    orders).  (The stand-in's values hold zeros: here every value is replaced
    by a positive one, same structure.)"""
    import torch
    from spgemm_amd.device import Context, DeviceCSR
    m, n, rp, ci, _, cum = lj
    vv = (np.arange(len(ci)) % 7 + 1) / 4.0
    blocks = tdist.product_blocks(cum, 0, m, 1.5e9, 16)  # (bench.py's --block-products)
    assert len(blocks) >= 80
    dB = DeviceCSR.from_host(m, n, rp, ci, vv)
    ctx = Context(0)
    assert ctx.rows_sorted(dB)
    g = torch.Generator(device="cuda").manual_seed(7)
    xs = [torch.rand(n, dtype=torch.float64, device="cuda", generator=g) + 0.5 for _ in range(2)]
    bxs = [_spmv(dB.rowptr, dB.col, dB.val, x) for x in xs]
    total = 0
    for bi, (b0, b1) in enumerate(blocks):
        mb, rpb, cib, vvb = tdist.slice_rows(m, rp, ci, vv, b0, b1)
        dA = DeviceCSR.from_host(mb, n, rpb, cib, vvb)
        ctx.reset()
        c, st = ctx.spgemm(dA, dB, 16, 16, b_sorted=bi > 0)
        assert st["nnzCub"] == 0 or st["nnzCub"] == cum[b1] - cum[b0]
        C = ctx.view_torch(c)
        assert C.m == mb and int(C.rowptr[0]) == 0 and int(C.rowptr[-1]) == c.nnz
        if c.nnz:
            assert int(C.col.min()) >= 0 and int(C.col.max()) < n
            asc = C.col[1:] > C.col[:-1]
            starts = C.rowptr[1:-1].long()
            starts = starts[(starts > 0) & (starts < c.nnz)]
            asc[starts - 1] = True  # (a row's first entry against the previous row's last)
            assert bool(asc.all()), f"block {bi}: a C row not strictly column-sorted"
        for x, bx in zip(xs, bxs):
            got = _spmv(C.rowptr, C.col, C.val, x)
            ref = _spmv(dA.rowptr, dA.col, dA.val, bx)
            err = float(((got - ref).abs() / ref.clamp_min(1e-300)).max()) if mb else 0.0
            assert err <= 1e-10, f"block {bi} rows [{b0}, {b1}): C x off by {err:.3g}"
        total += c.nnz
        del C, dA
    ctx.reset()
    assert total > 6e10  # (nnz(C) of the whole product: 6.5e10)


def test_mawi_full_scale_prefix_vs_scipy():
    """Full-scale mawi stand-in: the longest row prefix within 2e8 products
    (19 hub-neighbour rows of 10^7 products each, the dominant-run kernels'
    rows at their benched size) times the whole matrix, default route.  Values
    pos % 10 + 1 (no zero values: every structural entry is a nonzero sum, so
    scipy -- which drops zero sums -- keeps it; small integers: every sum exact
    whatever its order).  Row pointers, columns and values array for array."""
    import scipy.sparse as sp
    m, n, rp, ci, _ = synth.mawi()
    vv = (np.arange(len(ci)) % 10 + 1).astype(np.float64)
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    r = int(np.searchsorted(cum, 2e8, side="right") - 1)
    P = np.diff(cum[:r + 1])
    assert P.max() >= 10 ** 7 and (P > 65536).sum() >= 10, (r, P.max())
    A = T.Matrix.from_csr(r, n, rp[:r + 1].copy(), ci[:rp[r]].copy(), vv[:rp[r]].copy())
    B = T.Matrix.from_csr(m, n, rp, ci, vv)
    Cm, st = T.spgemm(A, B)
    assert st["path"] == T.PATH_ROWS
    got = Cm.csr()
    del Cm, A, B
    ref = (sp.csr_matrix((vv[:rp[r]], ci[:rp[r]], rp[:r + 1]), shape=(r, n)) @
           sp.csr_matrix((vv, ci, rp), shape=(m, n))).tocsr()
    ref.sort_indices()
    np.testing.assert_array_equal(got[2], ref.indptr)
    np.testing.assert_array_equal(got[3], ref.indices)
    np.testing.assert_array_equal(got[4], ref.data)


def test_mawi_bench_prefix_full_size_properties():
    """The mawi prefix at the size bench.py times (the longest row prefix
    within 1.5e9 products: 3,360 rows, C of 1.49e9 nonzeros, ~150 hub
    neighbours on the grouped dominant-run fill), checked whole through
    properties the oracle can afford: row pointers and every column against
    the oracle's SPA (the reference's CPU symbolic, spgemm_serialref_spa_new.h:
    7-105, restated in oracle/tsg_oracle.c), and each row's value sum against
    linearity -- rowsum(C)_i = sum_k A_ik rowsum(B)_k, exact here (values
    pos % 10 + 1: every sum an integer below 2^53); then every value of every
    48th row element for element against scipy."""
    m, n, rp, ci, _ = synth.mawi()
    vv = (np.arange(len(ci)) % 10 + 1).astype(np.float64)
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    r = int(np.searchsorted(cum, 1.5e9, side="right") - 1)
    assert cum[r] > 10 ** 9
    A = T.Matrix.from_csr(r, n, rp[:r + 1].copy(), ci[:rp[r]].copy(), vv[:rp[r]].copy())
    B = T.Matrix.from_csr(m, n, rp, ci, vv)
    Cm, st = T.spgemm(A, B)
    assert st["path"] == T.PATH_ROWS
    got = Cm.csr()
    del Cm, A, B
    oA = O.OMat.from_csr(r, n, rp[:r + 1].copy(), ci[:rp[r]].copy(), vv[:rp[r]].copy())
    oB = O.OMat.from_csr(m, n, rp, ci, vv)
    srp, sci = O.spa(oA, oB, 0, r)
    np.testing.assert_array_equal(got[2], srp)
    assert len(got[3]) == len(sci) > 10 ** 9
    assert np.array_equal(got[3], sci)
    del sci
    # (prefix sums of integer values: exact in fp64, and empty rows need no care)
    cs = np.concatenate([[0.0], np.cumsum(vv)])
    rowsum_b = cs[rp[1:].astype(np.int64)] - cs[rp[:-1].astype(np.int64)]
    na = int(rp[r])
    cs = np.concatenate([[0.0], np.cumsum(vv[:na] * rowsum_b[ci[:na]])])
    expect = cs[rp[1:r + 1].astype(np.int64)] - cs[rp[:r].astype(np.int64)]
    del cs
    gc = np.concatenate([[0.0], np.cumsum(got[4])])
    grp = got[2].astype(np.int64)
    np.testing.assert_array_equal(gc[grp[1:]] - gc[grp[:-1]], expect)
    del gc
    # and every value of a strided sample of the rows (every 48th: ~70 rows, a
    # few of them hub neighbours on the dominant-run fill) element for element
    # against scipy's SpGEMM of those rows (exact: small integer sums)
    import scipy.sparse as sp
    rows = np.arange(0, r, 48)
    lens = (rp[rows + 1] - rp[rows]).astype(np.int64)
    idx = np.concatenate([np.arange(rp[i], rp[i + 1]) for i in rows])
    As = sp.csr_matrix((vv[idx], ci[idx], np.concatenate([[0], np.cumsum(lens)])), shape=(len(rows), n))
    ref = (As @ sp.csr_matrix((vv, ci, rp), shape=(m, n))).tocsr()
    ref.sort_indices()
    assert (np.diff(ref.indptr) > 65536).any()  # (hub neighbours among them)
    for j, i in enumerate(rows):
        a, b = int(grp[i]), int(grp[i + 1])
        np.testing.assert_array_equal(got[3][a:b], ref.indices[ref.indptr[j]:ref.indptr[j + 1]])
        np.testing.assert_array_equal(got[4][a:b], ref.data[ref.indptr[j]:ref.indptr[j + 1]])
