"""BASELINE configs that the full-size tests cannot hold in one int32 C.

com-LiveJournal (config 4): the R-MAT stand-in's A^2 has 1.3e11 intermediate
products -- past the reference's `int nnzC` (src/tilespgemm-cuda.h:2327) -- so
the product runs as sequential tile-row blocks (spgemm_amd.dist.product_blocks,
what `bench.py --matrix lj` times).  Here: the block with the most work (the
hub rows, the load-imbalanced case) and two strided blocks, each C against the
numeric Gustavson oracle at 1e8-product blocks (host-checkable sizes).
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
    pick = [int(np.argmax(dens)), len(blocks) // 3, 2 * len(blocks) // 3]
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
