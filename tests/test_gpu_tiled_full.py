"""The drop-in tiled path at the BASELINE sizes (synthetic stand-ins).

What the reference's `./test` runs (src/main.cu:168-327): csr2tile of A
(row-major) and B (col-major), tilespgemm (src/tilespgemm-cuda.h:2220-2844:
the tile-pattern step 1 WITH structurally empty C tiles, step 2 masks + scan,
step 3 values), tile2csr -- here tsg_csr2tile_row_major/col_major ->
tsg_tilespgemm -> tsg_tile2csr through the C ABI, on the full-size cant,
webbase and mc2depi (A*A^T) stand-ins and on the heaviest LiveJournal row
block.  Compared, as the reference's own end-of-run check does for the whole
C (src/main.cu:325-350), but field by field:

  * C's tile structure (tile_ptr, tile_columnidx, empty tiles included) and
    every C tile field (tile_nnz, tile_csr_Ptr, tile_csr_Col, tile_csr_Value)
    against the oracle's tiled product (tests/_oracle.py tilespgemm, pinned to
    the reference's host code by tests/test_oracle.py); integer fields
    bit-exact, values within rtol 1e-10 (exact in practice: value = pos % 10);
  * the CSR C from tsg_tile2csr against the numeric Gustavson oracle.
"""
import numpy as np
import pytest

import _oracle as O
from spgemm_amd import dist as tdist
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu
RTOL = 1e-10
C_FIELDS = ("tile_nnz", "tile_csr_Ptr", "tile_csr_Col")


def _operands(m, n, rp, ci, vv, aat, B_csr=None):
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    if B_csr is not None:
        mb, nb, rpb, cib, vvb = B_csr
        return A, T.Matrix.from_csr(mb, nb, rpb, cib, vvb), oA, O.OMat.from_csr(mb, nb, rpb, cib, vvb)
    if aat:
        return A, T.transpose(A), oA, O.transpose(oA)
    return A, T.Matrix.alias(A), oA, O.OMat.alias(oA)


def _check_dropin(A, B, oA, oB, tm=16):
    T.csr2tile_row_major(A, tm, tm)
    T.csr2tile_col_major(B, tm, tm)
    Cm, info = T.tilespgemm(A, B, tm, tm)
    ct = Cm.tiles(tm, tm // 16)
    O.csr2tile_row_major(oA, tm, tm)
    O.csr2tile_col_major(oB, tm, tm)
    oC = O.tilespgemm(oA, oB, tm, tm)
    oct_ = O.c_tiles(oC, tm)
    # step 1: the tile-pattern structure, structurally empty C tiles included
    assert ct["numtile"] == oct_["numtile"]
    np.testing.assert_array_equal(ct["tile_ptr"], oct_["tile_ptr"])
    np.testing.assert_array_equal(ct["tile_columnidx"], oct_["tile_columnidx"])
    empty = int(np.count_nonzero(np.diff(oct_["tile_nnz"]) == 0))
    # steps 2 and 3: every C tile field
    for k in C_FIELDS:
        np.testing.assert_array_equal(ct[k], oct_[k], err_msg="C " + k)
    np.testing.assert_allclose(ct["tile_csr_Value"], oct_["tile_csr_Value"], rtol=RTOL, atol=0)
    assert info["nnzC"] == oC.s.nnz
    del ct, oct_, oC
    # tile2csr -> CSR C against Gustavson
    T.tile2csr(Cm, tm, tm)
    _, _, grp, gci, gvv = Cm.csr()
    _, _, rrp, rci, rvv = O.gustavson(oA, oB).csr()
    np.testing.assert_array_equal(grp, rrp)
    np.testing.assert_array_equal(gci, rci)
    np.testing.assert_allclose(gvv, rvv, rtol=RTOL, atol=0)
    return info, empty


@pytest.mark.parametrize("name", ["cant", "mc2depi", "webbase"])
def test_dropin_tiled_path_full_size_vs_oracle(name):
    m, n, rp, ci, vv = synth.GENERATORS[name]()
    A, B, oA, oB = _operands(m, n, rp, ci, vv, aat=name == "mc2depi")
    info, empty = _check_dropin(A, B, oA, oB)
    assert info["time_tile"] > 0
    if name == "webbase":  # the reference's tile-pattern step 1 keeps empty C tiles
        assert empty > 1_000_000


def test_dropin_tiled_path_lj_heaviest_block_vs_oracle():
    """The LiveJournal stand-in's densest 1e8-product row block (the hub rows)
    through the drop-in path, B = the whole matrix."""
    m, n, rp, ci, vv = synth.rmat()
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    blocks = tdist.product_blocks(cum, 0, m, 1e8, 16)
    dens = np.array([(cum[b1] - cum[b0]) / (b1 - b0) for b0, b1 in blocks])
    b0, b1 = blocks[int(np.argmax(dens))]
    mb, rpb, cib, vvb = tdist.slice_rows(m, rp, ci, vv, b0, b1)
    A, B, oA, oB = _operands(mb, n, rpb, cib, vvb, aat=False, B_csr=(m, n, rp, ci, vv))
    _check_dropin(A, B, oA, oB)
