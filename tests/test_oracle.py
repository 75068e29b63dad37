"""Pin the CPU oracle (oracle/tsg_oracle.c) against the reference's own host code.

Goldens in tests/golden/ref were produced by oracle/_ref/ref_driver (the
reference's mmio_allinone / csr2tile_row_major / csr2tile_col_major /
spgemm_spa compiled from /root/reference/src) -- see tests/golden/make_golden.py.
Values of C are cross-checked against scipy.sparse (an independent product).
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import _oracle as O
from conftest import FIXTURES, golden_cases

CASES = golden_cases()


def load_pair(name, aat):
    A = O.OMat.load(os.path.join(FIXTURES, name + ".mtx"))
    B = O.transpose(A) if aat else O.OMat.alias(A)
    return A, B


def g(npz, key):
    return npz[key.replace(".", "__")]


@pytest.mark.parametrize("path,name,aat,tm,tn", CASES)
def test_oracle_matches_reference_host_code(path, name, aat, tm, tn):
    ref = np.load(path)
    A, B = load_pair(name, aat)
    # CSR after load + value overwrite (mmio_highlevel.h:593-759, main.cu:111-112)
    m, n, rp, ci, vv = A.csr()
    assert (m, n) == (int(g(ref, "A.m")), int(g(ref, "A.n")))
    np.testing.assert_array_equal(rp, g(ref, "A.rowpointer"))
    np.testing.assert_array_equal(ci, g(ref, "A.columnindex"))
    np.testing.assert_array_equal(vv, g(ref, "A.value"))
    mb, nb, rpb, cib, vvb = B.csr()
    np.testing.assert_array_equal(rpb, g(ref, "B.rowpointer"))
    np.testing.assert_array_equal(cib, g(ref, "B.columnindex"))
    np.testing.assert_array_equal(vvb, g(ref, "B.value"))
    assert O.nnzcub(A, B) == int(g(ref, "nnzCub"))

    # tiled layouts (csr2tile.h:205-506), every field bit-exact
    O.csr2tile_row_major(A, tm, tn)
    O.csr2tile_col_major(B, tm, tn)
    at = A.tiles(tm, tn // 16)
    bt = B.tiles(tn, tm // 16, csc=True)
    for k in ("tilem", "tilen", "numtile"):
        assert at[k] == int(g(ref, "At." + k)), k
        assert bt[k] == int(g(ref, "Bt." + k)), k
    for k in ("tile_ptr", "tile_columnidx", "tile_nnz", "tile_csr_Ptr", "tile_csr_Col",
              "tile_csr_Value", "mask"):
        np.testing.assert_array_equal(at[k], g(ref, "At." + k), err_msg="A " + k)
        np.testing.assert_array_equal(bt[k], g(ref, "Bt." + k), err_msg="B " + k)
    np.testing.assert_array_equal(bt["csc_tile_ptr"], g(ref, "Bt.csc_tile_ptr"))
    np.testing.assert_array_equal(bt["csc_tile_rowidx"], g(ref, "Bt.csc_tile_rowidx"))

    # tiled C: step-1 structure vs reference SPA over tile patterns
    Cm = O.tilespgemm(A, B, tm, tn)
    ct = O.c_tiles(Cm, tm)
    np.testing.assert_array_equal(ct["tile_ptr"], g(ref, "Ct.tile_ptr"))
    np.testing.assert_array_equal(ct["tile_columnidx"], g(ref, "Ct.tile_columnidx"))

    # tile2csr pattern vs reference SPA pattern (spgemm_serialref_spa_new.h)
    O.tile2csr(Cm, tm, tm)
    _, _, crp, cci, cvv = Cm.csr()
    np.testing.assert_array_equal(crp, g(ref, "C.rowpointer"))
    np.testing.assert_array_equal(cci, g(ref, "C.columnindex"))

    # values vs an independent product (scipy), structural pattern kept
    As = sp.csr_matrix((vv, ci, rp), shape=(m, n))
    Bs = sp.csr_matrix((vvb, cib, rpb), shape=(mb, nb))
    Cs = (As @ Bs).tocsr()
    dense_ref = Cs.toarray()
    dense_got = np.zeros((m, nb))
    for i in range(m):
        dense_got[i, cci[crp[i]:crp[i + 1]]] = cvv[crp[i]:crp[i + 1]]
    np.testing.assert_allclose(dense_got, dense_ref, rtol=1e-10, atol=0)

    # numeric Gustavson oracle agrees with the tiled oracle bit for bit
    Gm = O.gustavson(A, B)
    _, _, grp, gci, gvv = Gm.csr()
    np.testing.assert_array_equal(grp, crp)
    np.testing.assert_array_equal(gci, cci)
    np.testing.assert_array_equal(gvv, cvv)


def test_bitmask_known_answer():
    """UnitTest/CSR2TILE/bitmask.h: 36 uint64 row masks (MSB = column 0) equal the
    row pattern of random_0.1_36x36.mtx -- the known answer for the MSB-first
    mask convention of csr2tile.h:193-195 (there at u16 width)."""
    expect = [
        0x0000000000410000, 0x000000040C440244, 0x00000001AD040320, 0x0000000288124002,
        0x0000000331011923, 0x000000002198200A, 0x00000002C0000000, 0x0000000080102400,
        0x0000000702320604, 0x0000000602100036, 0x000000000C080090, 0x00000002C0010105,
        0x0000000040808332, 0x0000000C00008800, 0x0000000008082000, 0x000000015C064A04,
        0x0000000042210000, 0x0000000600102810, 0x0000000108100300, 0x0000000881081094,
        0x0000000000C00148, 0x0000000100100680, 0x0000000050242020, 0x0000000080010480,
        0x0000000080540885, 0x0000000018005002, 0x0000000608924008, 0x0000000281828072,
        0x0000000002015800, 0x0000000400008101, 0x0000000284802125, 0x0000000006850115,
        0x000000004000820F, 0x000000040D11083D, 0x00000001C4800509, 0x000000008100087F,
    ]
    A = O.OMat.load(os.path.join(FIXTURES, "random_0.1_36x36.mtx"))
    O.csr2tile_row_major(A, 16, 16)
    t = A.tiles(16, 1)
    # rebuild 36-bit rows from the 16x16 tile masks (3x3 tiles, MSB-first)
    rows = [0] * 36
    for ti in range(t["tilem"]):
        for p in range(t["tile_ptr"][ti], t["tile_ptr"][ti + 1]):
            tc = int(t["tile_columnidx"][p])
            for r in range(16):
                R = ti * 16 + r
                if R >= 36:
                    continue
                w = int(t["mask"][p * 16 + r])
                for b in range(16):
                    if (w >> (15 - b)) & 1:
                        rows[R] |= 1 << (35 - (tc * 16 + b))
    # bitmask.h stores the 36 columns in the low 36 bits, MSB of that field = col 0
    assert rows == expect
