"""The fused element path (spgemm_amd/csrc/tsg_fused.hip): steps 1-3 and
tile2csr in one persistent kernel over row units, C tile row-segments (one
16-bit row mask of a 16x16 C tile) in an LDS hash, ranks by mask popcount,
unit offsets by a decoupled look-back.  Since round 3 the library's default
route sends short-row products to the row-merge path (faster there now);
TSG_PATH=fused forces the fused path on every input here, covering its heavy-row column windows
(histogram-merged windows, global-atomic values past the LDS accumulator).
Pattern bit-exact, values within 1e-10 relative, against the oracle."""
import os

import numpy as np
import pytest

import _oracle as O
from conftest import FIXTURES, golden_cases
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu


@pytest.fixture
def fused(monkeypatch):
    monkeypatch.setenv("TSG_PATH", "fused")


def _check(m, n, rp, ci, vv, aat=False):
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    if aat:
        B, oB = T.transpose(A), O.transpose(oA)
    else:
        B, oB = T.Matrix.alias(A), O.OMat.alias(oA)
    Cm, st = T.spgemm(A, B)
    got, ref = Cm.csr(), O.gustavson(oA, oB).csr()
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=0)
    assert st["nnzC"] == len(ref[3])
    return st


FIX = sorted({c.values[1] for c in golden_cases()})


@pytest.mark.parametrize("aat", [0, 1])
@pytest.mark.parametrize("name", FIX)
def test_fused_golden_fixtures(name, aat, fused):
    A = O.OMat.load(os.path.join(FIXTURES, name + ".mtx"))
    m, n, rp, ci, vv = A.csr()
    if aat == 0 and m != n:
        pytest.skip("A^2 needs a square matrix")
    if aat and A.s.isSymmetric:
        pytest.skip("the CLI refuses A*A^T of a symmetric-flagged matrix")
    st = _check(m, n, rp, ci, vv, aat=bool(aat))
    if aat:  # B = A^T: rows column-sorted by construction
        assert st["numtileA"] == -1  # the fused path ran
    else:  # B = A keeps the file's in-row order; unsorted B rows take the staged pipeline
        srt = all(np.all(np.diff(ci[rp[i]:rp[i + 1]]) > 0) for i in range(m))
        assert (st["numtileA"] == -1) == srt


@pytest.mark.parametrize("case", ["empty", "one", "rand_sparse", "dense", "rect_aat", "empty_rows"])
def test_fused_edge_cases(case, fused):
    if case == "empty":
        m, n, rp, ci, vv = 40, 40, np.zeros(41, np.int32), np.zeros(0, np.int32), np.zeros(0)
    elif case == "one":
        m, n, rp, ci, vv = synth.random_csr(1, 1, density=1.0, seed=1)
    elif case == "rand_sparse":
        m, n, rp, ci, vv = synth.random_csr(5000, 5000, density=0.0008, seed=21)
    elif case == "dense":  # every row heavy: a single-bin window per row, products past the slot cache
        m, n, rp, ci, vv = synth.random_csr(600, 600, density=0.2, seed=22)
    elif case == "rect_aat":
        m, n, rp, ci, vv = synth.random_csr(700, 2500, density=0.004, seed=23)
    else:
        m, n, rp, ci, vv = synth.random_csr(3000, 3000, density=0.001, seed=25)
    _check(m, n, rp, ci, vv, aat=(case == "rect_aat"))


@pytest.mark.parametrize("name", ["mc2depi", "webbase", "cant"])
def test_fused_full_size_stand_ins(name, fused):
    """webbase: 4,537 heavy rows cut into column windows; cant: every row heavy
    (one dense bin per row); mc2depi A*A^T: short rows only."""
    m, n, rp, ci, vv = synth.GENERATORS[name]()
    _check(m, n, rp, ci, vv, aat=(name == "mc2depi"))


def test_fused_mawi_hub_windows(fused):
    m, n, rp, ci, vv = synth.mawi(scale=3e-4)
    _check(m, n, rp, ci, vv)


def test_fused_real_values(fused):
    """non-integer fp64 values through LDS ds_add_f64 and the global-atomic
    window path: |c - ref| <= 1e-10 * (|A||B|)_ij"""
    m, n, rp, ci, _ = synth.random_csr(2000, 2000, density=0.05, seed=31)
    rng = np.random.default_rng(5)
    vv = rng.uniform(-1, 1, len(ci))
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    Cm, _ = T.spgemm(A, T.Matrix.alias(A))
    got = Cm.csr()
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    ref = O.gustavson(oA, O.OMat.alias(oA)).csr()
    oM = O.OMat.from_csr(m, n, rp, ci, np.abs(vv))
    mag = O.gustavson(oM, O.OMat.alias(oM)).csr()[4]
    np.testing.assert_array_equal(got[3], ref[3])
    assert np.all(np.abs(got[4] - ref[4]) <= 1e-10 * mag)


def test_default_routing_short_rows_go_to_row_merge():
    """mc2depi A*A^T (rows of <= 4 entries on both sides) and long rows spread
    over the columns both take the row-merge path by default (the fused path
    only when forced)."""
    m, n, rp, ci, vv = synth.mc2depi()
    st = _check(m, n, rp, ci, vv, aat=True)
    assert st["path"] == T.PATH_ROWS
    m, n, rp, ci, vv = synth.random_csr(3000, 3000, density=0.01, seed=4)  # ~30-entry rows
    st = _check(m, n, rp, ci, vv)
    assert st["path"] == T.PATH_ROWS
