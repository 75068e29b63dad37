"""fp64 value parity with non-integer values (north_star: values within 1e-10
relative).  The reference's value[k] = k % 10 makes every sum a small integer,
so these tests give A and B real values -- uniform(-1, 1), and signed values
spread over 16 decades -- and compare against the numeric Gustavson oracle
(a restatement of src/external/cusparse/spgemm_serialref_spa.h:7-119).

Tolerance: the GPU accumulates each C entry with LDS fp64 atomics, whose order
is run-dependent, and the oracle sums in CSR order; both are exact sums of the
same products up to rounding, so the bound is relative to the entry's
magnitude sum:  |c_gpu - c_ref| <= 1e-10 * (|A| |B|)_ij  (+0 absolute).  That
is the 1e-10 relative bar of north_star, stated for sums with cancellation.
The pattern (row pointers, columns, nnz) stays bit-exact.
"""
import os

import numpy as np
import pytest

import _oracle as O
from conftest import FIXTURES
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu
RTOL = 1e-10


def _vals(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        return rng.uniform(-1.0, 1.0, n)
    sign = np.where(rng.random(n) < 0.5, -1.0, 1.0)
    return sign * 10.0 ** rng.uniform(-8.0, 8.0, n)


def _check(m, n, rp, ci, va, mb, nb, rpb, cib, vb, alias=False):
    A = T.Matrix.from_csr(m, n, rp, ci, va)
    B = T.Matrix.alias(A) if alias else T.Matrix.from_csr(mb, nb, rpb, cib, vb)
    Cm, st = T.spgemm(A, B)
    gm, gn, grp, gci, gvv = Cm.csr()
    oA = O.OMat.from_csr(m, n, rp, ci, va)
    oB = O.OMat.from_csr(mb, nb, rpb, cib, vb)
    _, _, rrp, rci, rvv = O.gustavson(oA, oB).csr()
    np.testing.assert_array_equal(grp, rrp)
    np.testing.assert_array_equal(gci, rci)
    mag = O.gustavson(O.OMat.from_csr(m, n, rp, ci, np.abs(va)), O.OMat.from_csr(mb, nb, rpb, cib, np.abs(vb)))
    amag = mag.csr()[4]
    err = np.abs(gvv - rvv)
    bad = err > RTOL * amag
    assert not bad.any(), f"{bad.sum()} entries off; worst {np.max(err / np.maximum(amag, 1e-300))}"
    return gvv, st


@pytest.mark.parametrize("kind", ["uniform", "wide"])
@pytest.mark.parametrize("name", ["random_0.1_36x36", "banded_36x36", "x_powerlaw_400", "x_banded_500",
                                  "x_rect_50x130"])
def test_fixtures_real_values(name, kind):
    A0 = T.mmio_allinone(os.path.join(FIXTURES, name + ".mtx"))
    m, n, rp, ci, _ = A0.csr()
    va = _vals(kind, len(ci), 1)
    if m != n:  # A * A^T for the rectangular fixture
        import scipy.sparse as sp
        Bt = sp.csr_matrix((_vals(kind, len(ci), 2), ci, rp), shape=(m, n)).T.tocsr()
        Bt.sort_indices()
        _check(m, n, rp, ci, va, n, m, Bt.indptr.astype(np.int32), Bt.indices.astype(np.int32), Bt.data)
    else:
        _check(m, n, rp, ci, va, m, n, rp, ci, va, alias=True)


@pytest.mark.parametrize("mode", ["elem", "tile"])
@pytest.mark.parametrize("name", ["webbase", "cant"])
def test_full_size_real_values_both_step2_modes(name, mode, monkeypatch):
    monkeypatch.setenv("TSG_STEP2_MODE", mode)
    monkeypatch.setenv("TSG_PATH", "tiles")  # the staged pipeline's step-2 modes
    m, n, rp, ci, _ = synth.GENERATORS[name]()
    va = _vals("uniform", len(ci), 3)
    _check(m, n, rp, ci, va, m, n, rp, ci, va, alias=True)


def test_wide_magnitude_random_and_rerun_spread():
    """Wide-magnitude values on a random product; two runs agree within the
    same bound (the LDS atomic order may differ between runs)."""
    m, n, rp, ci, _ = synth.random_csr(3000, 3000, density=0.004, seed=9)
    va = _vals("wide", len(ci), 4)
    g1, _ = _check(m, n, rp, ci, va, m, n, rp, ci, va, alias=True)
    g2, _ = _check(m, n, rp, ci, va, m, n, rp, ci, va, alias=True)
    oA = O.OMat.from_csr(m, n, rp, ci, np.abs(va))
    mag = O.gustavson(oA, O.OMat.alias(oA)).csr()[4]
    assert np.all(np.abs(g1 - g2) <= 2 * RTOL * mag)


def test_full_size_real_values_default_routes():
    """cant's default route (the banded path) with real values."""
    m, n, rp, ci, _ = synth.GENERATORS["cant"]()
    va = _vals("uniform", len(ci), 7)
    _, st = _check(m, n, rp, ci, va, m, n, rp, ci, va, alias=True)
    assert st["numblkC"] == -1
