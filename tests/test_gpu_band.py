"""The banded path (spgemm_amd/csrc/tsg_band.hip): every C row's reachable
columns inside one window of <= 2,048 columns with at least as many element
products as columns (FEM-like rows, e.g. cant).  One walk per row
accumulates a*b at acc[col - lo] in LDS and marks a hit byte per column; the
row's nonzeros go to a staging slot at the prefix of the window widths, a scan
of the row counts gives the CSR offsets and a compaction kernel moves them.  The library routes such products to it; TSG_PATH=band
forces it whenever the window check passes.  Pattern bit-exact, values within
1e-10 relative, against the oracle."""
import numpy as np
import pytest

import _oracle as O
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu


def _sorted_rows(m, n, rp, ci, vv):
    order = np.concatenate([rp[i] + np.argsort(ci[rp[i]:rp[i + 1]], kind="stable") for i in range(m)]
                           ).astype(np.int64) if len(ci) else np.zeros(0, np.int64)
    return m, n, rp, ci[order], vv[order]


def _banded(m, half, seed, fill=1.0):
    """rows i with columns |j - i| <= half (each kept with probability fill)"""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for i in range(m):
        js = np.arange(max(0, i - half), min(m, i + half + 1))
        js = js[rng.random(len(js)) < fill] if fill < 1.0 else js
        rows.append(np.full(len(js), i))
        cols.append(js)
    r = np.concatenate(rows)
    c = np.concatenate(cols).astype(np.int32)
    rp = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=m))]).astype(np.int32)
    vv = (np.arange(len(c)) % 10).astype(np.float64)
    return m, m, rp, c, vv


def _check(m, n, rp, ci, vv, aat=False, real=False):
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
    if real:
        oM = O.OMat.from_csr(m, n, rp, ci, np.abs(vv))
        oMb = O.transpose(oM) if aat else O.OMat.alias(oM)
        mag = O.gustavson(oM, oMb).csr()[4]
        assert np.all(np.abs(got[4] - ref[4]) <= 1e-10 * mag)
    else:
        np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=0)
    assert st["nnzC"] == len(ref[3])
    return st


@pytest.fixture
def band(monkeypatch):
    monkeypatch.setenv("TSG_PATH", "band")


@pytest.mark.parametrize("case", ["narrow", "wide_window", "gappy", "one_row", "empty_rows", "dense_block"])
def test_band_forced_vs_oracle(case, band):
    if case == "narrow":
        m, n, rp, ci, vv = _banded(3000, 8, 1)
    elif case == "wide_window":  # windows near the 2,048-column limit
        m, n, rp, ci, vv = _banded(4000, 500, 2, fill=0.3)
    elif case == "gappy":  # sparse band: window check may fail -> another path, same C
        m, n, rp, ci, vv = _banded(3000, 40, 3, fill=0.2)
    elif case == "one_row":
        m, n, rp, ci, vv = synth.random_csr(1, 1, density=1.0, seed=1)
    elif case == "empty_rows":
        m, n, rp, ci, vv = _banded(2000, 16, 4)
        keep = np.ones(m, bool)
        keep[::7] = False  # every 7th row empty
        lens = np.diff(rp) * keep
        mask = np.repeat(keep, np.diff(rp))
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        ci, vv = ci[mask], vv[mask]
    else:
        m, n, rp, ci, vv = _sorted_rows(*synth.random_csr(600, 600, density=0.2, seed=22))
    st = _check(m, n, rp, ci, vv)
    if case in ("narrow", "empty_rows", "dense_block"):
        assert st["path"] == T.PATH_BAND and st["numblkC"] == -1  # the banded path ran


def test_band_aat_and_real_values(band):
    m, n, rp, ci, _ = _banded(2500, 12, 5)
    vv = np.random.default_rng(6).uniform(-1, 1, len(ci))
    st = _check(m, n, rp, ci, vv, aat=True, real=True)
    assert st["path"] == T.PATH_BAND


def test_cant_routes_to_band_and_matches_oracle():
    """The cant stand-in (banded FEM-like, ~64 entries per row) takes the banded
    path by default; rows spread over all columns take the row-merge path."""
    m, n, rp, ci, vv = synth.GENERATORS["cant"]()
    st = _check(m, n, rp, ci, vv)
    assert st["path"] == T.PATH_BAND and st["numblkC"] == -1
    m, n, rp, ci, vv = synth.random_csr(3000, 3000, density=0.01, seed=4)  # spread rows
    st = _check(m, n, rp, ci, vv)
    assert st["path"] == T.PATH_ROWS
