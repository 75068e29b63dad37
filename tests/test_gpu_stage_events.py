"""Stage markers on request (TSG_STAGE_EVENTS=1, tsg_api.cpp): without it the
row-merge and banded paths record only the numeric phase's bracket (each
marker cost a few us of GPU time on sub-millisecond calls), so their stage
times are 0 and the numeric phase's time is filled; with it every stage time
is measured.  The tiled route's step times follow the same switch.  C is the
same either way (checked against the oracle)."""
import numpy as np
import pytest

import _oracle as O
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu


def _banded(m, half):
    """rows i with columns |j - i| <= half (FEM-like: the banded path's input)"""
    lo = np.maximum(0, np.arange(m) - half)
    hi = np.minimum(m, np.arange(m) + half + 1)
    rp = np.concatenate([[0], np.cumsum(hi - lo)]).astype(np.int32)
    ci = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]).astype(np.int32)
    return m, m, rp, ci, (np.arange(len(ci)) % 10).astype(np.float64)


def _product(monkeypatch, on, name):
    if on:
        monkeypatch.setenv("TSG_STAGE_EVENTS", "1")
    else:
        monkeypatch.delenv("TSG_STAGE_EVENTS", raising=False)
    monkeypatch.delenv("TSG_PATH", raising=False)
    m, n, rp, ci, vv = synth.random_csr(3000, 3000, density=0.004, seed=81) if name == "rows" else \
        _banded(3000, 8)
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    C, st = T.spgemm(A, T.Matrix.alias(A))
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    ref = O.gustavson(oA, O.OMat.alias(oA)).csr()
    got = C.csr()
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=0)
    return st


@pytest.mark.parametrize("name", ["rows", "band"])
def test_stage_times_only_on_request(monkeypatch, name):
    for _ in range(2):  # (the second call: the context's allocations warm)
        off = _product(monkeypatch, False, name)
    on = _product(monkeypatch, True, name)
    assert off["path"] == on["path"] == (T.PATH_ROWS if name == "rows" else T.PATH_BAND)
    assert off["t_step3_kernel_ms"] > 0 and on["t_step3_kernel_ms"] > 0
    assert off["t_step1_ms"] == 0 and off["t_step3_ms"] == 0 and off["t_kern_ms"] == 0
    assert on["t_step1_ms"] > 0 and on["t_step3_ms"] > 0 and on["t_kern_ms"] > 0


def test_tiled_route_step_times_on_request(monkeypatch):
    m, n, rp, ci, vv = synth.random_csr(2000, 2000, density=0.005, seed=83)
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    B = T.Matrix.alias(A)
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    monkeypatch.delenv("TSG_STAGE_EVENTS", raising=False)
    _, off = T.tilespgemm(A, B, 16, 16)
    monkeypatch.setenv("TSG_STAGE_EVENTS", "1")
    _, on = T.tilespgemm(A, B, 16, 16)
    assert off["time_tile"] > 0 and on["time_tile"] > 0
    assert off["time_step2"] == 0 and off["time_step3"] == 0
    assert on["time_step2"] > 0 and on["time_step3"] > 0
