"""GPU: the less common step-1 paths of the element pipeline.

* the second element walk (no unit buffers, no stored bitmasks), forced with
  TSG_ABLATE=768 in a child process (the library reads TSG_ABLATE once);
* a B too wide for its (tile row, window) count units (mawi-like: 2^31 units),
  whose tile count is then reported as -1 while steps 1-3 read B's CSR.

Expected C from scipy (the products are small integers: exact in fp64).
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _check(m, n, rp, ci, vv, mb, nb, rpb, cib, vvb):
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    B = T.Matrix.from_csr(mb, nb, rpb, cib, vvb)
    Cm, st = T.spgemm(A, B)
    cm, cn, crp, cci, cvv = Cm.csr()
    ref = (sp.csr_matrix((vv, ci, rp), shape=(m, n)) @ sp.csr_matrix((vvb, cib, rpb), shape=(mb, nb))).tocsr()
    ref.sort_indices()
    assert (cm, cn) == ref.shape
    np.testing.assert_array_equal(crp, ref.indptr)
    np.testing.assert_array_equal(cci, ref.indices)
    np.testing.assert_allclose(cvv, ref.data, rtol=1e-10, atol=0)  # explicit zeros: none (values >= 1)
    return st


_CHILD = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
from test_gpu_step1_paths import _check
from spgemm_amd import synth
for (m, n, seed) in [(3000, 3000, 1), (600, 1_200_000, 2)]:
    mm, nn, rp, ci, vv = synth.random_csr(m, n, nnz_per_row=4, seed=seed)
    vv = vv + 1.0
    mb, nb, rpb, cib, vvb = synth.random_csr(n, n, nnz_per_row=3, seed=seed + 10)
    vvb = vvb + 1.0
    _check(mm, nn, rp, ci, vv, mb, nb, rpb, cib, vvb)
print("child ok")
"""


def test_second_element_walk_and_multiwindow():
    """TSG_ABLATE=768: no unit buffers (512) and no stored bitmasks (256), so
    step 1 emits by a second element walk; one case has 2 column windows."""
    env = dict(os.environ, TSG_ABLATE="768", TSG_PATH="tiles")
    code = _CHILD.format(repo=REPO, tests=os.path.join(REPO, "tests"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_b_too_wide_for_tile_counts(monkeypatch):
    """B with n = 2e8 (12.5 M tile rows x 191 windows > 2^31 count units):
    the element path runs on B's CSR; numtileB is reported as -1."""
    monkeypatch.setenv("TSG_PATH", "tiles")
    n = 200_000_000
    rng = np.random.default_rng(5)
    # A: 40 rows over the first 2,000 columns; B: rows < 2,000 hold 3 columns
    # spread over all of [0, n), the other rows are empty
    m, k = 40, 2000
    ci = np.sort(rng.choice(k, size=(m, 5), replace=True), axis=1).astype(np.int32)
    rows_a = [np.unique(r) for r in ci]
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows_a])]).astype(np.int32)
    ci = np.concatenate(rows_a).astype(np.int32)
    vv = (np.arange(len(ci)) % 10 + 1).astype(np.float64)
    rows_b = [np.unique(rng.integers(0, n, size=3)) for _ in range(k)]
    cnt = np.zeros(n + 1, dtype=np.int64)
    cnt[1:k + 1] = [len(r) for r in rows_b]
    rpb = np.cumsum(cnt).astype(np.int32)
    cib = np.concatenate(rows_b).astype(np.int32)
    vvb = (np.arange(len(cib)) % 10 + 1).astype(np.float64)
    st = _check(m, n, rp, ci, vv, n, n, rpb, cib, vvb)
    assert st["path"] == T.PATH_TILES and st["numtileB"] == -1


@pytest.mark.parametrize("nb", [300_000, 1_200_000])
def test_wide_b_tile_mode_step1_vs_oracle(nb):
    """The reference switches step 1 to the nsparse hash at > 16,384 B tile
    columns (src/tilespgemm-cuda.h:2379-2395).  Through the reference-layout
    host path (tsg_tilespgemm), C's tile-PATTERN structure (tile_ptr,
    tile_columnidx, empty tiles included) and every C tile field must equal the
    oracle's at 18,750 tile columns (one step-1 window) and 75,000 (two
    windows of 65,536)."""
    import _oracle as O
    m, k = 300, 3000
    mm, kk, rp, ci, vv = synth.random_csr(m, k, nnz_per_row=4, seed=nb % 97)
    _, _, rpb, cib, vvb = synth.random_csr(k, nb, nnz_per_row=3, seed=nb % 89)
    A = T.Matrix.from_csr(m, k, rp, ci, vv)
    B = T.Matrix.from_csr(k, nb, rpb, cib, vvb)
    oA = O.OMat.from_csr(m, k, rp, ci, vv)
    oB = O.OMat.from_csr(k, nb, rpb, cib, vvb)
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    O.csr2tile_row_major(oA, 16, 16)
    O.csr2tile_col_major(oB, 16, 16)
    Cm, _ = T.tilespgemm(A, B, 16, 16)
    oC = O.tilespgemm(oA, oB, 16, 16)
    ct, oct_ = Cm.tiles(16, 1), O.c_tiles(oC, 16)
    assert ct["numtile"] == oct_["numtile"]
    for key in ("tile_ptr", "tile_columnidx", "tile_nnz", "tile_csr_Ptr", "tile_csr_Col", "tile_csr_Value"):
        np.testing.assert_array_equal(ct[key], oct_[key], err_msg=key)
