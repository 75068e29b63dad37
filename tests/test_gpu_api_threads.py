"""Host API threading: each reference-named host call leases
its own context and stream for the calling thread's device, so host threads
calling tsg_spgemm_csr / the tile API concurrently on one device get exact
results (ctypes releases the GIL around the foreign call)."""
import threading

import numpy as np
import pytest

import _oracle as O
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu


def _run(seed, results, idx, reps=4):
    m, n, rp, ci, vv = synth.random_csr(4000 + 37 * seed, 4000 + 37 * seed, density=0.002, seed=seed)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    ref = O.gustavson(oA, O.OMat.alias(oA)).csr()
    ok = True
    try:
        for r in range(reps):
            A = T.Matrix.from_csr(m, n, rp, ci, vv)
            if r % 2 == 0:
                Cm, _ = T.spgemm(A, T.Matrix.alias(A))
            else:  # the reference's tiled path: csr2tile + tilespgemm + tile2csr
                B = T.Matrix.from_csr(m, n, rp, ci, vv)
                T.csr2tile_row_major(A, 16, 16)
                T.csr2tile_col_major(B, 16, 16)
                Cm, _ = T.tilespgemm(A, B, 16, 16)
                T.tile2csr(Cm, 16, 16)
            got = Cm.csr()
            ok &= np.array_equal(got[2], ref[2]) and np.array_equal(got[3], ref[3])
            ok &= np.allclose(got[4], ref[4], rtol=1e-10, atol=0)
        results[idx] = ok
    except Exception as e:  # surfaced by the assertion below
        results[idx] = e


def test_concurrent_host_threads_same_device():
    nth = 4
    results = [None] * nth
    ths = [threading.Thread(target=_run, args=(s, results, i)) for i, s in enumerate(range(1, nth + 1))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert all(r is True for r in results), results
