"""Independent on-GPU cross-check: libtsg's C against rocSPARSE SpGEMM on the
BASELINE configs' synthetic stand-ins (the reference's
own cuSPARSE check, src/spgemm_cu.h:5-41, checks the pattern only).  Pattern
bit-exact, fp64 values within rtol 1e-10.  rocSPARSE is test infrastructure
(tests/rocsparse), never on the product path."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_bin", "librs_spgemm.so")


@pytest.fixture(scope="module")
def rs():
    import torch  # noqa: F401  (one HIP runtime per process)
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(HERE, "rocsparse")], check=True, capture_output=True)
    L = C.CDLL(LIB)
    P = C.POINTER
    L.rs_spgemm.argtypes = [C.c_int] * 4 + [C.c_void_p] * 3 + [C.c_int] + [C.c_void_p] * 3 + [
        P(C.c_longlong), P(P(C.c_int)), P(P(C.c_int)), P(P(C.c_double))]
    L.rs_free.argtypes = [C.c_void_p]
    return L


def rocsparse_product(L, A, B):
    m, k, rpa, cia, va = A
    k2, n, rpb, cib, vb = B
    assert k == k2
    arrs = [np.ascontiguousarray(x) for x in (rpa, cia, va, rpb, cib, vb)]
    nnz = C.c_longlong()
    prp, pci, pv = C.POINTER(C.c_int)(), C.POINTER(C.c_int)(), C.POINTER(C.c_double)()
    rc = L.rs_spgemm(m, k, n, len(cia), arrs[0].ctypes.data, arrs[1].ctypes.data, arrs[2].ctypes.data, len(cib),
                     arrs[3].ctypes.data, arrs[4].ctypes.data, arrs[5].ctypes.data, C.byref(nnz), C.byref(prp),
                     C.byref(pci), C.byref(pv))
    assert rc == 0, rc
    nz = nnz.value
    out = (np.ctypeslib.as_array(prp, (m + 1,)).copy(),
           np.ctypeslib.as_array(pci, (max(nz, 1),))[:nz].copy(),
           np.ctypeslib.as_array(pv, (max(nz, 1),))[:nz].copy())
    for p in (prp, pci, pv):
        L.rs_free(C.cast(p, C.c_void_p))
    return out


def _transpose(m, n, rp, ci, vv):
    import scipy.sparse as sp
    t = sp.csr_matrix((vv, ci, rp), shape=(m, n)).T.tocsr()
    t.sort_indices()
    return n, m, t.indptr.astype(np.int32), t.indices.astype(np.int32), t.data


def _rows(mat, rows):
    m, n, rp, ci, vv = mat
    return rows, n, rp[:rows + 1].copy(), ci[:rp[rows]].copy(), vv[:rp[rows]].copy()


@pytest.mark.parametrize("name", ["webbase", "cant", "mc2depi", "lj_prefix"])
def test_matches_rocsparse(rs, name):
    if name == "lj_prefix":
        full = synth.GENERATORS["lj"]()
        A, B = _rows(full, 20000), full
    else:
        A = synth.GENERATORS[name]()
        B = _transpose(*A) if name == "mc2depi" else A
    Cm, st = T.spgemm(T.Matrix.from_csr(*A), T.Matrix.from_csr(*B))
    _, _, rp, ci, vv = Cm.csr()
    rrp, rci, rvv = rocsparse_product(rs, A, B)
    np.testing.assert_array_equal(rp, rrp)
    np.testing.assert_array_equal(ci, rci)
    np.testing.assert_allclose(vv, rvv, rtol=1e-10, atol=0)
    assert st["nnzC"] == len(rci)
