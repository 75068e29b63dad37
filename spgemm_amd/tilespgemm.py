"""Host-side mirror of the reference's TileSpGEMM operator interface.

Same names, argument meaning and error behaviour as the reference's host
functions (paths under /root/reference/src), each running the gfx950 HIP
kernels of libtsg.so through the C ABI (include/tsg.h):

  mmio_allinone(path)                -> Matrix        mmio_highlevel.h:593-759
  values_pos_mod10(A)                                  main.cu:111-112
  transpose(A)                       -> Matrix        utils.h:161-198 (on the GPU)
  nnzcub(A, B)                       -> int           main.cu:155-162 (on the GPU)
  csr2tile_row_major(A, tm, tn)                        csr2tile.h:205-277
  csr2tile_col_major(B, tm, tn)                        csr2tile.h:279-506
  tilespgemm(A, B, tm, tn, nnzCub)   -> (C, info)     tilespgemm-cuda.h:2220-2844
  tile2csr(C, tm, tn)                                  tile2csr.h:72-140
  spgemm(A, B, tm, tn)               -> (Matrix, stats)  one-shot CSR -> CSR

Errors raise TsgError (the reference exits or silently misbehaves instead).
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import SMatrix, Stats, check, lib

_CSR_FIELDS = ("rowpointer", "columnindex", "value")

# stats["path"]: the CSR-in -> CSR-out route that ran (include/tsg.h TSG_PATH_*)
PATH_TILES, PATH_BAND, PATH_ROWS = 0, 2, 3  # (1: the retired fused path)


def _view(ptr, n, dt):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dt)
    return np.ctypeslib.as_array(ptr, shape=(int(n),)).astype(dt, copy=True)


class Matrix:
    """Owns one SMatrix.  Arrays set from numpy are borrowed (kept alive here and
    detached before tsg_matrix_destroy); library-filled arrays are owned."""

    def __init__(self):
        self.s = SMatrix()
        self._keep = []
        self._borrowed = set()

    def __del__(self):
        try:
            for f in self._borrowed:
                setattr(self.s, f, None)
            if _lib._lib is not None:
                _lib._lib.tsg_matrix_destroy(C.byref(self.s))
        except Exception:
            pass

    @classmethod
    def from_csr(cls, m, n, rowptr, col, val, is_symmetric=0):
        o = cls()
        rp = np.ascontiguousarray(rowptr, dtype=np.int32)
        ci = np.ascontiguousarray(col, dtype=np.int32)
        vv = np.ascontiguousarray(val, dtype=np.float64)
        if rp.shape[0] != m + 1 or ci.shape[0] != vv.shape[0] or int(rp[-1]) != ci.shape[0]:
            raise ValueError("inconsistent CSR arrays")
        o._keep = [rp, ci, vv]
        o._borrowed = set(_CSR_FIELDS)
        o.s.m, o.s.n, o.s.nnz, o.s.isSymmetric = m, n, ci.shape[0], is_symmetric
        o.s.rowpointer = rp.ctypes.data_as(C.POINTER(C.c_int))
        o.s.columnindex = ci.ctypes.data_as(C.POINTER(C.c_int))
        o.s.value = vv.ctypes.data_as(C.POINTER(C.c_double))
        return o

    @classmethod
    def alias(cls, A):
        """B := A sharing A's CSR arrays (src/main.cu:145-151)."""
        o = cls()
        o._keep = [A]
        o._borrowed = set(_CSR_FIELDS)
        o.s.m, o.s.n, o.s.nnz = A.s.m, A.s.n, A.s.nnz
        o.s.rowpointer, o.s.columnindex, o.s.value = A.s.rowpointer, A.s.columnindex, A.s.value
        return o

    @property
    def shape(self):
        return (self.s.m, self.s.n)

    def csr(self):
        s = self.s
        return (s.m, s.n, _view(s.rowpointer, s.m + 1, np.int32),
                _view(s.columnindex, s.nnz, np.int32), _view(s.value, s.nnz, np.float64))

    def tiles(self, ptr_rows, mask_words, csc=False):
        s = self.s
        d = dict(tilem=s.tilem, tilen=s.tilen, numtile=s.numtile,
                 tile_ptr=_view(s.tile_ptr, s.tilem + 1, np.int32),
                 tile_columnidx=_view(s.tile_columnidx, s.numtile, np.int32),
                 tile_rowidx=_view(s.tile_rowidx, s.numtile, np.int32),
                 tile_nnz=_view(s.tile_nnz, s.numtile + 1, np.int32),
                 tile_csr_Ptr=_view(s.tile_csr_Ptr, s.numtile * ptr_rows, np.uint16),
                 tile_csr_Col=_view(s.tile_csr_Col, s.nnz, np.uint16),
                 tile_csr_Value=_view(s.tile_csr_Value, s.nnz, np.float64),
                 mask=_view(s.mask, s.numtile * ptr_rows * mask_words, np.uint16))
        if csc:
            d["csc_tile_ptr"] = _view(s.csc_tile_ptr, s.tilen + 1, np.int32)
            d["csc_tile_rowidx"] = _view(s.csc_tile_rowidx, s.numtile, np.int32)
        return d


def mmio_allinone(path):
    A = Matrix()
    check("tsg_mmio_allinone", lib().tsg_mmio_allinone(path.encode(), C.byref(A.s)))
    return A


def values_pos_mod10(A):
    lib().tsg_values_pos_mod10(C.byref(A.s))


def transpose(A):
    B = Matrix()
    check("tsg_transpose", lib().tsg_transpose(C.byref(A.s), C.byref(B.s)))
    return B


def nnzcub(A, B):
    out = C.c_ulonglong(0)
    check("tsg_nnzcub", lib().tsg_nnzcub(C.byref(A.s), C.byref(B.s), C.byref(out)))
    return int(out.value)


def csr2tile_row_major(A, tile_size_m=16, tile_size_n=16):
    check("tsg_csr2tile_row_major", lib().tsg_csr2tile_row_major(C.byref(A.s), tile_size_m, tile_size_n))


def csr2tile_col_major(B, tile_size_m=16, tile_size_n=16):
    check("tsg_csr2tile_col_major", lib().tsg_csr2tile_col_major(C.byref(B.s), tile_size_m, tile_size_n))


def tilespgemm(A, B, tile_size_m=16, tile_size_n=16, nnzCub=0, filename=None):
    """C = A*B on tiled inputs; returns (C, info) where info mirrors the
    reference's out-parameters (src/tilespgemm-cuda.h:2228-2235)."""
    Cm = Matrix()
    nnzC = C.c_ulonglong(0)
    outs = [C.c_double(0) for _ in range(7)]
    rc = lib().tsg_tilespgemm(C.byref(A.s), C.byref(B.s), C.byref(Cm.s), None, None, 0, 0.0, 0.0,
                              C.c_ulonglong(nnzCub), C.byref(nnzC), C.byref(outs[0]), C.byref(outs[1]),
                              C.byref(outs[2]), (filename or "").encode(), C.byref(outs[3]),
                              C.byref(outs[4]), C.byref(outs[5]), C.byref(outs[6]),
                              tile_size_m, tile_size_n)
    check("tsg_tilespgemm", rc)
    info = dict(nnzC=int(nnzC.value), compression_rate=outs[0].value, time_tile=outs[1].value,
                gflops_tile=outs[2].value, time_step1=outs[3].value, time_step2=outs[4].value,
                time_step3=outs[5].value, time_malloc=outs[6].value)
    return Cm, info


def tile2csr(Cm, tile_size_m=16, tile_size_n=16):
    check("tsg_tile2csr", lib().tsg_tile2csr(C.byref(Cm.s), tile_size_m, tile_size_n))


def spgemm(A, B, tile_size_m=16, tile_size_n=16):
    """One-shot CSR -> CSR on the GPU; returns (C Matrix, stats dict)."""
    Cm = Matrix()
    st = Stats()
    check("tsg_spgemm_csr", lib().tsg_spgemm_csr(C.byref(A.s), C.byref(B.s), C.byref(Cm.s),
                                                 tile_size_m, tile_size_n, C.byref(st)))
    return Cm, st.as_dict()
