"""ctypes binding of oracle/libtsg_oracle.so -- TEST INFRASTRUCTURE ONLY.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / reported CPU baseline.  Builds the oracle with `make -C oracle` on
first use if the .so is missing (gcc is available here and on the GPU box).
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "libtsg_oracle.so")
# diagnostics: another build of the same restatement (e.g. the ASan build, tools/asan_cpu.sh)
LIB_PATH = os.environ.get("TSG_ORACLE_LIB", LIB_PATH)


class TsgoMat(C.Structure):
    _fields_ = [
        ("m", C.c_int), ("n", C.c_int), ("nnz", C.c_int), ("isSymmetric", C.c_int),
        ("value", C.POINTER(C.c_double)), ("columnindex", C.POINTER(C.c_int)),
        ("rowpointer", C.POINTER(C.c_int)),
        ("tilem", C.c_int), ("tilen", C.c_int),
        ("tile_ptr", C.POINTER(C.c_int)), ("tile_columnidx", C.POINTER(C.c_int)),
        ("tile_rowidx", C.POINTER(C.c_int)), ("tile_nnz", C.POINTER(C.c_int)),
        ("numtile", C.c_int),
        ("tile_csr_Value", C.POINTER(C.c_double)), ("tile_csr_Col", C.POINTER(C.c_uint16)),
        ("tile_csr_Ptr", C.POINTER(C.c_uint16)), ("mask", C.POINTER(C.c_uint16)),
        ("csc_tile_ptr", C.POINTER(C.c_int)), ("csc_tile_rowidx", C.POINTER(C.c_int)),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "tsg_oracle.c")
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "libtsg_oracle.so"])
        L = C.CDLL(LIB_PATH)
        P = C.POINTER(TsgoMat)
        L.tsgo_mmio_load.argtypes = [C.c_char_p, P]
        L.tsgo_values_pos_mod10.argtypes = [P]
        L.tsgo_make_transpose.argtypes = [P, P]
        L.tsgo_nnzcub.argtypes = [P, P]
        L.tsgo_nnzcub.restype = C.c_ulonglong
        L.tsgo_csr2tile_row_major.argtypes = [P, C.c_int, C.c_int]
        L.tsgo_csr2tile_col_major.argtypes = [P, C.c_int, C.c_int]
        L.tsgo_tilespgemm.argtypes = [P, P, P, C.c_int, C.c_int]
        L.tsgo_tile2csr.argtypes = [P, C.c_int, C.c_int]
        L.tsgo_spa.argtypes = [P, P, C.c_void_p, C.c_void_p, C.POINTER(C.c_longlong),
                               C.c_int, C.c_int, C.c_int]
        L.tsgo_gustavson.argtypes = [P, P, P]
        L.tsgo_gustavson_rows.argtypes = [P, P, C.c_int, C.c_int]
        L.tsgo_gustavson_rows.restype = C.c_longlong
        L.tsgo_free.argtypes = [P]
        L.tsgo_num_threads.restype = C.c_int
        _lib = L
    return _lib


def _arr(ptr, n, dt):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dt)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt, copy=True)


class OMat:
    """Owns a TsgoMat; numpy inputs are kept alive while the struct points at them."""

    def __init__(self):
        self.s = TsgoMat()
        self._keep = []
        self._borrowed = set()

    def __del__(self):
        try:
            if _lib is not None:
                # borrowed arrays (numpy-owned or another OMat's) are detached first
                for name in self._borrowed:
                    setattr(self.s, name, None)
                _lib.tsgo_free(C.byref(self.s))
        except Exception:
            pass

    @classmethod
    def from_csr(cls, m, n, rowptr, col, val):
        o = cls()
        rp = np.ascontiguousarray(rowptr, dtype=np.int32)
        ci = np.ascontiguousarray(col, dtype=np.int32)
        vv = np.ascontiguousarray(val, dtype=np.float64)
        o._keep = [rp, ci, vv]
        o._borrowed = {"rowpointer", "columnindex", "value"}
        o.s.m, o.s.n, o.s.nnz = m, n, len(ci)
        o.s.rowpointer = rp.ctypes.data_as(C.POINTER(C.c_int))
        o.s.columnindex = ci.ctypes.data_as(C.POINTER(C.c_int))
        o.s.value = vv.ctypes.data_as(C.POINTER(C.c_double))
        return o

    @classmethod
    def alias(cls, A):
        """B := A sharing A's CSR arrays (src/main.cu:145-151)."""
        o = cls()
        o._keep = [A]
        o._borrowed = {"rowpointer", "columnindex", "value"}
        o.s.m, o.s.n, o.s.nnz = A.s.m, A.s.n, A.s.nnz
        o.s.rowpointer, o.s.columnindex, o.s.value = A.s.rowpointer, A.s.columnindex, A.s.value
        return o

    @classmethod
    def load(cls, path, pos_mod10=True):
        o = cls()
        rc = lib().tsgo_mmio_load(path.encode(), C.byref(o.s))
        if rc != 0:
            raise RuntimeError(f"oracle mmio load failed rc={rc} for {path}")
        if pos_mod10:
            lib().tsgo_values_pos_mod10(C.byref(o.s))
        return o

    def csr(self):
        s = self.s
        return (s.m, s.n, _arr(s.rowpointer, s.m + 1, np.int32),
                _arr(s.columnindex, s.nnz, np.int32), _arr(s.value, s.nnz, np.float64))

    def tiles(self, ptr_rows, mask_words, csc=False):
        s = self.s
        d = dict(tilem=s.tilem, tilen=s.tilen, numtile=s.numtile,
                 tile_ptr=_arr(s.tile_ptr, s.tilem + 1, np.int32),
                 tile_columnidx=_arr(s.tile_columnidx, s.numtile, np.int32),
                 tile_nnz=_arr(s.tile_nnz, s.numtile + 1, np.int32),
                 tile_csr_Ptr=_arr(s.tile_csr_Ptr, s.numtile * ptr_rows, np.uint16),
                 tile_csr_Col=_arr(s.tile_csr_Col, s.nnz if not csc else s.nnz, np.uint16),
                 tile_csr_Value=_arr(s.tile_csr_Value, s.nnz, np.float64),
                 mask=_arr(s.mask, s.numtile * ptr_rows * mask_words, np.uint16))
        if csc:
            d["csc_tile_ptr"] = _arr(s.csc_tile_ptr, s.tilen + 1, np.int32)
            d["csc_tile_rowidx"] = _arr(s.csc_tile_rowidx, s.numtile, np.int32)
        return d


def transpose(A):
    B = OMat()
    lib().tsgo_make_transpose(C.byref(A.s), C.byref(B.s))
    return B


def nnzcub(A, B):
    return int(lib().tsgo_nnzcub(C.byref(A.s), C.byref(B.s)))


def csr2tile_row_major(A, tm, tn):
    rc = lib().tsgo_csr2tile_row_major(C.byref(A.s), tm, tn)
    assert rc == 0, rc


def csr2tile_col_major(B, tm, tn):
    rc = lib().tsgo_csr2tile_col_major(C.byref(B.s), tm, tn)
    assert rc == 0, rc


def tilespgemm(A, B, tm, tn):
    Cm = OMat()
    rc = lib().tsgo_tilespgemm(C.byref(A.s), C.byref(B.s), C.byref(Cm.s), tm, tn)
    assert rc == 0, rc
    return Cm


def c_tiles(Cm, tm):
    s = Cm.s
    wpr = tm // 16
    nnz = s.nnz
    return dict(tilem=s.tilem, tilen=s.tilen, numtile=s.numtile,
                tile_ptr=_arr(s.tile_ptr, s.tilem + 1, np.int32),
                tile_columnidx=_arr(s.tile_columnidx, s.numtile, np.int32),
                tile_nnz=_arr(s.tile_nnz, s.numtile + 1, np.int32),
                tile_csr_Ptr=_arr(s.tile_csr_Ptr, s.numtile * tm, np.uint16),
                tile_csr_Col=_arr(s.tile_csr_Col, nnz, np.uint16),
                tile_csr_Value=_arr(s.tile_csr_Value, nnz, np.float64),
                mask=_arr(s.mask, s.numtile * tm * wpr, np.uint16))


def tile2csr(Cm, tm, tn):
    rc = lib().tsgo_tile2csr(C.byref(Cm.s), tm, tn)
    assert rc == 0, rc


def spa(A, B, row_begin=0, row_end=None):
    if row_end is None:
        row_end = A.s.m
    rp = np.zeros(A.s.m + 1, dtype=np.int32)
    nnz = C.c_longlong(0)
    rc = lib().tsgo_spa(C.byref(A.s), C.byref(B.s), rp.ctypes.data, None, C.byref(nnz), 1,
                        row_begin, row_end)
    if rc == -2:
        raise OverflowError(f"spa: nnz(C) of rows [{row_begin},{row_end}) = {nnz.value} exceeds int32")
    assert rc == 0, rc
    ci = np.zeros(max(int(nnz.value), 1), dtype=np.int32)
    lib().tsgo_spa(C.byref(A.s), C.byref(B.s), rp.ctypes.data, ci.ctypes.data, C.byref(nnz), 0,
                   row_begin, row_end)
    return rp, ci[: int(nnz.value)]


def gustavson(A, B):
    Cm = OMat()
    rc = lib().tsgo_gustavson(C.byref(A.s), C.byref(B.s), C.byref(Cm.s))
    assert rc == 0, rc
    return Cm


def gustavson_rows(A, B, r0, r1):
    return int(lib().tsgo_gustavson_rows(C.byref(A.s), C.byref(B.s), r0, r1))


def num_threads():
    return int(lib().tsgo_num_threads())
