"""ctypes binding of spgemm_amd/lib/libtsg.so (the C ABI in include/tsg.h).

The library is built in-tree (spgemm_amd/csrc/Makefile).  Loading fails loudly
if it is missing; calls fail loudly (TsgError) on a non-zero status, including
TSG_ERR_NO_DEVICE when no MI355X is visible -- there is no CPU fallback.
"""
import ctypes as C
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_PATH = os.path.join(PKG, "lib", "libtsg.so")
# A/B diagnostics only: load another build of the same C ABI
LIB_PATH = os.environ.get("TSG_LIB_PATH", LIB_PATH)
HEADER = os.path.join(REPO, "include", "tsg.h")

TSG_OK = 0
STATUS = {0: "TSG_OK", -1: "TSG_ERR_INVALID", -2: "TSG_ERR_HIP", -3: "TSG_ERR_OOM",
          -4: "TSG_ERR_OVERFLOW", -5: "TSG_ERR_NO_DEVICE", -6: "TSG_ERR_UNSUPPORTED",
          -7: "TSG_ERR_IO"}


class TsgError(RuntimeError):
    def __init__(self, fn, rc):
        super().__init__(f"{fn} failed: {STATUS.get(rc, rc)} ({rc})")
        self.rc = rc


class SMatrix(C.Structure):
    """Field-for-field tsg_smatrix == the reference SMatrix (src/common.h:150-172)."""
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


class Stats(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "t_csr2tile_ms", "t_step1_ms", "t_step2_ms", "t_step3_ms", "t_tile2csr_ms",
        "t_malloc_ms", "t_kern_ms", "t_e2e_ms")] + [(n, C.c_longlong) for n in (
            "nnzCub", "numtileA", "numtileB", "numblkC", "nnzC", "tile_products")] + [
            ("t_step3_kernel_ms", C.c_double), ("path", C.c_longlong)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DevCSR(C.Structure):
    _fields_ = [("m", C.c_int), ("n", C.c_int), ("nnz", C.c_int),
                ("rowpointer", C.c_void_p), ("columnindex", C.c_void_p), ("value", C.c_void_p)]


class DevTiles(C.Structure):
    _fields_ = [("m", C.c_int), ("n", C.c_int), ("nnz", C.c_int),
                ("tile_m", C.c_int), ("tile_n", C.c_int),
                ("tilem", C.c_int), ("tilen", C.c_int), ("numtile", C.c_int)] + [
        (n, C.c_void_p) for n in ("tile_ptr", "tile_columnidx", "tile_rowidx", "tile_nnz",
                                  "tile_csr_Ptr", "tile_csr_Col", "tile_csr_Value", "mask",
                                  "csc_tile_ptr", "csc_tile_rowidx", "tile_rm2csc",
                                  "rm_mask", "rm_rowstart")]


_lib = None

_SIGS = {
    "tsg_version": ([], C.c_char_p),
    "tsg_device_count": ([C.POINTER(C.c_int)], C.c_int),
    "tsg_status_string": ([C.c_int], C.c_char_p),
    "tsg_mmio_allinone": ([C.c_char_p, C.POINTER(SMatrix)], C.c_int),
    "tsg_values_pos_mod10": ([C.POINTER(SMatrix)], None),
    "tsg_transpose": ([C.POINTER(SMatrix), C.POINTER(SMatrix)], C.c_int),
    "tsg_nnzcub": ([C.POINTER(SMatrix), C.POINTER(SMatrix), C.POINTER(C.c_ulonglong)], C.c_int),
    "tsg_csr2tile_row_major": ([C.POINTER(SMatrix), C.c_int, C.c_int], C.c_int),
    "tsg_csr2tile_col_major": ([C.POINTER(SMatrix), C.c_int, C.c_int], C.c_int),
    "tsg_tilespgemm": ([C.POINTER(SMatrix)] * 3 + [C.c_void_p, C.c_void_p, C.c_int, C.c_double,
                       C.c_double, C.c_ulonglong, C.POINTER(C.c_ulonglong)] +
                       [C.POINTER(C.c_double)] * 3 + [C.c_char_p] + [C.POINTER(C.c_double)] * 4 +
                       [C.c_int, C.c_int], C.c_int),
    "tsg_tile2csr": ([C.POINTER(SMatrix), C.c_int, C.c_int], C.c_int),
    "tsg_spgemm_csr": ([C.POINTER(SMatrix), C.POINTER(SMatrix), C.POINTER(SMatrix), C.c_int, C.c_int,
                        C.POINTER(Stats)], C.c_int),
    "tsg_matrix_destroy": ([C.POINTER(SMatrix)], None),
    "tsg_context_create": ([C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "tsg_context_destroy": ([C.c_void_p], C.c_int),
    "tsg_context_reset": ([C.c_void_p], C.c_int),
    "tsg_dev_csr2tile_row_major": ([C.c_void_p, C.POINTER(DevCSR), C.c_int, C.c_int, C.c_void_p,
                                    C.POINTER(DevTiles)], C.c_int),
    "tsg_dev_csr2tile_col_major": ([C.c_void_p, C.POINTER(DevCSR), C.c_int, C.c_int, C.c_void_p,
                                    C.POINTER(DevTiles)], C.c_int),
    "tsg_dev_tilespgemm": ([C.c_void_p, C.POINTER(DevTiles), C.POINTER(DevTiles), C.c_void_p,
                            C.POINTER(DevTiles), C.POINTER(Stats)], C.c_int),
    "tsg_dev_tile2csr": ([C.c_void_p, C.POINTER(DevTiles), C.c_void_p, C.POINTER(DevCSR)], C.c_int),
    "tsg_dev_transpose": ([C.c_void_p, C.POINTER(DevCSR), C.c_void_p, C.POINTER(DevCSR)], C.c_int),
    "tsg_dev_spgemm": ([C.c_void_p, C.POINTER(DevCSR), C.POINTER(DevCSR), C.c_int, C.c_int, C.c_void_p,
                        C.POINTER(DevCSR), C.POINTER(Stats)], C.c_int),
    "tsg_dev_spgemm_sorted_b": ([C.c_void_p, C.POINTER(DevCSR), C.POINTER(DevCSR), C.c_int, C.c_int, C.c_int,
                                 C.c_void_p, C.POINTER(DevCSR), C.POINTER(Stats)], C.c_int),
    "tsg_dev_csr_rows_sorted": ([C.c_void_p, C.POINTER(DevCSR), C.c_void_p, C.POINTER(C.c_int)], C.c_int),
    "tsg_memcpy_h2d": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p], C.c_int),
    "tsg_memcpy_d2h": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p], C.c_int),
    "tsg_memcpy_d2d": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p], C.c_int),
    "tsg_dev_malloc": ([C.c_void_p, C.POINTER(C.c_void_p), C.c_size_t], C.c_int),
    "tsg_dev_free": ([C.c_void_p, C.c_void_p], C.c_int),
}


def header_symbols():
    """Every function the C ABI header declares."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tsg_[a-z0-9_]+)\s*\(", txt)))


def build(quiet=True):
    """Build libtsg.so + the CLI in-tree (hipcc --offload-arch=gfx950)."""
    cmd = ["make", "-C", os.path.join(PKG, "csrc"), "-j4"]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libtsg.so not built ({LIB_PATH}); run spgemm_amd._lib.build() "
                              "or `make -C spgemm_amd/csrc`")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7.
        # Loading torch first makes libtsg.so's NEEDED libamdhip64.so.7 resolve to
        # that already-loaded copy; the other order would put two runtimes (and
        # two device views) in the process and torch then sees no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(fn, rc):
    if rc != TSG_OK:
        raise TsgError(fn, rc)
    return rc


def device_count():
    n = C.c_int(0)
    lib().tsg_device_count(C.byref(n))
    return n.value
