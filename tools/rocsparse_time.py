"""Context only: device time of rocSPARSE SpGEMM (buffer-size + nnz + compute
stages, incl. its allocations) on a synthetic config, next to libtsg's e2e.
usage (GPU box): python tools/rocsparse_time.py [webbase|cant|mc2depi] [reps]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import torch  # noqa: E402,F401
import test_gpu_rocsparse as R  # noqa: E402
from spgemm_amd import synth  # noqa: E402
from spgemm_amd.device import Context, DeviceCSR  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "webbase"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
A = synth.GENERATORS[name]()
B = R._transpose(*A) if name == "mc2depi" else A
L = C.CDLL(R.LIB)
P = C.POINTER
L.rs_spgemm.argtypes = [C.c_int] * 4 + [C.c_void_p] * 3 + [C.c_int] + [C.c_void_p] * 3 + [
    P(C.c_longlong), P(P(C.c_int)), P(P(C.c_int)), P(P(C.c_double))]
L.rs_free.argtypes = [C.c_void_p]
L.rs_last_ms.restype = C.c_double
rs = []
for _ in range(reps + 1):
    R.rocsparse_product(L, A, B)
    rs.append(L.rs_last_ms())
ctx = Context(0)
dA, dB = DeviceCSR.from_host(*A), DeviceCSR.from_host(*B)
ts = []
for _ in range(reps + 1):
    ctx.reset()
    _, st = ctx.spgemm(dA, dB)
    ts.append(st["t_e2e_ms"])
blen = np.diff(B[2].astype(np.int64))
cub = int(blen[A[3]].sum())
print(f"{name}: nnzCub {cub}  rocSPARSE {np.median(rs[1:]):.3f} ms ({2 * cub / np.median(rs[1:]) / 1e6:.2f} GFLOPS)"
      f"  libtsg e2e {np.median(ts[1:]):.3f} ms ({2 * cub / np.median(ts[1:]) / 1e6:.2f} GFLOPS)")
