"""Per-call wall time vs the library's own t_e2e on a stand-in (host overhead check).
usage: python tools/step_overhead.py mc2depi [path]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import scipy.sparse as sp
import torch
from spgemm_amd import synth
from spgemm_amd.device import Context, DeviceCSR

name = sys.argv[1]
if len(sys.argv) > 2:
    os.environ["TSG_PATH"] = sys.argv[2]
m, n, rp, ci, vv = synth.GENERATORS[name]()
dA = DeviceCSR.from_host(m, n, rp, ci, vv)
if name == "mc2depi":
    T = sp.csr_matrix((vv, ci, rp), shape=(m, n)).T.tocsr(); T.sort_indices()
    dB = DeviceCSR.from_host(n, m, T.indptr, T.indices, T.data)
else:
    dB = dA
ctx = Context(0)
walls, e2e = [], []
for i in range(30):
    t0 = time.perf_counter()
    ctx.reset()
    c, st = ctx.spgemm(dA, dB)
    t1 = time.perf_counter()
    walls.append((t1 - t0) * 1e3)
    e2e.append(st["t_e2e_ms"])
torch.cuda.synchronize()
print(f"{name} path {int(st['path'])}: wall {np.median(walls[5:]):.3f} ms, t_e2e {np.median(e2e[5:]):.3f} ms")
ctx.close()
