"""Time the staged (tiles) and fused paths on the light rows and on the heavy
rows of a stand-in (the other rows emptied; B = the full matrix)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from spgemm_amd import synth
from spgemm_amd.device import Context, DeviceCSR


def keep_rows(m, rp, ci, vv, keep):
    lens = np.diff(rp) * keep
    nrp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    mask = np.repeat(keep, np.diff(rp))
    return nrp, ci[mask], vv[mask]


name = sys.argv[1]
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
m, n, rp, ci, vv = synth.GENERATORS[name]()
blen = np.diff(rp.astype(np.int64))
cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
P = np.diff(cum)
dB = DeviceCSR.from_host(m, n, rp, ci, vv)
ctx = Context(0)
for part, keep in (("light", P <= cap), ("heavy", P > cap), ("all", P >= 0)):
    nrp, nci, nvv = keep_rows(m, rp, ci, vv, keep)
    dA = DeviceCSR.from_host(m, n, nrp, nci, nvv)
    for path in ("fused", "tiles"):
        os.environ["TSG_PATH"] = path
        sts = []
        for i in range(6):
            ctx.reset()
            c, st = ctx.spgemm(dA, dB)
            sts.append(st)
        torch.cuda.synchronize()
        med = lambda k: float(np.median([s[k] for s in sts[2:]]))
        print(f"{name} {part} ({int(P[keep].sum())} products) {path}: e2e {med('t_e2e_ms'):.3f} kern {med('t_kern_ms'):.3f} "
              f"k3 {med('t_step3_kernel_ms'):.3f} nnzC {sts[-1]['nnzC']}", flush=True)
