"""Warm timing of the device pipeline (fused vs staged tiles) on stand-ins.
usage: python tools/fz_time.py webbase [cant mc2depi ...] [--light] [--path=fused,tiles]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from spgemm_amd import synth
from spgemm_amd.device import Context, DeviceCSR


def light_only(m, n, rp, ci, vv, cap=2048):
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    keep = np.diff(cum) <= cap
    lens = np.diff(rp) * keep
    nrp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    mask = np.repeat(keep, np.diff(rp))
    return m, n, nrp, ci[mask], vv[mask]


def run(name, light, reps=8):
    m, n, rp, ci, vv = synth.GENERATORS[name]()
    if light:
        m, n, rp, ci, vv = light_only(m, n, rp, ci, vv)
    aat = name == "mc2depi"
    dA = DeviceCSR.from_host(m, n, rp, ci, vv)
    if aat:
        import scipy.sparse as sp
        T = sp.csr_matrix((vv, ci, rp), shape=(m, n)).T.tocsr(); T.sort_indices()
        dB = DeviceCSR.from_host(n, m, T.indptr, T.indices, T.data)
    else:
        dB = dA
    ctx = Context(0)
    for path in PATHS:
        os.environ["TSG_PATH"] = path
        sts = []
        for i in range(reps):
            ctx.reset()
            c, st = ctx.spgemm(dA, dB)
            sts.append(st)
        torch.cuda.synchronize()
        med = lambda k: float(np.median([s[k] for s in sts[2:]]))
        print(f"{name}{'(light)' if light else ''} {path}: e2e {med('t_e2e_ms'):.3f} kern {med('t_kern_ms'):.3f} "
              f"s1 {med('t_step1_ms'):.3f} s2 {med('t_step2_ms'):.3f} s3 {med('t_step3_ms'):.3f} "
              f"k3 {med('t_step3_kernel_ms'):.3f} c2t {med('t_csr2tile_ms'):.3f} malloc {med('t_malloc_ms'):.3f} "
              f"nnzC {sts[-1]['nnzC']}", flush=True)
    ctx.close()


PATHS = ("fused", "tiles")

if __name__ == "__main__":
    light = "--light" in sys.argv
    for a in sys.argv[1:]:
        if a.startswith("--path="):
            PATHS = tuple(a[7:].split(","))
    for nm in [a for a in sys.argv[1:] if not a.startswith("--")]:
        run(nm, light)
