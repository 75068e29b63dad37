"""Round 4 debug: per-class row-count mismatches of the default route vs the oracle."""
import sys
import numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import _oracle as O
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

def classes(rp, ci, rpb):
    blen = np.diff(rpb).astype(np.int64)
    prod = blen[ci]
    P = np.add.reduceat(np.concatenate([prod, [0]]), rp[:-1]) * (np.diff(rp) > 0)
    k = np.diff(rp).astype(np.int64)
    c = np.full(len(P), 7)
    for cc, (pc, kc) in reversed(list(enumerate([(16, 16), (64, 64), (256, 62), (512, 124), (1024, 248), (2048, 504), (4096, 512)]))):
        c[(P <= pc) & (k <= kc)] = cc
    c[P == 0] = -1
    return c, P

def run(name, A_):
    m, n, rp, ci, vv = A_
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    Cm, st = T.spgemm(A, T.Matrix.alias(A))
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    ref = O.gustavson(oA, O.OMat.alias(oA)).csr()
    got = Cm.csr()
    cg, cr = np.diff(got[2].astype(np.int64)), np.diff(ref[2].astype(np.int64))
    c, P = classes(rp, ci, rp)
    print(name, "path", st["path"], "nnz", got[2][-1], ref[2][-1])
    for cc in range(-1, 8):
        s = c == cc
        bad = (cg[s] != cr[s]).sum()
        print(f"  class {cc}: rows {s.sum()} bad {bad} got {cg[s].sum()} ref {cr[s].sum()}")
    bad = np.nonzero(cg != cr)[0]
    print("  first bad rows", bad[:10], cg[bad[:10]], cr[bad[:10]], P[bad[:10]], c[bad[:10]])
    if len(bad) == 0:
        ok = np.array_equal(got[3], ref[3]) and np.allclose(got[4], ref[4], rtol=1e-10, atol=0)
        print("  cols/vals ok", ok)

run("random", synth.random_csr(3000, 3000, nnz_per_row=6, seed=3))
run("webbase", synth.webbase())
