import sys, time, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import _oracle as O
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T
def chk(name, m, n, rp, ci, vv, aat=False):
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    if aat: B, oB = T.transpose(A), O.transpose(oA)
    else: B, oB = T.Matrix.alias(A), O.OMat.alias(oA)
    t = time.time(); Cm, st = T.spgemm(A, B); t = time.time() - t
    got = Cm.csr(); ref = O.gustavson(oA, oB).csr()
    ok = np.array_equal(got[2], ref[2]) and np.array_equal(got[3], ref[3]) and np.allclose(got[4], ref[4], rtol=1e-10, atol=0)
    print(f"{name}: ok={ok} nnzC={st['nnzC']} ref={len(ref[3])} kern={st['t_step3_kernel_ms']:.3f} s1={st['t_step1_ms']:.3f} e2e={st['t_e2e_ms']:.3f} segs={st['numblkC']}", flush=True)
    if not ok:
        bad = np.nonzero(got[2] != ref[2])[0] if len(got[2]) == len(ref[2]) else []
        print("  rowptr mismatch rows", bad[:10], flush=True)
        sys.exit(1)
which = sys.argv[1:]
if 'small' in which:
    chk('rand300', *synth.random_csr(300, 300, density=0.02, seed=1))
    chk('rand1', *synth.random_csr(1, 1, density=1.0, seed=1))
    chk('empty', 40, 40, np.zeros(41, np.int32), np.zeros(0, np.int32), np.zeros(0))
    chk('rand2048', *synth.random_csr(2048, 2048, density=0.002, seed=3))
    chk('rect_aat', *synth.random_csr(700, 2500, density=0.004, seed=23), aat=True)
    chk('dense600', *synth.random_csr(600, 600, density=0.2, seed=22))
if 'big' in which:
    chk('mawi3e-4', *synth.mawi(scale=3e-4))
    for g in ['mc2depi', 'webbase', 'cant']:
        chk(g, *synth.GENERATORS[g](), aat=(g == 'mc2depi'))
print("done")
