"""Warm timing of the drop-in tiled path (tsg_tilespgemm: tiles in, the
reference's tiled C out) on a stand-in; usage: python tools/tiled_time.py webbase [reps] [tile]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

name = sys.argv[1] if len(sys.argv) > 1 else "webbase"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
tm = int(sys.argv[3]) if len(sys.argv) > 3 else 16
os.environ["TSG_QUIET"] = "1"
m, n, rp, ci, vv = synth.GENERATORS[name]()
A = T.Matrix.from_csr(m, n, rp, ci, vv)
B = T.transpose(A) if name == "mc2depi" else T.Matrix.from_csr(m, n, rp, ci, vv)
T.csr2tile_row_major(A, tm, tm)
T.csr2tile_col_major(B, tm, tm)
runs = []
for i in range(reps + 1):
    Cm, info = T.tilespgemm(A, B, tm, tm)
    runs.append(info)
    nt = Cm.s.numtile
    del Cm
med = lambda k: float(np.median([r[k] for r in runs[1:]]))
print(f"{name} tile {tm}: t_tile {med('time_tile'):.3f} ms  s1 {med('time_step1'):.3f} s2 {med('time_step2'):.3f} "
      f"s3 {med('time_step3'):.3f} malloc {med('time_malloc'):.3f}  numblkC {nt} nnzC {runs[-1]['nnzC']}", flush=True)
