"""A/B of the windowed-row kernels' options on the LiveJournal stand-in's
heaviest row block (rows [1883808, 1885408)): one matrix generation, each
option set timed warm in the same process (the options are read per call).
usage: python tools/w_ab.py [reps]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from spgemm_amd import synth
from spgemm_amd import dist as tdist
from spgemm_amd.device import Context, DeviceCSR

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
m, n, rp, ci, vv = synth.rmat()
mb, rpb, cib, vvb = tdist.slice_rows(m, rp, ci, vv, 1883808, 1883808 + 1600)
dA = DeviceCSR.from_host(mb, n, rpb, cib, vvb)
dB = DeviceCSR.from_host(m, n, rp, ci, vv)
ctx = Context(0)
os.environ["TSG_PATH"] = "rows"
cfgs = [("unit 8192", "8192"), ("unit 4096", "4096")]
for rnd in range(2):
    for name, un in cfgs:
        os.environ["TSG_W_UNIT"] = un
        ts = []
        for i in range(reps):
            ctx.reset()
            c, st = ctx.spgemm(dA, dB)
            ts.append(st["t_e2e_ms"])
            del c
        torch.cuda.synchronize()
        print(f"round {rnd} {name}: e2e median {np.median(ts[1:]):.3f} ms  nnzC {st['nnzC']}", flush=True)
ctx.close()
