"""Build tests/golden/ref/*.npz from the reference's OWN host code.

The reference's host path (mmio_allinone, csr2tile_row_major/col_major,
spgemm_spa) is compiled in place from /root/reference/src by
`make -C oracle ref` into oracle/_ref/ref_driver (see oracle/ref_driver.cpp).
This script runs it on every fixture (the reference's UnitTest/CSR2TILE .mtx
files, copied here as data, plus tests/golden/fixtures/x_*.mtx from
gen_extra_mtx.py) for C = A*A and C = A*A^T at several tile sizes and freezes
the outputs.  Only this container has /root/reference; the GPU box and the CPU
test suite read the frozen .npz files.

Run:  python tests/golden/make_golden.py
"""
import glob
import os
import shutil
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
FIX = os.path.join(HERE, "fixtures")
OUT = os.path.join(HERE, "ref")
REF_UNITTEST = "/root/reference/UnitTest/CSR2TILE"
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")
TILES = [(16, 16), (32, 16), (32, 32)]
# the remaining reference tile sides (16 | t <= 64), on a subset of fixtures
TILES_EXTRA = [(48, 16), (16, 48), (48, 48), (64, 64), (64, 16)]
EXTRA_FIXTURES = ("x_powerlaw_400", "x_banded_500", "x_rect_50x130", "x_dense_48", "random_0.1_36x36")

_DT = {"i": np.int32, "h": np.uint16, "d": np.float64, "q": np.int64}


def read_records(path):
    out = {}
    with open(path, "rb") as f:
        buf = f.read()
    off = 0
    while off < len(buf):
        (nl,) = struct.unpack_from("<I", buf, off)
        off += 4
        name = buf[off:off + nl].decode()
        off += nl
        code = chr(buf[off])
        off += 1
        (cnt,) = struct.unpack_from("<Q", buf, off)
        off += 8
        dt = np.dtype(_DT[code])
        arr = np.frombuffer(buf, dtype=dt, count=cnt, offset=off).copy()
        off += cnt * dt.itemsize
        out[name] = arr[0] if code == "q" else arr
    return out


def banner(path):
    with open(path) as f:
        toks = f.readline().lower().split()
    with open(path) as f:
        for line in f:
            if not line.startswith("%"):
                m, n, _ = map(int, line.split())
                break
    return toks, m, n


def main():
    os.makedirs(FIX, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    if os.path.isdir(REF_UNITTEST):
        for p in glob.glob(os.path.join(REF_UNITTEST, "*.mtx")):
            shutil.copy(p, FIX)
    subprocess.check_call([sys.executable, os.path.join(HERE, "gen_extra_mtx.py")])
    subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "ref"])
    n_cases = 0
    for mtx in sorted(glob.glob(os.path.join(FIX, "*.mtx"))):
        name = os.path.basename(mtx)[:-4]
        toks, m, n = banner(mtx)
        sym = toks[4] in ("symmetric", "hermitian")
        for aat in (0, 1):
            if aat == 0 and m != n:
                continue  # src/main.cu:102-106
            if aat == 1 and m == n and sym:
                continue  # src/main.cu:120-124
            for tm, tn in TILES + (TILES_EXTRA if name in EXTRA_FIXTURES else []):
                tmp = os.path.join(OUT, "_tmp.bin")
                subprocess.check_call([DRIVER, mtx, str(aat), str(tm), str(tn), tmp],
                                      stdout=subprocess.DEVNULL)
                rec = read_records(tmp)
                os.remove(tmp)
                np.savez_compressed(os.path.join(OUT, f"{name}_aat{aat}_{tm}x{tn}.npz"),
                                    **{k.replace(".", "__"): np.asarray(v) for k, v in rec.items()})
                n_cases += 1
    print(f"wrote {n_cases} golden cases to {OUT}")


if __name__ == "__main__":
    main()
