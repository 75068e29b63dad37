"""GPU parity: every stage of the HIP path against the oracle, through the C ABI.

Bar (north_star): C's nnz, row pointers, column pattern and the tiled layouts
bit-exact; fp64 values within rtol 1e-10 (here exact in practice: with the
reference's value[k] = k % 10 every product and sum is a small integer).
The structural oracle is pinned to the reference's own host code by
tests/test_oracle.py; goldens in tests/golden/ref come from that code.
"""
import ctypes
import os

import numpy as np
import pytest

import _oracle as O
from conftest import FIXTURES, golden_cases
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu
RTOL = 1e-10
TILE_KEYS = ("tile_ptr", "tile_columnidx", "tile_nnz", "tile_csr_Ptr", "tile_csr_Col", "tile_csr_Value", "mask")
# C's masks are device-internal in the reference too (never copied back, src/tilespgemm-cuda.h:2749-2775)
C_KEYS = TILE_KEYS[:-1]
SUPPORTED = {(16, 16), (32, 16), (32, 32), (48, 16), (16, 48), (48, 48), (64, 64), (64, 16)}  # all golden sizes


def g(npz, key):
    return npz[key.replace(".", "__")]


def both(path, aat):
    """(product A, product B, oracle A, oracle B) for a fixture."""
    A = T.mmio_allinone(path)
    T.values_pos_mod10(A)
    B = T.transpose(A) if aat else T.Matrix.alias(A)
    oA = O.OMat.load(path)
    oB = O.transpose(oA) if aat else O.OMat.alias(oA)
    return A, B, oA, oB


def assert_csr_equal(got, ref, values=True):
    gm, gn, grp, gci, gvv = got
    rm, rn, rrp, rci, rvv = ref
    assert (gm, gn) == (rm, rn)
    np.testing.assert_array_equal(grp, rrp)
    np.testing.assert_array_equal(gci, rci)
    if values:
        np.testing.assert_allclose(gvv, rvv, rtol=RTOL, atol=0)


CASES = [c for c in golden_cases() if (c.values[3], c.values[4]) in SUPPORTED]


@pytest.mark.parametrize("path,name,aat,tm,tn", CASES)
def test_pipeline_stages_vs_reference_goldens(path, name, aat, tm, tn):
    ref = np.load(path)
    A, B, oA, oB = both(os.path.join(FIXTURES, name + ".mtx"), aat)
    # GPU transpose (-aat 1) vs the reference's matrix_transposition
    _, _, brp, bci, bvv = B.csr()
    np.testing.assert_array_equal(brp, g(ref, "B.rowpointer"))
    np.testing.assert_array_equal(bci, g(ref, "B.columnindex"))
    np.testing.assert_array_equal(bvv, g(ref, "B.value"))
    assert T.nnzcub(A, B) == int(g(ref, "nnzCub"))
    # GPU csr2tile vs the reference's csr2tile (bit-exact, every field)
    T.csr2tile_row_major(A, tm, tn)
    T.csr2tile_col_major(B, tm, tn)
    at, bt = A.tiles(tm, tn // 16), B.tiles(tn, tm // 16, csc=True)
    for k in ("tilem", "tilen", "numtile"):
        assert at[k] == int(g(ref, "At." + k)), k
        assert bt[k] == int(g(ref, "Bt." + k)), k
    for k in TILE_KEYS:
        np.testing.assert_array_equal(at[k], g(ref, "At." + k), err_msg="A " + k)
        np.testing.assert_array_equal(bt[k], g(ref, "Bt." + k), err_msg="B " + k)
    np.testing.assert_array_equal(bt["csc_tile_ptr"], g(ref, "Bt.csc_tile_ptr"))
    np.testing.assert_array_equal(bt["csc_tile_rowidx"], g(ref, "Bt.csc_tile_rowidx"))
    # GPU steps 1-3 vs oracle tiled C (every field) and the reference step-1 structure
    Cm, info = T.tilespgemm(A, B, tm, tn, nnzCub=int(g(ref, "nnzCub")))
    O.csr2tile_row_major(oA, tm, tn)
    O.csr2tile_col_major(oB, tm, tn)
    oC = O.tilespgemm(oA, oB, tm, tn)
    ct, oct_ = Cm.tiles(tm, tm // 16), O.c_tiles(oC, tm)
    np.testing.assert_array_equal(ct["tile_ptr"], g(ref, "Ct.tile_ptr"))
    np.testing.assert_array_equal(ct["tile_columnidx"], g(ref, "Ct.tile_columnidx"))
    assert ct["numtile"] == oct_["numtile"]
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], oct_[k], err_msg="C " + k)
    assert info["nnzC"] == oC.s.nnz
    # GPU tile2csr vs the reference SPA pattern + oracle values
    T.tile2csr(Cm, tm, tm)
    O.tile2csr(oC, tm, tm)
    got = Cm.csr()
    np.testing.assert_array_equal(got[2], g(ref, "C.rowpointer"))
    np.testing.assert_array_equal(got[3], g(ref, "C.columnindex"))
    assert_csr_equal(got, oC.csr())


@pytest.mark.parametrize("path,name,aat,tm,tn", CASES)
def test_one_shot_spgemm_vs_oracle(path, name, aat, tm, tn):
    A, B, oA, oB = both(os.path.join(FIXTURES, name + ".mtx"), aat)
    Cm, st = T.spgemm(A, B, tm, tn)
    ref = O.gustavson(oA, oB)
    assert_csr_equal(Cm.csr(), ref.csr())
    assert st["nnzC"] == ref.s.nnz


def _synthetic_cases():
    out = []
    for (m, n, d, uns, dup) in [(1, 1, 1.0, False, False), (17, 17, 0.2, False, False),
                                (300, 300, 0.02, False, False), (1000, 1000, 0.004, True, False),
                                (999, 999, 0.01, False, True), (2048, 2048, 0.002, True, True),
                                (513, 513, 0.3, False, False)]:
        out.append(pytest.param(m, n, d, uns, dup, id=f"rand{m}x{n}_d{d}_u{int(uns)}_dup{int(dup)}"))
    return out


@pytest.mark.parametrize("m,n,density,unsorted,dups", _synthetic_cases())
def test_random_matrices_tiled_and_csr(m, n, density, unsorted, dups):
    mm, nn, rp, ci, vv = synth.random_csr(m, n, density=density, seed=7 + m, unsorted=unsorted, dups=dups)
    A = T.Matrix.from_csr(mm, nn, rp, ci, vv)
    B = T.Matrix.alias(A)
    oA = O.OMat.from_csr(mm, nn, rp, ci, vv)
    oB = O.OMat.alias(oA)
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    O.csr2tile_row_major(oA, 16, 16)
    O.csr2tile_col_major(oB, 16, 16)
    at, oat = A.tiles(16, 1), oA.tiles(16, 1)
    bt, obt = B.tiles(16, 1, csc=True), oB.tiles(16, 1, csc=True)
    for k in TILE_KEYS:
        np.testing.assert_array_equal(at[k], oat[k], err_msg="A " + k)
        np.testing.assert_array_equal(bt[k], obt[k], err_msg="B " + k)
    Cm, _ = T.tilespgemm(A, B, 16, 16)
    oC = O.tilespgemm(oA, oB, 16, 16)
    ct, oct_ = Cm.tiles(16, 1), O.c_tiles(oC, 16)
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], oct_[k], err_msg="C " + k)
    T.tile2csr(Cm, 16, 16)
    ref = O.gustavson(oA, oB)
    assert_csr_equal(Cm.csr(), ref.csr())


def test_aat_rectangular_and_empty():
    # A*A^T of a wide matrix with empty rows, and an all-empty matrix
    mm, nn, rp, ci, vv = synth.random_csr(130, 777, density=0.01, seed=3)
    A = T.Matrix.from_csr(mm, nn, rp, ci, vv)
    B = T.transpose(A)
    oA = O.OMat.from_csr(mm, nn, rp, ci, vv)
    oB = O.transpose(oA)
    assert_csr_equal(B.csr(), oB.csr())
    Cm, _ = T.spgemm(A, B)
    assert_csr_equal(Cm.csr(), O.gustavson(oA, oB).csr())
    E = T.Matrix.from_csr(40, 40, np.zeros(41, np.int32), np.zeros(0, np.int32), np.zeros(0))
    Ce, st = T.spgemm(E, T.Matrix.alias(E))
    m, n, rp, ci, vv = Ce.csr()
    assert (m, n) == (40, 40) and rp.sum() == 0 and len(ci) == 0 and st["nnzC"] == 0


def test_mawi_star_small_scale_vs_oracle():
    """mawi stand-in at 3e-4 scale (68 K nodes, hub degree 3,000): the hub's
    neighbours each receive the hub's whole row in C."""
    m, n, rp, ci, vv = synth.mawi(scale=3e-4)
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    Cm, st = T.spgemm(A, T.Matrix.alias(A))
    ref = O.gustavson(oA, O.OMat.alias(oA))
    assert_csr_equal(Cm.csr(), ref.csr())
    assert st["nnzC"] == ref.s.nnz


@pytest.mark.parametrize("path", [None, "tiles"])
@pytest.mark.parametrize("name", ["cant", "mc2depi", "webbase"])
def test_full_size_synthetic_vs_oracle(name, path, monkeypatch):
    """BASELINE configs at full size (synthetic stand-ins): pattern bit-exact,
    values exact, against the numeric Gustavson oracle -- on the default route
    (cant: banded path, mc2depi and webbase: row-merge path) and forced
    through the staged tile pipeline."""
    if path:
        monkeypatch.setenv("TSG_PATH", path)
    m, n, rp, ci, vv = synth.GENERATORS[name]()
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    if name == "mc2depi":  # config 3 is C = A*A^T
        B = T.transpose(A)
        oA = O.OMat.from_csr(m, n, rp, ci, vv)
        oB = O.transpose(oA)
    else:
        B = T.Matrix.alias(A)
        oA = O.OMat.from_csr(m, n, rp, ci, vv)
        oB = O.OMat.alias(oA)
    Cm, st = T.spgemm(A, B)
    ref = O.gustavson(oA, oB)
    assert_csr_equal(Cm.csr(), ref.csr())
    assert st["nnzC"] == ref.s.nnz
    # the staged pipeline's A/B tile counts (wave hash sets + bitmap fallback for
    # tile rows over 256 entries) equal the oracle csr2tile's numtile (the fused,
    # banded and row-merge paths build no A/B tiles and report -1)
    if path is None:  # the default routes
        assert st["path"] == {"cant": T.PATH_BAND, "mc2depi": T.PATH_ROWS, "webbase": T.PATH_ROWS}[name]
        assert st["numtileA"] == -1
        return
    assert st["path"] == T.PATH_TILES
    tA = O.OMat.from_csr(m, n, rp, ci, vv)
    O.csr2tile_row_major(tA, 16, 16)
    assert st["numtileA"] == tA.s.numtile
    tB = O.transpose(tA) if name == "mc2depi" else O.OMat.from_csr(m, n, rp, ci, vv)
    O.csr2tile_col_major(tB, 16, 16)
    assert st["numtileB"] == tB.s.numtile


def test_device_api_matches_host_api():
    import torch
    from spgemm_amd.device import Context, DeviceCSR
    m, n, rp, ci, vv = synth.random_csr(3000, 3000, density=0.003, seed=11)
    ctx = Context(0)
    dA = DeviceCSR.from_host(m, n, rp, ci, vv)
    c, st = ctx.spgemm(dA, dA)
    got = ctx.to_host(c)
    torch.cuda.synchronize()
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    assert_csr_equal(got, O.gustavson(oA, O.OMat.alias(oA)).csr())
    # repeated calls reuse the cached pool and stay exact
    for _ in range(3):
        ctx.reset()
        c2, _ = ctx.spgemm(dA, dA)
        assert_csr_equal(ctx.to_host(c2), got)
    # B's sortedness checked once, then the calls that skip it
    # (tsg_dev_csr_rows_sorted, tsg_dev_spgemm_sorted_b): the same C
    assert ctx.rows_sorted(dA)
    ctx.reset()
    c3, st3 = ctx.spgemm(dA, dA, b_sorted=True)
    assert_csr_equal(ctx.to_host(c3), got)
    assert st3["path"] == st["path"]
    # an unsorted B is reported as such, and the checking call routes it to the
    # staged tile pipeline with the right C
    mu, nu_, rpu, ciu, vvu = synth.random_csr(3000, 3000, density=0.003, seed=12, unsorted=True)
    dU = DeviceCSR.from_host(mu, nu_, rpu, ciu, vvu)
    assert not ctx.rows_sorted(dU)
    ctx.reset()
    c4, st4 = ctx.spgemm(dA, dU)
    oU = O.OMat.from_csr(mu, nu_, rpu, ciu, vvu)
    assert_csr_equal(ctx.to_host(c4), O.gustavson(oA, oU).csr())
    assert st4["path"] == T.PATH_TILES
    ctx.close()


@pytest.mark.parametrize("aat,tiles", [(0, ("16", "16")), (1, ("16", "16")), (0, ("32", "32")), (0, ("64", "16"))])
def test_cli_reports_reference_lines(aat, tiles, tmp_path):
    """./test -d 0 -aat X <mtx> 16 16 prints the reference's key lines with the
    oracle's nnzCub / nnzC and writes the CSV (creating the directory)."""
    import re
    import subprocess
    cli = os.path.join(os.path.dirname(T._lib.LIB_PATH), "..", "bin", "test")
    path = os.path.join(FIXTURES, "banded_36x36.mtx")
    out = tmp_path / "data"
    r = subprocess.run([cli, "-d", "0", "-aat", str(aat), path, *tiles], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, TSG_DATA_DIR=str(out)))
    assert r.returncode == 0, r.stderr
    oA = O.OMat.load(path)
    oB = O.transpose(oA) if aat else O.OMat.alias(oA)
    ref = O.gustavson(oA, oB)
    assert f"SpGEMM nnzCub = {O.nnzcub(oA, oB)}" in r.stdout
    assert re.search(rf"nnzC = {ref.s.nnz}\b", r.stdout), r.stdout
    assert re.search(r"TileSpGEMM runtime is [0-9.]+ ms, gflops = [0-9.]+", r.stdout), r.stdout
    assert any(out.iterdir())


@pytest.mark.parametrize("mode", ["elem", "tile"])
@pytest.mark.parametrize("case", ["rand_sparse", "rand_dense", "banded", "rect_aat", "unsorted"])
def test_step2_modes_match_oracle(mode, case, monkeypatch):
    """Both step-2 variants of the device pipeline (element-streamed masks from
    the CSR operands vs tile-level mask ORs) give the oracle's product; an
    unsorted B falls back to the tile payload path in either mode."""
    monkeypatch.setenv("TSG_STEP2_MODE", mode)
    monkeypatch.setenv("TSG_PATH", "tiles")  # the staged pipeline (the banded input would route elsewhere)
    if case == "rand_sparse":
        m, n, rp, ci, vv = synth.random_csr(5000, 5000, density=0.0008, seed=21)
    elif case == "rand_dense":
        m, n, rp, ci, vv = synth.random_csr(600, 600, density=0.2, seed=22)
    elif case == "banded":
        m, n, rp, ci, vv = synth.cant(dims=(4, 4, 63))
    elif case == "rect_aat":
        m, n, rp, ci, vv = synth.random_csr(700, 2500, density=0.004, seed=23)
    else:
        m, n, rp, ci, vv = synth.random_csr(1500, 1500, density=0.01, seed=24, unsorted=True, dups=True)
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    if case == "rect_aat":
        B, oB = T.transpose(A), O.transpose(oA)
    else:
        B, oB = T.Matrix.alias(A), O.OMat.alias(oA)
    Cm, st = T.spgemm(A, B)
    ref = O.gustavson(oA, oB)
    assert_csr_equal(Cm.csr(), ref.csr())
    assert st["nnzC"] == ref.s.nnz


@pytest.mark.parametrize("tm,tn", [(48, 16), (16, 48), (48, 48), (64, 64), (64, 16), (32, 64)])
@pytest.mark.parametrize("aat", [0, 1])
def test_other_tile_sizes_vs_oracle(tm, tn, aat):
    """Every reference tile size (sides 16..64): csr2tile of A and B, the host
    tilespgemm's C tiles and tile2csr, field by field against the oracle."""
    mm, nn, rp, ci, vv = synth.random_csr(700, 700 if not aat else 420, density=0.01, seed=tm * 7 + tn + aat)
    A = T.Matrix.from_csr(mm, nn, rp, ci, vv)
    oA = O.OMat.from_csr(mm, nn, rp, ci, vv)
    if aat:
        B, oB = T.transpose(A), O.transpose(oA)
    else:
        B, oB = T.Matrix.alias(A), O.OMat.alias(oA)
    T.csr2tile_row_major(A, tm, tn)
    T.csr2tile_col_major(B, tm, tn)
    O.csr2tile_row_major(oA, tm, tn)
    O.csr2tile_col_major(oB, tm, tn)
    at, oat = A.tiles(tm, tn // 16), oA.tiles(tm, tn // 16)
    bt, obt = B.tiles(tn, tm // 16, csc=True), oB.tiles(tn, tm // 16, csc=True)
    for k in TILE_KEYS:
        np.testing.assert_array_equal(at[k], oat[k], err_msg="A " + k)
        np.testing.assert_array_equal(bt[k], obt[k], err_msg="B " + k)
    Cm, _ = T.tilespgemm(A, B, tm, tn)
    oC = O.tilespgemm(oA, oB, tm, tn)
    ct, oct_ = Cm.tiles(tm, tm // 16), O.c_tiles(oC, tm)
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], oct_[k], err_msg="C " + k)
    T.tile2csr(Cm, tm, tm)
    assert_csr_equal(Cm.csr(), O.gustavson(oA, oB).csr())


@pytest.mark.parametrize("tm,tn", [(32, 32), (64, 64), (48, 16), (64, 32)])
def test_dense_accumulator_tiles(tm, tn):
    """Tiles of C with more than 512 nonzeros (possible from 32x32 up) take the
    dense per-wave LDS accumulator -- the reference's dns/ful bins
    (src/tilespgemm-cuda.h:1954-2218) -- natively at tm x tm; every C tile
    field against the oracle, and C's CSR against Gustavson."""
    mm, nn, rp, ci, vv = synth.random_csr(300, 300, density=0.35, seed=tm + tn)
    A = T.Matrix.from_csr(mm, nn, rp, ci, vv)
    B = T.Matrix.alias(A)
    oA = O.OMat.from_csr(mm, nn, rp, ci, vv)
    oB = O.OMat.alias(oA)
    T.csr2tile_row_major(A, tm, tn)
    T.csr2tile_col_major(B, tm, tn)
    O.csr2tile_row_major(oA, tm, tn)
    O.csr2tile_col_major(oB, tm, tn)
    Cm, info = T.tilespgemm(A, B, tm, tn)
    oC = O.tilespgemm(oA, oB, tm, tn)
    ct, oct_ = Cm.tiles(tm, tm // 16), O.c_tiles(oC, tm)
    assert np.diff(ct["tile_nnz"]).max() > 512  # the dense accumulator ran
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], oct_[k], err_msg="C " + k)
    assert info["time_step2"] > 0 and info["time_step3"] > 0
    T.tile2csr(Cm, tm, tm)
    assert_csr_equal(Cm.csr(), O.gustavson(oA, oB).csr())


CASES16 = [c for c in CASES if (c.values[3], c.values[4]) == (16, 16)]


@pytest.mark.parametrize("path,name,aat,tm,tn", CASES16)
def test_tiled_api_csr_streaming_and_tile_payload_agree(path, name, aat, tm, tn, monkeypatch):
    """tsg_tilespgemm at 16x16 streams element products from the SMatrix's CSR
    when B's rows are sorted (TSG_TILED_CSR unset) and reads the tile payloads
    otherwise (TSG_TILED_CSR=0); both must give the reference's tiled C, every
    field bit-exact.  A sorted-row copy of the fixture makes the CSR path run
    for A^2 as well (the file's in-row order is kept in the first pass)."""
    ref = np.load(path)
    for srt in (False, True):
        A, B, oA, oB = both(os.path.join(FIXTURES, name + ".mtx"), aat)
        if srt:
            m, n, rp, ci, vv = A.csr()
            order = np.concatenate([rp[i] + np.argsort(ci[rp[i]:rp[i + 1]], kind="stable") for i in range(m)]
                                   ).astype(np.int64) if len(ci) else np.zeros(0, np.int64)
            A = T.Matrix.from_csr(m, n, rp, ci[order], vv[order])
            B = T.transpose(A) if aat else T.Matrix.alias(A)
            oA = O.OMat.from_csr(m, n, rp, ci[order], vv[order])
            oB = O.transpose(oA) if aat else O.OMat.alias(oA)
        T.csr2tile_row_major(A, tm, tn)
        T.csr2tile_col_major(B, tm, tn)
        O.csr2tile_row_major(oA, tm, tn)
        O.csr2tile_col_major(oB, tm, tn)
        oct_ = O.c_tiles(O.tilespgemm(oA, oB, tm, tn), tm)
        for mode in (None, "0"):
            if mode is None:
                monkeypatch.delenv("TSG_TILED_CSR", raising=False)
            else:
                monkeypatch.setenv("TSG_TILED_CSR", mode)
            Cm, info = T.tilespgemm(A, B, tm, tn, nnzCub=int(g(ref, "nnzCub")))
            ct = Cm.tiles(tm, tm // 16)
            np.testing.assert_array_equal(ct["tile_ptr"], g(ref, "Ct.tile_ptr"))
            for k in C_KEYS:
                np.testing.assert_array_equal(ct[k], oct_[k], err_msg=f"C {k} (sorted={srt}, mode={mode})")
            del Cm


def test_tiled_api_csr_streaming_real_values():
    """The tiled host API on the CSR-streaming path with real fp64 values: C's
    tile values within 1e-10 of the oracle's magnitude sums (pattern exact)."""
    m, n, rp, ci, _ = synth.random_csr(1500, 1500, density=0.01, seed=41)
    vv = np.random.default_rng(3).uniform(-1, 1, len(ci))
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    B = T.Matrix.alias(A)
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    Cm, _ = T.tilespgemm(A, B, 16, 16)
    T.tile2csr(Cm, 16, 16)
    got = Cm.csr()
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    ref = O.gustavson(oA, O.OMat.alias(oA)).csr()
    oM = O.OMat.from_csr(m, n, rp, ci, np.abs(vv))
    mag = O.gustavson(oM, O.OMat.alias(oM)).csr()[4]
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    assert np.all(np.abs(got[4] - ref[4]) <= RTOL * mag)


def test_tiled_csr_route_wide_tile_rows_and_empty_tiles():
    """The 16x16 tiled route through the CSR C (tsg_ctiles.hip): one tile row
    spanning ~20 units of <= 992 tiles (B's row 0 reaches 20,000 tile columns),
    several rows of the tile row in the same tiles (multi-row masks and Ptr),
    and step-1 tiles whose element product is empty (A's column 1 selects an
    empty B row inside a tile pair that the tile pattern matches).  Every C
    tile array against the oracle's tiled product, CSR C against Gustavson."""
    nt = 20000
    n = 16 * nt
    rows = {0: [0, 1], 3: [0], 7: [0, 2], 15: [2], 16: [0], 40: [1, 2]}
    m = 48
    rp = np.zeros(m + 1, np.int64)
    for r, cs in rows.items():
        rp[r + 1] = len(cs)
    rp = np.cumsum(rp).astype(np.int32)
    ci = np.concatenate([np.array(rows[r], np.int32) for r in sorted(rows)])
    va = np.arange(1, len(ci) + 1, dtype=np.float64)
    # B (n x n, only rows 0 and 2 non-empty): row 0 hits column 16j + (j % 16) for
    # every tile column j, row 2 every 7th tile column; row 1 is empty
    b0 = 16 * np.arange(nt) + np.arange(nt) % 16
    b2 = 16 * np.arange(0, nt, 7) + 3
    brp = np.zeros(n + 1, np.int64)
    brp[1] = len(b0)
    brp[3] = len(b2)
    brp = np.cumsum(brp).astype(np.int32)
    bci = np.concatenate([b0, b2]).astype(np.int32)
    bvv = (np.arange(len(bci)) % 10 + 1).astype(np.float64)
    A = T.Matrix.from_csr(m, n, rp, ci, va)
    B = T.Matrix.from_csr(n, n, brp, bci, bvv)
    oA = O.OMat.from_csr(m, n, rp, ci, va)
    oB = O.OMat.from_csr(n, n, brp, bci, bvv)
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    O.csr2tile_row_major(oA, 16, 16)
    O.csr2tile_col_major(oB, 16, 16)
    Cm, info = T.tilespgemm(A, B, 16, 16)
    oC = O.tilespgemm(oA, oB, 16, 16)
    ct, oct_ = Cm.tiles(16, 1), O.c_tiles(oC, 16)
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], oct_[k], err_msg="C " + k)
    assert int(ct["tile_ptr"][1]) > 5 * 992  # the first tile row spans several units
    tn = np.diff(ct["tile_nnz"][: len(ct["tile_columnidx"]) + 1])
    assert (tn == 0).any()  # structurally present, numerically empty tiles
    T.tile2csr(Cm, 16, 16)
    assert_csr_equal(Cm.csr(), O.gustavson(oA, oB).csr())


@pytest.mark.parametrize("which", ["A", "B"])
def test_tiled_csr_disagreeing_with_tiles_takes_the_payload_route(which):
    """tsg_tilespgemm's CSR route reads the CSR that the SMatrix carries beside
    its tiles (src/main.cu:261-276 builds both from one CSR).  When that CSR
    disagrees with the tiles -- here A's (or B's) CSR lost its last nonzero
    after csr2tile, so its nnz no longer equals the tiles' tile_nnz[numtile] --
    the call must fall back to the tile payloads: C is the product of the
    TILES, every C tile field equal to the oracle's tiled product of the
    original operands."""
    m, n, rp, ci, vv = synth.random_csr(700, 700, density=0.006, seed=17)
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    B = T.Matrix.from_csr(m, n, rp.copy(), ci.copy(), vv.copy())
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    oB = O.OMat.from_csr(m, n, rp, ci, vv)
    O.csr2tile_row_major(oA, 16, 16)
    O.csr2tile_col_major(oB, 16, 16)
    want = O.c_tiles(O.tilespgemm(oA, oB, 16, 16), 16)
    # the operand's CSR without its last nonzero (row pointers only: the arrays keep
    # their length), swapped in beside the unchanged tiles (whose nnz stays)
    M = A if which == "A" else B
    rp2 = rp.astype(np.int32).copy()
    rp2[-1] -= 1
    ci2, vv2 = ci.astype(np.int32).copy(), vv.copy()
    M._keep += [rp2, ci2, vv2]
    M.s.rowpointer = rp2.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    M.s.columnindex = ci2.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    M.s.value = vv2.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    Cm, _ = T.tilespgemm(A, B, 16, 16)
    ct = Cm.tiles(16, 1)
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], want[k], err_msg=f"C {k} ({which}'s CSR disagrees)")
    T.tile2csr(Cm, 16, 16)
    assert_csr_equal(Cm.csr(), O.gustavson(oA, oB).csr())


def test_tiled_csr_with_other_columns_reruns_on_the_payload_route():
    """A CSR with the tiles' counts but another column (so csr_matches_tiles
    passes): one A entry moved to a column c2 whose B row reaches a C tile
    that step 1's structure (from the tiles) does not hold.  The CSR route
    finds a product outside step 1's tiles and the call reruns on the tile
    payloads: C is the tiles' product, every C tile field equal to the
    oracle's (it used to return TSG_ERR_INVALID)."""
    m, n, rp, ci, vv = synth.random_csr(1200, 1200, density=0.0015, seed=23)
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    B = T.Matrix.from_csr(m, n, rp.copy(), ci.copy(), vv.copy())
    T.csr2tile_row_major(A, 16, 16)
    T.csr2tile_col_major(B, 16, 16)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    oB = O.OMat.from_csr(m, n, rp, ci, vv)
    O.csr2tile_row_major(oA, 16, 16)
    O.csr2tile_col_major(oB, 16, 16)
    want = O.c_tiles(O.tilespgemm(oA, oB, 16, 16), 16)
    # C's tile structure per tile row (step 1's, empty tiles included)
    tp, tc = want["tile_ptr"], want["tile_columnidx"]
    have = [set(tc[tp[i]:tp[i + 1]].tolist()) for i in range(len(tp) - 1)]
    pick = None
    for r in range(m):
        if rp[r + 1] == rp[r]:
            continue
        for c2 in range(n):
            if c2 in ci[rp[r]:rp[r + 1]] or rp[c2 + 1] == rp[c2]:
                continue
            if any(int(j) // 16 not in have[r // 16] for j in ci[rp[c2]:rp[c2 + 1]]):
                pick = (r, c2)
                break
        if pick:
            break
    assert pick, "no column reaching outside C's tiles"
    r, c2 = pick
    ci2 = ci.astype(np.int32).copy()
    ci2[rp[r]] = c2  # (same counts everywhere; A's rows need not stay sorted)
    A._keep += [ci2]
    A.s.columnindex = ci2.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    Cm, _ = T.tilespgemm(A, B, 16, 16)
    ct = Cm.tiles(16, 1)
    for k in C_KEYS:
        np.testing.assert_array_equal(ct[k], want[k], err_msg=f"C {k}")
    T.tile2csr(Cm, 16, 16)
    assert_csr_equal(Cm.csr(), O.gustavson(oA, oB).csr())


@pytest.mark.parametrize("where", ["unreferenced", "referenced", "long_row_tail", "none"])
def test_row_block_checks_only_referenced_b_rows(monkeypatch, where):
    """A row block far smaller than B (nnz(A) * 64 < B's rows: the mawi prefix)
    checks the column order of the B rows A references only
    (dev_rows_sorted_shares_ref).  An out-of-order B row that A never reads
    leaves the row-merge path in place; one that A reads -- a short row, or the
    tail of a row of 10,000 entries (three queued chunks of 4,096 pairs) --
    sends the product to the staged tile pipeline, which re-checks all of B.
    Each C against the oracle."""
    monkeypatch.delenv("TSG_PATH", raising=False)
    rng = np.random.default_rng(71)
    nb, n = 40000, 30000
    brows = [np.sort(rng.choice(n, size=int(rng.integers(1, 12)), replace=False)) for _ in range(nb)]
    brows[7] = np.sort(rng.choice(n, size=10000, replace=False))  # a long row
    bad = {"unreferenced": 12345, "referenced": 3, "long_row_tail": 7, "none": None}[where]
    if bad is not None:
        r = brows[bad]
        if len(r) < 2:
            r = np.array([5, 9])
        r = r.copy()
        k = len(r) - 2 if where == "long_row_tail" else 0
        r[k], r[k + 1] = r[k + 1], r[k]  # two neighbours swapped
        brows[bad] = r
    lens = [len(r) for r in brows]
    brp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    bci = np.concatenate(brows).astype(np.int32)
    bvv = rng.uniform(-1, 1, len(bci))
    arows = [np.array([3, 7, 100 + i]) for i in range(40)]  # rows 3, 7 and 100..139 of B
    arp = np.concatenate([[0], np.cumsum([len(r) for r in arows])]).astype(np.int32)
    aci = np.concatenate(arows).astype(np.int32)
    avv = rng.uniform(-1, 1, len(aci))
    assert len(aci) * 64 < nb
    A = T.Matrix.from_csr(40, nb, arp, aci, avv)
    B = T.Matrix.from_csr(nb, n, brp, bci, bvv)
    Cm, st = T.spgemm(A, B)
    ref = O.gustavson(O.OMat.from_csr(40, nb, arp, aci, avv), O.OMat.from_csr(nb, n, brp, bci, bvv)).csr()
    got = Cm.csr()
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=1e-12)
    expect = T.PATH_TILES if where in ("referenced", "long_row_tail") else T.PATH_ROWS
    assert st["path"] == expect
