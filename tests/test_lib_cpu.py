"""CPU-side checks of the product library (no compute call needs a GPU here):
the C ABI library builds for gfx950, loads, exports every symbol include/tsg.h
declares, refuses to run without a device (no CPU fallback), and its host-only
Matrix-Market reader reproduces mmio_allinone's CSR order (pinned through the
oracle on the reference fixtures)."""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from conftest import FIXTURES
import _oracle as O
from spgemm_amd import _lib
from spgemm_amd import tilespgemm as T


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def test_exports_every_header_symbol(L):
    syms = _lib.header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), f"libtsg.so does not export {s}"


def test_code_object_is_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"gfx90a" not in data and b"gfx942" not in data


def test_status_strings(L):
    assert L.tsg_status_string(0) == b"ok"
    assert b"device" in L.tsg_status_string(-5)
    assert L.tsg_version().startswith(b"tsg-mi355x")


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present")
def test_fails_loudly_without_device(L):
    A = T.Matrix.from_csr(2, 2, [0, 1, 2], [0, 1], [1.0, 2.0])
    with pytest.raises(_lib.TsgError) as ei:
        T.csr2tile_row_major(A, 16, 16)
    assert ei.value.rc == -5
    with pytest.raises(_lib.TsgError):
        T.spgemm(A, T.Matrix.alias(A))


def test_invalid_tile_size_rejected(L):
    A = T.Matrix.from_csr(2, 2, [0, 1, 2], [0, 1], [1.0, 2.0])
    for tm, tn in [(8, 16), (16, 24), (0, 16), (128, 16)]:
        with pytest.raises(_lib.TsgError) as ei:
            T.csr2tile_row_major(A, tm, tn)
        assert ei.value.rc == -1


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(FIXTURES, "*.mtx"))),
                         ids=lambda p: os.path.basename(p))
def test_mmio_reader_matches_oracle(L, path):
    A = T.mmio_allinone(path)
    T.values_pos_mod10(A)
    ref = O.OMat.load(path)
    m, n, rp, ci, vv = A.csr()
    om, on, orp, oci, ovv = ref.csr()
    assert (m, n) == (om, on)
    assert A.s.isSymmetric == ref.s.isSymmetric
    np.testing.assert_array_equal(rp, orp)
    np.testing.assert_array_equal(ci, oci)
    np.testing.assert_array_equal(vv, ovv)


@pytest.mark.parametrize("kind", ["real general", "pattern symmetric", "integer general"])
def test_mmio_reader_parallel_chunks_match_oracle(L, tmp_path, kind):
    """A file large enough for the multi-threaded parse (>= 4 MiB per chunk):
    same CSR order and values as the oracle's mmio_allinone restatement."""
    rng = np.random.default_rng(5)
    m = 60000
    nz = 900000
    i = rng.integers(1, m + 1, nz)
    j = rng.integers(1, m + 1, nz)
    if "symmetric" in kind:
        i, j = np.maximum(i, j), np.minimum(i, j)
    path = tmp_path / "big.mtx"
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {kind}\n% generated\n{m} {m} {nz}\n")
        if kind.startswith("pattern"):
            np.savetxt(f, np.stack([i, j], 1), fmt="%d")
        elif kind.startswith("integer"):
            np.savetxt(f, np.stack([i, j, rng.integers(-9, 10, nz)], 1), fmt="%d")
        else:
            np.savetxt(f, np.stack([i, j, rng.standard_normal(nz)], 1), fmt="%d %d %.17g")
    assert os.path.getsize(path) > (8 << 20)
    A = T.mmio_allinone(str(path))
    ref = O.OMat.load(str(path), pos_mod10=False)  # file values, not k % 10
    m1, n1, rp, ci, vv = A.csr()
    m2, n2, orp, oci, ovv = ref.csr()
    assert (m1, n1) == (m2, n2)
    np.testing.assert_array_equal(rp, orp)
    np.testing.assert_array_equal(ci, oci)
    np.testing.assert_array_equal(vv, ovv)


def test_mmio_csr_cache_roundtrip(L, tmp_path, monkeypatch):
    path = os.path.join(FIXTURES, "x_powerlaw_400.mtx")
    monkeypatch.setenv("TSG_CSR_CACHE_DIR", str(tmp_path))
    first = T.mmio_allinone(path).csr()
    files = list(tmp_path.glob("x_powerlaw_400.mtx.*.tsgcsr"))
    assert len(files) == 1
    second = T.mmio_allinone(path).csr()  # served from the cache
    for a, b in zip(first, second):
        np.testing.assert_array_equal(a, b)
    monkeypatch.delenv("TSG_CSR_CACHE_DIR")
    for a, b in zip(first, T.mmio_allinone(path).csr()):
        np.testing.assert_array_equal(a, b)


def test_mmio_reader_errors(L, tmp_path):
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    with pytest.raises(_lib.TsgError) as ei:
        T.mmio_allinone(str(bad))
    assert ei.value.rc == -6
    with pytest.raises(_lib.TsgError) as ei:
        T.mmio_allinone(str(tmp_path / "missing.mtx"))
    assert ei.value.rc == -7
    oob = tmp_path / "oob.mtx"
    oob.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n")
    with pytest.raises(_lib.TsgError):
        T.mmio_allinone(str(oob))


CLI = os.path.join(os.path.dirname(_lib.LIB_PATH), "..", "bin", "test")


def _cli(*args, env=None):
    import subprocess
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=120, env=env)


def test_cli_usage_exits_zero():
    # fewer than 7 args: usage line and exit 0 (src/main.cu:16-20)
    r = _cli()
    assert r.returncode == 0 and "./test -d 0 -aat 0 matrix.mtx" in r.stdout


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present")
def test_cli_fails_loudly_without_device(tmp_path):
    r = _cli("-d", "0", "-aat", "0", os.path.join(FIXTURES, "banded_36x36.mtx"), "16", "16",
             env=dict(os.environ, TSG_DATA_DIR=str(tmp_path)))
    assert r.returncode != 0 and "no HIP device" in r.stderr
