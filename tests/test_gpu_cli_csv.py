"""The CLI's four result CSVs follow the reference's schemas
(src/main.cu:283-320): same column count, the same integer / `%f` float
kinds per column, the first six columns (file, m, n, nnz, nnzCub, nnzC) equal
to the oracle's values, and one appended row per run.  The reference rows in
tests/golden/csv/*.row (data from /root/reference/data/*.csv) pin the format."""
import os
import re
import subprocess

import pytest

import _oracle as O
from conftest import FIXTURES, GOLDEN
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu
FILES = ("results_tile", "step_runtime", "mem-cost", "preprocessing")
INT = re.compile(r"^-?[0-9]+$")
FLT = re.compile(r"^-?[0-9]+\.[0-9]{6}$")  # printf %f


def kinds(row):
    out = []
    for tok in row.split(",")[1:]:
        out.append("i" if INT.match(tok) else "f" if FLT.match(tok) else "?")
    return out


def ref_row(name):
    return open(os.path.join(GOLDEN, "csv", name + ".row")).read().strip()


def test_reference_rows_parse():
    for f in FILES:
        k = kinds(ref_row(f))
        assert "?" not in k, (f, k)
        assert k[:5] == ["i"] * 5 and all(x == "f" for x in k[5:]), (f, k)


@pytest.mark.parametrize("aat", [0, 1])
def test_cli_csv_schemas(aat, tmp_path):
    cli = os.path.join(os.path.dirname(T._lib.LIB_PATH), "..", "bin", "test")
    path = os.path.join(FIXTURES, "random_0.1_36x36.mtx")
    out = tmp_path / "data"
    env = dict(os.environ, TSG_DATA_DIR=str(out))
    for run in range(2):  # rows are appended, one per run
        r = subprocess.run([cli, "-d", "0", "-aat", str(aat), path, "16", "16"], capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stderr
    oA = O.OMat.load(path)
    oB = O.transpose(oA) if aat else O.OMat.alias(oA)
    ref = O.gustavson(oA, oB)
    want_head = [path, str(oA.s.m), str(oA.s.n), str(oA.s.nnz), str(O.nnzcub(oA, oB)), str(ref.s.nnz)]
    for f in FILES:
        rows = (out / (f + ".csv")).read_text().strip().splitlines()
        assert len(rows) == 2, (f, rows)
        rr = ref_row(f)
        for row in rows:
            assert len(row.split(",")) == len(rr.split(",")), (f, row, rr)
            assert kinds(row) == kinds(rr), (f, row, rr)
            assert row.split(",")[:6] == want_head, (f, row)
            comp = float(row.split(",")[6])
            assert abs(comp - O.nnzcub(oA, oB) / ref.s.nnz) < 1e-5
