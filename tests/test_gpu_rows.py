"""The row-merge path (spgemm_amd/csrc/tsg_rows.hip): rows binned by element
products (and A entries) into eight classes -- S16 / S64 (<= 16 / 64
products: ranks by counting in 16 or 64 lanes), M0..M4 (<= 256 / 512 /
1,024 / 2,048 / 4,096 products and <= 62 / 124 / 248 / 504 / 512 entries:
bitonic sorts of packed (column, position) keys in registers and LDS, or
merge-path rounds when the row's column span is too wide for packed keys) and
H (longer rows or more entries: an LDS column bitmap per window of 1,048,576
columns; rows of one window and <= 2,048 entries walk their products once --
registers, then scratch past 16,384 -- and take columns and values through the
bitmap's LDS by rank; other rows walk twice with f64 atomics for the values;
hub rows past 65,536 products and rows past the one-walk kernel's runs or
span: the windowed kernels -- (row, column window) units, products bucketed
per unit, an LDS bitmap per unit, values added in LDS -- or, for hub rows that
one run dominates, the dominant-run kernels).  TSG_PATH=rows forces the path.  Pattern
bit-exact, values within 1e-10 relative, against the oracle (the reference's
semantics: steps 1-3 + tile2csr, tilespgemm-cuda.h:279-2218)."""
import numpy as np
import pytest

import _oracle as O
from spgemm_amd import synth
from spgemm_amd import tilespgemm as T

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def rows_path(monkeypatch):
    monkeypatch.setenv("TSG_PATH", "rows")


def _csr(m, n, rows):
    """CSR from a list of per-row column arrays (kept in the given order)"""
    lens = [len(c) for c in rows]
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = (np.concatenate(rows) if sum(lens) else np.zeros(0)).astype(np.int32)
    vv = (np.arange(len(ci)) % 10).astype(np.float64)
    return m, n, rp, ci, vv


def _check(A_, B_=None, aat=False, real=False, seed=0, path=None):
    m, n, rp, ci, vv = A_
    if real:
        vv = np.random.default_rng(seed).uniform(-1, 1, len(ci))
    A = T.Matrix.from_csr(m, n, rp, ci, vv)
    oA = O.OMat.from_csr(m, n, rp, ci, vv)
    if aat:
        B, oB = T.transpose(A), O.transpose(oA)
    elif B_ is None:
        B, oB = T.Matrix.alias(A), O.OMat.alias(oA)
    else:
        bm, bn, brp, bci, bvv = B_
        if real:
            bvv = np.random.default_rng(seed + 1).uniform(-1, 1, len(bci))
        B, oB = T.Matrix.from_csr(bm, bn, brp, bci, bvv), O.OMat.from_csr(bm, bn, brp, bci, bvv)
    Cm, st = T.spgemm(A, B)
    got, ref = Cm.csr(), O.gustavson(oA, oB).csr()
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    if real:
        oM = O.OMat.from_csr(m, n, rp, ci, np.abs(vv))
        oMb = O.transpose(oM) if aat else (O.OMat.alias(oM) if B_ is None else
                                           O.OMat.from_csr(bm, bn, brp, bci, np.abs(bvv)))
        mag = O.gustavson(oM, oMb).csr()[4]
        assert np.all(np.abs(got[4] - ref[4]) <= 1e-10 * mag)
    else:
        np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=0)
    assert st["nnzC"] == len(ref[3])
    if path is None:
        assert st["path"] == T.PATH_ROWS and st["numblkC"] == -1 and st["numtileA"] == -1
    else:
        assert st["path"] == path
    return st


# (products, A entries) caps of the classes S16, S64, M0..M4 (tsg_rows.hip
# row_class); longer rows are class H
CAPS = [(16, 16), (64, 64), (256, 62), (512, 124), (1024, 248), (2048, 504), (4096, 512)]
H = len(CAPS)
M3, M4 = H - 2, H - 1


def _classes(m, n, rp, ci, rpB):
    """per row: (products, runs) -> class as tsg_rows.hip bins them (-1: no products)"""
    blen = np.diff(rpB.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])
    P = cum[rp[1:]] - cum[rp[:-1]]
    k = np.diff(rp)
    c = np.full(m, -1)
    c[(P > 0)] = H
    for i in range(len(CAPS) - 1, -1, -1):
        c[(P > 0) & (P <= CAPS[i][0]) & (k <= CAPS[i][1])] = i
    return c


@pytest.mark.parametrize("name", ["webbase", "cant", "mc2depi"])
def test_rows_full_size_synthetic(name):
    m, n, rp, ci, vv = synth.GENERATORS[name]()
    cls = _classes(m, n, rp, ci, rp)
    if name == "webbase":  # every class is populated
        assert all((cls == c).any() for c in range(H + 1))
    _check((m, n, rp, ci, vv), aat=name == "mc2depi")


def test_rows_webbase_real_values():
    _check(synth.GENERATORS["webbase"](), real=True, seed=3)


def test_rows_random_mixed_classes_real_values():
    rng = np.random.default_rng(11)
    n = 5000
    rows = []
    for i in range(3000):  # row lengths spread over 0..600 so every class appears
        L = int(rng.choice([0, 1, 2, 3, 5, 8, 20, 60, 150, 600], p=[.1, .2, .15, .15, .1, .1, .08, .06, .04, .02]))
        rows.append(np.sort(rng.choice(n, size=min(L, n), replace=False)))
    A = _csr(3000, n, rows)
    Bm = synth.random_csr(n, 7000, density=0.003, seed=12)
    B = (Bm[0], Bm[1], Bm[2], np.concatenate([np.sort(Bm[3][Bm[2][i]:Bm[2][i + 1]]) for i in range(n)]).astype(np.int32),
         Bm[4])
    cls = _classes(3000, n, A[2], A[3], B[2])
    assert all((cls == c).any() for c in range(H))
    _check(A, B, real=True, seed=5)


def test_rows_edge_cases():
    # empty matrix rows, a single row, a row selecting empty B rows only
    _check(_csr(5, 5, [[], [0, 1], [], [4], []]))
    _check(_csr(1, 1, [[0]]))
    B = _csr(4, 6, [[], [1, 5], [], [0, 2, 3]])
    _check(_csr(3, 4, [[0, 2], [1, 3], [0]]), B)


def test_rows_duplicate_runs_sum():
    # an A row naming the same B row twice (duplicate entries): equal keys of two
    # runs merge and sum
    A = _csr(2, 3, [[1, 1, 2], [0, 2, 2, 2]])
    B = _csr(3, 8, [[0, 7], [1, 3, 4], [3, 4, 6]])
    _check(A, B, real=True, seed=9)


def test_rows_many_runs_go_to_bitmap():
    # 2,000 runs of one column each (k > 1,024 -> class H) + a dense tail
    n = 40000
    rng = np.random.default_rng(4)
    hub = np.sort(rng.choice(n, size=2000, replace=False))
    rows = [hub] + [np.sort(rng.choice(n, size=3, replace=False)) for _ in range(200)]
    A = _csr(201, n, rows)
    Bm, Bn, Brp, Bci, Bvv = synth.random_csr(n, n, density=3e-5, seed=6)
    Bci = np.concatenate([np.sort(Bci[Brp[i]:Brp[i + 1]]) for i in range(n)]).astype(np.int32)
    assert _classes(201, n, A[2], A[3], Brp)[0] == H
    _check(A, (Bm, Bn, Brp, Bci, Bvv), real=True, seed=8)


def test_rows_bitmap_several_windows():
    # class H rows over 3,000,000 columns: three windows of 1,048,576 columns,
    # including an empty window in between
    n = 3_000_000
    rng = np.random.default_rng(7)
    k = 20
    Brows = []
    for j in range(k):
        lo = 0 if j % 2 == 0 else 2_500_000
        Brows.append(np.sort(rng.choice(np.arange(lo, lo + 400_000), size=400, replace=False)))
    B = _csr(k, n, Brows)
    A = _csr(3, k, [np.arange(k), np.arange(0, k, 2), np.array([1, 3])])
    assert _classes(3, k, A[2], A[3], B[2])[0] == H
    _check(A, B, real=True, seed=2)


def test_rows_merge_long_runs_and_collisions():
    # class M3 / M4 rows whose runs collide heavily (banded B): many equal columns
    rows = [np.arange(max(0, i - 30), min(2000, i + 31)) for i in range(2000)]
    A = _csr(2000, 2000, rows)
    cls = _classes(2000, 2000, A[2], A[3], A[2])
    assert (cls == M4).any() and (cls == M3).any() and (cls >= M3).all()
    _check(A, real=True, seed=4)


def test_rows_aat_lj_prefix():
    m, n, rp, ci, vv = synth.GENERATORS["lj"]()
    r = 20000
    e = int(rp[r])
    _check((r, n, rp[:r + 1].copy(), ci[:e].copy(), vv[:e].copy()), aat=True)


@pytest.mark.parametrize("checked", [False, True])
def test_default_routing_hub_rows_windowed(monkeypatch, checked):
    """A product with a hub row (past kRowsHubProducts = 65,536 products) that no
    single run dominates stays on the row-merge path: the windowed kernels
    (k_rows_w*) take the hub row (checked: through the fill lists, as above)."""
    monkeypatch.delenv("TSG_PATH", raising=False)
    if checked:
        monkeypatch.setenv("TSG_ROWS_CHECKED_SCAN", "1")
    n, nb = 300, 100_000
    rng = np.random.default_rng(21)
    # row 0 names every B row (300 runs of 300 columns spread over 100,000:
    # 90,000 products, no band window); 40 short rows
    rows = [np.arange(n)] + [np.array([i % n, (7 * i) % n]) for i in range(1, 41)]
    A = _csr(41, n, [np.unique(r) for r in rows])
    B = _csr(n, nb, [np.sort(rng.choice(nb, size=300, replace=False)) for _ in range(n)])
    m, _, rp, ci, vv = A
    Am = T.Matrix.from_csr(41, n, rp, ci, vv)
    Bm = T.Matrix.from_csr(n, nb, B[2], B[3], B[4])
    Cm, st = T.spgemm(Am, Bm)
    ref = O.gustavson(O.OMat.from_csr(41, n, rp, ci, vv), O.OMat.from_csr(n, nb, B[2], B[3], B[4])).csr()
    got = Cm.csr()
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    np.testing.assert_allclose(got[4], ref[4], rtol=1e-10, atol=0)
    assert st["path"] == T.PATH_ROWS


def test_default_routing_short_rows_row_merge(monkeypatch):
    """Short C rows (a 100-entry A row over 1-entry B rows, beside a 40-entry B
    row that no long A row selects) take the row-merge path by default."""
    monkeypatch.delenv("TSG_PATH", raising=False)
    n = 200
    brows = [np.array([(3 * j) % n]) for j in range(n)]
    brows[150] = np.arange(40)  # long B row, selected only by short A rows
    B = _csr(n, n, [np.unique(r) for r in brows])
    arows = [np.arange(100)] + [np.array([150, (i * 11) % 100]) for i in range(1, 60)]
    A = _csr(60, n, [np.unique(r) for r in arows])
    _check(A, B, real=True, seed=13, path=T.PATH_ROWS)


def test_rows_class_boundaries_by_entries():
    """Rows at each merge class's entry cap and one past it (62/63, 124/125,
    248/249, 504/505, 512/513 A entries of two products each): the class
    changes at the cap exactly (the LDS run tables are sized by it)."""
    n = 20000
    rng = np.random.default_rng(31)
    rows = []
    for cap in (62, 124, 248, 504, 512):
        for k in (cap, cap + 1):
            rows.append(np.sort(rng.choice(n, size=k, replace=False)))
    A = _csr(len(rows), n, rows)
    B = _csr(n, 50000, [np.sort(np.array([(7 * j) % 50000, (7 * j + 3) % 50000])) for j in range(n)])
    cls = _classes(len(rows), n, A[2], A[3], B[2])
    assert list(cls[0::2]) == [2, 3, 4, 5, 6] and list(cls[1::2]) == [3, 4, 5, 6, H]
    _check(A, B, real=True, seed=17)


@pytest.mark.parametrize("cls_products", [800, 1600, 3500])
def test_rows_unpacked_wide_span(cls_products):
    """M2 / M3 / M4 rows whose column span (20,000,000 columns) is too wide for
    packed u32 keys: the merge-path branch with moved (run, position) payloads
    and values gathered after the merge.  Runs sit at both ends of the range and
    collide (equal columns in several runs)."""
    n = 20_000_000
    rng = np.random.default_rng(cls_products)
    nb = 40
    Brows = []
    for j in range(nb):
        lo = 0 if j % 2 == 0 else n - 200_000
        Brows.append(np.sort(rng.choice(np.arange(lo, lo + 200_000, 50), size=cls_products // 20,
                                        replace=False)))
    B = _csr(nb, n, Brows)
    A = _csr(4, nb, [np.arange(0, 20), np.arange(20, 40), np.arange(0, 40, 3), np.array([1, 2, 5])])
    cls = _classes(4, nb, A[2], A[3], B[2])
    assert cls.max() >= 4 and cls.max() < H
    _check(A, B, real=True, seed=cls_products)


@pytest.mark.parametrize("checked", [False, True])
def test_rows_hub_rows_windowed_and_dominant_run(monkeypatch, checked):
    """Hub rows (past 65,536 products): without a dominant run the windowed
    kernels ((row, window) units, products bucketed per unit, per-unit LDS
    bitmaps, LDS values) -- many runs over 1,500,000 columns with heavy collisions (several
    buckets, windows with more nonzeros than one LDS value chunk), two long
    colliding runs; with one (all but <= 4,096 products in one run) the DR
    kernels -- one long run with a few short ones (the mawi pattern) and a row
    of one run -- beside ordinary rows.  checked: the large products' path
    (TSG_ROWS_CHECKED_SCAN=1: nnz(C) read back first), where the windowed units
    are filled from lists -- units of at most 1,024 products by the sort fill
    (k_rows_wsort), the rest by the bitmap fill, longest first."""
    if checked:
        monkeypatch.setenv("TSG_ROWS_CHECKED_SCAN", "1")
    rng = np.random.default_rng(41)
    n = 1_500_000
    nb = 3000
    Brows = [np.sort(rng.choice(n, size=int(rng.integers(20, 120)), replace=False)) for _ in range(nb - 3)]
    Brows.append(np.sort(rng.choice(n, size=200_000, replace=False)))  # a hub's long row
    Brows.append(np.sort(rng.choice(np.arange(1000, 1000 + 150_000), size=90_000, replace=False)))  # narrow
    Brows.append(np.arange(0, n, 7)[:80_000])
    B = _csr(nb, n, Brows)
    arows = [np.sort(rng.choice(nb - 3, size=1500, replace=False)),   # ~100k products, many runs
             np.array([5, 17, nb - 3]),                                # long run + short ones
             np.array([nb - 2, nb - 1]),                               # two long runs, colliding
             np.array([nb - 2])]                                       # one run, one window
    # class-H rows of a few thousand products over the whole span: windows of
    # 2^18 columns, units of ~700 / ~1,050 / ~2,300 products (the sort fill's
    # and the bitmap fill's sizes on either side of 1,024)
    arows += [np.sort(rng.choice(nb - 3, size=k, replace=False)) for k in (60, 90, 200)]
    arows += [np.sort(rng.choice(nb - 3, size=5, replace=False)) for _ in range(50)]
    A = _csr(len(arows), nb, arows)
    blen = np.diff(B[2].astype(np.int64))
    P = np.array([blen[r].sum() for r in arows])
    assert (P[:4] > 65536).all()
    _check(A, B, real=True, seed=43)


@pytest.mark.parametrize("pool", [None, 3000])
def test_rows_windowed_sort_fill_unit_sizes(monkeypatch, pool):
    """The checked-scan path's fill lists across unit sizes: class-H rows of
    4,100 .. 20,000 products over a 1.5 M-column span (windows of 2^18
    columns, units of ~700 .. ~3,300 products: the sort fill up to 1,024, the
    bitmap fill past it), with B's columns drawn from the whole span (few
    repeats) or from a pool of 3,000 columns (long runs of equal columns in
    the sort fill's summing walk), plus the npow boundaries 256 / 257 and
    1,024 / 1,025 of single-window rows.  Pattern exact, values within 1e-10
    of |A||B|."""
    monkeypatch.setenv("TSG_ROWS_CHECKED_SCAN", "1")
    rng = np.random.default_rng(61 if pool is None else 62)
    n, nb = 1_500_000, 3000
    cols = np.arange(n) if pool is None else np.sort(rng.choice(n, size=pool, replace=False))
    Brows = [np.sort(rng.choice(cols, size=int(rng.integers(50, 150)), replace=False)) for _ in range(nb - 4)]
    # single-window rows: one B row each of 256 / 257 / 1,024 / 1,025 columns inside 2^18
    for k in (256, 257, 1024, 1025):
        Brows.append(np.sort(rng.choice(200_000, size=k, replace=False)))
    B = _csr(nb, n, Brows)
    blen = np.diff(B[2].astype(np.int64))
    arows = []
    for target in (4100, 5000, 6500, 9000, 13000, 20000):
        k = int(target / blen[:nb - 4].mean())
        arows.append(np.sort(rng.choice(nb - 4, size=k, replace=False)))
    # (a row over the single-window B rows and a few short ones: class H by its products)
    arows.append(np.array([nb - 4, nb - 3, nb - 2, nb - 1] + list(range(10, 40))))
    arows += [np.sort(rng.choice(nb - 4, size=4, replace=False)) for _ in range(30)]
    A = _csr(len(arows), nb, arows)
    _check(A, B, real=True, seed=67)


@pytest.mark.parametrize("per_row", [False, True])
def test_rows_dominant_run_rows_grouped_by_run(monkeypatch, per_row):
    """Many dominant-run rows sharing a run (the mawi pattern: every hub
    neighbour's C row holds the hub's whole B row): k_rows_dr_group sorts them
    by run and cuts each run's rows into blocks of DR_GR = 16 whose chunks of
    DR_CH = 16,384 elements read the run once for the block.  71 + 32 rows on
    two runs of 120,000 / 70,001 columns (blocks of 16, 16, 16, 16, 7 and 16,
    16: a partial last block on the first run), their
    inserted columns before, inside (some L holds: a sum) and past the run, in
    one range or many; with TSG_DR_PER_ROW the per-row chunks instead."""
    if per_row:
        monkeypatch.setenv("TSG_DR_PER_ROW", "1")
    rng = np.random.default_rng(61)
    n = 1_500_000
    nb = 4000
    Brows = [np.sort(rng.choice(n, size=int(rng.integers(1, 40)), replace=False)) for _ in range(nb - 4)]
    h1 = np.sort(rng.choice(np.arange(1000, n - 1000), size=120_000, replace=False))
    h2 = np.sort(rng.choice(n, size=70_001, replace=False))
    Brows += [h1, h2, np.array([0, 1, 2]), np.array([n - 3, n - 2, n - 1])]  # (before / past h1)
    B = _csr(nb, n, Brows)
    arows = []
    for i in range(70):
        extra = rng.choice(nb - 4, size=int(rng.integers(0, 6)), replace=False)
        if i % 7 == 0:
            extra = np.concatenate([extra, [nb - 2, nb - 1]])
        arows.append(np.sort(np.concatenate([extra, [nb - 4]])))
    arows.append(np.sort(np.concatenate([rng.choice(nb - 4, size=120, replace=False), [nb - 4]])))  # many ranges
    for i in range(32):
        arows.append(np.sort(np.concatenate([rng.choice(nb - 4, size=int(rng.integers(0, 4)), replace=False),
                                             [nb - 3]])))
    arows += [np.sort(rng.choice(nb - 4, size=5, replace=False)) for _ in range(20)]  # ordinary rows
    order = rng.permutation(len(arows))  # (the runs' rows interleaved)
    arows = [arows[i] for i in order]
    A = _csr(len(arows), nb, arows)
    blen = np.diff(B[2].astype(np.int64))
    P = np.array([blen[r].sum() for r in arows])
    assert (P > 65536).sum() == 103
    _check(A, B, real=True, seed=67)


def test_rows_mawi_prefix_hub_rows():
    """The mawi stand-in at 1e-2 scale (hub degree 1e5): a row prefix holding
    hub-neighbour rows (each C row receives the hub's whole row) through the
    row-merge path, against the oracle."""
    m, n, rp, ci, vv = synth.mawi(scale=0.01)
    blen = np.diff(rp.astype(np.int64))
    cum = np.concatenate([[0], np.cumsum(blen[ci])])[rp]
    r = int(np.searchsorted(cum, 3e7, side="right") - 1)
    P = np.diff(cum[:r + 1])
    assert P.max() > 65536
    _check((r, n, rp[:r + 1].copy(), ci[:rp[r]].copy(), vv[:rp[r]].copy()), (m, n, rp, ci, vv), real=True, seed=47)


def test_default_routing_very_wide_b(monkeypatch):
    """Short C rows with B wider than 2^28 columns take the row-merge path by
    default (unpacked keys).  Checked against a per-row numpy product (the
    oracle's dense row accumulator would need B.n doubles per thread)."""
    monkeypatch.delenv("TSG_PATH", raising=False)
    rng = np.random.default_rng(51)
    n = (1 << 28) + 1000
    nb = 300
    Brows = [np.sort(rng.choice(n, size=int(rng.integers(1, 6)), replace=False)) for _ in range(nb)]
    B = _csr(nb, n, Brows)
    arows = [np.sort(rng.choice(nb, size=int(rng.integers(0, 5)), replace=False)) for _ in range(200)]
    A = _csr(200, nb, arows)
    av = rng.uniform(-1, 1, len(A[3]))
    bv = rng.uniform(-1, 1, len(B[3]))
    Am = T.Matrix.from_csr(200, nb, A[2], A[3], av)
    Bm = T.Matrix.from_csr(nb, n, B[2], B[3], bv)
    Cm, st = T.spgemm(Am, Bm)
    assert st["path"] == T.PATH_ROWS
    _, _, grp, gci, gvv = Cm.csr()
    want_rp, want_ci, want_v = [0], [], []
    for i in range(200):
        cols, vals = [], []
        for p in range(A[2][i], A[2][i + 1]):
            j = A[3][p]
            cols.append(B[3][B[2][j]:B[2][j + 1]])
            vals.append(av[p] * bv[B[2][j]:B[2][j + 1]])
        if cols:
            c = np.concatenate(cols)
            v = np.concatenate(vals)
            u, inv = np.unique(c, return_inverse=True)
            s = np.zeros(len(u))
            np.add.at(s, inv, v)
            want_ci.append(u)
            want_v.append(s)
            want_rp.append(want_rp[-1] + len(u))
        else:
            want_rp.append(want_rp[-1])
    np.testing.assert_array_equal(grp, np.array(want_rp))
    np.testing.assert_array_equal(gci, np.concatenate(want_ci))
    np.testing.assert_allclose(gvv, np.concatenate(want_v), rtol=1e-12, atol=1e-15)


def test_rows_class_h_one_walk_rows():
    """Class H's one-walk rows (tsg_rows.hip k_rows_bitmap: one gather walk, the
    first 16,384 products in registers and the rest in the row's scratch slots,
    columns and values through the bitmap's LDS by rank passes of 32,768 /
    16,384): rows at the register boundary (16,384 and 16,385 products), past it
    with up to 2,048 runs (two passes of column ranks, four of values), a row
    of 2,049 runs and one spanning two column windows (both the windowed
    bitmap walk), with repeated columns and real values."""
    rng = np.random.default_rng(21)
    nb, ncol = 6000, 3_000_000
    lens = np.where(np.arange(nb) % 2 == 0, rng.integers(1, 5, nb), rng.integers(20, 60, nb))
    brows = []
    for i in range(nb):
        lo = 0 if i % 3 else 40_000  # clustered and spread columns: repeats and unique ones
        hi = 200_000 if i % 3 else 900_000
        brows.append(np.sort(rng.choice(np.arange(lo, hi), size=int(lens[i]), replace=False)))
    brows[nb - 1] = np.array([0, 2_500_000])  # the two-window row's far column
    Bc = _csr(nb, ncol, brows)
    blen = np.diff(Bc[2].astype(np.int64))

    def pick(target, must=None, long_only=False):
        """distinct B rows whose lengths sum to exactly `target` products"""
        order = rng.permutation(nb - 1)
        if long_only:
            order = order[blen[order] >= 8]
        sel, tot = set(), 0
        for b in order:
            if tot + blen[b] <= target - 4:
                sel.add(int(b))
                tot += blen[b]
        for b in rng.permutation(nb - 1):  # close the gap exactly with rows of 1-4 products
            if tot == target:
                break
            if b not in sel and blen[b] <= target - tot:
                sel.add(int(b))
                tot += blen[b]
        if must is not None:
            sel.add(must)
        return np.sort(np.array(sorted(sel)))

    rows = [pick(16384), pick(16385), pick(24000), pick(61000, long_only=True), pick(9000)]
    # 2,049 runs (past the one-walk run table): short B rows only
    short = np.nonzero(blen <= 4)[0]
    rows.append(np.sort(rng.choice(short[short < nb - 1], 2049, replace=False)))
    rows.append(pick(6000, must=nb - 1))  # two column windows
    A = _csr(len(rows), nb, rows)
    P = [int(blen[r].sum()) for r in rows]
    assert P[0] == 16384 and P[1] == 16385 and all(4096 < p <= 65536 for p in P)
    assert max(len(r) for r in rows[:5]) <= 2048 and len(rows[5]) == 2049, [len(r) for r in rows]
    cls = _classes(len(rows), nb, A[2], A[3], Bc[2])
    assert (cls == H).all()
    _check(A, Bc, real=True, seed=9)


def test_repeated_column_in_b_row_routes_to_tiles(monkeypatch):
    """A B row that repeats a column (here a long hub row, the dominant-run
    kind) is not strictly column-sorted: the sortedness check flags it and the
    default route sends the product to the staged tile pipeline, whose C sums
    the repeated column's products like the oracle (the dominant-run kernels
    copy a run as it stands and would emit the column twice)."""
    monkeypatch.delenv("TSG_PATH", raising=False)
    rng = np.random.default_rng(61)
    n = 5000
    hub = np.sort(rng.choice(n, size=3000, replace=False))
    hub = np.sort(np.concatenate([hub, hub[1500:1501]]))  # one column twice, adjacent
    brows = [hub] + [np.sort(rng.choice(n, size=int(rng.integers(1, 8)), replace=False)) for _ in range(n - 1)]
    B = _csr(n, n, brows)
    arows = [np.sort(np.concatenate([[0], rng.choice(np.arange(1, n), size=3, replace=False)])) for _ in range(40)]
    A = _csr(40, n, arows)
    _check(A, B, real=True, seed=62, path=T.PATH_TILES)


def test_rows_scans_past_the_fused_tiles():
    """More than RS_INLINE_MAX = 2,048 tiles of 4,096 A entries and of row
    counts (9 * 10^6 rows, one entry each: A a permutation with two shuffled
    blocks, C = A*A): the setup's entry scan and the row-pointer scan take the
    generic three-launch scans and k_rows_cfirst instead of the fused kernels.
    C is A's permutation applied twice -- checked exactly with numpy."""
    m = 9_000_000
    rng = np.random.default_rng(5)
    ci = rng.permutation(m).astype(np.int32)
    rp = np.arange(m + 1, dtype=np.int32)
    vv = rng.uniform(0.5, 2.0, m)
    A = T.Matrix.from_csr(m, m, rp, ci, vv)
    Cm, st = T.spgemm(A, T.Matrix.alias(A))
    got = Cm.csr()
    np.testing.assert_array_equal(got[2], rp)
    np.testing.assert_array_equal(got[3], ci[ci])
    np.testing.assert_array_equal(got[4], vv * vv[ci])  # one product per entry: exact
    assert st["path"] == T.PATH_ROWS and st["nnzC"] == m
