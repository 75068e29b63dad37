"""Seeded synthetic stand-ins for the BASELINE.json matrices.

The SuiteSparse files are not available (no network); when a real .mtx is
present it is used instead (bench.py --mtx / $TSG_MTX_DIR).  Every generator is
deterministic for a given seed (default 20260116, the reference snapshot date)
and returns a CSR with ascending column indices per row -- the order
mmio_allinone produces for SuiteSparse files, which are stored column-major
(src/mmio_highlevel.h:707-741).  Values follow src/main.cu:111-112
(value[k] = k % 10 by CSR position).

  webbase   n = 1,000,005, nnz 3.09 M: web crawl -- power-law out-degree
            (P(d) ~ (d+c)^-2.1, d <= 4700) correlated with popularity, 60 % of
            links to nearby pages (same host, |delta| ~ geometric, mean 24), 40 %
            to pages drawn from a Zipf(1.0) popularity law; calibrated to
            webbase-1M's A^2 work (nnzCub 69.1 M vs 69.5 M published)
  cant      n = 62,451, 3-D FEM cantilever: 9 x 9 x 257 nodes x 3 dof, 27-point
            hexahedral couplings (3 x 3 blocks, 92 % kept); calibrated to the
            reference's pinned cant A^2 (nnzCub 269.5 M, nnzC 17.4 M)
  mc2depi   n = 525,825, unsymmetric 4-point stencil on a 725 x 725 grid + tail
  lj        n = 3,997,962, R-MAT (a=.57, b=c=.19), avg 17.3, symmetrised
  mawi      n = 226,196,185 (x scale), symmetric star + noise: one hub adjacent
            to 10^7 (x scale) random nodes, plus uniform random edges for an
            average degree of ~2 (nnz ~472 M at scale 1; the real matrix has 480 M)
"""
import numpy as np

SEED = 20260116


def _finish(n_rows, n_cols, rows, cols):
    """Dedupe (row, col) pairs, sort row-major, build CSR with pos % 10 values."""
    key = rows.astype(np.int64) * n_cols + cols.astype(np.int64)
    key = np.unique(key)
    r = (key // n_cols).astype(np.int64)
    c = (key % n_cols).astype(np.int32)
    rowptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.add.at(rowptr, r + 1, 1)
    rowptr = np.cumsum(rowptr)
    if rowptr[-1] >= 2 ** 31:
        raise ValueError("nnz exceeds int32")
    val = (np.arange(len(c), dtype=np.int64) % 10).astype(np.float64)
    return rowptr.astype(np.int32), c, val


def _powerlaw_degrees(rng, n, mean, alpha, dmax):
    d = np.arange(0, dmax + 1, dtype=np.float64)
    lo, hi = 0.01, 100.0
    for _ in range(60):  # bisection on the offset c for the requested mean
        c = 0.5 * (lo + hi)
        p = (d + c) ** (-alpha)
        p /= p.sum()
        mu = (p * d).sum()
        if mu > mean:
            hi = c
        else:
            lo = c
    return rng.choice(d.astype(np.int64), size=n, p=p)


def webbase(n=1_000_005, seed=SEED, mean_deg=4.0, sigma=5.5, p_local=0.6):
    """Calibrated so that n, nnz and the A^2 work match webbase-1M's published
    figures (nnz 3.1 M, 2*nnzCub = 139 MFLOP): this model gives nnz 3.09 M,
    nnzCub 69.1 M, nnzC 64.9 M.  Out-degree ~ (d+c)^-2.1; pages are ranked by a
    noisy popularity score (log-rank + N(0, sigma)) and the largest out-degrees go
    to the most popular pages (in/out-degree correlation of real crawls)."""
    rng = np.random.default_rng(seed)
    deg = _powerlaw_degrees(rng, n, mean_deg, 2.1, 4700)
    perm = rng.permutation(n)  # popularity rank -> page id
    score = np.log1p(np.arange(n)) + rng.normal(0.0, sigma, n)
    deg_by_page = np.empty(n, dtype=np.int64)
    deg_by_page[perm[np.argsort(score)]] = np.sort(deg)[::-1]
    rows = np.repeat(np.arange(n, dtype=np.int64), deg_by_page)
    m = len(rows)
    local = rng.random(m) < p_local
    delta = rng.geometric(1.0 / 24.0, size=m) * np.where(rng.random(m) < 0.5, -1, 1)
    loc_cols = np.clip(rows + delta, 0, n - 1)
    # Zipf(1) popularity: rank = floor(n^u) - 1
    ranks = np.floor(np.exp(rng.random(m) * np.log(n))).astype(np.int64) - 1
    glob_cols = perm[np.clip(ranks, 0, n - 1)]
    cols = np.where(local, loc_cols, glob_cols)
    rowptr, col, val = _finish(n, n, rows, cols)
    return n, n, rowptr, col, val


def cant(seed=SEED, dims=(9, 9, 257), keep=0.9225):
    """3-D FEM cantilever stand-in: a 9 x 9 x 257 grid of nodes (20,817 nodes x 3
    degrees of freedom = 62,451 rows, as cant.mtx), each node coupled to its
    27-point (hexahedral-element) neighbourhood by dense 3 x 3 blocks, every
    node-node coupling kept with probability `keep` (symmetrically).  Calibrated
    to the reference's only pinned figures for cant A^2 (data/results_tile.csv:1:
    nnzCub 269,486,473, nnzC 17,440,029): this model gives nnz 4,005,045 (cant.mtx:
    4,007,383), nnzCub 269,494,911 (+0.003 %) and nnzC 17,301,501 (-0.8 %)."""
    rng = np.random.default_rng(seed)
    nx, ny, nz = dims
    nn = nx * ny * nz
    idx = np.arange(nn, dtype=np.int64).reshape(nz, ny, nx)
    pr, pc = [np.arange(nn, dtype=np.int64)], [np.arange(nn, dtype=np.int64)]
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if (dz, dy, dx) <= (0, 0, 0):
                    continue  # each unordered neighbour pair once, mirrored below
                a = idx[max(0, -dz):nz - max(0, dz), max(0, -dy):ny - max(0, dy), max(0, -dx):nx - max(0, dx)]
                b = idx[max(0, dz):nz - max(0, -dz), max(0, dy):ny - max(0, -dy), max(0, dx):nx - max(0, -dx)]
                k = rng.random(a.size) < keep
                pr += [a.ravel()[k], b.ravel()[k]]
                pc += [b.ravel()[k], a.ravel()[k]]
    nr, nc = np.concatenate(pr), np.concatenate(pc)
    # node pair (u, v) -> the 3 x 3 block of rows 3u..3u+2, columns 3v..3v+2
    di = np.repeat(np.arange(3), 3)
    dj = np.tile(np.arange(3), 3)
    rows = (3 * nr[:, None] + di[None, :]).ravel()
    cols = (3 * nc[:, None] + dj[None, :]).ravel()
    n = 3 * nn
    rowptr, col, val = _finish(n, n, rows, cols)
    return n, n, rowptr, col, val


def mc2depi(n=525_825, seed=SEED):
    rng = np.random.default_rng(seed)
    g = 725
    idx = np.arange(n, dtype=np.int64)
    x, y = idx % g, idx // g
    rows, cols = [idx], [idx]
    for dx, dy in ((1, 0), (0, 1), (-1, 0)):
        xx, yy = x + dx, y + dy
        ok = (xx >= 0) & (xx < g) & (yy >= 0) & (yy * g + xx < n) & (rng.random(n) < 0.75)
        rows.append(idx[ok])
        cols.append((yy * g + xx)[ok])
    rowptr, col, val = _finish(n, n, np.concatenate(rows), np.concatenate(cols))
    return n, n, rowptr, col, val


def rmat(scale_n=3_997_962, avg=17.3, seed=SEED, a=0.57, b=0.19, c=0.19):
    rng = np.random.default_rng(seed)
    levels = int(np.ceil(np.log2(scale_n)))
    m = int(scale_n * avg / 2)
    r = np.zeros(m, dtype=np.int64)
    q = np.zeros(m, dtype=np.int64)
    for _ in range(levels):
        u = rng.random(m)
        bit_r = (u >= a + b).astype(np.int64)
        bit_c = (((u >= a) & (u < a + b)) | (u >= a + b + c)).astype(np.int64)
        r = (r << 1) | bit_r
        q = (q << 1) | bit_c
    perm = rng.permutation(1 << levels)
    r, q = perm[r], perm[q]
    ok = (r < scale_n) & (q < scale_n)
    r, q = r[ok], q[ok]
    rows = np.concatenate([r, q])
    cols = np.concatenate([q, r])
    rowptr, col, val = _finish(scale_n, scale_n, rows, cols)
    return scale_n, scale_n, rowptr, col, val


def random_csr(m, n, density=None, nnz_per_row=None, seed=SEED, unsorted=False, dups=False):
    """Small generic matrices for parity tests (optionally unsorted / duplicates)."""
    rng = np.random.default_rng(seed)
    if nnz_per_row is None:
        nnz_per_row = max(1, int(density * n))
    deg = rng.integers(0, 2 * nnz_per_row + 1, size=m)
    rows = np.repeat(np.arange(m, dtype=np.int64), deg)
    cols = rng.integers(0, n, size=len(rows))
    if not dups:
        rowptr, col, val = _finish(m, n, rows, cols)
    else:
        order = np.lexsort((cols, rows))
        rows, cols = rows[order], cols[order]
        rowptr = np.zeros(m + 1, dtype=np.int64)
        np.add.at(rowptr, rows + 1, 1)
        rowptr = np.cumsum(rowptr).astype(np.int32)
        col = cols.astype(np.int32)
        val = (np.arange(len(col)) % 10).astype(np.float64)
    if unsorted:
        col = col.copy()
        for i in range(m):
            s, e = rowptr[i], rowptr[i + 1]
            col[s:e] = col[s:e][rng.permutation(e - s)]
    return m, n, rowptr, col, val


def mawi(scale=1.0, seed=SEED, hub_deg=10_000_000, noise_deg=2.0):
    """Packet-trace graph stand-in: its A^2 is dominated by the hub (every hub
    neighbour's row of C receives the hub's whole row), so the full product is
    far beyond int32 nnz(C) -- bench.py runs the largest feasible row prefix."""
    rng = np.random.default_rng(seed)
    n = max(16, int(226_196_185 * scale))
    hd = max(1, int(hub_deg * scale))
    hub = int(rng.integers(n // 2, n))  # late, so row prefixes before it stay feasible
    nb = rng.choice(n, size=hd, replace=False)
    nb = nb[nb != hub]
    m_noise = int(n * noise_deg / 2)
    u = rng.integers(0, n, m_noise)
    v = rng.integers(0, n, m_noise)
    rows = np.concatenate([np.full(len(nb), hub, np.int64), nb, u, v])
    cols = np.concatenate([nb, np.full(len(nb), hub, np.int64), v, u])
    rowptr, col, val = _finish(n, n, rows, cols)
    return n, n, rowptr, col, val


GENERATORS = {"webbase": webbase, "cant": cant, "mc2depi": mc2depi, "lj": rmat, "mawi": mawi}
