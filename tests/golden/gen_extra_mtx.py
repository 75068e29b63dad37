"""Generate extra Matrix-Market fixtures (seeded) that exercise loader and tiling
edge cases the reference's own UnitTest/CSR2TILE fixtures do not cover:
symmetric mirroring, pattern / integer value types, unsorted file order with
duplicate entries, rectangular shapes (A*A^T), empty rows and empty tile rows,
fully dense tiles, and multi-tile-row banded / power-law structure.

Run:  python tests/golden/gen_extra_mtx.py   (writes tests/golden/fixtures/x_*.mtx)
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "fixtures")


def write(name, m, n, entries, field="real", sym="general", rng=None):
    path = os.path.join(OUT, name + ".mtx")
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {field} {sym}\n")
        f.write(f"% tsg extra fixture {name}\n")
        f.write(f"{m} {n} {len(entries)}\n")
        for (i, j) in entries:
            if field == "pattern":
                f.write(f"{i + 1} {j + 1}\n")
            elif field == "integer":
                f.write(f"{i + 1} {j + 1} {int(rng.integers(-9, 10))}\n")
            else:
                f.write(f"{i + 1} {j + 1} {rng.uniform(-1, 1):.6f}\n")


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20260116)

    # symmetric pattern, lower triangle stored column-major (SuiteSparse style)
    m = 100
    ent = set()
    for j in range(m):
        ent.add((j, j))
        for i in rng.choice(np.arange(j, m), size=min(4, m - j), replace=False):
            ent.add((int(i), j))
    ent = sorted(ent, key=lambda e: (e[1], e[0]))
    write("x_sym_pattern_100", m, m, ent, field="pattern", sym="symmetric", rng=rng)

    # symmetric real with mirrored entries crossing tile boundaries
    m = 70
    ent = sorted({(int(i), int(j)) for i, j in zip(rng.integers(0, m, 300), rng.integers(0, m, 300)) if i >= j},
                 key=lambda e: (e[1], e[0]))
    write("x_sym_real_70", m, m, ent, sym="symmetric", rng=rng)

    # integer values, entries in shuffled file order, with duplicates
    m = 77
    base = [(int(i), int(j)) for i, j in zip(rng.integers(0, m, 500), rng.integers(0, m, 500))]
    base += base[:40]  # duplicates
    order = rng.permutation(len(base))
    write("x_int_unsorted_dup_77", m, m, [base[k] for k in order], field="integer", rng=rng)

    # rectangular (A*A^T only)
    mr, nr = 50, 130
    ent = sorted({(int(i), int(j)) for i, j in zip(rng.integers(0, mr, 700), rng.integers(0, nr, 700))})
    write("x_rect_50x130", mr, nr, ent, rng=rng)

    # empty rows and a completely empty tile row (rows 16..31)
    m = 64
    ent = []
    for i in range(m):
        if 16 <= i < 32 or i % 7 == 3:
            continue
        for j in rng.choice(m, size=3, replace=False):
            ent.append((i, int(j)))
    write("x_empty_rows_64", m, m, sorted(ent), rng=rng)

    # dense 48x48: full 16x16 tiles, C tiles with 256 nonzeros
    m = 48
    write("x_dense_48", m, m, [(i, j) for i in range(m) for j in range(m)], rng=rng)

    # banded 500x500, half bandwidth 12 (FEM-like, cant stand-in in miniature)
    m, hb = 500, 12
    ent = [(i, j) for i in range(m) for j in range(max(0, i - hb), min(m, i + hb + 1))]
    write("x_banded_500", m, m, ent, rng=rng)

    # power-law out/in degree 400x400 (webbase stand-in in miniature)
    m = 400
    deg = np.minimum((rng.pareto(1.1, m) + 1).astype(int), 120)
    ent = set()
    w = 1.0 / np.arange(1, m + 1) ** 1.1
    w /= w.sum()
    perm = rng.permutation(m)
    for i in range(m):
        for j in rng.choice(m, size=int(deg[i]), replace=True, p=w):
            ent.add((i, int(perm[j])))
    write("x_powerlaw_400", m, m, sorted(ent), rng=rng)


if __name__ == "__main__":
    main()
