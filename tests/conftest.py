import glob
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)

GOLDEN = os.path.join(TESTS, "golden")
FIXTURES = os.path.join(GOLDEN, "fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden_cases():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "ref", "*.npz"))):
        base = os.path.basename(p)[:-4]
        name, aat, tiles = base.rsplit("_", 2)
        tm, tn = map(int, tiles.split("x"))
        out.append(pytest.param(p, name, int(aat[3:]), tm, tn, id=base))
    return out
