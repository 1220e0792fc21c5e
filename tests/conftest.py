import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-resolution C3 cases")


@pytest.fixture(scope="session")
def scene_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("scenes"))


def ulp_diff(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Distance in units in the last place between two float32 arrays (monotone int map)."""
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return np.abs(ai - bi)


def assert_parity(got: np.ndarray, ref: np.ndarray, what: str = "", max_ulp: int = 1):
    """North-star tolerance: every channel within 1 ULP (and 1e-4 absolute) of the reference.
    Reports how many channels are not bit-identical."""
    assert got.shape == ref.shape, (got.shape, ref.shape)
    nan_got, nan_ref = np.isnan(got), np.isnan(ref)
    assert np.array_equal(nan_got, nan_ref), f"{what}: NaN pattern differs"
    g = np.where(nan_got, 0, got).astype(np.float32)
    r = np.where(nan_ref, 0, ref).astype(np.float32)
    d = ulp_diff(g, r)
    bad = int((d > 0).sum())
    worst = int(d.max()) if d.size else 0
    if worst > max_ulp or not np.allclose(g, r, rtol=0, atol=1e-4):
        idx = np.unravel_index(int(d.argmax()), d.shape)
        raise AssertionError(f"{what}: {bad} channels differ, worst {worst} ulp at {idx}: "
                             f"got {g[idx]!r} ref {r[idx]!r}")
    return bad
