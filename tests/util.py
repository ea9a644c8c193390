"""Small assertion helpers: compare integer arrays bit for bit without pytest's (slow) list diffs."""
import numpy as np


def assert_same(got, exp, what=""):
    g = np.asarray(got, dtype=np.int64)
    e = np.asarray(exp, dtype=np.int64)
    assert g.shape == e.shape, f"{what}: shape {g.shape} != {e.shape}"
    bad = np.flatnonzero(g.reshape(-1) != e.reshape(-1))
    if bad.size:
        i = int(bad[0])
        raise AssertionError(f"{what}: {bad.size} of {g.size} elements differ; first at flat index {i}: "
                             f"got {int(g.reshape(-1)[i])}, expected {int(e.reshape(-1)[i])}")
