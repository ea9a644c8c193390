"""Synthetic inputs: value(r, c) = lo + splitmix64_at(seed, r*cols + c) % (hi - lo).

The device generator is sda_synth_fill_dev (csrc/elementwise.hip); this numpy twin produces the
same values on the host so CPU baselines and parity tests can regenerate any slice of a
benchmark matrix without copying it back from HBM.
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

SEED_BASE = 0x5DA          # config c uses SEED_BASE + c


def splitmix64_at(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def fill(rows: int, cols: int, seed: int, lo: int, hi: int, row0: int = 0) -> np.ndarray:
    """Rows [row0, row0 + rows) of the (.., cols) synthetic matrix, as int64."""
    rng = np.uint64((hi - lo) % (1 << 64))
    idx = (np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row0)) * np.uint64(cols) + \
        np.arange(cols, dtype=np.uint64)[None, :]
    z = splitmix64_at(seed, idx)
    with np.errstate(over="ignore"):
        v = np.uint64(lo % (1 << 64)) + z % rng
    return v.view(np.int64).reshape(rows, cols)
