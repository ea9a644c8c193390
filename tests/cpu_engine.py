"""Host stand-in for the device entry points sda_amd.distributed calls (CPU / gloo tests only).

Same method names and arguments as sda_amd.Engine's `_dev` entry points, but the pointers are
host addresses of CPU torch tensors and the oracle does the arithmetic.  This lets the world-2
gloo tests run the product functions of sda_amd.distributed themselves (shard split, reduce,
finalize, all-gather) with nothing but the per-rank compute swapped out.
"""
import ctypes

import numpy as np

from oracle import oracle as O


def _view(ptr: int, n: int, ctype=ctypes.c_int64) -> np.ndarray:
    if n == 0:
        return np.zeros(0, np.int64)
    return np.ctypeslib.as_array((ctype * n).from_address(ptr))


def _rows(ptr: int, n: int, dim: int, stride: int) -> np.ndarray:
    if n == 0 or dim == 0:
        return np.zeros((n, dim), np.int64)
    flat = _view(ptr, (n - 1) * stride + dim)
    return np.lib.stride_tricks.as_strided(flat, (n, dim), (stride * 8, 8)).copy()


class CpuEngine:
    def __init__(self):
        self.calls = []

    def combine_dev(self, modulus, shares_ptr, n, dim, row_stride, out_ptr, stream=None):
        self.calls.append("combine_dev")
        _view(out_ptr, dim)[:] = O.combine(modulus, _rows(shares_ptr, n, dim, row_stride))

    def combine_accumulate_dev(self, modulus, shares_ptr, n, dim, row_stride, inout_ptr, stream=None):
        # continuing from r (|r| < m) == one pass whose first row is r: (0 + r) % m == r
        self.calls.append("combine_accumulate_dev")
        acc = _view(inout_ptr, dim)
        acc[:] = O.combine(modulus, np.vstack([acc[None, :], _rows(shares_ptr, n, dim, row_stride)]))

    def combine_finalize_dev(self, modulus, sums_ptr, dim, out_ptr, stream=None):
        # canonical residue of the two's-complement u64 sums (launch_mod_canonical)
        self.calls.append("combine_finalize_dev")
        s = _view(sums_ptr, dim).view(np.uint64)
        _view(out_ptr, dim)[:] = (s % np.uint64(abs(modulus))).astype(np.int64)

    def chacha_mask_combine_dev(self, modulus, dimension, seeds_ptr, w, n_seeds, out_ptr, stream=None):
        self.calls.append("chacha_mask_combine_dev")
        seeds = _view(seeds_ptr, n_seeds * w, ctypes.c_uint32).reshape(n_seeds, w).astype(np.int64) \
            if n_seeds else np.zeros((0, w), np.int64)
        _view(out_ptr, dimension)[:] = O.chacha_mask_combine(modulus, dimension, seeds)
