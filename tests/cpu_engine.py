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
        # canonical residue of the (signed) int64 sums (launch_mod_canonical)
        self.calls.append("combine_finalize_dev")
        _view(out_ptr, dim)[:] = np.mod(_view(sums_ptr, dim), abs(modulus))

    # ---- participation split (include/sda_engine.h), restated independently of the device kernels ----
    def combine_split_dev(self, modulus, shares_ptr, n, dim, row_stride, inout_ptr, flags_ptr, stream=None):
        self.calls.append("combine_split_dev")
        rows = _rows(shares_ptr, n, dim, row_stride)
        acc = _view(inout_ptr, dim)
        acc[:] = O.combine(modulus, np.vstack([acc[None, :], rows]))
        lim = (1 << 63) - abs(modulus)
        fl = _view(flags_ptr, 2)
        if rows.size and rows.min() < 0:
            fl[0] = 1
        if rows.size and (int(rows.min()) < -lim or int(rows.max()) > lim):
            fl[1] = 1

    def combine_split_prefix_dev(self, modulus, gathered_ptr, world, rank, dim, c_in_ptr, total_ptr, code_ptr,
                                 stream=None):
        self.calls.append("combine_split_prefix_dev")
        m = abs(modulus)
        g = _view(gathered_ptr, world * dim).reshape(world, dim)
        _view(c_in_ptr, dim)[:] = [sum(int(x) for x in g[:rank, j]) % m for j in range(dim)]
        _view(total_ptr, dim)[:] = [sum(int(x) for x in g[:, j]) % m for j in range(dim)]
        _view(code_ptr, dim, ctypes.c_int32)[:] = (1 + (g[0] < 0)) if rank == 0 else 0

    def combine_split_replay_dev(self, modulus, shares_ptr, n, dim, row_stride, rank, state_ptr, code_ptr,
                                 stream=None):
        # The chunk maps the sign s of the running value r = c - m s through s -> f(s).  Run the
        # reference recurrence (the oracle) from BOTH hypotheses, r = c_in and r = c_in - m, and read f:
        # f(0) == f(1) is an event (set / reset), f(0) != f(1) none.  (c_in = 0 forces s = 0: f(0) decides.)
        self.calls.append("combine_split_replay_dev")
        m = abs(modulus)
        rows = _rows(shares_ptr, n, dim, row_stride)
        c = _view(state_ptr, dim)
        code = _view(code_ptr, dim, ctypes.c_int32)
        r0 = O.combine(modulus, np.vstack([c[None, :], rows]))
        r1 = O.combine(modulus, np.vstack([np.where(c > 0, c - m, 0)[None, :], rows]))
        f0, f1 = r0 < 0, r1 < 0
        event = (c == 0) | (f0 == f1)
        code[:] = np.where(event, 2 * rank + 1 + f0.astype(np.int32), code)
        c[:] = np.mod(r0, m)

    def combine_split_resolve_dev(self, modulus, total_ptr, code_ptr, dim, out_ptr, stream=None):
        self.calls.append("combine_split_resolve_dev")
        code = _view(code_ptr, dim, ctypes.c_int32)
        _view(out_ptr, dim)[:] = _view(total_ptr, dim) - np.where((code - 1) % 2 == 1, abs(modulus), 0)

    def chacha_mask_combine_dev(self, modulus, dimension, seeds_ptr, w, n_seeds, out_ptr, stream=None):
        self.calls.append("chacha_mask_combine_dev")
        seeds = _view(seeds_ptr, n_seeds * w, ctypes.c_uint32).reshape(n_seeds, w).astype(np.int64) \
            if n_seeds else np.zeros((0, w), np.int64)
        _view(out_ptr, dimension)[:] = O.chacha_mask_combine(modulus, dimension, seeds)
