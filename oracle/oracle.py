"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference (baajur/sda) hot path; see sda_oracle.h
for what each function restates and how it is pinned.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_i64p = C.POINTER(C.c_int64)
_u32p = C.POINTER(C.c_uint32)
_szp = C.POINTER(C.c_size_t)


class PackedParams(C.Structure):
    _fields_ = [("secret_count", C.c_size_t), ("share_count", C.c_size_t),
                ("privacy_threshold", C.c_size_t), ("prime", C.c_int64),
                ("omega_secrets", C.c_int64), ("omega_shares", C.c_int64)]


class ChaChaRng(C.Structure):
    _fields_ = [("state", C.c_uint32 * 16), ("buffer", C.c_uint32 * 16), ("index", C.c_size_t)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle not built: {_LIB_PATH} (run `make oracle`)")
        L = C.CDLL(_LIB_PATH)
        L.or_rem.restype = C.c_int64
        L.or_rem.argtypes = [C.c_int64, C.c_int64]
        L.or_combine.argtypes = [C.c_int64, _i64p, C.c_size_t, C.c_size_t, _i64p]
        L.or_combine_mt.argtypes = [C.c_int64, _i64p, C.c_size_t, C.c_size_t, _i64p, C.c_int]
        L.or_combine_mt.restype = C.c_int
        L.or_combine_rows.argtypes = [C.c_int64, C.POINTER(_i64p), _szp, C.c_size_t, _i64p, _szp]
        L.or_combine_rows.restype = C.c_int
        L.or_additive_generate.argtypes = [C.c_int64, C.c_size_t, _i64p, C.c_size_t, _i64p, _i64p]
        L.or_mod_pow.restype = C.c_int64
        L.or_mod_pow.argtypes = [C.c_int64, C.c_uint32, C.c_int64]
        L.or_mod_inverse.restype = C.c_int64
        L.or_mod_inverse.argtypes = [C.c_int64, C.c_int64]
        L.or_packed_share.argtypes = [C.POINTER(PackedParams), _i64p, _i64p, _i64p]
        L.or_packed_generate.argtypes = [C.POINTER(PackedParams), _i64p, C.c_size_t, _i64p, _i64p]
        L.or_packed_reconstruct.argtypes = [C.POINTER(PackedParams), C.c_size_t, _szp, C.c_size_t, _i64p, _i64p]
        L.or_packed_reconstruct.restype = C.c_int
        L.or_chacha20_core.argtypes = [_u32p, _u32p]
        L.or_chacha_rng_from_seed.argtypes = [C.POINTER(ChaChaRng), _u32p, C.c_size_t]
        L.or_chacha_next_u32.restype = C.c_uint32
        L.or_chacha_next_u32.argtypes = [C.POINTER(ChaChaRng)]
        L.or_chacha_next_u64.restype = C.c_uint64
        L.or_chacha_next_u64.argtypes = [C.POINTER(ChaChaRng)]
        L.or_chacha_gen_range.restype = C.c_int64
        L.or_chacha_gen_range.argtypes = [C.POINTER(ChaChaRng), C.c_int64, C.c_int64]
        L.or_chacha_mask.argtypes = [C.c_int64, _u32p, C.c_size_t, _i64p, C.c_size_t, _i64p]
        L.or_chacha_mask_combine.argtypes = [C.c_int64, C.c_size_t, _i64p, C.c_size_t, C.c_size_t, _i64p]
        L.or_unmask.argtypes = [C.c_int64, _i64p, _i64p, C.c_size_t, _i64p]
        L.or_full_mask.argtypes = [C.c_int64, _i64p, _i64p, C.c_size_t, _i64p]
        L.or_positive.argtypes = [C.c_int64, _i64p, C.c_size_t, _i64p]
        L.or_varint_encode.restype = C.c_size_t
        L.or_varint_encode.argtypes = [_i64p, C.c_size_t, C.POINTER(C.c_uint8)]
        L.or_varint_decode.restype = C.c_size_t
        L.or_varint_decode.argtypes = [C.POINTER(C.c_uint8), C.c_size_t, _i64p, C.c_size_t]
        L.or_snapshot_transpose.argtypes = [C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.c_size_t, C.c_size_t,
                                            C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)]
        _lib = L
    return _lib


def _i64(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(_i64p)


def _u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a, a.ctypes.data_as(_u32p)


def rem(a: int, m: int) -> int:
    return lib().or_rem(a, m)


def combine(m: int, shares) -> np.ndarray:
    """combiner.rs:16-28 over a dense [N][dim] array."""
    s, sp = _i64(shares)
    n, dim = (s.shape if s.ndim == 2 else (0, 0))
    out, op = _i64(np.zeros(dim, np.int64))
    lib().or_combine(m, sp, n, dim, op)
    return out


def combine_mt(m: int, shares, threads: int) -> np.ndarray:
    """combine() with the columns split over `threads` POSIX threads (CPU baseline, all cores)."""
    s, sp = _i64(shares)
    n, dim = (s.shape if s.ndim == 2 else (0, 0))
    out, op = _i64(np.zeros(dim, np.int64))
    lib().or_combine_mt(m, sp, n, dim, op, threads)
    return out


def combine_rows(m: int, rows):
    """combiner.rs:16-28 over a ragged list; returns (err_code, result)."""
    arrs = [np.ascontiguousarray(r, dtype=np.int64) for r in rows]
    ptrs = (_i64p * max(1, len(arrs)))(*[a.ctypes.data_as(_i64p) for a in arrs])
    lens = (C.c_size_t * max(1, len(arrs)))(*[len(a) for a in arrs])
    cap = len(arrs[0]) if arrs else 0
    out, op = _i64(np.zeros(max(cap, 1), np.int64))
    olen = C.c_size_t(0)
    rc = lib().or_combine_rows(m, ptrs, lens, len(arrs), op, C.byref(olen))
    return rc, out[: olen.value]


def additive_generate(m: int, n: int, secrets, draws) -> np.ndarray:
    s, sp = _i64(secrets)
    d, dp = _i64(draws)
    assert d.size == s.size * (n - 1)
    out, op = _i64(np.zeros((n, s.size), np.int64))
    lib().or_additive_generate(m, n, sp, s.size, dp, op)
    return out


def packed_params(k, n, t, p, ws, wn) -> PackedParams:
    return PackedParams(k, n, t, p, ws, wn)


def packed_share(pp: PackedParams, secrets, randomness) -> np.ndarray:
    s, sp = _i64(secrets)
    r, rp = _i64(randomness)
    out, op = _i64(np.zeros(pp.share_count, np.int64))
    lib().or_packed_share(C.byref(pp), sp, rp, op)
    return out


def packed_generate(pp: PackedParams, secrets, randomness) -> np.ndarray:
    s, sp = _i64(secrets)
    B = (s.size + pp.secret_count - 1) // pp.secret_count
    r, rp = _i64(randomness)
    assert r.size == B * pp.privacy_threshold
    out, op = _i64(np.zeros((pp.share_count, B), np.int64))
    lib().or_packed_generate(C.byref(pp), sp, s.size, rp, op)
    return out


def packed_reconstruct(pp: PackedParams, dimension: int, indices, shares):
    idx = np.ascontiguousarray(indices, dtype=np.uint64)
    s, sp = _i64(shares)
    out, op = _i64(np.zeros(max(dimension, 1), np.int64))
    rc = lib().or_packed_reconstruct(C.byref(pp), dimension, idx.ctypes.data_as(_szp), idx.size, sp, op)
    return rc, out[:dimension]


def chacha20_core(state16) -> np.ndarray:
    s, sp = _u32(state16)
    out, op = _u32(np.zeros(16, np.uint32))
    lib().or_chacha20_core(sp, op)
    return out


class Rng:
    """rand-0.3 ChaChaRng restated (from_seed, next_u32, next_u64, gen_range)."""

    def __init__(self, seed_words):
        self._st = ChaChaRng()
        s, sp = _u32(seed_words)
        lib().or_chacha_rng_from_seed(C.byref(self._st), sp, s.size)

    def next_u32(self) -> int:
        return lib().or_chacha_next_u32(C.byref(self._st))

    def next_u64(self) -> int:
        return lib().or_chacha_next_u64(C.byref(self._st))

    def gen_range(self, low: int, high: int) -> int:
        return lib().or_chacha_gen_range(C.byref(self._st), low, high)


def chacha_mask(m: int, seed_words, secrets) -> np.ndarray:
    sw, swp = _u32(seed_words)
    s, sp = _i64(secrets)
    out, op = _i64(np.zeros(s.size, np.int64))
    lib().or_chacha_mask(m, swp, sw.size, sp, s.size, op)
    return out


def chacha_mask_combine(m: int, dimension: int, seeds_as_i64) -> np.ndarray:
    s, sp = _i64(seeds_as_i64)
    N, w = s.shape if s.ndim == 2 else (0, 0)
    out, op = _i64(np.zeros(max(dimension, 1), np.int64))
    lib().or_chacha_mask_combine(m, dimension, sp, w, N, op)
    return out[:dimension]


def unmask(q: int, masks, masked) -> np.ndarray:
    a, ap = _i64(masks)
    b, bp = _i64(masked)
    out, op = _i64(np.zeros(a.size, np.int64))
    lib().or_unmask(q, ap, bp, a.size, op)
    return out


def full_mask(m: int, masks, secrets) -> np.ndarray:
    a, ap = _i64(masks)
    b, bp = _i64(secrets)
    out, op = _i64(np.zeros(a.size, np.int64))
    lib().or_full_mask(m, ap, bp, a.size, op)
    return out


def positive(m: int, vals) -> np.ndarray:
    a, ap = _i64(vals)
    out, op = _i64(np.zeros(a.size, np.int64))
    lib().or_positive(m, ap, a.size, op)
    return out


def varint_encode(vals) -> bytes:
    a, ap = _i64(vals)
    buf = (C.c_uint8 * (10 * max(1, a.size)))()
    n = lib().or_varint_encode(ap, a.size, buf)
    return bytes(buf[:n])


def varint_decode(data: bytes) -> np.ndarray:
    src = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    out, op = _i64(np.zeros(max(1, len(data)), np.int64))
    n = lib().or_varint_decode(src, len(data), op, out.size)
    return out[:n]


def snapshot_transpose(blobs):
    """server/src/stores.rs:86-101 iter_snapshot_clerk_jobs_data: blobs[p][c] (bytes) ->
    per clerk the list of its blobs in snapshot order (restated in C: or_snapshot_transpose)."""
    P = len(blobs)
    n = len(blobs[0]) if P else 0
    flat = b"".join(b for row in blobs for b in row)
    off = np.concatenate([[0], np.cumsum([len(b) for row in blobs for b in row])]).astype(np.uint64)
    src = (C.c_uint8 * max(1, len(flat))).from_buffer_copy(flat or b"\0")
    out = (C.c_uint8 * max(1, len(flat)))()
    coff = np.zeros(max(1, n * (P + 1)), np.uint64)
    lib().or_snapshot_transpose(src, off.ctypes.data_as(C.POINTER(C.c_uint64)), P, n, out,
                                coff.ctypes.data_as(C.POINTER(C.c_uint64)))
    data = bytes(out[:len(flat)])
    coff = coff[:n * (P + 1)].reshape(n, P + 1)
    return [[data[coff[c, p]:coff[c, p + 1]] for p in range(P)] for c in range(n)]
