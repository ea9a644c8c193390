"""ctypes binding of libsda_engine.so (include/sda_engine.h).

This is the Python-side consumer of the C ABI: the parity tests and bench.py call the MI355X
engine only through it.  There is deliberately no CPU fallback: if the shared library is
missing or a call fails, an exception is raised.

Trait mirrors (reference: client/src/crypto/{sharing,masking}/mod.rs):
    share_generate     ShareGenerator::generate        (sharing/mod.rs:14-17)
    share_combine      ShareCombiner::combine          (sharing/mod.rs:23-25)
    secret_reconstruct SecretReconstructor::reconstruct (sharing/mod.rs:31-33)
    secret_mask        SecretMasker::mask              (masking/mod.rs:13-15)
    mask_combine       MaskCombiner::combine           (masking/mod.rs:21-23)
    secret_unmask      SecretUnmasker::unmask          (masking/mod.rs:29-31)
    positive           RecipientOutput::positive       (receive.rs:14-20)
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from typing import Optional, Sequence

import numpy as np

from . import schemes as S

# SDA_ENGINE_LIB: developer override (A/B builds of the same ABI); the default is the in-tree build.
LIB_PATH = os.environ.get("SDA_ENGINE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsda_engine.so")

OK = 0
ERR_BATCH_INPUT_WRONG_LENGTH = 1
ERR_PACKED_SHARING_FAILED = 2
ERR_WRONG_DIMENSION = 3
ERR_MISMATCHING_DIMENSION = 4
ERR_INPUTS_MUST_HAVE_SAME_LENGTH = 5
ERR_NOT_ENOUGH_SHARES = 6
ERR_PRECONDITION = 64
ERR_INVALID_ARGUMENT = 65
ERR_UNSUPPORTED = 66
ERR_DEVICE = 67
ERR_OUT_OF_MEMORY = 68

REVEAL_EXACT = 0
REVEAL_CANONICAL = 1

_i64p = C.POINTER(C.c_int64)
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p
_st = C.c_int

# (name, restype, argtypes) for every symbol declared in include/sda_engine.h
SIGNATURES = [
    ("sda_abi_version", C.c_int, []),
    ("sda_engine_create", _st, [C.c_int, C.POINTER(_vp)]),
    ("sda_engine_destroy", None, [_vp]),
    ("sda_engine_create_multi", _st, [C.POINTER(C.c_int), C.c_int, C.POINTER(_vp)]),
    ("sda_engine_device_count", C.c_int, [_vp]),
    ("sda_engine_synchronize", _st, [_vp]),
    ("sda_last_error_message", C.c_char_p, []),
    ("sda_status_string", C.c_char_p, [C.c_int]),
    ("sda_scheme_input_size", C.c_uint64, [C.POINTER(S.SharingSchemeC)]),
    ("sda_scheme_output_size", C.c_uint64, [C.POINTER(S.SharingSchemeC)]),
    ("sda_scheme_privacy_threshold", C.c_uint64, [C.POINTER(S.SharingSchemeC)]),
    ("sda_scheme_reconstruction_threshold", C.c_uint64, [C.POINTER(S.SharingSchemeC)]),
    ("sda_share_length", C.c_uint64, [C.POINTER(S.SharingSchemeC), C.c_uint64]),
    ("sda_share_generate", _st, [_vp, C.POINTER(S.SharingSchemeC), _i64p, C.c_uint64, _i64p, C.c_uint64,
                                 _i64p, C.c_uint64]),
    ("sda_share_combine", _st, [_vp, C.POINTER(S.SharingSchemeC), C.POINTER(_i64p), _u64p, C.c_uint64,
                                _i64p, C.c_uint64, _u64p]),
    ("sda_secret_reconstruct", _st, [_vp, C.POINTER(S.SharingSchemeC), C.c_uint64, _u64p, C.POINTER(_i64p),
                                     _u64p, C.c_uint64, _i64p, C.c_uint64, _u64p]),
    ("sda_secret_mask", _st, [_vp, C.POINTER(S.MaskingSchemeC), _i64p, C.c_uint64, _u32p, C.c_uint64, _i64p,
                              _i64p, C.c_uint64, _u64p, _i64p]),
    ("sda_mask_combine", _st, [_vp, C.POINTER(S.MaskingSchemeC), C.POINTER(_i64p), _u64p, C.c_uint64, _i64p,
                               C.c_uint64, _u64p]),
    ("sda_secret_unmask", _st, [_vp, C.POINTER(S.MaskingSchemeC), _i64p, C.c_uint64, _i64p, C.c_uint64, _i64p,
                                C.c_uint64, _u64p]),
    ("sda_recipient_positive", _st, [_vp, C.c_int64, _i64p, C.c_uint64, _i64p]),
    ("sda_combine_dev", _st, [_vp, C.c_int64, _vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp, _vp]),
    ("sda_combine_finalize_dev", _st, [_vp, C.c_int64, _vp, C.c_uint64, _vp, _vp]),
    ("sda_combine_accumulate_dev", _st, [_vp, C.c_int64, _vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp, _vp]),
    ("sda_combine_split_dev", _st, [_vp, C.c_int64, _vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp, _vp, _vp]),
    ("sda_combine_split_prefix_dev", _st, [_vp, C.c_int64, _vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp, _vp, _vp,
                                           _vp]),
    ("sda_combine_split_replay_dev", _st, [_vp, C.c_int64, _vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                           _vp, _vp, _vp]),
    ("sda_combine_split_resolve_dev", _st, [_vp, C.c_int64, _vp, _vp, C.c_uint64, _vp, _vp]),
    ("sda_packed_generate_dev", _st, [_vp, C.POINTER(S.SharingSchemeC), _vp, C.c_uint64, C.c_uint64, _vp, _vp,
                                      _vp]),
    ("sda_packed_generate_mode_dev", _st, [_vp, C.POINTER(S.SharingSchemeC), _vp, C.c_uint64, C.c_uint64, _vp,
                                           _vp, C.c_int32, _vp]),
    ("sda_packed_reconstruct_dev", _st, [_vp, C.POINTER(S.SharingSchemeC), C.c_uint64, _u64p, C.c_uint64,
                                         C.c_uint64, _vp, _vp, C.c_int32, _vp]),
    ("sda_additive_generate_dev", _st, [_vp, C.c_int64, C.c_uint64, _vp, C.c_uint64, _vp, _vp, _vp]),
    ("sda_chacha_mask_combine_dev", _st, [_vp, C.c_int64, C.c_uint64, _vp, C.c_uint64, C.c_uint64, _vp, _vp]),
    ("sda_synth_fill_dev", _st, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int64, C.c_int64, _vp]),
    ("sda_hbm_alloc", _st, [C.c_int, C.c_uint64, C.POINTER(_vp)]),
    ("sda_hbm_free", _st, [_vp]),
    ("sda_hbm_trim", _st, [C.c_int, C.c_uint64]),
    ("sda_hbm_stats", _st, [C.c_int, _u64p, _u64p, _u64p]),
    ("sda_varint_encode", _st, [_vp, _i64p, C.c_uint64, _u8p, C.c_uint64, _u64p]),
    ("sda_varint_decode", _st, [_vp, _u8p, C.c_uint64, _i64p, C.c_uint64, _u64p]),
    ("sda_clerk_decode_combine", _st, [_vp, C.POINTER(S.SharingSchemeC), C.POINTER(_u8p), _u64p, C.c_uint64,
                                       _i64p, C.c_uint64, _u64p]),
    ("sda_varint_decode_dev", _st, [_vp, _vp, _u64p, C.c_uint64, _vp, C.c_uint64, _u64p, _vp]),
    ("sda_clerk_decode_combine_dev", _st, [_vp, C.c_int64, _vp, _u64p, C.c_uint64, _vp, C.c_uint64, _u64p, _vp]),
    ("sda_varint_encode_dev", _st, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp, C.c_uint64, _u64p, _vp]),
    ("sda_snapshot_transpose_dev", _st, [_vp, _vp, _u64p, C.c_uint64, C.c_uint64, _vp, C.c_uint64, _u64p, _u64p,
                                         _u64p, _vp]),
    ("sda_recipient_reveal_dev", _st, [_vp, C.POINTER(S.MaskingSchemeC), _vp, C.c_uint64, C.c_uint64,
                                       C.POINTER(S.SharingSchemeC), C.c_uint64, _u64p, _vp, C.c_uint64, C.c_uint64,
                                       C.c_int64, C.c_int32, _vp, C.c_uint64, _u64p, _vp]),
    ("sda_recipient_reveal", _st, [_vp, C.POINTER(S.MaskingSchemeC), C.POINTER(_i64p), _u64p, C.c_uint64,
                                   C.POINTER(S.SharingSchemeC), C.c_uint64, _u64p, C.POINTER(_i64p), _u64p,
                                   C.c_uint64, C.c_int64, C.c_int32, _i64p, C.c_uint64, _u64p]),
    ("sda_participant_share_dev", _st, [_vp, C.POINTER(S.MaskingSchemeC), _u32p, C.c_uint64, _vp,
                                        C.POINTER(S.SharingSchemeC), _vp, C.c_uint64, _vp, C.c_int32, _vp, _vp,
                                        C.c_uint64, _u64p, _vp]),
]

_lib = None


def load_library():
    """Load the in-tree engine library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"MI355X engine not built: {LIB_PATH} is missing (run `make` / __graft_entry__.build())")
        lib = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


class SdaError(Exception):
    """A non-OK sda_status.  `.status` is the code; for 1..6 str(e) starts with the reference's string."""

    def __init__(self, status: int, message: str):
        self.status = status
        super().__init__(message)


def _check(st: int):
    if st != OK:
        lib = load_library()
        detail = lib.sda_last_error_message().decode()
        base = lib.sda_status_string(st).decode()
        raise SdaError(st, f"{base}: {detail}" if detail and detail != base else base)


def _arr(a, dtype=np.int64):
    return np.ascontiguousarray(np.asarray(a, dtype=dtype))


def _ptr(a, t=_i64p):
    return a.ctypes.data_as(t)


def _rows(rows):
    arrs = [_arr(r) for r in rows]
    n = len(arrs)
    ptrs = (_i64p * max(n, 1))(*[_ptr(a) for a in arrs])
    lens = (C.c_uint64 * max(n, 1))(*[a.size for a in arrs])
    return arrs, ptrs, lens, n


class _HbmBlock:
    """One sda_hbm_alloc buffer, exposed through __cuda_array_interface__ so torch.as_tensor wraps it
    without a copy; torch keeps this object alive as long as the tensor, and its release frees the buffer."""

    _TYPESTR = {"torch.int64": "<i8", "torch.int32": "<i4", "torch.uint8": "|u1", "torch.float64": "<f8",
                "torch.float32": "<f4"}

    def __init__(self, lib, device, shape, dtype, nbytes):
        typestr = self._TYPESTR.get(str(dtype))
        if typestr is None:
            raise ValueError(f"hbm_empty: unsupported dtype {dtype}")
        self.lib = lib
        p = _vp()
        _check(lib.sda_hbm_alloc(device, nbytes, C.byref(p)))
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (self.ptr, False),
                                         "version": 2, "strides": None}

    def __del__(self):
        # sda_hbm_free does not wait for the device (the buffer is only pooled); at interpreter shutdown the
        # HIP runtime may already be gone, and the process exit releases everything anyway
        if getattr(self, "ptr", None) and not sys.is_finalizing():
            self.lib.sda_hbm_free(self.ptr)
        self.ptr = None


class Engine:
    """One engine handle = one HIP device + one stream (sda_engine_create), or, with `devices`, one handle over
    several devices (sda_engine_create_multi): the host trait calls then split over them; the `_dev` entry points
    run on devices[0]."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        # torch (when the caller uses it) ships its own HIP runtime; it has to open the device before
        # the engine's ROCm runtime does, or torch later reports "No HIP GPUs are available"
        t = sys.modules.get("torch")
        if t is not None and t.cuda.is_available():
            t.cuda.init()
        self.lib = load_library()
        h = _vp()
        if devices is None:
            _check(self.lib.sda_engine_create(device, C.byref(h)))
        else:
            devs = (C.c_int * max(len(devices), 1))(*devices)
            _check(self.lib.sda_engine_create_multi(devs, len(devices), C.byref(h)))
            device = int(devices[0])
        self.h = h
        self.device = device

    def device_count(self) -> int:
        """Devices the handle's host calls use (sda_engine_device_count)."""
        return int(self.lib.sda_engine_device_count(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.lib.sda_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------- trait mirrors ----------------
    def share_generate(self, scheme, secrets, draws) -> np.ndarray:
        s = scheme.c()
        sec = _arr(secrets)
        dr = _arr(draws).reshape(-1)
        B = self.lib.sda_share_length(C.byref(s), sec.size)
        n = scheme.output_size()
        out = np.zeros(max(n * B, 1), np.int64)
        _check(self.lib.sda_share_generate(self.h, C.byref(s), _ptr(sec), sec.size, _ptr(dr), dr.size, _ptr(out),
                                           out.size))
        return out[: n * B].reshape(n, B)

    def share_combine(self, scheme, rows: Sequence) -> np.ndarray:
        s = scheme.c()
        arrs, ptrs, lens, n = _rows(rows)
        cap = arrs[0].size if arrs else 0
        out = np.zeros(max(cap, 1), np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_share_combine(self.h, C.byref(s), ptrs, lens, n, _ptr(out), out.size, C.byref(olen)))
        return out[: olen.value]

    def secret_reconstruct(self, scheme, dimension: int, indexed_shares) -> np.ndarray:
        s = scheme.c()
        idx = _arr([i for i, _ in indexed_shares], np.uint64)
        arrs, ptrs, lens, n = _rows([r for _, r in indexed_shares])
        cap = max(dimension, arrs[0].size if arrs else 0, 1)
        out = np.zeros(cap, np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_secret_reconstruct(self.h, C.byref(s), dimension, _ptr(idx, _u64p), ptrs, lens, n,
                                               _ptr(out), out.size, C.byref(olen)))
        return out[: olen.value]

    def secret_mask(self, scheme, secrets, seed: Optional[Sequence[int]] = None, full_masks=None):
        s = scheme.c()
        sec = _arr(secrets)
        sd = _arr(seed if seed is not None else [], np.uint32)
        fm = _arr(full_masks) if full_masks is not None else None
        mask = np.zeros(max(sec.size, sd.size, 1), np.int64)
        masked = np.zeros(max(sec.size, 1), np.int64)
        mlen = C.c_uint64(0)
        _check(self.lib.sda_secret_mask(self.h, C.byref(s), _ptr(sec), sec.size, _ptr(sd, _u32p), sd.size,
                                        _ptr(fm) if fm is not None else None, _ptr(mask), mask.size,
                                        C.byref(mlen), _ptr(masked)))
        return mask[: mlen.value], masked[: sec.size]

    def mask_combine(self, scheme, rows: Sequence) -> np.ndarray:
        s = scheme.c()
        arrs, ptrs, lens, n = _rows(rows)
        cap = max(getattr(scheme, "dimension", 0), arrs[0].size if arrs else 0, 1)
        out = np.zeros(cap, np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_mask_combine(self.h, C.byref(s), ptrs, lens, n, _ptr(out), out.size, C.byref(olen)))
        return out[: olen.value]

    def secret_unmask(self, scheme, values) -> np.ndarray:
        s = scheme.c()
        mask, masked = _arr(values[0]), _arr(values[1])
        out = np.zeros(max(masked.size, 1), np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_secret_unmask(self.h, C.byref(s), _ptr(mask), mask.size, _ptr(masked), masked.size,
                                          _ptr(out), out.size, C.byref(olen)))
        return out[: olen.value]

    def positive(self, modulus: int, values) -> np.ndarray:
        v = _arr(values)
        out = np.zeros(max(v.size, 1), np.int64)
        _check(self.lib.sda_recipient_positive(self.h, modulus, _ptr(v), v.size, _ptr(out)))
        return out[: v.size]

    # ---------------- share payload codec (sodium.rs:36-41 / :82-88) ----------------
    def varint_encode(self, values) -> bytes:
        v = _arr(values)
        out = (C.c_uint8 * max(10 * v.size, 1))()
        olen = C.c_uint64(0)
        _check(self.lib.sda_varint_encode(self.h, _ptr(v), v.size, out, len(out), C.byref(olen)))
        return bytes(out[: olen.value])

    def varint_decode(self, data: bytes) -> np.ndarray:
        src = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
        out = np.zeros(max(len(data), 1), np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_varint_decode(self.h, src, len(data), _ptr(out), out.size, C.byref(olen)))
        return out[: olen.value]

    def clerk_decode_combine_packed(self, scheme, payload: np.ndarray, blob_off) -> np.ndarray:
        """sda_clerk_decode_combine over blobs that sit back to back in one host uint8 array (blob i =
        payload[blob_off[i]:blob_off[i + 1]]), passed as pointers into it: no per-blob copy on the Python side."""
        s = scheme.c()
        pay = np.ascontiguousarray(payload, dtype=np.uint8)
        off = _arr(blob_off, np.uint64)
        n = off.size - 1
        base = pay.ctypes.data
        ptrs = (_u8p * max(n, 1))(*[C.cast(base + int(o), _u8p) for o in off[:-1]])
        lens = (C.c_uint64 * max(n, 1))(*[int(off[i + 1] - off[i]) for i in range(n)])
        cap = int(max(np.diff(off).max(initial=0), 1))
        out = np.zeros(cap, np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_clerk_decode_combine(self.h, C.byref(s), ptrs, lens, n, _ptr(out), out.size, C.byref(olen)))
        return out[: olen.value]

    def clerk_decode_combine(self, scheme, blobs: Sequence[bytes]) -> np.ndarray:
        """clerk.rs:79-86 after the sealed-box opens: decode each participation, combine."""
        s = scheme.c()
        bufs = [(C.c_uint8 * max(len(b), 1)).from_buffer_copy(b or b"\0") for b in blobs]
        n = len(bufs)
        ptrs = (_u8p * max(n, 1))(*[C.cast(b, _u8p) for b in bufs])
        lens = (C.c_uint64 * max(n, 1))(*[len(b) for b in blobs])
        cap = max([len(b) for b in blobs] + [1])
        out = np.zeros(cap, np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_clerk_decode_combine(self.h, C.byref(s), ptrs, lens, n, _ptr(out), out.size,
                                                 C.byref(olen)))
        return out[: olen.value]

    # ---------------- fused role pipelines ----------------
    def recipient_reveal(self, masking, mask_rows, sharing, dimension: int, indexed_shares, output_modulus: int,
                         mode=REVEAL_EXACT) -> np.ndarray:
        """receive.rs:80-157 + positive() (:14-20) as one device pipeline."""
        ms, ss = masking.c(), sharing.c()
        marrs, mptrs, mlens, nm = _rows(mask_rows)
        idx = _arr([i for i, _ in indexed_shares], np.uint64)
        sarrs, sptrs, slens, ns = _rows([r for _, r in indexed_shares])
        cap = max(dimension, sarrs[0].size if sarrs else 0, 1)
        out = np.zeros(cap, np.int64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_recipient_reveal(self.h, C.byref(ms), mptrs, mlens, nm, C.byref(ss), dimension,
                                             _ptr(idx, _u64p), sptrs, slens, ns, output_modulus, mode, _ptr(out),
                                             out.size, C.byref(olen)))
        return out[: olen.value]

    def synchronize(self):
        _check(self.lib.sda_engine_synchronize(self.h))

    def hbm_empty(self, shape, dtype=None):
        """An uninitialised torch tensor on this engine's device, in an sda_hbm_alloc buffer (fixed-size
        physical chunks, DESIGN.md "HBM backing"); the buffer is released when the tensor is."""
        import torch
        dtype = dtype or torch.int64
        shape = tuple(int(s) for s in shape)
        count = 1
        for s in shape:
            count *= s
        nbytes = max(count * torch.empty((), dtype=dtype).element_size(), 1)
        return torch.as_tensor(_HbmBlock(self.lib, self.device, shape, dtype, nbytes),
                               device=torch.device("cuda", self.device))

    def hbm_trim(self, keep_bytes: int = 0):
        """Release this device's pooled sda_hbm_alloc buffers down to keep_bytes (sda_hbm_trim)."""
        _check(self.lib.sda_hbm_trim(self.device, keep_bytes))

    def hbm_stats(self):
        """(live, pooled, retired) bytes of this device's sda_hbm_alloc buffers (sda_hbm_stats)."""
        v = [C.c_uint64() for _ in range(3)]
        _check(self.lib.sda_hbm_stats(self.device, *[C.byref(x) for x in v]))
        return tuple(int(x.value) for x in v)

    # ---------------- device-resident entry points (raw device pointers, hipStream_t) ----------------
    def combine_dev(self, modulus, shares_ptr, n, dim, row_stride, out_ptr, stream=None):
        _check(self.lib.sda_combine_dev(self.h, modulus, shares_ptr, n, dim, row_stride, out_ptr, stream))

    def combine_accumulate_dev(self, modulus, shares_ptr, n, dim, row_stride, inout_ptr, stream=None):
        _check(self.lib.sda_combine_accumulate_dev(self.h, modulus, shares_ptr, n, dim, row_stride, inout_ptr,
                                                   stream))

    def combine_finalize_dev(self, modulus, sums_ptr, dim, out_ptr, stream=None):
        _check(self.lib.sda_combine_finalize_dev(self.h, modulus, sums_ptr, dim, out_ptr, stream))

    # participation split of the combine (sda_amd.distributed; include/sda_engine.h "participation split")
    def combine_split_dev(self, modulus, shares_ptr, n, dim, row_stride, inout_ptr, flags_ptr, stream=None):
        _check(self.lib.sda_combine_split_dev(self.h, modulus, shares_ptr, n, dim, row_stride, inout_ptr, flags_ptr,
                                              stream))

    def combine_split_prefix_dev(self, modulus, gathered_ptr, world, rank, dim, c_in_ptr, total_ptr, code_ptr,
                                 stream=None):
        _check(self.lib.sda_combine_split_prefix_dev(self.h, modulus, gathered_ptr, world, rank, dim, c_in_ptr,
                                                     total_ptr, code_ptr, stream))

    def combine_split_replay_dev(self, modulus, shares_ptr, n, dim, row_stride, rank, state_ptr, code_ptr,
                                 stream=None):
        _check(self.lib.sda_combine_split_replay_dev(self.h, modulus, shares_ptr, n, dim, row_stride, rank,
                                                     state_ptr, code_ptr, stream))

    def combine_split_resolve_dev(self, modulus, total_ptr, code_ptr, dim, out_ptr, stream=None):
        _check(self.lib.sda_combine_split_resolve_dev(self.h, modulus, total_ptr, code_ptr, dim, out_ptr, stream))

    def packed_generate_dev(self, scheme, secrets_ptr, dimension, n_vectors, draws_ptr, out_ptr, stream=None):
        s = scheme.c()
        _check(self.lib.sda_packed_generate_dev(self.h, C.byref(s), secrets_ptr, dimension, n_vectors, draws_ptr,
                                                out_ptr, stream))

    def packed_generate_mode_dev(self, scheme, secrets_ptr, dimension, n_vectors, draws_ptr, out_ptr, mode,
                                 stream=None):
        s = scheme.c()
        _check(self.lib.sda_packed_generate_mode_dev(self.h, C.byref(s), secrets_ptr, dimension, n_vectors,
                                                     draws_ptr, out_ptr, mode, stream))

    def packed_reconstruct_dev(self, scheme, dimension, indices, n_vectors, shares_ptr, out_ptr,
                               mode=REVEAL_EXACT, stream=None):
        s = scheme.c()
        idx = _arr(indices, np.uint64)
        _check(self.lib.sda_packed_reconstruct_dev(self.h, C.byref(s), dimension, _ptr(idx, _u64p), idx.size,
                                                   n_vectors, shares_ptr, out_ptr, mode, stream))

    def additive_generate_dev(self, modulus, share_count, secrets_ptr, dimension, draws_ptr, out_ptr, stream=None):
        _check(self.lib.sda_additive_generate_dev(self.h, modulus, share_count, secrets_ptr, dimension, draws_ptr,
                                                  out_ptr, stream))

    def chacha_mask_combine_dev(self, modulus, dimension, seeds_ptr, w, n_seeds, out_ptr, stream=None):
        _check(self.lib.sda_chacha_mask_combine_dev(self.h, modulus, dimension, seeds_ptr, w, n_seeds, out_ptr,
                                                    stream))

    def synth_fill_dev(self, dst_ptr, rows, cols, seed, lo, hi, stream=None):
        _check(self.lib.sda_synth_fill_dev(self.h, dst_ptr, rows, cols, seed, lo, hi, stream))

    def varint_decode_dev(self, bytes_ptr, blob_off, out_ptr, out_stride, stream=None) -> np.ndarray:
        off = _arr(blob_off, np.uint64)
        n = off.size - 1
        counts = np.zeros(max(n, 1), np.uint64)
        _check(self.lib.sda_varint_decode_dev(self.h, bytes_ptr, _ptr(off, _u64p), n, out_ptr, out_stride,
                                              _ptr(counts, _u64p), stream))
        return counts[:n]

    def clerk_decode_combine_dev(self, modulus, bytes_ptr, blob_off, out_ptr, out_cap, stream=None) -> int:
        off = _arr(blob_off, np.uint64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_clerk_decode_combine_dev(self.h, modulus, bytes_ptr, _ptr(off, _u64p), off.size - 1,
                                                     out_ptr, out_cap, C.byref(olen), stream))
        return olen.value

    def varint_encode_dev(self, vals_ptr, rows, length, stride, dst_ptr, dst_cap, stream=None) -> np.ndarray:
        rb = np.zeros(max(rows, 1), np.uint64)
        _check(self.lib.sda_varint_encode_dev(self.h, vals_ptr, rows, length, stride, dst_ptr, dst_cap,
                                              _ptr(rb, _u64p), stream))
        return rb[:rows]

    def snapshot_transpose_dev(self, src_ptr, part_off, n_participations, n_clerks, dst_ptr=None, dst_cap=0,
                               stream=None):
        """AggregationsStore::iter_snapshot_clerk_jobs_data (server/src/stores.rs:86-101) on device.

        part_off: [P*n + 1] offsets of the [participation][clerk] blobs in src.  Returns
        (dst_len, clerk_base [n], clerk_off [n][P+1]); dst_ptr None = sizing query."""
        off = _arr(part_off, np.uint64)
        P, n = n_participations, n_clerks
        if off.size != P * n + 1:
            raise ValueError("part_off must have n_participations * n_clerks + 1 entries")
        base = np.zeros(max(n, 1), np.uint64)
        coff = np.zeros(max(n * (P + 1), 1), np.uint64)
        dlen = C.c_uint64(0)
        _check(self.lib.sda_snapshot_transpose_dev(self.h, src_ptr, _ptr(off, _u64p), P, n, dst_ptr, dst_cap,
                                                   C.byref(dlen), _ptr(base, _u64p), _ptr(coff, _u64p), stream))
        return dlen.value, base[:n], coff[:n * (P + 1)].reshape(n, P + 1)

    def recipient_reveal_dev(self, masking, mask_ptr, n_masks, mask_width, sharing, dimension, indices, shares_ptr,
                             share_len, output_modulus, out_ptr, out_cap, mode=REVEAL_EXACT, stream=None) -> int:
        ms, ss = masking.c(), sharing.c()
        idx = _arr(indices, np.uint64)
        olen = C.c_uint64(0)
        _check(self.lib.sda_recipient_reveal_dev(self.h, C.byref(ms), mask_ptr, n_masks, mask_width, C.byref(ss),
                                                 dimension, _ptr(idx, _u64p), shares_ptr, idx.size, share_len,
                                                 output_modulus, mode, out_ptr, out_cap, C.byref(olen), stream))
        return olen.value

    def participant_share_dev(self, masking, sharing, secrets_ptr, dimension, draws_ptr, shares_ptr, seed=None,
                              full_masks_ptr=None, payload_ptr=None, payload_cap=0, mode=REVEAL_EXACT, stream=None):
        """participate.rs:53-76 (+ payload encoding) on device; returns per-clerk payload byte counts."""
        ms, ss = masking.c(), sharing.c()
        sd = _arr(seed if seed is not None else [], np.uint32)
        n = sharing.output_size()
        rb = np.zeros(max(n, 1), np.uint64)
        _check(self.lib.sda_participant_share_dev(self.h, C.byref(ms), _ptr(sd, _u32p), sd.size, full_masks_ptr,
                                                  C.byref(ss), secrets_ptr, dimension, draws_ptr, mode, shares_ptr,
                                                  payload_ptr, payload_cap, _ptr(rb, _u64p), stream))
        return rb[:n]
