"""Trait-mirror API over the CPU oracle (test infrastructure only).

Same method names and error behaviour as sda_amd.Engine so the KAT pipeline can run on either.
Error codes follow include/sda_engine.h; the oracle reports the reference's Err cases and this
wrapper re-creates the reference's panics (assert!) as PRECONDITION errors.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from sda_amd import schemes as S
from sda_amd.engine import (ERR_MISMATCHING_DIMENSION, ERR_NOT_ENOUGH_SHARES, ERR_PRECONDITION,
                            ERR_WRONG_DIMENSION, SdaError)


class OracleBackend:
    def share_generate(self, scheme, secrets, draws):
        secrets = np.asarray(secrets, np.int64)
        if isinstance(scheme, S.Additive):
            return O.additive_generate(scheme.modulus, scheme.share_count, secrets, draws)
        pp = O.packed_params(scheme.secret_count, scheme.share_count, scheme.privacy_threshold(),
                             scheme.prime_modulus, scheme.omega_secrets, scheme.omega_shares)
        return O.packed_generate(pp, secrets, draws)

    def share_combine(self, scheme, rows):
        rc, out = O.combine_rows(scheme.modulus, rows)
        if rc:
            raise SdaError(ERR_WRONG_DIMENSION, "Wrong dimension")
        return out

    def secret_reconstruct(self, scheme, dimension, indexed_shares):
        if isinstance(scheme, S.Additive):
            rc, out = O.combine_rows(scheme.modulus, [r for _, r in indexed_shares])
            if rc:
                raise SdaError(ERR_MISMATCHING_DIMENSION, "Mismatching dimension")
            return out
        pp = O.packed_params(scheme.secret_count, scheme.share_count, scheme.privacy_threshold(),
                             scheme.prime_modulus, scheme.omega_secrets, scheme.omega_shares)
        B = (dimension + scheme.secret_count - 1) // scheme.secret_count
        if B == 0:
            return np.zeros(0, np.int64)
        rows = [np.asarray(r, np.int64) for _, r in indexed_shares]
        if any(r.size < B for r in rows):
            raise SdaError(ERR_PRECONDITION, "index out of bounds")
        shares = np.stack([r[:B] for r in rows]) if rows else np.zeros((0, B), np.int64)
        rc, out = O.packed_reconstruct(pp, dimension, [i for i, _ in indexed_shares], shares)
        if rc == 6:
            raise SdaError(ERR_NOT_ENOUGH_SHARES, "Not enough shares to reconstruct")
        return out

    def secret_mask(self, scheme, secrets, seed=None, full_masks=None):
        secrets = np.asarray(secrets, np.int64)
        if isinstance(scheme, S.NoMasking):
            return np.zeros(0, np.int64), secrets.copy()
        if isinstance(scheme, S.FullMasking):
            return np.asarray(full_masks, np.int64), O.full_mask(scheme.modulus, full_masks, secrets)
        if scheme.dimension != secrets.size:
            raise SdaError(ERR_PRECONDITION, "assertion failed: dimension == secrets.len()")
        seed = np.asarray(seed, np.uint32)
        return seed.astype(np.int64), O.chacha_mask(scheme.modulus, seed, secrets)

    def mask_combine(self, scheme, rows):
        if isinstance(scheme, S.NoMasking):
            if any(len(r) for r in rows):
                raise SdaError(ERR_PRECONDITION, "assertion failed")
            return np.zeros(0, np.int64)
        if isinstance(scheme, S.FullMasking):
            rc, out = O.combine_rows(scheme.modulus, rows)
            if rc:
                raise SdaError(ERR_PRECONDITION, "assertion failed: mask.len() == dimension")
            return out
        w = max([len(r) for r in rows] + [1])
        seeds = np.zeros((len(rows), w), np.int64)
        for i, r in enumerate(rows):
            seeds[i, : len(r)] = r
        return O.chacha_mask_combine(scheme.modulus, scheme.dimension, seeds)

    def secret_unmask(self, scheme, values):
        mask, masked = (np.asarray(v, np.int64) for v in values)
        if isinstance(scheme, S.NoMasking):
            if mask.size:
                raise SdaError(ERR_PRECONDITION, "assertion failed")
            return masked.copy()
        if mask.size != masked.size:
            raise SdaError(ERR_PRECONDITION, "assertion failed: mask.len() == masked_secrets.len()")
        return O.unmask(scheme.modulus, mask, masked)

    def positive(self, modulus, values):
        return O.positive(modulus, values)
