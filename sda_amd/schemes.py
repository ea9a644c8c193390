"""Scheme descriptors mirroring the reference protocol enums.

protocol/src/crypto.rs:43-64   LinearMaskingScheme  { None, Full{modulus}, ChaCha{modulus, dimension, seed_bitsize} }
protocol/src/crypto.rs:79-114  LinearSecretSharingScheme { Additive{share_count, modulus}, PackedShamir{...} }
protocol/src/crypto.rs:117-155 derived sizes (input_size, output_size, privacy_threshold, reconstruction_threshold)
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

SHARING_ADDITIVE = 0
SHARING_PACKED_SHAMIR = 1
MASKING_NONE = 0
MASKING_FULL = 1
MASKING_CHACHA = 2


class SharingSchemeC(C.Structure):
    _fields_ = [("kind", C.c_int32), ("share_count", C.c_uint64), ("modulus", C.c_int64),
                ("secret_count", C.c_uint64), ("privacy_threshold", C.c_uint64),
                ("omega_secrets", C.c_int64), ("omega_shares", C.c_int64)]


class MaskingSchemeC(C.Structure):
    _fields_ = [("kind", C.c_int32), ("modulus", C.c_int64), ("dimension", C.c_uint64),
                ("seed_bitsize", C.c_uint64)]


@dataclass(frozen=True)
class Additive:
    share_count: int
    modulus: int

    def input_size(self) -> int: return 1                               # crypto.rs:120-126
    def output_size(self) -> int: return self.share_count               # crypto.rs:129-135
    def privacy_threshold(self) -> int: return self.share_count - 1     # crypto.rs:138-144
    def reconstruction_threshold(self) -> int: return self.share_count  # crypto.rs:147-153

    def c(self) -> SharingSchemeC:
        return SharingSchemeC(SHARING_ADDITIVE, self.share_count, self.modulus, 0, 0, 0, 0)


@dataclass(frozen=True)
class PackedShamir:
    secret_count: int
    share_count: int
    privacy_threshold_: int
    prime_modulus: int
    omega_secrets: int
    omega_shares: int

    def input_size(self) -> int: return self.secret_count
    def output_size(self) -> int: return self.share_count
    def privacy_threshold(self) -> int: return self.privacy_threshold_
    def reconstruction_threshold(self) -> int: return self.privacy_threshold_ + self.secret_count

    @property
    def modulus(self) -> int:
        return self.prime_modulus

    def c(self) -> SharingSchemeC:
        return SharingSchemeC(SHARING_PACKED_SHAMIR, self.share_count, self.prime_modulus, self.secret_count,
                              self.privacy_threshold_, self.omega_secrets, self.omega_shares)


@dataclass(frozen=True)
class NoMasking:
    def has_mask(self) -> bool: return False                            # crypto.rs:68-74
    def c(self) -> MaskingSchemeC: return MaskingSchemeC(MASKING_NONE, 0, 0, 0)


@dataclass(frozen=True)
class FullMasking:
    modulus: int
    def has_mask(self) -> bool: return True
    def c(self) -> MaskingSchemeC: return MaskingSchemeC(MASKING_FULL, self.modulus, 0, 0)


@dataclass(frozen=True)
class ChaChaMasking:
    modulus: int
    dimension: int
    seed_bitsize: int
    def has_mask(self) -> bool: return True
    def seed_words(self) -> int: return (self.seed_bitsize + 31) // 32  # chacha.rs:30
    def c(self) -> MaskingSchemeC:
        return MaskingSchemeC(MASKING_CHACHA, self.modulus, self.dimension, self.seed_bitsize)


# BASELINE.json configs[2] parameters (k=8, n=26, t=7): 16 | p-1 and 27 | p-1, p < 2^31
CONFIG_PACKED = PackedShamir(secret_count=8, share_count=26, privacy_threshold_=7, prime_modulus=2147482801,
                             omega_secrets=50280738, omega_shares=1761728707)
# integration-tests/tests/full_loop.rs:55-67
FULL_LOOP_PACKED = PackedShamir(secret_count=3, share_count=8, privacy_threshold_=4, prime_modulus=433,
                                omega_secrets=354, omega_shares=150)
