"""End-to-end aggregation flow used by the KAT tests, over any backend with the trait-mirror API
(sda_amd.Engine, or tests.oracle_backend.OracleBackend).

It follows the reference workflows step by step:
  participate  client/src/participate.rs:53-76   mask -> share-generate (per participant)
  snapshot     server/src/stores.rs:86-101       transpose [participation][clerk] -> [clerk][participation]
  clerk        client/src/clerk.rs:79-86         combine the clerk's shares in snapshot order
  reveal       client/src/receive.rs:102-152     mask-combine, reconstruct(indexed), unmask
  output       client/src/receive.rs:14-20       RecipientOutput::positive
OsRng draws are replaced by explicit randomness from a deterministic generator (`Draws`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from sda_amd import schemes as S
from sda_amd.synth import splitmix64_at


class Draws:
    """Deterministic stand-in for OsRng: a splitmix64 stream, mapped into [0, hi)."""

    def __init__(self, seed: int):
        self.seed = seed
        self.pos = 0

    def u64(self, n: int) -> np.ndarray:
        v = splitmix64_at(self.seed, np.arange(self.pos, self.pos + n, dtype=np.uint64))
        self.pos += n
        return v

    def below(self, hi: int, n: int) -> np.ndarray:
        return (self.u64(n) % np.uint64(hi)).astype(np.int64)

    def u32(self, n: int) -> np.ndarray:
        return (self.u64(n) >> np.uint64(32)).astype(np.uint32)


@dataclass
class AggregationTrace:
    masks: List[np.ndarray] = field(default_factory=list)
    masked: List[np.ndarray] = field(default_factory=list)
    draws: List[np.ndarray] = field(default_factory=list)
    shares: List[np.ndarray] = field(default_factory=list)          # per participant [n][B]
    clerk_results: List[np.ndarray] = field(default_factory=list)   # per clerk [B]
    combined_mask: Optional[np.ndarray] = None
    masked_output: Optional[np.ndarray] = None
    output: Optional[np.ndarray] = None
    positive: Optional[np.ndarray] = None


def sharing_draws(sharing, dimension: int, rng: Draws) -> np.ndarray:
    if isinstance(sharing, S.Additive):          # additive.rs:42-44 gen_range(0, modulus)
        return rng.below(sharing.modulus, dimension * (sharing.share_count - 1))
    k, t = sharing.secret_count, sharing.privacy_threshold()
    B = (dimension + k - 1) // k                  # tss Range::new(0, p - 1)
    return rng.below(sharing.prime_modulus - 1, B * t)


def run_aggregation(be, masking, sharing, modulus: int, dimension: int, inputs, rng: Draws,
                    clerk_order=None, trace: Optional[AggregationTrace] = None) -> AggregationTrace:
    tr = trace or AggregationTrace()
    n = sharing.output_size()
    for secrets in inputs:
        secrets = np.asarray(secrets, dtype=np.int64)
        if isinstance(masking, S.NoMasking):
            mask, masked = be.secret_mask(masking, secrets)
        elif isinstance(masking, S.FullMasking):
            mask, masked = be.secret_mask(masking, secrets, full_masks=rng.below(masking.modulus, dimension))
        else:
            mask, masked = be.secret_mask(masking, secrets, seed=rng.u32(masking.seed_words()))
        draws = sharing_draws(sharing, dimension, rng)
        shares = be.share_generate(sharing, masked, draws)
        tr.masks.append(np.asarray(mask))
        tr.masked.append(np.asarray(masked))
        tr.draws.append(np.asarray(draws))
        tr.shares.append(np.asarray(shares))
    # clerks: one combine per committee member, participations in snapshot order
    tr.clerk_results = [np.asarray(be.share_combine(sharing, [sh[c] for sh in tr.shares])) for c in range(n)]
    if masking.has_mask():
        tr.combined_mask = np.asarray(be.mask_combine(masking, tr.masks))
        mask = tr.combined_mask
    else:
        mask = np.zeros(0, np.int64)
    order = list(range(n)) if clerk_order is None else list(clerk_order)
    indexed = [(c, tr.clerk_results[c]) for c in order]
    tr.masked_output = np.asarray(be.secret_reconstruct(sharing, dimension, indexed))
    tr.output = np.asarray(be.secret_unmask(masking, (mask, tr.masked_output)))
    tr.positive = np.asarray(be.positive(modulus, tr.output))
    return tr


# integration-tests/tests/full_loop.rs:11-67 -- the four aggregation variants
def full_loop_variants():
    add = S.Additive(share_count=3, modulus=433)
    return {
        "simple": (S.NoMasking(), add),
        "with_fullmask": (S.FullMasking(modulus=433), add),
        "with_chachamask": (S.ChaChaMasking(modulus=433, dimension=4, seed_bitsize=128), add),
        "with_packedshamir": (S.NoMasking(), S.FULL_LOOP_PACKED),
    }


FULL_LOOP_INPUTS = [[1, 2, 3, 4], [1, 2, 3, 4]]          # full_loop.rs:114
FULL_LOOP_EXPECTED = [2, 4, 6, 8]                          # full_loop.rs:148
README_INPUTS = [[0, 1, 2, 3, 4, 5, 6, 7, 8, 9], [0] * 10, [0, 1] * 5]   # README.md:105-107
README_EXPECTED = [0, 2, 2, 4, 4, 6, 6, 8, 8, 10]                         # README.md:157
