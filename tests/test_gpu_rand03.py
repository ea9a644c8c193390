"""The device ChaCha stream against rand 0.3's own ChaChaRng known answers (tests/golden/rand03_chacharng.json,
from the crate's test_rng_true_values).  With m = 2^32, gen_range(0, m) returns the low word of
next_u64 = (next_u32 << 32) | next_u32, i.e. stream word 2i + 1 for element i (no pair is rejected: none of
these high words is 0xFFFFFFFF).  So SecretMasker::mask (chacha.rs:25-53) over zero secrets exposes the odd
words of the stream, and MaskCombiner::combine (chacha.rs:57-76) of one seed the same."""
import json
import os

import numpy as np
import pytest

from sda_amd import schemes as S

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rand03_chacharng.json")


def _v():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("call", ["mask", "mask_combine"])
def test_device_stream_matches_rand03_known_answers(engine, call):
    v = _v()
    m = 1 << 32
    cases = [([0] * 8, {i: v["zero_key_first_32_u32"][2 * i + 1] for i in range(16)}),
             (list(range(8)), {(17 * i - 1) // 2: v["seed_0_to_7_word_17i"][i] for i in range(1, 16, 2)})]
    for seed, want in cases:
        D = max(want) + 1
        ms = S.ChaChaMasking(m, D, 256)
        if call == "mask":
            _, got = engine.secret_mask(ms, np.zeros(D, np.int64), seed=seed)
        else:
            got = engine.mask_combine(ms, [seed])
        for i, w in want.items():
            assert int(got[i]) == w, (seed, i, hex(int(got[i])), hex(w))
