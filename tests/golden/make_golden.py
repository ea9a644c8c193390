"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Pinning:
  * full_loop_kat.json / readme_walkthrough.json end in the reference's own known answers
    (integration-tests/tests/full_loop.rs:148 -> [2,4,6,8]; README.md:157 -> 0 2 2 4 4 6 6 8 8 10);
    this script asserts them before writing.
  * chacha_rfc7539.json holds the RFC 7539 block-function vectors (section 2.3.2 and A.1 #1),
    typed in from the RFC, not produced by the oracle; the oracle is asserted against them.
  * rand03_chacharng.json holds the known answers of rand 0.3's own ChaChaRng test (`test_rng_true_values`
    in the crate's src/chacha.rs: 32 words of the zero key, then the i-th word of the i-th block for the
    seed [0, 1, .., 7]), typed in from that test (the crate is absent from the image); the oracle is
    asserted against them.  They pin ChaChaRng::from_seed's key layout, the block counter and next_u32's
    order, i.e. the stream chacha.rs:36/67 draws from.
  * every other value is the oracle's restatement output (a regression pin for the GPU path).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from sda_amd import schemes as S  # noqa: E402
from tests.oracle_backend import OracleBackend  # noqa: E402
from tests.pipeline import (FULL_LOOP_EXPECTED, FULL_LOOP_INPUTS, README_EXPECTED, README_INPUTS,  # noqa: E402
                            Draws, full_loop_variants, run_aggregation)

RFC7539 = {
    # section 2.3.2: key 00..1f, counter 1, nonce 000000090000004a00000000
    "2.3.2": {
        "state": [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574, 0x03020100, 0x07060504, 0x0B0A0908, 0x0F0E0D0C,
                  0x13121110, 0x17161514, 0x1B1A1918, 0x1F1E1D1C, 0x00000001, 0x09000000, 0x4A000000, 0x00000000],
        "out": [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
                0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2],
    },
    # appendix A.1 test vector #1: zero key, counter 0, zero nonce
    "A.1#1": {
        "state": [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + [0] * 12,
        "out": [0xADE0B876, 0x903DF1A0, 0xE56A5D40, 0x28BD8653, 0xB819D2BD, 0x1AED8DA0, 0xCCEF36A8, 0xC70D778B,
                0x7C5941DA, 0x8D485751, 0x3FE02477, 0x374AD8B8, 0xF4B8436A, 0x1CA11815, 0x69B687C3, 0x8665EEB2],
    },
}


def scheme_json(s):
    if isinstance(s, S.Additive):
        return {"Additive": {"share_count": s.share_count, "modulus": s.modulus}}
    if isinstance(s, S.PackedShamir):
        return {"PackedShamir": {"secret_count": s.secret_count, "share_count": s.share_count,
                                 "privacy_threshold": s.privacy_threshold(), "prime_modulus": s.prime_modulus,
                                 "omega_secrets": s.omega_secrets, "omega_shares": s.omega_shares}}
    if isinstance(s, S.NoMasking):
        return "None"
    if isinstance(s, S.FullMasking):
        return {"Full": {"modulus": s.modulus}}
    return {"ChaCha": {"modulus": s.modulus, "dimension": s.dimension, "seed_bitsize": s.seed_bitsize}}


def L(a):
    return np.asarray(a).tolist()


def trace_json(tr):
    return {"masks": [L(m) for m in tr.masks], "masked": [L(m) for m in tr.masked],
            "draws": [L(d) for d in tr.draws], "shares": [L(s) for s in tr.shares],
            "clerk_results": [L(c) for c in tr.clerk_results],
            "combined_mask": None if tr.combined_mask is None else L(tr.combined_mask),
            "masked_output": L(tr.masked_output), "output": L(tr.output), "positive": L(tr.positive)}


# rand 0.3, src/chacha.rs, test_rng_true_values: ChaChaRng::from_seed(&[0u32; 8]), 32 x next_u32 (RFC 7539
# test vectors 1 and 2: blocks 0 and 1 of the zero key) ...
RAND03_ZERO_KEY = [
    0xade0b876, 0x903df1a0, 0xe56a5d40, 0x28bd8653, 0xb819d2bd, 0x1aed8da0, 0xccef36a8, 0xc70d778b,
    0x7c5941da, 0x8d485751, 0x3fe02477, 0x374ad8b8, 0xf4b8436a, 0x1ca11815, 0x69b687c3, 0x8665eeb2,
    0xbee7079f, 0x7a385155, 0x7c97ba98, 0x0d082d73, 0xa0290fcb, 0x6965e348, 0x3e53c612, 0xed7aee32,
    0x7621b729, 0x434ee69c, 0xb03371d5, 0xd539d874, 0x281fed31, 0x45fb0a51, 0x1f0ae1ac, 0x6f4d794b]
# ... and from_seed(&[0, 1, 2, 3, 4, 5, 6, 7]): "the 17*i-th 32-bit word, i.e., the i-th word of the i-th
# 16-word block" for i = 0..15
RAND03_SEED_0_7_STRIDE17 = [
    0xf225c81a, 0x6ab1be57, 0x04d42951, 0x70858036, 0x49884684, 0x64efec72, 0x4be2d186, 0x3615b384,
    0x11cfa18e, 0xd3c50049, 0x75c775f6, 0x434c6530, 0x2c5bad8f, 0x898881dc, 0x5f1c86d9, 0xc1f8e7f4]


def checksum(words: np.ndarray):
    """sum_i w_i k_i and sum_i (w_i ^ k_i) mod 2^64, k_i = splitmix64_at(0xC5C5, i) | 1 (tests/abi_c/hbm_cycle.c)."""
    from sda_amd.synth import splitmix64_at
    w = np.ascontiguousarray(words, np.int64).reshape(-1).view(np.uint64)
    k = splitmix64_at(0xC5C5, np.arange(w.size, dtype=np.uint64)) | np.uint64(1)
    with np.errstate(over="ignore"):
        return int(np.sum(w * k, dtype=np.uint64)), int(np.sum(w ^ k, dtype=np.uint64))


def abi_c_sharegen():
    from sda_amd import synth
    sch = S.CONFIG_PACKED
    p, k, t, n, D = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count, 1_000_000
    B = D // k
    secrets = synth.fill(1, D, 0x5DA + 2, 0, p).reshape(-1)
    draws = synth.fill(B, t, 0x5DA + 3, 0, p - 1).reshape(-1)
    pp = O.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    shares = O.packed_generate(pp, secrets, draws)
    # the shares reveal to the secrets (a property check of the fixture itself)
    rc, rec = O.packed_reconstruct(pp, 4 * k, list(range(k + t)), shares[:k + t, :4])
    assert rc == 0 and (np.mod(rec, p) == secrets[:4 * k]).all()
    c1, c2 = checksum(shares)
    return {"scheme": scheme_json(sch), "dimension": D, "secret_seed": 0x5DA + 2, "draw_seed": 0x5DA + 3,
            "layout": "[n][B] clerk-major, i64", "checksum": [c1, c2],
            "secrets_checksum": list(checksum(secrets)), "draws_checksum": list(checksum(draws))}


def main():
    be = OracleBackend()
    out = {}

    # 1. full_loop.rs KAT, four variants, deterministic draws
    kat = {}
    for i, (name, (masking, sharing)) in enumerate(full_loop_variants().items()):
        seed = 0x5DA + 100 + i
        tr = run_aggregation(be, masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(seed))
        assert tr.positive.tolist() == FULL_LOOP_EXPECTED, (name, tr.positive)
        kat[name] = {"masking": scheme_json(masking), "sharing": scheme_json(sharing), "draw_seed": seed,
                     "inputs": FULL_LOOP_INPUTS, "expected": FULL_LOOP_EXPECTED, "trace": trace_json(tr)}
    out["full_loop_kat.json"] = kat

    # 2. README walkthrough (3 x 10, m = 433, Additive over 3 clerks, no masking)
    tr = run_aggregation(be, S.NoMasking(), S.Additive(3, 433), 433, 10, README_INPUTS, Draws(0x5DA + 1))
    assert tr.positive.tolist() == README_EXPECTED, tr.positive
    out["readme_walkthrough.json"] = {"masking": "None", "sharing": scheme_json(S.Additive(3, 433)),
                                      "draw_seed": 0x5DA + 1, "inputs": README_INPUTS,
                                      "expected": README_EXPECTED, "trace": trace_json(tr)}

    # 3. RFC 7539 ChaCha20 block vectors (external pin) + rand-0.3 stream-derived values
    for name, v in RFC7539.items():
        got = O.chacha20_core(np.array(v["state"], np.uint32)).tolist()
        assert got == v["out"], (name, [hex(x) for x in got])
    streams = []
    for seed_words, m, n in [([0, 0, 0, 0], 433, 16), ([1, 2, 3, 4], 433, 10), ([7], 2147482801, 24),
                             ([0xDEADBEEF, 1, 2, 3, 4, 5, 6, 7, 8, 9], 1 << 40, 12)]:
        r = O.Rng(seed_words)
        u32 = [r.next_u32() for _ in range(8)]
        r = O.Rng(seed_words)
        streams.append({"seed": seed_words, "modulus": m, "first_u32": u32,
                        "gen_range": [r.gen_range(0, m) for _ in range(n)]})
    out["chacha_rfc7539.json"] = {"rfc7539": RFC7539, "rand03_streams": streams}

    # 3b. rand 0.3 ChaChaRng's own known answers (external pin, typed in; see the module doc)
    r = O.Rng([0] * 8)
    got = [r.next_u32() for _ in range(32)]
    assert got == RAND03_ZERO_KEY, [hex(x) for x in got]
    r = O.Rng(list(range(8)))
    got = []
    for _ in range(16):
        got.append(r.next_u32())
        for _ in range(16):
            r.next_u32()
    assert got == RAND03_SEED_0_7_STRIDE17, [hex(x) for x in got]
    out["rand03_chacharng.json"] = {
        "source": "rand 0.3 src/chacha.rs test_rng_true_values (crate absent from the image; typed in)",
        "zero_key_first_32_u32": RAND03_ZERO_KEY,
        "seed_0_to_7_word_17i": RAND03_SEED_0_7_STRIDE17}

    # 4. combine order / overflow cases (combiner.rs:16-28)
    cases = [
        {"m": 10, "rows": [[5], [5], [-3]]},
        {"m": 10, "rows": [[-3], [5], [5]]},
        {"m": 433, "rows": [[432, -432, 0, 431], [432, -432, -1, 3], [-500, 1000, 433, -866]]},
        {"m": 2147482801, "rows": [[2**63 - 1, -2**63, 5], [2**63 - 1, -2**63, -7], [1, -1, 2**62]]},
        {"m": 1, "rows": [[5, -5], [7, 8]]},
        {"m": 2**62 + 3, "rows": [[2**62, -2**62, 2**63 - 1], [2**62, -2**62, 2**63 - 1]]},
    ]
    for c in cases:
        c["expected"] = O.combine(c["m"], np.array(c["rows"], np.int64)).tolist()
    out["combine_cases.json"] = cases

    # 5. additive generate with fixed draws (additive.rs:32-51): secret 3, draws [400, 10], m = 433
    add = O.additive_generate(433, 3, [3, -5, 1000], [400, 10, 0, 432, 432, 432])
    out["additive_cases.json"] = {"m": 433, "n": 3, "secrets": [3, -5, 1000], "draws": [400, 10, 0, 432, 432, 432],
                                  "expected": add.tolist()}

    # 6. packed shamir share / reconstruct at both parameter sets
    packed = []
    for sch, seed in [(S.FULL_LOOP_PACKED, 11), (S.CONFIG_PACKED, 12)]:
        pp = O.packed_params(sch.secret_count, sch.share_count, sch.privacy_threshold(), sch.prime_modulus,
                             sch.omega_secrets, sch.omega_shares)
        rng = Draws(seed)
        D = 5 * sch.secret_count - 1                # ragged tail batch
        secrets = rng.below(sch.prime_modulus, D) - sch.prime_modulus // 2
        B = (D + sch.secret_count - 1) // sch.secret_count
        draws = rng.below(sch.prime_modulus - 1, B * sch.privacy_threshold())
        shares = O.packed_generate(pp, secrets, draws)
        reveals = []
        n = sch.share_count
        for subset in [list(range(n)), list(range(n))[::-1],
                       list(range(1, n)),
                       list(range(n - sch.reconstruction_threshold(), n))]:
            rc, rec = O.packed_reconstruct(pp, D, subset, shares[subset])
            assert rc == 0
            reveals.append({"indices": subset, "expected": rec.tolist()})
            assert (np.mod(rec, sch.prime_modulus) == np.mod(secrets, sch.prime_modulus)).all()
        packed.append({"scheme": scheme_json(sch), "secrets": secrets.tolist(), "draws": draws.tolist(),
                       "shares": shares.tolist(), "reveals": reveals})
    out["packed_cases.json"] = packed

    # 7. configs[2] at 1M-dim for the torch-free C consumer (tests/abi_c/hbm_cycle.c `gen`): the inputs of
    #    sda_synth_fill_dev (seeds 0x5DA + 2 / + 3), the oracle's tss shares, two order-sensitive checksums
    out["abi_c_sharegen.json"] = abi_c_sharegen()

    for name, obj in out.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
