"""CPU: the oracle against the reference's known answers and the committed golden fixtures."""
import json
import os

import numpy as np
import pytest

from sda_amd import schemes as S
from tests.oracle_backend import OracleBackend
from tests.pipeline import (FULL_LOOP_EXPECTED, FULL_LOOP_INPUTS, README_EXPECTED, README_INPUTS, Draws,
                            full_loop_variants, run_aggregation)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("variant", list(full_loop_variants()))
def test_full_loop_kat(oracle, variant):
    """integration-tests/tests/full_loop.rs:148: output.positive().values == [2, 4, 6, 8]."""
    masking, sharing = full_loop_variants()[variant]
    for seed in range(5):   # any injected randomness must give the KAT answer
        tr = run_aggregation(OracleBackend(), masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(1000 + seed))
        assert tr.positive.tolist() == FULL_LOOP_EXPECTED


def test_full_loop_packed_with_t_plus_k_clerks(oracle):
    """PackedShamir result_ready at t+k clerk results (protocol/src/crypto.rs:147-153)."""
    masking, sharing = full_loop_variants()["with_packedshamir"]
    for order in ([0, 2, 3, 4, 5, 6, 7], [7, 6, 5, 4, 3, 1, 0], [1, 2, 3, 4, 5, 6, 7]):
        tr = run_aggregation(OracleBackend(), masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(7), clerk_order=order)
        assert tr.positive.tolist() == FULL_LOOP_EXPECTED


def test_readme_walkthrough(oracle):
    """README.md:157: `0 2 2 4 4 6 6 8 8 10`."""
    tr = run_aggregation(OracleBackend(), S.NoMasking(), S.Additive(3, 433), 433, 10, README_INPUTS, Draws(3))
    assert tr.positive.tolist() == README_EXPECTED


def test_golden_traces_reproduce(oracle):
    kat = load("full_loop_kat.json")
    for name, v in kat.items():
        masking, sharing = full_loop_variants()[name]
        tr = run_aggregation(OracleBackend(), masking, sharing, 433, 4, v["inputs"], Draws(v["draw_seed"]))
        t = v["trace"]
        assert [s.tolist() for s in tr.shares] == t["shares"]
        assert [c.tolist() for c in tr.clerk_results] == t["clerk_results"]
        assert tr.masked_output.tolist() == t["masked_output"]
        assert tr.positive.tolist() == v["expected"]


def test_rfc7539_block(oracle):
    for name, v in load("chacha_rfc7539.json")["rfc7539"].items():
        assert oracle.chacha20_core(np.array(v["state"], np.uint32)).tolist() == v["out"], name


def test_rand03_streams(oracle):
    for st in load("chacha_rfc7539.json")["rand03_streams"]:
        r = oracle.Rng(st["seed"])
        assert [r.next_u32() for _ in range(8)] == st["first_u32"]
        r = oracle.Rng(st["seed"])
        assert [r.gen_range(0, st["modulus"]) for _ in st["gen_range"]] == st["gen_range"]


def test_rand03_chacharng_known_answers(oracle):
    """rand 0.3's own ChaChaRng test (src/chacha.rs test_rng_true_values): the zero key's first 32 words and,
    for the seed [0, 1, .., 7], the i-th word of the i-th block -- ChaChaRng::from_seed's key layout, its block
    counter and next_u32's order, the stream chacha.rs:36/67 draws from."""
    v = load("rand03_chacharng.json")
    r = oracle.Rng([0] * 8)
    assert [r.next_u32() for _ in range(32)] == v["zero_key_first_32_u32"]
    r = oracle.Rng(list(range(8)))
    got = []
    for _ in range(16):
        got.append(r.next_u32())
        for _ in range(16):
            r.next_u32()
    assert got == v["seed_0_to_7_word_17i"]


def test_stream_layout(oracle):
    """next_u64 = (next_u32 << 32) | next_u32; block counter starts at 0 (ChaCha20 zero key = RFC A.1#1)."""
    r = oracle.Rng([0, 0, 0, 0])
    assert r.next_u64() == (0xADE0B876 << 32) | 0x903DF1A0


def test_gen_range_rejection(oracle):
    """gen_range rejects v >= zone = u64::MAX - u64::MAX % m and draws again."""
    m = (1 << 63) + 1 if False else (1 << 62) + 1      # zone = 3 * 2^62 + 3: ~25% rejections
    zone = (2**64 - 1) - (2**64 - 1) % m
    r1, r2 = oracle.Rng([9]), oracle.Rng([9])
    got = [r1.gen_range(0, m) for _ in range(50)]
    exp = []
    while len(exp) < 50:
        v = r2.next_u64()
        if v < zone:
            exp.append(v % m)
    assert got == exp


def test_combine_cases(oracle):
    for c in load("combine_cases.json"):
        assert oracle.combine(c["m"], np.array(c["rows"], np.int64)).tolist() == c["expected"]
    # combiner.rs: the signed result depends on the participation order
    assert oracle.combine(10, np.array([[5], [5], [-3]])).tolist() == [-3]
    assert oracle.combine(10, np.array([[-3], [5], [5]])).tolist() == [7]


def test_combine_ragged_and_empty(oracle):
    rc, out = oracle.combine_rows(433, [])
    assert rc == 0 and out.size == 0
    rc, _ = oracle.combine_rows(433, [[1, 2], [3]])
    assert rc == 3                     # "Wrong dimension"


def test_additive_fixture(oracle):
    a = load("additive_cases.json")
    got = oracle.additive_generate(a["m"], a["n"], a["secrets"], a["draws"])
    assert got.tolist() == a["expected"]
    assert got[:, 0].tolist() == [400, 10, -407]          # (3 - 400) % 433 = -397; (-397 - 10) % 433 = -407


def _pp(O, sch):
    return O.packed_params(sch.secret_count, sch.share_count, sch.privacy_threshold(), sch.prime_modulus,
                           sch.omega_secrets, sch.omega_shares)


def test_packed_fixture(oracle):
    for c in load("packed_cases.json"):
        p = c["scheme"]["PackedShamir"]
        sch = S.PackedShamir(p["secret_count"], p["share_count"], p["privacy_threshold"], p["prime_modulus"],
                             p["omega_secrets"], p["omega_shares"])
        pp = _pp(oracle, sch)
        shares = oracle.packed_generate(pp, c["secrets"], c["draws"])
        assert shares.tolist() == c["shares"]
        for r in c["reveals"]:
            rc, rec = oracle.packed_reconstruct(pp, len(c["secrets"]), r["indices"], shares[r["indices"]])
            assert rc == 0 and rec.tolist() == r["expected"]


@pytest.mark.parametrize("sch", [S.FULL_LOOP_PACKED, S.CONFIG_PACKED])
def test_packed_math(oracle, sch):
    """Canonical shares are evaluations of the degree < k+t+1 polynomial through (1,0), the secrets at
    omega_secrets^i and the randomness at omega_secrets^(k+j) -- the tss definition."""
    p = sch.prime_modulus
    pp = _pp(oracle, sch)
    rng = Draws(5)
    secrets = rng.below(p, sch.secret_count)
    rand = rng.below(p - 1, sch.privacy_threshold())
    shares = oracle.packed_share(pp, secrets, rand)
    L = sch.secret_count + sch.privacy_threshold() + 1
    xs = [pow(sch.omega_secrets, i, p) for i in range(L)]
    ys = [0] + secrets.tolist() + rand.tolist()

    def f(x):   # Lagrange evaluation mod p
        acc = 0
        for i in range(L):
            num = den = 1
            for j in range(L):
                if j != i:
                    num = num * (x - xs[j]) % p
                    den = den * (xs[i] - xs[j]) % p
            acc = (acc + ys[i] * num * pow(den, p - 2, p)) % p
        return acc
    for j in range(sch.share_count):
        assert shares[j] % p == f(pow(sch.omega_shares, j + 1, p))
        assert -p < shares[j] < p


def test_config_prime_parameters():
    """configs[2]: 16 | p - 1 and 27 | p - 1; omega orders exactly 16 and 27."""
    s = S.CONFIG_PACKED
    p = s.prime_modulus
    assert p < 2**31 and all(p % d for d in range(2, int(p ** 0.5) + 1, 1) if d < 50000)
    assert pow(s.omega_secrets, 16, p) == 1 and pow(s.omega_secrets, 8, p) != 1
    assert pow(s.omega_shares, 27, p) == 1 and pow(s.omega_shares, 9, p) != 1
    f = S.FULL_LOOP_PACKED
    assert pow(f.omega_secrets, 8, 433) == 1 and pow(f.omega_secrets, 4, 433) != 1
    assert pow(f.omega_shares, 9, 433) == 1 and pow(f.omega_shares, 3, 433) != 1


def test_reconstruct_errors(oracle):
    sch = S.FULL_LOOP_PACKED
    pp = _pp(oracle, sch)
    shares = oracle.packed_generate(pp, [1, 2, 3], [1, 2, 3, 4])
    rc, _ = oracle.packed_reconstruct(pp, 3, [0, 1, 2, 3, 4, 5], shares[:6])
    assert rc == 6                     # "Not enough shares to reconstruct" (t + k = 7)


def test_masking_roundtrip(oracle):
    rng = Draws(77)
    for m in (433, 2147482801, 1 << 40):
        secrets = rng.below(m, 64)
        seed = rng.u32(4)
        masked = oracle.chacha_mask(m, seed, secrets)
        r = oracle.Rng(seed)
        mask = np.array([r.gen_range(0, m) for _ in range(64)])
        assert (oracle.unmask(m, mask, masked) % m == secrets % m).all()
        comb = oracle.chacha_mask_combine(m, 64, np.array([seed], np.int64))
        assert comb.tolist() == mask.tolist()


def test_varint_known_answers(oracle):
    """integer-encoding 1.0 VarInt for i64 = protobuf sint64: ZigZag table and LEB128 examples from
    the Protocol Buffers encoding guide (0->0, -1->1, 1->2, -2->3, 2^31-1 -> 2^32-2,
    -2^31 -> 2^32-1; 300 -> ac 02)."""
    zz = {0: 0, -1: 1, 1: 2, -2: 3, 2**31 - 1: 2**32 - 2, -(2**31): 2**32 - 1}
    for v, z in zz.items():
        enc = oracle.varint_encode(np.array([v], np.int64))
        dec, shift = 0, 0
        for b in enc:
            dec |= (b & 0x7F) << shift
            shift += 7
        assert dec == z and all(b & 0x80 for b in enc[:-1]) and not enc[-1] & 0x80
    assert oracle.varint_encode(np.array([150], np.int64)) == bytes([0xAC, 0x02])   # zigzag(150) = 300
    assert oracle.varint_encode(np.array([-2**63, 2**63 - 1], np.int64)) == bytes([0xFF] * 9 + [0x01] + [0xFE] + [0xFF] * 8 + [0x01])
    # the decode loop of sodium.rs:82-88 over malformed input (u64::decode_var: shift > 70 stops)
    assert oracle.varint_decode(bytes([0x80])).tolist() == [0]
    assert oracle.varint_decode(bytes([0xFF] * 11 + [0x01])).tolist() == [-2**63, -1]


def test_varint_codec(oracle):
    vals = np.array([0, -1, 1, 63, -64, 64, 2**62, -2**63, 2**63 - 1, 433, -432], np.int64)
    enc = oracle.varint_encode(vals)
    assert enc[:3] == bytes([0, 1, 2])          # zigzag: 0 -> 0, -1 -> 1, 1 -> 2
    assert oracle.varint_decode(enc).tolist() == vals.tolist()


def test_chacha_reject_seeds_reject_where_found(oracle):
    """tests/golden/chacha_rejects.json (the GPU search of tools/chacha_reject_search.hip): the oracle's
    rand-0.3 stream of every listed seed rejects a draw (v >= u64::MAX - u64::MAX % m) exactly at the
    reported pair and at no earlier one -- so the rejection tests' inputs really exercise the fix-up."""
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "chacha_rejects.json")))
    for m, hits in g["moduli"].items():
        m = int(m)
        zone = (2**64 - 1) - (2**64 - 1) % m
        assert len(hits) >= 5
        for s, pair in hits:
            r = oracle.Rng([s, 0x5DA, 7, 11])
            assert [i for i in range(pair + 1) if r.next_u64() >= zone] == [pair]
