"""GPU parity: the MI355X engine (through the C ABI) against the CPU oracle and golden fixtures.

Bar: bit-exact (integer work).  Sizes are ones the oracle finishes in seconds; the full-size
configurations are covered by size-independent properties in test_gpu_device.py.
"""
import json
import math
import os

import numpy as np
import pytest

from sda_amd import SdaError, schemes as S
from sda_amd import engine as E
from tests.oracle_backend import OracleBackend
from tests.util import assert_same
from tests.pipeline import (FULL_LOOP_EXPECTED, FULL_LOOP_INPUTS, README_EXPECTED, README_INPUTS, Draws,
                            full_loop_variants, run_aggregation)

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
I64_MIN, I64_MAX = -(2**63), 2**63 - 1


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _pp(O, sch):
    return O.packed_params(sch.secret_count, sch.share_count, sch.privacy_threshold(), sch.prime_modulus,
                           sch.omega_secrets, sch.omega_shares)


# ------------------------------------------------------------------ end-to-end KATs
@pytest.mark.parametrize("variant", list(full_loop_variants()))
def test_full_loop_kat_trace(engine, variant):
    """Every stage of integration-tests/tests/full_loop.rs, bit-exact against the golden trace."""
    v = load("full_loop_kat.json")[variant]
    masking, sharing = full_loop_variants()[variant]
    tr = run_aggregation(engine, masking, sharing, 433, 4, v["inputs"], Draws(v["draw_seed"]))
    t = v["trace"]
    assert [m.tolist() for m in tr.masks] == t["masks"]
    assert [m.tolist() for m in tr.masked] == t["masked"]
    assert [s.tolist() for s in tr.shares] == t["shares"]
    assert [c.tolist() for c in tr.clerk_results] == t["clerk_results"]
    assert (None if tr.combined_mask is None else tr.combined_mask.tolist()) == t["combined_mask"]
    assert tr.masked_output.tolist() == t["masked_output"]
    assert tr.output.tolist() == t["output"]
    assert tr.positive.tolist() == FULL_LOOP_EXPECTED


@pytest.mark.parametrize("variant", list(full_loop_variants()))
def test_full_loop_kat_many_draws(engine, oracle, variant):
    masking, sharing = full_loop_variants()[variant]
    for seed in range(4):
        a = run_aggregation(engine, masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(seed))
        b = run_aggregation(OracleBackend(), masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(seed))
        assert_same(a.masked_output, b.masked_output)
        assert a.positive.tolist() == FULL_LOOP_EXPECTED


def test_full_loop_packed_subsets(engine, oracle):
    masking, sharing = full_loop_variants()["with_packedshamir"]
    for order in ([0, 2, 3, 4, 5, 6, 7], [7, 6, 5, 4, 3, 1, 0], [1, 2, 3, 4, 5, 6, 7]):
        a = run_aggregation(engine, masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(7), clerk_order=order)
        b = run_aggregation(OracleBackend(), masking, sharing, 433, 4, FULL_LOOP_INPUTS, Draws(7), clerk_order=order)
        assert_same(a.masked_output, b.masked_output)
        assert a.positive.tolist() == FULL_LOOP_EXPECTED


def test_readme_walkthrough(engine):
    v = load("readme_walkthrough.json")
    tr = run_aggregation(engine, S.NoMasking(), S.Additive(3, 433), 433, 10, README_INPUTS, Draws(v["draw_seed"]))
    assert [c.tolist() for c in tr.clerk_results] == v["trace"]["clerk_results"]
    assert tr.positive.tolist() == README_EXPECTED


# ------------------------------------------------------------------ combine (north-star kernel 1)
def test_combine_golden_cases(engine):
    for c in load("combine_cases.json"):
        got = engine.share_combine(S.Additive(3, c["m"]), c["rows"])
        assert got.tolist() == c["expected"], c


@pytest.mark.parametrize("m", [433, 2147482801, 1, 2, (1 << 40) + 7, (1 << 62) + 3, I64_MAX])
@pytest.mark.parametrize("N,D", [(1, 1), (3, 10), (17, 1001), (64, 4096), (300, 2049), (2, 100003)])
def test_combine_random(engine, oracle, m, N, D):
    rng = np.random.default_rng(N * 7919 + D + m % 1000)
    for kind in ("canonical", "signed", "wide"):
        if kind == "canonical":
            x = rng.integers(0, m, size=(N, D), dtype=np.int64, endpoint=False)
        elif kind == "signed":
            x = rng.integers(-(m - 1), m, size=(N, D), dtype=np.int64) if m > 1 else np.zeros((N, D), np.int64)
        else:
            x = rng.integers(I64_MIN, I64_MAX, size=(N, D), dtype=np.int64, endpoint=True)
        got = engine.share_combine(S.Additive(3, m), list(x))
        assert_same(got, oracle.combine(m, x), kind)


def test_combine_negative_modulus_and_errors(engine, oracle):
    x = np.array([[5, -7, 12], [9, 3, -20]], np.int64)
    assert_same(engine.share_combine(S.Additive(3, -10), list(x)), oracle.combine(-10, x))
    assert engine.share_combine(S.Additive(3, 433), []).tolist() == []
    with pytest.raises(SdaError) as ei:
        engine.share_combine(S.Additive(3, 433), [[1, 2], [3]])
    assert ei.value.status == E.ERR_WRONG_DIMENSION and str(ei.value).startswith("Wrong dimension")
    with pytest.raises(SdaError) as ei:
        engine.share_combine(S.Additive(3, 0), [[1, 2]])
    assert ei.value.status == E.ERR_PRECONDITION
    # m = 0 with a later row of another length: combiner.rs:20-25 folds row 0 first, so `%= 0` panics
    # before row 1's length is checked; with an empty row 0 nothing is folded and the length check wins
    with pytest.raises(SdaError) as ei:
        engine.share_combine(S.Additive(3, 0), [[1, 2], [3]])
    assert ei.value.status == E.ERR_PRECONDITION
    with pytest.raises(SdaError) as ei:
        engine.share_combine(S.Additive(3, 0), [[], [3]])
    assert ei.value.status == E.ERR_WRONG_DIMENSION
    with pytest.raises(SdaError) as ei:
        engine.secret_reconstruct(S.Additive(3, 0), 2, [(0, [1, 2]), (1, [1])])
    assert ei.value.status == E.ERR_PRECONDITION


def test_additive_reconstruct_is_combine(engine, oracle):
    rows = [np.array([1, -2, 400]), np.array([432, 5, 100]), np.array([-431, 0, -1])]
    got = engine.secret_reconstruct(S.Additive(3, 433), 3, [(2, rows[0]), (0, rows[1]), (1, rows[2])])
    assert_same(got, oracle.combine(433, np.stack(rows)))
    with pytest.raises(SdaError) as ei:
        engine.secret_reconstruct(S.Additive(3, 433), 3, [(0, [1, 2]), (1, [1])])
    assert ei.value.status == E.ERR_MISMATCHING_DIMENSION


# ------------------------------------------------------------------ additive generate
def test_additive_fixture(engine):
    a = load("additive_cases.json")
    got = engine.share_generate(S.Additive(a["n"], a["m"]), a["secrets"], a["draws"])
    assert got.tolist() == a["expected"]


@pytest.mark.parametrize("n", [1, 2, 3, 26])
@pytest.mark.parametrize("m", [433, 2147482801, (1 << 62) + 3])
def test_additive_generate_random(engine, oracle, n, m):
    rng = np.random.default_rng(n * 31 + m % 97)
    D = 5000
    secrets = rng.integers(I64_MIN, I64_MAX, size=D, dtype=np.int64, endpoint=True)
    secrets[: D // 2] = rng.integers(-(m - 1), m, size=D // 2, dtype=np.int64)
    draws = rng.integers(0, m, size=D * (n - 1), dtype=np.int64)
    got = engine.share_generate(S.Additive(n, m), secrets, draws)
    assert_same(got, oracle.additive_generate(m, n, secrets, draws))


# ------------------------------------------------------------------ packed Shamir (north-star kernel 2)
def _roots(p, L, N3):
    """order-L and order-N3 roots of unity mod p (smallest generator)."""
    fac, x, d = set(), p - 1, 2
    while d * d <= x:
        while x % d == 0:
            fac.add(d)
            x //= d
        d += 1
    if x > 1:
        fac.add(x)
    g = next(g for g in range(2, p) if all(pow(g, (p - 1) // q, p) != 1 for q in fac))
    return pow(g, (p - 1) // L, p), pow(g, (p - 1) // N3, p)


def _prime_for(L, N3, below=2**31):
    step = L * N3 // math.gcd(L, N3)
    c = (below - 1) // step
    while True:
        p = c * step + 1
        if p < below and all(p % q for q in range(2, int(p**0.5) + 1)):
            return p
        c -= 1


def packed_schemes():
    out = [S.FULL_LOOP_PACKED, S.CONFIG_PACKED]
    for k, t, n in [(1, 0, 2), (3, 4, 26), (7, 8, 26), (1, 2, 8), (15, 16, 80), (8, 7, 80), (31, 32, 80)]:
        L, N3 = k + t + 1, n + 1
        p = _prime_for(L, N3) if (L, N3) != (8, 27) else 433
        ws, wn = _roots(p, L, N3)
        out.append(S.PackedShamir(k, n, t, p, ws, wn))
    return out


def test_packed_fixture(engine):
    for c in load("packed_cases.json"):
        p = c["scheme"]["PackedShamir"]
        sch = S.PackedShamir(p["secret_count"], p["share_count"], p["privacy_threshold"], p["prime_modulus"],
                             p["omega_secrets"], p["omega_shares"])
        shares = engine.share_generate(sch, c["secrets"], c["draws"])
        assert shares.tolist() == c["shares"]
        for r in c["reveals"]:
            got = engine.secret_reconstruct(sch, len(c["secrets"]), [(i, shares[i]) for i in r["indices"]])
            assert got.tolist() == r["expected"]


@pytest.mark.parametrize("sch", packed_schemes(), ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_generate_random(engine, oracle, sch):
    p = sch.prime_modulus
    rng = np.random.default_rng(p % 1000 + sch.share_count)
    D = 37 * sch.secret_count + 1 if sch.secret_count > 1 else 300
    B = (D + sch.secret_count - 1) // sch.secret_count
    secrets = rng.integers(-(p - 1), p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    got = engine.share_generate(sch, secrets, draws)
    exp = oracle.packed_generate(_pp(oracle, sch), secrets, draws)
    assert_same(got, exp)
    # raw i64 secrets outside (-p, p): generic exact path (wrapping i64, tss order)
    wide = secrets.copy()
    wide[::5] = rng.integers(-(2**40), 2**40, size=wide[::5].size, dtype=np.int64)
    got = engine.share_generate(sch, wide, draws)
    assert_same(got, oracle.packed_generate(_pp(oracle, sch), wide, draws))


@pytest.mark.parametrize("sch", packed_schemes(), ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_reconstruct_random(engine, oracle, sch):
    p, n = sch.prime_modulus, sch.share_count
    n_max = n                      # batched.rs:75 uses every supplied share: up to all n clerks
    rng = np.random.default_rng(p % 777 + n)
    D = 23 * sch.secret_count + 1
    B = (D + sch.secret_count - 1) // sch.secret_count
    secrets = rng.integers(0, p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    shares = oracle.packed_generate(_pp(oracle, sch), secrets, draws)
    need = sch.reconstruction_threshold()
    for trial in range(5):
        size = n_max if trial == 0 else int(rng.integers(need, n_max + 1))
        idx = rng.permutation(n)[:size].tolist()
        got = engine.secret_reconstruct(sch, D, [(i, shares[i]) for i in idx])
        rc, exp = oracle.packed_reconstruct(_pp(oracle, sch), D, idx, shares[idx])
        assert rc == 0
        assert_same(got, exp)
        assert (got % p == secrets % p).all()
    # shares outside (-p, p) (e.g. combined shares fed in raw): generic exact path
    idx = list(range(need))
    raw = shares[idx].copy()
    raw[0, ::3] += 5 * p
    got = engine.secret_reconstruct(sch, D, [(i, raw[j]) for j, i in enumerate(idx)])
    rc, exp = oracle.packed_reconstruct(_pp(oracle, sch), D, idx, raw)
    assert_same(got, exp)


def test_packed_errors(engine):
    sch = S.FULL_LOOP_PACKED
    shares = engine.share_generate(sch, [1, 2, 3], [1, 2, 3, 4])
    with pytest.raises(SdaError) as ei:
        engine.secret_reconstruct(sch, 3, [(i, shares[i]) for i in range(6)])
    assert ei.value.status == E.ERR_NOT_ENOUGH_SHARES
    assert engine.secret_reconstruct(sch, 0, [(0, [])]).tolist() == []     # no batch => no check
    with pytest.raises(SdaError) as ei:
        engine.share_generate(S.PackedShamir(3, 8, 5, 433, 354, 150), [1, 2, 3], [0] * 5)
    assert ei.value.status == E.ERR_UNSUPPORTED                             # L = 9 not a power of 2


# ------------------------------------------------------------------ masking (north-star kernel 3)
# (1 << 62) + 1: ~25 % of draws rejected; 0x5555555555555556: ~33 % rejected and, above 2^62, the
# reference's `result[i] += m` wraps i64 (chacha.rs:70), so the combine is signed and order
# dependent; I64_MAX: wrapping with almost no rejections
@pytest.mark.parametrize("m", [433, 2147482801, (1 << 40) + 7, (1 << 62) + 1, 0x5555555555555556, I64_MAX])
@pytest.mark.parametrize("words", [0, 1, 4, 8, 10])
def test_chacha_mask_and_combine(engine, oracle, m, words):
    rng = np.random.default_rng(m % 991 + words)
    D = 1000 if m > (1 << 61) else 3001
    sch = S.ChaChaMasking(m, D, 32 * words)
    secrets = rng.integers(0, m, size=D, dtype=np.int64)
    seeds = [rng.integers(0, 2**32, size=words, dtype=np.uint64).astype(np.uint32) for _ in range(5)]
    for sd in seeds[:2]:
        mask, masked = engine.secret_mask(sch, secrets, seed=sd)
        assert_same(mask, sd.astype(np.int64))
        assert_same(masked, oracle.chacha_mask(m, sd, secrets))
    rows = [sd.astype(np.int64) for sd in seeds]
    got = engine.mask_combine(sch, rows)
    exp = oracle.chacha_mask_combine(m, D, np.stack(rows) if words else np.zeros((5, 0), np.int64))
    assert_same(got, exp)


def test_chacha_wrapping_moduli_many_seeds(engine, oracle):
    """m > 2^62: 40 seeds, so the running i64 sum wraps often; bit-exact with the reference's
    sequential recurrence (the engine walks the seeds in order on its exact stream path)."""
    rng = np.random.default_rng(62)
    for m in (0x5555555555555556, I64_MAX - 24):
        rows = [rng.integers(0, 2**32, size=4, dtype=np.uint64).astype(np.int64) for _ in range(40)]
        got = engine.mask_combine(S.ChaChaMasking(m, 513, 128), rows)
        exp = oracle.chacha_mask_combine(m, 513, np.stack(rows))
        assert_same(got, exp)
        assert (exp < 0).any()            # the wrap did happen


def test_chacha_many_seeds(engine, oracle):
    m, D, N = 2147482801, 777, 300
    rng = np.random.default_rng(5)
    rows = [rng.integers(0, 2**32, size=4, dtype=np.uint64).astype(np.int64) for _ in range(N)]
    got = engine.mask_combine(S.ChaChaMasking(m, D, 128), rows)
    assert_same(got, oracle.chacha_mask_combine(m, D, np.stack(rows)))


def test_chacha_ragged_seed_lengths(engine, oracle):
    m, D = 433, 100
    rows = [np.array([1, 2, 3, 4]), np.array([5]), np.array([], np.int64), np.array([7, 8])]
    got = engine.mask_combine(S.ChaChaMasking(m, D, 128), rows)
    padded = np.zeros((4, 4), np.int64)
    for i, r in enumerate(rows):
        padded[i, : len(r)] = r
    assert_same(got, oracle.chacha_mask_combine(m, D, padded))


def test_chacha_dimension_assert(engine):
    with pytest.raises(SdaError) as ei:
        engine.secret_mask(S.ChaChaMasking(433, 5, 128), [1, 2, 3], seed=[1, 2, 3, 4])
    assert ei.value.status == E.ERR_PRECONDITION


@pytest.mark.parametrize("m", [433, 2147482801, (1 << 62) + 3])
def test_full_mask_unmask_positive(engine, oracle, m):
    rng = np.random.default_rng(m % 313)
    D = 4097
    secrets = rng.integers(I64_MIN // 2, I64_MAX // 2, size=D, dtype=np.int64)
    masks = rng.integers(0, m, size=D, dtype=np.int64)
    mk, masked = engine.secret_mask(S.FullMasking(m), secrets, full_masks=masks)
    assert_same(mk, masks)
    assert_same(masked, oracle.full_mask(m, masks, secrets))
    rows = [rng.integers(0, m, size=D, dtype=np.int64) for _ in range(7)]
    assert_same(engine.mask_combine(S.FullMasking(m), rows), oracle.combine(m, np.stack(rows)))
    un = engine.secret_unmask(S.FullMasking(m), (masks, masked))
    assert_same(un, oracle.unmask(m, masks, masked))
    assert_same(engine.positive(m, un), oracle.positive(m, un))
    assert_same(engine.secret_unmask(S.NoMasking(), ([], secrets)), secrets)
    with pytest.raises(SdaError):
        engine.secret_unmask(S.FullMasking(m), (masks[:-1], masked))


@pytest.mark.parametrize("sch", packed_schemes(), ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_generate_canonical_mode(engine, oracle, sch):
    """SDA_REVEAL_CANONICAL share-gen == the oracle's tss shares mod p (incl. raw i64 secrets)."""
    import torch
    p = sch.prime_modulus
    rng = np.random.default_rng(p % 991 + sch.share_count)
    D = 41 * sch.secret_count + 3
    B = (D + sch.secret_count - 1) // sch.secret_count
    secrets = rng.integers(-(p - 1), p, size=D, dtype=np.int64)
    secrets[::7] = rng.integers(-(2**40), 2**40, size=secrets[::7].size, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    exp = np.mod(oracle.packed_generate(_pp(oracle, sch), secrets, draws), p)
    for extra in (0, 1):                          # odd and even B (narrow and paired-wide stores)
        s_ = np.concatenate([secrets, np.zeros(extra * sch.secret_count, np.int64)])
        d_ = np.concatenate([draws, np.zeros(extra * sch.privacy_threshold(), np.int64)])
        Bx = B + extra
        ds, dd = torch.as_tensor(s_).cuda(), torch.as_tensor(d_).cuda()
        out = torch.empty((sch.share_count, Bx), dtype=torch.int64, device="cuda")
        engine.packed_generate_mode_dev(sch, ds.data_ptr(), s_.size, 1, dd.data_ptr(), out.data_ptr(),
                                        E.REVEAL_CANONICAL)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert_same(got[:, :B], exp)
        assert got.min() >= 0


def _bitrev(i, bits):
    return int(format(i, f"0{bits}b")[::-1], 2) if bits else 0


@pytest.mark.parametrize("sch", [s for s in packed_schemes() if s.prime_modulus >= 2**24 and
                                 s.secret_count + s.privacy_threshold() + 1 >= 4],
                         ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_generate_negative_multiple_of_p(engine, oracle, sch):
    """Exact share-gen where a first-stage dividend is exactly -p (tss: `-p % p == 0`).

    The exact kernel for p >= 2^24 truncates lazily (packed_gen.hip: Trunc<true>) and must send
    such batches to the generic fix-up; every other batch stays on the fast path.  The traps sit
    in the radix-2 stage-1 butterflies (x[2m] +- x[2m+1] over bit-reversed inputs).
    """
    p, k, t = sch.prime_modulus, sch.secret_count, sch.privacy_threshold()
    L = k + t + 1
    lb = L.bit_length() - 1
    rng = np.random.default_rng(p % 4099 + L)
    B = 96
    D = B * k
    secrets = rng.integers(-(p - 1), p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * t, dtype=np.int64)

    def put(b, r, v):          # raw index r of batch b: [0, secrets(k), randomness(t)]
        if r <= k:
            secrets[b * k + r - 1] = v
        else:
            draws[b * t + r - 1 - k] = v

    for b in range(0, B, 3):   # two of three batches trapped, the rest stay random
        if b + 1 < B:
            b_list = (b, b + 1)
        else:
            b_list = (b,)
        for bb in b_list:
            m = int(rng.integers(1, L // 2))
            u, c = _bitrev(2 * m, lb), _bitrev(2 * m + 1, lb)
            a = int(rng.integers(1, p))
            put(bb, u, -a)
            put(bb, c, (p - a) if bb % 2 else -(p - a))     # u - c == -p   /   u + c == -p
    got = engine.share_generate(sch, secrets, draws)
    assert_same(got, oracle.packed_generate(_pp(oracle, sch), secrets, draws))


@pytest.mark.parametrize("sch", [s for s in packed_schemes() if s.prime_modulus >= 2**24],
                         ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_generate_structured_values(engine, oracle, sch):
    """Exact share-gen on structured batches that stress the sign-bit radix-2 half (packed_gen.hip,
    SIGNBIT) and its traps: sparse vectors (zero secrets; all-zero batches), tiny values (+-1, +-2, where
    the twiddle products no longer dominate), values a and p - a of either sign (butterfly sums that are
    exact multiples of p, where tss truncates to 0), and p - 1 -- mixed with random batches.  Every batch
    must equal the oracle (tss' operation order) whatever path -- fast or fix-up -- it took."""
    p, k, t = sch.prime_modulus, sch.secret_count, sch.privacy_threshold()
    L = k + t + 1
    rng = np.random.default_rng(p % 7919 + 3 * L)
    B = 4096
    raw = rng.integers(-(p - 1), p, size=(B, L), dtype=np.int64)
    a = int(rng.integers(3, p - 3))
    pool = np.array([0, 1, -1, 2, -2, a, -a, p - a, -(p - a), p - 1, -(p - 1)], dtype=np.int64)
    for b in range(B):
        kind = b % 4
        if kind == 0:                        # sparse: a few pool values, the rest zero
            raw[b] = 0
            pos = rng.choice(np.arange(1, L), size=int(rng.integers(1, min(4, L - 1) + 1)), replace=False)
            raw[b, pos] = rng.choice(pool, size=pos.size)
        elif kind == 1:                      # every value from the pool
            raw[b] = rng.choice(pool, size=L)
        elif kind == 2:                      # zero secrets, random draws
            raw[b, 1:k + 1] = 0
        raw[b, 0] = 0                        # values[0] = 0 (the inserted point)
    raw[-1] = 0                              # an all-zero batch
    secrets = raw[:, 1:k + 1].reshape(-1).copy()
    draws = raw[:, k + 1:].reshape(-1).copy()
    got = engine.share_generate(sch, secrets, draws)
    assert_same(got, oracle.packed_generate(_pp(oracle, sch), secrets, draws))


@pytest.mark.parametrize("sch", [s for s in packed_schemes() if s.prime_modulus >= 2**24 and
                                 s.secret_count <= 8 and s.reconstruction_threshold() <= 15],
                         ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_reconstruct_traps(engine, oracle, sch):
    """Exact reveal where a Newton difference is exactly -p, or a coefficient is 0 (all-zero
    shares): the lazily truncating kernel (p >= 2^24, k <= 8, <= 16 points) must fall back to the
    generic exact path for those batches only."""
    p, n = sch.prime_modulus, sch.share_count
    rng = np.random.default_rng(p % 3001 + n)
    k = sch.secret_count
    B = 150
    D = B * k - (1 if k > 1 else 0)               # ragged tail batch where k allows it
    need = sch.reconstruction_threshold()
    for size in sorted({need, min(n, 15)}):
        idx = rng.permutation(n)[:size].tolist()
        sh = rng.integers(-(p - 1), p, size=(size, B), dtype=np.int64)
        for b in range(0, B, 2):                  # share[r] - share[r-1] == -p (first Newton level)
            if size >= 2:
                r = int(rng.integers(1, size))
                a = int(rng.integers(1, p))
                sh[r, b], sh[r - 1, b] = -a, p - a
        sh[:, 3] = 0                              # zero Newton coefficients
        sh[:, 7] = 0
        got = engine.secret_reconstruct(sch, D, [(i, sh[j]) for j, i in enumerate(idx)])
        rc, exp = oracle.packed_reconstruct(_pp(oracle, sch), D, idx, sh)
        assert rc == 0
        assert_same(got, exp)


def _reveal_points(sch, idx):
    p, wn = sch.prime_modulus, sch.omega_shares
    return [1] + [pow(wn, i + 1, p) for i in idx]         # packed::reconstruct inserts (1, 0) first


def _newton_values(C, xs, p):
    """Values at xs[1:] of the Newton-form polynomial with coefficients C over the nodes xs."""
    out = []
    for xj in xs[1:]:
        acc, basis = 0, 1
        for l, c in enumerate(C):
            acc = (acc + c * basis) % p
            basis = basis * (xj - xs[l]) % p
        out.append(acc)
    return out


@pytest.mark.parametrize("sch", [s for s in packed_schemes() if s.prime_modulus >= 2**24 and
                                 s.secret_count <= 8 and s.reconstruction_threshold() <= 15],
                         ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_reconstruct_zero_residues(engine, oracle, sch):
    """The sign-bit reveal path is exact unless a residue on the way is 0 mod p; those batches must be
    caught and recomputed.  Planted per batch, with random signs on the shares:
      (a) a newton_evaluate partial sum = 0 mod p (the fold's exact value then is 0 or +-p), at a
          random secret e and step i (i = last: the secret itself is 0 mod p);
      (b) a divided difference over a random window = 0 mod p (its Newton step's exact difference
          is 0 or +-p)."""
    p, n, k = sch.prime_modulus, sch.share_count, sch.secret_count
    ws = sch.omega_secrets
    rng = np.random.default_rng(p % 7919 + n)
    size = min(n, 15)
    idx = rng.permutation(n)[:size].tolist()
    xs = _reveal_points(sch, idx)
    m = size + 1
    B = 240
    sh = np.zeros((size, B), np.int64)
    for b in range(B):
        if b % 2 == 0:                                   # (a) zero partial sum of the fold
            e = int(rng.integers(0, k))
            i = int(rng.integers(2, m)) if b % 6 else m - 1
            X = pow(ws, e + 1, p)
            npb = [1]
            for l in range(m - 1):
                npb.append(npb[-1] * (X - xs[l]) % p)
            C = [0] + [int(v) for v in rng.integers(1, p, size=m - 1)]
            part = sum(C[l] * npb[l] for l in range(1, i)) % p
            C[i] = (-part) * pow(npb[i], -1, p) % p
            if C[i] == 0:
                C[i] = 1
            y = _newton_values(C, xs, p)
        else:                                            # (b) zero divided difference over a window
            L = int(rng.integers(2, m))                  # window of L + 1 nodes: a Newton level L step
            a = int(rng.integers(0, m - L))
            y = [int(v) for v in rng.integers(0, p, size=m - 1)]
            nodes = list(range(a, a + L + 1))
            w = []
            for q in nodes:
                d = 1
                for r in nodes:
                    if r != q:
                        d = d * (xs[q] - xs[r]) % p
                w.append(pow(d, -1, p))
            vals = [0] + y                                # node 0 carries value 0
            s = sum(w[j] * vals[q] for j, q in enumerate(nodes[:-1])) % p
            last = nodes[-1]
            vals[last] = (-s) * pow(w[-1], -1, p) % p
            y = vals[1:]
        neg = rng.random(size) < 0.5
        sh[:, b] = [(v - p) if (ng and v) else v for v, ng in zip(y, neg)]
    D = B * k
    got = engine.secret_reconstruct(sch, D, [(i, sh[j]) for j, i in enumerate(idx)])
    rc, exp = oracle.packed_reconstruct(_pp(oracle, sch), D, idx, sh)
    assert rc == 0
    assert_same(got, exp)


# ------------------------------------------------------------------ packed Shamir past the register kernels
# tss takes any power-of-2 k + t + 1 and power-of-3 n + 1; past 64 / 81 (and past 95 shares per reveal)
# the engine runs packed_wide.hip's workspace kernels.  (k, t, n): L = 128 / 256 over 243 / 729 points,
# and a small L over 243 points (reveals from up to 242 shares through the wide Newton path).
def wide_schemes():
    out = []
    for k, t, n in [(100, 27, 242), (64, 63, 242), (5, 2, 242), (200, 55, 728), (1, 0, 242)]:
        L, N3 = k + t + 1, n + 1
        p = _prime_for(L, N3)
        ws, wn = _roots(p, L, N3)
        out.append(S.PackedShamir(k, n, t, p, ws, wn))
    return out


@pytest.mark.parametrize("sch", wide_schemes(), ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_wide_generate(engine, oracle, sch):
    """Share-gen at k + t + 1 > 64 or n + 1 > 81 == tss (oracle), signed and canonical, raw i64 secrets too."""
    import torch
    p, k = sch.prime_modulus, sch.secret_count
    rng = np.random.default_rng(p % 1009 + sch.share_count)
    D = 9 * k + 1
    B = (D + k - 1) // k
    secrets = rng.integers(-(p - 1), p, size=D, dtype=np.int64)
    secrets[::5] = rng.integers(-(2**40), 2**40, size=secrets[::5].size, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    exp = oracle.packed_generate(_pp(oracle, sch), secrets, draws)
    assert_same(engine.share_generate(sch, secrets, draws), exp)
    ds, dd = torch.as_tensor(secrets).cuda(), torch.as_tensor(draws).cuda()
    out = torch.empty((2, sch.share_count, B), dtype=torch.int64, device="cuda")
    dd2 = torch.cat([dd, dd])
    ds2 = torch.cat([ds, ds])                   # two vectors per launch
    engine.packed_generate_mode_dev(sch, ds2.data_ptr(), D, 2, dd2.data_ptr(), out.data_ptr(), E.REVEAL_CANONICAL)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert_same(got[0], np.mod(exp, p))
    assert_same(got[1], np.mod(exp, p))


@pytest.mark.parametrize("sch", wide_schemes(), ids=lambda s: f"k{s.secret_count}t{s.privacy_threshold()}n{s.share_count}")
def test_packed_wide_reconstruct(engine, oracle, sch):
    """Reveal from every share (batched.rs:75) and from random subsets, through the register kernels
    (<= 95 shares) and the wide Newton path (more), both modes, == tss (oracle)."""
    import torch
    p, n, k = sch.prime_modulus, sch.share_count, sch.secret_count
    rng = np.random.default_rng(p % 331 + n)
    D = 5 * k + 1
    B = (D + k - 1) // k
    secrets = rng.integers(0, p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    shares = oracle.packed_generate(_pp(oracle, sch), secrets, draws)
    need = sch.reconstruction_threshold()
    sizes = [n, max(need, 96), max(need, 95), need] + [int(rng.integers(need, n + 1)) for _ in range(2)]
    for size in sizes:
        idx = rng.permutation(n)[:size].tolist()
        got = engine.secret_reconstruct(sch, D, [(i, shares[i]) for i in idx])
        rc, exp = oracle.packed_reconstruct(_pp(oracle, sch), D, idx, shares[idx])
        assert rc == 0
        assert_same(got, exp)
        assert (got % p == secrets % p).all()
        dsh = torch.as_tensor(np.ascontiguousarray(shares[idx])).cuda()
        out = torch.empty(D, dtype=torch.int64, device="cuda")
        engine.packed_reconstruct_dev(sch, D, idx, 1, dsh.data_ptr(), out.data_ptr(), mode=E.REVEAL_CANONICAL)
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy(), np.mod(exp, p))
    # shares outside (-p, p): tss' wrapping arithmetic on the wide path as well
    idx = list(range(max(need, min(n, 120))))
    raw = shares[idx].copy()
    raw[0, ::3] += 5 * p
    got = engine.secret_reconstruct(sch, D, [(i, raw[j]) for j, i in enumerate(idx)])
    rc, exp = oracle.packed_reconstruct(_pp(oracle, sch), D, idx, raw)
    assert_same(got, exp)


def test_packed_wide_domain_limits(engine):
    """Past the engine's domain (k + t + 1 > 1024, n + 1 > 729) the call is refused, not approximated."""
    with pytest.raises(SdaError) as ei:
        engine.share_generate(S.PackedShamir(1000, 2186, 1047, 2147483647 - 12, 3, 5), [1], [0] * 1047)
    assert ei.value.status == E.ERR_UNSUPPORTED


def _random_packed_scheme(rng):
    """A random tss-valid scheme: k + t + 1 = L (power of 2), n + 1 = N3 (power of 3) with k + t <= n, a
    random prime p = 1 mod lcm(L, N3) below 2^31 from one of three magnitude bands (so both the lazy and
    the verbatim truncation paths run), and roots of unity from a random generator."""
    L = int(rng.choice([2, 4, 8, 16, 32, 64]))
    N3 = int(rng.choice([n3 for n3 in (3, 9, 27, 81) if n3 > L]))
    k = int(rng.integers(1, L))
    t = L - 1 - k
    step = L * N3 // math.gcd(L, N3)
    lo, hi = [(N3 + 2, 1 << 16), (1 << 16, 1 << 24), (1 << 24, 1 << 31)][int(rng.integers(0, 3))]
    while True:
        c = int(rng.integers(max(1, lo // step), (hi - 1) // step))
        p = c * step + 1
        if lo <= p < hi and all(p % q for q in range(2, int(p**0.5) + 1)):
            break
    ws, wn = _roots(p, L, N3)
    e = int(rng.integers(1, p - 1))
    while math.gcd(e, p - 1) != 1:
        e += 1
    return S.PackedShamir(k, N3 - 1, t, p, pow(ws, e, p), pow(wn, e, p))


@pytest.mark.parametrize("seed", range(16))
def test_packed_random_schemes(engine, oracle, seed):
    """Random schemes (sizes, primes from 2^9 to 2^31, any primitive roots of the right orders):
    share-gen with signed secrets in (-p, p) and reconstruct from random subsets of at least t + k
    shares, against the oracle's tss restatement (bit-exact signed representatives)."""
    rng = np.random.default_rng(0xC0FFEE + seed)
    sch = _random_packed_scheme(rng)
    p, n, k = sch.prime_modulus, sch.share_count, sch.secret_count
    D = int(rng.integers(1, 300)) * k + int(rng.integers(0, k))
    D = max(D, 1)
    B = (D + k - 1) // k
    secrets = rng.integers(-(p - 1), p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    pp = _pp(oracle, sch)
    shares = engine.share_generate(sch, secrets, draws)
    assert_same(shares, oracle.packed_generate(pp, secrets, draws), f"gen {sch}")
    need = sch.reconstruction_threshold()
    for _ in range(3):
        idx = rng.permutation(n)[:int(rng.integers(need, n + 1))].tolist()
        got = engine.secret_reconstruct(sch, D, [(i, shares[i]) for i in idx])
        rc, exp = oracle.packed_reconstruct(pp, D, idx, shares[idx])
        assert rc == 0
        assert_same(got, exp, f"reveal {sch} from {len(idx)}")
        assert (got % p == secrets % p).all()


@pytest.mark.parametrize("seed", range(8))
def test_packed_wide_random_schemes(engine, oracle, seed):
    """Random schemes past the register kernels (L up to 1024 over 243 or 729 points, primes from the
    smallest valid one up to 2^31, random primitive roots): gen and reveal from random subsets (register
    and workspace reveal paths) bit-exact vs the oracle."""
    rng = np.random.default_rng(0xBEEF + seed)
    N3 = int(rng.choice([243, 729]))
    L = int(rng.choice([l for l in (2, 8, 64, 128, 256, 512, 1024) if l < N3]))
    k = int(rng.integers(1, L))
    t = L - 1 - k
    step = L * N3
    small = bool(rng.integers(0, 2))
    lo, hi = (step + 1, 1 << 24) if small and step < (1 << 23) else (1 << 24, 1 << 31)
    while True:
        c = int(rng.integers(max(1, lo // step), (hi - 1) // step))
        p = c * step + 1
        if lo <= p < hi and all(p % q for q in range(2, int(p**0.5) + 1)):
            break
    ws, wn = _roots(p, L, N3)
    e = int(rng.integers(1, p - 1))
    while math.gcd(e, p - 1) != 1:
        e += 1
    sch = S.PackedShamir(k, N3 - 1, t, p, pow(ws, e, p), pow(wn, e, p))
    n = sch.share_count
    D = int(rng.integers(1, 4)) * k + int(rng.integers(0, k))
    D = max(D, 1)
    B = (D + k - 1) // k
    secrets = rng.integers(-(p - 1), p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * sch.privacy_threshold(), dtype=np.int64)
    pp = _pp(oracle, sch)
    shares = engine.share_generate(sch, secrets, draws)
    assert_same(shares, oracle.packed_generate(pp, secrets, draws), f"gen {sch}")
    need = sch.reconstruction_threshold()
    for size in (need, int(rng.integers(need, n + 1))):
        idx = rng.permutation(n)[:size].tolist()
        got = engine.secret_reconstruct(sch, D, [(i, shares[i]) for i in idx])
        rc, exp = oracle.packed_reconstruct(pp, D, idx, shares[idx])
        assert rc == 0
        assert_same(got, exp, f"reveal {sch} from {size}")
