"""GPU parity of the fused role pipelines against the oracle.

  recipient   receive.rs:80-157 + :14-20   mask combine -> reconstruct -> unmask -> positive
  participant participate.rs:53-76         mask -> share-generate -> per-clerk payload encoding
and the whole aggregation on device: participants -> clerk decode+combine -> recipient reveal.
Expected values come from the step-by-step oracle flow (tests/pipeline.py over OracleBackend),
which the full_loop / README KATs pin.  Bit-exact.
"""
import numpy as np
import pytest

from sda_amd import SdaError, schemes as S
from sda_amd import engine as E
from tests.oracle_backend import OracleBackend
from tests.pipeline import (FULL_LOOP_EXPECTED, FULL_LOOP_INPUTS, README_EXPECTED, README_INPUTS, Draws,
                            full_loop_variants, run_aggregation, sharing_draws)
from tests.util import assert_same

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

P = S.CONFIG_PACKED.prime_modulus


def _cases():
    out = [(name, ms, ss, 433, 4, FULL_LOOP_INPUTS, FULL_LOOP_EXPECTED) for name, (ms, ss) in full_loop_variants().items()]
    out.append(("readme", S.NoMasking(), S.Additive(3, 433), 433, 10, README_INPUTS, README_EXPECTED))
    rng = np.random.default_rng(11)
    D = 8 * 97 + 3
    inputs = [rng.integers(0, 1000, size=D) for _ in range(5)]
    exp = list(np.sum(inputs, axis=0) % P)
    out.append(("packed_chacha", S.ChaChaMasking(P, D, 128), S.CONFIG_PACKED, P, D, inputs, exp))
    out.append(("packed_full", S.FullMasking(P), S.CONFIG_PACKED, P, D, inputs, exp))
    out.append(("additive_chacha", S.ChaChaMasking(P, D, 96), S.Additive(5, P), P, D, inputs, exp))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_recipient_reveal_matches_stepwise(engine, case):
    name, ms, ss, m, D, inputs, expected = case
    tr = run_aggregation(OracleBackend(), ms, ss, m, D, inputs, Draws(0x5DA))
    assert tr.positive.tolist() == list(expected)
    n = ss.output_size()
    for order in (list(range(n)), list(reversed(range(n)))):
        if isinstance(ss, S.PackedShamir):
            order = order[: ss.reconstruction_threshold() + 1]
        indexed = [(c, tr.clerk_results[c]) for c in order]
        got = engine.recipient_reveal(ms, tr.masks, ss, D, indexed, m)
        # the stepwise oracle flow with the same clerk order
        be = OracleBackend()
        mo = be.secret_reconstruct(ss, D, indexed)
        mask = be.mask_combine(ms, tr.masks) if ms.has_mask() else np.zeros(0, np.int64)
        exp = be.positive(m, be.secret_unmask(ms, (mask, mo)))
        assert_same(got, exp, name)
        assert (np.mod(got, m) == np.mod(expected, m)).all()


def test_recipient_reveal_errors(engine):
    tr = run_aggregation(OracleBackend(), S.NoMasking(), S.FULL_LOOP_PACKED, 433, 4, FULL_LOOP_INPUTS, Draws(1))
    few = [(c, tr.clerk_results[c]) for c in range(S.FULL_LOOP_PACKED.reconstruction_threshold() - 1)]
    with pytest.raises(SdaError) as ei:
        engine.recipient_reveal(S.NoMasking(), [], S.FULL_LOOP_PACKED, 4, few, 433)
    assert ei.value.status == E.ERR_NOT_ENOUGH_SHARES
    add = S.Additive(3, 433)
    with pytest.raises(SdaError) as ei:
        engine.recipient_reveal(S.NoMasking(), [], add, 4, [(0, [1, 2, 3]), (1, [1, 2])], 433)
    assert ei.value.status == E.ERR_MISMATCHING_DIMENSION
    with pytest.raises(SdaError) as ei:                      # full.rs:58 assert_eq! (mask length 3 vs 2)
        engine.recipient_reveal(S.FullMasking(433), [[1, 2, 3]], add, 2, [(0, [1, 2]), (1, [3, 4])], 433)
    assert ei.value.status == E.ERR_PRECONDITION


def _device(a, dtype=torch.int64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


@pytest.mark.parametrize("ms", [S.NoMasking(), S.FullMasking(P), S.ChaChaMasking(P, 4099, 128)],
                         ids=["none", "full", "chacha"])
@pytest.mark.parametrize("ss", [S.Additive(4, P), S.CONFIG_PACKED], ids=["additive", "packed"])
def test_participant_share_dev(engine, oracle, ms, ss):
    D = 4099
    rng = Draws(0xABC)
    secrets = np.random.default_rng(5).integers(-(P - 1), P, size=D, dtype=np.int64)
    be = OracleBackend()
    full = seed = None
    if isinstance(ms, S.FullMasking):
        full = rng.below(P, D)
        mask, masked = be.secret_mask(ms, secrets, full_masks=full)
    elif isinstance(ms, S.ChaChaMasking):
        seed = rng.u32(ms.seed_words())
        mask, masked = be.secret_mask(ms, secrets, seed=seed)
    else:
        masked = secrets
    draws = sharing_draws(ss, D, rng)
    exp = be.share_generate(ss, masked, draws)
    n, B = exp.shape
    d_sec, d_dr = _device(secrets), _device(draws)
    d_full = _device(full) if full is not None else None
    out = torch.empty((n, B), dtype=torch.int64, device="cuda")
    cap = n * B * 10 + 32
    pay = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    rb = engine.participant_share_dev(ms, ss, d_sec.data_ptr(), D, d_dr.data_ptr(), out.data_ptr(), seed=seed,
                                      full_masks_ptr=d_full.data_ptr() if d_full is not None else None,
                                      payload_ptr=pay.data_ptr(), payload_cap=cap)
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), exp)
    host = pay.cpu().numpy().tobytes()
    off = np.concatenate([[0], np.cumsum(rb)]).astype(np.int64)
    for c in range(n):
        assert host[off[c]:off[c + 1]] == oracle.varint_encode(exp[c])


@pytest.mark.parametrize("gen_mode", [E.REVEAL_EXACT, E.REVEAL_CANONICAL], ids=["gen_exact", "gen_canon"])
@pytest.mark.parametrize("mode", [E.REVEAL_EXACT, E.REVEAL_CANONICAL], ids=["rev_exact", "rev_canon"])
def test_aggregation_end_to_end_on_device(engine, mode, gen_mode):
    """participants (device) -> clerks: decode + combine their payloads (device) -> recipient reveal
    (device) == sum of the inputs mod p (integration-tests/tests/full_loop.rs's property at scale)."""
    ms, ss = S.ChaChaMasking(P, 80_000, 128), S.CONFIG_PACKED
    D, N = 80_000, 6
    n, B = ss.share_count, (D + ss.secret_count - 1) // ss.secret_count
    rng = Draws(0x5DA + 4)
    inputs = np.random.default_rng(6).integers(0, 1 << 20, size=(N, D), dtype=np.int64)
    cap = n * B * 10 + 32
    payloads, seeds = [], []
    for i in range(N):
        seed = rng.u32(ms.seed_words())
        seeds.append(seed)
        sec, dr = _device(inputs[i]), _device(sharing_draws(ss, D, rng))
        sh = torch.empty((n, B), dtype=torch.int64, device="cuda")
        pay = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        rb = engine.participant_share_dev(ms, ss, sec.data_ptr(), D, dr.data_ptr(), sh.data_ptr(), seed=seed,
                                          payload_ptr=pay.data_ptr(), payload_cap=cap, mode=gen_mode)
        off = np.concatenate([[0], np.cumsum(rb)]).astype(np.int64)
        h = pay.cpu().numpy().tobytes()
        payloads.append([h[off[c]:off[c + 1]] for c in range(n)])
    # clerk c: the N participations' payloads for c, back to back (snapshot order), decode + combine
    results = torch.empty((n, B), dtype=torch.int64, device="cuda")
    for c in range(n):
        blobs = [payloads[i][c] for i in range(N)]
        off = np.concatenate([[0], np.cumsum([len(b) for b in blobs])]).astype(np.uint64)
        buf = torch.frombuffer(bytearray(b"".join(blobs) + bytes(32)), dtype=torch.uint8).cuda()
        got = engine.clerk_decode_combine_dev(P, buf.data_ptr(), off, results[c].data_ptr(), B)
        assert got == B
    seeds_d = _device(np.stack(seeds).view(np.int32), torch.int32)
    idx = list(range(n - 1, n - 1 - ss.reconstruction_threshold(), -1))
    sub = results[idx].contiguous()
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    L = engine.recipient_reveal_dev(ms, seeds_d.data_ptr(), N, ms.seed_words(), ss, D, idx, sub.data_ptr(), B, P,
                                    out.data_ptr(), D, mode=mode)
    torch.cuda.synchronize()
    assert L == D
    assert_same(out.cpu().numpy(), inputs.sum(axis=0) % P)


def test_recipient_reveal_wide_scheme(engine):
    """The recipient pipeline over a scheme past the register kernels (n + 1 = 243, all 242 clerk
    results: the workspace reveal of packed_wide.hip) == the step-wise oracle flow."""
    from tests.test_gpu_parity import wide_schemes
    ss = next(s for s in wide_schemes() if s.secret_count == 5)
    m = ss.prime_modulus
    rng = np.random.default_rng(12)
    D = 5 * 41 + 2
    inputs = [rng.integers(0, 1000, size=D) for _ in range(3)]
    ms = S.ChaChaMasking(m, D, 128)
    tr = run_aggregation(OracleBackend(), ms, ss, m, D, inputs, Draws(0x5DB))
    assert tr.positive.tolist() == list(np.sum(inputs, axis=0) % m)
    for order in (list(range(ss.share_count)), list(range(ss.share_count))[::-2]):
        indexed = [(c, tr.clerk_results[c]) for c in order]
        got = engine.recipient_reveal(ms, tr.masks, ss, D, indexed, m)
        be = OracleBackend()
        mo = be.secret_reconstruct(ss, D, indexed)
        exp = be.positive(m, be.secret_unmask(ms, (be.mask_combine(ms, tr.masks), mo)))
        assert_same(got, exp, "wide")


def _signed_clerk_results(ss, D, seed):
    """Arbitrary signed clerk results in (-p, p) for every clerk: the reveal interpolates whatever it gets."""
    p, n = ss.prime_modulus, ss.share_count
    B = (D + ss.secret_count - 1) // ss.secret_count
    rng = np.random.default_rng(seed)
    return [rng.integers(-(p - 1), p, size=B, dtype=np.int64) for _ in range(n)]


def _stepwise(ms, masks, ss, D, indexed, m):
    be = OracleBackend()
    mo = be.secret_reconstruct(ss, D, indexed)                # tss' exact signed representatives
    mask = be.mask_combine(ms, masks) if ms.has_mask() else np.zeros(0, np.int64)
    return be.positive(m, be.secret_unmask(ms, (mask, mo))), mo, mask


@pytest.mark.parametrize("ms_kind", ["none", "full", "chacha"])
def test_recipient_residue_only_runs_canonical_identically(engine, monkeypatch, ms_kind):
    """Masking modulus (or no mask) == output modulus == p: the pipeline runs the canonical reveal for an EXACT
    request.  On signed clerk results its output equals the step-wise oracle flow over tss'
    exact reveal, and the forced-EXACT pipeline (SDA_RECIPIENT_EXACT=1), byte for byte."""
    ss = S.CONFIG_PACKED
    D = 8 * 523 + 5
    ms = {"none": S.NoMasking(), "full": S.FullMasking(P), "chacha": S.ChaChaMasking(P, D, 128)}[ms_kind]
    rng = Draws(0x77)
    masks = [] if ms_kind == "none" else ([rng.below(P, D) for _ in range(3)] if ms_kind == "full"
                                          else [rng.u32(4) for _ in range(3)])
    res = _signed_clerk_results(ss, D, 3)
    indexed = [(c, res[c]) for c in (25, 3, 17, 8, 0, 11, 20, 6, 14, 1, 22, 9, 5, 19, 12, 24)]
    exp, _, _ = _stepwise(ms, masks, ss, D, indexed, P)
    got = engine.recipient_reveal(ms, masks, ss, D, indexed, P)
    monkeypatch.setenv("SDA_RECIPIENT_EXACT", "1")
    forced = engine.recipient_reveal(ms, masks, ss, D, indexed, P)
    assert_same(got, exp, ms_kind)
    assert_same(forced, exp, ms_kind + " forced exact")


@pytest.mark.parametrize("which", ["mask_modulus", "output_modulus"])
def test_recipient_keeps_exact_when_moduli_differ(engine, which):
    """A masking modulus or output modulus other than p makes the output depend on the reveal's signed
    representative, so the pipeline keeps tss' exact reveal: the output equals the exact step-wise flow and
    differs from what a canonical reveal would give on some elements."""
    ss = S.CONFIG_PACKED
    D = 8 * 301 + 1
    q = P + 2 if which == "mask_modulus" else P
    m_out = P if which == "mask_modulus" else 1 << 40
    ms = S.FullMasking(q)
    rng = Draws(0x78)
    masks = [rng.below(q, D) for _ in range(2)]
    res = _signed_clerk_results(ss, D, 4)
    indexed = [(c, res[c]) for c in range(ss.reconstruction_threshold())]
    exp, mo, mask = _stepwise(ms, masks, ss, D, indexed, m_out)
    be = OracleBackend()
    canon = be.positive(m_out, be.secret_unmask(ms, (mask, np.mod(mo, P))))
    assert (np.asarray(canon) != np.asarray(exp)).any()      # the representative matters here
    got = engine.recipient_reveal(ms, masks, ss, D, indexed, m_out)
    assert_same(got, exp, which)


def test_recipient_duplicate_points_fall_back_to_exact(engine):
    """Equal moduli but a repeated clerk index (no Lagrange form): the pipeline falls back to the exact reveal
    and matches the step-wise flow (tss' Newton over the repeated point)."""
    ss = S.FULL_LOOP_PACKED
    p = ss.prime_modulus
    D = 3 * 5
    res = _signed_clerk_results(ss, D, 5)
    indexed = [(c, res[c]) for c in (0, 1, 2, 3, 4, 5, 2)]
    exp, _, _ = _stepwise(S.NoMasking(), [], ss, D, indexed, p)
    got = engine.recipient_reveal(S.NoMasking(), [], ss, D, indexed, p)
    assert_same(got, exp, "duplicate points")
