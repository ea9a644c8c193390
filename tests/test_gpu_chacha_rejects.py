"""GPU: the ChaCha fast path's gen_range rejection fix-up (chacha.rs:37-39, 68-69: gen_range(0, m)
rejects a draw v >= u64::MAX - u64::MAX % m and takes the next pair), on seeds whose streams really
reject a draw.

Rejections are rare by construction (< 2^-28 per draw on the fast path; 2^-42.5 for the field prime),
so the seeds were searched for on the GPU with tools/chacha_reject_search.hip (scripts/
gpu_reject_search.sh) and each hit was confirmed with the oracle's rand-0.3 ChaChaRng
(tests/test_oracle_golden.py pins it).  Two moduli cover both fast-path kernels:
  4294901761 = 2^32 - 2^16 + 1   lazy accumulation (m <= 2^32), 2^-32 rejections per draw
  68719676673                     64-bit Barrett path (2^32 < m <= 2^62), 2^-28 per draw (the path's limit)
Checked against the oracle: the combine (counter mode + fix-up), a single stream (the participant's
mask), and the two device pipelines that now read the rejection count at the END of the call and
redo their dependent steps (recipient: unmask; participant: mask add, share-gen, payloads).
"""
import json
import os

import numpy as np
import pytest

from sda_amd import schemes as S
from tests.oracle_backend import OracleBackend
from tests.pipeline import Draws, sharing_draws
from tests.util import assert_same

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

# seed words (s, 0x5DA, 7, 11) -> the first rejected pair of that stream (tests/golden/chacha_rejects.json;
# tests/test_oracle_golden.py checks the hits against the oracle's stream)
_G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "chacha_rejects.json")))
REJECTS = {int(m): [tuple(h) for h in hits] for m, hits in _G["moduli"].items()}
MODULI = sorted(REJECTS)


def _seed(s):
    return np.array([s, 0x5DA, 7, 11], np.int64)


def _seeds(m, extra=3):
    rng = np.random.default_rng(m % 1009)
    rows = [_seed(s) for s, _ in REJECTS[m]]
    rows += [rng.integers(0, 2**32, size=4, dtype=np.uint64).astype(np.int64) for _ in range(extra)]
    return np.stack(rows)


@pytest.mark.parametrize("m", MODULI)
@pytest.mark.parametrize("D", [65536, 3391, 2687])
def test_combine_with_rejections(engine, oracle, m, D):
    """Combine over the found seeds (+3 random): D = 65536 holds every hit; 3391 / 2687 put one hit in
    the stream's last element, so the fix-up must extend that stream past D."""
    rows = _seeds(m)
    exp = oracle.chacha_mask_combine(m, D, rows)
    got = engine.mask_combine(S.ChaChaMasking(m, D, 128), list(rows))
    assert_same(got, exp)
    seeds = torch.as_tensor(rows.astype(np.uint32).view(np.int32)).cuda()
    out = torch.full((D,), 7, dtype=torch.int64, device="cuda")
    engine.chacha_mask_combine_dev(m, D, seeds.data_ptr(), 4, rows.shape[0], out.data_ptr())
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), exp)


@pytest.mark.parametrize("m", MODULI)
def test_single_stream_with_rejection(engine, oracle, m):
    """One rejecting stream (the participant's own mask): masked = (secret + draw) % m."""
    D = 65536
    rng = np.random.default_rng(3)
    secrets = rng.integers(-(m - 1), m, size=D, dtype=np.int64)
    for s, _ in REJECTS[m][:3]:
        mask, masked = engine.secret_mask(S.ChaChaMasking(m, D, 128), secrets, seed=_seed(s))
        assert_same(masked, oracle.chacha_mask(m, _seed(s).astype(np.uint32), secrets))


@pytest.mark.parametrize("m", MODULI)
def test_recipient_reveal_with_rejections(engine, m):
    """sda_recipient_reveal{,_dev}: the mask combine's rejections are resolved after the reconstruct and
    unmask were queued -- the result equals the oracle's step-wise flow."""
    D = 65536
    ms, ss = S.ChaChaMasking(m, D, 128), S.Additive(3, m)
    rng = np.random.default_rng(m % 97)
    clerks = [(c, rng.integers(-(m - 1), m, size=D, dtype=np.int64)) for c in range(3)]
    masks = list(_seeds(m))
    be = OracleBackend()
    exp = be.positive(m, be.secret_unmask(ms, (be.mask_combine(ms, masks), be.secret_reconstruct(ss, D, clerks))))
    assert_same(engine.recipient_reveal(ms, masks, ss, D, clerks, m), exp)
    seeds = torch.as_tensor(np.stack(masks).astype(np.uint32).view(np.int32)).cuda()
    sh = torch.as_tensor(np.stack([v for _, v in clerks])).cuda()
    out = torch.full((D,), 7, dtype=torch.int64, device="cuda")
    n = engine.recipient_reveal_dev(ms, seeds.data_ptr(), len(masks), 4, ss, D, [0, 1, 2], sh.data_ptr(), D, m,
                                    out.data_ptr(), D)
    torch.cuda.synchronize()
    assert n == D
    assert_same(out.cpu().numpy(), exp)


@pytest.mark.parametrize("m", MODULI)
def test_participant_share_with_rejection(engine, oracle, m):
    """sda_participant_share_dev with a rejecting mask stream: mask add, share-gen and payloads are
    redone after the fix-up -- shares and payload bytes equal the oracle's."""
    D = 65536
    ms, ss = S.ChaChaMasking(m, D, 128), S.Additive(4, m)
    secrets = np.random.default_rng(9).integers(-(m - 1), m, size=D, dtype=np.int64)
    be = OracleBackend()
    for s, _ in REJECTS[m][:2]:
        seed = _seed(s)
        _, masked = be.secret_mask(ms, secrets, seed=seed)
        draws = sharing_draws(ss, D, Draws(s))
        exp = be.share_generate(ss, masked, draws)
        n, B = exp.shape
        d_sec = torch.as_tensor(secrets).cuda()
        d_dr = torch.as_tensor(np.ascontiguousarray(draws)).cuda()
        out = torch.empty((n, B), dtype=torch.int64, device="cuda")
        cap = n * B * 10 + 32
        pay = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        rb = engine.participant_share_dev(ms, ss, d_sec.data_ptr(), D, d_dr.data_ptr(), out.data_ptr(), seed=seed,
                                          payload_ptr=pay.data_ptr(), payload_cap=cap)
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy(), exp)
        host = pay.cpu().numpy().tobytes()
        off = np.concatenate([[0], np.cumsum(rb)]).astype(np.int64)
        for c in range(n):
            assert host[off[c]:off[c + 1]] == oracle.varint_encode(exp[c])
