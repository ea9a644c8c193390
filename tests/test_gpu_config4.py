"""GPU: BASELINE.json configs[4] at its own size -- the full clerk path with ChaCha (LinearMaskingScheme
PRG) masking + packed Shamir (k = 8, n = 26, t = 7) at 10,000,000-dim -- through the C ABI.

  participant  participate.rs:53-76   mask (chacha.rs:25-53) -> share-generate -> per-clerk payloads
  recipient    receive.rs:80-157      mask combine (chacha.rs:57-76) -> reconstruct -> unmask -> positive

At 10M-dim the oracle runs the ChaCha streams in full (a few seconds per seed) and recomputes sampled
share batches; the rest is checked by size-independent properties: payload encode -> decode round
trips, linearity of the mask combine over a split seed set, and the recipient's output equal to the
secrets on every element.
"""
import numpy as np
import pytest

from sda_amd import schemes as S
from tests.util import assert_same

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SS = S.CONFIG_PACKED
P, K, T, N = SS.prime_modulus, SS.secret_count, SS.privacy_threshold(), SS.share_count
D = 10_000_000
B = D // K


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _draws(rng, rows, cols, hi):
    return torch.from_numpy(rng.integers(0, hi, size=(rows, cols), dtype=np.int64)).cuda()


def test_config4_participant_10M(engine, oracle):
    """sda_participant_share_dev at configs[4]'s size: the ChaCha(128) mask of the participant's seed,
    packed share generation of the masked vector (tss' exact signed shares), and the 26 clerk payloads.
    Sampled batches equal oracle.packed_share of the oracle's masked secrets; every payload decodes
    back to its clerk's share row, and two rows are byte-identical to the oracle's encoding."""
    rng = np.random.default_rng(0x5DA + 40)
    ms = S.ChaChaMasking(P, D, 128)
    sec_h = rng.integers(0, 1 << 20, size=D, dtype=np.int64)
    seed = [int(v) for v in rng.integers(0, 1 << 32, size=4, dtype=np.uint64)]
    sec = torch.from_numpy(sec_h).cuda()
    drw = _draws(rng, B, T, P - 1)
    sh = torch.empty((N, B), dtype=torch.int64, device="cuda")
    cap = N * B * 6 + 32
    pay = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    rb = engine.participant_share_dev(ms, SS, sec.data_ptr(), D, drw.data_ptr(), sh.data_ptr(), seed=seed,
                                      payload_ptr=pay.data_ptr(), payload_cap=cap, stream=_stream())
    torch.cuda.synchronize()
    masked = oracle.chacha_mask(P, np.array(seed, np.uint32), sec_h)          # chacha.rs:36-45
    pp = oracle.packed_params(K, N, T, P, SS.omega_secrets, SS.omega_shares)
    sh_h, dr_h = sh.cpu().numpy(), drw.cpu().numpy()
    for b in sorted(set(int(x) for x in rng.integers(0, B, 2048)) | {0, B - 1}):
        assert_same(sh_h[:, b], oracle.packed_share(pp, masked[b * K:(b + 1) * K], dr_h[b]))
    # payloads: back to back per clerk (sodium.rs:36-41 encoding), decode -> the share rows
    off = np.concatenate([[0], np.cumsum(rb)]).astype(np.uint64)
    dec = torch.empty((N, B), dtype=torch.int64, device="cuda")
    counts = engine.varint_decode_dev(pay.data_ptr(), off, dec.data_ptr(), B, _stream())
    torch.cuda.synchronize()
    assert (counts == B).all()
    assert torch.equal(dec, sh)
    host = pay[: int(off[-1])].cpu().numpy().tobytes()
    for c in (0, N - 1):
        assert host[int(off[c]):int(off[c + 1])] == oracle.varint_encode(sh_h[c])


def test_config4_recipient_10M(engine, oracle):
    """sda_recipient_reveal_dev at configs[4]'s size with 32 participant seeds: the combined ChaCha mask
    equals the oracle's over 4 full seeds, the 32-seed combine is the sum mod p of its two 16-seed halves,
    and reveal (exact, 15 clerks) -> unmask -> positive returns the secrets on every element."""
    rng = np.random.default_rng(0x5DA + 41)
    ms = S.ChaChaMasking(P, D, 128)
    seeds_h = rng.integers(0, 1 << 32, size=(32, 4), dtype=np.uint64).astype(np.uint32)
    seeds = torch.from_numpy(seeds_h.view(np.int32)).cuda()
    m4 = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.chacha_mask_combine_dev(P, D, seeds.data_ptr(), 4, 4, m4.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert_same(m4.cpu().numpy(), oracle.chacha_mask_combine(P, D, seeds_h[:4].astype(np.int64)))
    mask = torch.empty(D, dtype=torch.int64, device="cuda")
    lo = torch.empty(D, dtype=torch.int64, device="cuda")
    hi = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.chacha_mask_combine_dev(P, D, seeds.data_ptr(), 4, 32, mask.data_ptr(), _stream())
    engine.chacha_mask_combine_dev(P, D, seeds[:16].data_ptr(), 4, 16, lo.data_ptr(), _stream())
    engine.chacha_mask_combine_dev(P, D, seeds[16:].data_ptr(), 4, 16, hi.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert int(mask.min()) >= 0 and int(mask.max()) < P
    assert torch.equal(mask, torch.remainder(lo + hi, P))
    del lo, hi, m4
    # the clerks' combined shares of (secret + mask) mod p, as a participant population would leave them
    sec = torch.from_numpy(rng.integers(0, 1 << 20, size=D, dtype=np.int64)).cuda()
    masked = torch.remainder(sec + mask, P)
    drw = _draws(rng, B, T, P - 1)
    sh = torch.empty((N, B), dtype=torch.int64, device="cuda")
    engine.packed_generate_dev(SS, masked.data_ptr(), D, 1, drw.data_ptr(), sh.data_ptr(), _stream())
    idx = list(range(N - 1, N - 1 - (T + K), -1))
    sub = sh[idx].contiguous()
    del masked, drw, sh
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    got = engine.recipient_reveal_dev(ms, seeds.data_ptr(), 32, 4, SS, D, idx, sub.data_ptr(), B, P, out.data_ptr(),
                                      D, stream=_stream())
    torch.cuda.synchronize()
    assert got == D
    assert torch.equal(out, sec)
