"""GPU: engine-handle behaviour -- calls on several streams, the two exact ChaCha paths, and the
empty / zero-dimension edge cases of the device entry points.
"""
import os

import numpy as np
import pytest

from sda_amd import SdaError, schemes as S
from sda_amd import engine as E
from tests.util import assert_same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def test_calls_on_two_streams_share_scratch_safely(engine, oracle):
    """Packed share-gen uses the handle's fix-up log: a second call on another stream must not reset
    it while the first call's fix-up is still queued (the handle orders the streams)."""
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    B = 20_000
    D = B * k
    rng = np.random.default_rng(21)
    sec_a = rng.integers(-(2**40), 2**40, size=D, dtype=np.int64)      # every batch takes the fix-up
    sec_b = rng.integers(0, p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * t, dtype=np.int64)
    da, db, dd = (torch.from_numpy(x).cuda() for x in (sec_a, sec_b, draws))
    oa = torch.empty((n, B), dtype=torch.int64, device="cuda")
    ob = torch.empty((n, B), dtype=torch.int64, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):
        engine.packed_generate_dev(sch, da.data_ptr(), D, 1, dd.data_ptr(), oa.data_ptr(), s1.cuda_stream)
        engine.packed_generate_dev(sch, db.data_ptr(), D, 1, dd.data_ptr(), ob.data_ptr(), s2.cuda_stream)
    torch.cuda.synchronize()
    pp = oracle.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    ga, gb = oa.cpu().numpy(), ob.cpu().numpy()
    dr = draws.reshape(B, t)
    for b in (0, 1, B // 2, B - 1):
        assert_same(ga[:, b], oracle.packed_share(pp, sec_a[b * k:(b + 1) * k], dr[b]))
        assert_same(gb[:, b], oracle.packed_share(pp, sec_b[b * k:(b + 1) * k], dr[b]))


def test_stream_destroyed_between_calls(engine, oracle):
    """A caller that creates and destroys a HIP stream per call (a C consumer, a torch ExternalStream):
    the next call on another stream orders itself after the previous call through an event recorded
    when that call returned, so it never touches the destroyed stream."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")          # the runtime torch already loaded (one soname)
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    m, N, D = 2147482801, 33, 10_001
    x = np.random.default_rng(5).integers(-(m - 1), m, size=(N, D), dtype=np.int64)
    xd = torch.from_numpy(x).cuda()
    exp = oracle.combine(m, x)
    outs = []
    torch.cuda.synchronize()
    for i in range(4):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        o = torch.empty(D, dtype=torch.int64, device="cuda")
        engine.combine_dev(m, xd.data_ptr(), N, D, D, o.data_ptr(), s.value)
        if i % 2:
            assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0      # destroyed with (i even) or without its work drained
        outs.append(o)
    o = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.combine_dev(m, xd.data_ptr(), N, D, D, o.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for r in outs + [o]:
        assert_same(r.cpu().numpy(), exp)


@pytest.mark.parametrize("m", [2147482801, (1 << 40) + 7])
def test_chacha_stream_path_equals_fast_path(engine, m, monkeypatch):
    """Both exact ChaCha implementations (counter mode + rejection fix-up, and per-stream expansion +
    the sequential combine) agree on a size the oracle cannot finish quickly (96 seeds x 1M)."""
    N, D = 96, 1_000_003
    seeds = torch.randint(0, 2**31 - 1, (N, 4), dtype=torch.int32, device="cuda",
                          generator=torch.Generator(device="cuda").manual_seed(m % 1000))
    fast = torch.empty(D, dtype=torch.int64, device="cuda")
    slow = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.chacha_mask_combine_dev(m, D, seeds.data_ptr(), 4, N, fast.data_ptr())
    torch.cuda.synchronize()
    monkeypatch.setenv("SDA_CHACHA_PATH", "stream")
    engine.chacha_mask_combine_dev(m, D, seeds.data_ptr(), 4, N, slow.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(fast, slow)


def test_chacha_high_rejection_large_dimension(engine, oracle):
    """m = 2^62 + 1 rejects ~25 % of draws: a 1M-dim stream has ~330k rejections, far beyond the
    fast path's log; the stream path handles it (checked on a prefix and on the suffix)."""
    m, D = (1 << 62) + 1, 1_000_000
    seed = [11, 22, 33, 44]
    sch = S.ChaChaMasking(m, D, 128)
    secrets = np.zeros(D, np.int64)
    _, masked = engine.secret_mask(sch, secrets, seed=seed)
    exp = oracle.chacha_mask(m, np.array(seed, np.uint32), secrets)     # (0 + mask) % m == mask
    assert_same(masked, exp)


def test_chacha_dev_zero_dimension_and_no_seeds(engine):
    out = torch.full((5,), 7, dtype=torch.int64, device="cuda")
    seeds = torch.zeros((3, 4), dtype=torch.int32, device="cuda")
    engine.chacha_mask_combine_dev(433, 0, seeds.data_ptr(), 4, 3, out.data_ptr())     # D = 0: nothing
    engine.chacha_mask_combine_dev(433, 5, seeds.data_ptr(), 4, 0, out.data_ptr())     # no seeds: zeros
    torch.cuda.synchronize()
    assert out.tolist() == [0] * 5


def test_reveal_dev_zero_dimension_runs_no_check(engine):
    """batched.rs:77-81: dimension 0 runs no batch, so even too few shares is not an error."""
    sch = S.CONFIG_PACKED
    out = torch.empty(1, dtype=torch.int64, device="cuda")
    engine.packed_reconstruct_dev(sch, 0, [0, 1], 1, out.data_ptr(), out.data_ptr())
    n = engine.recipient_reveal_dev(S.NoMasking(), 0, 0, 0, sch, 0, [0, 1], out.data_ptr(), 0, 433,
                                    out.data_ptr(), 1)
    assert n == 0
    with pytest.raises(SdaError) as ei:
        engine.packed_reconstruct_dev(sch, 8, [0, 1], 1, out.data_ptr(), out.data_ptr())
    assert ei.value.status == E.ERR_NOT_ENOUGH_SHARES
