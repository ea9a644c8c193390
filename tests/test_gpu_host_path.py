"""The streaming, multi-device host path of the C ABI (include/sda_engine.h, engine.cpp "host path" section)
against the oracle, through the host trait entry points the Rust shim calls:

  sda_share_combine     ShareCombiner::combine   (clerk.rs:85-86 -> combiner.rs:16-28)
  sda_mask_combine      MaskCombiner::combine    (receive.rs:113-116 -> full.rs:38-50, chacha.rs:57-76)
  sda_share_generate    ShareGenerator::generate (participate.rs:75-76 -> batched.rs:19-53)
  sda_secret_reconstruct SecretReconstructor::reconstruct (receive.rs:140-145 -> batched.rs:69-97)

Rows stream in row tiles through pinned double buffers (a forced 1 MiB stage makes every case many tiles and,
for wide rows, column chunks); a handle over several devices splits by columns / batches / seeds.  Ordinals
may repeat, so the splits run here on one MI355X (the ChaCha seed split then stays on one device; a one-device
handle reduces through a one-rank RCCL communicator).  Bit-exact against oracle/sda_oracle.c."""
import numpy as np
import pytest

from sda_amd import Engine, schemes as S
from tests.util import assert_same

pytestmark = pytest.mark.gpu

P = S.CONFIG_PACKED.prime_modulus


@pytest.fixture(scope="module")
def multi3():
    e = Engine(devices=[0, 0, 0])
    yield e
    e.close()


@pytest.fixture(scope="module")
def multi1():
    e = Engine(devices=[0])
    yield e
    e.close()


def _rows(N, D, seed, signed=True, m=P):
    rng = np.random.default_rng(seed)
    lo = -(m - 1) if signed else 0
    return [rng.integers(lo, m, size=D, dtype=np.int64) for _ in range(N)]


@pytest.mark.parametrize("stage_mb", ["1", "256"])
@pytest.mark.parametrize("N,D", [(1, 5), (37, 100_003), (5, 300_001), (64, 2)])
def test_share_combine_streams_row_tiles(engine, oracle, monkeypatch, stage_mb, N, D):
    """Signed rows through the streaming path: a 1 MiB stage (a few rows per tile, and column chunks for the
    300k-wide rows) and the default stage give the reference's recurrence bit for bit."""
    monkeypatch.setenv("SDA_HOST_STAGE_MB", stage_mb)
    rows = _rows(N, D, N * 7 + D)
    got = engine.share_combine(S.Additive(3, P), rows)
    assert_same(got, oracle.combine(P, np.stack(rows)), f"N={N} D={D} stage={stage_mb}")


def test_share_combine_larger_than_stage_small_modulus(engine, oracle, monkeypatch):
    """A job 24x the staging tile with a small modulus (a sign event in almost every step) and rows that are
    not contiguous in host memory."""
    monkeypatch.setenv("SDA_HOST_STAGE_MB", "1")
    m = 7
    big = np.random.default_rng(3).integers(-6, 7, size=(200, 2 * 65_536 + 9), dtype=np.int64)
    rows = [big[i, :] for i in range(0, 200, 2)] + [big[i, :].copy() for i in range(1, 200, 2)]
    got = engine.share_combine(S.Additive(3, m), rows)
    assert_same(got, oracle.combine(m, np.stack(rows)), "small m")


@pytest.mark.parametrize("D", [1, 2, 3, 10_001, 65_538])
def test_multi_column_split_combine(multi3, oracle, monkeypatch, D):
    """Three column slices (on one GPU): ShareCombiner, Full MaskCombiner and Additive reconstruct equal the
    single-pass oracle, slices of 1-2 columns and empty slices included."""
    monkeypatch.setenv("SDA_HOST_STAGE_MB", "1")
    assert multi3.device_count() == 3
    rows = _rows(23, D, D)
    exp = oracle.combine(P, np.stack(rows))
    assert_same(multi3.share_combine(S.Additive(3, P), rows), exp, "share_combine")
    assert_same(multi3.secret_reconstruct(S.Additive(23, P), D, list(enumerate(rows))), exp, "additive reveal")
    masks = _rows(9, D, D + 1, signed=False)
    assert_same(multi3.mask_combine(S.FullMasking(P), masks), oracle.combine(P, np.stack(masks)), "full masks")


def test_multi_errors_match_single(multi3, engine):
    """Validation runs before any split: the reference's errors, unchanged."""
    from sda_amd import SdaError
    from sda_amd import engine as E
    for eng in (engine, multi3):
        with pytest.raises(SdaError) as ei:
            eng.share_combine(S.Additive(3, P), [[1, 2, 3], [1, 2]])
        assert ei.value.status == E.ERR_WRONG_DIMENSION
        assert eng.share_combine(S.Additive(3, P), []).size == 0


@pytest.mark.parametrize("handle", ["multi1", "multi3", "single"])
def test_chacha_mask_combine_seed_split(request, oracle, handle):
    """ChaCha MaskCombiner::combine: a one-device multi handle takes the seed split with a one-rank RCCL reduce,
    the repeated-ordinal handle and the plain handle run on one device; all equal the oracle."""
    eng = request.getfixturevalue("engine" if handle == "single" else handle)
    D = 4099
    seeds = np.random.default_rng(9).integers(0, 1 << 32, size=(7, 4), dtype=np.int64)
    ms = S.ChaChaMasking(P, D, 128)
    got = eng.mask_combine(ms, [list(s) for s in seeds])
    assert_same(got, oracle.chacha_mask_combine(P, D, seeds), handle)


@pytest.mark.parametrize("handle", ["multi1", "multi3"])
def test_multi_generate_and_reconstruct(request, engine, oracle, handle):
    """Batch split of packed share-gen and exact reconstruct, column split of additive share-gen: the same
    bytes as the one-device handle and the oracle (ragged last batch included)."""
    eng = request.getfixturevalue(handle)
    ss = S.CONFIG_PACKED
    k, t, n = ss.secret_count, ss.privacy_threshold(), ss.share_count
    D = 8 * 1001 + 3
    B = (D + k - 1) // k
    rng = np.random.default_rng(21)
    sec = rng.integers(-(P - 1), P, size=D, dtype=np.int64)
    draws = rng.integers(0, P - 1, size=B * t, dtype=np.int64)
    got = eng.share_generate(ss, sec, draws)
    pp = oracle.packed_params(k, n, t, P, ss.omega_secrets, ss.omega_shares)
    exp = oracle.packed_generate(pp, sec, draws)
    assert_same(got, exp, "packed generate")
    assert_same(got, engine.share_generate(ss, sec, draws), "vs one device")
    idx = [25, 2, 14, 7, 19, 0, 11, 23, 5, 16, 9, 21, 3, 13, 18]
    indexed = [(c, exp[c]) for c in idx]
    assert_same(eng.secret_reconstruct(ss, D, indexed), oracle.packed_reconstruct(pp, D, idx, exp[idx])[1], "reveal")
    add = S.Additive(4, P)
    adraws = rng.integers(0, P, size=D * 3, dtype=np.int64)
    assert_same(eng.share_generate(add, sec, adraws), oracle.additive_generate(P, 4, sec, adraws), "additive")


def test_share_combine_host_rows_large(engine, oracle):
    """A clerk job from host rows at 1M-dim, 400 participations (3.2 GB: 12 default tiles): the streamed
    result equals the device combine of the same rows and the oracle on sampled columns."""
    import torch
    N, D = 400, 1_000_000
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 77, -(P - 1), P, torch.cuda.current_stream().cuda_stream)
    dev_out = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.combine_dev(P, x.data_ptr(), N, D, D, dev_out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    host = x.cpu().numpy()
    del x
    got = engine.share_combine(S.Additive(3, P), [host[i] for i in range(N)])
    assert_same(got, dev_out.cpu().numpy(), "host vs device")
    cols = np.random.default_rng(1).choice(D, 512, replace=False)
    assert_same(got[cols], oracle.combine(P, np.ascontiguousarray(host[:, cols])), "oracle sample")


def test_clerk_decode_combine_streams_blob_groups(engine, oracle, monkeypatch):
    """sda_clerk_decode_combine (clerk.rs:79-86 after the sealed-box opens) through the streaming path: a 1 MiB
    stage puts the 120 payloads in ~60 groups; signed field shares, a few raw i64 participations (10-byte
    varints) and a malformed one (a run of continuation bytes, decoded as sodium.rs:82-88 does) give the
    oracle's decode + combine bit for bit; the errors keep the reference's order across groups."""
    from sda_amd import SdaError
    from sda_amd import engine as E
    monkeypatch.setenv("SDA_HOST_STAGE_MB", "1")
    rng = np.random.default_rng(5)
    N, D = 120, 100_003
    x = rng.integers(-(P - 1), P, size=(N, D), dtype=np.int64)
    x[17] = rng.integers(-(1 << 62), 1 << 62, size=D, dtype=np.int64)
    x[90, :5] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, -1, 0, 1 << 40]
    blobs = [oracle.varint_encode(r) for r in x]
    mal = bytearray(blobs[64])
    mal[1000:1000 + 12] = b"\x80" * 12                       # one 11+-byte run: sodium.rs decodes it anyway
    blobs[64] = bytes(mal)
    rows = [oracle.varint_decode(b) for b in blobs]
    same_len = all(r.size == D for r in rows)
    got = None
    if same_len:
        got = engine.clerk_decode_combine(S.Additive(3, P), blobs)
        assert_same(got, oracle.combine(P, np.stack(rows)), "streamed decode+combine")
    else:                                                    # the malformed run changed the length: Wrong dimension
        with pytest.raises(SdaError) as ei:
            engine.clerk_decode_combine(S.Additive(3, P), blobs)
        assert ei.value.status == E.ERR_WRONG_DIMENSION and "participation 64" in str(ei.value)
        blobs[64] = oracle.varint_encode(x[64])
        got = engine.clerk_decode_combine(S.Additive(3, P), blobs)
        assert_same(got, oracle.combine(P, x), "streamed decode+combine")
    # a participation in a late group of another length: Err("Wrong dimension") naming it
    bad = list(blobs)
    bad[101] = oracle.varint_encode(x[101][:-1])
    with pytest.raises(SdaError) as ei:
        engine.clerk_decode_combine(S.Additive(3, P), bad)
    assert ei.value.status == E.ERR_WRONG_DIMENSION and "participation 101" in str(ei.value)
    # m = 0: participation 0 is folded before any other length is checked (combiner.rs:20-25)
    with pytest.raises(SdaError) as ei:
        engine.clerk_decode_combine(S.Additive(3, 0), bad)
    assert ei.value.status == E.ERR_PRECONDITION
    assert engine.clerk_decode_combine(S.Additive(3, 0), [b"", b""]).size == 0


@pytest.mark.parametrize("handle", ["multi1", "multi3"])
def test_recipient_reveal_multi_handle(request, handle):
    """sda_recipient_reveal (receive.rs:80-157 + positive()) on a multi-device handle: the ChaCha mask combine runs
    through the seed split (one-rank RCCL reduce on multi1, one device on the repeated-ordinal multi3), the rest on
    device 0 with the combined mask as a Full row; equal to the step-wise oracle flow for every ChaCha case of
    test_gpu_pipelines (the full_loop KAT included), both clerk orders."""
    from tests.oracle_backend import OracleBackend
    from tests.pipeline import Draws, run_aggregation
    from tests.test_gpu_pipelines import _cases
    eng = request.getfixturevalue(handle)
    for name, ms, ss, m, D, inputs, expected in _cases():
        if not isinstance(ms, S.ChaChaMasking):
            continue
        tr = run_aggregation(OracleBackend(), ms, ss, m, D, inputs, Draws(0x5DA))
        n = ss.output_size()
        for order in (list(range(n)), list(reversed(range(n)))):
            if isinstance(ss, S.PackedShamir):
                order = order[: ss.reconstruction_threshold() + 1]
            indexed = [(c, tr.clerk_results[c]) for c in order]
            be = OracleBackend()
            exp = be.positive(m, be.secret_unmask(ms, (be.mask_combine(ms, tr.masks), be.secret_reconstruct(ss, D, indexed))))
            assert_same(eng.recipient_reveal(ms, tr.masks, ss, D, indexed, m), exp, f"{handle} {name}")
