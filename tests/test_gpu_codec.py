"""GPU parity of the share payload codec against the oracle.

Reference: client/src/crypto/encryption/sodium.rs:36-41 (encode), :82-88 (decode) with
integer-encoding 1.0 VarInt for i64 (zigzag + LEB128; third-party, restated in the oracle and
pinned by the protobuf sint64 known answers in test_oracle_golden.py).  Bit-exact.
"""
import os

import numpy as np
import pytest

from sda_amd import SdaError, schemes as S
from sda_amd import engine as E
from tests.util import assert_same

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

I64_MIN, I64_MAX = -(2**63), 2**63 - 1
EDGE = [0, -1, 1, 63, -64, 64, -65, 8191, -8192, 8192, 2**31 - 1, -(2**31), 2**62, -(2**62) - 1,
        I64_MIN, I64_MAX, 433, -432, 2147482800, -2147482800]


def _values(rng, n):
    """a mix of byte lengths: small, field-sized (~31 bit) and full-range values"""
    kind = rng.integers(0, 4, size=n)
    v = np.where(kind == 0, rng.integers(-200, 200, size=n),
                 np.where(kind == 1, rng.integers(-(2**31), 2**31, size=n),
                          np.where(kind == 2, rng.integers(-(2**45), 2**45, size=n),
                                   rng.integers(I64_MIN, I64_MAX, size=n, dtype=np.int64))))
    return v.astype(np.int64)


def test_encode_matches_oracle(engine, oracle):
    rng = np.random.default_rng(1)
    for vals in (np.array(EDGE, np.int64), _values(rng, 1), _values(rng, 4095), _values(rng, 4096),
                 _values(rng, 70_001), np.zeros(0, np.int64)):
        assert engine.varint_encode(vals) == oracle.varint_encode(vals)


def test_decode_matches_oracle(engine, oracle):
    rng = np.random.default_rng(2)
    for vals in (np.array(EDGE, np.int64), _values(rng, 3), _values(rng, 10_000), _values(rng, 123_457)):
        data = oracle.varint_encode(vals)
        got = engine.varint_decode(data)
        assert_same(got, vals)
        assert_same(got, oracle.varint_decode(data))
    assert engine.varint_decode(b"").size == 0


@pytest.mark.parametrize("blob", [
    bytes([0x80]),                                   # truncated final varint -> partial value
    bytes([0x05, 0xFF, 0xFF]),                        # value, then a truncated tail
    bytes([0xFF] * 10 + [0x01]),                      # 10 continuation + terminator = one 11-byte element
    bytes([0xFF] * 11 + [0x01]),                      # 11 continuation bytes: an 11-byte element, then 0x01
    bytes([0xFF] * 25 + [0x02, 0x03]),                # long run: sequential (irregular) path
    bytes([0xFF] * 10),                               # 10-byte truncated tail
    bytes([0x80] * 9 + [0x00]),                       # overlong zero
])
def test_decode_malformed_like_reference(engine, oracle, blob):
    assert_same(engine.varint_decode(blob), oracle.varint_decode(blob))


def _pack(blobs, pad_to=16):
    """concatenate blobs at arbitrary (unaligned) offsets into one 16-byte aligned device buffer"""
    off = [0]
    for b in blobs:
        off.append(off[-1] + len(b))
    host = b"".join(blobs) + bytes(32)
    t = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    assert t.data_ptr() % 16 == 0
    return t, off


def test_decode_dev_many_blobs(engine, oracle):
    rng = np.random.default_rng(3)
    rows = [_values(rng, int(n)) for n in (0, 1, 5, 700, 4096, 9000, 1, 33_333)]
    blobs = [oracle.varint_encode(r) for r in rows]
    blobs[3] = blobs[3] + bytes([0xFF] * 14 + [0x7F])        # an irregular blob among regular ones
    rows[3] = oracle.varint_decode(blobs[3])
    t, off = _pack(blobs)
    stride = max(r.size for r in rows)
    out = torch.full((len(rows), stride), 7, dtype=torch.int64, device="cuda")
    counts = engine.varint_decode_dev(t.data_ptr(), off, out.data_ptr(), stride)
    assert counts.tolist() == [r.size for r in rows]
    o = out.cpu().numpy()
    for i, r in enumerate(rows):
        assert_same(o[i, :r.size], r, f"blob {i}")


def test_clerk_decode_combine(engine, oracle):
    """clerk.rs:79-86: decrypted payloads -> decode -> ShareCombiner::combine (signed, order-dependent)"""
    rng = np.random.default_rng(4)
    m = 2147482801
    x = rng.integers(-(m - 1), m, size=(37, 5003), dtype=np.int64)
    blobs = [oracle.varint_encode(r) for r in x]
    got = engine.clerk_decode_combine(S.Additive(3, m), blobs)
    assert_same(got, oracle.combine(m, x))
    # a participation of a different length: Err("Wrong dimension") (combiner.rs:21)
    bad = blobs[:5] + [oracle.varint_encode(x[5][:-1])] + blobs[6:]
    with pytest.raises(SdaError) as ei:
        engine.clerk_decode_combine(S.Additive(3, m), bad)
    assert ei.value.status == 3
    assert engine.clerk_decode_combine(S.Additive(3, m), []).size == 0
    # m = 0: blob 0 is folded before blob 1's length is checked (combiner.rs:20-25) -> the panic wins
    for path in ("slots", "matrix"):
        os.environ["SDA_CODEC_PATH"] = path
        try:
            with pytest.raises(SdaError) as ei:
                engine.clerk_decode_combine(S.Additive(3, 0), bad)
            assert ei.value.status == E.ERR_PRECONDITION, path
        finally:
            os.environ.pop("SDA_CODEC_PATH", None)


def test_clerk_decode_combine_dev_and_encode_dev(engine, oracle):
    """device round trip at a larger size: encode_dev -> decode+combine_dev == combine"""
    m = 2147482801
    N, D = 64, 100_003
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 0x5DA + 7, -(m - 1), m)
    cap = N * D * 10 + 32
    buf = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    row_bytes = engine.varint_encode_dev(x.data_ptr(), N, D, D, buf.data_ptr(), cap)
    off = np.concatenate([[0], np.cumsum(row_bytes)]).astype(np.uint64)
    xh = x.cpu().numpy()
    host = buf[: int(off[-1])].cpu().numpy().tobytes()
    for i in (0, 17, N - 1):                                   # bytes equal the oracle's encoding
        assert host[int(off[i]):int(off[i + 1])] == oracle.varint_encode(xh[i])
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    n = engine.clerk_decode_combine_dev(m, buf.data_ptr(), off, out.data_ptr(), D)
    torch.cuda.synchronize()
    assert n == D
    assert_same(out.cpu().numpy(), oracle.combine(m, xh))


@pytest.mark.parametrize("vec", ["2", "4"])
def test_clerk_decode_combine_narrow_and_wide(engine, oracle, monkeypatch, vec):
    """The clerk's decode -> combine keeps the decoded matrix as int32 when every value fits (field
    shares), and falls back to int64 when one does not: both give combiner.rs:16-28's exact result.
    Edges: -2^31 and 2^31 - 1 fit; 2^31 and -2^31 - 1 do not."""
    monkeypatch.setenv("SDA_COMBINE32_VEC", vec)
    m = 2147482801
    rng = np.random.default_rng(5)
    N, D = 23, 8004
    x = rng.integers(-(m - 1), m, size=(N, D), dtype=np.int64)
    x[3, 5], x[4, 6], x[7, D - 1] = -(2**31), 2**31 - 1, -(2**31)
    cases = {"fits": x}
    for name, big in (("above", 2**31), ("below", -(2**31) - 1), ("i64", I64_MIN + 5)):
        y = x.copy()
        y[N - 1, D // 2] = big
        cases[name] = y
    for name, rows in cases.items():
        blobs = [oracle.varint_encode(r) for r in rows]
        t, off = _pack(blobs)
        out = torch.empty(D, dtype=torch.int64, device="cuda")
        n = engine.clerk_decode_combine_dev(m, t.data_ptr(), off, out.data_ptr(), D)
        torch.cuda.synchronize()
        assert n == D
        assert_same(out.cpu().numpy(), oracle.combine(m, rows), name)
        monkeypatch.setenv("SDA_CODEC_NARROW", "0")                      # the int64 path alone
        out.fill_(7)
        engine.clerk_decode_combine_dev(m, t.data_ptr(), off, out.data_ptr(), D)
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy(), oracle.combine(m, rows), name + " (int64)")
        monkeypatch.delenv("SDA_CODEC_NARROW")


@pytest.mark.parametrize("run", [4, 5, 6, 10, 11, 12, 25])
def test_continuation_runs_at_every_alignment(engine, oracle, monkeypatch, run):
    """Runs of `run` continuation bytes placed at every byte offset of a 16-byte word (and across word
    and 4 KiB sub-region boundaries): the count pass classifies a blob from them -- 11 in a row make it
    irregular (sequential decoder, as u64::decode_var stops at shift > 70), 5 or more mark elements of
    >= 6 bytes (the fused path's multi-round variant).  Both decode paths and both decode+combine paths
    must equal the oracle whatever the alignment."""
    rng = np.random.default_rng(100 + run)
    m = 2147482801
    S = 4200                                        # elements per blob (past one 4 KiB sub-region)
    rows, blobs = [], []
    for shift in list(range(0, 34)) + [4070, 4085, 4090, 4095, 4100]:
        pre = bytes(shift)                          # `shift` one-byte zeros
        mid = bytes([0xFF] * run + [0x01])
        base = oracle.varint_decode(pre + mid)      # the run's element(s) as the reference decodes them
        tail = oracle.varint_encode(rng.integers(-(m - 1), m, size=S - base.size, dtype=np.int64))
        blob = pre + mid + tail
        r = oracle.varint_decode(blob)
        assert r.size == S
        rows.append(r)
        blobs.append(blob)
    rows = np.stack(rows)
    t, off = _pack(blobs)
    out = torch.full((len(blobs), S), 7, dtype=torch.int64, device="cuda")
    counts = engine.varint_decode_dev(t.data_ptr(), off, out.data_ptr(), S)
    assert counts.tolist() == [S] * len(blobs)
    assert_same(out.cpu().numpy(), rows, f"decode run={run}")
    exp = oracle.combine(m, rows)
    for path in ("matrix", "fused", "slots"):
        monkeypatch.setenv("SDA_CODEC_PATH", path)
        res = torch.full((S,), 7, dtype=torch.int64, device="cuda")
        assert engine.clerk_decode_combine_dev(m, t.data_ptr(), off, res.data_ptr(), S) == S
        torch.cuda.synchronize()
        assert_same(res.cpu().numpy(), exp, f"{path} run={run}")


@pytest.mark.parametrize("case", ["one_byte", "one_region", "exact_cap", "mixed_blobs"])
def test_slot_cap_overflow_falls_back(engine, oracle, monkeypatch, case):
    """The slot decode keeps 4096 slots per 16 KiB region (every element of >= 4 bytes fits); a region
    with more elements (short ones) raises the wide flag and the job takes the matrix path.  Either way
    the result is combiner.rs:16-28's exact one.  exact_cap: 4-byte elements fill a region to exactly
    4096 (no fallback, gap 0)."""
    rng = np.random.default_rng(77)
    m = 2147482801
    N, D = 6, 40_000
    x = rng.integers(-(m - 1), m, size=(N, D), dtype=np.int64)
    if case == "one_byte":                       # every element one byte: 16,384 per region
        x = rng.integers(-64, 64, size=(N, D), dtype=np.int64)
    elif case == "one_region":                   # a run of 9,000 one-byte elements inside a normal blob
        x[2, 10_000:19_000] = rng.integers(-64, 64, size=9_000)
    elif case == "exact_cap":                    # zigzag in [2^21, 2^28): 4 bytes each, blob 0 region-aligned
        mag = rng.integers(2**20, 2**27, size=(N, D), dtype=np.int64)
        x = np.where(rng.integers(0, 2, size=(N, D)) == 1, mag, -mag - 1)
    else:                                        # blobs alternate between short and field-size elements
        x[1::2] = rng.integers(-8000, 8000, size=(N // 2, D), dtype=np.int64)
    blobs = [oracle.varint_encode(r) for r in x]
    if case == "exact_cap":
        assert all(len(b) == 4 * D for b in blobs)
    t, off = _pack(blobs)
    exp = oracle.combine(m, x)
    for path in ("slots", "matrix"):
        monkeypatch.setenv("SDA_CODEC_PATH", path)
        res = torch.full((D,), 7, dtype=torch.int64, device="cuda")
        assert engine.clerk_decode_combine_dev(m, t.data_ptr(), off, res.data_ptr(), D) == D
        torch.cuda.synchronize()
        assert_same(res.cpu().numpy(), exp, f"{case} {path}")


def test_encode_dev_capacity(engine, oracle):
    """The encode places its rows on the device; a dst_cap one byte short of the rows' total is refused
    (ERR_INVALID_ARGUMENT) with nothing written, and the exact capacity works."""
    m = 2147482801
    rng = np.random.default_rng(21)
    x = rng.integers(-(m - 1), m, size=(5, 3001), dtype=np.int64)
    total = sum(len(oracle.varint_encode(r)) for r in x)
    xd = torch.as_tensor(x).cuda()
    buf = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    with pytest.raises(SdaError) as ei:
        engine.varint_encode_dev(xd.data_ptr(), 5, 3001, 3001, buf.data_ptr(), total - 1)
    assert ei.value.status == E.ERR_INVALID_ARGUMENT
    torch.cuda.synchronize()
    assert (buf.cpu().numpy() == 0xA5).all()
    rb = engine.varint_encode_dev(xd.data_ptr(), 5, 3001, 3001, buf.data_ptr(), total)
    torch.cuda.synchronize()
    assert int(rb.sum()) == total
    host = buf.cpu().numpy().tobytes()
    assert host[:total] == b"".join(oracle.varint_encode(r) for r in x)
    assert (buf.cpu().numpy()[total:] == 0xA5).all()


@pytest.mark.parametrize("path", ["slots", "matrix"])
def test_decode_combine_errors_leave_output(engine, oracle, monkeypatch, path):
    """The slot path queues its combine before the host has seen the element counts; the combine exits on
    the device when the blobs decode to different lengths, when the dimension exceeds out_cap, or when the
    modulus is invalid -- the call then returns the reference's error and `out` is untouched.  (m = 0 with
    only empty blobs is no error: combiner.rs computes no %.)"""
    monkeypatch.setenv("SDA_CODEC_PATH", path)
    m = 2147482801
    rng = np.random.default_rng(31)
    rows = [rng.integers(-(m - 1), m, size=5000, dtype=np.int64) for _ in range(4)]
    good = [oracle.varint_encode(r) for r in rows]
    out = torch.full((5000,), 7, dtype=torch.int64, device="cuda")

    def run(blobs, modulus, cap):
        t, off = _pack(blobs)
        return engine.clerk_decode_combine_dev(modulus, t.data_ptr(), off, out.data_ptr(), cap)

    bad = good[:2] + [oracle.varint_encode(rows[2][:4999])] + good[3:]
    for blobs, modulus, cap, status in ((bad, m, 5000, E.ERR_WRONG_DIMENSION), (good, m, 4999, E.ERR_INVALID_ARGUMENT),
                                        (good, 0, 5000, E.ERR_PRECONDITION)):
        with pytest.raises(SdaError) as ei:
            run(blobs, modulus, cap)
        assert ei.value.status == status
        torch.cuda.synchronize()
        assert (out.cpu().numpy() == 7).all()
    assert run([b"", b""], 0, 5000) == 0
    assert run(good, m, 5000) == 5000
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), oracle.combine(m, np.stack(rows)))


@pytest.mark.parametrize("irregular", [False, True])
def test_decode_dev_capacity_leaves_output(engine, oracle, irregular):
    """sda_varint_decode_dev counts, checks out_stride and decodes without a host wait in between: a blob
    with more values than out_stride (a regular one, or a malformed one the sequential decoder takes) stops
    every write on the device -- the call fails with nothing written; out_stride = the longest blob works."""
    rng = np.random.default_rng(41)
    rows = [rng.integers(-(2**40), 2**40, size=n, dtype=np.int64) for n in (3000, 3100, 2900)]
    blobs = [oracle.varint_encode(r) for r in rows]
    if irregular:                                   # 12 continuation bytes: u64::decode_var's shift > 70 stop
        blobs[1] = bytes([0xFF] * 12 + [0x01]) + blobs[1]
    exp = [oracle.varint_decode(b) for b in blobs]
    longest = max(e.size for e in exp)
    t, off = _pack(blobs)
    out = torch.full((3, longest), 7, dtype=torch.int64, device="cuda")
    with pytest.raises(SdaError) as ei:
        engine.varint_decode_dev(t.data_ptr(), off, out.data_ptr(), longest - 1)
    assert ei.value.status == E.ERR_INVALID_ARGUMENT
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == 7).all()
    counts = engine.varint_decode_dev(t.data_ptr(), off, out.data_ptr(), longest)
    torch.cuda.synchronize()
    assert counts.tolist() == [e.size for e in exp]
    got = out.cpu().numpy()
    for i, e in enumerate(exp):
        assert_same(got[i, :e.size], e)


@pytest.mark.parametrize("group", ["1", "3", "7", "64"])
def test_grouped_slot_path(engine, oracle, monkeypatch, group):
    """SDA_CODEC_GROUP: the slot path decoded and combined a group of blobs at a time, the recurrence's state
    carried between groups.  Results equal combiner.rs:16-28's for signed shares; a blob of another length
    in the LAST group, a short out_cap and a wide element (matrix fall-back) behave as the one-pass path
    (error, out untouched / the exact result)."""
    monkeypatch.setenv("SDA_CODEC_PATH", "slots")
    monkeypatch.setenv("SDA_CODEC_GROUP", group)
    m = 2147482801
    rng = np.random.default_rng(91)
    N, D = 23, 20_011
    x = rng.integers(-(m - 1), m, size=(N, D), dtype=np.int64)
    x[::4, :50] = rng.integers(-64, 64, size=(len(range(0, N, 4)), 50))     # short elements too
    blobs = [oracle.varint_encode(r) for r in x]
    t, off = _pack(blobs)
    out = torch.full((D,), 7, dtype=torch.int64, device="cuda")
    assert engine.clerk_decode_combine_dev(m, t.data_ptr(), off, out.data_ptr(), D) == D
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), oracle.combine(m, x), f"group {group}")
    # the last blob one element short: Wrong dimension, out untouched
    bad = blobs[:-1] + [oracle.varint_encode(x[-1][:-1])]
    tb, offb = _pack(bad)
    out.fill_(7)
    with pytest.raises(SdaError) as ei:
        engine.clerk_decode_combine_dev(m, tb.data_ptr(), offb, out.data_ptr(), D)
    assert ei.value.status == E.ERR_WRONG_DIMENSION
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == 7).all()
    with pytest.raises(SdaError) as ei:
        engine.clerk_decode_combine_dev(m, t.data_ptr(), off, out.data_ptr(), D - 1)
    assert ei.value.status == E.ERR_INVALID_ARGUMENT
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == 7).all()
    # a value past int32 in the last blob: the job takes the matrix path, still exact
    y = x.copy()
    y[-1, D // 2] = 2**40
    ty, offy = _pack([oracle.varint_encode(r) for r in y])
    assert engine.clerk_decode_combine_dev(m, ty.data_ptr(), offy, out.data_ptr(), D) == D
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), oracle.combine(m, y), f"group {group} wide")
