"""GPU parity of the clerk's fused decode -> combine (codec.hip varint_decode_combine_kernel) against
the oracle: clerk.rs:79-86 decodes every decrypted participation (sodium.rs:82-88, integer-encoding
VarInt) and folds it into ShareCombiner::combine (combiner.rs:16-28), exact and order-dependent for
signed shares.  Bit-exact.

The fused path walks column tiles of 1,536 elements; its plan locates each tile's first element in
every payload through the count pass's 256-byte sub-chunk counts.  The cases below put tile edges on
every kind of byte position: element lengths 1..10 (zeros, field shares, full-range i64), dimensions
either side of a tile, payloads at unaligned offsets, truncated final varints, jobs with elements of
>= 6 bytes (the multi-round variant, slices longer than one word per lane), and moduli from 1 to
i64::MAX (negative ones as |m|, as Rust's `%`).
`SDA_CODEC_PATH=fused` selects it (it measured slower, profiles/r02d/ab_codec_fused.txt, so it is opt-in);
`=matrix` the count pass + dense int32 matrix + combine; `=slots` (or unset: the default) the single
decode into int32 slots per 16 KiB region + the combine over the slots (round 3).  All three must agree
with the oracle on every case; elements longer than 5 bytes send the slot path to the matrix path.
"""
import numpy as np
import pytest

from tests.util import assert_same

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

I64_MIN, I64_MAX = -(2**63), 2**63 - 1
M31 = 2147482801


def _pack(blobs):
    off = [0]
    for b in blobs:
        off.append(off[-1] + len(b))
    host = b"".join(blobs) + bytes(32)
    t = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    assert t.data_ptr() % 16 == 0
    return t, off


def _run(engine, m, blobs, dim, path, monkeypatch):
    monkeypatch.setenv("SDA_CODEC_PATH", path)
    t, off = _pack(blobs)
    out = torch.full((max(dim, 1),), 7, dtype=torch.int64, device="cuda")
    n = engine.clerk_decode_combine_dev(m, t.data_ptr(), off, out.data_ptr(), out.numel())
    torch.cuda.synchronize()
    assert n == dim
    return out[:dim].cpu().numpy()


def _rows(rng, kind, n, d):
    if kind == "field":
        return rng.integers(-(M31 - 1), M31, size=(n, d), dtype=np.int64)
    if kind == "zeros":                                    # 1-byte elements: 16 per word
        return np.zeros((n, d), np.int64)
    if kind == "small":
        return rng.integers(-64, 64, size=(n, d), dtype=np.int64)
    if kind == "wide":                                     # 10-byte elements: slices of 2+ rounds (multi)
        return rng.choice(np.array([I64_MIN, I64_MAX, I64_MIN + 1, -(2**62) - 7, 2**63 - 9], np.int64), size=(n, d))
    # mixed lengths 1..10, a different pattern per row
    k = rng.integers(0, 4, size=(n, d))
    return np.where(k == 0, rng.integers(-200, 200, size=(n, d)),
                    np.where(k == 1, rng.integers(-(2**31), 2**31, size=(n, d)),
                             np.where(k == 2, rng.integers(-(2**45), 2**45, size=(n, d)),
                                      rng.integers(I64_MIN, I64_MAX, size=(n, d), dtype=np.int64)))).astype(np.int64)


@pytest.mark.parametrize("kind", ["field", "zeros", "small", "wide", "mixed"])
@pytest.mark.parametrize("dim", [1, 2, 1535, 1536, 1537, 3072, 5003])
def test_fused_decode_combine_shapes(engine, oracle, monkeypatch, kind, dim):
    rng = np.random.default_rng(dim * 7 + len(kind))
    n = 5 if kind in ("wide", "mixed") else 9
    x = _rows(rng, kind, n, dim)
    blobs = [oracle.varint_encode(r) for r in x]
    exp = oracle.combine(M31, x)
    for path in ("fused", "matrix", "slots"):
        assert_same(_run(engine, M31, blobs, dim, path, monkeypatch), exp, f"{kind} {path}")


@pytest.mark.parametrize("m", [1, 2, 7, -M31, 2**31 + 11, 2**62 + 1, I64_MAX])
def test_fused_decode_combine_moduli(engine, oracle, monkeypatch, m):
    """combiner.rs:22-25 for any modulus: wrapping add, truncated %, |m| for negative m"""
    rng = np.random.default_rng(abs(m) % 1000)
    x = _rows(rng, "mixed", 6, 3001)
    x[0, :8] = [I64_MAX, I64_MAX, I64_MIN, -1, 0, 1, I64_MIN, I64_MAX]
    blobs = [oracle.varint_encode(r) for r in x]
    for path in ("fused", "slots"):
        assert_same(_run(engine, m, blobs, 3001, path, monkeypatch), oracle.combine(m, x), path)


def test_fused_decode_combine_truncated_tails(engine, oracle, monkeypatch):
    """a truncated final varint decodes to its partial value (sodium.rs:82-88 + integer-encoding):
    every payload ends in one, so all decode to the same count"""
    rng = np.random.default_rng(11)
    x = _rows(rng, "field", 7, 2047)
    blobs = [oracle.varint_encode(r) + bytes([0x80 | int(rng.integers(0, 128))] * int(rng.integers(1, 9)))
             for r in x]
    rows = np.stack([oracle.varint_decode(b) for b in blobs])
    assert rows.shape == (7, 2048)
    for path in ("fused", "slots"):
        assert_same(_run(engine, M31, blobs, 2048, path, monkeypatch), oracle.combine(M31, rows), path)


def test_fused_decode_combine_many_blobs_ragged_offsets(engine, oracle, monkeypatch):
    """100 participations with different byte lengths (unaligned offsets), more blobs than one prefetch
    ring and a dimension past 16 KiB regions"""
    rng = np.random.default_rng(12)
    D = 12_345
    x = np.concatenate([_rows(rng, "field", 60, D), _rows(rng, "mixed", 25, D), _rows(rng, "zeros", 15, D)])
    x = x[rng.permutation(x.shape[0])]
    blobs = [oracle.varint_encode(r) for r in x]
    exp = oracle.combine(M31, x)
    for path in ("fused", "matrix", "slots"):
        assert_same(_run(engine, M31, blobs, D, path, monkeypatch), exp, path)


def test_fused_decode_combine_at_scale(engine, oracle, monkeypatch):
    """64 x 400,003 field shares on the device (encode_dev -> decode+combine_dev), both paths, equal to the
    oracle's combine on every column"""
    N, D = 64, 400_003
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 0xF05ED, -(M31 - 1), M31)
    cap = N * D * 10 + 32
    buf = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    row_bytes = engine.varint_encode_dev(x.data_ptr(), N, D, D, buf.data_ptr(), cap)
    off = np.concatenate([[0], np.cumsum(row_bytes)]).astype(np.uint64)
    exp = oracle.combine(M31, x.cpu().numpy())
    for path in ("fused", "matrix", "slots"):
        monkeypatch.setenv("SDA_CODEC_PATH", path)
        out = torch.full((D,), 7, dtype=torch.int64, device="cuda")
        assert engine.clerk_decode_combine_dev(M31, buf.data_ptr(), off, out.data_ptr(), D) == D
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy(), exp, path)


def test_fused_decode_combine_irregular_falls_back(engine, oracle, monkeypatch):
    """a blob with a run of 11+ continuation bytes (malformed) takes the sequential exact decoder even
    when the fused path is forced"""
    rng = np.random.default_rng(13)
    x = _rows(rng, "field", 4, 1500)
    blobs = [oracle.varint_encode(r) for r in x]
    blobs[2] = oracle.varint_encode(x[2][:-2]) + bytes([0xFF] * 12 + [0x01])   # 1498 + 2 elements
    rows = np.stack([oracle.varint_decode(b) for b in blobs])
    assert rows.shape == (4, 1500)
    for path in ("fused", "slots"):
        assert_same(_run(engine, M31, blobs, 1500, path, monkeypatch), oracle.combine(M31, rows), path)


@pytest.mark.parametrize("ones", [0, 1, 7, 3001, 8999])
def test_slot_decode_combine_region_edges(engine, oracle, monkeypatch, ones):
    """The slot path's tiles around 16 KiB region edges: the first payload mixes `ones` one-byte elements
    with five-byte field shares, which moves every later payload's region boundaries, so tiles of 512
    elements start near a region's end (or in a short first region) and continue in the next one."""
    rng = np.random.default_rng(ones + 3)
    D = 9_000
    x = _rows(rng, "field", 12, D)
    x[0, :ones] = 0
    x[6] = 0                                                # a payload of 1-byte elements only
    blobs = [oracle.varint_encode(r) for r in x]
    exp = oracle.combine(M31, x)
    for path in ("slots", "matrix"):
        assert_same(_run(engine, M31, blobs, D, path, monkeypatch), exp, path)
