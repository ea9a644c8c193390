"""Snapshot transposition: [participation][clerk] payloads -> clerking jobs.

Reference: server/src/stores.rs:86-101 (AggregationsStore::iter_snapshot_clerk_jobs_data: for every
participation in snapshot order, `shares[ix].push(share)` per clerk index) and the Mongo store's
$unwind/$group/$sort (server-store-mongodb/src/aggregations.rs:164-195), which yields the same
grouping.  Pure data movement, so the bar is byte-exact.  The reference has no test of its own for
this function; the CPU tests pin the C restatement against a literal Python restatement of the
stores.rs loop (parity of the loop itself unpinned by reference fixtures).
"""
import numpy as np
import pytest

from sda_amd import SdaError
from tests.util import assert_same


def _reference_loop(blobs, clerks_number):
    """stores.rs:89-99 verbatim in Python"""
    shares = [[] for _ in range(clerks_number)]
    for participation in blobs:
        for ix, share in enumerate(participation):
            shares[ix].append(share)
    return shares


def _ragged(rng, P, n, lo=0, hi=200):
    return [[rng.integers(0, 256, size=int(rng.integers(lo, hi)), dtype=np.uint8).tobytes() for _ in range(n)]
            for _ in range(P)]


@pytest.mark.parametrize("P,n,lo,hi", [(0, 3, 0, 10), (1, 1, 0, 5), (7, 3, 0, 40), (13, 26, 0, 300),
                                       (5, 8, 0, 1)])
def test_oracle_matches_reference_loop(oracle, P, n, lo, hi):
    blobs = _ragged(np.random.default_rng(P * 31 + n), P, n, lo, hi)
    assert oracle.snapshot_transpose(blobs) == (_reference_loop(blobs, n) if P else [])


def test_oracle_readme_shaped_snapshot(oracle):
    """three participations, three clerks (README.md walkthrough shape), distinguishable payloads"""
    blobs = [[bytes([p, c]) * (c + 1) for c in range(3)] for p in range(3)]
    got = oracle.snapshot_transpose(blobs)
    assert got[1] == [bytes([0, 1]) * 2, bytes([1, 1]) * 2, bytes([2, 1]) * 2]
    assert got == _reference_loop(blobs, 3)


# ---------------------------------------------------------------- GPU (through the C ABI)

def _run_device(engine, blobs, pad_front=0):
    import torch
    P = len(blobs)
    n = len(blobs[0]) if P else 0
    flat = bytes(pad_front) + b"".join(b for row in blobs for b in row)
    lens = [len(b) for row in blobs for b in row]
    off = (np.concatenate([[0], np.cumsum(lens)]) + pad_front).astype(np.uint64) if P * n else \
        np.array([pad_front], np.uint64)
    src = torch.frombuffer(bytearray(flat + bytes(32)), dtype=torch.uint8).cuda()
    need, _, _ = engine.snapshot_transpose_dev(src.data_ptr(), off, P, n)      # sizing query
    dst = torch.full((max(need, 16),), 0xA5, dtype=torch.uint8, device="cuda")
    dlen, base, coff = engine.snapshot_transpose_dev(src.data_ptr(), off, P, n, dst.data_ptr(), dst.numel())
    torch.cuda.synchronize()
    assert dlen == need
    host = dst.cpu().numpy().tobytes()
    return [[host[int(base[c] + coff[c, p]):int(base[c] + coff[c, p + 1])] for p in range(P)] for c in range(n)], \
        base, coff


@pytest.mark.gpu
@pytest.mark.parametrize("P,n,lo,hi", [(1, 1, 1, 2), (7, 3, 0, 40), (13, 26, 0, 300), (5, 8, 0, 1),
                                       (3, 4, 16_000, 40_000), (200, 26, 0, 64)])
@pytest.mark.parametrize("pad_front", [0, 5])
def test_gpu_transpose_matches_oracle(engine, oracle, P, n, lo, hi, pad_front):
    """every source/destination misalignment, blobs shorter than a quad, blobs across 16 KiB chunks"""
    blobs = _ragged(np.random.default_rng(P * 7 + n + pad_front), P, n, lo, hi)
    got, base, coff = _run_device(engine, blobs, pad_front)
    assert got == oracle.snapshot_transpose(blobs)
    assert all(int(b) % 16 == 0 for b in base)


@pytest.mark.gpu
def test_gpu_transpose_empty_snapshot(engine):
    got, _, _ = _run_device(engine, [])
    assert got == []


@pytest.mark.gpu
def test_gpu_transpose_rejects_bad_args(engine):
    import torch
    src = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(SdaError):        # decreasing offsets
        engine.snapshot_transpose_dev(src.data_ptr(), [0, 8, 4], 1, 2)
    dst = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(SdaError):        # dst too small
        engine.snapshot_transpose_dev(src.data_ptr(), [0, 8, 16], 1, 2, dst.data_ptr(), 8)
    with pytest.raises(SdaError):        # misaligned src
        engine.snapshot_transpose_dev(src.data_ptr() + 1, [0, 8, 16], 1, 2, dst.data_ptr(), 64)


@pytest.mark.gpu
def test_gpu_server_colocated_clerk_path(engine, oracle):
    """participants' varint payloads (device) -> snapshot transposition (device) -> every clerk's
    decode + combine (device) == the oracle's combine of each clerk's decoded shares"""
    import torch
    P, n, D, m = 40, 5, 3000, 2147482801
    rng = np.random.default_rng(0x5DA + 4)
    shares = rng.integers(-(m - 1), m, size=(P, n, D), dtype=np.int64)
    blobs = [[oracle.varint_encode(shares[p, c]) for c in range(n)] for p in range(P)]
    flat = b"".join(b for row in blobs for b in row)
    off = np.concatenate([[0], np.cumsum([len(b) for row in blobs for b in row])]).astype(np.uint64)
    src = torch.frombuffer(bytearray(flat + bytes(32)), dtype=torch.uint8).cuda()
    need, _, _ = engine.snapshot_transpose_dev(src.data_ptr(), off, P, n)
    dst = torch.empty(need, dtype=torch.uint8, device="cuda")
    _, base, coff = engine.snapshot_transpose_dev(src.data_ptr(), off, P, n, dst.data_ptr(), need)
    out = torch.empty((n, D), dtype=torch.int64, device="cuda")
    for c in range(n):
        got = engine.clerk_decode_combine_dev(m, dst.data_ptr() + int(base[c]), coff[c], out[c].data_ptr(), D)
        assert got == D
    torch.cuda.synchronize()
    exp = np.stack([oracle.combine(m, shares[:, c, :]) for c in range(n)])
    assert_same(out.cpu().numpy(), exp, "clerk results")


@pytest.mark.gpu
def test_gpu_transpose_large_is_permutation(engine):
    """a clerking-job-sized snapshot (1,000 participations x 26 clerks of ~40 KB): every clerk job
    is the byte concatenation of its column, checked by per-blob checksums"""
    import torch
    P, n = 1000, 26
    rng = np.random.default_rng(9)
    lens = rng.integers(38_000, 42_000, size=P * n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    total = int(off[-1])
    g = torch.Generator(device="cuda").manual_seed(3)
    src = torch.randint(0, 256, (total + 32,), dtype=torch.uint8, device="cuda", generator=g)
    need, _, _ = engine.snapshot_transpose_dev(src.data_ptr(), off, P, n)
    dst = torch.empty(need, dtype=torch.uint8, device="cuda")
    _, base, coff = engine.snapshot_transpose_dev(src.data_ptr(), off, P, n, dst.data_ptr(), need)
    torch.cuda.synchronize()
    s64, d64 = src.to(torch.int64), dst.to(torch.int64)
    cs = torch.cumsum(s64, 0)
    cd = torch.cumsum(d64, 0)

    def seg(c, lo, hi):
        return (int(c[hi - 1]) - (int(c[lo - 1]) if lo else 0)) if hi > lo else 0
    for c in range(0, n, 5):
        for p in range(0, P, 97):
            b = p * n + c
            exp = seg(cs, int(off[b]), int(off[b + 1]))
            lo = int(base[c] + coff[c, p])
            hi = int(base[c] + coff[c, p + 1])
            assert hi - lo == int(lens[b])
            assert seg(cd, lo, hi) == exp
    # and one full clerk job byte for byte
    c = 7
    exp = torch.cat([src[int(off[p * n + c]):int(off[p * n + c + 1])] for p in range(P)])
    assert torch.equal(dst[int(base[c]):int(base[c] + coff[c, P])], exp)
    assert_same([int(coff[c, P])], [int(exp.numel())])
