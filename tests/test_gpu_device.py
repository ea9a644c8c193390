"""GPU: device-resident entry points (the ones bench.py times) at larger sizes.

Full-size results are checked through properties that do not need the oracle to finish the
whole job: column independence (the oracle recomputes a random sample of columns / batches
exactly), encode -> decode round trips, and torch int64 column sums for non-negative inputs.
"""
import numpy as np
import pytest

from sda_amd import schemes as S
from sda_amd import engine as E
from sda_amd import synth
from tests.util import assert_same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def test_synth_fill_matches_numpy(engine):
    rows, cols, seed, lo, hi = 37, 1001, 0x5DA + 2, -2147482800, 2147482801
    t = torch.empty((rows, cols), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(t.data_ptr(), rows, cols, seed, lo, hi, _stream())
    torch.cuda.synchronize()
    assert (t.cpu().numpy() == synth.fill(rows, cols, seed, lo, hi)).all()


@pytest.mark.parametrize("dim,stride", [(1_000_000, 1_000_000), (1_000_003, 1_000_003), (500_000, 500_016)])
def test_combine_dev_large(engine, oracle, dim, stride):
    m, N = 2147482801, 1024
    x = torch.empty((N, stride), dtype=torch.int64, device="cuda")
    # signed inputs in (-m, m): the order-dependent case
    engine.synth_fill_dev(x.data_ptr(), N, stride, 0x5DA + 9, -(m - 1), m, _stream())
    out = torch.empty(dim, dtype=torch.int64, device="cuda")
    engine.combine_dev(m, x.data_ptr(), N, dim, stride, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    cols = np.random.default_rng(dim).choice(dim, 512, replace=False)
    xs = x[:, torch.from_numpy(cols).cuda()].cpu().numpy()
    assert_same(got[cols], oracle.combine(m, xs))
    # property: residue equals the column sum mod m
    col_sum = x[:, :dim].sum(dim=0)           # |sum| < N * m < 2^63
    assert (torch.remainder(col_sum, m).cpu().numpy() == np.mod(got, m)).all()


def test_combine_dev_config1_full_size(engine, oracle):
    """configs[1] at its own size on one GPU: 10,000 participations x 1M-dim (80 GB resident), signed
    (-m, m) shares -- the order-dependent case.  1,024 sampled columns equal the oracle's sequential
    recurrence bit for bit; every column's residue equals its int64 column sum mod m."""
    m, N, D = 2147482801, 10_000, 1_000_000
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 0x5DA + 31, -(m - 1), m, _stream())
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.combine_dev(m, x.data_ptr(), N, D, D, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    cols = np.sort(np.random.default_rng(31).choice(D, 1024, replace=False))
    xs = x[:, torch.from_numpy(cols).cuda()].cpu().numpy()
    got = out.cpu().numpy()
    assert_same(got[cols], oracle.combine(m, xs))
    col_sum = x.sum(dim=0)                    # |sum| < N * m < 2^63
    del x
    assert torch.equal(torch.remainder(col_sum, m), torch.remainder(out, m))


def test_combine_dev_canonical_and_finalize(engine):
    m, N, D = 2147482801, 512, 1_000_000
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 0x5DA + 1, 0, m, _stream())
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.combine_dev(m, x.data_ptr(), N, D, D, out.data_ptr(), _stream())
    exp = torch.remainder(x.sum(dim=0), m)
    torch.cuda.synchronize()
    assert torch.equal(out, exp)
    # two "ranks": halves combined separately, summed as int64, finalized on device
    a = torch.empty(D, dtype=torch.int64, device="cuda")
    b = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.combine_dev(m, x.data_ptr(), N // 2, D, D, a.data_ptr(), _stream())
    engine.combine_dev(m, x[N // 2:].data_ptr(), N - N // 2, D, D, b.data_ptr(), _stream())
    s = a + b
    fin = torch.empty(D, dtype=torch.int64, device="cuda")
    engine.combine_finalize_dev(m, s.data_ptr(), D, fin.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert torch.equal(fin, exp)


@pytest.mark.parametrize("mode", [E.REVEAL_EXACT, E.REVEAL_CANONICAL])
def test_packed_dev_roundtrip_config(engine, oracle, mode):
    """configs[2]: k=8, n=26, t=7 at 1M-dim, several participant vectors per launch."""
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    V, D = 3, 1_000_000
    B = D // k
    sec = torch.empty((V, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(sec.data_ptr(), V, D, 0x5DA + 2, 0, p, _stream())
    draws = torch.empty((V, B, t), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(draws.data_ptr(), V * B, t, 0x5DA + 22, 0, p - 1, _stream())
    shares = torch.empty((V, n, B), dtype=torch.int64, device="cuda")
    engine.packed_generate_dev(sch, sec.data_ptr(), D, V, draws.data_ptr(), shares.data_ptr(), _stream())
    torch.cuda.synchronize()
    # batches are independent: check a sample against the oracle (tss op order, signed)
    pp = oracle.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    sec_h, dr_h, sh_h = sec.cpu().numpy(), draws.cpu().numpy(), shares.cpu().numpy()
    for v, b in zip(np.random.default_rng(1).integers(0, V, 64), np.random.default_rng(2).integers(0, B, 64)):
        exp = oracle.packed_share(pp, sec_h[v, b * k:(b + 1) * k], dr_h[v, b])
        assert_same(sh_h[v, :, b], exp)
    # reveal from a t+k subset (reversed) and from all clerks: round trip to the secrets
    for idx in (list(range(n - 1, n - 1 - (t + k), -1)), list(range(n))):
        sub = shares[:, idx, :].contiguous()
        out = torch.empty((V, D), dtype=torch.int64, device="cuda")
        engine.packed_reconstruct_dev(sch, D, idx, V, sub.data_ptr(), out.data_ptr(), mode, _stream())
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert (np.mod(got, p) == sec_h).all()
        if mode == E.REVEAL_CANONICAL:
            assert got.min() >= 0
        else:
            # exact representatives on a batch sample
            for v, b in zip(range(V), (5, B // 2, B - 1)):
                rc, exp = oracle.packed_reconstruct(pp, k, idx, sh_h[v][idx][:, b:b + 1])
                assert_same(got[v, b * k:(b + 1) * k], exp)


def test_chacha_combine_dev(engine, oracle):
    m, D, N = 2147482801, 100_003, 48
    seeds = np.random.default_rng(3).integers(0, 2**32, size=(N, 4), dtype=np.uint64).astype(np.uint32)
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    sd = _dev(seeds.view(np.int32)).view(torch.int32)
    engine.chacha_mask_combine_dev(m, D, sd.data_ptr(), 4, N, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), oracle.chacha_mask_combine(m, D, seeds.astype(np.int64)))


def test_additive_generate_dev(engine, oracle):
    m, n, D = 433, 3, 200_001
    rng = np.random.default_rng(4)
    sec = rng.integers(-(2**40), 2**40, size=D, dtype=np.int64)
    draws = rng.integers(0, m, size=D * (n - 1), dtype=np.int64)
    out = torch.empty((n, D), dtype=torch.int64, device="cuda")
    dsec, ddr = _dev(sec), _dev(draws)          # keep the device buffers alive across the launch
    engine.additive_generate_dev(m, n, dsec.data_ptr(), D, ddr.data_ptr(), out.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == oracle.additive_generate(m, n, sec, draws)).all()


def test_packed_generate_fixup_overflow(engine, oracle):
    """More out-of-range batches than the fix-up log holds: every batch is recomputed exactly."""
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    B = 70_001                                  # > kGenLogCap (65536) logged batches, odd => narrow stores
    D = B * k - 3
    rng = np.random.default_rng(0x5DA)
    sec = rng.integers(-(2**40), 2**40, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=(B, t), dtype=np.int64)
    shares = engine.share_generate(sch, sec, draws.reshape(-1))
    pp = oracle.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    padded = np.concatenate([sec, np.zeros(B * k - D, dtype=np.int64)])
    for b in list(np.random.default_rng(3).integers(0, B, 48)) + [0, B - 1]:
        exp = oracle.packed_share(pp, padded[b * k:(b + 1) * k], draws[b])
        assert_same(shares[:, b], exp)


@pytest.mark.parametrize("D", [3001, 3000], ids=["odd_dim", "even_dim_pipelined"])
def test_combine_accumulate_tiles(engine, oracle, D):
    """sda_combine_accumulate_dev: a job streamed in row tiles == one pass (signed, order-dependent); an even
    dimension runs the software-pipelined kernel (2 columns per lane), an odd one the 1-column kernel."""
    m = 2147482801
    N = 37
    x = np.random.default_rng(9).integers(-(m - 1), m, size=(N, D), dtype=np.int64)
    xd = torch.as_tensor(x).cuda()
    acc = torch.zeros(D, dtype=torch.int64, device="cuda")
    for t0 in range(0, N, 10):
        n = min(10, N - t0)
        engine.combine_accumulate_dev(m, xd[t0].data_ptr(), n, D, D, acc.data_ptr())
    torch.cuda.synchronize()
    assert_same(acc.cpu().numpy(), oracle.combine(m, x))


def test_distributed_helpers_single_rank(engine, oracle):
    """sda_amd.distributed's device paths at world size 1 (the multi-rank reduce is covered with
    gloo in test_host.py): seed-split ChaCha mask combine and the column-split signed combine."""
    from sda_amd import distributed as Dd
    m, D = 2147482801, 5001
    seeds = torch.randint(0, 2**31 - 1, (7, 4), dtype=torch.int32, device="cuda",
                          generator=torch.Generator(device="cuda").manual_seed(3))
    part = torch.empty(D, dtype=torch.int64, device="cuda")
    out = torch.empty(D, dtype=torch.int64, device="cuda")
    Dd.mask_combine_sharded(engine, m, D, seeds, part, out)
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), oracle.chacha_mask_combine(m, D, seeds.cpu().numpy().astype(np.int64)))
    x = np.random.default_rng(12).integers(-(m - 1), m, size=(19, D), dtype=np.int64)
    xd = torch.as_tensor(x).cuda()
    Dd.combine_columns_sharded(engine, m, xd, out)
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), oracle.combine(m, x))


def test_packed_reveal_fixup_overflow(engine, oracle):
    """More out-of-range (raw i64) share batches than the reveal's fix-up log holds: every batch is
    recomputed exactly by the fix-up kernel (one wave per batch)."""
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    B = 70_001                                  # > kGenLogCap (65536) logged batches
    D = B * k
    rng = np.random.default_rng(0x5DB)
    idx = list(range(3, 3 + t + k))
    raw = rng.integers(-(2**40), 2**40, size=(len(idx), B), dtype=np.int64)
    got = engine.secret_reconstruct(sch, D, [(c, raw[j]) for j, c in enumerate(idx)])
    pp = oracle.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    sample = sorted(set(int(b) for b in np.random.default_rng(4).integers(0, B, 40)) | {0, B - 1})
    rc, exp = oracle.packed_reconstruct(pp, k * len(sample), idx, raw[:, sample])
    assert rc == 0
    for j, b in enumerate(sample):
        assert_same(got[b * k:(b + 1) * k], exp[j * k:(j + 1) * k])


def _split_on_one_gpu(engine, m, x, G, tile=None):
    """The participation split of sda_amd.distributed run for G simulated ranks on one GPU, every step
    through the C ABI: pass 1 + flags per rank, the all-gather / SUM / MAX exchanges done with torch
    on the device, prefix + replay + resolve per rank.  Returns (flags, result seen by every rank)."""
    from sda_amd import distributed as Dd
    N, D = x.shape
    spans = [Dd.shard_range(N, g, G) for g in range(G)]
    tile = tile or N

    def tiles(g):
        s0, cnt = spans[g]
        return [(x[s0 + t0].data_ptr(), min(tile, cnt - t0)) for t0 in range(0, cnt, tile)]

    parts = torch.zeros((G, D), dtype=torch.int64, device="cuda")
    flags = torch.zeros((G, 2), dtype=torch.int64, device="cuda")
    for g in range(G):
        for ptr, n in tiles(g):
            engine.combine_split_dev(m, ptr, n, D, x.stride(0), parts[g].data_ptr(), flags[g].data_ptr(), _stream())
    fl = flags.sum(dim=0).tolist()
    states = torch.empty((G, D), dtype=torch.int64, device="cuda")
    totals = torch.empty((G, D), dtype=torch.int64, device="cuda")
    codes = torch.empty((G, D), dtype=torch.int32, device="cuda")
    for g in range(G):
        engine.combine_split_prefix_dev(m, parts.data_ptr(), G, g, D, states[g].data_ptr(), totals[g].data_ptr(),
                                        codes[g].data_ptr(), _stream())
        if g:
            for ptr, n in tiles(g):
                engine.combine_split_replay_dev(m, ptr, n, D, x.stride(0), g, states[g].data_ptr(),
                                                codes[g].data_ptr(), _stream())
    code = codes.max(dim=0).values.contiguous()
    outs = torch.empty((G, D), dtype=torch.int64, device="cuda")
    for g in range(G):
        engine.combine_split_resolve_dev(m, totals[g].data_ptr(), code.data_ptr(), D, outs[g].data_ptr(), _stream())
    torch.cuda.synchronize()
    assert (outs == outs[0]).all()            # every rank resolves the same result
    return fl, outs[0].cpu().numpy()


@pytest.mark.parametrize("m,N,D,lo,hi,G,tile", [
    (2147482801, 2000, 100_003, -(2147482801 - 1), 2147482801, 8, None),   # signed field shares, 8 ranks
    (2147482801, 999, 50_000, -(2147482801 - 1), 2147482801, 3, 100),      # row tiles, ragged ranks
    (7, 1200, 20_002, -6, 7, 8, None),                                     # sign events almost every step
    ((1 << 62) - 57, 400, 10_001, -((1 << 62) - 58), (1 << 62) - 57, 2, 64),  # largest fast-path moduli
    (1000003, 300, 9_999, -(1 << 61), 1 << 61, 5, None),                   # raw i64: the generic path
    (433, 1, 1_001, -432, 433, 1, None),                                   # one rank, one row
    (433, 3, 4_096, -432, 433, 8, None),                                   # ranks with no rows
])
def test_participation_split_signed_exact(engine, oracle, m, N, D, lo, hi, G, tile):
    """The exact signed participation split (SURVEY §7 hard part 1 (b)): pass-1 flags,
    prefix, replay of the sign events and their MAX resolution give the reference's single sequential
    pass (combiner.rs:16-28) bit for bit on signed inputs, whose result depends on the order."""
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 0x5DA + 31, lo, hi, _stream())
    fl, got = _split_on_one_gpu(engine, m, x, G, tile)
    xh = x.cpu().numpy()
    exp = oracle.combine(m, xh)
    assert fl[0] > 0 and fl[1] == 0
    assert (exp < 0).any() and (exp > 0).any()
    assert_same(got, exp)


def test_participation_split_flags(engine):
    """Pass-1 flags: none for non-negative inputs (the one-reduce path), [neg] for a single negative
    value, [wrap] for a value past 2^63 - m (the split refuses it), in any column and row."""
    m, N, D = 2147482801, 70, 3_001
    x = torch.empty((N, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, D, 0x5DA + 32, 0, m, _stream())

    def flags():
        f = torch.zeros(2, dtype=torch.int64, device="cuda")
        acc = torch.zeros(D, dtype=torch.int64, device="cuda")
        engine.combine_split_dev(m, x.data_ptr(), N, D, D, acc.data_ptr(), f.data_ptr(), _stream())
        torch.cuda.synchronize()
        return f.tolist(), acc
    f, acc = flags()
    assert f == [0, 0]
    assert torch.equal(acc, torch.remainder(x.sum(dim=0), m))
    x[69, 3000] = -1
    assert flags()[0] == [1, 0]
    x[69, 3000] = 5
    x[13, 1] = (1 << 63) - m + 1            # just past the no-wrap range
    assert flags()[0] == [0, 1]
    x[13, 1] = (1 << 63) - m                # the range's edge: fine
    assert flags()[0] == [0, 0]
    x[0, 0] = -(1 << 63)
    assert flags()[0] == [1, 1]


def test_finalize_signed_sums(engine):
    """sda_combine_finalize_dev takes signed int64 sums (the all-reduced per-rank results) to their
    canonical residue -- negative sums included (it once read them as u64)."""
    m = 2147482801
    s = torch.tensor([-1, -m, -(m + 1), -(8 * (m - 1)), 8 * (m - 1), 0, m - 1, -(1 << 62)], dtype=torch.int64,
                     device="cuda")
    out = torch.empty_like(s)
    engine.combine_finalize_dev(m, s.data_ptr(), s.numel(), out.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert out.tolist() == [int(v) % m for v in s.tolist()]


@pytest.mark.parametrize("pipe", ["1", "0"], ids=["pipelined", "unpipelined"])
def test_combine_pipelined_row_counts(engine, oracle, monkeypatch, pipe):
    """combine.hip's software-pipelined i64 kernel (two buffers of 4 rows, the last whole batch peeled off) at
    every row count from 1 to 21 -- no whole batch, an odd and an even number of them, each with 0-3 tail rows --
    plain and accumulating, signed inputs (the order-dependent case), against the reference recurrence."""
    monkeypatch.setenv("SDA_COMBINE_PIPE", pipe)
    m, D = 2147482801, 2 * 1543
    rng = np.random.default_rng(1543)
    x = rng.integers(-(m - 1), m, size=(21, D), dtype=np.int64)
    xd = torch.as_tensor(x).cuda()
    for N in range(1, 22):
        out = torch.empty(D, dtype=torch.int64, device="cuda")
        engine.combine_dev(m, xd.data_ptr(), N, D, D, out.data_ptr(), _stream())
        torch.cuda.synchronize()
        assert_same(out.cpu().numpy(), oracle.combine(m, x[:N]), f"N={N}")
    for N in range(1, 21):
        acc = torch.as_tensor(x[0]).cuda()                   # the state after row 0; then rows 1..N
        engine.combine_accumulate_dev(m, xd[1].data_ptr(), N, D, D, acc.data_ptr(), _stream())
        torch.cuda.synchronize()
        assert_same(acc.cpu().numpy(), oracle.combine(m, x[:N + 1]), f"accumulate N={N}")


@pytest.mark.parametrize("balance", ["1", "0"], ids=["balanced", "plain_grid"])
@pytest.mark.parametrize("dim", [262_146, 1_048_560, 1_048_578], ids=["one_wide_wg", "widths_248_256", "two_rounds"])
def test_combine_balanced_grid_widths(engine, oracle, monkeypatch, balance, dim):
    """combine.hip's balanced grid (workgroups of wlo or wlo + 8 lanes, starting at g wlo + 8 min(g, nwide)) at its
    edge cases -- a single wide workgroup, widths capped at 248 / 256 lanes, a second round of workgroups -- plain
    and accumulating, signed inputs, against the reference recurrence on every column."""
    monkeypatch.setenv("SDA_COMBINE_BALANCE", balance)
    m, N = 2147482801, 9
    x = torch.empty((N, dim), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), N, dim, 0x5DA + dim, -(m - 1), m, _stream())
    out = torch.empty(dim, dtype=torch.int64, device="cuda")
    engine.combine_dev(m, x.data_ptr(), N, dim, dim, out.data_ptr(), _stream())
    acc = x[0].clone()
    engine.combine_accumulate_dev(m, x[1].data_ptr(), N - 1, dim, dim, acc.data_ptr(), _stream())
    torch.cuda.synchronize()
    exp = oracle.combine(m, x.cpu().numpy())
    assert_same(out.cpu().numpy(), exp)
    assert_same(acc.cpu().numpy(), exp)
