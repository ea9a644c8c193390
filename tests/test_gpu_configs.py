"""GPU: BASELINE.json configs at full dimension, checked against the oracle on samples and through
size-independent properties.

  configs[3]  federated aggregation, 10M-dim: the clerk job streamed through HBM in row tiles with
              sda_combine_accumulate_dev (client/src/crypto/sharing/combiner.rs:16-28 called at
              client/src/clerk.rs:79-86), signed inputs; and the participation split + finalize the
              multi-GPU path uses, on one GPU.
  configs[2]  packed Shamir k=8 n=26 t=7 at 1M-dim: the CANONICAL share / reveal modes end in the same
              recipient output as the EXACT (tss-order) ones -- the full_loop.rs:148-style sum.
"""
import numpy as np
import pytest

from sda_amd import distributed as Dd
from sda_amd import engine as E
from sda_amd import schemes as S
from tests.util import assert_same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
M = 2147482801
D10M = 10_000_000


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_config3_tiled_accumulate_signed_10M(engine, oracle):
    """configs[3] per-GPU job shape: 10M-dim, participations streamed as row tiles through the
    accumulating combine; signed shares (the order-dependent case).  Exact on sampled columns (the
    oracle replays all rows), residue property on every column."""
    R, T = 24, 3
    tile = torch.empty((R, D10M), dtype=torch.int64, device="cuda")
    acc = torch.zeros(D10M, dtype=torch.int64, device="cuda")
    colsum = torch.zeros(D10M, dtype=torch.int64, device="cuda")
    cols = np.sort(np.random.default_rng(31).choice(D10M, 2048, replace=False))
    cols_d = torch.from_numpy(cols).cuda()
    sample = []
    for t in range(T):
        engine.synth_fill_dev(tile.data_ptr(), R, D10M, 0x5DA + 3 + t, -(M - 1), M, _stream())
        engine.combine_accumulate_dev(M, tile.data_ptr(), R, D10M, D10M, acc.data_ptr(), _stream())
        colsum += tile.sum(dim=0)                      # |sum| < 72 m < 2^63
        sample.append(tile[:, cols_d].cpu().numpy())
    torch.cuda.synchronize()
    got = acc.cpu().numpy()
    assert_same(got[cols], oracle.combine(M, np.vstack(sample)))
    assert torch.equal(torch.remainder(acc, M), torch.remainder(colsum, M))
    assert int(acc.abs().max()) < M


def test_config3_participation_split_finalize_10M(engine):
    """The multi-GPU reduction on one GPU: two participation halves combined separately (tiles through
    sda_amd.distributed.combine_tiles_sharded), summed as int64 (what the RCCL all-reduce does),
    finalized on device -- equal to one pass over all rows for non-negative inputs (configs[3])."""
    R = 32
    x = torch.empty((R, D10M), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(x.data_ptr(), R, D10M, 0x5DA + 4, 0, M, _stream())
    one = torch.empty(D10M, dtype=torch.int64, device="cuda")
    engine.combine_dev(M, x.data_ptr(), R, D10M, D10M, one.data_ptr(), _stream())
    halves = []
    for lo, hi in ((0, 13), (13, R)):
        part = torch.empty(D10M, dtype=torch.int64, device="cuda")
        out = torch.empty(D10M, dtype=torch.int64, device="cuda")
        tiles = [(x[r].data_ptr(), min(5, hi - r)) for r in range(lo, hi, 5)]
        Dd.combine_tiles_sharded(engine, M, tiles, D10M, D10M, part, out)
        halves.append(out)
    s = halves[0] + halves[1]
    fin = torch.empty(D10M, dtype=torch.int64, device="cuda")
    engine.combine_finalize_dev(M, s.data_ptr(), D10M, fin.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert torch.equal(fin, one)
    assert torch.equal(one, torch.remainder(x.sum(dim=0), M))


def test_config2_canonical_equals_exact_end_to_end(engine, oracle):
    """configs[2] (k=8, n=26, t=7, 1M-dim): V participants share their vectors in EXACT and in
    CANONICAL mode, every clerk combines its column, the recipient reveals from a t+k clerk subset;
    both modes give positive() == the sum of the secrets mod p -- the full_loop.rs:148 invariant --
    and the canonical shares are the exact ones mod p."""
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    V, D = 4, 1_000_000
    B = D // k
    sec = torch.empty((V, D), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(sec.data_ptr(), V, D, 0x5DA + 2, 0, p, _stream())
    drw = torch.empty((V, B, t), dtype=torch.int64, device="cuda")
    engine.synth_fill_dev(drw.data_ptr(), V * B, t, 0x5DA + 22, 0, p - 1, _stream())
    expect = torch.remainder(sec.sum(dim=0), p)
    idx = [25, 3, 17, 0, 9, 11, 24, 6, 1, 20, 14, 22, 5, 8, 19]          # t + k = 15 clerks, any order
    outs = {}
    shares = {}
    for mode in (E.REVEAL_EXACT, E.REVEAL_CANONICAL):
        sh = torch.empty((V, n, B), dtype=torch.int64, device="cuda")
        engine.packed_generate_mode_dev(sch, sec.data_ptr(), D, V, drw.data_ptr(), sh.data_ptr(), mode, _stream())
        shares[mode] = sh
        clerk = torch.empty((len(idx), B), dtype=torch.int64, device="cuda")
        for j, c in enumerate(idx):                     # clerk c combines the V participations
            col = sh[:, c, :].contiguous()
            engine.combine_dev(p, col.data_ptr(), V, B, B, clerk[j].data_ptr(), _stream())
        out = torch.empty(D, dtype=torch.int64, device="cuda")
        engine.packed_reconstruct_dev(sch, D, idx, 1, clerk.data_ptr(), out.data_ptr(), mode, _stream())
        torch.cuda.synchronize()
        outs[mode] = out
    assert torch.equal(torch.remainder(shares[E.REVEAL_EXACT], p), shares[E.REVEAL_CANONICAL])
    pos = {m: torch.where(o < 0, o + p, o) for m, o in outs.items()}   # RecipientOutput::positive
    assert torch.equal(pos[E.REVEAL_EXACT], expect) and torch.equal(pos[E.REVEAL_CANONICAL], expect)
    # exact mode also reproduces tss' signed representatives (sampled batches vs the oracle)
    pp = oracle.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    sh_h = shares[E.REVEAL_EXACT].cpu().numpy()
    for b in (0, 7, B // 2, B - 1):
        clerk_b = np.array([[oracle.combine(p, sh_h[:, c, b:b + 1])[0]] for c in idx], np.int64)
        rc, exp = oracle.packed_reconstruct(pp, k, idx, clerk_b)
        assert rc == 0
        assert_same(outs[E.REVEAL_EXACT][b * k:(b + 1) * k].cpu().numpy(), exp)


@pytest.mark.parametrize("mode", [E.REVEAL_EXACT, E.REVEAL_CANONICAL])
def test_packed_reveal_all_80_clerks(engine, oracle, mode):
    """n = 80 (n + 1 = 81): the reference reconstructs from every share it is given (batched.rs:75),
    up to all 80 clerks -- 81 Newton points."""
    from tests.test_gpu_parity import packed_schemes
    sch = next(s for s in packed_schemes() if s.share_count == 80 and s.secret_count == 8)
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    D = 8 * 40_001
    B = D // k
    rng = np.random.default_rng(80)
    secrets = rng.integers(0, p, size=D, dtype=np.int64)
    draws = rng.integers(0, p - 1, size=B * t, dtype=np.int64)
    shares = engine.share_generate(sch, secrets, draws)
    pp = oracle.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    for idx in (list(range(n)), rng.permutation(n)[:77].tolist()):
        sub = torch.from_numpy(np.ascontiguousarray(shares[idx])).cuda()
        out = torch.empty(D, dtype=torch.int64, device="cuda")
        engine.packed_reconstruct_dev(sch, D, idx, 1, sub.data_ptr(), out.data_ptr(), mode, _stream())
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert (np.mod(got, p) == secrets).all()
        if mode == E.REVEAL_EXACT:
            for b in (0, 1, B // 3, B - 1):
                rc, exp = oracle.packed_reconstruct(pp, k, idx, shares[idx][:, b:b + 1])
                assert rc == 0
                assert_same(got[b * k:(b + 1) * k], exp)
