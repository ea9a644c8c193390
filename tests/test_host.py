"""CPU: host-side logic -- synthetic inputs, sharding, reduce headroom, world-size-2 gloo reduce."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sda_amd import distributed as Dd
from sda_amd import synth


def test_splitmix_reference_values():
    # splitmix64 with state 0: first outputs of the published generator
    z = synth.splitmix64_at(0, np.arange(3, dtype=np.uint64))
    assert [int(x) for x in z] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_fill_ranges_and_slices():
    a = synth.fill(5, 7, 0x5DA, -10, 10)
    assert a.dtype == np.int64 and a.min() >= -10 and a.max() < 10
    assert (synth.fill(2, 7, 0x5DA, -10, 10, row0=3) == a[3:5]).all()


@pytest.mark.parametrize("n,world", [(10, 3), (100000, 8), (7, 8), (0, 2)])
def test_shard_range_partitions(n, world):
    spans = [Dd.shard_range(n, r, world) for r in range(world)]
    assert sum(c for _, c in spans) == n
    pos = 0
    for s, c in spans:
        assert s == pos
        pos += c


def test_reduce_headroom():
    assert Dd.reduce_headroom_ok(8, 2147482801)
    assert not Dd.reduce_headroom_ok(8, 2**62)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world2(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    return res


def _split_cases():
    """(name, modulus, N, D, lo, hi): non-negative (configs[3]), signed field shares (real Additive
    clerk jobs, additive.rs:46), a tiny modulus (sign events in almost every step), a 2^40-class
    modulus, and raw i64 values far outside (-m, m) (the generic path; within the no-wrap range)."""
    return [("nonneg", 2147482801, 37, 129, 0, 2147482801),
            ("signed", 2147482801, 37, 129, -(2147482801 - 1), 2147482801),
            ("small_m", 7, 41, 66, -6, 7),
            ("m2_40", (1 << 40) + 15, 29, 50, -(1 << 40), (1 << 40) + 15),
            ("raw_i64", 1000003, 23, 31, -(1 << 61), 1 << 61)]


def _worker_rows(rank, world, port, q):
    """sda_amd.distributed.combine_rows_sharded / combine_tiles_sharded themselves (participation
    split: pass 1 + flags, one int64 all-reduce, finalize -- or, for signed inputs, the two-pass
    replay + MAX-resolved sign events) with the oracle as the per-rank compute (tests/cpu_engine)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Dd.EXCHANGE_AT_WORLD_1 = world == 1          # world 1: the exchange path over a one-rank group
    from oracle import oracle as O
    from tests.cpu_engine import CpuEngine
    res = {}
    for name, m, N, D, lo, hi in _split_cases():
        eng = CpuEngine()
        full = torch.from_numpy(synth.fill(N, D, 0x5DA + 4, lo, hi))
        start, count = Dd.shard_range(N, rank, world)
        mine = full[start:start + count].contiguous()
        part, out = torch.empty(D, dtype=torch.int64), torch.empty(D, dtype=torch.int64)
        exp = O.combine(m, full.numpy()).tolist()
        st = Dd.SplitStats()
        Dd.combine_rows_sharded(eng, m, mine.data_ptr(), count, D, D, part, out, stats=st)
        res[name + "/rows"] = (out.tolist(), exp, st.signed)
        # the same rows streamed as 5-row tiles (configs[3]'s tiled accumulate on each rank)
        tiles = [(mine[t0].data_ptr(), min(5, count - t0)) for t0 in range(0, count, 5)]
        Dd.combine_tiles_sharded(eng, m, tiles, D, D, part, out, stats=st)
        res[name + "/tiles"] = (out.tolist(), exp, st.signed)
        calls = [None] * world
        dist.all_gather_object(calls, sorted(set(eng.calls)))
        res[name + "/calls"] = sorted(set(c for cs in calls for c in cs))
    # deferred tickets (defer=True): a non-negative job, whose result is final once finish() has read the
    # flags, then two signed jobs through ONE partial buffer before either is finished -- the first signed
    # ticket's pass-1 result was overwritten, so its finish() recomputes pass 1
    m, D = 2147482801, 77
    jobs = [synth.fill(19, D, 0x5DA + 40 + j, lo, m) for j, lo in enumerate((0, -(m - 1), -(m - 1)))]
    part = torch.empty(D, dtype=torch.int64)
    outs, tickets, stats = [], [], []
    for x in jobs:
        start, count = Dd.shard_range(x.shape[0], rank, world)
        mine = torch.from_numpy(x[start:start + count].copy())
        outs.append(torch.empty(D, dtype=torch.int64))
        stats.append(Dd.SplitStats())
        tickets.append((Dd.combine_rows_sharded(CpuEngine(), m, mine.data_ptr(), count, D, D, part, outs[-1],
                                                stats=stats[-1], defer=True), mine))
    for t, _ in tickets:
        t.finish()
        t.finish()                                   # idempotent
    res["deferred"] = [(o.tolist(), O.combine(m, x).tolist(), s.signed, s.redo_pass1, s.passes)
                       for o, x, s in zip(outs, jobs, stats)]
    # a signed deferred job whose `out` a later split reuses before finish(): refused with ValueError on
    # every rank (never the earlier job's exact result written over the later job's); the later job is intact
    x_s, x_n = jobs[1], jobs[0]
    start, count = Dd.shard_range(x_s.shape[0], rank, world)
    ms_, mn_ = (torch.from_numpy(v[start:start + count].copy()) for v in (x_s, x_n))
    shared_out = torch.empty(D, dtype=torch.int64)
    part2 = torch.empty(D, dtype=torch.int64)
    t_s = Dd.combine_rows_sharded(CpuEngine(), m, ms_.data_ptr(), count, D, D, part, shared_out, defer=True)
    t_n = Dd.combine_rows_sharded(CpuEngine(), m, mn_.data_ptr(), count, D, D, part2, shared_out, defer=True)
    try:
        t_s.finish()
        res["out_reuse_refused"] = False
    except ValueError:
        res["out_reuse_refused"] = True
    t_n.finish()
    res["out_reuse_later_intact"] = shared_out.tolist() == O.combine(m, x_n).tolist()
    # an input the reference's running sum could wrap on: the split refuses it (never a wrong value)
    m = 1000003
    x = torch.from_numpy(synth.fill(4, 8, 1, 0, 100))
    if rank == world - 1:
        x[2, 3] = (1 << 63) - 5
    part, out = torch.empty(8, dtype=torch.int64), torch.empty(8, dtype=torch.int64)
    try:
        Dd.combine_rows_sharded(CpuEngine(), m, x.data_ptr(), 4, 8, 8, part, out)
        res["wrap_refused"] = False
    except ValueError:
        res["wrap_refused"] = True
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_gloo_sharded_combine_matches_single_pass(world):
    """combine_rows_sharded and combine_tiles_sharded at world sizes 2, 3 and 8 (gloo; 8 = the
    driver's node), and at world 1 with the exchange forced (EXCHANGE_AT_WORLD_1), equal the reference's single sequential pass (combiner.rs:16-28) bit for bit --
    non-negative AND signed inputs (the two-pass split), raw i64 inputs, tiny moduli -- and refuse
    inputs where the reference's own sum may wrap."""
    res = _run_world2(_worker_rows, world)
    assert res.pop("wrap_refused") is True
    assert res.pop("out_reuse_refused") is True
    assert res.pop("out_reuse_later_intact") is True
    deferred = res.pop("deferred")
    for got, exp, *_ in deferred:
        assert got == exp
    # (signed, pass 1 recomputed, passes): the second job's buffer was reused by the third before its finish()
    assert [tuple(d[2:]) for d in deferred] == [(False, False, 1), (True, True, 3), (True, False, 2)]
    split = ["combine_finalize_dev", "combine_split_dev"]
    two_pass = ["combine_split_dev", "combine_split_prefix_dev", "combine_split_replay_dev",
                "combine_split_resolve_dev"]
    for name, *_ in _split_cases():
        for kind in ("rows", "tiles"):
            got, exp, signed = res[name + "/" + kind]
            assert got == exp, (name, kind)
            assert signed == (name != "nonneg"), (name, kind)
        calls = res[name + "/calls"]
        # the finalize is queued before the flags are read, so signed jobs run it too (then resolve)
        exp_calls = split if name == "nonneg" else sorted(set(split) | {c for c in two_pass
                                                                         if world > 1 or "replay" not in c})
        assert calls == exp_calls, (name, calls)           # (world 1 has no rank > 0 to replay)


def _worker_mask_columns(rank, world, port, q):
    """mask_combine_sharded (seed split + reduce) and combine_columns_sharded (signed column split +
    all-gather), the product functions, with the oracle as the per-rank compute."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Dd.EXCHANGE_AT_WORLD_1 = world == 1
    from oracle import oracle as O
    from tests.cpu_engine import CpuEngine
    eng = CpuEngine()
    m, D = 2147482801, 301
    seeds = (np.arange(10 * 4, dtype=np.int64).reshape(10, 4) * 7919) % (1 << 31)
    s0, c = Dd.shard_range(10, rank, world)
    mine = torch.from_numpy(seeds[s0:s0 + c].astype(np.int32))
    part, out = torch.empty(D, dtype=torch.int64), torch.empty(D, dtype=torch.int64)
    Dd.mask_combine_sharded(eng, m, D, mine, part, out)
    res = {"mask": (out.tolist(), O.chacha_mask_combine(m, D, seeds).tolist())}
    x = synth.fill(23, D, 0x5DA + 9, -(m - 1), m)         # signed: order-dependent exact result
    full = torch.empty(D, dtype=torch.int64)
    Dd.combine_columns_sharded(eng, m, torch.from_numpy(x), full)
    res["columns"] = (full.tolist(), O.combine(m, x).tolist())
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 8])
def test_gloo_mask_reduce_and_column_split(world):
    """sda_amd.distributed: ChaCha mask combine split over seeds + reduce, and the signed combine
    split over columns + all-gather, equal the single-pass reference (gloo, world 2 and 8)."""
    res = _run_world2(_worker_mask_columns, world)
    for k, (got, exp) in res.items():
        assert got == exp, k


def test_exchange_at_world1_is_off_by_default():
    """The forced one-rank exchange is a test hook: product callers at world size 1 never run a collective."""
    assert Dd.EXCHANGE_AT_WORLD_1 is False
    assert not Dd._exchange(1) and Dd._exchange(2)


def test_world1_helpers_return_exact_signed_result():
    """At world size 1 no reduce runs: the exact single-pass result is returned unchanged, signed
    values included (no canonicalising finalize)."""
    from oracle import oracle as O
    from tests.cpu_engine import CpuEngine
    m, N, D = 433, 9, 50
    x = torch.from_numpy(synth.fill(N, D, 0x5DA + 3, -(m - 1), m))
    part, out = torch.empty(D, dtype=torch.int64), torch.empty(D, dtype=torch.int64)
    Dd.combine_rows_sharded(CpuEngine(), m, x.data_ptr(), N, D, D, part, out)
    assert out.tolist() == O.combine(m, x.numpy()).tolist() and min(out.tolist()) < 0


@pytest.mark.parametrize("dim,world", [(1, 2), (7, 3), (1000, 8), (5, 8)])
def test_column_slice_partitions(dim, world):
    sl = [Dd.column_slice(dim, r, world) for r in range(world)]
    cols = [c for lo, n in sl for c in range(lo, lo + n)]
    assert cols == list(range(dim)) and all(lo % 2 == 0 for lo, n in sl if n)
