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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    m, N, D = 2147482801, 37, 129
    full = synth.fill(N, D, 0x5DA + 4, 0, m)             # non-negative inputs (configs[3])
    start, count = Dd.shard_range(N, rank, world)
    part = torch.from_numpy(O.combine(m, full[start:start + count]))   # per-rank exact combine (CPU stand-in)
    dist.all_reduce(part, op=dist.ReduceOp.SUM)          # int64 sum == u64 two's-complement sum
    got = part.numpy() % m
    if rank == 0:
        q.put((got.tolist(), O.combine(m, full).tolist()))
    dist.destroy_process_group()


def test_gloo_world2_sharded_combine_matches_single_pass():
    """The N-split + int64 all-reduce + final mod of sda_amd.distributed equals the reference's
    single sequential pass for non-negative inputs (world size 2, gloo on CPU)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, exp = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert got == exp


def _worker2(rank, world, port, q):
    """reduce_canonical over the ChaCha mask N-split, and the column split of a signed combine,
    with the oracle as the per-rank compute stand-in."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    m, D = 2147482801, 301
    seeds = (np.arange(10 * 4, dtype=np.int64).reshape(10, 4) * 7919) % (1 << 31)
    s0, c = Dd.shard_range(10, rank, world)
    part = torch.from_numpy(O.chacha_mask_combine(m, D, seeds[s0:s0 + c]))
    out = torch.empty(D, dtype=torch.int64)
    Dd.reduce_canonical(part, m, lambda p, o: o.copy_(torch.remainder(p, m)), out)
    res = {"mask": (out.tolist(), O.chacha_mask_combine(m, D, seeds).tolist())}
    x = synth.fill(23, D, 0x5DA + 9, -(m - 1), m)         # signed: order-dependent exact result
    lo, cnt = Dd.column_slice(D, rank, world)
    width = max(Dd.column_slice(D, r, world)[1] for r in range(world))
    mine = torch.zeros(width, dtype=torch.int64)
    mine[:cnt] = torch.from_numpy(O.combine(m, np.ascontiguousarray(x[:, lo:lo + cnt])))
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    full = torch.cat([parts[r][:Dd.column_slice(D, r, world)[1]] for r in range(world)])
    res["columns"] = (full.tolist(), O.combine(m, x).tolist())
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


def test_gloo_world2_mask_reduce_and_column_split():
    """sda_amd.distributed: ChaCha mask combine split over seeds + reduce_canonical, and the signed
    combine split over columns + all-gather, equal the single-pass reference (gloo, world 2)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker2, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    for k, (got, exp) in res.items():
        assert got == exp, k


@pytest.mark.parametrize("dim,world", [(1, 2), (7, 3), (1000, 8), (5, 8)])
def test_column_slice_partitions(dim, world):
    sl = [Dd.column_slice(dim, r, world) for r in range(world)]
    cols = [c for lo, n in sl for c in range(lo, lo + n)]
    assert cols == list(range(dim)) and all(lo % 2 == 0 for lo, n in sl if n)
