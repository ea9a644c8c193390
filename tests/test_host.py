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
