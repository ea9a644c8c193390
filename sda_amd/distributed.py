"""Multi-GPU sharding of the clerk combine (one process per GPU).

Participations are independent, so a clerking job's N rows split across the G ranks of one
node with no data-path exchange.  Each rank runs the exact combine (combiner.rs:16-28) on its
row range; the per-rank results are non-negative residues in [0, m) whenever the inputs are
non-negative (masks, canonicalised shares -- and the benchmark configs), so their sum over
ranks, taken as u64/two's-complement i64 by ONE all-reduce over RCCL (xGMI), followed by a
final `% m` on device, equals the reference's single-pass result bit for bit.

Overflow headroom (proved before the reduce): the reduced value is at most G * (m - 1), which
must stay below 2^63.  For signed inputs the exact result is order dependent; those use the
column split (each rank owns a slice of D and walks all N rows) instead, which needs no
reduction, only an all-gather of the slices.  At world size 1 no reduce runs and the exact
single-pass result is returned as is (signed inputs included).

The same N-split + one reduce serves the recipient's ChaCha mask combine (chacha.rs:57-76):
every draw is >= 0, so per-rank canonical partial sums reduce exactly (moduli up to 2^62; above
that the reference's own sum wraps and is order dependent, and the headroom check refuses G > 1).
Packed share-gen and reveal shard by participant vector / batch with no collective at all
(shard_range).

`engine` is anything with the device entry points used here (sda_amd.Engine; the CPU tests pass
a stand-in that runs the oracle on host tensors).
"""
from __future__ import annotations

from typing import Iterable, Tuple

I64_MAX = (1 << 63) - 1


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous near-equal split of n items: (start, count) for `rank`."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def reduce_headroom_ok(world: int, modulus: int) -> bool:
    """Sum of `world` residues in [0, m) must not overflow the i64 all-reduce."""
    return world * (abs(modulus) - 1) <= I64_MAX


def _world(group):
    import torch.distributed as dist
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _stream(t, stream):
    """The caller's stream, else torch's current stream on t's device (engine launches and the
    collective are then ordered on one stream); host tensors (CPU tests) have none."""
    if stream is not None or not t.is_cuda:
        return stream
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def reduce_canonical(partial, modulus: int, finalize, out, group=None):
    """One all-reduce(SUM) over int64 of per-rank residues in [0, m), then `finalize(partial, out)`
    (the device `% m`).  Exact for non-negative inputs within the headroom.  World size 1: out is
    the single-pass result itself."""
    import torch.distributed as dist

    world = _world(group)
    if world == 1:
        out.copy_(partial)
        return
    if not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    finalize(partial, out)


def combine_tiles_sharded(engine, modulus: int, tiles: Iterable[Tuple[int, int]], dim: int, row_stride: int,
                          partial, out, group=None, stream=None):
    """This rank's participations as row tiles [(shares_ptr, n_rows), ...] streamed through the exact
    combine (sda_combine_accumulate_dev continues the recurrence, so the tiles act as one pass), then
    the all-reduce + device finalize across ranks.  `partial` / `out`: int64 [dim] on this rank's
    device.  World size > 1 requires non-negative inputs (see module doc)."""
    world = _world(group)
    if world > 1 and not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    st = _stream(partial, stream)
    partial.zero_()
    for ptr, n in tiles:
        engine.combine_accumulate_dev(modulus, ptr, n, dim, row_stride, partial.data_ptr(), st)
    reduce_canonical(partial, modulus,
                     lambda p, o: engine.combine_finalize_dev(modulus, p.data_ptr(), dim, o.data_ptr(), st),
                     out, group)


def combine_rows_sharded(engine, modulus: int, shares_ptr: int, n_local: int, dim: int, row_stride: int,
                         partial, out, group=None, stream=None):
    """Exact per-rank combine of [n_local][row_stride] rows + all-reduce(SUM) over int64 + device
    finalize (combiner.rs:16-28 over the participation split)."""
    world = _world(group)
    if world > 1 and not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    st = _stream(partial, stream)
    engine.combine_dev(modulus, shares_ptr, n_local, dim, row_stride, partial.data_ptr(), st)
    reduce_canonical(partial, modulus,
                     lambda p, o: engine.combine_finalize_dev(modulus, p.data_ptr(), dim, o.data_ptr(), st),
                     out, group)


def mask_combine_sharded(engine, modulus: int, dim: int, seeds, partial, out, group=None, stream=None):
    """Recipient ChaCha mask combine with the seeds split over the ranks: each rank expands and
    sums its own seeds ([n_local][w] int32 tensor), then one int64 all-reduce + final mod."""
    world = _world(group)
    if world > 1 and not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    st = _stream(partial, stream)
    n_local, w = (seeds.shape[0], seeds.shape[1]) if seeds.dim() == 2 else (0, 4)
    engine.chacha_mask_combine_dev(modulus, dim, seeds.data_ptr() if n_local else 0, w, n_local,
                                   partial.data_ptr(), st)
    reduce_canonical(partial, modulus,
                     lambda p, o: engine.combine_finalize_dev(modulus, p.data_ptr(), dim, o.data_ptr(), st),
                     out, group)


def column_slice(dim: int, rank: int, world: int) -> Tuple[int, int]:
    """Even column split for the signed (order-dependent) combine; slices start on even columns so
    every rank keeps the 16-byte vector path."""
    pairs = (dim + 1) // 2
    start, count = shard_range(pairs, rank, world)
    lo = 2 * start
    return lo, max(0, min(dim, 2 * (start + count)) - lo)


def combine_columns_sharded(engine, modulus: int, shares, out, group=None, stream=None):
    """Signed inputs: each rank runs the exact combine over ALL rows of its column slice (no
    reduction, bit-exact), then the slices are all-gathered into `out` ([dim] int64)."""
    import torch
    import torch.distributed as dist

    st = _stream(out, stream)
    world = _world(group)
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n, dim = shares.shape
    lo, cnt = column_slice(dim, rank, world)
    width = max(column_slice(dim, r, world)[1] for r in range(world))
    mine = torch.zeros(width, dtype=torch.int64, device=out.device)
    if cnt:
        engine.combine_dev(modulus, shares[:, lo:].data_ptr(), n, cnt, shares.stride(0), mine.data_ptr(), st)
    parts = [torch.empty_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(parts, mine, group=group)
    else:
        parts = [mine]
    for r in range(world):
        l, c = column_slice(dim, r, world)
        out[l:l + c] = parts[r][:c]
