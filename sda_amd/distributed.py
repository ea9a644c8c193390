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
reduction, only an all-gather of the slices.

The same N-split + one reduce serves the recipient's ChaCha mask combine (chacha.rs:57-76):
every draw is >= 0, so per-rank canonical partial sums reduce exactly.  Packed share-gen and
reveal shard by participant vector / batch with no collective at all (shard_range).
"""
from __future__ import annotations

from typing import Tuple

I64_MAX = (1 << 63) - 1


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous near-equal split of n items: (start, count) for `rank`."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def reduce_headroom_ok(world: int, modulus: int) -> bool:
    """Sum of `world` residues in [0, m) must not overflow the i64 all-reduce."""
    return world * (abs(modulus) - 1) <= I64_MAX


def combine_rows_sharded(engine, modulus: int, shares_ptr: int, n_local: int, dim: int, row_stride: int,
                         partial, out, group=None, stream=None):
    """Exact per-rank combine + all-reduce(SUM) over int64 + device finalize.

    `partial` / `out` are int64 torch tensors of length `dim` on this rank's device; shares_ptr
    points at this rank's [n_local][row_stride] slice.  Requires non-negative inputs."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if stream is None:   # stay on torch's current stream so the collective is ordered after the kernel
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    if not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    engine.combine_dev(modulus, shares_ptr, n_local, dim, row_stride, partial.data_ptr(), stream)
    if world > 1:
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    engine.combine_finalize_dev(modulus, partial.data_ptr(), dim, out.data_ptr(), stream)


def reduce_canonical(partial, modulus: int, finalize, out, group=None):
    """One all-reduce(SUM) over int64 of per-rank residues in [0, m), then `finalize(partial, out)`
    (the device `% m`).  Exact for non-negative inputs within the headroom."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    if world > 1:
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    finalize(partial, out)


def mask_combine_sharded(engine, modulus: int, dim: int, seeds, partial, out, group=None, stream=None):
    """Recipient ChaCha mask combine with the seeds split over the ranks: each rank expands and
    sums its own seeds ([n_local][w] int32 device tensor), then one int64 all-reduce + final mod."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    n_local, w = (seeds.shape[0], seeds.shape[1]) if seeds.dim() == 2 else (0, 4)
    engine.chacha_mask_combine_dev(modulus, dim, seeds.data_ptr() if n_local else 0, w, n_local,
                                   partial.data_ptr(), stream)
    reduce_canonical(partial, modulus,
                     lambda p, o: engine.combine_finalize_dev(modulus, p.data_ptr(), dim, o.data_ptr(), stream),
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
    reduction, bit-exact), then the slices are all-gathered into `out` ([dim] int64 device)."""
    import torch
    import torch.distributed as dist

    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n, dim = shares.shape
    lo, cnt = column_slice(dim, rank, world)
    width = max(column_slice(dim, r, world)[1] for r in range(world))
    mine = torch.zeros(width, dtype=torch.int64, device=out.device)
    if cnt:
        engine.combine_dev(modulus, shares[:, lo:].data_ptr(), n, cnt, dim, mine.data_ptr(), stream)
    parts = [torch.empty_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(parts, mine, group=group)
    else:
        parts = [mine]
    for r in range(world):
        l, c = column_slice(dim, r, world)
        out[l:l + c] = parts[r][:c]
