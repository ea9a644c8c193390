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
reduction at all.
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
