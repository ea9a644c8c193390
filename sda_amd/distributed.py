"""Multi-GPU sharding of the clerk combine (one process per GPU).

Participations are independent, so a clerking job's N rows split across the G ranks of one node
(rank g holds a contiguous range, in participation order).  Each rank runs the exact combine
(combiner.rs:16-28) on its rows (pass 1).  The reference's result is r = (sum of inputs) mod m as a
canonical residue when every input is >= 0, but a SIGNED, order-dependent value in (-m, m) as soon as
one input is negative -- and real Additive clerk jobs are signed (the last share is
`(secret - x) % m`, additive.rs:46).  So pass 1 also raises two device flags (an input < 0; an input
so large that the reference's own `r + v` may wrap i64), and one all-reduce carries the flags with the
ranks' results:

* no negative input anywhere: the int64 SUM of the ranks' canonical results, taken by that ONE
  all-reduce over RCCL (xGMI), then a device `% m` (sda_combine_finalize_dev), IS the reference's
  result.  Overflow headroom (proved before the reduce): |sum| <= G (m - 1) <= 2^63 - 1.
* some negative input: exact two-pass split (SURVEY §7 hard part 1 option (b)).  The
  pass-1 results are all-gathered; each rank g > 0 gets its incoming residue c_in = canonical sum of
  ranks < g and replays its rows from c_in, recording only the LAST sign event (set / reset / none) of
  the reference's running value; an all-reduce MAX over per-rank event codes picks the last event in
  participation order; the result is the canonical total, minus m when that event set the sign.
  Bit-exact with one sequential pass; costs a second read of the rows.
* an input outside [-(2^63 - m), 2^63 - m]: the reference's running sum may wrap there, which no
  split reproduces -- ValueError (use one rank, or the column split).

At world size 1 no exchange runs and the exact single-pass result is returned as is
(`EXCHANGE_AT_WORLD_1` = True runs the full exchange path instead, over a one-rank group: how a one-GPU
box drives RCCL through the very calls of the 8-GPU run, tests/test_gpu_multirank.py).  The column split
(combine_columns_sharded: each rank owns a slice of D and walks all N rows) stays for callers that
hold whole columns.

The same N-split + one reduce serves the recipient's ChaCha mask combine (chacha.rs:57-76): every
draw is >= 0, so per-rank canonical partial sums reduce exactly (moduli up to 2^62; above that the
reference's own sum wraps and is order dependent, and the headroom check refuses G > 1).  Packed
share-gen and reveal shard by participant vector / batch with no collective at all (shard_range).

`engine` is anything with the device entry points used here (sda_amd.Engine; the CPU tests pass a
stand-in that runs the oracle on host tensors).  Everything a helper enqueues -- engine launches,
copies and collectives -- runs on one stream: `stream` when given, else torch's current stream.
"""
from __future__ import annotations

from typing import Iterable, Tuple

I64_MAX = (1 << 63) - 1
EXCHANGE_AT_WORLD_1 = False     # run the collectives even in a one-rank group (module doc)


def _exchange(world: int) -> bool:
    return world > 1 or EXCHANGE_AT_WORLD_1


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


def _on(t, st):
    """Context that makes `st` torch's current stream on t's device (so torch copies and the
    collectives queue behind the engine's launches on it); a no-op for host tensors."""
    import contextlib
    if st is None or not t.is_cuda:
        return contextlib.nullcontext()
    import torch
    if st == torch.cuda.current_stream(t.device).cuda_stream:
        return contextlib.nullcontext()
    return torch.cuda.stream(torch.cuda.ExternalStream(st, device=t.device))


def reduce_canonical(partial, modulus: int, finalize, out, group=None):
    """One all-reduce(SUM) over int64 of per-rank residues in [0, m), then `finalize(partial, out)`
    (the device `% m`).  Exact for non-negative inputs within the headroom.  World size 1: out is
    the single-pass result itself.  Call on the stream the inputs were produced on."""
    import torch.distributed as dist

    world = _world(group)
    if not _exchange(world):
        out.copy_(partial)
        return
    if not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    finalize(partial, out)


class SplitStats:
    """What the last participation split did on this rank (bench.py and the tests read it)."""
    signed = False      # some rank saw a negative input -> the two-pass path ran
    passes = 1


def _combine_split(engine, modulus: int, tiles, dim: int, row_stride: int, partial, out, group, stream,
                   stats: SplitStats = None):
    """The participation split of combiner.rs:16-28 (module doc): this rank's rows as row tiles
    [(ptr, n_rows), ...] in participation order; `partial` int64 [dim] receives this rank's pass-1
    result, `out` int64 [dim] the job's result on every rank."""
    import torch
    import torch.distributed as dist

    tiles = list(tiles)
    world = _world(group)
    st = _stream(partial, stream)
    stats = stats if stats is not None else SplitStats()
    stats.signed, stats.passes = False, 1
    with _on(partial, st):
        if not _exchange(world):     # one sequential pass: the exact result, signed values included
            if len(tiles) == 1:
                engine.combine_dev(modulus, tiles[0][0], tiles[0][1], dim, row_stride, partial.data_ptr(), st)
            else:
                partial.zero_()
                for ptr, n in tiles:
                    engine.combine_accumulate_dev(modulus, ptr, n, dim, row_stride, partial.data_ptr(), st)
            out.copy_(partial)
            return
        partial.zero_()
        if not reduce_headroom_ok(world, modulus):
            raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
        rank = dist.get_rank(group)
        # pass 1 + the flags, then ONE all-reduce of [partial | flags]
        work = torch.zeros(dim + 2, dtype=torch.int64, device=partial.device)
        for ptr, n in tiles:
            engine.combine_split_dev(modulus, ptr, n, dim, row_stride, partial.data_ptr(),
                                     work[dim:].data_ptr(), st)
        work[:dim].copy_(partial)
        dist.all_reduce(work, op=dist.ReduceOp.SUM, group=group)
        neg, risk = (int(v) for v in work[dim:].tolist())          # host sync: 16 bytes
        if risk:
            raise ValueError("participation split: an input lies outside [-(2^63 - m), 2^63 - m], where the "
                             "reference's running sum may wrap; combine on one rank or split by columns")
        if not neg:
            engine.combine_finalize_dev(modulus, work.data_ptr(), dim, out.data_ptr(), st)
            return
        # signed inputs: the exact two-pass split
        stats.signed, stats.passes = True, 2
        gathered = torch.empty((world, dim), dtype=torch.int64, device=partial.device)
        dist.all_gather(list(gathered.unbind(0)), partial, group=group)
        state = torch.empty(dim, dtype=torch.int64, device=partial.device)
        total = torch.empty(dim, dtype=torch.int64, device=partial.device)
        code = torch.empty(dim, dtype=torch.int32, device=partial.device)
        engine.combine_split_prefix_dev(modulus, gathered.data_ptr(), world, rank, dim, state.data_ptr(),
                                        total.data_ptr(), code.data_ptr(), st)
        if rank > 0:                 # rank 0's sign is its own pass-1 result's (the prefix kernel set it)
            for ptr, n in tiles:
                engine.combine_split_replay_dev(modulus, ptr, n, dim, row_stride, rank, state.data_ptr(),
                                                code.data_ptr(), st)
        dist.all_reduce(code, op=dist.ReduceOp.MAX, group=group)
        engine.combine_split_resolve_dev(modulus, total.data_ptr(), code.data_ptr(), dim, out.data_ptr(), st)


def combine_tiles_sharded(engine, modulus: int, tiles: Iterable[Tuple[int, int]], dim: int, row_stride: int,
                          partial, out, group=None, stream=None, stats: SplitStats = None):
    """This rank's participations as row tiles [(shares_ptr, n_rows), ...] (the recurrence continues
    across tiles, so they act as one pass; the signed path reads them twice) through the exact
    participation split.  `partial` / `out`: int64 [dim] on this rank's device.  Any inputs: signed
    ones take the two-pass path; inputs the reference's sum could wrap on raise ValueError."""
    _combine_split(engine, modulus, tiles, dim, row_stride, partial, out, group, stream, stats)


def combine_rows_sharded(engine, modulus: int, shares_ptr: int, n_local: int, dim: int, row_stride: int,
                         partial, out, group=None, stream=None, stats: SplitStats = None):
    """Exact participation split of combiner.rs:16-28 over this rank's [n_local][row_stride] rows."""
    _combine_split(engine, modulus, [(shares_ptr, n_local)], dim, row_stride, partial, out, group, stream, stats)


def mask_combine_sharded(engine, modulus: int, dim: int, seeds, partial, out, group=None, stream=None):
    """Recipient ChaCha mask combine with the seeds split over the ranks: each rank expands and
    sums its own seeds ([n_local][w] int32 tensor), then one int64 all-reduce + final mod."""
    world = _world(group)
    if world > 1 and not reduce_headroom_ok(world, modulus):
        raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
    st = _stream(partial, stream)
    n_local, w = (seeds.shape[0], seeds.shape[1]) if seeds.dim() == 2 else (0, 4)
    with _on(partial, st):
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
    with _on(out, st):
        mine = torch.zeros(width, dtype=torch.int64, device=out.device)
        if cnt:
            engine.combine_dev(modulus, shares[:, lo:].data_ptr(), n, cnt, shares.stride(0), mine.data_ptr(), st)
        parts = [torch.empty_like(mine) for _ in range(world)]
        if _exchange(world):
            dist.all_gather(parts, mine, group=group)
        else:
            parts = [mine]
        for r in range(world):
            l, c = column_slice(dim, r, world)
            out[l:l + c] = parts[r][:c]
