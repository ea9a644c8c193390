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
  result.  Overflow headroom (proved before the reduce): |sum| <= G (m - 1) <= 2^63 - 1.  The step
  queues pass 1, the all-reduce and the finalize back to back with no host read between them; the two
  flags reach the host by an asynchronous copy that SplitTicket.finish() checks afterwards (at the end
  of the call, or later with defer=True), and only a flagged job does more work.
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
    world = 1           # ranks in the group the split ran over
    redo_pass1 = False  # the two-pass path recomputed pass 1 (its buffer was reused before finish())


# Per (device, dim, stream) exchange buffer [dim results | 2 flags], kept across calls: a step allocates
# nothing.  Calls on one stream are ordered by the stream, so one buffer per stream is race-free.
_WORK = {}
# partial buffer -> generation of the last pass 1 written into it (a deferred ticket's pass-1 result is
# still there only if no later split wrote the same buffer)
_GEN = {}
# out buffer -> generation of the last split that queued its result into it: a deferred ticket whose job
# turns out signed rewrites `out` in finish(), which would clobber a LATER job's result in the same buffer
# (never cleared: a dropped entry would fail a ticket still in flight; the keys are the allocator's addresses)
_OUT_GEN = {}


def _workspace(t, dim: int, st):
    import torch
    key = (str(t.device), dim, st)
    w = _WORK.get(key)
    if w is None:
        if len(_WORK) > 16:
            _WORK.clear()
        w = _WORK[key] = torch.empty(dim + 2, dtype=torch.int64, device=t.device)
    return w


class SplitTicket:
    """A participation-split step whose sign flags are still in flight (module doc; the pattern of the
    engine's chacha_combine_begin/_end).  The step has already ENQUEUED everything the non-negative case
    needs -- pass 1, the one all-reduce, the finalize into `out` -- and an asynchronous copy of the two
    all-reduced flags into pinned host memory.  finish() waits for that 16-byte copy only, then:
    risk flag -> ValueError; negative flag -> the exact two-pass split, which rewrites `out`.
    `out` holds the job's result once finish() has returned.  Every rank must call finish() (the signed
    path runs collectives), in the same order relative to its other collectives.  Idempotent.
    Until finish() returns, the job's share rows must stay as they are (the signed path reads them again)
    and `out` must not be handed to another split: finish() raises ValueError for a signed job whose `out`
    a later split has reused (its exact result would overwrite the later job's); a reused `partial` only
    costs a recomputed pass 1."""

    def __init__(self, engine, modulus, tiles, dim, row_stride, partial, out, group, st, stats, flags_h, event,
                 gen, out_gen):
        self._args = (engine, modulus, tiles, dim, row_stride, partial, out, group, st, stats)
        self._flags_h, self._event, self._gen, self._out_gen = flags_h, event, gen, out_gen
        self._finished = False

    def done(self) -> bool:
        """True once the flags have landed on the host (finish() will not block)."""
        return self._event is None or self._event.query()

    def finish(self) -> None:
        if self._finished:
            return
        self._finished = True
        if self._event is not None:
            self._event.synchronize()             # the 16-byte flag copy, queued after the finalize
        neg, risk = int(self._flags_h[0]), int(self._flags_h[1])
        if risk:
            raise ValueError("participation split: an input lies outside [-(2^63 - m), 2^63 - m], where the "
                             "reference's running sum may wrap; combine on one rank or split by columns")
        if neg:
            if _OUT_GEN.get(self._args[6].data_ptr()) != self._out_gen:
                raise ValueError("participation split: this signed job's `out` was reused by a later split before "
                                 "finish(); its exact result would overwrite that job's (one `out` per ticket in "
                                 "flight)")
            _two_pass(*self._args, redo=_GEN.get(self._args[5].data_ptr()) != self._gen)


def _two_pass(engine, modulus, tiles, dim, row_stride, partial, out, group, st, stats, redo):
    """Signed inputs somewhere: the exact two-pass split (module doc).  `partial` holds this rank's pass-1
    result unless `redo` (a later split reused the buffer before a deferred finish()): pass 1 again."""
    import torch
    import torch.distributed as dist

    world, rank = _world(group), dist.get_rank(group)
    stats.signed, stats.passes, stats.redo_pass1 = True, 3 if redo else 2, redo
    with _on(partial, st):
        if redo:                     # into a scratch buffer: `partial` may hold a later ticket's pass 1
            flags = torch.zeros(2, dtype=torch.int64, device=partial.device)
            partial = torch.zeros(dim, dtype=torch.int64, device=partial.device)
            for ptr, n in tiles:
                engine.combine_split_dev(modulus, ptr, n, dim, row_stride, partial.data_ptr(), flags.data_ptr(), st)
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


def _combine_split(engine, modulus: int, tiles, dim: int, row_stride: int, partial, out, group, stream,
                   stats: SplitStats = None, defer: bool = False):
    """The participation split of combiner.rs:16-28 (module doc): this rank's rows as row tiles
    [(ptr, n_rows), ...] in participation order; `partial` int64 [dim] receives this rank's pass-1
    result, `out` int64 [dim] the job's result on every rank.  The non-negative case makes no blocking
    host read: pass 1, the all-reduce and the finalize are queued back to back and the flags travel
    to the host asynchronously (SplitTicket).  defer=False checks them before returning (after all
    the work is queued); defer=True returns the ticket and the caller finishes it later."""
    import torch
    import torch.distributed as dist

    tiles = list(tiles)
    world = _world(group)
    st = _stream(partial, stream)
    stats = stats if stats is not None else SplitStats()
    stats.signed, stats.passes, stats.world, stats.redo_pass1 = False, 1, world, False
    with _on(partial, st):
        if not _exchange(world):     # one sequential pass: the exact result, signed values included
            if len(tiles) == 1:
                engine.combine_dev(modulus, tiles[0][0], tiles[0][1], dim, row_stride, partial.data_ptr(), st)
            else:
                partial.zero_()
                for ptr, n in tiles:
                    engine.combine_accumulate_dev(modulus, ptr, n, dim, row_stride, partial.data_ptr(), st)
            out.copy_(partial)
            return None
        if not reduce_headroom_ok(world, modulus):
            raise ValueError(f"reduce headroom: {world} * (m - 1) exceeds 2^63 - 1")
        # pass 1 into `partial` (kept for the signed path) + the flags, then ONE all-reduce of
        # [results | flags] in the cached exchange buffer
        work = _workspace(partial, dim, st)
        partial.zero_()
        work[dim:].zero_()
        for ptr, n in tiles:
            engine.combine_split_dev(modulus, ptr, n, dim, row_stride, partial.data_ptr(),
                                     work[dim:].data_ptr(), st)
        if len(_GEN) > 1024:
            _GEN.clear()
        gen = _GEN[partial.data_ptr()] = _GEN.get(partial.data_ptr(), 0) + 1
        out_gen = _OUT_GEN[out.data_ptr()] = _OUT_GEN.get(out.data_ptr(), 0) + 1
        work[:dim].copy_(partial)
        dist.all_reduce(work, op=dist.ReduceOp.SUM, group=group)
        # the finalize is the result whenever no rank saw a negative input: queue it now, read the
        # flags later (a signed job rewrites `out` in finish())
        engine.combine_finalize_dev(modulus, work.data_ptr(), dim, out.data_ptr(), st)
        if work.is_cuda:
            flags_h = torch.empty(2, dtype=torch.int64, pin_memory=True)
            flags_h.copy_(work[dim:], non_blocking=True)
            event = torch.cuda.Event()
            event.record()                       # on `st` (the current stream inside _on)
        else:                                    # host tensors (CPU / gloo tests): already there
            flags_h, event = work[dim:].clone(), None
    ticket = SplitTicket(engine, modulus, tiles, dim, row_stride, partial, out, group, st, stats, flags_h, event,
                         gen, out_gen)
    if defer:
        return ticket
    ticket.finish()
    return None


def combine_tiles_sharded(engine, modulus: int, tiles: Iterable[Tuple[int, int]], dim: int, row_stride: int,
                          partial, out, group=None, stream=None, stats: SplitStats = None, defer: bool = False):
    """This rank's participations as row tiles [(shares_ptr, n_rows), ...] (the recurrence continues
    across tiles, so they act as one pass; the signed path reads them twice) through the exact
    participation split.  `partial` / `out`: int64 [dim] on this rank's device.  Any inputs: signed
    ones take the two-pass path; inputs the reference's sum could wrap on raise ValueError.
    defer=True returns a SplitTicket (N > 1; None at world size 1): `out` is final after its finish()."""
    return _combine_split(engine, modulus, tiles, dim, row_stride, partial, out, group, stream, stats, defer)


def combine_rows_sharded(engine, modulus: int, shares_ptr: int, n_local: int, dim: int, row_stride: int,
                         partial, out, group=None, stream=None, stats: SplitStats = None, defer: bool = False):
    """Exact participation split of combiner.rs:16-28 over this rank's [n_local][row_stride] rows
    (defer: see combine_tiles_sharded)."""
    return _combine_split(engine, modulus, [(shares_ptr, n_local)], dim, row_stride, partial, out, group, stream,
                          stats, defer)


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
