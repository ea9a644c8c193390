"""One rank of tests/test_gpu_multirank.py: the product's multi-GPU helpers (sda_amd.distributed) on the
HIP engine, two or four ranks sharing one MI355X (cuda:0) over gloo -- or one rank over RCCL
(SDA_MR_BACKEND=nccl) with the exchange path forced at world size 1.

Not a test module: test_gpu_multirank starts two of these as plain child processes (RANK 0 and 1),
so the collective path of bench.py --gpus N runs with the real device kernels and real device tensors;
only the transport differs from the 8-GPU node (gloo instead of RCCL, since RCCL refuses two ranks on
one device).  Rank 0 writes every result to $SDA_MR_OUT (.npz); the parent compares with the oracle.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MOD = 2147482801
# participation-split cases (name, rows, dim, modulus, lo, hi): non-negative shares (one reduce) and
# signed shares (real Additive clerk jobs, additive.rs:46: the exact two-pass split), ragged and 1000 x 100k,
# a tiny modulus (sign events almost every step) and raw i64 values outside (-m, m) (generic kernel path)
CASES = [("nonneg", 37, 129, MOD, 0, MOD), ("nonneg", 1000, 100_003, MOD, 0, MOD),
         ("signed", 37, 129, MOD, -(MOD - 1), MOD), ("signed", 1000, 100_003, MOD, -(MOD - 1), MOD),
         ("small_m", 203, 4_099, 7, -6, 7), ("raw_i64", 64, 20_001, 1000003, -(1 << 61), 1 << 61)]
TILE = 128
SEEDS = (np.arange(48 * 4, dtype=np.int64).reshape(48, 4) * 7919 + 11) % (1 << 31)
SIGNED = (301, 50_001)
SEEDS10M = (np.arange(8 * 4, dtype=np.int64).reshape(8, 4) * 104729 + 7) % (1 << 31)


def main():
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    torch.cuda.init()
    backend = os.environ.get("SDA_MR_BACKEND", "gloo")
    if backend == "nccl":          # RCCL: one rank per device, so world 1 here
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from sda_amd import Engine, synth
    from sda_amd import distributed as Dd
    Dd.EXCHANGE_AT_WORLD_1 = world == 1     # world 1: the same collectives over a one-rank group

    eng = Engine(0)
    dev = torch.device("cuda", 0)
    res = {}
    for name, N, D, m, lo, hi in CASES:
        s0, cnt = Dd.shard_range(N, rank, world)
        mine = torch.from_numpy(synth.fill(cnt, D, 0x5DA + 21, lo, hi, row0=s0)).to(dev)
        part = torch.empty(D, dtype=torch.int64, device=dev)
        out = torch.empty(D, dtype=torch.int64, device=dev)
        st = Dd.SplitStats()
        Dd.combine_rows_sharded(eng, m, mine.data_ptr(), cnt, D, D, part, out, stats=st)
        res[f"rows_{name}_{N}x{D}"] = out.cpu().numpy()
        res[f"signed_{name}_{N}x{D}"] = np.array(st.signed)
        # the same participations streamed as row tiles (configs[3]'s accumulate on every rank)
        tiles = [(mine[t0].data_ptr(), min(TILE, cnt - t0)) for t0 in range(0, cnt, TILE)]
        out2 = torch.empty(D, dtype=torch.int64, device=dev)
        Dd.combine_tiles_sharded(eng, m, tiles, D, D, part, out2)
        res[f"tiles_{name}_{N}x{D}"] = out2.cpu().numpy()
        del mine

    if backend == "nccl":
        # a non-negative split step makes no blocking host read: with ~0.1 s of GPU work queued ahead of
        # it, the deferred step (pass 1, RCCL all-reduce, finalize, async flag copy) returns to the host
        # long before that work ends, its ticket still pending; finish() then yields the exact result
        N, D = 64, 100_003
        mine = torch.from_numpy(synth.fill(N, D, 0x5DA + 23, 0, MOD)).to(dev)
        part = torch.empty(D, dtype=torch.int64, device=dev)
        out = torch.empty(D, dtype=torch.int64, device=dev)
        Dd.combine_rows_sharded(eng, MOD, mine.data_ptr(), N, D, D, part, out)      # warm the caches
        torch.cuda.synchronize()
        torch.cuda._sleep(200_000_000)
        t0 = time.perf_counter()
        tk = Dd.combine_rows_sharded(eng, MOD, mine.data_ptr(), N, D, D, part, out, defer=True)
        res["deferred_host_s"] = np.array(time.perf_counter() - t0)
        res["deferred_pending"] = np.array(not tk.done())
        tk.finish()
        t1 = time.perf_counter()
        res["deferred_wait_s"] = np.array(t1 - t0)
        res["deferred_out"] = out.cpu().numpy()
        del mine

    # recipient's ChaCha mask combine, seeds split over the ranks + one reduce
    s0, cnt = Dd.shard_range(SEEDS.shape[0], rank, world)
    seeds = torch.from_numpy(SEEDS[s0:s0 + cnt].astype(np.int32)).to(dev)
    D = 70_001
    part = torch.empty(D, dtype=torch.int64, device=dev)
    out = torch.empty(D, dtype=torch.int64, device=dev)
    Dd.mask_combine_sharded(eng, MOD, D, seeds, part, out)
    res["mask"] = out.cpu().numpy()
    # configs[4]'s dimension: 8 seeds x 10M-dim, split over the ranks
    D = 10_000_000
    s0, cnt = Dd.shard_range(SEEDS10M.shape[0], rank, world)
    seeds = torch.from_numpy(SEEDS10M[s0:s0 + cnt].astype(np.int32)).to(dev)
    part = torch.empty(D, dtype=torch.int64, device=dev)
    out = torch.empty(D, dtype=torch.int64, device=dev)
    Dd.mask_combine_sharded(eng, MOD, D, seeds, part, out)
    res["mask10M"] = out.cpu().numpy()
    del part, out

    # signed (order-dependent) combine: column split + all-gather
    N, D = SIGNED
    x = torch.from_numpy(synth.fill(N, D, 0x5DA + 22, -(MOD - 1), MOD)).to(dev)
    full = torch.empty(D, dtype=torch.int64, device=dev)
    Dd.combine_columns_sharded(eng, MOD, x, full)
    res["columns"] = full.cpu().numpy()

    torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        np.savez(os.environ["SDA_MR_OUT"], **res)
    dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
