"""GPU: the multi-GPU helpers (sda_amd.distributed) at world size 2 and 4 on the HIP engine.

Child processes (tests/multirank_worker.py, one per RANK) share cuda:0 and a gloo process group:
each runs the engine's device kernels on its own participations / seeds / column slice, and the
product functions do the exchange (int64 all-reduce + device finalize, or all-gather) on device
tensors -- the code path of `bench.py --gpus N`, with gloo standing in for RCCL (RCCL refuses two
ranks on one device; the 8-GPU node runs the same calls over RCCL).  The third case runs ONE rank over
RCCL with the exchange forced at world size 1 (distributed.EXCHANGE_AT_WORLD_1): every RCCL call of the
8-GPU path -- int64 SUM all-reduce, the flag readback, all-gather into row views, int32 MAX all-reduce --
on real device tensors, against the same oracle results.  The results must equal the
reference's single sequential pass (combiner.rs:16-28, chacha.rs:57-76), recomputed by the oracle.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from sda_amd import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import multirank_worker as W  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module", params=[(2, "gloo"), (4, "gloo"), (1, "nccl")],
                ids=["world2", "world4", "rccl_world1"])
def results(request, tmp_path_factory):
    world, backend = request.param
    out = str(tmp_path_factory.mktemp("mr") / "res.npz")
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               SDA_MR_OUT=out, SDA_MR_BACKEND=backend, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "multirank_worker.py")],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    with np.load(out) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name,N,D,m,lo,hi", W.CASES)
def test_sharded_rows_and_tiles_equal_single_pass(results, oracle, name, N, D, m, lo, hi):
    """combine_rows_sharded / combine_tiles_sharded: participation split == the single sequential pass
    over all N rows -- non-negative shares through one int64 all-reduce + device `% m`, signed shares
    through the exact two-pass split (replay + MAX-resolved sign events)."""
    full = synth.fill(N, D, 0x5DA + 21, lo, hi)
    exp = oracle.combine(m, full)
    assert bool(results[f"signed_{name}_{N}x{D}"]) == (lo < 0)
    if lo < 0:
        assert (exp < 0).any()
    assert np.array_equal(results[f"rows_{name}_{N}x{D}"], exp)
    assert np.array_equal(results[f"tiles_{name}_{N}x{D}"], exp)


def test_split_step_makes_no_blocking_host_read(results, oracle):
    """rccl_world1: the non-negative participation-split step (defer=True) returns to the host while
    ~0.1 s of earlier GPU work is still running -- no host read between its RCCL all-reduce and its
    finalize -- and its ticket's finish() then gives the exact result."""
    if "deferred_out" not in results:
        pytest.skip("RCCL case only")
    host_s, wait_s = float(results["deferred_host_s"]), float(results["deferred_wait_s"])
    assert bool(results["deferred_pending"]), "the step's flags were already on the host: it waited"
    assert host_s < wait_s / 2, (host_s, wait_s)
    x = synth.fill(64, 100_003, 0x5DA + 23, 0, W.MOD)
    assert np.array_equal(results["deferred_out"], oracle.combine(W.MOD, x))


def test_sharded_mask_combine_seed_split(results, oracle):
    """mask_combine_sharded: the recipient's ChaCha mask combine over seeds split across ranks."""
    exp = oracle.chacha_mask_combine(W.MOD, 70_001, W.SEEDS)
    assert np.array_equal(results["mask"], exp)


def test_sharded_mask_combine_10M(results, oracle):
    """mask_combine_sharded at configs[4]'s dimension (8 seeds x 10M-dim split over the ranks)."""
    exp = oracle.chacha_mask_combine(W.MOD, 10_000_000, W.SEEDS10M)
    assert np.array_equal(results["mask10M"], exp)


def test_sharded_signed_column_split(results, oracle):
    """combine_columns_sharded: signed shares (order-dependent exact result), column split +
    all-gather, bit-exact with the sequential recurrence."""
    N, D = W.SIGNED
    x = synth.fill(N, D, 0x5DA + 22, -(W.MOD - 1), W.MOD)
    exp = oracle.combine(W.MOD, x)
    assert (exp < 0).any()
    assert np.array_equal(results["columns"], exp)


def test_bench_spawns_its_own_ranks(tmp_path):
    """`bench.py --gpus 2` with no launcher starts its two ranks itself (gloo rehearsal: both share
    cuda:0) and rank 0 prints the JSON line with n_gpus = 2; the signed participation-split leg runs
    and checks itself.  A mismatched WORLD_SIZE exits non-zero instead of benchmarking one GPU."""
    import json
    root = os.path.dirname(HERE)
    env = dict(os.environ, SDA_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--no-side", "--no-cpu", "--steps", "2",
           "--warmup", "1", "--rows", "64", "--dim", "200000"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    assert rec["dist"]["world_size"] == 2 and [r["rank"] for r in rec["dist"]["ranks"]] == [0, 1]
    assert rec["combine_signed_split"]["passes"] == 2
    bad = subprocess.run(cmd, env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True,
                         text=True, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr
