#!/usr/bin/env python3
"""bench.py -- clerk share-combine throughput on MI355X (BASELINE.json metric), plus packed-Shamir
share-gen / reveal and ChaCha mask-combine side legs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Step = one exact clerk combine (combiner.rs:16-28) of this rank's 10,000 x 1,000,000 i64 share
matrix (BASELINE.json configs[1]), HBM-resident before timing starts.  With N > 1 ranks every rank
combines its own 10k x 1M block (weak scaling: participations shard across GPUs) and the per-rank
results are summed by one RCCL all-reduce over int64 (== u64 two's complement) and reduced on
device (sda_amd.distributed).  value = bytes combined by all ranks / max-over-ranks wall time.
Rank 0 prints ONE JSON line; everything else goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "clerk share-combine GB/s + packed-Shamir shares/s at 1M-dim, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0           # MI355X_MICROARCH.md: 8.0 TB/s spec
MODULUS = 2147482801             # m = p = 2147482801
SEED_BASE = 0x5DA


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, choices=[1, 3, 4], default=1,
                    help="1: configs[1] (10k x 1M per GPU, weak scaling); 3: configs[3] (100k x 10M in total, "
                         "split over the GPUs, streamed through a resident 1000-row tile); 4: configs[4]'s "
                         "recipient (100k ChaCha seeds x 10M-dim mask combine split over the GPUs + packed "
                         "reveal, unmask, positive)")
    ap.add_argument("--seeds", type=int, default=100_000, help="configs[4]: participant seeds in total")
    ap.add_argument("--rows", type=int, default=10_000, help="participations per GPU (configs[1]: 10k)")
    ap.add_argument("--dim", type=int, default=1_000_000, help="vector dimension (configs[1]: 1M)")
    ap.add_argument("--shamir-vectors", type=int, default=1000,
                    help="participant vectors per share-gen / reveal launch (BASELINE.md C3: P = 1,000)")
    ap.add_argument("--chacha-seeds", type=int, default=256)
    ap.add_argument("--no-side", action="store_true", help="skip packed-Shamir / ChaCha legs")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-path leg (sda_share_combine from host rows at the headline size)")
    ap.add_argument("--host-calls", type=int, default=2, help="timed sda_share_combine calls in the host-path leg")
    ap.add_argument("--no-multi-device", action="store_true",
                    help="skip the in-process multi-GPU leg (one engine handle over every visible GPU, N = 1 only)")
    ap.add_argument("--multi-device-leg", default=None, help=argparse.SUPPRESS)   # internal: the child's ordinals
    ap.add_argument("--no-signed-split", action="store_true",
                    help="N > 1: skip the signed-shares leg of the participation split (two-pass path)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-check", action="store_true", help="A/B helper: skip the side-leg round-trip checks")
    ap.add_argument("--codec-rows", type=int, default=1000, help="participations in the codec leg")
    ap.add_argument("--snapshot-participations", type=int, default=1000,
                    help="participations in the snapshot transposition leg")
    ap.add_argument("--pipeline-dim", type=int, default=10_000_000, help="vector dimension of the role pipelines")
    ap.add_argument("--only", choices=["combine", "shamir", "chacha", "codec", "snapshot", "pipelines"], default=None,
                    help="profile helper: run just one leg (no JSON contract)")
    return ap.parse_args()


class Timer:
    """HIP events on torch's current stream -- the stream every engine launch here is issued on."""

    def __init__(self, torch):
        self.torch = torch
        self.pairs = []

    def record(self, fn):
        s = self.torch.cuda.Event(enable_timing=True)
        e = self.torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        self.pairs.append((s, e))

    def mean_ms(self):
        self.torch.cuda.synchronize()
        return statistics.fmean(s.elapsed_time(e) for s, e in self.pairs)


def host_model():
    """The host the CPU baseline ran on: CPU model, the CPUs this process may use, and the thread
    budget (the GPU box exports OMP_NUM_THREADS = its CPU share per GPU)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity, "thread_budget": min(share, affinity)}


def cpu_baseline(dim: int, budget_s: float):
    """oracle/ C restatement of combiner.rs:16-28 (real `%` per element, -O2) on a bounded sample of
    the same synthetic matrix: (i) 1 core -- the reference is single-threaded; (ii) all the host
    cores this job may use, columns split over POSIX threads."""
    from oracle import oracle as O
    from sda_amd import synth
    host = host_model()
    threads = host["thread_budget"]

    def timed(rows, fn):
        x = synth.fill(rows, dim, SEED_BASE + 1, 0, MODULUS)
        times = []
        t_start = time.perf_counter()
        while (len(times) < 5 and (time.perf_counter() - t_start) < budget_s) or len(times) < 2:
            t0 = time.perf_counter()
            fn(x)
            times.append(time.perf_counter() - t0)
        return 8.0 * rows * dim / statistics.median(times) / 1e9, len(times)

    one, n1 = timed(100, lambda x: O.combine(MODULUS, x))
    allc, n2 = timed(400, lambda x: O.combine_mt(MODULUS, x, threads))
    return {"value": round(allc, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"400 x {dim:,} i64 rows of the headline matrix (uniform [0, m)), oracle/sda_oracle.c "
                      f"or_combine_mt at -O2 over {threads} threads (column split), median of {n2} runs",
            "single_core": {"value": round(one, 4), "unit": "GB/s", "cores": 1,
                            "sample": f"100 x {dim:,} rows, or_combine (the reference loop, 1 thread), "
                                      f"median of {n1} runs"},
            "shamir": cpu_baseline_shamir(threads, budget_s),
            "chacha": cpu_baseline_chacha(threads, budget_s),
            "host": host}


def _median_time(fn, budget_s, runs=3):
    """Median wall time of fn() over up to `runs` runs (at least 2) within about budget_s seconds."""
    times = []
    t_start = time.perf_counter()
    while (len(times) < runs and (time.perf_counter() - t_start) < budget_s) or len(times) < 2:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return statistics.median(times), len(times)


def _threaded(threads, jobs):
    """Run the oracle calls in `jobs` on `threads` host threads (ctypes releases the GIL in the C code)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for f in [ex.submit(j) for j in jobs]:
            f.result()


def cpu_baseline_shamir(threads: int, budget_s: float):
    """The second half of the metric on the host: oracle/sda_oracle.c's restatement of tss 0.2 share
    (packed_shamir.rs:40-43 via batched.rs:19-53) and reconstruct (packed_shamir.rs:73-77 via
    batched.rs:69-97) at configs[2]'s scheme, 1 core (the reference is single-threaded) and `threads`
    cores (one participant vector per thread)."""
    from oracle import oracle as O
    from sda_amd import schemes as S
    from sda_amd import synth
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    pp = O.packed_params(k, n, t, p, sch.omega_secrets, sch.omega_shares)
    Dg, Dr = 1_000_000, 250_000
    vecs = max(1, threads)
    sec = synth.fill(vecs, Dg, SEED_BASE + 2, 0, p)
    drw = synth.fill(vecs, (Dg // k) * t, SEED_BASE + 22, 0, p - 1)
    idx = list(range(n - (t + k), n))
    shares = [O.packed_generate(pp, sec[v, :Dr], drw[v, :(Dr // k) * t])[idx] for v in range(vecs)]
    g1, ng1 = _median_time(lambda: O.packed_generate(pp, sec[0], drw[0]), budget_s / 4)
    ga, nga = _median_time(lambda: _threaded(threads, [lambda v=v: O.packed_generate(pp, sec[v], drw[v])
                                                       for v in range(vecs)]), budget_s / 4)
    r1, nr1 = _median_time(lambda: O.packed_reconstruct(pp, Dr, idx, shares[0]), budget_s / 4)
    ra, nra = _median_time(lambda: _threaded(threads, [lambda v=v: O.packed_reconstruct(pp, Dr, idx, shares[v])
                                                       for v in range(vecs)]), budget_s / 4)
    B = Dg // k
    return {"unit": "shares/s (gen), secrets/s (reveal)", "kind": "port",
            "gen_shares_per_s": {"single_core": round(n * B / g1, 1), "all_cores": round(vecs * n * B / ga, 1),
                                 "cores": threads},
            "reveal_secrets_per_s": {"single_core": round(Dr / r1, 1), "all_cores": round(vecs * Dr / ra, 1),
                                     "cores": threads, "clerks": len(idx)},
            "sample": f"k=8 n=26 t=7 p={p}: share-gen of 1M-dim vectors (1 vector on 1 core, {vecs} on "
                      f"{threads} threads), exact reveal of 250k-dim vectors from {len(idx)} clerks; "
                      f"median of {ng1}/{nga}/{nr1}/{nra} runs; oracle/sda_oracle.c at -O2"}


def cpu_baseline_chacha(threads: int, budget_s: float):
    """chacha.rs:57-76 (MaskCombiner::combine) on the host: oracle/sda_oracle.c's rand-0.3 ChaChaRng +
    gen_range restatement, seeds over 1M-dim; 1 core, and `threads` cores (seeds split over threads; every
    draw is >= 0, so the per-thread canonical sums add exactly)."""
    from oracle import oracle as O
    D, per = 1_000_000, 2
    seeds = (np.arange(threads * per * 4, dtype=np.int64).reshape(-1, 4) * 7919 + 13) % (1 << 31)
    t1, n1 = _median_time(lambda: O.chacha_mask_combine(MODULUS, D, seeds[:per]), budget_s / 4)
    ta, na = _median_time(lambda: _threaded(threads, [lambda i=i: O.chacha_mask_combine(
        MODULUS, D, seeds[i * per:(i + 1) * per]) for i in range(threads)]), budget_s / 4)
    return {"unit": "mask elements/s", "kind": "port", "single_core": round(per * D / t1, 1),
            "all_cores": round(threads * per * D / ta, 1), "cores": threads,
            "sample": f"{per} seeds x 1M-dim on 1 core, {threads * per} on {threads} threads; median of {n1}/{na} "
                      "runs; oracle/sda_oracle.c at -O2"}


def multi_device_leg(args):
    """The drop-in boundary over every GPU of the node from ONE process (sda_engine_create_multi):
    runs in a child process (started before this one touches a GPU; killed after 150 s: a first cross-device RCCL run that hangs must not hold up the line) and returns its record,
    or None with one visible GPU.  SDA_BENCH_MULTI_DEVICES="0,0" rehearses it on one GPU (slices on one device)."""
    import subprocess
    forced = os.environ.get("SDA_BENCH_MULTI_DEVICES")
    if forced:
        devs = forced
    else:
        import torch
        n = torch.cuda.device_count()          # counts devices without initialising them
        if n < 2:
            return None
        devs = ",".join(str(i) for i in range(n))
    cmd = [sys.executable, os.path.abspath(__file__), "--multi-device-leg", devs, "--rows", str(args.rows),
           "--dim", str(args.dim)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=150)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 150 s", "devices": devs}
    sys.stderr.write(r.stderr[-4000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}: {r.stderr.strip().splitlines()[-1] if r.stderr.strip() else ''}",
                "devices": devs}
    return json.loads(lines[-1])


def multi_device_child(args):
    """multi_device_leg's process: one engine handle over the given ordinals.
    (1) ShareCombiner::combine (clerk.rs:85-86) over the headline job's N x D i64 rows in host memory: the
        handle streams a column slice per GPU; timed against a one-GPU handle on the same rows, bit-exact.
    (2) MaskCombiner::combine (chacha.rs:57-76) of 2048 ChaCha seeds over a 10M-dim mask: seeds split over the
        GPUs and one RCCL ncclReduce (int64) over xGMI; bit-exact against the one-GPU handle."""
    import torch
    from sda_amd import Engine, schemes as S
    devs = [int(x) for x in args.multi_device_leg.split(",")]
    N, D, m = args.rows, args.dim, MODULUS
    one = Engine(devs[0])
    eng = Engine(devices=devs)
    dev = torch.device("cuda", devs[0])
    host = torch.empty((N, D), dtype=torch.int64)
    tile = max(1, min(N, (8 << 30) // (8 * D)))
    t = torch.empty((tile, D), dtype=torch.int64, device=dev)
    for r0 in range(0, N, tile):
        r = min(tile, N - r0)
        one.synth_fill_dev(t.data_ptr(), r, D, SEED_BASE + 1 + r0, -(m - 1), m, torch.cuda.current_stream().cuda_stream)
        host[r0:r0 + r].copy_(t[:r])
    del t
    torch.cuda.synchronize()
    hn = host.numpy()
    rows = [hn[i] for i in range(N)]
    sch = S.Additive(3, m)

    def timed(e, calls=2):
        ts, res = [], None
        for i in range(1 + calls):
            t0 = time.perf_counter()
            res = e.share_combine(sch, rows)
            if i:
                ts.append(time.perf_counter() - t0)
        return statistics.median(ts), res
    t1, r1 = timed(one)
    tg, rg = timed(eng)
    ok = bool(np.array_equal(r1, rg))
    Dc, Ns = 10_000_000, 2048
    seeds = [list(map(int, row)) for row in np.random.default_rng(SEED_BASE + 5).integers(0, 1 << 32, size=(Ns, 4))]
    ms = S.ChaChaMasking(m, Dc, 128)
    def timed_mask(e, calls=3):                    # one warm call, then the median of `calls`
        ts, res = [], e.mask_combine(ms, seeds)
        for _ in range(calls):
            t0 = time.perf_counter()
            res = e.mask_combine(ms, seeds)
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts), res
    tc1, c1 = timed_mask(one)
    tcg, cg = timed_mask(eng)
    okc = bool(np.array_equal(c1, cg))
    rec = {"devices": devs, "device_count": eng.device_count(),
           "share_combine": {"config": f"{N:,} host rows x {D:,} i64, signed (the headline job from host memory)",
                             "one_gpu_s": round(t1, 3), "one_gpu_GBps": round(8.0 * N * D / t1 / 1e9, 2),
                             "all_gpus_s": round(tg, 3), "all_gpus_GBps": round(8.0 * N * D / tg / 1e9, 2),
                             "split": "columns", "bit_exact_vs_one_gpu": ok},
           "chacha_mask_combine": {"config": f"{Ns} seeds x {Dc:,}-dim (host call)",
                                   "one_gpu_s": round(tc1, 4), "all_gpus_s": round(tcg, 4),
                                   "all_gpus_mask_elems_per_s": Ns * Dc / tcg,
                                   "split": "seeds + RCCL ncclReduce int64 onto ordinals[0]", "bit_exact_vs_one_gpu": okc}}
    print(json.dumps(rec), flush=True)
    if not (ok and okc):
        sys.exit(3)


def host_path_leg(args, torch, eng, shares, N, D, m, dev, st):
    """The drop-in boundary at the headline size: ShareCombiner::combine (clerk.rs:85-86 -> combiner.rs:16-28)
    through the HOST entry point the Rust shim calls, sda_share_combine, over the same N x D i64 rows held in
    host memory as N separate row buffers (a Vec<Vec<i64>>).  The engine streams them through pinned double
    buffers in row tiles (engine.cpp, host path), so the call is bound by the host -> device link; the leg
    reports it beside the measured pinned and pageable H2D rates of the same box.  Bit-exact check: the call's
    result equals the device-resident combine of the same rows (the buffer holds the signed leg's rows by now)."""
    from sda_amd import schemes as S
    dev_out = torch.empty(D, dtype=torch.int64, device=dev)
    eng.combine_dev(m, shares.data_ptr(), N, D, D, dev_out.data_ptr(), st)
    t0 = time.perf_counter()
    host = torch.empty((N, D), dtype=torch.int64)          # pageable host memory, like the Rust Vecs
    host.copy_(shares)
    torch.cuda.synchronize()
    fill_s = time.perf_counter() - t0
    hn = host.numpy()
    rows = [hn[i] for i in range(N)]
    sch = S.Additive(3, m)
    times = []
    got = None
    for i in range(1 + max(1, args.host_calls)):
        t0 = time.perf_counter()
        got = eng.share_combine(sch, rows)
        if i:
            times.append(time.perf_counter() - t0)
    ok = bool(np.array_equal(got, dev_out.cpu().numpy()))
    if not ok:
        raise SystemExit("host-path combine check FAILED")
    # the link's own rates on this box: 1 GiB pinned and pageable host buffers -> HBM
    def h2d(pinned):
        src = torch.empty(1 << 27, dtype=torch.int64, pin_memory=pinned)
        src.fill_(1)
        dst = torch.empty(1 << 27, dtype=torch.int64, device=dev)
        dst.copy_(src, non_blocking=pinned)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=pinned)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return 8.0 * (1 << 27) / statistics.median(ts) / 1e9
    pinned_gbps, pageable_gbps = h2d(True), h2d(False)
    t = statistics.median(times)
    gbps = 8.0 * N * D / t / 1e9
    del host, hn, rows
    return {"config": f"sda_share_combine (host entry point) over {N:,} host rows x {D:,} i64"
                      + (" (the headline job)" if D == 1_000_000 else " (configs[3]'s resident tile)"),
            "ms_per_call": round(t * 1e3, 1), "GBps": round(gbps, 2), "calls": len(times),
            "h2d_pinned_GBps": round(pinned_gbps, 2), "h2d_pageable_GBps": round(pageable_gbps, 2),
            "frac_of_pinned_h2d": round(gbps / pinned_gbps, 4),
            "stage_mb": int(os.environ.get("SDA_HOST_STAGE_MB", "256")),
            "host_threads": int(os.environ.get("SDA_HOST_THREADS", "0")) or min(os.cpu_count() or 1, 16),
            "host_fill_s": round(fill_s, 2),
            "check": "bit-exact: equals the device-resident combine of the same rows, all columns"}


class TimedEngine:
    """Wraps the engine for sda_amd.distributed: HIP events around every combine launch, on the
    stream the launch is issued on (the kernel's own duration for the roofline)."""

    def __init__(self, eng, timer):
        self.eng, self.timer = eng, timer
        self.timing = False

    def __getattr__(self, name):
        return getattr(self.eng, name)

    def _timed(self, fn, *a):
        if self.timing:
            self.timer.record(lambda: fn(*a))
        else:
            fn(*a)

    def combine_dev(self, *a):
        self._timed(self.eng.combine_dev, *a)

    def combine_accumulate_dev(self, *a):
        self._timed(self.eng.combine_accumulate_dev, *a)

    def combine_split_dev(self, *a):            # pass 1 of the participation split (N > 1)
        self._timed(self.eng.combine_split_dev, *a)


def exact_sample_check(torch, shares, cols, m, got, reps=1, rows=None):
    """Bit-exact check of combiner.rs:22-25 on sampled columns: the sequential recurrence
    r = (r + v) % m (np.fmod = Rust's truncated %) replayed on the host over the rows in order
    (`reps` passes over the resident tile for the tiled workload, then its first `rows` rows)."""
    xs = shares[:, cols].cpu().numpy()
    r = np.zeros(xs.shape[1], dtype=np.int64)
    for _ in range(reps):
        for i in range(xs.shape[0]):
            r = np.fmod(r + xs[i], m)
    for i in range(rows or 0):
        r = np.fmod(r + xs[i], m)
    return bool((r == got[cols].cpu().numpy()).all())


def spawn_ranks(n: int) -> int:
    """`--gpus N` (N > 1) started without a launcher: start N ranks of this same command, one per GPU
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them), wait for all of them
    and return the first failing exit code (0 if all passed).  Rank 0 prints the JSON line to the
    inherited stdout.  Runs before this process touches the GPU (only the device COUNT is read, which
    does not initialise it), so the ranks own their devices."""
    import signal
    import socket
    import subprocess
    if os.environ.get("SDA_DIST_BACKEND", "nccl") == "nccl":
        import torch
        have = torch.cuda.device_count()
        if have < n:
            log(f"bench.py: --gpus {n} needs {n} GPUs, {have} visible (SDA_DIST_BACKEND=gloo rehearses "
                f"N ranks on fewer devices)")
            return 2
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks")
                for q in alive:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def main():
    args = parse()
    if args.multi_device_leg is not None:
        multi_device_child(args)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    multi = None
    if (os.environ.get("WORLD_SIZE", "1") == "1" and args.only is None and args.config == 1 and not args.no_multi_device
            and not args.no_host_path):
        multi = multi_device_leg(args)         # before this process touches a GPU (a child process of its own)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch with --nproc-per-node equal to --gpus")
        sys.exit(2)

    import torch
    import torch.distributed as dist

    from sda_amd import Engine, schemes as S
    from sda_amd import distributed as Dd
    from sda_amd import engine as E
    # one rank per GPU; SDA_DIST_BACKEND=gloo rehearses N ranks on fewer devices (RCCL refuses two
    # ranks on one device): ranks then share GPUs round-robin, and the collectives run over gloo
    backend = os.environ.get("SDA_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    eng = Engine(local)
    stream = lambda: torch.cuda.current_stream().cuda_stream   # noqa: E731
    dev = torch.device("cuda", local)

    def barrier():
        if world > 1:
            dist.barrier()

    # The side legs' resident buffers come from sda_hbm_alloc: one virtual range over fixed-size physical
    # chunks, so share-gen's rate does not depend on how fragmented the box's free VRAM is (DESIGN.md "HBM
    # backing", profiles/r04t, r04u).  SDA_BENCH_ALLOC=torch switches back to torch's allocator (A/B).
    alloc_kind = "torch" if os.environ.get("SDA_BENCH_ALLOC", "hbm") == "torch" else "hbm"

    def hbm(shape, dtype=torch.int64):
        if alloc_kind == "torch":
            return torch.empty(shape, dtype=dtype, device=dev)
        return eng.hbm_empty(shape if isinstance(shape, tuple) else (shape,), dtype)

    if args.config == 4:
        run_config4(args, torch, dist, eng, dev, stream, barrier, world, rank, backend)
        if world > 1:
            dist.destroy_process_group()
        return

    # ---------------- workload: configs[1] (or configs[3]), HBM-resident ----------------
    N, D, m = args.rows, args.dim, MODULUS
    tile = 0
    value = achieved = kernel_ms = dt = 0.0
    if args.config == 3:
        # configs[3]: 100k participations x 10M-dim, participations split over the ranks; 8 TB do not
        # fit, so each rank streams its share through one resident 1000 x 10M tile (80 GB) with the
        # accumulating combine (bit-identical to one pass over the rows).
        D, total = 10_000_000, 100_000
        N = (total + world - 1) // world
        tile = 1000
    run_combine = args.only in (None, "combine")
    side = {}
    if run_combine:
        R = tile if tile else N
        # torch.empty (one hipMalloc) here: the combine ran 1.5 % faster on it than on sda_hbm_alloc's chunks
        # (12.80 vs 12.98 ms, 4 interleaved rounds, profiles/r04w), the reverse of share-gen
        shares = torch.empty((R, D), dtype=torch.int64, device=dev)
        eng.synth_fill_dev(shares.data_ptr(), R, D, SEED_BASE + 1 + 1000 * rank, 0, m, stream())
        partial = torch.empty(D, dtype=torch.int64, device=dev)
        out = torch.empty(D, dtype=torch.int64, device=dev)
        ktimer = Timer(torch)
        teng = TimedEngine(eng, ktimer)
        # the product's multi-GPU path (sda_amd.distributed): per-rank exact combine of this rank's
        # participations (row tiles for configs[3]), one int64 all-reduce over RCCL, device finalize
        tiles = [(shares.data_ptr(), min(tile, N - t0)) for t0 in range(0, N, tile)] if tile else None

        # N > 1: each step's sign flags come back asynchronously (SplitTicket); a step finishes the
        # PREVIOUS step's ticket after queueing its own work, so no host read sits between a step's
        # all-reduce and its finalize, and the GPU never waits for the host
        # (two `out` buffers, alternating: a ticket in flight never shares its `out` with the next step's)
        pending = []
        outs = [out, torch.empty(D, dtype=torch.int64, device=dev)]
        nstep = [0]

        def step(timed):
            nonlocal out
            teng.timing = timed
            out = outs[nstep[0] % 2]
            nstep[0] += 1
            if tile:
                t = Dd.combine_tiles_sharded(teng, m, tiles, D, D, partial, out, defer=True)
            else:
                t = Dd.combine_rows_sharded(teng, m, shares.data_ptr(), N, D, D, partial, out, defer=True)
            while pending:
                pending.pop().finish()
            if t is not None:
                pending.append(t)

        for _ in range(args.warmup):
            step(False)
        while pending:
            pending.pop().finish()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(True)
        while pending:
            pending.pop().finish()
        torch.cuda.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        kernel_ms = ktimer.mean_ms()
        # check the last step's result on 4096 sampled columns
        cols = torch.randint(0, D, (4096,), device=dev, generator=torch.Generator(device=dev).manual_seed(7))
        if args.no_check:
            ok = True
        elif world == 1:     # bit-exact: the sequential recurrence replayed on the host
            ok = exact_sample_check(torch, shares, cols, m, out, reps=(N // tile) if tile else 1,
                                    rows=(N % tile) if tile else 0)
        else:                # non-negative inputs: (sum over ranks of column sums) mod m
            ref = (N // tile) * shares[:, cols].sum(dim=0) + shares[: N % tile, cols].sum(dim=0) if tile \
                else shares[:, cols].sum(dim=0)
            dist.all_reduce(ref, op=dist.ReduceOp.SUM)
            ok = torch.equal(torch.remainder(ref, m), out[cols])
        if not ok:
            raise SystemExit("combine result check FAILED")
        rows_per_launch = tile if tile else N
        # one launch reads its rows and writes D results; an accumulating launch (row tiles, and the
        # participation split's pass 1 at N > 1) also reads the running partial (16 D).  `value` counts
        # the job's own bytes only: N x D shares in, D out.
        bytes_per_launch = 8.0 * rows_per_launch * D + (16.0 if (tile or world > 1) else 8.0) * D
        total_bytes = (8.0 * N * D + 8.0 * D) * args.steps * world
        value = total_bytes / dt / 1e9
        achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
        log(f"[combine] rank {rank}: {args.steps} steps in {dt*1e3:.1f} ms, kernel {kernel_ms:.3f} ms "
            f"({achieved:.0f} GB/s per launch)")

        # the signed worst case -- uniform (-m, m) shares, whose exact result is
        # order dependent -- through the same kernel on the same resident buffer
        if not args.no_side and world == 1 and not tile:
            eng.synth_fill_dev(shares.data_ptr(), N, D, SEED_BASE + 12, -(m - 1), m, stream())
            st = Timer(torch)
            sg = lambda: eng.combine_dev(m, shares.data_ptr(), N, D, D, partial.data_ptr(), stream())  # noqa
            for i in range(1 + max(3, args.steps // 4)):
                st.record(sg) if i else sg()
            s_ms = st.mean_ms()
            if not args.no_check and not exact_sample_check(torch, shares, cols, m, partial):
                raise SystemExit("signed combine result check FAILED")
            side["combine_signed"] = {
                "config": "configs[1] with uniform (-m, m) shares (SURVEY 8(d) C2(ii)), exact signed result",
                "kernel_ms": s_ms, "GBps": bytes_per_launch / (s_ms * 1e-3) / 1e9,
                "roofline_frac": bytes_per_launch / (s_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                "check": "bit-exact on 4096 sampled columns (sequential recurrence replayed on the host)"}
            log(f"[combine_signed] {json.dumps(side['combine_signed'])}")
        if not args.no_signed_split and world > 1 and not tile:
            # the same signed worst case through the participation split at N > 1: the exact two-pass
            # path (pass 1 + flags, all-gather, replay of the sign events, MAX-resolve)
            eng.synth_fill_dev(shares.data_ptr(), N, D, SEED_BASE + 12 + 1000 * rank, -(m - 1), m, stream())
            sst = Dd.SplitStats()
            sstep = lambda: Dd.combine_rows_sharded(eng, m, shares.data_ptr(), N, D, D, partial, out, stats=sst)  # noqa
            sstep()
            torch.cuda.synchronize()
            barrier()
            reps = max(3, args.steps // 4)
            ts = time.perf_counter()
            for _ in range(reps):
                sstep()
            torch.cuda.synchronize()
            barrier()
            tt = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            s_dt = float(tt.item()) / reps
            ok = True
            if not args.no_check:     # replay the reference recurrence over all ranks' rows, in rank order
                c256 = cols[:256]
                mine = shares[:, c256].contiguous()
                allr = [torch.empty_like(mine) for _ in range(world)]
                dist.all_gather(allr, mine)
                r = np.zeros(256, dtype=np.int64)
                for blk in allr:
                    for row in blk.cpu().numpy():
                        r = np.fmod(r + row, m)
                ok = bool((r == out[c256].cpu().numpy()).all()) and sst.signed
            if not ok:
                raise SystemExit("signed participation split check FAILED")
            side["combine_signed_split"] = {
                "config": f"configs[1] with uniform (-m, m) shares on each of {world} ranks: exact participation "
                          "split of a signed job (two passes over the rows, all-gather + MAX all-reduce)",
                "ms_per_step": s_dt * 1e3, "GBps_all_gpus": 8.0 * (N * D + D) * world / s_dt / 1e9,
                "passes": sst.passes,
                "check": "bit-exact on 256 sampled columns: the reference recurrence over all ranks' rows in order"}
            log(f"[combine_signed_split] {json.dumps(side['combine_signed_split'])}")
        if not args.no_host_path and world == 1 and args.only is None:
            # configs[1]: the whole job from host rows.  configs[3]: the resident 1000-row tile from host rows
            # (80 GB), and the PCIe-inclusive time of this GPU's whole share projected at that rate (SURVEY
            # §8(d) C4: report kernel-only and end-to-end separately)
            R = tile if tile else N
            side["host_path"] = host_path_leg(args, torch, eng, shares, R, D, m, dev, stream())
            if tile:
                job = 8.0 * N * D
                side["host_path"]["job_bytes_per_gpu"] = job
                side["host_path"]["projected_job_s_host_path"] = round(job / (side["host_path"]["GBps"] * 1e9), 2)
                side["host_path"]["job_s_hbm_resident"] = round(dt / args.steps, 3)
            log(f"[host_path] {json.dumps(side['host_path'])}")
        del shares
        torch.cuda.empty_cache()         # the next leg gets fresh allocations, not a reused segment

    # ---------------- side legs (rank-local, reported by rank 0) ----------------
    if not args.no_side and args.only in (None, "shamir"):
        sch = S.CONFIG_PACKED
        p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
        V, Dm = args.shamir_vectors, 1_000_000
        B = Dm // k
        sec = hbm((V, Dm))
        eng.synth_fill_dev(sec.data_ptr(), V, Dm, SEED_BASE + 2, 0, p, stream())
        drw = hbm((V, B, t))
        eng.synth_fill_dev(drw.data_ptr(), V * B, t, SEED_BASE + 22, 0, p - 1, stream())
        sh = hbm((V, n, B))
        idx = list(range(n - (t + k), n))           # a t+k clerk subset (result_ready threshold)
        sub = hbm((V, len(idx), B))
        rev = hbm((V, Dm))
        gen_t, rex_t, rca_t, gca_t = Timer(torch), Timer(torch), Timer(torch), Timer(torch)
        # canonical-mode share-gen first (its shares are overwritten by the exact ones below)
        genc = lambda: eng.packed_generate_mode_dev(sch, sec.data_ptr(), Dm, V, drw.data_ptr(), sh.data_ptr(),  # noqa
                                                    E.REVEAL_CANONICAL, stream())
        for i in range(args.warmup + args.steps):
            gca_t.record(genc) if i >= args.warmup else genc()
        torch.cuda.synchronize()
        if not args.no_check:     # canonical shares: in [0, p) and a canonical reveal returns the secrets
            sub0 = sh[:, n - (t + k):, :].contiguous()
            rv = torch.empty((V, Dm), dtype=torch.int64, device=dev)
            eng.packed_reconstruct_dev(sch, Dm, list(range(n - (t + k), n)), V, sub0.data_ptr(), rv.data_ptr(),
                                       E.REVEAL_CANONICAL, stream())
            torch.cuda.synchronize()
            if int(sh.min()) < 0 or not torch.equal(rv, sec):
                raise SystemExit("canonical share-gen round trip FAILED")
            del sub0, rv
        gen = lambda: eng.packed_generate_dev(sch, sec.data_ptr(), Dm, V, drw.data_ptr(), sh.data_ptr(), stream())  # noqa
        for i in range(args.warmup + args.steps):
            gen_t.record(gen) if i >= args.warmup else gen()
        sub.copy_(sh[:, idx, :])
        for mode, tm in ((E.REVEAL_EXACT, rex_t), (E.REVEAL_CANONICAL, rca_t)):
            f = lambda: eng.packed_reconstruct_dev(sch, Dm, idx, V, sub.data_ptr(), rev.data_ptr(), mode, stream())  # noqa
            for i in range(args.warmup + args.steps):
                tm.record(f) if i >= args.warmup else f()
            torch.cuda.synchronize()
            if not args.no_check and not torch.equal(torch.remainder(rev, p), sec):
                raise SystemExit(f"packed reveal round-trip FAILED (mode {mode})")
        g_ms, x_ms, c_ms, gc_ms = gen_t.mean_ms(), rex_t.mean_ms(), rca_t.mean_ms(), gca_t.mean_ms()
        gen_bytes = 8.0 * V * (Dm + t * B + n * B)
        rev_bytes = 8.0 * V * (len(idx) * B + Dm)
        side["shamir"] = {
            "config": "PackedShamir k=8 n=26 t=7 p=2147482801, 1M-dim, %d vectors/launch" % V,
            "buffers": alloc_kind,
            "shares_per_s": V * n * B / (g_ms * 1e-3),
            "gen_ms": g_ms, "gen_GBps": gen_bytes / (g_ms * 1e-3) / 1e9,
            "gen_roofline_frac": gen_bytes / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "gen_canonical_ms": gc_ms, "gen_canonical_GBps": gen_bytes / (gc_ms * 1e-3) / 1e9,
            "gen_canonical_roofline_frac": gen_bytes / (gc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "reveal_exact_ms": x_ms, "reveal_exact_GBps": rev_bytes / (x_ms * 1e-3) / 1e9,
            "reveal_canonical_ms": c_ms, "reveal_canonical_GBps": rev_bytes / (c_ms * 1e-3) / 1e9,
            "reveal_clerks": len(idx),
        }
        waves = V * ((B + 255) // 256) * 4              # 256-lane workgroups (L = 16 share-gen and reveal)
        for key, ms in (("gen_exact", g_ms), ("gen_canonical", gc_ms), ("reveal_exact", x_ms),
                        ("reveal_canonical", c_ms)):
            r = valu_roofline(key, ms, waves)
            if r:
                side["shamir"][key + "_valu"] = r
        ex = side["shamir"].get("gen_exact_valu")
        if ex:      # integer-op throughput of share-gen (north star: "integer-op throughput in rocprof")
            side["shamir"]["int_ops_per_s"] = ex["achieved"] * 1e12
        if world > 1:
            # "packed-Shamir shares/s at 1/2/4/8 GPUs": every rank generates its own participants'
            # shares at once (vector split, no collective); whole-job rate over the max-over-ranks time
            torch.cuda.synchronize()
            barrier()
            t_all = time.perf_counter()
            for _ in range(args.steps):
                gen()
            torch.cuda.synchronize()
            barrier()
            tt = torch.tensor([time.perf_counter() - t_all], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            side["shamir"]["shares_per_s_all_gpus"] = world * V * n * B * args.steps / float(tt.item())
            side["shamir"]["n_gpus"] = world
        log(f"[shamir] {json.dumps(side['shamir'])}")
        del sec, drw, sh, sub, rev
        torch.cuda.empty_cache()         # the next leg gets fresh allocations, not a reused segment
    if not args.no_side and args.only in (None, "chacha"):
        Dc, Ns = 1_000_000, args.chacha_seeds
        seeds = torch.randint(0, 2**31 - 1, (Ns, 4), dtype=torch.int32, device=dev,
                              generator=torch.Generator(device=dev).manual_seed(SEED_BASE + 5))
        cout = torch.empty(Dc, dtype=torch.int64, device=dev)
        ct = Timer(torch)
        f = lambda: eng.chacha_mask_combine_dev(m, Dc, seeds.data_ptr(), 4, Ns, cout.data_ptr(), stream())  # noqa
        for i in range(2 + max(2, args.steps // 4)):
            ct.record(f) if i >= 2 else f()
        c_ms = ct.mean_ms()
        side["chacha"] = {"config": f"ChaCha mask combine, {Ns} seeds x 1M-dim", "ms": c_ms,
                          "mask_elems_per_s": Ns * Dc / (c_ms * 1e-3),
                          "chacha_blocks_per_s": Ns * Dc / 8 / (c_ms * 1e-3)}
        r = valu_roofline("chacha_combine", c_ms, None)
        if r:
            side["chacha"]["roofline"] = r
        log(f"[chacha] {json.dumps(side['chacha'])}")

    if not args.no_side and args.only in (None, "codec"):
        # clerk payload path (clerk.rs:79-86 after the sealed-box opens): varint payloads of
        # signed field shares -> decode -> exact combine; plus the encode of the same matrix.
        Nc, Dc = args.codec_rows, 1_000_000
        x = hbm((Nc, Dc))
        eng.synth_fill_dev(x.data_ptr(), Nc, Dc, SEED_BASE + 6, -(m - 1), m, stream())
        cap = Nc * Dc * 6 + 32                          # |v| < 2^31 -> zigzag < 2^32 -> <= 5 bytes
        buf = hbm(cap, torch.uint8)
        buf.zero_()
        et, dt_, ct = Timer(torch), Timer(torch), Timer(torch)
        rb = None
        for i in range(3):
            f = lambda: eng.varint_encode_dev(x.data_ptr(), Nc, Dc, Dc, buf.data_ptr(), cap, stream())  # noqa
            if i:
                et.record(f)
            else:
                rb = f()
        rb = eng.varint_encode_dev(x.data_ptr(), Nc, Dc, Dc, buf.data_ptr(), cap, stream())
        off = np.concatenate([[0], np.cumsum(rb)]).astype(np.uint64)
        payload = float(off[-1])
        mat = hbm((Nc, Dc))
        cout = torch.empty(Dc, dtype=torch.int64, device=dev)
        for i in range(4):
            f = lambda: eng.varint_decode_dev(buf.data_ptr(), off, mat.data_ptr(), Dc, stream())  # noqa
            dt_.record(f) if i else f()
        for i in range(4):
            f = lambda: eng.clerk_decode_combine_dev(m, buf.data_ptr(), off, cout.data_ptr(), Dc, stream())  # noqa
            ct.record(f) if i else f()
        # the other two exact paths, timed beside the default (SDA_CODEC_PATH knob): the count pass + dense
        # int32 matrix + combine (round 2's default), and the fused column-tile decode+combine (opt-in)
        alt = {}
        cout_m = torch.empty(Dc, dtype=torch.int64, device=dev)
        prev = os.environ.get("SDA_CODEC_PATH")
        for pname in ("matrix", "fused"):
            alt[pname] = Timer(torch)
            os.environ["SDA_CODEC_PATH"] = pname
            try:
                for i in range(4):
                    f = lambda: eng.clerk_decode_combine_dev(m, buf.data_ptr(), off, cout_m.data_ptr(), Dc, stream())  # noqa
                    alt[pname].record(f) if i else f()
            finally:
                if prev is None:
                    del os.environ["SDA_CODEC_PATH"]
                else:
                    os.environ["SDA_CODEC_PATH"] = prev
            torch.cuda.synchronize()
            if not args.no_check and not torch.equal(cout, cout_m):
                raise SystemExit(f"codec {pname} vs default decode+combine FAILED")
        torch.cuda.synchronize()
        if not args.no_check:
            if not torch.equal(mat, x):
                raise SystemExit("codec round trip FAILED")
            # size-independent property of the exact combine: r in (-m, m), r == column sum (mod m)
            cols = torch.randint(0, Dc, (4096,), device=dev)
            r = cout[cols]
            if not (torch.equal(torch.remainder(r, m), torch.remainder(x[:, cols].sum(0), m))
                    and bool((r.abs() < m).all())):
                raise SystemExit("codec decode+combine FAILED")
        # the clerk's HOST entry point over the same payloads (the Rust shim's call after the sealed-box opens):
        # the payload bytes cross PCIe, the decode and combine run on device (engine.cpp host_decode_combine)
        host_dc = None
        if not args.no_host_path and world == 1:
            from sda_amd import schemes as S_
            hpay = buf[:int(payload) + 32].cpu().numpy()
            hts = []
            for i in range(3):
                t0 = time.perf_counter()
                hres = eng.clerk_decode_combine_packed(S_.Additive(3, m), hpay, off)
                if i:
                    hts.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            if not args.no_check and not np.array_equal(hres, cout.cpu().numpy()):
                raise SystemExit("host decode+combine FAILED")
            ht = statistics.median(hts)
            host_dc = {"ms_per_call": round(ht * 1e3, 1), "payload_GBps": round(payload / ht / 1e9, 2),
                       "shares_per_s": Nc * Dc / ht,
                       "note": "sda_clerk_decode_combine from host memory: payload over PCIe (4.94 B/share instead "
                               "of 8 for decoded rows), decoded + combined on device; equals the device path"}
            del hpay
        e_ms, d_ms, c_ms = et.mean_ms(), dt_.mean_ms(), ct.mean_ms()
        mx_ms, cm_ms = alt["matrix"].mean_ms(), alt["fused"].mean_ms()
        default_path = os.environ.get("SDA_CODEC_PATH", "slots")
        side["codec"] = {
            "config": f"varint payloads of {Nc} participations x 1M-dim signed field shares "
                      f"({payload / Nc / Dc:.2f} B/share)",
            "payload_bytes": payload,
            "decode_ms": d_ms, "decode_payload_GBps": payload / (d_ms * 1e-3) / 1e9,
            "decode_hbm_GBps": (payload + 8.0 * Nc * Dc) / (d_ms * 1e-3) / 1e9,
            "decode_combine_ms": c_ms, "decode_combine_shares_per_s": Nc * Dc / (c_ms * 1e-3),
            "decode_combine_payload_GBps": payload / (c_ms * 1e-3) / 1e9,
            "decode_combine_roofline_frac": (payload + 8.0 * Dc) / (c_ms * 1e-3) / 8.0e12,
            # bytes the default path moves: payload read once, int32 slots written and read back, the i64
            # result written (the matrix path reads the payload twice: count pass + decode)
            "decode_combine_hbm_GBps": ((payload if default_path == "slots" else 2 * payload) + 8.0 * Nc * Dc
                                        + 8.0 * Dc) / (c_ms * 1e-3) / 1e9,
            "decode_combine_path": {"slots": "decode once into int32 slots per 16 KiB region, exact combine over "
                                             "the slots", "matrix": "count pass, decode to an int32 matrix, exact "
                                             "combine", "fused": "count pass, fused column-tile decode+combine"
                                    }.get(default_path, default_path),
            "buffers": alloc_kind + " (payload, matrix); engine scratch (slots): "
                       + ("sda_hbm_alloc chunks" if os.environ.get("SDA_SCRATCH_HBM") == "1" else "hipMalloc"),
            "decode_combine_matrix_ms": mx_ms,
            "decode_combine_fused_ms": cm_ms,
            "encode_ms": e_ms, "encode_hbm_GBps": (payload + 8.0 * Nc * Dc) / (e_ms * 1e-3) / 1e9,
            **({"host_decode_combine": host_dc} if host_dc else {}),
        }
        log(f"[codec] {json.dumps(side['codec'])}")
        del x, buf, mat
        torch.cuda.empty_cache()         # the next leg gets fresh allocations, not a reused segment

    if not args.no_side and args.only in (None, "snapshot"):
        # server side (stores.rs:86-101): a snapshot of Ps participations x 26 clerk payloads of
        # packed-Shamir 1M-dim shares (B = 125,000 varint shares, ~4.94 B each -> ~617 KB per payload,
        # ragged) regrouped into 26 clerking jobs.  Algorithmic bytes = read + write of every payload.
        Ps, ncl = args.snapshot_participations, 26
        g = np.random.default_rng(SEED_BASE + 11)
        lens = g.integers(600_000, 635_000, size=Ps * ncl)
        poff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        total = int(poff[-1])
        src = hbm(total + 32, torch.uint8)
        eng.synth_fill_dev(src.data_ptr(), 1, (total + 32) // 8, SEED_BASE + 11, -(2**61), 2**61, stream())
        need, _, _ = eng.snapshot_transpose_dev(src.data_ptr(), poff, Ps, ncl)
        dst = hbm(need, torch.uint8)
        stt = Timer(torch)
        for i in range(2 + max(2, args.steps // 4)):
            f = lambda: eng.snapshot_transpose_dev(src.data_ptr(), poff, Ps, ncl, dst.data_ptr(), need, stream())  # noqa
            stt.record(f) if i >= 2 else f()
        _, base, coff = eng.snapshot_transpose_dev(src.data_ptr(), poff, Ps, ncl, None, 0)
        torch.cuda.synchronize()
        if not args.no_check:
            for c, pp in ((0, 0), (7, Ps // 3), (ncl - 1, Ps - 1), (13, Ps // 2)):
                b = pp * ncl + c
                lo = int(base[c] + coff[c, pp])
                if not torch.equal(dst[lo:lo + int(lens[b])], src[int(poff[b]):int(poff[b + 1])]):
                    raise SystemExit("snapshot transposition FAILED")
        s_ms = stt.mean_ms()
        cpt = Timer(torch)                               # same-size device-to-device copy: the copy ceiling
        for i in range(4):
            f = lambda: dst[:total].copy_(src[:total])  # noqa
            cpt.record(f) if i else f()
        cp_ms = cpt.mean_ms()
        side["snapshot"] = {
            "config": f"{Ps} participations x {ncl} clerk payloads of ~617 KB (ragged), {total / 1e9:.2f} GB",
            "ms": s_ms, "payload_GBps": total / (s_ms * 1e-3) / 1e9,
            "hbm_GBps": 2.0 * total / (s_ms * 1e-3) / 1e9,
            "roofline_frac": 2.0 * total / (s_ms * 1e-3) / 8.0e12,
            "d2d_copy_ms": cp_ms, "d2d_copy_hbm_GBps": 2.0 * total / (cp_ms * 1e-3) / 1e9, "buffers": alloc_kind,
            "note": "call time (host plan of one entry per blob + upload + kernel), HIP events",
        }
        log(f"[snapshot] {json.dumps(side['snapshot'])}")
        del src, dst
        torch.cuda.empty_cache()         # the next leg gets fresh allocations, not a reused segment

    if not args.no_side and args.only in (None, "pipelines"):
        # configs[4] per GPU: participant = ChaCha mask -> packed share-gen -> per-clerk payload encoding
        # (participate.rs:53-76); recipient = ChaCha mask combine over Ns seeds -> exact reveal from t+k
        # clerks -> unmask + positive (receive.rs:80-157).  One participant round trip is checked.
        sch = S.CONFIG_PACKED
        p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
        Dp = args.pipeline_dim
        B = (Dp + k - 1) // k
        msk = S.ChaChaMasking(p, Dp, 128)
        sec = torch.empty(Dp, dtype=torch.int64, device=dev)
        eng.synth_fill_dev(sec.data_ptr(), 1, Dp, SEED_BASE + 8, 0, 1 << 20, stream())
        drw = torch.empty((B, t), dtype=torch.int64, device=dev)
        eng.synth_fill_dev(drw.data_ptr(), B, t, SEED_BASE + 9, 0, p - 1, stream())
        sh = torch.empty((n, B), dtype=torch.int64, device=dev)
        cap = n * B * 6 + 32
        pay = torch.zeros(cap, dtype=torch.uint8, device=dev)
        seed = [0x5DA, 1, 2, 3]
        pt, rt = Timer(torch), Timer(torch)
        for i in range(3):
            f = lambda: eng.participant_share_dev(msk, sch, sec.data_ptr(), Dp, drw.data_ptr(), sh.data_ptr(),  # noqa
                                                  seed=seed, payload_ptr=pay.data_ptr(), payload_cap=cap,
                                                  stream=stream())
            pt.record(f) if i else f()
        pct = Timer(torch)
        for i in range(3):
            f = lambda: eng.participant_share_dev(msk, sch, sec.data_ptr(), Dp, drw.data_ptr(), sh.data_ptr(),  # noqa
                                                  seed=seed, payload_ptr=pay.data_ptr(), payload_cap=cap,
                                                  mode=E.REVEAL_CANONICAL, stream=stream())
            pct.record(f) if i else f()
        eng.participant_share_dev(msk, sch, sec.data_ptr(), Dp, drw.data_ptr(), sh.data_ptr(), seed=seed,
                                  stream=stream())       # the exact shares again for the round trip below
        idx = list(range(n - 1, n - 1 - (t + k), -1))
        sub = sh[idx].contiguous()
        out = torch.empty(Dp, dtype=torch.int64, device=dev)
        one = torch.tensor([seed], dtype=torch.int32, device=dev)
        eng.recipient_reveal_dev(msk, one.data_ptr(), 1, 4, sch, Dp, idx, sub.data_ptr(), B, p, out.data_ptr(), Dp,
                                 stream=stream())
        torch.cuda.synchronize()
        if not args.no_check and not torch.equal(out, sec):
            raise SystemExit("participant -> recipient round trip FAILED")
        Ns = args.chacha_seeds
        seeds = torch.randint(0, 2**31 - 1, (Ns, 4), dtype=torch.int32, device=dev,
                              generator=torch.Generator(device=dev).manual_seed(SEED_BASE + 10))
        for i in range(3):
            f = lambda: eng.recipient_reveal_dev(msk, seeds.data_ptr(), Ns, 4, sch, Dp, idx, sub.data_ptr(), B, p,  # noqa
                                                 out.data_ptr(), Dp, stream=stream())
            rt.record(f) if i else f()
        p_ms, r_ms, pc_ms = pt.mean_ms(), rt.mean_ms(), pct.mean_ms()
        side["pipelines"] = {
            "config": f"configs[4] per GPU: ChaCha(128-bit) masking + PackedShamir k=8 n=26 t=7 at {Dp:,}-dim",
            "participant_ms": p_ms, "participant_secrets_per_s": Dp / (p_ms * 1e-3),
            "participant_canonical_ms": pc_ms,
            "recipient_seeds": Ns, "recipient_ms": r_ms,
            "buffers": "torch.empty (inputs, shares, payloads); engine scratch: "
                       + ("sda_hbm_alloc chunks >= 256 MiB" if os.environ.get("SDA_SCRATCH_HBM") == "1" else "hipMalloc"),
            "recipient_mask_elems_per_s": Ns * Dp / (r_ms * 1e-3),
        }
        log(f"[pipelines] {json.dumps(side['pipelines'])}")
        del sec, drw, sh, pay, sub, out

    dist_info = None
    if world > 1:     # who took part: the driver's SCALE run can check that the communicator saw N ranks
        props = torch.cuda.get_device_properties(local)
        me = {"rank": rank, "local_rank": local, "device": local, "name": props.name,
              "pci_bus_id": getattr(props, "pci_bus_id", None), "pci_device_id": getattr(props, "pci_device_id", None)}
        allr = [None] * world
        dist.all_gather_object(allr, me)
        dist_info = {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": allr}
    if args.only is not None:
        return
    if rank == 0:
        traffic = traffic_from_profile(tile if tile else N, D)
        tr = roofline_trace(traffic[2], bytes_per_launch, kernel_ms)
        rec = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if tile else "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic: splitmix64 uniform [0, m) i64 shares, HBM-resident (no checkpoints/datasets)",
            "config": {"workload": ("AdditiveSharing clerk combine, 10k participations x 1M-dim i64 shares per GPU "
                                    "(BASELINE.json configs[1])") if not tile else
                                   ("Federated aggregation combine, 100k participations x 10M-dim in total, split over "
                                    "the GPUs, streamed through a resident 1000-row tile (BASELINE.json configs[3])"),
                       "participations_per_gpu": N, "dim": D, "modulus": m,
                       **({"tile_rows": tile, "participations_total": 100_000} if tile else {}),
                       "parallelism": f"participation split x{world}" + ((", RCCL int64 all-reduce" if backend == "nccl" else f", {backend} int64 all-reduce (rehearsal)")
                                                                       if world > 1 else ""),
                       "exact": "combiner.rs:16-28 recurrence, bit-exact",
                       "buffers": "torch.empty"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic[0], "traffic_source": traffic[1],
                         **({"trace": tr} if tr else {})},
            "kernel_ms": round(kernel_ms, 4),
            "kernel_bytes_per_launch": bytes_per_launch,
        }
        if dist_info is not None:
            rec["dist"] = dist_info
        rec.update(side)
        if multi is not None:
            rec["multi_device"] = multi
        if world == 1 and not args.no_cpu:
            rec["cpu_baseline"] = cpu_baseline(min(D, 1_000_000), args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_config4(args, torch, dist, eng, dev, stream, barrier, world, rank, backend):
    """BASELINE.json configs[4] from the recipient's side (receive.rs:80-157): 100k participants'
    128-bit ChaCha seeds expanded and combined over a 10M-dim vector (chacha.rs:57-76), the seeds split
    over the ranks with one int64 all-reduce + device finalize (sda_amd.distributed.mask_combine_sharded),
    then the packed reveal (k = 8, n = 26, t = 7, 15 clerks, exact) + unmask + positive() of each rank's
    slice of the batches (sda_recipient_reveal_dev with the combined mask as a Full mask row).  Step = all
    of it; value = mask elements expanded per second by all ranks."""
    from sda_amd import distributed as Dd, schemes as S
    from sda_amd import engine as E
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    D, total = 10_000_000, args.seeds
    B = D // k
    s0, cnt = Dd.shard_range(total, rank, world)
    allseeds = torch.randint(0, 2**31 - 1, (total, 4), dtype=torch.int32, device=dev,
                             generator=torch.Generator(device=dev).manual_seed(SEED_BASE + 5))
    seeds = allseeds[s0:s0 + cnt].contiguous()
    del allseeds
    partial = torch.empty(D, dtype=torch.int64, device=dev)
    mask = torch.empty(D, dtype=torch.int64, device=dev)
    # this rank's slice of the batches, and its clerks' shares of (secret + mask) mod p
    b0, nb = Dd.shard_range(B, rank, world)
    Dl = nb * k
    sec = torch.empty(Dl, dtype=torch.int64, device=dev)
    eng.synth_fill_dev(sec.data_ptr(), 1, Dl, SEED_BASE + 4, 0, p, stream())
    kt = Timer(torch)
    teng = TimedMask(eng, kt)
    Dd.mask_combine_sharded(teng, p, D, seeds, partial, mask)            # untimed: the shares' mask
    masked = torch.remainder(sec + mask[b0 * k:b0 * k + Dl], p)
    drw = torch.empty((nb, t), dtype=torch.int64, device=dev)
    eng.synth_fill_dev(drw.data_ptr(), nb, t, SEED_BASE + 44, 0, p - 1, stream())
    sh = torch.empty((n, nb), dtype=torch.int64, device=dev)
    eng.packed_generate_dev(sch, masked.data_ptr(), Dl, 1, drw.data_ptr(), sh.data_ptr(), stream())
    idx = list(range(n - (t + k), n))
    sub = sh[idx].contiguous()
    del masked, drw, sh
    out = torch.empty(Dl, dtype=torch.int64, device=dev)
    full = S.FullMasking(p)
    rt = Timer(torch)

    def step(timed):
        teng.timing = timed
        Dd.mask_combine_sharded(teng, p, D, seeds, partial, mask)
        f = lambda: eng.recipient_reveal_dev(full, mask[b0 * k:].data_ptr(), 1, Dl, sch, Dl, idx,  # noqa: E731
                                             sub.data_ptr(), nb, p, out.data_ptr(), Dl, E.REVEAL_EXACT, stream())
        rt.record(f) if timed else f()

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ok = torch.equal(out, sec)                 # positive(unmask(reveal)) == the secrets, every element
    if world > 1:
        okt = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    if not ok:
        raise SystemExit("configs[4] recipient round trip FAILED")
    mc_ms, rv_ms = kt.mean_ms(), rt.mean_ms()
    draws = float(total) * D
    log(f"[config4] rank {rank}: {args.steps} steps in {dt * 1e3:.1f} ms, mask combine {mc_ms:.2f} ms "
        f"({cnt} seeds), reveal {rv_ms:.3f} ms ({nb} batches)")
    if rank != 0:
        return
    rec = {
        "metric": "configs[4] recipient: ChaCha mask elements/s (seeds x 10M-dim mask combine + packed reveal)",
        "value": round(draws * args.steps / dt, 1), "unit": "mask elements/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic: device-generated 128-bit seeds and secrets (no datasets)",
        "config": {"workload": "BASELINE.json configs[4], recipient side: ChaCha(128-bit) mask combine of "
                               f"{total:,} seeds x {D:,}-dim + PackedShamir k=8 n=26 t=7 exact reveal from 15 "
                               "clerks + unmask + positive",
                   "seeds_per_gpu": cnt, "dim": D, "modulus": p,
                   "parallelism": f"seed split x{world}" + ((", RCCL int64 all-reduce" if backend == "nccl" else
                                                             f", {backend} int64 all-reduce (rehearsal)")
                                                            if world > 1 else "") + ", batch split reveal"},
        "mask_combine_kernel_ms": round(mc_ms, 3), "reveal_ms": round(rv_ms, 3),
        "chacha_blocks_per_s_per_gpu": cnt * D / 8 / (mc_ms * 1e-3),
        "check": "recipient output == the secrets on every element (all ranks)",
    }
    r = valu_roofline("chacha_combine", mc_ms, None, blocks=cnt * D / 8)
    if r:
        rec["roofline"] = r
    print(json.dumps(rec), flush=True)


class TimedMask:
    """HIP events around the ChaCha mask-combine launches of sda_amd.distributed.mask_combine_sharded."""

    def __init__(self, eng, timer):
        self.eng, self.timer = eng, timer
        self.timing = False

    def __getattr__(self, name):
        return getattr(self.eng, name)

    def chacha_mask_combine_dev(self, *a):
        if self.timing:
            self.timer.record(lambda: self.eng.chacha_mask_combine_dev(*a))
        else:
            self.eng.chacha_mask_combine_dev(*a)


def valu_roofline(key, ms, waves, blocks=None):
    """VALU issue roofline of an integer kernel (scripts/valu_mix.py -> profiles/valu_roofline.json):
    lane-ops per launch = SQ_INSTS_VALU (PMC, at this configuration) x 64, or the static VALU count of
    the straight-line kernel x its waves; achieved = lane-ops / live kernel time; peak = the kernel's
    instruction mix priced at the measured tools/ubench_int issue rates."""
    try:
        with open(os.path.join(ROOT, "profiles", "valu_roofline.json")) as f:
            k = json.load(f)["kernels"][key]
    except (OSError, ValueError, KeyError):
        return None
    if blocks is not None and k.get("pmc_valu_insts_per_launch") and k.get("pmc_blocks"):
        # another launch size of the same kernel: the PMC instruction count per ChaCha block, scaled
        insts = k["pmc_valu_insts_per_launch"] / k["pmc_blocks"] * blocks
        src = "PMC SQ_INSTS_VALU per block (256 x 1M launch) x blocks"
    elif blocks is None and k.get("pmc_valu_insts_per_launch") and (waves is None or k.get("pmc_waves") == waves):
        insts, src = k["pmc_valu_insts_per_launch"], "PMC SQ_INSTS_VALU"
    elif waves is not None:
        insts, src = k["static_valu"] * waves, "static VALU count x waves"
    else:
        return None
    achieved = insts * 64 / (ms * 1e-3) / 1e12
    r = {"bound": "valu", "achieved": round(achieved, 3), "peak": k["mix_ceiling_T_lane_ops"],
         "unit": "T lane-ops/s", "frac": round(achieved / k["mix_ceiling_T_lane_ops"], 4),
         "valu_insts_per_launch": insts, "source": src}
    if k.get("pattern_ceiling_T_lane_ops"):      # the kernel's dependent pattern timed alone (tools/ubench_bank)
        r["pattern_peak"] = k["pattern_ceiling_T_lane_ops"]
        r["pattern_frac"] = round(achieved / k["pattern_ceiling_T_lane_ops"], 4)
        r["pattern_source"] = k.get("pattern_source")
    return r


def traffic_from_profile(N, D):
    """(HBM bytes per combine launch, the profiles/ session they come from, that session's trace record) from
    the committed rocprofv3 PMC pass, if it was collected for this exact workload; FETCH_SIZE doubled per
    MI355X_MICROARCH.md §HBM.  (None, None, None) otherwise."""
    path = os.path.join(ROOT, "profiles", "combine_traffic.json")
    try:
        with open(path) as f:
            for t in json.load(f)["launches"]:
                if t.get("rows") == N and t.get("dim") == D:
                    return t["hbm_bytes_per_launch"], t.get("source"), t.get("trace")
    except (OSError, ValueError, KeyError):
        pass
    return None, None, None


def roofline_trace(trace, bytes_per_launch, kernel_ms):
    """The dominant kernel as the committed profile session saw it, beside this run's live HIP-event figure:
    that session's rocprofv3 kernel-trace average and the fraction it gives, and the same session's untraced
    HIP-event kernel time, so a difference between this line and the profile splits into tracing overhead
    (traced vs untraced on the profiled box) and box-to-box spread (untraced there vs live here)."""
    if not trace or not trace.get("kernel_avg_ms"):
        return None
    avg = trace["kernel_avg_ms"]
    r = {"session": trace.get("session"), "kernel_avg_ms": round(avg, 4),
         "frac": round(bytes_per_launch / (avg * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
         "dispatches": trace.get("dispatches")}
    un = trace.get("untraced_bench_kernel_ms")
    if un:
        r["untraced_kernel_ms_same_box"] = round(un, 4)
        r["tracing_overhead"] = round(avg / un - 1.0, 4)
        r["live_vs_profiled_box"] = round(kernel_ms / un - 1.0, 4)
    return r


if __name__ == "__main__":
    main()
