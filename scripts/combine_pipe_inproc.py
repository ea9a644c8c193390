"""In-process A/B of the combine kernel's software pipelining (SDA_COMBINE_PIPE, read per launch; "0" = off; during
round 6's tuning the knob also took the depths 2 / 4 / 6 / 8, profiles/r06m): one
10k x 1M i64 buffer, the variants interleaved launch block by launch block, HIP events on the launch stream, so
buffer placement and box state are shared by every variant.  Also checks the variants agree bit for bit.
    python scripts/combine_pipe_inproc.py [rounds] [variants ...]
SDA_INPROC_SHAPE=acc times the accumulating kernel on configs[3]'s 1000 x 10M tile instead; SDA_INPROC_KNOB names
the variable the variants set (default SDA_COMBINE_PIPE; e.g. SDA_COMBINE_BALANCE).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd import Engine  # noqa: E402

M = 2147482801
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
variants = sys.argv[2:] or ["0", "1"]
knob = os.environ.get("SDA_INPROC_KNOB", "SDA_COMBINE_PIPE")
torch.cuda.init()
eng = Engine(0)
acc = os.environ.get("SDA_INPROC_SHAPE") == "acc"
N, D = (1_000, 10_000_000) if acc else (10_000, 1_000_000)
x = torch.empty((N, D), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
eng.synth_fill_dev(x.data_ptr(), N, D, 0x5DB, -(M - 1), M, st)      # signed: the order-dependent worst case
outs = {v: torch.zeros(D, dtype=torch.int64, device="cuda") for v in variants}


def launch(v):
    if acc:
        eng.combine_accumulate_dev(M, x.data_ptr(), N, D, D, outs[v].data_ptr(), st)
    else:
        eng.combine_dev(M, x.data_ptr(), N, D, D, outs[v].data_ptr(), st)


res = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        os.environ[knob] = v
        launch(v)                                                                   # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            launch(v)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[v].append(ms)
        print(f"round {r} {knob}={v} {ms:.4f} ms  {8.0 * N * D / ms / 1e9:.3f} TB/s", flush=True)
same = all(torch.equal(outs[v], outs[variants[0]]) for v in variants)
for v in variants:
    s = sorted(res[v])
    print(f"{knob}={v}: median {s[len(s) // 2]:.4f} ms, min {s[0]:.4f}, max {s[-1]:.4f}")
print("bit-identical across variants:", same)
